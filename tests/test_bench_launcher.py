"""bench.py's multi-rank entry point (the driver's `bench.py --gpus N` contract).

`python bench.py --gpus 2` run outside a launcher must start 2 ranks (one process per GPU,
scripts/run.py:84-100's DDP plugin) as a child `torch.distributed.run`, relay rank 0's JSON line
and exit code, and report n_gpus from the process group.  `--cpu-stub` keeps the launcher,
sharding (R / world rays per rank) and the timed-region contract but replaces the HIP step by a
CPU stub on gloo, so this runs without a GPU.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-stub", "--steps", "3", "--warmup", "1",
                        *args], capture_output=True, text=True, timeout=240, env=env, cwd="/tmp")
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


def test_gpus2_launches_two_ranks():
    p, lines = _run("--gpus", "2")
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["rays_per_step"] == 131072
    assert out["config"]["rays_per_rank"] == 131072 // 2
    assert out["config"]["parallelism"] == "ray-dp2"
    assert out["value"] > 0 and out["steps"] == 3 and out["warmup"] == 1


def test_gpus1_single_process():
    p, lines = _run("--gpus", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(lines[-1])
    assert out["n_gpus"] == 1 and out["config"]["rays_per_rank"] == 131072


def test_world_mismatch_fails_loudly():
    # a launcher that started fewer ranks than --gpus asks for is an error, not a 1-rank line
    p, lines = _run("--gpus", "2", env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and not lines
    assert "WORLD_SIZE" in p.stderr
