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


def test_gpus8_stub_shards_eight_ranks():
    # the driver's largest scaling point: 8 ranks (gloo on the CPU here), R / 8 rays each
    p, lines = _run("--gpus", "8")
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "ray-dp8"
    assert out["config"]["rays_per_rank"] * 8 == out["config"]["rays_per_step"] == 131072


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _FakeDist:
    def __init__(self, world):
        self.world, self.calls = world, []

    def init_process_group(self, backend, **kw):
        self.calls.append((backend, kw))

    def get_world_size(self):
        return self.world


class _FakeCuda:
    def __init__(self, count):
        self.count, self.bound = count, []

    def device_count(self):
        return self.count

    def set_device(self, d):
        self.bound.append(d)


def test_rccl_branch_wiring_eight_ranks(monkeypatch):
    """The nccl (= RCCL) branch bench.py takes on an 8-GPU node: every local rank binds its own
    device and joins the group on it; the dmabuf IPC mode is set for RCCL."""
    import argparse
    import torch
    bench = _bench_module()
    monkeypatch.delenv("HSA_ENABLE_IPC_MODE_LEGACY", raising=False)
    a = argparse.Namespace(dist_backend="nccl")
    for local in range(8):
        fd, fc = _FakeDist(8), _FakeCuda(8)
        world, dev = bench.init_ranks(a, 8, local, dist_mod=fd, cuda=fc)
        assert world == 8 and dev == torch.device("cuda", local)
        assert fc.bound == [local]
        assert fd.calls == [("nccl", {"device_id": torch.device("cuda", local)})]
    assert os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # the gloo rehearsal folds 8 ranks onto the card(s) present
    fd, fc = _FakeDist(8), _FakeCuda(1)
    world, dev = bench.init_ranks(argparse.Namespace(dist_backend="gloo"), 8, 5, dist_mod=fd, cuda=fc)
    assert dev == torch.device("cuda", 0) and fd.calls == [("gloo", {})]
    # one rank: no process group at all
    fd, fc = _FakeDist(1), _FakeCuda(1)
    assert bench.init_ranks(a, 1, 0, dist_mod=fd, cuda=fc) == (1, torch.device("cuda", 0)) and not fd.calls


def test_launcher_command_for_eight_gpus(monkeypatch):
    """`bench.py --gpus 8` outside a launcher starts torch.distributed.run with 8 ranks on
    127.0.0.1 as a child process, relaying its exit code."""
    bench = _bench_module()
    seen = {}

    class _P:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return _P()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5"])
    a = bench.parse()
    assert a.gpus == 8
    assert bench.launch_ranks(a) == 7
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_gpus_defaults_to_world_size(monkeypatch):
    bench = _bench_module()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.parse().gpus == 4
    monkeypatch.delenv("WORLD_SIZE")
    a = bench.parse()
    assert a.gpus == 1 and a.psnr_steps == bench.PSNR_LEG["steps"]
