"""Diagnostic: does the configs[1] step's speed depend on where in HBM its workspace lands?  Bench
processes run back to back alternate between two speeds (profiles/r06t_ab.jsonl, r06z_ab.jsonl: the
hidden launches ~5 % apart by position, identical ISA).  Here one process times the step and its
kernel classes with the workspace allocated first, then re-allocated behind dummy allocations of
several sizes (so it lands on other physical pages), each measured twice.
usage: python profiles/placement_probe.py [steps]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402

def measure(ts, steps):
    for _ in range(2):
        ts.step()
    torch.cuda.synchronize()
    nat.timing_enable(True)
    nat.timing_collect()
    t0 = time.perf_counter()
    for _ in range(steps):
        ts.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    got = nat.timing_collect()
    nat.timing_enable(False)
    return round(ms, 3), {k: round(t / n, 4) for k, (t, n) in got.items() if n}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ts, _ = bench.build_step(a, dev)
    nbytes = ts.ws.numel()
    free0, total = torch.cuda.mem_get_info(dev)
    out = {"ws_gb": round(nbytes / 1e9, 2), "free_gb_after_ws": round(free0 / 1e9, 2), "total_gb": round(total / 1e9, 2),
           "rows": []}
    dummies = [0, 0, 40, 80, 120, 0]
    for dgb in dummies:
        del ts.ws
        torch.cuda.empty_cache()
        dummy = torch.empty(int(dgb * 1e9), dtype=torch.uint8, device=dev) if dgb else None
        ts.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        ms, avg = measure(ts, steps)
        row = {"dummy_gb": dgb, "ws_ptr_gb": round(ts.ws.data_ptr() / 2 ** 30, 1), "ms_per_step": ms, "avg_ms": avg}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
        del dummy
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
