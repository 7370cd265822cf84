"""Diagnostic: do two workspaces of one process, allocated side by side (so on different physical
pages), run the configs[1] step at different speeds?  Allocates the TrainStep's workspace, then a
second of the same size, and times the step on each alternately (den_timing per kernel class).
usage: python profiles/placement_probe2.py [steps] [rounds]"""
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
from placement_probe import measure  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ts, _ = bench.build_step(a, dev)
    ws = [ts.ws, torch.empty_like(ts.ws)]
    free, total = torch.cuda.mem_get_info(dev)
    out = {"ws_gb": round(ts.ws.numel() / 1e9, 1), "free_gb": round(free / 1e9, 1), "rows": []}
    for r in range(rounds):
        for i in (0, 1) if r % 2 == 0 else (1, 0):
            ts.ws = ws[i]
            ms, avg = measure(ts, steps)
            row = {"round": r, "ws": i, "ms_per_step": ms, "hidden": avg.get("hidden_bwd_kernel"),
                   "lb": avg.get("hidden_bwd_lb_kernel"), "dwstream": avg.get("dw_gemm_kernel"),
                   "fwd": avg.get("render_fwd_kernel"), "head": avg.get("render_bwd_kernel")}
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
