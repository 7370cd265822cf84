"""Diagnostic: the first steps of a bench process run slower (profiles/r06al_placement2*.jsonl: the
first 10 steps after the TrainStep is built, hidden 4.81-4.84 ms and forward 23.2-23.3 ms, every later
measurement 4.49-4.53 / 22.4-22.6 ms, on either of two workspaces).  This times consecutive windows of
steps from the start under one settle policy applied right after the workspace is allocated:
  none   -- as bench.py before r06
  zero   -- the workspace written once (ws.zero_(), every page touched) and synchronised
  sleep  -- 2 s idle
  second -- a second buffer of the workspace's size allocated and kept (never used)
usage: python profiles/settle_probe.py POLICY [windows] [steps_per_window]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "profiles"))

import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402


def main():
    policy = sys.argv[1]
    windows = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    t_alloc = time.perf_counter()
    ts, _ = bench.build_step(a, dev)
    torch.cuda.synchronize()
    if policy == "zero":
        ts.ws.zero_()
        torch.cuda.synchronize()
    elif policy == "sleep":
        time.sleep(2.0)
    elif policy == "second":
        spare = torch.empty_like(ts.ws)  # noqa: F841 (kept alive for the whole run)
    out = {"policy": policy, "setup_s": round(time.perf_counter() - t_alloc, 2), "windows": []}
    nat.timing_enable(True)
    nat.timing_collect()
    for w in range(windows):
        t0 = time.perf_counter()
        for _ in range(per):
            ts.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / per * 1e3
        got = nat.timing_collect()
        row = {"window": w, "ms_per_step": round(ms, 2),
               "hidden": round(got["hidden_bwd_kernel"][0] / max(got["hidden_bwd_kernel"][1], 1), 3),
               "fwd": round(got["render_fwd_kernel"][0] / max(got["render_fwd_kernel"][1], 1), 3)}
        out["windows"].append(row)
    nat.timing_enable(False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
