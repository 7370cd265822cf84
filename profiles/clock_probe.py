"""Diagnostic: the clock each hot kernel holds inside the configs[1] training step (MI355X_MICROARCH.md
'DVFS give-back' item 6).  Needs the DEN_CLOCK build (make variant NAME=clock DEFS=-DDEN_CLOCK),
selected with DEN_LIB: every kernel stamps s_memtime / s_memrealtime once at start and end per
workgroup into a buffer of its own.  Runs the BF16 step back to back for >= `secs` seconds on the
benchmark's synthetic data (random-init weights, so random operands), then reads the last step's
stamps: clock = delta memtime / delta realtime x 100 MHz, median / min / max over workgroups, and
the stamped span against the kernel's own wall.
usage: DEN_LIB=deblur-e-nerf_amd/libden_clock.so python profiles/clock_probe.py [secs] [tag]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402

KERNELS = ["render_fwd", "render_head_bwd", "hidden_bwd (L1, the step's last)", "hidden_bwd Lb", "dwstream"]


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    tag = sys.argv[2] if len(sys.argv) > 2 else "probe"
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ts, _ = bench.build_step(a, dev)
    lib = nat.lib()
    lib.den_debug_clock.argtypes = [ctypes.c_void_p]
    for _ in range(3):
        ts.step()
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < secs:
        ts.step()
        n += 1
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    buf = np.zeros(5 * 512 * 4, dtype=np.uint64)
    assert lib.den_debug_clock(buf.ctypes.data) == 0
    st = buf.reshape(5, 512, 4).astype(np.float64)
    out = {"tag": tag, "steps": n, "ms_per_step": round(wall, 3), "kernels": {}}
    for k, name in enumerate(KERNELS):
        s = st[k]
        ok = (s[:, 3] > s[:, 1]) & (s[:, 2] > s[:, 0])
        if not ok.any():
            continue
        s = s[ok]
        ghz = (s[:, 2] - s[:, 0]) / (s[:, 3] - s[:, 1]) * 100e6 / 1e9
        span_ms = (s[:, 3].max() - s[:, 1].min()) / 100e6 * 1e3
        out["kernels"][name] = {"workgroups": int(ok.sum()), "ghz_median": round(float(np.median(ghz)), 4),
                                "ghz_min": round(float(ghz.min()), 4), "ghz_max": round(float(ghz.max()), 4),
                                "span_ms": round(float(span_ms), 3),
                                "wg_ms_median": round(float(np.median((s[:, 3] - s[:, 1]) / 1e5)), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
