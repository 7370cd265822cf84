"""Experiment: per-wave cycle split of the layer-major hidden backward (den_hidden.hip HbProf marks):
DMA issue, chain (dz fragments + W^T MFMAs), epilogue (activation derivative + dz stores), dW / db,
Lb's sigma weight-gradient row, the vmcnt wait for the next block, the barrier -- for the last L7..L1
launch of a step (L1) and for Lb.  Needs the DEN_HIDDEN_PROF build
(make variant NAME=hidprof DEFS=-DDEN_HIDDEN_PROF), selected with DEN_LIB.  Runs the configs[1] BF16
step (bench.build_step) a few times and reads the last step's marks.
usage: DEN_LIB=deblur-e-nerf_amd/libden_hidprof.so python profiles/hidden_prof.py [steps]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402

PHASES = ["dma_issue", "chain", "epilogue", "dW", "sigma_row", "vm_wait", "barrier"]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    ts, _ = bench.build_step(a, torch.device("cuda", 0))
    lib = nat.lib()
    lib.den_debug_hidden_prof.argtypes = [ctypes.c_void_p]
    for _ in range(steps):
        ts.step()
    torch.cuda.synchronize()
    nat.timing_enable(True)
    ts.step()
    torch.cuda.synchronize()
    nat.timing_enable(False)
    kt = nat.timing_collect()
    buf = np.zeros(2 * 256 * 8 * 8, dtype=np.uint64)
    assert lib.den_debug_hidden_prof(buf.ctypes.data) == 0
    p = buf.reshape(2, 256, 8, 8).astype(np.float64)
    out = {"kernel_ms": {k: round(v[0] / max(v[1], 1), 4) for k, v in kt.items() if v[1]}, "launches": {}}
    n_blocks = a.rays * a.samples // 32
    for s, name in enumerate(("L1", "Lb")):
        tot = p[s, :, :, 7]
        row = {"cycles_per_wave": round(float(tot.mean()), 0), "blocks_per_wg": n_blocks / 256}
        for q, ph in enumerate(PHASES):
            v = p[s, :, :, q]
            row[ph] = {"cyc_per_block": round(float(v.mean()) / (n_blocks / 256), 1),
                       "share": round(float(v.mean() / tot.mean()), 4)}
        # by wave (8, two per SIMD): the barrier share tells which wave finishes its block last
        row["barrier_share_by_wave"] = [round(float(p[s, :, w, 6].mean() / tot.mean()), 4) for w in range(8)]
        row["dma_issue_share_by_wave"] = [round(float(p[s, :, w, 0].mean() / tot.mean()), 4) for w in range(8)]
        out["launches"][name] = row
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
