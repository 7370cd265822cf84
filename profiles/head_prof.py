"""Experiment: per-wave cycle split of the BF16 head backward (render_head_bwd_kernel, s_memtime
between its phases: 0 compositing adjoint, 1 the barrier after it, 2 the Lr^T chain (+ fused Lr dW),
3 dz_g staging + the ve tile, 4 the Lg^T chain + sigma's dz, 5 the fused Lg weight-gradient loop;
6 the whole launch; 7 items of the workgroup).  Needs a DEN_HEAD_PROF build (make variant NAME=hprof
DEFS=-DDEN_HEAD_PROF), selected with DEN_LIB.
usage: DEN_LIB=deblur-e-nerf_amd/libden_hprof.so python profiles/head_prof.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deblur-e-nerf_amd")]
import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402

NAMES = ["adjoint", "adjoint_barrier", "lr_chain", "stage_ve", "lg_chain", "lg_dw", "launch", "items"]


def main():
    sys.argv = ["bench.py", "--no-cpu-baseline", "--no-extra-legs", "--psnr-steps", "0"]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ts, _ = bench.build_step(a, dev, 0, 1)
    for _ in range(3):
        ts.step()
    torch.cuda.synchronize()
    lib = nat.lib()
    lib.den_debug_head_prof.argtypes = [ctypes.c_void_p]
    buf = np.zeros(256 * 8 * 8, dtype=np.uint64)
    nat._check(lib.den_debug_head_prof(buf.ctypes.data))
    p = buf.reshape(256, 8, 8).astype(np.float64)
    items = p[:, 0, 7].mean()
    out = {"items_per_wg": items, "launch_cycles_mean": p[:, :, 6].mean(),
           "per_item_cycles_by_wave": {NAMES[q]: [round(float(p[:, w, q].mean() / items)) for w in range(8)]
                                        for q in range(6)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
