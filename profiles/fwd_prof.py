"""Experiment: per-wave cycle split of the BF16 render forward (s_memtime around each weight-chunk
step: body = MFMA chain + epilogue + stores, wait = vmcnt wait for the next chunk, barrier).
Needs a DEN_FWD_PROF build of libden (make variant NAME=prof DEFS=-DDEN_FWD_PROF), selected with
DEN_LIB.  usage: DEN_LIB=deblur-e-nerf_amd/libden_prof.so python profiles/fwd_prof.py [train]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from deblur_e_nerf import _native as nat  # noqa: E402
from _util import flat_from_params, synthetic_rays  # noqa: E402
from oracle import nerf as onerf  # noqa: E402


def main():
    train = len(sys.argv) < 2 or sys.argv[1] == "train"
    R, S, rd = 131072, 128, 1
    o, d, u = synthetic_rays(R, seed=5, device="cuda")
    flat = flat_from_params(onerf.build_params(rd, 1), rd).cuda().requires_grad_(train)
    packed = nat.PackedWeights("bf16", rd, "cuda")
    packed.pack(flat.detach())
    cfg = dict(mode=nat.mode_id("bf16"), rd=rd, aabb=list(onerf.AABB_CHAIR), near=1.43, far=6.63)
    lib = nat.lib()
    lib.den_debug_fwd_prof.argtypes = [ctypes.c_void_p]
    buf = np.zeros(512 * 8 * 8, dtype=np.uint64)
    ms = []
    for it in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.set_grad_enabled(train):
            e0.record()
            c, op, dp = nat.render(o, d, u, None, flat, cfg, packed, S)
            e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        del c, op, dp
    print(f"render call ms (incl. host glue): {['%.2f' % m for m in ms]}")
    assert lib.den_debug_fwd_prof(buf.ctypes.data) == 0
    p = buf.reshape(512, 8, 8).astype(np.float64)
    waves = p[:, :, 6] > 0
    # persistent kernel (r04): [0..2] summed body / vmcnt wait / barrier cycles of the weight-chunk
    # steps, [3] kernel start, [4] summed item prologues (sampling + encoding), [5] summed item
    # tails (activations + compositing), [6] kernel end
    start, end = p[:, :, 3], p[:, :, 6]
    tot = (end - start)[waves]
    print(f"train={train} waves={waves.sum()} (first 512 workgroups) wave cycles mean {tot.mean():.0f}")
    for name, v in (("prologues", p[:, :, 4][waves]), ("tails", p[:, :, 5][waves])):
        print(f"  {name:9s} {v.mean():10.0f} cyc/wave ({v.mean() / tot.mean() * 100:5.1f} %)")
    for q, name in enumerate(["body", "vm wait", "barrier"]):
        v = p[:, :, q][waves]
        print(f"    {name:8s} {v.mean():10.0f} cyc/wave ({v.mean() / tot.mean() * 100:5.1f} %)")
    # by wave index: waves w and w + 4 share SIMD w; waves 0 .. rays_per_wg - 1 composite a ray in each
    # item's tail (den_render.hip)
    # [7]: the per-sample outputs + record stores of the tail (r05bb on: the whole tail)
    v7 = p[:, :, 7][waves]
    print(f"  tail outputs {v7.mean():10.0f} cyc/wave ({v7.mean() / tot.mean() * 100:5.1f} %)")
    for name, q in (("tails", 5), ("barrier", 2), ("body", 0), ("pre-barrier tail", 7)):
        row = [p[:, w, q][waves[:, w]].mean() / tot.mean() * 100 for w in range(8)]
        print(f"  {name:8s} by wave: " + " ".join(f"{x:5.1f}" for x in row) + " %")
    per_wave = p[:, :, 0][waves]
    print(f"  body min/max over waves {per_wave.min():.0f} / {per_wave.max():.0f}")
    wg0 = start[:, 0][waves[:, 0]]
    wg1 = end.max(1)[waves[:, 0]]
    span = (wg1.max() - wg0.min())
    print(f"  512 workgroups span {span:.0f} cycles; sum of their lifetimes / span = "
          f"{(wg1 - wg0).sum() / span:.1f} workgroups resident on average")


if __name__ == "__main__":
    main()
