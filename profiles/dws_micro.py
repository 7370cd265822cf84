"""r05: the streamed weight-gradient launch (den_render_bwd_part part 2) timed alone, repeatedly, after
one full step -- versus its time inside the step (bench.py's phase timing): does the launch's cost
depend on what ran before it?"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deblur-e-nerf_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402


def main():
    sys.argv = ["bench.py", "--no-cpu-baseline", "--no-extra-legs", "--psnr-steps", "0"]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ts, _ = bench.build_step(a, dev, 0, 1)
    for _ in range(3):
        ts.step()
    torch.cuda.synchronize()
    L = nat.lib()
    st = nat._stream(dev)
    gr = nat.RenderGrad(nat._ptr(ts.d_rgb), None, None, nat._ptr(ts.grad), nat._ptr(ts.grad_bkgd))
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    out = {}
    for name, part in (("part2_alone", 2), ("part1_alone", 1), ("part2_alone_again", 2)):
        ts_ = []
        for _ in range(6):
            e0, e1 = ev(), ev()
            e0.record()
            nat._check(L.den_render_bwd_part(ctypes.byref(ts.desc), ctypes.byref(ts.io), ctypes.byref(gr), part, st))
            e1.record()
            torch.cuda.synchronize()
            ts_.append(round(e0.elapsed_time(e1), 3))
        out[name] = ts_
    # part 2 right after part 1, alternating
    seq = []
    for _ in range(4):
        e = [ev() for _ in range(3)]
        e[0].record()
        nat._check(L.den_render_bwd_part(ctypes.byref(ts.desc), ctypes.byref(ts.io), ctypes.byref(gr), 1, st))
        e[1].record()
        nat._check(L.den_render_bwd_part(ctypes.byref(ts.desc), ctypes.byref(ts.io), ctypes.byref(gr), 2, st))
        e[2].record()
        torch.cuda.synchronize()
        seq.append((round(e[0].elapsed_time(e[1]), 3), round(e[1].elapsed_time(e[2]), 3)))
    out["part1_then_part2"] = seq
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
