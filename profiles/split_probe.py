"""Diagnostic: does the configs[1] step gain from running one half's forward beside the other half's
backward?  The 4N rays split into the diff groups [0, 2N) and the TV groups [2N, 4N), whose losses
and gradients are independent (den_misc.hip event_step_*).  Sequential (the product step's render
part): fwd(all) ; bwd(all).  Split: fwd(A) on every CU ; [fwd(B) on <= gf workgroups, stream 2] beside
[bwd(A) on <= gb workgroups, stream 1] ; bwd(B) on every CU.  Times the render part only (the loss
kernels take microseconds), alternating the two orders, with the gradients of the split summed and
compared against the sequential gradient (f32 summation order only) and the radiance bit for bit.
usage: python profiles/split_probe.py [reps] [gf:gb ...]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from deblur_e_nerf import _native as nat  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    splits = [tuple(int(v) for v in s.split(":")) for s in sys.argv[2:]] or [(128, 128), (112, 144), (96, 160)]
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    ts, _ = bench.build_step(a, dev)
    for _ in range(2):
        ts.step()
    ts.forward()  # d_rgb of the current weights
    torch.cuda.synchronize()
    L = nat.lib()
    R, S, P = ts.R, ts.S, ts.P
    full = nat._desc(ts.cfg, R, S, True, ts.has_bkgd)
    half = nat._desc(ts.cfg, R // 2, S, True, ts.has_bkgd)
    hb = nat.render_workspace_bytes(half)
    hb = (hb + 4095) // 4096 * 4096
    fb = nat.render_workspace_bytes(full)
    del ts.ws
    torch.cuda.empty_cache()
    ws = torch.empty(max(fb, 2 * hb), dtype=torch.uint8, device=dev)
    bkgd = torch.nn.functional.softplus(ts.bkgd_orig) if ts.has_bkgd else None
    rgb, op, dep = torch.empty_like(ts.rgb), torch.empty_like(ts.opacity), torch.empty_like(ts.depth)
    d_rgb = ts.d_rgb.clone()
    pk = ts.packed

    def io(r0, r1, w):
        return nat.RenderIO(nat._ptr(ts.rays_o[r0:r1]), nat._ptr(ts.rays_d[r0:r1]), nat._ptr(ts.jitter[r0:r1]),
                            nat._ptr(pk.fwd), nat._ptr(pk.bwd), nat._ptr(pk.bias), nat._ptr(bkgd), ctypes.c_void_p(w),
                            nat._ptr(rgb[r0:r1]), nat._ptr(op[r0:r1]), nat._ptr(dep[r0:r1]))

    def grad(r0, r1, g):
        gb = torch.zeros(ts.rd, device=dev)
        return nat.RenderGrad(nat._ptr(d_rgb[r0:r1]), None, None, nat._ptr(g), nat._ptr(gb) if ts.has_bkgd else None), gb

    io_full = io(0, R, ws.data_ptr())
    io_a, io_b = io(0, R // 2, ws.data_ptr()), io(R // 2, R, ws.data_ptr() + hb)
    g_full, g_a, g_b = (torch.zeros(P, device=dev) for _ in range(3))
    gr_full, _ = grad(0, R, g_full)
    gr_a, _ = grad(0, R // 2, g_a)
    gr_b, _ = grad(R // 2, R, g_b)
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(dev)
    h1, h2 = ctypes.c_void_p(s1.cuda_stream), ctypes.c_void_p(s2.cuda_stream)

    def seq():
        full.max_workgroups = 0
        nat._check(L.den_render_fwd(ctypes.byref(full), ctypes.byref(io_full), h1))
        nat._check(L.den_render_bwd(ctypes.byref(full), ctypes.byref(io_full), ctypes.byref(gr_full), h1))

    da, db = nat._desc(ts.cfg, R // 2, S, True, ts.has_bkgd), nat._desc(ts.cfg, R // 2, S, True, ts.has_bkgd)

    def split(gf, gb):
        da.max_workgroups = 0
        nat._check(L.den_render_fwd(ctypes.byref(da), ctypes.byref(io_a), h1))
        e1 = torch.cuda.Event()
        e1.record(s1)
        s2.wait_event(e1)
        db.max_workgroups = gf
        nat._check(L.den_render_fwd(ctypes.byref(db), ctypes.byref(io_b), h2))
        da.max_workgroups = gb
        nat._check(L.den_render_bwd(ctypes.byref(da), ctypes.byref(io_a), ctypes.byref(gr_a), h1))
        e2 = torch.cuda.Event()
        e2.record(s2)
        s1.wait_event(e2)
        db.max_workgroups = 0
        nat._check(L.den_render_bwd(ctypes.byref(db), ctypes.byref(io_b), ctypes.byref(gr_b), h1))

    def timed(fn, *args):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(s1)
        fn(*args)
        t1.record(s1)
        t1.synchronize()
        return t0.elapsed_time(t1)

    # correctness: the split's radiance bit for bit, its summed gradient against the sequential one
    seq()
    torch.cuda.synchronize()
    rgb_seq, g_seq = rgb.clone(), g_full.clone()
    split(*splits[0])
    torch.cuda.synchronize()
    g_sum = g_a + g_b
    out = {"rgb_equal": bool(torch.equal(rgb, rgb_seq)),
           "grad_rel": float((g_sum - g_seq).norm() / g_seq.norm()), "reps": reps, "runs": {}}
    print(json.dumps(out), flush=True)
    for _ in range(2):
        seq()
        split(*splits[0])
    torch.cuda.synchronize()
    res = {"seq": []}
    for sp in splits:
        res[f"{sp[0]}:{sp[1]}"] = []
    for _ in range(reps):
        res["seq"].append(timed(seq))
        for sp in splits:
            res[f"{sp[0]}:{sp[1]}"].append(timed(split, *sp))
    for k, v in res.items():
        v = sorted(v)
        out["runs"][k] = {"median_ms": round(v[len(v) // 2], 3), "min_ms": round(v[0], 3), "max_ms": round(v[-1], 3)}
    # the phases alone: the half forward on all CUs and on gf, the half backward on all CUs and on gb
    ph = {}
    for name, d_, i_, g_, cap in [("fwdA_all", da, io_a, None, 0), ("bwdA_all", da, io_a, gr_a, 0)] + \
            [(f"fwdB_{gf}", db, io_b, None, gf) for gf, _ in splits] + [(f"bwdA_{gb}", da, io_a, gr_a, gb) for _, gb in splits]:
        d_.max_workgroups = cap
        if g_ is None:
            f = lambda: nat._check(L.den_render_fwd(ctypes.byref(d_), ctypes.byref(i_), h1))
        else:
            nat._check(L.den_render_fwd(ctypes.byref(d_), ctypes.byref(i_), h1))  # fresh activations
            f = lambda: nat._check(L.den_render_bwd(ctypes.byref(d_), ctypes.byref(i_), ctypes.byref(g_), h1))
        ph[name] = round(timed(f), 3)
    out["phases_ms"] = ph
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
