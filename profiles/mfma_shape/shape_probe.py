"""A/B of the two bf16 MFMA shapes on the forward's layer body (shape_probe.hip): wall time and the
clock held, on random data, after >= `warm` seconds of back-to-back launches, alternating shapes.
usage: python profiles/mfma_shape/shape_probe.py [rounds] [warm_s] [layers]   (build: make -C profiles/mfma_shape;
PROBE_LIB=<path> selects another build, e.g. libshape_probe_pf.so: the 16x16x32 body with its A fragments
one k-block ahead, make -C profiles/mfma_shape pf)"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
WAVES = 8


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    warm = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    layers = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    lib = ctypes.CDLL(os.environ.get("PROBE_LIB", os.path.join(HERE, "libshape_probe.so")))
    lib.shape_probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    grid = torch.cuda.get_device_properties(dev).multi_processor_count
    g = torch.Generator().manual_seed(3)
    # weights ~ U(-1, 1) / 16 (PyTorch's default Linear bound for K = 256), activations ~ U(0, 4)
    w = ((torch.rand(256 * 256, generator=g) * 2 - 1) / 16).to(torch.bfloat16).to(dev)
    n_frag = grid * WAVES * 16 * 64 * 8
    b0 = (torch.rand(n_frag, generator=g) * 4).to(torch.bfloat16).to(dev)
    out = torch.empty_like(b0)
    clk = torch.zeros(grid * 4, dtype=torch.int64, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def launch(shape):
        rc = lib.shape_probe_launch(shape, grid, ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(b0.data_ptr()), 0.05,
                                    layers, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(clk.data_ptr()), stream)
        assert rc == 0, rc

    flop = 2.0 * 256 * 256 * 32 * WAVES * grid * layers
    res = {"grid": grid, "layers": layers, "flop_per_launch": flop, "rounds": []}
    outs = {}
    for shape in (32, 16):
        launch(shape)
        torch.cuda.synchronize()
        outs[shape] = out.float().cpu()
    # the two shapes compute the same layer function up to the k-order of the chain (different, since
    # the weights are read in each shape's own fragment order): record the output statistics only
    res["out_mean"] = {s: float(o.mean()) for s, o in outs.items()}
    res["out_finite"] = {s: bool(torch.isfinite(o).all()) for s, o in outs.items()}
    for r in range(rounds):
        for shape in ((32, 16) if r % 2 == 0 else (16, 32)):
            t_end = time.perf_counter() + warm
            while time.perf_counter() < t_end:
                launch(shape)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 10
            e0.record()
            for _ in range(n):
                launch(shape)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / n
            c = clk.cpu().numpy().reshape(grid, 4).astype(np.float64)
            ok = (c[:, 3] > c[:, 1]) & (c[:, 2] > c[:, 0])
            ghz = (c[ok, 2] - c[ok, 0]) / (c[ok, 3] - c[ok, 1]) * 0.1
            cyc = float(np.median(c[ok, 2] - c[ok, 0]))
            row = {"round": r, "shape": f"{shape}x{shape}x{512 // shape}", "ms": round(ms, 4),
                   "tflops": round(flop / ms / 1e9, 1), "ghz_median": round(float(np.median(ghz)), 4),
                   "ghz_min": round(float(ghz.min()), 4), "ghz_max": round(float(ghz.max()), 4),
                   "cycles_median": cyc}
            res["rounds"].append(row)
            print(json.dumps(row), flush=True)
    for shape in ("32x32x16", "16x16x32"):
        rows = [x for x in res["rounds"] if x["shape"] == shape]
        res[shape] = {"ms_median": float(np.median([x["ms"] for x in rows])),
                      "ghz_median": float(np.median([x["ghz_median"] for x in rows])),
                      "cycles_median": float(np.median([x["cycles_median"] for x in rows]))}
    res["ratio_wall_32_over_16"] = res["32x32x16"]["ms_median"] / res["16x16x32"]["ms_median"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
