"""Byte rate of the hidden backward's memory pattern (read two 16 KiB blocks, write one, per 32-sample
block; 2^19 blocks = configs[1]'s 25.8 GB per launch) issued several ways (stream_probe.hip).
usage: python profiles/stream_probe/stream_probe.py [reps]   (build: make -C profiles/stream_probe)"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
BLOCK = 16384

# (name, variant, grid, waves, layout): layout "sep" three tensors (the product's since r06n), "inplace"
# output over the second read (the product before r06n), "skew" the three tensors offset by 0 / 8 / 4 KiB
# + n 16 KiB, "inter48" one buffer with blocks [a | b | c] back to back, "bm128" one buffer of 8-slot
# block-major rows (a slot 5, b slot 3, c slot 4: the three activations of one layer launch)
CONFIGS = [
    ("lds_dma_inplace (before r06n)", 0, 256, 4, "inplace"),
    ("lds_dma_separate (r06n)", 1, 256, 4, "sep"),
    ("lds_dma_separate_depth2", 4, 256, 4, "sep"),
    ("lds_dma_separate_depth4", 5, 256, 4, "sep"),
    ("lds_dma_skew", 1, 256, 4, "skew"),
    ("lds_dma_interleaved48", 1, 256, 4, "inter48"),
    ("lds_dma_blockmajor128", 1, 256, 4, "bm128"),
    ("regs_nt_256x4", 2, 256, 4, "sep"),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lib = ctypes.CDLL(os.path.join(HERE, "libstream_probe.so"))
    lib.stream_probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_blocks = 1 << 19
    nb = n_blocks * BLOCK
    # one pool for every layout: 8 slots per block (bm128 needs them all)
    pool = torch.randint(0, 2 ** 31 - 1, (8 * nb // 4 + 3 * 8192,), dtype=torch.int32, device=dev)
    p0 = pool.data_ptr()

    def ptrs(layout):
        if layout in ("sep", "inplace"):
            a, b, c = p0, p0 + nb, p0 + 2 * nb
            return a, b, (b if layout == "inplace" else c), BLOCK
        if layout == "skew":
            return p0, p0 + nb + 8192 + 16384, p0 + 2 * nb + 4096 + 32768, BLOCK
        if layout == "inter48":
            return p0, p0 + BLOCK, p0 + 2 * BLOCK, 3 * BLOCK
        if layout == "bm128":
            return p0 + 5 * BLOCK, p0 + 3 * BLOCK, p0 + 4 * BLOCK, 8 * BLOCK
        raise ValueError(layout)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    moved = 3.0 * n_blocks * BLOCK
    out = {"n_blocks": n_blocks, "bytes_per_launch": moved, "rows": []}
    for rnd in range(2):
        for name, v, grid, waves, layout in (CONFIGS if rnd == 0 else CONFIGS[::-1]):
            a, b, c, stride = ptrs(layout)

            def go():
                rc = lib.stream_probe_launch(v, grid, waves, ctypes.c_void_p(a), ctypes.c_void_p(b), ctypes.c_void_p(c),
                                             n_blocks, stride, st)
                assert rc == 0, (name, rc)
            for _ in range(2):
                go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                go()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / reps
            row = {"round": rnd, "config": name, "ms": round(ms, 4), "tb_s": round(moved / ms / 1e9, 3)}
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
