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

CONFIGS = [  # (name, variant, grid, waves, in_place)
    ("lds_dma_inplace_256x4 (hidden_bwd_kernel's)", 0, 256, 4, True),
    ("lds_dma_separate_256x4", 1, 256, 4, False),
    ("regs_nt_256x4", 2, 256, 4, False),
    ("regs_nt_256x8", 2, 256, 8, False),
    ("regs_nt_512x8", 2, 512, 8, False),
    ("regs_nt_1024x8", 2, 1024, 8, False),
    ("regs_nt_512x8_inplace", 2, 512, 8, True),
    ("regs_cached_512x8", 3, 512, 8, False),
    ("regs_cached_512x8_inplace", 3, 512, 8, True),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lib = ctypes.CDLL(os.path.join(HERE, "libstream_probe.so"))
    lib.stream_probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_blocks = 1 << 19
    a = torch.randint(0, 2 ** 31 - 1, (n_blocks * BLOCK // 4,), dtype=torch.int32, device=dev)
    b = torch.randint(0, 2 ** 31 - 1, (n_blocks * BLOCK // 4,), dtype=torch.int32, device=dev)
    c = torch.empty_like(a)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    moved = 3.0 * n_blocks * BLOCK
    out = {"n_blocks": n_blocks, "bytes_per_launch": moved, "rows": []}
    for rnd in range(2):
        for name, v, grid, waves, inplace in (CONFIGS if rnd == 0 else CONFIGS[::-1]):
            cp = b if inplace else c

            def go():
                rc = lib.stream_probe_launch(v, grid, waves, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                             ctypes.c_void_p(cp.data_ptr()), n_blocks, st)
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
