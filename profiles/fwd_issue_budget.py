"""Issue budget of the BF16 training forward (render_fwd_kernel<1, true>) from its ISA.

The persistent forward's item body (all 11 layers of 256 samples) is fully unrolled, so the static
instruction counts of the kernel are, to within its prologue and compositing tail, the counts one
wave issues per item.  Each class is priced with MI355X_MICROARCH.md's measured vector-issue costs
(constants table: "vector-instruction ISSUE cost", "LDS-DMA piece issue cost", ds_read rows):

  v_mfma_f32_32x32x16_bf16     holds the SIMD's vector issue 8 of its 32 cycles
  transcendental (exp/log/...)  8 cycles       plain VALU (add/med3/fma/mov/...)  4
  v_pk_*_f32                    8 cycles       v_cvt_pk_bf16_f32                   4.5
  ds_read_b128 beside MFMAs     3 cycles       global_load_lds_dwordx4 (LDS-DMA)  60
  global_store_dwordx4          16 (store issue, T21 row)    s_nop               4

Two waves share each SIMD (8-wave workgroup, one per CU), so the SIMD issues 2x one wave's budget
while its matrix pipe needs 2 x 32 cycles per MFMA: MFMA busy <= 2*32*N_mfma / (2*issue).

    python profiles/fwd_issue_budget.py [path/to/libden.so]
"""
import collections
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_ZN3den17render_fwd_kernelILi1ELb1EEEvNS_10RenderArgsIXT_EEE"

PRICE = [  # (regex on the mnemonic, class, cycles)
    (r"^v_mfma_", "MFMA (issue hold)", 8.0),
    (r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", "transcendental", 8.0),
    (r"^v_pk_\w+_f32", "packed f32 (v_pk_*_f32)", 8.0),
    (r"^v_cvt_pk_bf16_f32", "v_cvt_pk_bf16_f32", 4.5),
    (r"^v_", "other VALU", 4.0),
    (r"^global_load_lds_dwordx4", "LDS-DMA piece", 60.0),
    (r"^ds_read", "ds_read", 3.0),
    (r"^ds_write", "ds_write", 8.0),
    (r"^global_store", "global_store", 16.0),
    (r"^global_load", "global_load", 8.0),
    (r"^s_nop", "s_nop", 4.0),
]


def isa(so):
    tmp = tempfile.mkdtemp()
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(so, lib)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], check=True, capture_output=True)
        co = [f for f in os.listdir(tmp) if "gfx950" in f]
        if not co:
            raise SystemExit("no gfx950 code object in " + so)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", os.path.join(tmp, co[0])],
                              check=True, capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(tmp)


def kernel_mnemonics(text, name):
    out, inside = [], False
    for line in text.splitlines():
        if re.match(r"^[0-9a-f]+ <.*>:$", line):
            inside = f"<{name}>:" in line
            continue
        if inside:
            m = re.match(r"^\s+([a-z_0-9]+)", line)
            if m:
                out.append(m.group(1))
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "deblur-e-nerf_amd",
                                                            "libden.so")
    mn = kernel_mnemonics(isa(so), KERNEL)
    counts, cycles = collections.Counter(), collections.Counter()
    for m in mn:
        for pat, cls, c in PRICE:
            if re.match(pat, m):
                counts[cls] += 1
                cycles[cls] += c
                break
    n_mfma = counts["MFMA (issue hold)"]
    issue = sum(cycles.values())
    print(f"render_fwd_kernel<1,true>: {len(mn)} instructions, {n_mfma} MFMAs per wave-item")
    print(f"{'class':28s} {'count':>7s} {'cycles':>9s} {'share':>6s}")
    for cls, c in sorted(cycles.items(), key=lambda kv: -kv[1]):
        print(f"{cls:28s} {counts[cls]:7d} {c:9.0f} {c / issue:6.1%}")
    valu = sum(v for k, v in counts.items() if k not in ("MFMA (issue hold)", "LDS-DMA piece", "ds_read", "ds_write",
                                                          "global_store", "global_load", "s_nop"))
    print(f"issue cycles per wave-item {issue:.0f}; matrix-pipe cycles {32 * n_mfma}")
    print(f"VALU instructions per MFMA {valu / n_mfma:.2f}")
    print(f"MFMA-busy ceiling at two waves per SIMD: {32 * n_mfma / issue:.3f}")


if __name__ == "__main__":
    main()
