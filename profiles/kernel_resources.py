"""Per-kernel register / LDS / spill summary of the built libden.so (its gfx950 code object's
AMDGPU metadata), e.g. to confirm a kernel change kept its register budget without spills.
usage: python profiles/kernel_resources.py [libden.so] [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else \
        os.path.join(root, "deblur-e-nerf_amd", "libden.so")
    pats = [a for a in sys.argv[1:] if not a.endswith(".so")]
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.o")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", lib], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    for blk in notes.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if pats and not any(p in name for p in pats):
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]  # noqa: E731
        agpr = blk.split("\n", 1)[0].split(":")[-1].strip()
        print(f"{name[:90]:90s} vgpr {get('vgpr_count'):>3} agpr {agpr:>3} vspill {get('vgpr_spill_count'):>3} "
              f"sspill {get('sgpr_spill_count'):>3} lds {get('group_segment_fixed_size'):>6} "
              f"scratch {get('private_segment_fixed_size'):>5}")


if __name__ == "__main__":
    main()
