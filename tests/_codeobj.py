"""The gfx950 code object inside a hipcc-built shared library (the clang offload bundle in its
.hip_fatbin section), for static checks of the built kernels (tests/test_codeobj.py)."""
import os
import struct
import subprocess
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
LLVM = "/opt/rocm/lib/llvm/bin"


def gfx950_code_object(so_path):
    """-> bytes of the amdgcn-amd-amdhsa--gfx950 ELF bundled in `so_path`."""
    data = open(so_path, "rb").read()
    start = data.find(MAGIC)
    if start < 0:
        raise ValueError(f"{so_path}: no offload bundle")
    pos = start + len(MAGIC)
    (n,) = struct.unpack_from("<Q", data, pos)
    pos += 8
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", data, pos)
        pos += 24
        triple = data[pos:pos + tlen].decode()
        pos += tlen
        if "gfx950" in triple:
            return data[start + off:start + off + size]
    raise ValueError(f"{so_path}: no gfx950 code object in the bundle")


def disassemble(so_path):
    """-> {kernel symbol: [instruction lines]} of the gfx950 code object (llvm-objdump -d)."""
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "co.elf")
        with open(co, "wb") as f:
            f.write(gfx950_code_object(so_path))
        out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                             capture_output=True, text=True, check=True).stdout
    funcs, cur = {}, None
    for ln in out.splitlines():
        if ln.endswith(">:") and "<" in ln:
            cur = ln[ln.index("<") + 1:-2]
            funcs[cur] = []
        elif cur and ln.strip():
            funcs[cur].append(ln.strip())
    return funcs


def kernel_descriptors(so_path):
    """-> {kernel name: private segment (scratch) bytes per work-item} from the code object's
    AMDGPU metadata note (llvm-readelf --notes)."""
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "co.elf")
        with open(co, "wb") as f:
            f.write(gfx950_code_object(so_path))
        out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True, text=True,
                             check=True).stdout
    res, name = {}, None
    for ln in out.splitlines():
        t = ln.strip()
        if t.startswith(".name:"):
            name = t.split(":", 1)[1].strip()
        elif t.startswith(".private_segment_fixed_size:") and name:
            res[name] = int(t.split(":", 1)[1])
            name = None
    return res
