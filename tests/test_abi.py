"""The C-ABI boundary (include/den_api.h <-> libden.so <-> _native.py), on CPU.

No compute call is made here (no GPU in this container): the library must
load, export every entry point the header declares, bind with the ctypes
signatures of the Python mirror, and answer the host-only queries.
"""
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "den_api.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \t\*]*?\b(den_\w+)\s*\(", src, flags=re.M)))


def _lib():
    from deblur_e_nerf import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libden.so not built (run python __graft_entry__.py)")
    return _native, _native.lib()


def test_header_declares_entry_points():
    names = _declared()
    assert "den_render_fwd" in names and "den_render_bwd" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    _, L = _lib()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    nat, _ = _lib()
    assert sorted(nat.exported_symbols()) == _declared()


def test_host_queries():
    nat, L = _lib()
    assert L.den_version() >= 1
    # 595,844 parameters for rd=3, 595,586 for rd=1
    assert nat.param_count(3) == 595844
    assert nat.param_count(1) == 595844 - 2 * 129
    assert L.den_packed_fwd_bytes(nat.MODE_BF16) > 0 and L.den_packed_fwd_bytes(nat.MODE_F32) > 0
    # render tile: the bench's 2^17 x 128 samples and its 8-way shard must tile it
    for mode in (nat.MODE_F32, nat.MODE_BF16):
        tile = L.den_render_tile_samples(mode)
        assert tile in (128, 256, 512) and (131072 * 128 // 8) % tile == 0
    assert L.den_render_tile_samples(7) == -1


def test_invalid_shapes_fail_with_error_text():
    """Argument validation happens before any HIP call: bad shapes come back as
    error codes with text, never an abort."""
    nat, L = _lib()
    cfg = dict(mode=nat.MODE_BF16, rd=1, aabb=[-1.5] * 3 + [1.5] * 3, near=1.43, far=6.63)
    desc = nat._desc(cfg, 3, 100, True, True)  # 100 samples do not tile a workgroup
    assert L.den_render_workspace_bytes(__import__("ctypes").byref(desc)) == 0
    assert len(L.den_last_error()) > 0
    # max_workgroups (ABI 7): a launch cap only -- the workspace does not depend on it; negative refused
    import ctypes
    desc = nat._desc(cfg, 4096, 128, True, True)
    ref = L.den_render_workspace_bytes(ctypes.byref(desc))
    desc.max_workgroups = 96
    assert ref > 0 and L.den_render_workspace_bytes(ctypes.byref(desc)) == ref
    desc.max_workgroups = -1
    assert L.den_render_workspace_bytes(ctypes.byref(desc)) == 0
    assert b"max_workgroups" in L.den_last_error()


def test_no_cpu_fallback():
    """Product ops refuse host tensors instead of computing on the CPU."""
    import torch
    nat, _ = _lib()
    with pytest.raises(nat.DenError):
        nat.adam_step(torch.zeros(4), torch.zeros(4), torch.zeros(4), torch.zeros(4), 1e-3, 0.9, 0.999, 1e-8, 0.0, 1)


def _param_counts():
    """{function: number of parameters} from the header's prototypes."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(den_\w+)\s*\(([^)]*)\)\s*;", src):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_ctypes_signatures_match_header_arity():
    """Every ctypes binding passes exactly as many arguments as the C prototype declares."""
    nat, _ = _lib()
    counts = _param_counts()
    bad = {n: (len(args), counts[n]) for n, (_, args) in nat._SIGS.items() if n in counts and len(args) != counts[n]}
    assert not bad, bad


def test_training_workspace_fits_the_benchmark_shard():
    """The BF16 training workspace (block-major rows of S_0..S_7 / dz_0..dz_7 / dz_b) stays
    at ~6.4 KB of activations per sample: configs[1]'s 2^17 x 128 samples and a 2^18-ray shard fit one
    288 GB MI355X (host-only query, no GPU)."""
    import ctypes
    nat, L = _lib()
    cfg = dict(mode=nat.MODE_BF16, rd=1, aabb=[-1.5] * 3 + [1.5] * 3, near=1.43, far=6.63)
    for rays in (131072, 262144):
        desc = nat._desc(cfg, rays, 128, True, True)
        b = L.den_render_workspace_bytes(ctypes.byref(desc))
        per_sample = b / (rays * 128)
        print(f"[{rays} rays] workspace {b / 1e9:.1f} GB = {per_sample:.0f} B per sample")
        assert 6000 < per_sample < 6700 and b < 250e9
    # the F32 parity layout keeps contiguous tensors (no rows): ~20 KB per sample
    desc = nat._desc(dict(cfg, mode=nat.MODE_F32), 4096, 128, True, True)
    assert L.den_render_workspace_bytes(ctypes.byref(desc)) / (4096 * 128) > 15000
