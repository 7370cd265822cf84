"""Static checks of the built gfx950 code object (libden.so, no GPU needed).

r05: the streamed weight-gradient kernel faulted on the GPU ("illegal memory access") when the
compiler outlined its block-fetch lambda into a real function call (s_swappc) -- the callee reads the
sampler's arguments through the kernarg-segment pointer, which the persistent kernels use to keep
argument words out of scalar registers.  The fetch is force-inlined now; this test keeps every
kernel of the BF16 training path call-free and scratch-free, so a change that makes the compiler
outline or spill to memory fails here, on the CPU, instead of on the GPU."""
import os

import pytest

from conftest import ROOT
import _codeobj

LIB = os.path.join(ROOT, "deblur-e-nerf_amd", "libden.so")
# the BF16 training step's kernels (den_api.hip render_fwd_impl / render_bwd_impl, hidden path)
HOT = ("render_fwd_kernelILi1ELb1E", "render_head_bwd_kernel", "hidden_bwd_kernelILb0E", "hidden_bwd_kernelILb1E",
       "dwstream_kernel", "dw_reduce_kernel", "lr_reduce1_kernel", "lr_reduce2_kernel")
# kernels allowed to contain calls (the F32 parity forward: its compositing helpers are outlined)
CALLS_ALLOWED = ("render_fwd_kernelILi0E",)


@pytest.fixture(scope="module")
def code():
    if not os.path.exists(LIB):
        pytest.skip("libden.so not built")
    return _codeobj.disassemble(LIB), _codeobj.kernel_descriptors(LIB)


def _calls(lines):
    return [ln for ln in lines if "s_swappc" in ln or "s_setpc" in ln]


def test_hot_kernels_are_call_free_and_scratch_free(code):
    funcs, scratch = code
    for pat in HOT:
        names = [k for k in funcs if pat in k]
        assert names, f"no kernel matching {pat} in libden.so"
        for k in names:
            assert not _calls(funcs[k]), f"{k} makes function calls"
            assert scratch.get(k, 0) == 0, f"{k} uses {scratch[k]} B of scratch per lane"


def test_no_unexpected_calls(code):
    funcs, _ = code
    bad = [k for k, v in funcs.items() if _calls(v) and not any(p in k for p in CALLS_ALLOWED)]
    assert not bad, f"kernels with function calls: {bad}"
