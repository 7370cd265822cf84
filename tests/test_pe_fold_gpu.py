"""The pe weight-gradient fold (den_hidden.hip PEM): with the rays not requiring grad, the BF16 backward
forms L0's weight / bias gradient and L5's pe-column weight gradient inside the L1 / L5 hidden launches
(dz_0 never reaches HBM); with the rays requiring grad (den_render_ray_grad reads dz_0) the same
gradients come from the streamed launch (den_dwstream.hip) over the stored dz_0 / dz_5 / pe.  Both read
the same BF16 operands and accumulate in f32 per workgroup over the same block ranges in the same
order, reduced by the same split-K kernel: the parameter gradients are bit-identical (measured r06bb;
asserted with torch.equal, and per tensor).  The den_timing launch counts show which path ran: the
streamed launch (timing class dw_gemm_kernel) once per backward without the fold, never with it.  Sizes: 1024 rays x 128 samples = 4096 wave blocks, 16 per
workgroup, so both rings (L5 two blocks ahead, L1 one) run many steps; plus a ragged 96-ray case.
Needs an MI355X (marked gpu)."""
import pytest
import torch

from _util import flat_from_params, norm_rel, synthetic_rays, unflat
from oracle import nerf as onerf

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grads(nat, rd, R, S, seed, rays_grad):
    p = onerf.build_params(rd, seed)
    flat = flat_from_params(p, rd).to(DEV).requires_grad_(True)
    packed = nat.PackedWeights("bf16", rd, DEV)
    packed.pack(flat.detach())
    o, d, u = synthetic_rays(R, seed=seed + 1)
    g = torch.Generator().manual_seed(seed + 2)
    gc, go, gd = torch.randn(R, rd, generator=g), torch.randn(R, generator=g), torch.randn(R, generator=g)
    od, dd = o.to(DEV).requires_grad_(rays_grad), d.to(DEV).requires_grad_(rays_grad)
    cfg = dict(mode=nat.mode_id("bf16"), rd=rd, aabb=list(onerf.AABB_CHAIR), near=1.43, far=6.63, contraction=0)
    c, op, dp = nat.render(od, dd, u.to(DEV), torch.full((rd,), 0.7, device=DEV), flat, cfg, packed, S)
    torch.cuda.synchronize()
    nat.timing_enable(True)
    nat.timing_collect()
    ((c * gc.to(DEV)).sum() + (op * go.to(DEV)).sum() + (dp * gd.to(DEV)).sum()).backward()
    torch.cuda.synchronize()
    kt = nat.timing_collect()
    nat.timing_enable(False)
    return flat.grad.detach().clone(), kt.get("dw_gemm_kernel", (0.0, 0))[1]


@pytest.mark.parametrize("R", [1024, 96])
@pytest.mark.parametrize("rd", [1, 3])
def test_pe_fold_matches_streamed(R, rd):
    from deblur_e_nerf import _native as nat
    S = 128
    folded, n_fold = _grads(nat, rd, R, S, 11, rays_grad=False)
    streamed, n_stream = _grads(nat, rd, R, S, 11, rays_grad=True)
    assert (n_fold, n_stream) == (0, 1), (n_fold, n_stream)
    assert torch.isfinite(folded).all()
    whole = norm_rel(folded, streamed)
    # per parameter tensor of the reference layout (the folded L0 / L5 tensors among them)
    uf, us = unflat(folded, rd), unflat(streamed, rd)
    worst = 0.0
    for name in us:
        a, b = uf[name], us[name]
        if b.abs().max() == 0:
            assert a.abs().max() == 0, name
            continue
        e = norm_rel(a, b)
        worst = max(worst, e)
        assert torch.equal(a, b), (name, e)
    print(f"[R {R} rd {rd}] folded vs streamed: whole {whole:.2e}, worst tensor {worst:.2e}")
    assert torch.equal(folded, streamed)
