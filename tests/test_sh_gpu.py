"""SHEncoder on the GPU (den_sh_encode_fwd / _bwd, den_sh.hip; external/ngp.py SHEncoder.forward)
against the reference module's outputs and autograd gradients (tests/golden/sh_encoder.npz,
make_golden.gen_sh) and the oracle (oracle/sh.py), degrees 1..8.

Tolerance: 4e-6 of the largest magnitude, outputs and coords gradients -- the kernel's recurrence
and the reference's written-out polynomials round differently in f32 (measured worst case
printed).  At 2^22 directions (beyond the oracle's reach) the addition theorem holds per band:
sum_m Y_l^m(u)^2 = (2l+1)/(4 pi) for unit u, and the gradient of sum(Y^2) over a band is then
radial (it vanishes tangentially)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 4e-6


def _enc(degree):
    from deblur_e_nerf.external import ngp
    return ngp.SHEncoder(n_input_dims=3, degree=degree)


@pytest.mark.parametrize("degree", range(1, 9))
def test_sh_encoder_matches_reference(golden_dir, degree):
    z = np.load(f"{golden_dir}/sh_encoder.npz")
    x = torch.from_numpy(z["coords"]).to(DEV).requires_grad_(True)
    out = _enc(degree)(x)
    ref = z[f"out_{degree}"]
    assert out.shape == ref.shape
    e_out = float(np.abs(out.detach().cpu().numpy() - ref).max() / np.abs(ref).max())
    (out * torch.from_numpy(z[f"g_{degree}"]).to(DEV)).sum().backward()
    gref = z[f"dcoords_{degree}"]
    e_g = float(np.abs(x.grad.cpu().numpy() - gref).max() / max(np.abs(gref).max(), 1.0))
    print(f"  degree {degree}: out {e_out:.2e}, d_coords {e_g:.2e}")
    assert e_out <= TOL and e_g <= TOL


def test_sh_encoder_matches_oracle_batched_shape():
    """(..., 3) batch dims, as the reference; random directions vs the f64 oracle."""
    from oracle import sh as osh
    g = torch.Generator().manual_seed(3)
    u = torch.randn(5, 7, 3, generator=g)
    u = u / u.norm(dim=-1, keepdim=True)
    out = _enc(6)(u.to(DEV))
    assert out.shape == (5, 7, 36)
    ref = osh.sh_encode(u.reshape(-1, 3).numpy(), 6).reshape(5, 7, 36)
    assert np.abs(out.cpu().numpy() - ref).max() <= TOL * np.abs(ref).max()


def test_sh_encoder_empty_and_degree_bounds():
    from deblur_e_nerf import _native as nat
    out = _enc(4)(torch.empty(0, 3, device=DEV))
    assert out.shape == (0, 16)
    with pytest.raises(nat.DenError):
        nat.sh_encode(torch.zeros(4, 3, device=DEV), 9)


def test_sh_encoder_addition_theorem_full_size():
    n = 1 << 22
    g = torch.Generator(device=DEV).manual_seed(5)
    u = torch.randn(n, 3, device=DEV, generator=g)
    u = (u / u.norm(dim=-1, keepdim=True)).requires_grad_(True)
    y = _enc(8)(u)
    worst = 0.0
    for l in range(8):
        band = (y[:, l * l:(l + 1) * (l + 1)].double() ** 2).sum(-1)
        worst = max(worst, float((band - (2 * l + 1) / (4 * math.pi)).abs().max()))
    (y ** 2).sum().backward()
    gr = u.grad.double()
    ud = u.detach().double()
    tangential = gr - (gr * ud).sum(-1, keepdim=True) * ud
    t_rel = float(tangential.norm(dim=-1).max() / gr.norm(dim=-1).max())
    print(f"  addition theorem worst |sum_m Y^2 - (2l+1)/4pi| {worst:.2e}, tangential gradient {t_rel:.2e}")
    assert worst < 2e-5 and t_rel < 5e-5
