"""The evaluation's intensity correction (the reference's deblur_e_nerf.py:705-935, CPU f64 as the
reference runs it): the affine log-intensity alignment (``affine_log_intensity_correction``) against
a known affine map and the closed-form regression; the black-level refinement
(``evaluation_correction``): ``OffsetGammaCorrection`` forward / jacobians against the reference
module's outputs (tests/golden/correction.npz, make_golden.gen_correction), the Levenberg-Marquardt
and Gauss-Newton refinements against scipy.optimize.least_squares (MINPACK "lm") on the same
residual -- pypose, whose optimizers the reference subclasses, is not installed: its per-step
trajectory is parity unpinned, the converged correction is pinned."""
import math

import torch

import numpy as np
import pytest

from deblur_e_nerf.models.deblur_e_nerf import affine_log_intensity_correction, evaluation_correction
from deblur_e_nerf.models.offset_gamma_correction import OffsetGammaCorrection
from deblur_e_nerf.utils.easydict import EasyDict


def test_recovers_known_affine_map_grayscale():
    g = torch.Generator().manual_seed(3)
    target = torch.rand(3, 20, 24, generator=g, dtype=torch.float64) * 0.9 + 0.05
    # pred = exp((log target - b) / a): the correction must find gamma = a, scale = e^b
    a, b = 0.7, -0.4
    pred = ((target.log() - b) / a).exp()
    corr, gamma, scale = affine_log_intensity_correction(pred, target)
    assert corr.shape == (3, 1, 20, 24)
    assert abs(float(gamma[0]) - a) < 1e-9 and abs(float(scale[0]) - math.exp(b)) < 1e-9
    assert float((corr[:, 0] - target.double()).abs().max()) < 1e-9


def test_matches_closed_form_regression_with_gain_exposure():
    g = torch.Generator().manual_seed(4)
    target = torch.rand(2, 16, 16, generator=g) * 0.8 + 0.1
    pred = (target + torch.rand(2, 16, 16, generator=g) * 0.05).clamp(0.01, 1)
    gep = torch.tensor([1.0, 2.0])
    corr, gamma, scale = affine_log_intensity_correction(pred, target, gain_exposure_prod=gep)
    lg = (gep / gep.mean()).log().view(2, 1, 1).double()
    x, y = pred.double().log().reshape(-1), (target.double().log() - lg).reshape(-1)
    xm, ym = x.mean(), y.mean()
    a = ((x - xm) * (y - ym)).sum() / ((x - xm) ** 2).sum()
    b = ym - a * xm
    assert abs(float(gamma[0] - a)) < 1e-6 and abs(float(scale[0].log() - b)) < 1e-6
    want = ((a * pred.double().log() + b) + lg).exp()
    assert float((corr[:, 0] - want).abs().max()) < 1e-6


def test_bayer_shared_scale_per_channel_offsets():
    g = torch.Generator().manual_seed(5)
    target = torch.rand(1, 3, 10, 12, generator=g, dtype=torch.float64) * 0.9 + 0.05
    offs = torch.tensor([0.1, -0.2, 0.3], dtype=torch.float64).view(1, 3, 1, 1)
    pred = ((target.log() - offs) / 1.25).exp()
    corr, gamma, scale = affine_log_intensity_correction(pred, target, has_bayer_filter=True)
    assert gamma.shape == (1,) and scale.shape == (3,)
    assert abs(float(gamma[0]) - 1.25) < 1e-9
    assert torch.allclose(scale.log(), offs.view(3).double(), atol=1e-9)
    # per-channel scale requested: one (gamma, scale) pair per channel
    _, gamma3, scale3 = affine_log_intensity_correction(pred, target, has_bayer_filter=True,
                                                        per_channel_log_it_scale=True)
    assert gamma3.shape == (3,) and scale3.shape == (3,)


@pytest.mark.parametrize("tag", ["pc", "shared_gamma", "scalar"])
def test_offset_gamma_correction_matches_reference(golden_dir, tag):
    z = np.load(f"{golden_dir}/correction.npz")
    x = torch.from_numpy(z["x"])
    m = OffsetGammaCorrection(torch.from_numpy(z["const_scale"]), torch.from_numpy(z[f"{tag}_scale"]),
                              torch.from_numpy(z[f"{tag}_gamma"]), torch.from_numpy(z[f"{tag}_offset"]))
    with torch.no_grad():
        assert np.array_equal(m(x).numpy(), z[f"{tag}_y"])
        np.testing.assert_allclose(m.jacobian(x)[0].numpy(), z[f"{tag}_jac"], rtol=1e-14, atol=0)
        for name, j in zip(("scale", "gamma", "offset"), m.param_jacobian(x)[0]):
            np.testing.assert_allclose(j.numpy(), z[f"{tag}_pjac_{name}"], rtol=1e-14, atol=0)


def _scene(seed, B=3, H=18, W=22, gep=(1.0, 2.0, 1.5), noise=0.01):
    """Targets = a known offset-gamma map of the predictions, with per-image gain-exposure and noise."""
    g = torch.Generator().manual_seed(seed)
    pred = torch.rand(B, H, W, generator=g) * 0.85 + 0.1
    nge = torch.tensor(gep, dtype=torch.float64)
    nge = (nge / nge.mean()).view(B, 1, 1)
    target = nge * (1.4 * pred.double().pow(0.8) - 0.06) + noise * torch.rand(B, H, W, generator=g, dtype=torch.float64)
    return pred, target.float().clamp_min(1e-3), torch.tensor(gep)


def _scipy_refine(res_pred, target, nge, x0):
    from scipy.optimize import least_squares
    p, t, c = res_pred.numpy().ravel(), target.double().numpy().ravel(), nge.numpy().ravel()

    def f(v):
        return c * (v[0] * p ** v[1] - v[2]) - t
    return least_squares(f, x0, method="lm", xtol=1e-15, ftol=1e-15, gtol=1e-15, max_nfev=10000).x


def test_gain_exposure_normalisation_in_its_own_dtype():
    """deblur_e_nerf.py:707-739 with an f32, non-constant gain-exposure product: normalised and its
    log taken in f32, subtracted from the f32 target logs, and only then cast to f64 for the least
    squares -- the corrected image equals that restatement to 1e-12 relative (an f64 normalisation
    differs at ~1e-7 relative; not bit for bit: the threaded LAPACK least squares is not bitwise
    reproducible from call to call, which made a torch.equal here flaky in the full suite)."""
    g = torch.Generator().manual_seed(11)
    target = torch.rand(3, 12, 14, generator=g) * 0.8 + 0.1
    pred = (target * 1.3 + torch.rand(3, 12, 14, generator=g) * 0.05).clamp(0.01, 2)
    gep = (torch.rand(3, generator=g) * 3 + 0.2).float() * torch.tensor(1 / 3.0)  # f32, not constant
    corr, gamma, scale = affine_log_intensity_correction(pred, target, gain_exposure_prod=gep)
    nge = gep.view(-1, 1, 1, 1) / gep.mean()                        # f32 (:709-711)
    lg = nge.log()                                                  # f32 (:737)
    plog = pred.unsqueeze(1).log().double()
    tlog = (target.unsqueeze(1).log() - lg).double()                # f32 subtraction, then f64 (:738-792)
    A = torch.nn.functional.pad(plog.unsqueeze(-1), (0, 1), value=1.0).transpose(0, 1).flatten(1, 3)
    sol = torch.linalg.lstsq(A, tlog.unsqueeze(-1).transpose(0, 1).flatten(1, 3)).solution
    want = ((A @ sol).view(1, 3, 12, 14).transpose(0, 1) + lg).exp()
    torch.testing.assert_close(corr, want, rtol=1e-12, atol=0.0)
    assert abs(float(gamma[0]) - float(sol[0, 0, 0])) <= 1e-12 * abs(float(sol[0, 0, 0]))
    # and the f64 normalisation is measurably different (so the test resolves the dtype)
    lg64 = (gep.double() / gep.double().mean()).log().view(-1, 1, 1, 1)
    assert not torch.equal(lg64.float(), lg) or not torch.equal((target.unsqueeze(1).log() - lg64).double(), tlog)


@pytest.mark.parametrize("algo", ["lm", "gn"])
def test_black_level_refinement_converges_to_least_squares(algo):
    pred, target, gep = _scene(7)
    cfg = EasyDict(per_channel_log_it_scale=False, black_level_offset=True,
                   optimizer=EasyDict(algo=algo, max_steps=60, lm=EasyDict(radius=1e6)))
    r = evaluation_correction(pred, target, gep, False, cfg)
    errs = r.errors.numpy()
    assert (np.diff(errs) <= 1e-15).all(), errs                 # LM and GN never raise the error here
    # the same problem for scipy: the refinement acts on the affine-corrected predictions
    base = evaluation_correction(pred, target, gep, False, EasyDict(per_channel_log_it_scale=False,
                                                                    black_level_offset=False))
    lg = (gep.double() / gep.double().mean()).log().view(-1, 1, 1, 1)
    res_pred = (base.pred.log() - lg).exp()                     # back to the normalised domain
    nge = (gep.double() / gep.double().mean()).view(-1, 1, 1, 1).expand_as(res_pred)
    x = _scipy_refine(res_pred, target.unsqueeze(1), nge, [1.0, 1.0, 0.0])
    sc, ga, of = (float(v.reshape(-1)[0]) for v in r.converged)
    print(f"  {algo}: {len(errs) - 1} steps, error {errs[0]:.3e} -> {errs[-1]:.3e}; "
          f"(scale, gamma, offset) {sc:.6f} {ga:.6f} {of:.6f} vs scipy {x[0]:.6f} {x[1]:.6f} {x[2]:.6f}")
    np.testing.assert_allclose([sc, ga, of], x, rtol=1e-6, atol=1e-9)
    # the effective correction composes the affine fit with the refinement (:920-928)
    assert torch.allclose(r.gamma, base.gamma * ga) and torch.allclose(r.offset, torch.tensor([of], dtype=torch.float64))


def test_black_level_refinement_config_steps_and_warm_start():
    """The shipped configs' refinement (lm, max_steps 10, radius 1e6): at most 10 steps, an early stop
    once error and parameters settle, and a warm start from the converged values stops at once."""
    pred, target, gep = _scene(8)
    cfg = EasyDict(per_channel_log_it_scale=False, black_level_offset=True,
                   optimizer=EasyDict(algo="lm", max_steps=10, lm=EasyDict(radius=1e6)))
    r = evaluation_correction(pred, target, gep, False, cfg)
    assert 2 <= len(r.errors) <= 11 and r.pred.shape == (3, 1, 18, 22)
    again = evaluation_correction(pred, target, gep, False, cfg, init=r.converged)
    assert len(again.errors) <= 3 and abs(float(again.errors[-1] - r.errors[-1])) <= 1e-12 * float(r.errors[-1])


def test_black_level_refinement_bayer_shapes():
    """A Bayer sensor without per-channel scale: scale / offset per channel, one gamma."""
    g = torch.Generator().manual_seed(9)
    pred = torch.rand(2, 3, 10, 12, generator=g) * 0.8 + 0.1
    target = (1.2 * pred.double().pow(0.9) - 0.02).float().clamp_min(1e-3)
    cfg = EasyDict(per_channel_log_it_scale=False, black_level_offset=True,
                   optimizer=EasyDict(algo="lm", max_steps=10, lm=EasyDict(radius=1e6)))
    r = evaluation_correction(pred, target, None, True, cfg)
    assert [tuple(v.shape) for v in r.converged] == [(3, 1, 1, 1), (1, 1, 1, 1), (3, 1, 1, 1)]
    assert r.scale.shape == (3,) and r.gamma.shape == (1,) and r.offset.shape == (3,)  # (:806-810, :924-928)
    assert float((r.pred - target.double()).abs().max()) < 1e-3


@pytest.mark.parametrize("name", ["eval_epoch_rd1", "eval_epoch_rd3_gn", "eval_epoch_rd1_affine"])
def test_correction_on_reference_eval_renders(name):
    """evaluation_correction on the renders and views of the reference's validation loop
    (tests/golden/eval_epoch_*.npz): the refinement's converged parameters -- the warm start the next
    evaluation starts from -- and its error log match the reference's evaluation_epoch_end
    (deblur_e_nerf.py:842-949, run on oracle/pypose.py) over two evaluations."""
    import os
    from test_posed_image import build_views_dir
    from deblur_e_nerf.data.datasets import PosedImage
    from deblur_e_nerf.models.deblur_e_nerf import init_correction_params
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", f"{name}.npz"))
    files = {k: z[k] for k in z.files}
    files["root"] = np.array(".")

    class _Z(dict):
        pass
    zz = _Z(files)
    zz.files = list(files)
    root = build_views_dir(zz)
    np.savez(os.path.join(root, "camera_calibration.npz"), **{k[4:]: z[k] for k in z.files if k.startswith("cal:")})
    rd = int(z["rd"])
    target = PosedImage(root, "val", int(z["eval_perm_seed"]), bool(z["alpha_over_white_bg"])).posed_imgs.img
    blo = bool(z["black_level_offset"])
    cfg = EasyDict(per_channel_log_it_scale=False, black_level_offset=blo,
                   optimizer=EasyDict(algo=str(z["algo"]), max_steps=10, lm=EasyDict(radius=1.0e6)))
    init = init_correction_params(rd == 3, False) if blo else None
    for ev in range(2):
        res = evaluation_correction(torch.from_numpy(z[f"ev{ev}:pred"]), target, None, rd == 3, cfg, init=init)
        if not blo:
            assert res.errors is None
            continue
        ref = z[f"ev{ev}:errors"]
        assert res.errors.shape == ref.shape and np.allclose(res.errors.numpy(), ref, rtol=1e-9, atol=0), \
            (res.errors.numpy(), ref)
        for got, nm in zip(res.converged, ("scale", "gamma", "offset")):
            assert got.shape == z[f"ev{ev}:init_{nm}"].shape
            assert np.allclose(got.numpy(), z[f"ev{ev}:init_{nm}"], rtol=1e-9, atol=1e-12), nm
        init = res.converged
