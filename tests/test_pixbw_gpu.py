"""Parity of the pixel-bandwidth kernels (den_pixbw_sample_ts / _fwd / _bwd, reached
through the PixelBandwidth module mirror) against (1) the reference's own
PixelBandwidth run in f32 and f64 (tests/golden/pixbw_*.npz, written by
tests/golden/make_golden.py from the imported reference module) and (2) the f64
CPU oracle on identical inputs.  Needs an MI355X (marked gpu).

Tolerances:
* vs the reference's f64 run (the kernels take the f32-rounded intensities):
  log-intensity |a-b| <= 2e-6 max(|b|, 1) -- the reference's own f32-vs-f64 gap is
  ~1e-6; intensity gradients 1e-4 of max|ref|; parameter
  gradients 1e-4 relative.
* vs the f64 oracle on the same f32-valued inputs, with the timestamp differences
  cast to f32 as the reference does (only the matrix-exponential algorithm, the
  summation order and the final f32 rounding differ): 2e-7 on outputs, 1e-6 (of
  max) on intensity gradients, 1e-5 on parameter gradients.
"""
import math
import os

import numpy as np
import pytest
import torch

from _util import norm_rel, rel_err
from oracle import pixbw as opb

pytestmark = pytest.mark.gpu
DEV = "cuda"
FILES = ["pixbw_S16_eds.npz", "pixbw_S30_eds.npz", "pixbw_S16_pert.npz"]
OMEGA = 2 * math.pi * 21.0


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def _module(calib, min_ts, tmp_path, originals=None):
    from deblur_e_nerf.models.pixel_bandwidth import PixelBandwidth
    np.savez(os.path.join(tmp_path, "camera_calibration.npz"), **calib)
    pb = PixelBandwidth(str(tmp_path), torch.tensor(min_ts), 21.0, _Cfg(max_sample_lifetime=0.95))
    if originals is not None:
        with torch.no_grad():
            for pn in opb.PARAM_NAMES:
                getattr(pb.parametrizations, pn).original.copy_(torch.as_tensor(originals[pn]))
    return pb.to(DEV)


def _run_sequence(pb, gen, call_ts, intensities, coef):
    """The golden's call sequence: reset at call 0 (diff start), then 3 decaying calls."""
    leaves = []

    def fn_for(c):
        def fn(ts):
            it = intensities[c].to(DEV).float().requires_grad_(True)
            leaves.append(it)
            return (it,)
        return fn

    outs = [pb(gen, call_ts[c], fn_for(c), reset_diff=(c == 0))[0] for c in range(len(intensities))]
    total = sum((outs[c] * coef[c]).sum() for c in range(len(outs)))
    pb.zero_grad()
    total.backward()
    torch.cuda.synchronize()
    return outs, leaves


@pytest.mark.parametrize("fname", FILES)
def test_sample_timestamps_match_oracle(golden_dir, fname):
    from deblur_e_nerf import _native as nat
    z = np.load(os.path.join(golden_dir, fname))
    call_ts = torch.from_numpy(z["call_ts"])
    for gname in ("gen_dirac", "gen_unif"):
        gen = torch.from_numpy(z[gname])
        for c in range(4):
            ref = opb.sample_timestamps(gen, call_ts[c], OMEGA, 0.95)
            got = nat.pixbw_sample_ts(gen.to(DEV), call_ts[c].to(DEV), OMEGA, 0.95).cpu()
            assert float((got - ref).abs().max()) <= 1e-6, (gname, c)  # ns, on timestamps ~1e8-1e9


@pytest.mark.parametrize("fname", FILES)
def test_pixel_bandwidth_matches_reference_golden(golden_dir, tmp_path, fname):
    z = np.load(os.path.join(golden_dir, fname))
    calib = {k.split(":", 1)[1]: z[k] for k in z.files if k.startswith("calib:")}
    pb = _module(calib, int(z["min_ts"]), tmp_path, {pn: z[f"orig_f32:{pn}"] for pn in opb.PARAM_NAMES})
    for pn in opb.PARAM_NAMES:  # the mirror's parametrisation gives the reference's values
        ref = float(z[f"param_f32:{pn}"])
        assert abs(float(getattr(pb, pn).detach()) - ref) <= 1e-6 * abs(ref), pn
    call_ts = torch.from_numpy(z["call_ts"]).to(DEV)
    coef = torch.from_numpy(z["coef"]).to(DEV).float()
    for gi, gname in enumerate(("gen_dirac", "gen_unif")):
        gen = torch.from_numpy(z[gname]).to(DEV)
        its = [torch.from_numpy(z[f"it_g{gi}_f32_c{c}"]) for c in range(4)]
        outs, leaves = _run_sequence(pb, gen, call_ts, its, coef)
        worst = [0.0, 0.0, 0.0]
        for c in range(4):
            e64 = rel_err(outs[c], z[f"logit_g{gi}_f64_c{c}"])
            e32 = rel_err(outs[c], z[f"logit_g{gi}_f32_c{c}"])
            # the reference's own f32 run is this far from its f64 run (up to ~3e-3 here)
            gap = rel_err(z[f"logit_g{gi}_f32_c{c}"], z[f"logit_g{gi}_f64_c{c}"])
            assert e64 <= 2e-6 and e32 <= gap + 2e-6, (gname, c, e64, e32, gap)
            ref = z[f"dit_g{gi}_f64_c{c}"]
            d = float(np.abs(leaves[c].grad.cpu().numpy() - ref).max() / np.abs(ref).max())
            assert d <= 1e-4, (gname, c, d)
            worst = [max(worst[0], e64), max(worst[1], e32), max(worst[2], d)]
        for pn in opb.PARAM_NAMES:
            ref = float(z[f"dparam_g{gi}_f64:{pn}"])
            got = float(getattr(pb.parametrizations, pn).original.grad)
            assert abs(got - ref) <= 1e-4 * max(abs(ref), 1e-30), (gname, pn, got, ref)
        print(f"[{fname} {gname}] log I err vs reference f64 {worst[0]:.1e} (vs its f32 run {worst[1]:.1e}); "
              f"dI err {worst[2]:.1e}")


def _eds_calib():
    return {k: np.array(v, dtype=np.float32) for k, v in dict(
        input_time_const_eff_it_prod=(35e-12 * 25e-3) / 2000e-12,
        miller_time_const_eff_it_prod=(0.6e-12 * 25e-3) / 2000e-12,
        amplifier_gain=140.0, closed_loop_gain=1 / 0.7, output_time_const=25e-6,
        sf_cutoff_freq=16400.0, diff_amp_cutoff_freq=82000.0).items()}


@pytest.mark.parametrize("S,N", [(3, 70), (16, 4096), (30, 300)])
def test_pixel_bandwidth_matches_oracle_f64(tmp_path, S, N):
    """Size-independent check against the f64 oracle on identical (f32-valued) inputs,
    including the smallest sample size the reference accepts (S = 3: with S = 2 its
    sample_intensity indexes an empty tensor, pixel_bandwidth.py:335-337) and N not a
    multiple of the 64-event block."""
    g = torch.Generator().manual_seed(100 + S)
    calib = _eds_calib()
    min_ts = 100_000_000
    pb = _module(calib, min_ts, tmp_path)
    gen = torch.rand(S - 1, N, generator=g, dtype=torch.float64)
    t_end = (torch.rand(N, generator=g, dtype=torch.float64) * 0.8e9 + 0.15e9).floor()
    call_ts = [t_end - 3e5, t_end, t_end - 1e5]
    its = [torch.exp(torch.rand(S, N, generator=g) * 6.9 - 4.6) for _ in call_ts]  # 0.01 .. 10
    coef = torch.randn(len(call_ts), N, generator=g)

    outs, leaves = _run_sequence(pb, gen.to(DEV), [t.to(DEV) for t in call_ts], its, coef.to(DEV))

    # oracle: f64 arithmetic on the same f32 values, dt cast to f32 like the reference
    # the post-softplus f32 values the kernels see, as f64 leaves
    prm = {"tau_in_it_eff_prod": torch.tensor(float(pb.tau_in_it_eff_prod), dtype=torch.float64)}
    for pn in opb.PARAM_NAMES:
        prm[pn] = torch.tensor(float(getattr(pb, pn).detach()), dtype=torch.float64, requires_grad=True)
    orc = opb.PixelBandwidthOracle(prm, min_ts, dt_dtype=torch.float32)
    leaves_o = []

    def fn_for(c):
        def fn(ts):
            it = its[c].double().requires_grad_(True)
            leaves_o.append(it)
            return it
        return fn

    outs_o = [orc(gen, call_ts[c], fn_for(c), reset_diff=(c == 0)) for c in range(len(call_ts))]
    total = sum((outs_o[c] * coef[c].double()).sum() for c in range(len(outs_o)))
    # gradients w.r.t. the post-softplus values (the oracle's leaves), chained below
    pvals = [prm[pn] for pn in opb.PARAM_NAMES]
    grads = torch.autograd.grad(total, leaves_o + pvals)
    for c in range(len(call_ts)):
        assert rel_err(outs[c], outs_o[c].detach()) <= 2e-7, c  # f32 outputs of an f64 computation
        ref = grads[c].numpy()
        d = float(np.abs(leaves[c].grad.cpu().double().numpy() - ref).max() / np.abs(ref).max())
        assert d <= 1e-6, (c, d)
    for k, pn in enumerate(opb.PARAM_NAMES):
        orig = getattr(pb.parametrizations, pn).original
        ref = float(grads[len(call_ts) + k]) * float(torch.sigmoid(orig.detach().double()))
        got = float(orig.grad)
        assert abs(got - ref) <= 1e-5 * max(abs(ref), 1e-30), (pn, got, ref)
