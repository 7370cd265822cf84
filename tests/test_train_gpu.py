"""Parity of the native train step (deblur_e_nerf.train.TrainStep: event target,
render fwd, fused event loss, render bwd, Adam, repack) against the CPU oracle's
step (oracle/train.py).  Needs an MI355X (marked gpu).

Tolerances: F32 parity mode -- losses 1e-4 relative (north_star).  Gradients are
judged against the oracle run in f64: the loss is a difference of log
intensities of two nearby renders, so its gradient cancels and even the f32
oracle sits up to a few 1e-4 from the f64 one on some layers.  Per layer the HIP
gradient must be within max(1e-4, 4 x the f32 oracle's own error) of f64.
BF16 -- 2.5e-3 on losses, 3e-2 on gradients (vs f64; ~2x the measured worst case).
Adam is checked against torch.optim.Adam fed the same gradient (1e-6).
"""
import pytest
import torch

from _util import norm_rel, unflat

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(mode, rd, N=64, S=128, seed=5):
    from deblur_e_nerf.train import TrainStep, synthetic_batch
    ts = TrainStep(N, n_samples=S, radiance_dim=rd, mode=mode, device=DEV, seed=seed)
    b = synthetic_batch(N, seed=seed)
    if rd == 3:  # colour sensor: one bayer channel per event
        b["channel"] = torch.randint(0, 3, (N,), generator=torch.Generator().manual_seed(seed))
    ts.load_batch(**b)
    return ts, b


@pytest.mark.parametrize("rd", [1, 3])
# BF16 bounds ~2x the measured worst case (r03 / r04 GPU logs): losses 1.1e-3 (the TV loss on the
# 1e-3 floor), the whole gradient 1.7e-2; tensor-wise 5e-2 (worst tensors, rd = 3: the colour head's
# output weights 3.5e-2, the bottleneck bias 3.3e-2)
@pytest.mark.parametrize("mode,tol_l,tol_g,tol_t", [("f32", 1e-4, 1e-4, 1e-4), ("bf16", 2.5e-3, 3e-2, 5e-2)])
def test_train_step_matches_oracle(mode, rd, tol_l, tol_g, tol_t):
    from oracle.train import flat_grad
    ts, b = _setup(mode, rd)
    flat_cpu = ts.flat.detach().cpu()
    p32 = {k: v.clone() for k, v in unflat(flat_cpu, rd).items()}
    p64 = {k: v.double() for k, v in unflat(flat_cpu, rd).items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
    bk = ts.bkgd_orig.detach().cpu()
    g32, (Ld, Lt, tot) = flat_grad(p32, bk, b, ts.S, rd)
    g64, _ = flat_grad(p64, bk.double(), b64, ts.S, rd)
    ts.forward()
    ts.backward()
    torch.cuda.synchronize()
    loss = ts.loss[:3].cpu().tolist()
    for a, r in zip(loss, (Ld, Lt, tot)):
        assert abs(a - r) <= tol_l * max(abs(r), 1e-3), (loss, (Ld, Lt, tot))
    g = ts.gbuf.detach().cpu().double()
    ga, g6, g3 = unflat(g[:-rd], rd), unflat(g64[:-rd], rd), unflat(g32[:-rd].double(), rd)
    rows = []
    for k in ga:
        if mode == "bf16" and ga[k].numel() < 8:
            continue  # a handful of bf16-rounded scalars: covered by the tensor-wide norm below
        e, e_cpu = norm_rel(ga[k], g6[k]), norm_rel(g3[k], g6[k])
        rows.append((k, e, e_cpu))
    print(f"[{mode} rd={rd}] loss {loss} vs {(Ld, Lt, tot)}")
    for k, e, e_cpu in rows:
        print(f"   {k:28s} HIP vs f64 {e:.2e}   f32 oracle vs f64 {e_cpu:.2e}")
    e_all = norm_rel(g, g64)
    print(f"   whole gradient               HIP vs f64 {e_all:.2e}")
    for k, e, e_cpu in rows:
        assert e <= max(tol_t, 4 * e_cpu), (k, e, e_cpu)
    assert e_all <= max(tol_g, 4 * norm_rel(g32.double(), g64))
    e_bk, e_bk_cpu = norm_rel(g[-rd:], g64[-rd:]), norm_rel(g32[-rd:].double(), g64[-rd:])
    print(f"   render bkgd                  HIP vs f64 {e_bk:.2e}   f32 oracle vs f64 {e_bk_cpu:.2e}")
    assert e_bk <= max(tol_g, 4 * e_bk_cpu)


@pytest.mark.parametrize("rd", [1, 3])
def test_train_step_from_raw_events_matches_oracle(rd):
    """TrainStep fed raw events (load_events: den_event_prep + den_pixel_rays on
    the device every step) against the oracle's event preparation + rays + step,
    F32 parity mode, with non-trivial C+/C- and refractory period."""
    from deblur_e_nerf.train import TrainStep, synthetic_events
    from oracle.train import flat_grad, prepare_batch
    N, S = 64, 128
    cts, tau = (0.27, 0.22), 1500.0
    ts = TrainStep(N, n_samples=S, radiance_dim=rd, mode="f32", device=DEV, seed=7, contrast_thresholds=cts,
                   refractory_period=tau, mean_contrast_threshold=0.245)
    raw = synthetic_events(N, seed=8)
    if rd == 3:
        raw["channel"] = torch.randint(0, 3, (N,), generator=torch.Generator().manual_seed(8))
    ts.load_events(**raw)
    b = prepare_batch(raw, cts, tau)
    if rd == 3:
        b["channel"] = raw["channel"]
    p32 = unflat(ts.flat.detach().cpu(), rd)
    p64 = {k: v.double() for k, v in p32.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
    bk = ts.bkgd_orig.detach().cpu()
    g32, (Ld, Lt, tot) = flat_grad({k: v.clone() for k, v in p32.items()}, bk, b, S, rd, mean_ct=0.245)
    g64, _ = flat_grad(p64, bk.double(), b64, S, rd, mean_ct=0.245)
    ts.forward()
    ts.backward()
    torch.cuda.synchronize()
    # the device-derived inputs themselves
    assert torch.equal(ts.lid.cpu(), b["lid"])
    assert torch.equal(ts.start_ts.cpu(), b["start_ts"])
    assert torch.allclose(ts.rays_d.cpu(), b["rays_d"], rtol=0, atol=1e-6)
    loss = ts.loss[:3].cpu().tolist()
    for a, r in zip(loss, (Ld, Lt, tot)):
        assert abs(a - r) <= 1e-4 * max(abs(r), 1e-3), (loss, (Ld, Lt, tot))
    g = ts.gbuf.detach().cpu().double()
    assert norm_rel(g, g64) <= max(1e-4, 4 * norm_rel(g32.double(), g64))


def test_adam_matches_torch():
    ts, _ = _setup("f32", 1)
    ts.forward()
    ts.backward()
    flat0 = ts.flat.detach().cpu().clone()
    grad = ts.grad.detach().cpu().clone()
    ts.optimizer_step()
    ts.forward()
    ts.backward()
    grad2 = ts.grad.detach().cpu().clone()
    ts.optimizer_step()
    torch.cuda.synchronize()
    w = flat0.clone().requires_grad_(True)
    opt = torch.optim.Adam([w], lr=ts.lr, weight_decay=ts.wd)
    for gg in (grad, grad2):
        w.grad = gg.clone()
        opt.step()
    assert torch.allclose(ts.flat.cpu(), w.detach(), rtol=1e-6, atol=1e-7)


def test_step_is_deterministic():
    """Fixed-order reductions (no float atomics): two identical steps give
    bit-identical gradients."""
    out = []
    for _ in range(2):
        ts, _ = _setup("bf16", 1, N=256)
        ts.forward()
        ts.backward()
        torch.cuda.synchronize()
        out.append(ts.gbuf.detach().cpu().clone())
    assert torch.equal(out[0], out[1])


def test_missed_rays_stay_finite_over_training():
    """Rays that miss the AABB (here: near-axis directions passing beside the box)
    render the background exactly, carry no gradient, and several Adam steps
    stay finite (regression: their clipped slab points once fed unbounded
    coordinates to the encoding)."""
    from deblur_e_nerf.train import TrainStep, synthetic_events
    N = 2048
    ts = TrainStep(N, n_samples=128, radiance_dim=1, mode="bf16", device=DEV, seed=3)
    raw = synthetic_events(N, seed=11)
    # force a quarter of the events to look past the box along a near-axis direction
    k = N // 4
    raw["T_wc_position"][:, :k] = torch.tensor([-1.96, -3.49, -0.58])
    raw["T_wc_orientation"][:, :k] = torch.eye(3)[[0, 2, 1]].T.contiguous()  # z axis ~ world y
    raw["position"][:k] = torch.tensor([400.6, 400.0])
    ts.load_events(**raw)
    for _ in range(6):
        ts.step()
        assert torch.isfinite(ts.loss[:3]).all(), ts.loss
    miss = ts.opacity[:k] == 0
    assert bool(miss.all())
    bk = ts.bkgd  # the background the last forward composited over (Adam has moved bkgd_orig since)
    assert torch.equal(ts.rgb[:k][miss], bk.expand(int(miss.sum()), 1))


@pytest.mark.parametrize("rd", [1, 3])
# BF16: the TV loss measured 2.4e-2 off (a difference of pixel-bandwidth filtered log intensities
# 1e-3 apart).  The BF16 gradient error is set by the forward's BF16 noise against the intensity
# change over the events' interval: with the camera on the pose trajectory (r05) it measured 13 / 6 /
# 2.1 / 0.86 % at 5 / 20 / 50 / 200 units/s, the layer-major and sample-major backward identical
# (profiles/probe_pixbw_bf16.py, gpurun_out r05h / r05i) -- conditioning, not the kernels; the test
# runs at 200 units/s, where the f32 oracle's own error is smallest too.
@pytest.mark.parametrize("mode,tol_l,tol_g", [("f32", 1e-4, 1e-4), ("bf16", 3e-2, 3e-2)])
def test_pixbw_train_step_matches_oracle(rd, mode, tol_l, tol_g):
    """Pixel-bandwidth-on step (BASELINE configs[2] shape, small): PixbwTrainStep
    (event prep, sample timestamps, rays, renders, pixel-bandwidth filter, losses,
    autograd backward through the HIP kernels) against the oracle's step; F32
    parity mode: losses 1e-4 relative, gradients judged against the f64 oracle
    as in test_train_step_matches_oracle; BF16 (the mode bench.py --pixbw runs):
    3e-2 on losses, 3e-2 on gradients."""
    from deblur_e_nerf.train import PixbwTrainStep, synthetic_pixbw_events
    from oracle import pixbw as opb
    from oracle.train import pixbw_flat_grad
    N, S, n_s = 4, 16, 128
    ts = PixbwTrainStep(N, it_sample_size=S, n_samples=n_s, radiance_dim=rd, mode=mode, device=DEV, seed=9)
    raw = synthetic_pixbw_events(N, it_sample_size=S, seed=13, speed=200.0)
    if rd == 3:
        raw["channel"] = torch.randint(0, 3, (N,), generator=torch.Generator().manual_seed(13))
    ts.load_events(**raw)
    prm32 = {"tau_in_it_eff_prod": float(ts.pb.tau_in_it_eff_prod)}
    for pn in opb.PARAM_NAMES:
        prm32[pn] = float(getattr(ts.pb, pn).detach())
    min_ts = float(ts.pb.min_ts)
    p32 = unflat(ts.flat.detach().cpu(), rd)
    bk = ts.bkgd_orig.detach().cpu()
    g32, (Ld, Lt, tot) = pixbw_flat_grad({k: v.clone() for k, v in p32.items()}, bk, raw, S, n_s, rd, prm32, min_ts)
    raw64 = {k: (v.double() if v.is_floating_point() and v.dtype == torch.float32 else v) for k, v in raw.items()}
    g64, l64 = pixbw_flat_grad({k: v.double() for k, v in p32.items()}, bk.double(), raw64, S, n_s, rd, prm32,
                               min_ts, dt_dtype=None)
    ts.forward()
    ts.backward()
    torch.cuda.synchronize()
    loss = ts.loss.cpu().tolist()
    # the TV term is an L1 of a log-intensity difference of two nearby renders (~1e-4): judged, like the
    # gradients, against the f64 oracle with the f32 oracle's own error as the floor
    g = ts.gbuf.detach().cpu().double()
    e, e_cpu = norm_rel(g, g64), norm_rel(g32.double(), g64)
    print(f"[pixbw {mode} rd={rd}] loss {loss} vs {(Ld, Lt, tot)}; grad HIP vs f64 {e:.2e}, "
          f"f32 oracle vs f64 {e_cpu:.2e}")
    for a, r32, r64 in zip(loss, (Ld, Lt, tot), l64):
        assert abs(a - r64) <= max(tol_l * abs(r64), 4 * abs(r32 - r64)), (loss, (Ld, Lt, tot), l64)
    assert e <= max(tol_g, 4 * e_cpu), (e, e_cpu)


def test_pixbw_slow_pose_stays_finite():
    """Regression (round-1 verdict): the pixel-bandwidth bench at a 0.5 units/s synthetic camera
    speed gave NaN losses.  Isolated on the commit that introduced PixbwTrainStep (f6c18db) by
    swapping in the compositing of its parent: NaN with the old compositing, finite with the
    overflow-robust one (exclusive optical depth as a sum, sigma selected, zero-length samples
    skipped) -- DESIGN.md section 6.  Full bench size, BF16, 6 Adam steps."""
    from deblur_e_nerf.train import PixbwTrainStep, synthetic_pixbw_events
    S = 16
    N = 131072 // (4 * S)
    ts = PixbwTrainStep(N, it_sample_size=S, n_samples=128, radiance_dim=1, mode="bf16", device=DEV, seed=0)
    ts.load_events(**synthetic_pixbw_events(N, S, speed=0.5))
    for _ in range(6):
        loss = ts.step()
        assert bool(torch.isfinite(loss).all()), loss
    assert bool(torch.isfinite(ts.flat).all())


def test_full_size_step_properties():
    """BASELINE configs[1] at full size (2^15 events = 2^17 rays x 128 samples, BF16), through
    size-independent properties: finite loss and gradients; every ray's render is bit-identical
    to the same ray rendered in a 256-event sub-batch (per-ray compute is independent of the
    batch); and the sub-batch loss matches the f64 oracle's at the BF16 bound."""
    from deblur_e_nerf.train import TrainStep, synthetic_batch
    from oracle.train import flat_grad
    N, n = 32768, 256
    full = TrainStep(N, n_samples=128, radiance_dim=1, mode="bf16", device=DEV, seed=5)
    full.load_batch(**synthetic_batch(N, seed=5))
    full.forward()
    full.backward()
    sub = TrainStep(n, n_samples=128, radiance_dim=1, mode="bf16", device=DEV, seed=5)
    b = synthetic_batch(n, seed=5, rank=0, world=N // n)
    sub.load_batch(**b)
    sub.forward()
    sub.backward()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(full.loss[:3]).all()) and bool(torch.isfinite(full.gbuf).all())
    assert float(full.gbuf.abs().max()) > 0
    for t_full, t_sub in ((full.rgb, sub.rgb), (full.opacity, sub.opacity), (full.depth, sub.depth)):
        a = t_full.reshape(4, N, -1)[:, :n].cpu()
        assert torch.equal(a, t_sub.reshape(4, n, -1).cpu())
    p64 = {k: v.double() for k, v in unflat(sub.flat.detach().cpu(), 1).items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
    g64, (Ld, Lt, tot) = flat_grad(p64, sub.bkgd_orig.detach().cpu().double(), b64, 128, 1)
    loss = sub.loss[:3].cpu().tolist()
    e_sub = norm_rel(sub.gbuf, g64)
    print(f"full-size loss {full.loss[:3].cpu().tolist()}; sub-batch {loss} vs f64 oracle {(Ld, Lt, tot)}; "
          f"sub-batch gradient vs f64 oracle {e_sub:.2e}")
    assert abs(loss[2] - tot) <= 1e-4 * abs(tot)  # measured 8e-6
    assert e_sub <= 3e-2  # the BF16 gradient bound of this file (measured 1.5e-2)
    # linearity at full size: the 2^24-sample gradient (persistent split-K over every CU, one
    # reduction) equals the event-weighted sum of the gradients of its K sub-batches computed
    # separately -- the loss is a mean over events, so g_full = sum_k (n_k / N) g_k (BF16
    # summation-order noise: measured 8.2e-5)
    K = 8
    acc = torch.zeros_like(full.gbuf, dtype=torch.float64)
    g_full = full.gbuf.detach().double().clone()
    del full
    torch.cuda.empty_cache()
    part = TrainStep(N // K, n_samples=128, radiance_dim=1, mode="bf16", device=DEV, seed=5)
    for k in range(K):
        part.load_batch(**synthetic_batch(N // K, seed=5, rank=k, world=K))
        part.forward()
        part.backward()
        acc += part.gbuf.double() / K
    e_lin = norm_rel(acc, g_full)
    print(f"full-size gradient vs the mean of {K} sub-batch gradients: {e_lin:.2e}")
    assert e_lin <= 2e-4


@pytest.mark.parametrize("cap", [1, 37])
def test_render_max_workgroups_cap(cap):
    """den_render_desc.max_workgroups (ABI 7) changes only the persistent grids: the BF16 forward's
    radiance is bit-identical and the gradient equal up to the weight gradients' f32 summation order,
    with 1 (one workgroup walks everything) and 37 (an odd split of the blocks).  Bound 1e-3: one
    workgroup sums all 8,192 blocks of a layer in one f32 accumulator chain instead of 256 partials
    (measured 9.5e-5 for cap 1, r06j), on a gradient that cancels (a difference of log intensities)."""
    ts, _ = _setup("bf16", 1, N=512)
    ts.forward()
    ts.backward()
    torch.cuda.synchronize()
    rgb0, g0 = ts.rgb.clone(), ts.grad.clone()
    ts.desc.max_workgroups = cap
    try:
        ts.forward()
        ts.backward()
    finally:
        ts.desc.max_workgroups = 0
    torch.cuda.synchronize()
    assert torch.equal(ts.rgb, rgb0)
    e = float((ts.grad - g0).norm() / g0.norm())
    print(f"[cap {cap}] gradient vs one workgroup per CU: {e:.2e}")
    assert e <= 1e-3
