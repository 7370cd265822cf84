"""Parity of the `ngp` radiance field on the GPU (den_ngp_fwd / den_ngp_bwd / den_hashgrid_*,
external/ngp.py NGPradianceField) against fixtures the REFERENCE's own NGPradianceField
produced (tests/golden/make_golden.py gen_ngp: external/ngp.py with oracle/tcnn.py standing in
for tcnn.Encoding -- the grid encoding is parity unpinned, tiny-cuda-nn being absent) and against
the oracle.  Needs an MI355X (marked gpu).

Tolerances: outputs 1e-5 relative (f32 MLP sums in a different order than torch's GEMMs),
MLP-weight gradients 1e-4 tensor-wise, hash-table gradients 1e-4 tensor-wise (f32 atomics in
any order, as tcnn's kernel_grid_backward), the standalone encoding 1e-6 / 1e-5.
"""
import numpy as np
import pytest
import torch

from _util import ngp_fixture, ngp_table_grad, rel_err
from oracle import ngp as ongp
from oracle import tcnn as otcnn

pytestmark = pytest.mark.gpu
DEV = "cuda"
FIXTURES = ["ngp_rd1_small", "ngp_rd3_small_sphere_relu_sigmoid", "ngp_rd3_small_tanh", "ngp_rd3_default",
            "ngp_rd1_small_shifted_softplus", "ngp_rd3_small_sphere_softplus"]
CT_NAMES = {0: "AABB", 1: "UN_BOUNDED_TANH", 2: "UN_BOUNDED_SPHERE"}


def _field(p, pos, base, head, rd, ctype, aabb):
    from deblur_e_nerf.external import marching, ngp
    act = {"softplus": torch.nn.Softplus(beta=100), "relu": torch.nn.ReLU()}
    ract = {"softplus": torch.nn.Softplus(beta=1), "sigmoid": torch.nn.Sigmoid()}
    from deblur_e_nerf.models import nerf
    dens = {"shifted_trunc_exp": ngp.shifted_trunc_exp, "softplus": torch.nn.Softplus(beta=1),
            "shifted_softplus": nerf.shifted_softplus}
    bcfg = dict(base, hidden_activation=act[base["hidden_activation"]],
                density_activation=dens[base.get("density_activation", "shifted_trunc_exp")])
    hcfg = dict(head, hidden_activation=act[head["hidden_activation"]],
                radiance_activation=ract[head["radiance_activation"]], output_dim=rd)
    f = ngp.NGPradianceField(aabb=[float(v) for v in aabb], num_dim=3, use_viewdirs=True,
                             contraction_type=getattr(marching.ContractionType, CT_NAMES[ctype]),
                             pos_encoding_config=pos, dir_encoding_config={"degree": 4}, mlp_base_config=bcfg,
                             mlp_head_config=hcfg)
    sd = f.state_dict()
    for k in p:
        assert sd[k].shape == p[k].shape, k
    f.load_state_dict(dict(p, aabb=f.aabb), strict=True)
    return f.to(DEV)


def _tensor_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("fixture", FIXTURES)
def test_ngp_field_matches_reference(golden_dir, fixture):
    z = np.load(f"{golden_dir}/{fixture}.npz")
    p, pos, base, head, rd, ctype = ngp_fixture(z)
    f = _field(p, pos, base, head, rd, ctype, z["aabb"])
    x = torch.from_numpy(z["x"]).to(DEV)
    d = torch.from_numpy(z["d"]).to(DEV)
    rgb, sig = f(x, d)
    assert rgb.shape == (x.shape[0], rd) and sig.shape == (x.shape[0], 1)
    assert rel_err(rgb.detach().cpu(), z["rgb"]) < 1e-5
    assert rel_err(sig.detach().cpu(), z["sigma"]) < 1e-5
    ((rgb * torch.from_numpy(z["g_rgb"]).to(DEV)).sum() + (sig * torch.from_numpy(z["g_sigma"]).to(DEV)).sum()).backward()
    torch.cuda.synchronize()
    grads = dict(f.named_parameters())
    errs = {}
    for k in p:
        ref = ngp_table_grad(z, p[k].numel()) if k == "mlp_base.0.params" else torch.from_numpy(z[f"grad:{k}"])
        errs[k] = (_tensor_rel(grads[k].grad, ref), float(grads[k].grad.abs().max()), float(ref.abs().max()))
    assert all(e < 1e-4 for e, _, _ in errs.values()), errs


@pytest.mark.parametrize("n_levels,n,rd,hidden,radiance", [
    (5, 1, 1, "softplus", "softplus"), (5, 33, 3, "relu", "sigmoid"), (13, 1000, 3, "softplus", "softplus"),
    (16, 4095, 1, "softplus", "sigmoid"), (1, 64, 3, "relu", "softplus")])
def test_ngp_field_ragged_matches_oracle(n_levels, n, rd, hidden, radiance):
    """The field kernels (32-sample tiles per wave, the two wave halves encoding levels
    [0, ceil(L/2)) and [ceil(L/2), L)) at sample counts that leave partial tiles and odd level
    counts, against oracle/ngp.field: outputs 1e-5, every gradient 1e-4 tensor-wise, and the
    density-only pass equal to the full pass's density."""
    pos = dict(ongp.POS_ENCODING, n_levels=n_levels, log2_hashmap_size=14)
    base = dict(ongp.MLP_BASE, hidden_activation=hidden)
    head = dict(ongp.MLP_HEAD, hidden_activation=hidden, radiance_activation=radiance)
    aabb = [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]
    p = ongp.build_params(rd, 11 + n_levels, pos, table_scale=0.1)
    f = _field(p, pos, base, head, rd, 0, aabb)
    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, 3, generator=g) * 3.2 - 1.6  # a few points outside the box (density 0)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=-1)
    g_rgb, g_sig = torch.randn(n, rd, generator=g), torch.randn(n, 1, generator=g)
    rgb, sig = f(x.to(DEV), d.to(DEV))
    ((rgb * g_rgb.to(DEV)).sum() + (sig * g_sig.to(DEV)).sum()).backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    rgb_r, sig_r = ongp.field(pr, x, d, rd, torch.tensor(aabb), 0, pos, base, head)
    ((rgb_r * g_rgb).sum() + (sig_r * g_sig).sum()).backward()
    assert _tensor_rel(rgb.detach(), rgb_r.detach()) < 1e-5 and _tensor_rel(sig.detach(), sig_r.detach()) < 1e-5
    grads = dict(f.named_parameters())
    errs = {k: _tensor_rel(grads[k].grad, pr[k].grad) for k in p}
    assert max(errs.values()) < 1e-4, errs
    with torch.no_grad():
        assert torch.equal(f.query_density(x.to(DEV)).reshape(-1), sig.detach().reshape(-1))


def test_ngp_field_large_batch_equals_chunks():
    """Past DEN_NGP_MF_GRID workgroups x 8 waves x 32 samples the field kernels loop over tiles: a
    140,000-sample call equals 4,096-sample chunks bit for bit in the forward (per-sample
    arithmetic does not depend on the grid) and to 1e-4 in the gradients (atomic and split order)."""
    from deblur_e_nerf.external import ngp
    torch.manual_seed(4)
    f = ngp.NGPradianceField(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], pos_encoding_config=dict(ongp.POS_ENCODING),
                             mlp_base_config=dict(ongp.MLP_BASE, hidden_activation=torch.nn.Softplus(beta=100),
                                                  density_activation=ngp.shifted_trunc_exp),
                             mlp_head_config=dict(ongp.MLP_HEAD, hidden_activation=torch.nn.Softplus(beta=100),
                                                  radiance_activation=torch.nn.Softplus(beta=1), output_dim=3)).to(DEV)
    with torch.no_grad():
        f.mlp_base[0].params.mul_(1e3)
    n = 140_000
    x = torch.rand(n, 3, device=DEV) * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(n, 3, device=DEV), dim=-1)
    g_rgb, g_sig = torch.randn(n, 3, device=DEV), torch.randn(n, 1, device=DEV)
    rgb, sig = f(x, d)
    ((rgb * g_rgb).sum() + (sig * g_sig).sum()).backward()
    full = {k: p.grad.clone() for k, p in f.named_parameters()}
    f.zero_grad()
    outs = []
    for s in range(0, n, 4096):
        r, q = f(x[s:s + 4096], d[s:s + 4096])
        ((r * g_rgb[s:s + 4096]).sum() + (q * g_sig[s:s + 4096]).sum()).backward()
        outs.append((r.detach(), q.detach()))
    assert torch.equal(rgb.detach(), torch.cat([o[0] for o in outs])) and torch.equal(sig.detach(), torch.cat([o[1] for o in outs]))
    errs = {k: _tensor_rel(full[k], p.grad) for k, p in f.named_parameters()}
    assert max(errs.values()) < 1e-4, errs


def test_ngp_query_density_under_autograd():
    """query_density with autograd on is differentiable (the reference's tcnn path is): sigma and its
    parameter and position gradients equal those of forward()'s density output; under no_grad it
    takes the density-only kernel and returns the same values."""
    from deblur_e_nerf.external import ngp
    torch.manual_seed(6)
    f = ngp.NGPradianceField(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], pos_encoding_config=dict(ongp.POS_ENCODING),
                             mlp_base_config=dict(ongp.MLP_BASE, hidden_activation=torch.nn.Softplus(beta=100),
                                                  density_activation=ngp.shifted_trunc_exp),
                             mlp_head_config=dict(ongp.MLP_HEAD, hidden_activation=torch.nn.Softplus(beta=100),
                                                  radiance_activation=torch.nn.Softplus(beta=1), output_dim=1)).to(DEV)
    with torch.no_grad():
        f.mlp_base[0].params.mul_(1e3)
    x = (torch.rand(3000, 3, device=DEV) * 3 - 1.5).requires_grad_(True)
    g = torch.randn(3000, 1, device=DEV)
    sig = f.query_density(x)
    (sig * g).sum().backward()
    gq = {k: p.grad.clone() for k, p in f.named_parameters()}
    gx = x.grad.clone()
    f.zero_grad()
    x.grad = None
    d = torch.zeros_like(x)
    d[:, 2] = 1.0
    _, sig_f = f(x, d)
    (sig_f * g).sum().backward()
    assert torch.equal(sig.detach(), sig_f.detach())
    assert all(torch.equal(gq[k], p.grad) or _tensor_rel(gq[k], p.grad) < 1e-5 for k, p in f.named_parameters())
    assert _tensor_rel(gx, x.grad) < 1e-5
    with torch.no_grad():
        assert torch.equal(f.query_density(x.detach()), sig.detach())


@pytest.mark.parametrize("otype,log2", [("HashGrid", 19), ("HashGrid", 12), ("DenseGrid", 19)])
def test_hashgrid_matches_oracle(otype, log2):
    """den_hashgrid_fwd / bwd (tcnn.Encoding) vs oracle/tcnn.py on random points, including
    points outside [0,1] (wrapping cells, as tcnn computes them)."""
    from deblur_e_nerf import _native
    n_levels = 16 if otype == "HashGrid" else 6
    pos = dict(ongp.POS_ENCODING, otype=otype, log2_hashmap_size=log2, n_levels=n_levels)
    desc = _native.ngp_desc(1, pos, "softplus", "softplus", 0, [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5])
    n_tab = _native.ngp_table_params(desc)
    assert n_tab == otcnn.n_params(pos)
    g = torch.Generator().manual_seed(7)
    table = torch.randn(n_tab, generator=g)
    x = torch.rand(4096, 3, generator=g) * 1.2 - 0.1
    dy = torch.randn(4096, 2 * n_levels, generator=g)
    tab_dev = table.to(DEV).requires_grad_(True)
    out = _native.hashgrid(tab_dev, desc, x.to(DEV))
    (out * dy.to(DEV)).sum().backward()
    tab = table.clone().requires_grad_(True)
    ref = otcnn.encode(x, tab, pos)
    (ref * dy).sum().backward()
    e_out = _tensor_rel(out.detach(), ref.detach())
    e_grad = _tensor_rel(tab_dev.grad, tab.grad)
    assert e_out < 1e-6 and e_grad < 1e-5, (e_out, e_grad, float(tab_dev.grad.abs().max()), float(tab.grad.abs().max()))


def test_ngp_packed_samples_match_points():
    """packed_samples (rays + ray_indices + t intervals) == forward at o + d (t0 + t1) / 2."""
    from deblur_e_nerf.external import ngp
    torch.manual_seed(3)
    f = ngp.NGPradianceField(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], pos_encoding_config=dict(ongp.POS_ENCODING),
                             mlp_base_config=dict(ongp.MLP_BASE, hidden_activation=torch.nn.Softplus(beta=100),
                                                  density_activation=ngp.shifted_trunc_exp),
                             mlp_head_config=dict(ongp.MLP_HEAD, hidden_activation=torch.nn.Softplus(beta=100),
                                                  radiance_activation=torch.nn.Softplus(beta=1), output_dim=3)).to(DEV)
    with torch.no_grad():
        f.mlp_base[0].params.mul_(1e3)
    R, n = 50, 3000
    o = torch.randn(R, 3, device=DEV)
    dd = torch.nn.functional.normalize(torch.randn(R, 3, device=DEV), dim=-1)
    ri = torch.randint(0, R, (n,), device=DEV).sort().values.int()
    t0 = torch.rand(n, device=DEV) * 3
    t1 = t0 + 0.01
    rgb_p, sig_p = f.packed_samples(o, dd, ri, t0[:, None], t1[:, None])
    pts = o[ri.long()] + dd[ri.long()] * (t0 + t1)[:, None] / 2.0
    rgb, sig = f(pts, dd[ri.long()])
    assert _tensor_rel(rgb_p.detach(), rgb.detach()) < 1e-6 and _tensor_rel(sig_p.detach(), sig.detach()) < 1e-6
    assert torch.equal(f.packed_samples(o, dd, ri, t0, t1, density_only=True)[:, 0], sig_p[:, 0].detach())


def test_ngp_sparse_gradient_scatter_matches_oracle():
    """The workgroup-aggregated table scatter (ngp_scatter_kernel) with ray-ordered samples whose
    upstream gradient is zero on every other sample (masked losses, dead samples): same-cell lanes
    fold before the scatter, and a zero-gradient lane must neither drop its partners' values nor
    absorb them.  Table gradient vs oracle/ngp.field at 1e-4 tensor-wise."""
    pos = dict(ongp.POS_ENCODING, n_levels=8, log2_hashmap_size=14)
    base = dict(ongp.MLP_BASE, hidden_activation="softplus")
    head = dict(ongp.MLP_HEAD, hidden_activation="softplus", radiance_activation="softplus")
    aabb = [-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]
    rd = 3
    p = ongp.build_params(rd, 77, pos, table_scale=0.1)
    f = _field(p, pos, base, head, rd, 0, aabb)
    g = torch.Generator().manual_seed(78)
    R, per = 16, 256  # ray-ordered: 256 closely spaced samples per ray share the coarse cells
    o = torch.rand(R, 3, generator=g) * 0.4 - 0.2
    dd = torch.nn.functional.normalize(torch.randn(R, 3, generator=g), dim=-1)
    t = (torch.arange(per, dtype=torch.float32) * 0.004)[None].expand(R, -1)
    x = (o[:, None, :] + dd[:, None, :] * t[..., None]).reshape(-1, 3)
    d = dd[:, None, :].expand(-1, per, -1).reshape(-1, 3).contiguous()
    n = x.shape[0]
    keep = (torch.arange(n) % 2 == 1).float()[:, None]
    g_sig = torch.randn(n, 1, generator=g) * keep
    rgb, sig = f(x.to(DEV), d.to(DEV))
    (sig * g_sig.to(DEV)).sum().backward()
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    _, sig_r = ongp.field(pr, x, d, rd, torch.tensor(aabb), 0, pos, base, head)
    (sig_r * g_sig).sum().backward()
    k = "mlp_base.0.params"
    e = _tensor_rel(dict(f.named_parameters())[k].grad, pr[k].grad)
    assert e < 1e-4, e


def test_ngp_density_only_refuses_grad():
    """The density-only kernel pass keeps no backward state: asked for a parameter gradient it raises
    instead of returning a zero one (query_density sends differentiable calls through the full field
    instead: test_ngp_query_density_under_autograd)."""
    from deblur_e_nerf import _native
    from deblur_e_nerf.external import ngp
    f = ngp.NGPradianceField(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5]).to(DEV)
    x = torch.zeros(64, 3, device=DEV)
    d = torch.zeros(64, 3, device=DEV)
    d[:, 2] = 1.0
    with pytest.raises(NotImplementedError):
        _native.ngp_field(f.flat_leaf(), f.desc, x, d, density_only=True)
    with torch.no_grad():
        assert f.query_density(x).shape[0] == 64


def test_ngp_rejects_host_tensors():
    from deblur_e_nerf import _native
    from deblur_e_nerf.external import ngp
    f = ngp.NGPradianceField(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5])
    with pytest.raises(_native.DenError):
        f(torch.zeros(4, 3), torch.zeros(4, 3))


def _ngp_nerf(z, sigma_shift=None):
    import json
    from deblur_e_nerf.external import marching
    from deblur_e_nerf.models import nerf as nerf_lib
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    rd = int(z["rd"])
    arch = ED(pos_encoding=json.loads(str(z["pos_encoding"])), dir_encoding=dict(degree=4),
              mlp_base=dict(hidden_activation="softplus", density_activation="shifted_trunc_exp", n_neurons=64,
                            n_hidden_layers=1, geo_feat_dim=15, weight_norm=False),
              mlp_head=dict(hidden_activation="softplus", radiance_activation="softplus", n_neurons=64,
                            n_hidden_layers=2, weight_norm=False))
    occ = ED(resolution=int(z["res"]), occ_thre=0.01, ema_decay=0.95, warmup_steps=256, n=16)
    ctype = {"aabb": "AABB", "sphere": "UN_BOUNDED_SPHERE", "tanh": "UN_BOUNDED_TANH"}[
        str(z["contraction"]) if "contraction" in z.files else "aabb"]
    cone = float(z["cone"]) if "cone" in z.files else 0.0
    nerf = nerf_lib.NeRF([float(v) for v in z["aabb"]], getattr(marching.ContractionType, ctype), occ, float(z["near"]),
                         float(z["far"]), float(z["step"]), "parameter", cone, 1e-4, 0.0, 16384, "ngp", arch, 3, rd)
    rf = nerf.radiance_field
    p = {k[len("param:"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param:")}
    p["mlp_base.0.params"] = torch.from_numpy(z["table"])
    rf.load_state_dict(dict(p, aabb=rf.aabb), strict=True)
    nerf = nerf.to(DEV)
    if sigma_shift is not None:
        with torch.no_grad():
            nerf.radiance_field.mlp_base[1].output_layer.bias[0] += sigma_shift
    return nerf


@pytest.mark.parametrize("rd", [1, 3])
def test_nerf_ngp_matches_reference(golden_dir, rd, monkeypatch):
    """NeRF(arch="ngp").forward through render_image (occupancy marching, early-stop pre-pass,
    packed compositing) against the reference's NeRF with the ngp field: the occupancy update at
    step 0, the training render (recorded jitter) and its gradients, the eval render.  F32;
    1e-4 on renders, 1e-3 tensor-wise on gradients (atomics + compositing order)."""
    from deblur_e_nerf.external import marching
    from test_nerfacc_gpu import _Draws
    z = np.load(f"{golden_dir}/render_ngp_rd{rd}.npz")
    nerf = _ngp_nerf(z)
    nerf.train()
    o = torch.from_numpy(z["rays_o"]).to(DEV)
    d = torch.from_numpy(z["rays_d"]).to(DEV)
    monkeypatch.setattr(marching, "_uniform", _Draws([z["occ_u"]]))
    nerf.update_occ_grid(step=0, T_wc_position=o)
    e_occ = rel_err(nerf.occupancy_grid.occs.cpu(), z["occs"])
    assert e_occ <= 1e-4, e_occ
    with torch.no_grad():
        nerf.radiance_field.mlp_base[1].output_layer.bias[0] += float(z["sigma_bias_shift"])
    nerf.occupancy_grid._binary.copy_(torch.from_numpy(z["binary_render"]).to(DEV))
    monkeypatch.setattr(marching, "_uniform", _Draws([z["train_jitter"]]))
    rad, op, dp, mspr = nerf(o, d)
    assert abs(mspr - float(z["train_mspr"])) <= 2.0 / o.shape[0], (mspr, float(z["train_mspr"]))
    errs = {k: rel_err(a, z[k]) for a, k in ((rad, "train_radiance"), (op, "train_opacity"), (dp, "train_depth"))}
    assert max(errs.values()) <= 1e-4, errs
    g = lambda k: torch.from_numpy(z[k]).to(DEV)  # noqa: E731
    ((rad * g("g_rad")).sum() + (op * g("g_op")).sum() + (dp * g("g_dp")).sum()).backward()
    gerr = {k: _tensor_rel(p.grad, torch.from_numpy(z[f"grad:{k}"])) for k, p in nerf.radiance_field.named_parameters()}
    gerr["bkgd"] = _tensor_rel(nerf.parametrizations.render_bkgd.original.grad, torch.from_numpy(z["grad_bkgd_orig"]))
    assert max(gerr.values()) <= 1e-3, gerr
    nerf.eval()
    with torch.no_grad():
        rad, op, dp, mspr = nerf(o, d)
    for a, k in ((rad, "eval_radiance"), (op, "eval_opacity"), (dp, "eval_depth")):
        assert rel_err(a, z[k]) <= 1e-4, k


def _check_grid(grid, z, occ_thre=0.01):
    """occs within 1e-4 relative of the reference's; the binary grid identical except cells whose
    reference occupancy lies within 1e-4 (relative) of the threshold (nerfacc: occs > min(mean,
    occ_thre))."""
    occs = grid.occs.detach().cpu().double()
    ref = torch.from_numpy(z["occs"]).double()
    e = float((occs - ref).norm() / ref.norm())
    thre = min(float(ref.mean()), occ_thre)
    flips = grid.binary.detach().cpu().reshape(-1) != torch.from_numpy(z["binary"]).reshape(-1)
    near = (ref - thre).abs() <= 1e-4 * thre
    print(f"  occs rel err {e:.2e} (max {float(ref.max()):.3e}), binary flips {int(flips.sum())} "
          f"({int((flips & ~near).sum())} away from the threshold)")
    assert e <= 1e-4, e
    assert not bool((flips & ~near).any())


def test_nerf_ngp_cone_update_and_render_matches_reference(golden_dir, monkeypatch):
    """configs[3]'s composition (07_ziggy_and_fuzz_hdr.yaml: unbounded-sphere contraction, near 0.01
    / far 13, cone_angle 0.004): the occupancy update's cone branch (nerf.py:176-193 -- a random
    camera per cell point, its cone step times the density) with the reference's recorded cell
    jitter and camera draws, then the eval render through cone-stepped marching.  F32."""
    from deblur_e_nerf.external import marching
    from deblur_e_nerf.models import nerf as nerf_lib
    from test_nerfacc_gpu import _Draws
    z = np.load(f"{golden_dir}/render_ngp_cone_rd1.npz")
    nerf = _ngp_nerf(z)
    nerf.train()
    cams = torch.from_numpy(z["cams"]).to(DEV)
    monkeypatch.setattr(marching, "_uniform", _Draws([z["occ_u"]]))
    ids = [torch.from_numpy(z["occ_randint_0"])]

    def replay(high, size, device=None):
        r = ids.pop(0)
        assert tuple(r.shape) == tuple(size) and int(r.max()) < high
        return r.to(device)
    monkeypatch.setattr(nerf_lib, "_randint", replay)
    nerf.update_occ_grid(step=0, T_wc_position=cams)
    assert not ids
    _check_grid(nerf.occupancy_grid, z)
    with torch.no_grad():
        nerf.radiance_field.mlp_base[1].output_layer.bias[0] += float(z["sigma_bias_shift"])
    # the render marches the reference's binary grid (cells at the threshold could flip)
    nerf.occupancy_grid._binary.copy_(torch.from_numpy(z["binary"]).to(DEV))
    nerf.eval()
    o = torch.from_numpy(z["rays_o"]).to(DEV)
    d = torch.from_numpy(z["rays_d"]).to(DEV)
    with torch.no_grad():
        rad, op, dp, mspr = nerf(o, d)
    assert abs(mspr - float(z["eval_mspr"])) <= 1e-3 * float(z["eval_mspr"]), (mspr, float(z["eval_mspr"]))
    errs = {k: rel_err(a, z[k]) for a, k in ((rad, "eval_radiance"), (op, "eval_opacity"), (dp, "eval_depth"))}
    print(f"  cone render: mean samples / ray {mspr:.2f} vs {float(z['eval_mspr']):.2f}; {errs}")
    assert max(errs.values()) <= 1e-4, errs
