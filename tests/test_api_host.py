"""Host-side logic of the reference-API mirror (no GPU): the module tree, constructors,
parameter names, EasyDict semantics, the optimizer's parameter grouping, and the oracle's
nerfacc / RoMa restatements against the reference-run fixtures."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import nerf as onerf
from oracle import nerfacc as onerfacc
from oracle import roma as oroma


def test_easydict_semantics():
    from deblur_e_nerf.utils.easydict import EasyDict
    b = EasyDict({"event": {"start_ts": 1}})
    b.diff = {}
    b.diff.ts_diff = 3
    assert b.event.start_ts == 1 and b["diff"]["ts_diff"] == 3
    assert isinstance(b.diff, EasyDict)
    b.pop("diff")
    assert "diff" not in b
    with pytest.raises(AttributeError):
        b.nothing


def test_loss_constructor_mirrors_reference():
    from deblur_e_nerf.loss_metric.loss import Loss
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    L = Loss(ED(log_intensity_diff=1.0, log_intensity_tv=1e-3), ED(log_intensity_diff="huber", log_intensity_tv="l1"),
             ED(log_intensity_diff=True, log_intensity_tv=True))
    assert L.error_fn.log_intensity_diff == "huber"
    # every error function of the reference (loss.py:25-30), mape included
    for fn in ("l1", "mse", "huber", "mape"):
        assert Loss(ED(log_intensity_diff=1.0, log_intensity_tv=1e-3), ED(log_intensity_diff=fn, log_intensity_tv="l1"),
                    ED(log_intensity_diff=True, log_intensity_tv=True)).error_fn.log_intensity_diff == fn
    with pytest.raises((NotImplementedError, KeyError, ValueError)):
        Loss(ED(log_intensity_diff=1.0, log_intensity_tv=1e-3), ED(log_intensity_diff="smape", log_intensity_tv="l1"),
             ED(log_intensity_diff=True, log_intensity_tv=True))


def test_deblur_e_nerf_constructs_with_reference_parameter_names(golden_dir):
    sys.path.insert(0, os.path.dirname(__file__))
    import test_deblur_gpu as t
    z = np.load(os.path.join(golden_dir, "step_pixbw_rd1.npz"))
    old = t.DEV
    t.DEV = "cpu"
    try:
        m = t.build_model(z)
    finally:
        t.DEV = old
    names = [n for n, _ in m.named_parameters()]
    assert "nerf.radiance_field.mlp.base.hidden_layers.5.weight" in names
    assert "nerf.parametrizations.render_bkgd.original" in names
    assert "pixel_bandwidth.parametrizations.tau_diff.original" in names
    assert "refractory_period.parametrizations._refractory_period.original" in names
    assert dict(m.named_parameters())["nerf.radiance_field.mlp.base.hidden_layers.5.weight"].shape == (256, 319)
    assert sum(p.numel() for p in m.parameters()) == 595586 + 2 + 1 + 1 + 6
    buffers = dict(m.named_buffers())
    assert buffers["nerf.occupancy_grid.occs"].numel() == 24 ** 3
    assert "trajectory.T_wc_timestamp" not in m.state_dict()  # non-persistent, as the reference's
    opt = m.configure_optimizers()["optimizer"]
    assert len(opt.param_groups) == 5
    # the refractory group's lr = max_refractory_period * relative lr (deblur_e_nerf.py:1063-1065)
    assert opt.param_groups[0]["lr"] == pytest.approx(1e6 * 1e-3)
    assert not m.pixel_bandwidth.parametrizations.tau_diff.original.requires_grad   # frozen (default: true)
    assert m.contrast_threshold.parametrizations.mean_contrast_threshold.original.requires_grad


def test_adam_flat_span_detection():
    from deblur_e_nerf.external import mlp
    from deblur_e_nerf.optim import _flat_span
    f = mlp.VanillaNeRFRadianceField([-1.5] * 3 + [1.5] * 3, radiance_dim=1,
                                     hidden_activation=torch.nn.Softplus(beta=100),
                                     density_activation=__import__("deblur_e_nerf.external.ngp",
                                                                   fromlist=["x"]).shifted_trunc_exp,
                                     radiance_activation=torch.nn.Softplus(beta=1))
    ps = list(f.mlp.parameters())
    span = _flat_span(ps)
    assert span is not None and span.numel() == 595586 and span.data_ptr() == f.flat_params.data_ptr()
    assert _flat_span([ps[1], ps[0]]) is None


def test_oracle_packed_composite_matches_dense():
    """oracle.nerfacc (packed, per-ray segments) == oracle.nerf.composite (dense rays)."""
    g = torch.Generator().manual_seed(3)
    R, N = 5, 37
    t0 = torch.sort(torch.rand(R, N, generator=g) * 4, dim=1).values
    t1 = t0 + torch.rand(R, N, generator=g) * 0.05 + 1e-3
    sig = torch.rand(R, N, generator=g) * 20
    rgb = torch.rand(R, N, 3, generator=g)
    bk = torch.tensor([0.3, 0.6, 0.9])
    c_d, o_d, d_d, _ = onerf.composite(t0, t1, rgb, sig, bk)
    ri = torch.arange(R).repeat_interleave(N)
    c_p, o_p, d_p = onerfacc.composite_packed(t0.reshape(-1, 1), t1.reshape(-1, 1), ri, R, sig.reshape(-1, 1),
                                              rgb.reshape(-1, 3), bk)
    assert torch.allclose(c_p, c_d, atol=1e-6) and torch.allclose(o_p[:, 0], o_d, atol=1e-6)
    assert torch.allclose(d_p[:, 0], d_d, atol=1e-5)


def test_oracle_march_reproduces_fixture(golden_dir):
    z = np.load(os.path.join(golden_dir, "render_rd1.npz"))
    ri, a0, a1, _ = onerfacc.march(z["rays_o"], z["rays_d"], z["train_t_min"], z["train_t_max"], z["binary_render"],
                                   z["aabb"].astype(np.float32), [int(z["res"])] * 3, 0, np.float32(z["step"]), 0.0)
    assert np.array_equal(ri, z["train_marched_ri"]) and np.array_equal(a0, z["train_marched_t0"])
    assert np.array_equal(a1, z["train_marched_t1"])
    # every kept sample is a marched one, and the early stop removed some
    assert len(z["train_kept_ri"]) < len(ri)


def test_oracle_roma_rotations_are_proper(golden_dir):
    z = np.load(os.path.join(golden_dir, "traj.npz"))
    r = torch.from_numpy(z["rotation"]).double()
    eye = torch.eye(3, dtype=torch.float64).expand_as(r)
    assert float((r @ r.transpose(-1, -2) - eye).abs().max()) < 5e-6
    assert float((torch.linalg.det(r) - 1).abs().max()) < 5e-6
    q = torch.nn.functional.normalize(torch.randn(8, 4, dtype=torch.float64), dim=-1)
    m = oroma.unitquat_to_rotmat(oroma.quat_product(q, oroma.quat_conjugation(q)))
    assert torch.allclose(m, torch.eye(3, dtype=torch.float64).expand(8, 3, 3), atol=1e-12)


def test_ngp_field_mirrors_reference_names(golden_dir):
    """NGPradianceField (external/ngp.py mirror) has the reference's parameter names, shapes and
    order (the golden's param_names come from the reference module), one flat buffer, and the
    table size of tcnn's sizing."""
    import numpy as np
    from deblur_e_nerf.external import marching, ngp
    from oracle import ngp as ongp
    from oracle import tcnn as otcnn
    z = np.load(os.path.join(golden_dir, "ngp_rd3_default.npz"))
    f = ngp.NGPradianceField(aabb=[-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], contraction_type=marching.ContractionType.AABB,
                             pos_encoding_config=dict(ongp.POS_ENCODING),
                             mlp_base_config=dict(ongp.MLP_BASE, hidden_activation=torch.nn.Softplus(beta=100),
                                                  density_activation=ngp.shifted_trunc_exp),
                             mlp_head_config=dict(ongp.MLP_HEAD, hidden_activation=torch.nn.Softplus(beta=100),
                                                  radiance_activation=torch.nn.Softplus(beta=1), output_dim=3))
    names = [k for k, _ in f.named_parameters()]
    assert names == [str(k) for k in z["param_names"]]
    assert f.mlp_base[0].params.numel() == otcnn.n_params(ongp.POS_ENCODING)
    for k, v in f.named_parameters():
        if k != "mlp_base.0.params":
            assert tuple(v.shape) == z[f"param:{k}"].shape, k
    flat = f.flat_params
    assert all(p.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr() for p in f.parameters())
    with pytest.raises(NotImplementedError):
        ngp.NGPradianceField(aabb=[-1, -1, -1, 1, 1, 1], mlp_base_config=dict(ongp.MLP_BASE, n_neurons=32,
                             hidden_activation=torch.nn.ReLU(), density_activation=ngp.shifted_trunc_exp))
