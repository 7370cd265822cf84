"""The evaluation loop through the module's own hooks -- DeblurENeRF.validation_step /
validation_epoch_end (deblur_e_nerf.py:588-1053) driven by run_evaluation (what Lightning's
Trainer.validate runs, scripts/run.py:114-118) on a DataModule built from a views directory --
against the reference's loop run on the same views and the same field (tests/golden/eval_epoch_*.npz,
make_golden.gen_eval_epoch): the per-view renders, the corrected predictions' metrics (l1, psnr,
ssim), the correction's warm start carried into a second evaluation, the correction-error log, the
logged images and the saved 8-bit predictions.

Fixtures: a monochrome sensor with the Levenberg-Marquardt refinement (the shipped configs'
``correction``), a Bayer sensor with Gauss-Newton and RGBA views alpha-composited over white, and the
affine correction alone (``black_level_offset`` false).  The reference's refinement ran on
oracle/pypose.py and its Metric on oracle/metrics.py (pypose / torchmetrics are not installed:
their arithmetic is parity unpinned; everything around it is the reference's code).

Tolerances: renders at the north star's 1e-4 (F32); with the reference's own renders fed in
(``test_epoch_end_on_reference_renders``) the CPU f64 correction agrees to 1e-7 and the metrics to
1e-6; end to end, the renders' f32 noise (~1e-6) passes through the correction: parameters 1e-4,
metrics 1e-4 relative, saved 8-bit predictions within one level."""
import os
import tempfile

import numpy as np
import pytest
import torch

from test_deblur_gpu import build_model
from test_nerfacc_gpu import _Draws

pytestmark = pytest.mark.gpu
DEV = "cuda"
FIXTURES = ["eval_epoch_rd1", "eval_epoch_rd3_gn", "eval_epoch_rd1_affine"]


class _ImgLogger:
    def __init__(self):
        self.images = {}
        self.experiment = self

    def add_image(self, tag, img, global_step=None):
        self.images[tag] = img.detach().cpu().numpy()


def _correction(z):
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    return ED(per_channel_log_it_scale=False, black_level_offset=bool(z["black_level_offset"]),
              optimizer=ED(algo=str(z["algo"]), max_steps=10, lm=ED(radius=1.0e6)))


def _model(z, monkeypatch):
    from deblur_e_nerf.external import marching
    m, d = build_model(z, correction=_correction(z), eval_save=True, return_dir=True)
    monkeypatch.setattr(marching, "_uniform", _Draws([z["occ_u"]]))
    m.nerf.update_occ_grid(step=0, T_wc_position=m.trajectory.T_wc_position)
    m._logger = _ImgLogger()
    m.trainer.log_dir = tempfile.mkdtemp(prefix="den_evallog_")
    return m, d


def _datamodule(z, d):
    from deblur_e_nerf.data.datamodule import DataModule
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    return DataModule(0, ["novel_view"], 1, [0], ED(enable=False), d, 1.0, 1.0, 1.0, None, int(z["eval_perm_seed"]),
                      bool(z["alpha_over_white_bg"]), 1, 131072, 1, 1, 0)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("name", FIXTURES)
def test_validation_loop_matches_reference(golden_dir, name, monkeypatch):
    from deblur_e_nerf.utils import image_io
    z = np.load(os.path.join(golden_dir, f"{name}.npz"))
    m, d = _model(z, monkeypatch)
    dm = _datamodule(z, d)
    # the renders of validation_step, view by view in the DataModule's (permuted) order
    dm.setup("validate")
    loader = dm.val_dataloader()
    m.eval()
    with torch.no_grad():
        preds = [m.validation_step({k: v.to(DEV) for k, v in b.items()}, i)["pred_intensity_img"]
                 for i, b in enumerate(loader)]
    got = torch.stack(preds).cpu().double()
    ref = torch.from_numpy(z["ev0:pred"]).double()
    e = float((got - ref).norm() / ref.norm())
    print(f"[{name}] renders {tuple(got.shape)} rel err {e:.2e}")
    assert got.shape == ref.shape and e <= 1e-4
    for ev in range(2):
        p = f"ev{ev}:"
        m._current_epoch = ev
        m._logger.images.clear()
        res = m.run_evaluation("val", dm)[0]
        want = {k[len(p + "log:val/"):]: float(z[k]) for k in z.files
                if k.startswith(p + "log:val/") and not k.endswith("/epoch") and not k.endswith("/lpips")}
        print(f"[{name}] eval {ev}: {res} vs reference {want}")
        assert set(res) >= {f"val/{k}" for k in want}
        for k, v in want.items():
            tol = 1e-4 * abs(v) if k != "ssim" else 1e-4
            assert abs(res[f"val/{k}"] - v) <= tol, (k, res[f"val/{k}"], v)
        if bool(z["black_level_offset"]):
            for nm, mine in (("scale", m.init_correction_scale), ("gamma", m.init_correction_gamma),
                             ("offset", m.init_correction_offset)):
                r = _rel(mine.numpy(), z[p + "init_" + nm])
                assert mine.shape == z[p + "init_" + nm].shape and r <= 1e-4, (ev, nm, r)
            log = np.loadtxt(os.path.join(m.trainer.log_dir, "correction-errors", f"{ev}.csv"), ndmin=1)
            ref_err = z[p + "errors"]
            print(f"[{name}] eval {ev} correction errors {log} vs {ref_err}")
            assert abs(len(log) - len(ref_err)) <= 1
            assert _rel(log[0], ref_err[0]) <= 1e-4 and _rel(log[-1], ref_err[-1]) <= 1e-4
        for k in z.files:
            if k.startswith(p + "image:"):
                tag = k[len(p + "image:"):]
                assert tag in m._logger.images, tag
                assert np.abs(m._logger.images[tag] - z[k]).max() <= 1e-4 * max(1.0, np.abs(z[k]).max()), tag
        saved = [k for k in z.files if k.startswith(p + "saved:")]
        assert saved
        for k in saved:
            fn = k[len(p + "saved:"):]
            img = image_io.imread_unchanged(os.path.join(m.trainer.log_dir, "predictions", fn))
            refimg = z[k][..., 0] if z[k].ndim == 3 and z[k].shape[2] == 1 else z[k]
            diff = np.abs(img.astype(np.int32) - refimg.astype(np.int32))
            assert img.shape == refimg.shape and diff.max() <= 1 and (diff == 0).mean() >= 0.99, (fn, diff.max())


@pytest.mark.parametrize("name", FIXTURES)
def test_epoch_end_on_reference_renders(golden_dir, name, monkeypatch):
    """validation_epoch_end fed the reference's own renders (the fixture's per-view predictions) with
    the loader's targets: the glue after the render in isolation."""
    z = np.load(os.path.join(golden_dir, f"{name}.npz"))
    m, d = _model(z, monkeypatch)
    dm = _datamodule(z, d)
    dm.setup("validate")
    for ev in range(2):
        p = f"ev{ev}:"
        m._current_epoch = ev
        m.logged.clear()
        outputs = []
        for i, b in enumerate(dm.val_dataloader()):
            b = {k: v.squeeze(0).to(DEV) for k, v in b.items()}
            outputs.append({"sample_id": b["sample_id"], "pred_intensity_img": torch.from_numpy(z[p + "pred"][i]).to(DEV),
                            "target_intensity_img": b["img"], "exposure_time": torch.tensor(1, device=DEV),
                            "gain": torch.tensor(1.0, device=DEV)})
        m.validation_epoch_end(outputs)
        for k in z.files:
            if k.startswith(p + "log:val/") and not k.endswith(("/epoch", "/lpips")):
                mine, ref = float(m.logged["val/" + k[len(p + "log:val/"):]]), float(z[k])
                assert abs(mine - ref) <= 1e-6 * max(1.0, abs(ref)), (ev, k, mine, ref)
        if bool(z["black_level_offset"]):
            assert np.array_equal(np.loadtxt(os.path.join(m.trainer.log_dir, "correction-errors", f"{ev}.csv"),
                                             ndmin=1).shape, z[p + "errors"].shape)
            for nm in ("scale", "gamma", "offset"):
                assert _rel(getattr(m, "init_correction_" + nm).numpy(), z[p + "init_" + nm]) <= 1e-7


def test_ssim_matches_torchmetrics_restatement():
    """den_ssim against oracle/metrics.py (torchmetrics 0.6.2's ssim restated) on random image pairs,
    grey and colour, several sizes (11 x 11 is the smallest that keeps a window)."""
    from oracle import metrics as om
    from deblur_e_nerf import _native
    g = torch.Generator().manual_seed(5)
    for shape in [(1, 1, 11, 11), (2, 1, 40, 56), (3, 3, 33, 17), (1, 3, 128, 96)]:
        t = torch.rand(*shape, generator=g) * 0.8 + 0.1
        p = (t + torch.randn(*shape, generator=g) * 0.05).clamp(0, 1)
        for rng in (1.0, 0.9):
            got = _native.ssim(p.to(DEV), t.to(DEV), rng).cpu()
            ref = torch.stack([om.ssim(p[i:i + 1], t[i:i + 1], data_range=rng) for i in range(shape[0])]).double()
            print(f"[ssim {shape} range {rng}] {got.tolist()} vs {ref.tolist()}")
            assert float((got - ref).abs().max()) <= 2e-6
    with pytest.raises(Exception):
        _native.ssim(torch.rand(1, 1, 10, 12, device=DEV), torch.rand(1, 1, 10, 12, device=DEV), 1.0)


def test_metric_compute_reports_reference_metrics():
    from deblur_e_nerf.loss_metric.metric import Metric
    from oracle import metrics as om
    g = torch.Generator().manual_seed(8)
    t = torch.rand(3, 24, 30, generator=g) * 0.8 + 0.1
    p = (t + torch.randn(3, 24, 30, generator=g) * 0.03).clamp(0.05, 0.95)
    got = Metric("alex").compute(p.to(DEV), t.to(DEV), 0.05, 0.95)
    assert abs(float(got.ssim) - float(om.ssim(p[None], t[None], data_range=0.95))) <= 2e-6
    assert abs(float(got.psnr) - float(om.psnr(p[None], t[None], data_range=0.9, dim=(1, 2, 3)))) <= 1e-4
    with pytest.raises(AssertionError):  # targets outside [min, max] (metric.py:41-42)
        Metric().compute(p.to(DEV), t.to(DEV), 0.2, 0.95)
