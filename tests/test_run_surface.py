"""scripts/run.py's import surface, on CPU: the package exposes ``den.data.datamodule.DataModule``
and ``den.models.deblur_e_nerf.DeblurENeRF`` through attribute access (deblur_e_nerf/__init__.py:1,
data/__init__.py, models/__init__.py of the reference), and both construct from the reference's
own YAML configs with run.py:38-66's exact argument mapping.  The configs are read from the
reference tree when it is present (this container), the dataset directory is replaced by a
synthetic one (the configs point to /data/wflow/...)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import yaml

REF_CONFIGS = "/root/reference/configs/train"
CONFIGS = ["synthetic.yaml", "07_ziggy_and_fuzz_hdr.yaml", "11_all_characters.yaml"]


def _dataset_dir(rd=1, n_events=5000):
    from _util import synthetic_dataset_arrays
    d = tempfile.mkdtemp(prefix="den_run_")
    cal, poses = synthetic_dataset_arrays(rd)
    np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
    np.savez(os.path.join(d, "camera_poses.npz"), **poses)
    torch.save(torch.tensor(1_000_000), os.path.join(d, "max_refractory_period.pt"))
    g = torch.Generator().manual_seed(3)
    end = (torch.rand(n_events, generator=g, dtype=torch.float64) * 8e8 + 1.5e8).long()
    pos = (torch.rand(n_events, generator=g) < 0.5).long()
    ev = dict(position=torch.rand(n_events, 2, generator=g) * 799, start_ts=end - 200_000, end_ts=end,
              num_pos=pos, num_neg=1 - pos)
    if rd == 3:
        ev["channel_idx"] = torch.randint(0, 3, (n_events,), generator=g, dtype=torch.int8)
    torch.save(ev, os.path.join(d, "events.pt"))
    return d


def _load(name):
    from deblur_e_nerf.utils.easydict import EasyDict
    path = os.path.join(REF_CONFIGS, name)
    if not os.path.isfile(path):
        pytest.skip("the reference configs are not in this environment")
    with open(path) as f:
        return EasyDict(yaml.safe_load(f))


@pytest.mark.parametrize("name", CONFIGS)
def test_run_py_constructs_datamodule_and_model(name):
    import deblur_e_nerf as den
    config = _load(name)
    config.data.dataset_directory = _dataset_dir(rd=1)
    config.git_head_hash = "test"
    config.seed = 0
    # scripts/run.py:38-66, verbatim argument mapping
    datamodule = den.data.datamodule.DataModule(
        config.seed, config.eval_target, config.trainer.num_nodes, config.trainer.gpus, config.model.pixel_bandwidth,
        **config.data)
    model = den.models.deblur_e_nerf.DeblurENeRF(
        config.git_head_hash, config.eval_target, config.trainer.num_nodes, config.trainer.gpus,
        config.model.min_modeled_intensity, config.model.eval_save_pred_intensity_img,
        config.model.checkpoint_filepath, config.model.contrast_threshold, config.model.refractory_period,
        config.model.pixel_bandwidth, config.model.nerf, config.model.correction, config.loss, config.metric,
        config.optimizer, config.lr_scheduler, config.data.dataset_directory, config.data.alpha_over_white_bg,
        config.data.train_eff_ray_sample_batch_size)
    assert model.nerf.radiance_field is not None
    assert model.train_ray_sample_batch_size == config.data.train_eff_ray_sample_batch_size // len(config.trainer.gpus)
    assert hasattr(model, "pixel_bandwidth") == bool(config.model.pixel_bandwidth.enable)
    names = [n for n, _ in model.named_parameters()]
    assert any(n.startswith("nerf.radiance_field.mlp") for n in names)
    # the training loaders: one event batch + the matching normalized samples
    datamodule.setup("fit")
    loaders = datamodule.train_dataloader()
    ev = next(iter(loaders["event"]))
    nz = next(iter(loaders["normalized"]))
    B = datamodule.train_batch_size
    assert ev["end_ts"].shape == (1, B) and ev["position"].shape == (1, B, 2)
    assert set(nz) >= {"ts_diff", "diff_start_ts", "ts_subdiff", "subdiff_start_ts"}
    assert nz["ts_diff"].dtype == torch.float64 and torch.all(nz["ts_diff"] == 1)
    assert float(nz["ts_subdiff"].min()) >= 0 and float(nz["ts_subdiff"].max()) <= 1
    if config.model.pixel_bandwidth.enable:
        S = config.model.pixel_bandwidth.it_sample_size
        assert nz["interval_gen"].shape == (1, S - 1, B) and torch.all(nz["interval_gen"] == 0.5)
    # update_train_batch_size's hook: the next batches follow the new size
    datamodule.train_dataset.batch_size = 17
    for s in datamodule.train_normalized_sampler.datasets:
        s.size = 17 if isinstance(s.size, int) else (*s.size[:-1], 17)
    assert next(iter(loaders["event"]))["end_ts"].shape == (1, 17)
    assert next(iter(loaders["normalized"]))["diff_start_ts"].shape == (1, 17)


def test_samplers_distributions():
    from deblur_e_nerf.data import samplers
    g = torch.Generator().manual_seed(0)
    tri = next(iter(samplers.TriangularSampler(0, 1, 200_000, 0, torch.float64, g)))
    # triangular(0, 0, 1): density 2(1 - x), mean 1/3, P(x < 0.5) = 3/4
    assert abs(float(tri.mean()) - 1 / 3) < 3e-3 and abs(float((tri < 0.5).double().mean()) - 0.75) < 3e-3
    uni = next(iter(samplers.UniformSampler(2, 4, (3, 1000), torch.float64, g)))
    assert uni.shape == (3, 1000) and float(uni.min()) >= 2 and float(uni.max()) < 4
    with pytest.raises(ValueError):
        samplers.TriangularSampler(0, 1, 4, 2)
    assert torch.equal(next(iter(samplers.DiracDeltaSampler(0.5, 3, torch.float64))),
                       torch.full((3,), 0.5, dtype=torch.float64))


def test_datamodule_rejects_workers():
    from deblur_e_nerf.data.datamodule import DataModule
    from deblur_e_nerf.utils.easydict import EasyDict
    with pytest.raises(ValueError):
        DataModule(0, ["novel_view"], 1, [0], EasyDict(enable=False), "/nonexistent", 1.0, 1.0, 1.0, None, 9, True,
                   256, 131072, 1, 1, 4)


@pytest.mark.parametrize("name", ["synthetic.yaml", "07_ziggy_and_fuzz_hdr.yaml"])
def test_run_py_val_test_surface(name):
    """run.py val|test (scripts/run.py:114-118): with a views/ folder the DataModule's val / test sets
    are PosedImage views (event_view: the training views' images; novel_view: transforms_val/test),
    the model holds each stage's intrinsics inverse, pixel grid and value range
    (deblur_e_nerf.py:96-162), and the loaders yield the batches validation_step / test_step take.
    Without views/, validation raises (the reference cannot even be constructed then)."""
    import deblur_e_nerf as den
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "eval_epoch_rd1.npz"))
    config = _load(name)
    d = _dataset_dir(rd=1)
    for k in z.files:
        if k.startswith("file:views/"):
            rel = k[len("file:"):]
            if config.eval_target == ["event_view"]:
                rel = rel.replace("transforms_val", "transforms_train")
            path = os.path.join(d, rel)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "wb") as f:
                f.write(z[k].tobytes())
    config.data.dataset_directory = d
    config.data.alpha_over_white_bg = False  # the views are RGB (no alpha channel)
    config.data.val_dataset_ratio = 1.0
    config.data.test_dataset_ratio = 1.0
    config.git_head_hash, config.seed = "test", 0
    datamodule = den.data.datamodule.DataModule(
        config.seed, config.eval_target, config.trainer.num_nodes, config.trainer.gpus, config.model.pixel_bandwidth,
        **config.data)
    model = den.models.deblur_e_nerf.DeblurENeRF(
        config.git_head_hash, config.eval_target, config.trainer.num_nodes, config.trainer.gpus,
        config.model.min_modeled_intensity, config.model.eval_save_pred_intensity_img,
        config.model.checkpoint_filepath, config.model.contrast_threshold, config.model.refractory_period,
        config.model.pixel_bandwidth, config.model.nerf, config.model.correction, config.loss, config.metric,
        config.optimizer, config.lr_scheduler, config.data.dataset_directory, config.data.alpha_over_white_bg,
        config.data.train_eff_ray_sample_batch_size)
    H, W = 20, 24
    assert model.val_img_pixel_pos.shape == (H, W, 2) and model.val_intrinsics_inv.shape == (3, 3)
    assert model.val_min_normalized_pixel_value == 0.5 / 256
    assert model.val_max_normalized_pixel_value == 1 - 0.5 / 256
    if config.eval_target == ["event_view"]:  # the test stage reuses the val views
        assert torch.equal(model.test_intrinsics_inv, model.val_intrinsics_inv)
    else:  # no transforms_test.json: the test stage stays empty (deblur_e_nerf.py:161-162)
        assert model.test_intrinsics_inv is None
    assert model.init_correction_gamma.shape == (1, 1, 1, 1)
    datamodule.setup("validate")
    b = next(iter(datamodule.val_dataloader()))
    assert b["img"].shape == (1, H, W) and b["sample_id"].shape == (1, 16)
    assert b["T_wc_position"].shape == (1, 3) and b["T_wc_orientation"].shape == (1, 3, 3)
    assert len(datamodule.val_dataset) == 3
    if config.eval_target == ["event_view"]:
        datamodule.setup("test")
        assert len(datamodule.test_dataset) == 3
    else:
        with pytest.raises(FileNotFoundError):
            datamodule.setup("test")
    if config.eval_target != ["event_view"]:
        with pytest.raises(RuntimeError):  # no test views: test_step names what is missing
            model.test_step(b, 0)


def test_val_without_views_raises():
    from deblur_e_nerf.data.datamodule import DataModule
    from deblur_e_nerf.utils.easydict import EasyDict
    dm = DataModule(0, ["novel_view"], 1, [0], EasyDict(enable=False), _dataset_dir(), 1.0, 1.0, 1.0, None, 9, True,
                    256, 131072, 1, 1, 0)
    dm.setup("fit")
    assert dm.val_dataset is None
    with pytest.raises(FileNotFoundError):
        dm.setup("validate")
