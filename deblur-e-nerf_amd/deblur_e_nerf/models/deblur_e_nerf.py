"""DeblurENeRF -- mirror of the reference's LightningModule (models/deblur_e_nerf.py:20-1308)
for the training path, so that scripts/run.py and PyTorch Lightning drive it unchanged.

Same constructor arguments (:32-53), the same component attributes and parameter names
(``contrast_threshold``, ``refractory_period``, ``pixel_bandwidth``, ``nerf``, ``trajectory``,
``loss``, ``metric``), the same ``training_step(batch, batch_index)`` (:396-586),
``render_log_intensity`` (:1129-1160), ``render_train_pixels`` (:1162-1183),
``render_pixels`` (:1185-1221), ``bayering`` (:1223-1235), ``derive_mean_value``
(:1237-1250), ``update_train_batch_size`` (:1252-1308) and ``configure_optimizers``
(:1055-1112).  Every array computation of the step runs in libden.so:

  den_event_prep(_bwd)   ContrastThreshold + RefractoryPeriod + the supervision timestamps
  den_trajectory         LinearTrajectory (poses at the render timestamps)
  den_pixel_rays         NeRF.pixel_params_to_ray
  den_march_* / den_render (points = 2) / den_composite_*   occupancy-grid marching, the fused
                         MLP at the packed samples, compositing (NeRF sampler "occupancy", the
                         reference's); or den_render_fwd/bwd with the fixed-count sampler
  den_pixbw_*            PixelBandwidth
  den_event_target(_bwd), den_event_loss_*   Loss.compute
  den_adam_step          optim.Adam (configure_optimizers)

The pixel-bandwidth-off step renders its four supervision groups (diff start / end, TV start /
end) in ONE render call of 4N rays instead of four: same results, one launch.

Without pytorch_lightning (absent in this image) the class derives from torch.nn.Module and
provides the few Trainer attributes the step reads (``trainer.accumulate_grad_batches``,
``global_step``, ``log``, ``all_gather``); ``fit_step`` runs one optimisation step (forward,
backward, DDP-style gradient all-reduce, optimizer) without a Trainer.

Evaluation: ``render_image_eval`` renders an image, ``evaluation_correction``
is the reference's CPU f64 intensity correction (affine log-intensity fit + the black-level
refinement by Gauss-Newton / Levenberg-Marquardt) and ``loss_metric.metric`` gives the PSNR; the
Lightning validation loop and SSIM / LPIPS are outside the scope.
"""
import functools
import math
import os

import numpy as np
import torch
import torch.distributed as dist

from .. import _native
from ..data import datasets
from ..external import marching
from ..loss_metric import loss as loss_lib
from ..loss_metric import metric as metric_lib
from ..optim import Adam
from ..utils import image_io, modules
from ..utils.easydict import EasyDict
from . import event_generation_params, nerf as nerf_lib, pixel_bandwidth as pixbw_lib, trajectories

try:  # the reference's base class when PyTorch Lightning is installed
    import pytorch_lightning as _pl
    _Base = _pl.LightningModule
    _HAS_PL = True
except ImportError:  # pragma: no cover - the image has no pytorch_lightning
    _Base = torch.nn.Module
    _HAS_PL = False


class _TrainerStub:
    """What the module's hooks read of a pytorch_lightning Trainer when there is none: training_step's
    ``accumulate_grad_batches`` / ``datamodule``, evaluation_epoch_end's ``log_dir``,
    ``is_global_zero`` and ``sanity_checking``."""

    def __init__(self, accumulate_grad_batches=1, datamodule=None, log_dir=None):
        self.accumulate_grad_batches = accumulate_grad_batches
        self.datamodule = datamodule
        self.log_dir = log_dir
        self.sanity_checking = False

    @property
    def is_global_zero(self):
        return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def _gather_collection(data, device):
    """pytorch_lightning's LightningModule.all_gather (1.4.9) over the default process group: every
    tensor of a (nested) list / tuple / dict gathered to a (world, ...) stack; with one process the
    tensors come back as they are (PL's single-device plugin), scalars as 0-d tensors."""
    if isinstance(data, dict):
        return type(data)({k: _gather_collection(v, device) for k, v in data.items()})
    if isinstance(data, (list, tuple)):
        return type(data)(_gather_collection(v, device) for v in data)
    t = torch.as_tensor(data, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = t.contiguous()
        out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(out, t)
        return torch.stack(out)
    return t


class DeblurENeRF(_Base):
    INTRINSICS_KEY = "intrinsics"
    NUM_DIM = 3
    MAX_NUM_SAMPLES_PER_RAY = 1024
    CORRECTION_ERRORS_FOLDER_NAME = "correction-errors"
    CORRECTION_ERRORS_EXTENSION = ".csv"
    PREDICTIONS_FOLDER_NAME = "predictions"
    PREDICTION_FILE_EXTENSION = ".png"
    PREDICTION_BIT_DEPTH = 8
    MODEL_COMPONENTS = ["contrast_threshold", "refractory_period", "nerf"]
    MULTI_PARAM_MODEL_COMPONENTS = ["contrast_threshold"]

    def __init__(self, git_head_hash, eval_target, num_nodes, gpus, min_modeled_intensity,
                 eval_save_pred_intensity_img, checkpoint_filepath, contrast_threshold, refractory_period,
                 pixel_bandwidth, nerf, correction, loss, metric, optimizer, lr_scheduler, dataset_directory,
                 alpha_over_white_bg, train_eff_ray_sample_batch_size):
        super().__init__()
        assert isinstance(min_modeled_intensity, (int, float)) and min_modeled_intensity > 0
        for cfg in (contrast_threshold, refractory_period, nerf):
            assert isinstance(cfg.load_state_dict, bool)
            assert isinstance(cfg.freeze, (bool, dict))
        assert isinstance(train_eff_ray_sample_batch_size, int) and train_eff_ray_sample_batch_size > 0
        if nerf.freeze:
            assert nerf.load_state_dict
        num_gpus = num_nodes * (len(gpus) if gpus is not None else 1)
        self.train_ray_sample_batch_size = train_eff_ray_sample_batch_size // num_gpus
        self.eval_save_pred_intensity_img = eval_save_pred_intensity_img
        self.correction = correction
        self.MODEL_COMPONENTS = list(type(self).MODEL_COMPONENTS)
        self.MULTI_PARAM_MODEL_COMPONENTS = list(type(self).MULTI_PARAM_MODEL_COMPONENTS)

        cal = datasets.Event.load_camera_calibration(dataset_directory)
        bayer = str(cal[datasets.Event.BAYER_PATTERN_KEY]) if datasets.Event.BAYER_PATTERN_KEY in cal else ""
        self.has_bayer_filter = bayer != datasets.Event.NULL_BAYER_PATTERN
        self.register_buffer("train_intrinsics_inv",
                             torch.linalg.inv(torch.from_numpy(np.asarray(cal[self.INTRINSICS_KEY])).float()),
                             persistent=False)
        self._init_eval_stages(dataset_directory, eval_target)
        self.render_bkgd = "parameter" if alpha_over_white_bg else None
        # the refinement correction's warm start, carried across evaluations (:171-197)
        if self.correction.black_level_offset:
            self.init_correction_scale, self.init_correction_gamma, self.init_correction_offset = \
                init_correction_params(self.has_bayer_filter, self.correction.per_channel_log_it_scale)

        hp = EasyDict(git_head_hash=git_head_hash, min_modeled_intensity=min_modeled_intensity,
                      checkpoint_filepath=checkpoint_filepath, contrast_threshold=contrast_threshold,
                      refractory_period=refractory_period, pixel_bandwidth=pixel_bandwidth, nerf=nerf, loss=loss,
                      metric=metric, optimizer=optimizer, lr_scheduler=lr_scheduler)
        if _HAS_PL:
            self.save_hyperparameters(dict(hp))
        else:
            self._hparams = hp
            self._trainer = _TrainerStub()
            self._global_step = 0
            self._current_epoch = 0
            self._logger = None
            self.logged = {}

        self.contrast_threshold = event_generation_params.ContrastThreshold(
            dataset_directory, self.hparams.contrast_threshold.parameterize_mean_ct)
        self.refractory_period = event_generation_params.RefractoryPeriod(dataset_directory)
        camera_poses = datasets.CameraPose(dataset_directory, None)
        if self.hparams.pixel_bandwidth.enable:
            self.pixel_bandwidth = pixbw_lib.PixelBandwidth(
                dataset_directory, camera_poses.camera_poses.T_wc_timestamp.min(),
                self.hparams.pixel_bandwidth.f_c_dominant_min, self.hparams.pixel_bandwidth.target_cumprob)
            self.MODEL_COMPONENTS.append("pixel_bandwidth")
            self.MULTI_PARAM_MODEL_COMPONENTS.append("pixel_bandwidth")
        self.nerf = self._build_nerf(camera_poses)
        self.trajectory = trajectories.LinearTrajectory(camera_poses)
        self._load_model_component_state_dicts()
        self._freeze_model_components()
        self.loss = loss_lib.Loss(loss.weight, loss.error_fn, loss.normalize)
        self.metric = metric_lib.Metric(getattr(metric, "lpips_net", None))

    # ------------------------------------------------------------------ trainer glue
    if not _HAS_PL:
        @property
        def hparams(self):
            return self._hparams

        @property
        def trainer(self):
            return self._trainer

        @trainer.setter
        def trainer(self, t):
            self._trainer = t

        @property
        def global_step(self):
            return self._global_step

        def log(self, name, value, **kwargs):
            self.logged[name] = value.detach() if torch.is_tensor(value) else value

        @property
        def current_epoch(self):
            return self._current_epoch

        @property
        def device(self):
            return self.train_intrinsics_inv.device

        @property
        def logger(self):
            """None (no TensorBoard logger) unless a test or driver sets ``_logger``: an object with
            ``experiment.add_image(tag, img, global_step=...)``."""
            return self._logger

        def all_gather(self, data):
            return _gather_collection(data, self.trajectory.T_wc_position.device)

    # ------------------------------------------------------------------ evaluation stages
    def _init_eval_stages(self, dataset_directory, eval_target):
        """deblur_e_nerf.py:96-162: the val views (the training views' images for an ``event_view``
        target, else ``views/transforms_val.json``) and, when present, the test views give each stage
        its intrinsics inverse, its (H, W, 2) pixel grid and its value range.  One deviation: the
        reference cannot be constructed without a ``views/`` folder (PosedImage joins a None path);
        here the stages are then left empty (None) and only validation / testing raise."""
        if set(eval_target) == {"event_view"}:
            val_stage = "train"
        elif set(eval_target) == {"novel_view"}:
            val_stage = "val"
        else:
            raise NotImplementedError(f"eval_target {eval_target}")
        for name in ("val", "test"):
            setattr(self, f"{name}_min_normalized_pixel_value", None)
            setattr(self, f"{name}_max_normalized_pixel_value", None)
            self.register_buffer(f"{name}_intrinsics_inv", None, persistent=False)
            self.register_buffer(f"{name}_img_pixel_pos", None, persistent=False)
        if datasets.PosedImage.posed_img_folder_path(dataset_directory) is None:
            return
        val = datasets.PosedImage(dataset_directory, val_stage, permutation_seed=None)
        self._set_eval_stage("val", val)
        try:
            test = val if val_stage == "train" else datasets.PosedImage(dataset_directory, "test", permutation_seed=None)
            self._set_eval_stage("test", test)
        except FileNotFoundError:
            pass

    def _set_eval_stage(self, name, posed):
        H, W = posed.posed_imgs.img.shape[-2:]
        setattr(self, f"{name}_min_normalized_pixel_value", posed.min_normalized_pixel_value)
        setattr(self, f"{name}_max_normalized_pixel_value", posed.max_normalized_pixel_value)
        dev = self.train_intrinsics_inv.device
        setattr(self, f"{name}_intrinsics_inv", posed.posed_imgs.intrinsics.inverse().to(dev))
        setattr(self, f"{name}_img_pixel_pos",
                torch.stack(torch.meshgrid(torch.arange(W), torch.arange(H), indexing="xy"), dim=2)
                .to(torch.get_default_dtype()).to(dev))

    # ------------------------------------------------------------------ components
    def _build_nerf(self, camera_poses):
        cfg = self.hparams.nerf
        if cfg.aabb == "auto":
            p = camera_poses.camera_poses.T_wc_position
            aabb = torch.cat((p.min(dim=0).values, p.max(dim=0).values)).tolist()
        else:
            aabb = list(cfg.aabb)
        ctype = {"aabb": nerf_lib.ContractionType.AABB, "sphere": nerf_lib.ContractionType.UN_BOUNDED_SPHERE,
                 "tanh": nerf_lib.ContractionType.UN_BOUNDED_TANH}[cfg.contraction_type]
        if cfg.render_step_size == "auto":
            a = torch.tensor(aabb)
            step = math.sqrt(self.NUM_DIM) * torch.max(a[3:] - a[:3]).item() / self.MAX_NUM_SAMPLES_PER_RAY
        else:
            step = cfg.render_step_size
        rd = 3 if self.has_bayer_filter else 1
        return nerf_lib.NeRF(aabb, ctype, cfg.occ_grid, cfg.near_plane, cfg.far_plane, step, self.render_bkgd,
                             cfg.cone_angle, cfg.early_stop_eps, cfg.alpha_thre, cfg.test_chunk_size, cfg.arch,
                             arch_config=cfg[cfg.arch], num_dim=self.NUM_DIM, radiance_dim=rd,
                             sampler=cfg.get("sampler", "occupancy"), n_samples=cfg.get("n_samples", 128),
                             mode=cfg.get("compute_mode", "f32"))

    def _load_model_component_state_dicts(self):
        if not any(self.hparams[c].load_state_dict for c in self.MODEL_COMPONENTS):
            return
        ckpt = torch.load(self.hparams.checkpoint_filepath, map_location="cpu", weights_only=True)
        for c in self.MODEL_COMPONENTS:
            if self.hparams[c].load_state_dict:
                prefix = c + "."
                sd = {k[len(prefix):]: v for k, v in ckpt["state_dict"].items() if k.startswith(prefix)}
                getattr(self, c).load_state_dict(sd)

    def _freeze_model_components(self):
        for c in self.MODEL_COMPONENTS:
            f = self.hparams[c].freeze
            if isinstance(f, dict):
                f = f.default
            if f:
                modules.freeze(getattr(self, c))
        for c in self.MULTI_PARAM_MODEL_COMPONENTS:
            if isinstance(self.hparams[c].freeze, bool):
                continue
            comp = getattr(self, c)
            for name, fr in self.hparams[c].freeze.items():
                if name == "default":
                    continue
                getattr(comp.parametrizations, name).original.requires_grad_(not fr)

    # ------------------------------------------------------------------ training step
    def forward(self, batch):
        pass

    def training_step(self, batch, batch_index):
        batch = EasyDict(batch)
        batch.size = batch.event.start_ts.numel()
        for v in batch.normalized.values():
            assert v.shape[-1] == batch.size
        for k, v in batch.event.items():
            batch.event[k] = v.squeeze(dim=0)
        for k, v in batch.normalized.items():
            batch.normalized[k] = v.squeeze(dim=0)
        if self.has_bayer_filter:
            batch.event.channel_idx = batch.event.channel_idx.to(torch.int64)
        else:
            batch.event.channel_idx = None
        w = self.hparams.loss.weight
        has_diff, has_tv = w.log_intensity_diff > 0, w.log_intensity_tv > 0
        dev = batch.event.end_ts.device
        N = batch.size

        # ContrastThreshold + RefractoryPeriod + supervision timestamps (deblur_e_nerf.py:414-455),
        # one fused kernel with its reverse mode (gradients into C+/C-/tau_r when unfrozen)
        zeros = torch.zeros(N, dtype=torch.float64, device=dev)
        nz = batch.normalized
        norm = torch.stack([nz.get("ts_diff", zeros), nz.get("diff_start_ts", zeros), nz.get("ts_subdiff", zeros),
                            nz.get("subdiff_start_ts", zeros)]).to(torch.float64).contiguous()
        ct = torch.stack([self.contrast_threshold.pos_contrast_threshold,
                          self.contrast_threshold.neg_contrast_threshold]).reshape(2)
        tau = self.refractory_period.refractory_period.reshape(1)
        ev = batch.event
        lid, start_ts, render_ts, ts_diff, ts_subdiff, _ = _native.EventPrepFunction.apply(
            ev.num_pos.to(torch.int64).contiguous(), ev.num_neg.to(torch.int64).contiguous(),
            ev.end_ts.to(torch.int64).contiguous(), ev.start_ts.to(torch.int64).contiguous(), norm, ct, tau, None,
            has_diff, has_tv)
        ev.log_intensity_diff = lid
        ev.start_ts = start_ts
        ev.pop("num_pos")
        ev.pop("num_neg")
        batch.diff = EasyDict(ts_diff=ts_diff, start_ts=render_ts[0], end_ts=render_ts[1]) if has_diff else None
        batch.subdiff = EasyDict(ts_diff=ts_subdiff, start_ts=render_ts[2], end_ts=render_ts[3]) if has_tv else None
        interval_gen = batch.normalized.get("interval_gen", None)
        batch.pop("normalized")

        if batch_index % self.trainer.accumulate_grad_batches == 0:
            self.nerf.update_occ_grid(step=self.global_step, T_wc_position=self.trajectory.T_wc_position)

        groups = [(batch.diff, "start"), (batch.diff, "end")] if has_diff else []
        groups += [(batch.subdiff, "start"), (batch.subdiff, "end")] if has_tv else []
        if self.hparams.pixel_bandwidth.enable:
            # stateful differencing-amplifier reset on the first call (pixel_bandwidth.py:419-446)
            for gi, (d, side) in enumerate(groups):
                li, occ, spr, valid = self.render_log_intensity(d[side + "_ts"], ev.position, ev.channel_idx,
                                                                interval_gen, reset_diff=(gi == 0))
                d[side + "_log_intensity"], d[side + "_mean_ray_occ_rate"] = li, occ
                d[side + "_mean_num_samples_per_ray"], d["is_" + side + "_valid"] = spr, valid
        else:
            # the four groups as ONE render of len(groups) x N rays
            ts = torch.stack([d[side + "_ts"] for d, side in groups])
            li, occ, spr, valid = self.render_log_intensity(ts, ev.position, ev.channel_idx)
            for gi, (d, side) in enumerate(groups):
                d[side + "_log_intensity"], d[side + "_mean_ray_occ_rate"] = li[gi], occ[gi]
                d[side + "_mean_num_samples_per_ray"], d["is_" + side + "_valid"] = spr, valid[gi]
        for d in (batch.diff, batch.subdiff):
            if d is None:
                continue
            d.log_intensity_diff = d.end_log_intensity - d.start_log_intensity
            d.is_valid = d.is_start_valid | d.is_end_valid
            for k in ("start_ts", "end_ts", "start_log_intensity", "end_log_intensity"):
                d.pop(k)
        ev.pop("position")
        if self.has_bayer_filter:
            ev.pop("channel_idx")

        batch.mean_num_samples_per_ray = self.update_train_batch_size(batch.diff, batch.subdiff, batch_index)
        batch.mean_loss = self.loss.compute(ev, batch.diff, batch.subdiff,
                                            self.contrast_threshold.mean_contrast_threshold)
        batch.weighted_mean_loss = EasyDict({k: v * self.hparams.loss.weight[k] for k, v in batch.mean_loss.items()})
        train_loss = sum(batch.weighted_mean_loss.values())

        self.log("train/loss", train_loss, prog_bar=True)
        for k, v in batch.mean_loss.items():
            self.log(f"train/{k}", v)
        for c in self.MULTI_PARAM_MODEL_COMPONENTS:
            comp = getattr(self, c)
            for name in comp.parametrizations.keys():
                p = getattr(comp, name)
                if p.requires_grad:
                    self.log(f"train/{c}/{name}", p)
        if not self.hparams.refractory_period.freeze:
            self.log("train/refractory_period", self.refractory_period.refractory_period)
        batch.mean_ray_occ_rate = self.derive_mean_value(
            [(batch.diff, ["start_mean_ray_occ_rate", "end_mean_ray_occ_rate"]),
             (batch.subdiff, ["start_mean_ray_occ_rate", "end_mean_ray_occ_rate"])])
        batch.mean_valid_rate = self.derive_mean_value(
            [(batch.diff, ["is_start_valid", "is_end_valid"]), (batch.subdiff, ["is_start_valid", "is_end_valid"])],
            value_transform=lambda b: b.to(torch.get_default_dtype()).mean())
        self.log("train/batch_size", batch.size)
        self.log("train/mean_num_samples_per_ray", batch.mean_num_samples_per_ray)
        self.log("train/mean_ray_occ_rate", batch.mean_ray_occ_rate)
        self.log("train/mean_valid_rate", batch.mean_valid_rate)
        return train_loss

    # ------------------------------------------------------------------ rendering
    def render_log_intensity(self, timestamp, pixel_position, pixel_channel_idx=None, normalized_interval_gen=None,
                             reset_diff=False):
        """deblur_e_nerf.py:1129-1160 -> (log intensity ([G,] N), mean ray occupancy rate, mean
        samples per ray, is_valid ([G,] N)).  ``timestamp`` may carry a leading group dim G
        (pixel bandwidth off) to render several supervision groups in one call."""
        if self.hparams.pixel_bandwidth.enable:
            fn = functools.partial(self.render_train_pixels, pixel_position=pixel_position,
                                   pixel_channel_idx=pixel_channel_idx)
            log_intensity, aux = self.pixel_bandwidth(normalized_interval_gen, timestamp, fn, reset_diff)
            mean_ray_occ_rate, mean_num_samples_per_ray, is_valid = aux
            is_valid = is_valid.any(dim=0)
        else:
            intensity, mean_ray_occ_rate, mean_num_samples_per_ray, is_valid = self.render_train_pixels(
                timestamp, pixel_position, pixel_channel_idx)
            log_intensity = intensity.log()
        return log_intensity, mean_ray_occ_rate, mean_num_samples_per_ray, is_valid

    def render_train_pixels(self, timestamp, pixel_position, pixel_channel_idx=None):
        """deblur_e_nerf.py:1162-1183: poses at the timestamps ([G,] N), rays, render, bayering."""
        T_wc_position, T_wc_orientation = self.trajectory(timestamp)
        intensity, opacity, _, mean_num_samples_per_ray, is_valid = self.render_pixels(
            self.train_intrinsics_inv, pixel_position, T_wc_position, T_wc_orientation)
        if self.has_bayer_filter:
            intensity = self.bayering(intensity, pixel_channel_idx)
        occ = (opacity > 0).to(torch.get_default_dtype())
        mean_ray_occ_rate = occ.mean() if timestamp.dim() == 1 else occ.reshape(occ.shape[0], -1).mean(dim=1)
        return intensity, mean_ray_occ_rate, mean_num_samples_per_ray, is_valid

    def render_pixels(self, intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation):
        """deblur_e_nerf.py:1185-1221 -> intensity ([3,] [M,] N), opacity, depth, mean samples per
        ray, is_valid."""
        ray_origin, ray_direction = self.nerf.pixel_params_to_ray(intrinsics_inverse, pixel_position,
                                                                   T_wc_position, T_wc_orientation)
        intensity, opacity, depth, mean_num_samples_per_ray = self.nerf(ray_origin, ray_direction)
        if intensity.dim() > opacity.dim():
            intensity = intensity.permute(-1, *range(opacity.dim()))
        intensity = intensity + self.hparams.min_modeled_intensity
        if self.render_bkgd is None:
            is_valid = opacity > 0
        else:
            is_valid = torch.ones_like(opacity, dtype=torch.bool)
        depth = depth * torch.sum(ray_direction * T_wc_orientation[..., 2], dim=-1)
        return intensity, opacity, depth, mean_num_samples_per_ray, is_valid

    def bayering(self, intensity, channel_idx):
        """deblur_e_nerf.py:1223-1235: (3, [S,] N) -> ([S,] N), the event's colour channel."""
        idx = channel_idx.unsqueeze(dim=0)
        if intensity.dim() == 3:
            idx = idx.unsqueeze(dim=0).expand(-1, intensity.shape[1], -1)
        return intensity.gather(dim=0, index=idx).squeeze(dim=0)

    @staticmethod
    def derive_mean_value(dict_keys_pairs, value_transform=lambda v: v):
        pairs = [(d, [k for k in keys if k in d.keys()]) for d, keys in dict_keys_pairs if d is not None]
        values = [value_transform(d[k]) for d, keys in pairs for k in keys]
        return sum(values) / len(values)

    def update_train_batch_size(self, batch_diff, batch_subdiff, batch_index):
        """deblur_e_nerf.py:1252-1308: the mean samples per ray over the renders, averaged over
        the ranks (all_gather), sets the next event batch size so that the samples per render
        call stay ~ train_eff_ray_sample_batch_size / gpus (on the second-to-last micro-batch of
        an accumulation group)."""
        mspr = self.derive_mean_value([(batch_diff, ["start_mean_num_samples_per_ray", "end_mean_num_samples_per_ray"]),
                                       (batch_subdiff, ["start_mean_num_samples_per_ray",
                                                        "end_mean_num_samples_per_ray"])])
        mspr = torch.mean(self.all_gather(torch.tensor(float(mspr))).float())
        acc = self.trainer.accumulate_grad_batches
        if acc > 1 and (batch_index % acc) != (acc - 2):
            return mspr
        new_size = int(self.train_ray_sample_batch_size / mspr)
        self.train_batch_size = new_size
        dm = getattr(self.trainer, "datamodule", None)
        if dm is not None and hasattr(dm, "train_dataset"):
            dm.train_dataset.batch_size = new_size
            for s in dm.train_normalized_sampler.datasets:
                s.size = new_size if isinstance(s.size, int) else (*s.size[:-1], new_size)
        return mspr

    # ------------------------------------------------------------------ optimisation
    def configure_optimizers(self):
        """deblur_e_nerf.py:1055-1112 with optim.Adam (den_adam_step) in place of torch.optim.Adam."""
        refr = list(self.refractory_period.parameters())
        mlp = [p for n, p in self.named_parameters() if n.startswith("nerf.radiance_field.mlp")]
        groups = [{"params": refr,
                   "lr": self.refractory_period.max_refractory_period.item()
                   * self.hparams.optimizer.relative_lr.refractory_period},
                  {"params": mlp, "weight_decay": self.hparams.loss.weight.nerf_mlp_weight_decay}]
        for c in self.MULTI_PARAM_MODEL_COMPONENTS:
            comp = getattr(self, c)
            groups.extend({"params": [getattr(comp.parametrizations, n).original], "lr": lr}
                          for n, lr in self.hparams.optimizer.lr[c].items())
        collated = set(p for g in groups for p in g["params"])
        other = [p for p in self.parameters() if p not in collated]
        groups.append({"params": other})
        if self.hparams.optimizer.algo != "adam":
            raise NotImplementedError
        optimizer = Adam(groups, lr=self.hparams.optimizer.lr.default)
        if self.hparams.lr_scheduler.algo != "multi_step_lr":
            raise NotImplementedError
        sched = torch.optim.lr_scheduler.MultiStepLR(optimizer,
                                                     milestones=self.hparams.lr_scheduler.multi_step_lr.milestones,
                                                     gamma=self.hparams.lr_scheduler.multi_step_lr.gamma)
        return {"optimizer": optimizer, "lr_scheduler": {"scheduler": sched,
                                                         "interval": self.hparams.lr_scheduler.interval}}

    def fit_step(self, batch, batch_index, optimizer):
        """One optimisation step without a Trainer: the occupancy grid from rank 0 (DDP's buffer
        broadcast), training_step, backward, the DDP gradient all-reduce (mean over ranks, one
        flat buffer), optimizer step on the last micro-batch of an accumulation group (PL's
        accumulate_grad_batches semantics: gradients summed over the group, each micro-batch loss
        scaled by 1 / accumulate_grad_batches).

        DDP (broadcast_buffers=True, run.py:86-88) broadcasts rank 0's buffers in a forward only
        when the previous forward ran with gradient sync on; PL runs micro-batches 0..acc-2 of a
        group under ``no_sync()``, so the broadcast happens before the FIRST micro-batch of each
        group only -- before training_step's grid update there (deblur_e_nerf.py:465), so the
        remaining micro-batches of the group march with each rank's own freshly updated grid."""
        acc = self.trainer.accumulate_grad_batches
        if batch_index % acc == 0:
            marching.sync_grid(getattr(self.nerf, "occupancy_grid", None))
        loss = self.training_step(batch, batch_index)
        (loss / acc).backward()
        if (batch_index + 1) % acc == 0:
            allreduce_gradients(self)
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)
            if not _HAS_PL:
                self._global_step += 1
        return loss

    # ------------------------------------------------------------------ evaluation (val / test)
    def on_train_epoch_start(self):
        """deblur_e_nerf.py:392-394: release the allocator's unoccupied cached blocks."""
        if torch.cuda.is_available():
            torch.cuda.empty_cache()

    def on_train_start(self):
        """deblur_e_nerf.py:1114-1127: the hyper-parameter metrics a logger tracks."""
        if self.logger is None or not hasattr(self.logger, "log_hyperparams"):
            return
        self.logger.log_hyperparams(self.hparams, {"val/l1": float("inf"), "val/psnr": float("-inf"), "val/ssim": -1,
                                                   "val/lpips": float("inf")})

    def _stage(self, name, keys):
        for k in keys:
            if getattr(self, f"{name}_{k}") is None:
                raise RuntimeError(f"no {name} views: the dataset directory has no views/ folder with "
                                   f"transforms_{'val' if name == 'val' else 'test'}.json (PosedImage)")
        return EasyDict({k: getattr(self, f"{name}_{k}") for k in keys})

    def validation_step(self, batch, batch_index):
        """deblur_e_nerf.py:588-593."""
        return self.evaluation_step(batch, batch_index, self._stage("val", ("intrinsics_inv", "img_pixel_pos")))

    def test_step(self, batch, batch_index):
        """deblur_e_nerf.py:595-600."""
        return self.evaluation_step(batch, batch_index, self._stage("test", ("intrinsics_inv", "img_pixel_pos")))

    def evaluation_step(self, batch, batch_index, stage):
        """deblur_e_nerf.py:602-652: one view (batch size 1) rendered at its camera pose over the
        stage's pixel grid (render_pixels: den_pixel_rays + the NeRF renders, chunked in eval mode)
        -> sample_id, pred_intensity_img ([3,] H, W), target_intensity_img, exposure_time, gain."""
        batch = EasyDict(batch)
        batch.size = len(batch.img)
        assert batch.size == 1
        for k, v in batch.items():
            if k != "size":
                batch[k] = v.squeeze(dim=0)
        target = batch.img
        H, W = target.shape[-2:]
        assert H == stage.img_pixel_pos.shape[0] and W == stage.img_pixel_pos.shape[1]
        pos = batch.T_wc_position.view(1, 1, 3).expand(H, W, -1)
        rot = batch.T_wc_orientation.view(1, 1, 3, 3).expand(H, W, -1, -1)
        pred, _, _, _, _ = self.render_pixels(stage.intrinsics_inv, stage.img_pixel_pos, pos, rot)
        if "exposure_time" not in batch.keys():
            batch.exposure_time = torch.tensor(1, dtype=torch.int64, device=self.device)
        if "gain" not in batch.keys():
            batch.gain = torch.tensor(1, dtype=torch.get_default_dtype(), device=self.device)
        return {"sample_id": batch.sample_id, "pred_intensity_img": pred, "target_intensity_img": target,
                "exposure_time": batch.exposure_time, "gain": batch.gain}

    def validation_epoch_end(self, outputs):
        """deblur_e_nerf.py:654-660."""
        stage = self._stage("val", ("min_normalized_pixel_value", "max_normalized_pixel_value"))
        stage.name = "val"
        return self.evaluation_epoch_end(outputs, stage)

    def test_epoch_end(self, outputs):
        """deblur_e_nerf.py:662-668."""
        stage = self._stage("test", ("min_normalized_pixel_value", "max_normalized_pixel_value"))
        stage.name = "test"
        return self.evaluation_epoch_end(outputs, stage)

    def evaluation_epoch_end(self, outputs, stage):
        """deblur_e_nerf.py:670-1053: gather the views of every rank; on global rank 0 the intensity
        correction on the CPU in f64 (``evaluation_correction``: the least-squares affine log-intensity
        fit, then -- ``correction.black_level_offset`` -- the OffsetGammaCorrection refinement by
        Gauss-Newton / Levenberg-Marquardt from the warm start of the previous evaluation, which is
        then carried on unless Lightning is sanity checking), the per-view metrics on the device
        (``Metric.compute``: den_image_error, den_ssim), their mean logged as ``<stage>/<metric>``, and
        -- with a logger -- the correction-error log, the first view as an image and, with
        ``eval_save_pred_intensity_img``, the 8-bit predictions as PNG files."""
        outputs = self.all_gather(outputs)
        dim = outputs[0]["sample_id"].dim()
        merge = torch.stack if dim == 1 else torch.cat
        sample_id = merge([o["sample_id"] for o in outputs])
        pred = merge([o["pred_intensity_img"] for o in outputs])
        target = merge([o["target_intensity_img"] for o in outputs])
        exposure_time = merge([o["exposure_time"] for o in outputs])
        gain = merge([o["gain"] for o in outputs])
        del outputs
        sample_id = self.unicode_code_pt_tensor_to_str(sample_id)
        log_dir = self.trainer.log_dir
        if not self.trainer.is_global_zero:
            return
        gain_exposure_prod = (gain * exposure_time).cpu()
        batch_size = len(target)
        res = evaluation_correction(pred.cpu(), target.cpu(), gain_exposure_prod, self.has_bayer_filter,
                                    self.correction,
                                    init=(self.init_correction_scale, self.init_correction_gamma,
                                          self.init_correction_offset) if self.correction.black_level_offset else None)
        pred, target = res.pred, res.target
        if self.correction.black_level_offset:
            if not self.trainer.sanity_checking:
                self.init_correction_scale, self.init_correction_gamma, self.init_correction_offset = res.converged
            if self.logger is not None:
                folder = os.path.join(log_dir, self.CORRECTION_ERRORS_FOLDER_NAME)
                os.makedirs(folder, exist_ok=True)
                np.savetxt(os.path.join(folder, str(self.current_epoch) + self.CORRECTION_ERRORS_EXTENSION),
                           res.errors.numpy(), fmt=("%.14f",))
        self.last_correction = res
        pred = pred.to(self.device)
        target = target.to(self.device)
        pred = pred.to(target.dtype)
        metric = self.metric.init_batch_metric()
        for p, t in zip(pred, target):
            sample = self.metric.compute(p, t, min_target_val=stage.min_normalized_pixel_value,
                                         max_target_val=stage.max_normalized_pixel_value)
            for k, v in sample.items():
                metric[k].append(v)
        for k, v in metric.items():
            metric[k] = sum(v) / batch_size
        self.log(f"{stage.name}/epoch", self.current_epoch, prog_bar=True, logger=False, rank_zero_only=True)
        for k, v in metric.items():
            self.log(f"{stage.name}/{k}", v, prog_bar=True, rank_zero_only=True)
        if self.logger is None:
            return
        lo, hi = stage.min_normalized_pixel_value, stage.max_normalized_pixel_value
        self.logger.experiment.add_image(f"{stage.name}/pred_intensity_img",
                                         ((pred[0] - lo) / (hi - lo)).clamp(min=0, max=1), global_step=self.global_step)
        if self.current_epoch == 0:
            self.logger.experiment.add_image(f"{stage.name}/target_intensity_img", (target[0] - lo) / (hi - lo),
                                             global_step=self.global_step)
        del target
        if not self.eval_save_pred_intensity_img:
            return
        max_pixel_value = 2 ** self.PREDICTION_BIT_DEPTH - 1
        img = (max_pixel_value * ((pred.cpu() - lo) / (hi - lo)).clamp(min=0, max=1)).round()
        img = img.numpy().astype({8: np.uint8, 16: np.uint16}[self.PREDICTION_BIT_DEPTH])
        img = img.transpose(0, 2, 3, 1)  # (B, H, W, 1 | 3) grey / RGB
        if self.has_bayer_filter:
            img = np.stack([image_io.bgr_to_rgb(x) for x in img], axis=0)  # RGB -> BGR, as cv2.imwrite expects
        folder = os.path.join(log_dir, self.PREDICTIONS_FOLDER_NAME)
        os.makedirs(folder, exist_ok=True)
        for sid, x in zip(sample_id, img):
            image_io.imwrite(os.path.join(folder, sid + self.PREDICTION_FILE_EXTENSION), x)

    @staticmethod
    def unicode_code_pt_tensor_to_str(batch_unicode_code_pt_tensor):
        """deblur_e_nerf.py:1310-1319: code points -> strings, trailing padding stripped."""
        return ["".join(map(chr, (int(c) for c in sample))).rstrip() for sample in batch_unicode_code_pt_tensor]

    @torch.no_grad()
    def run_evaluation(self, stage, datamodule):
        """What pytorch_lightning's ``Trainer.validate`` / ``Trainer.test`` run on this module
        (scripts/run.py:114-118), for use without Lightning: the stage's loader (sharded over the
        ranks of the default process group as Lightning's ``replace_sampler_ddp`` does, without
        shuffling), eval mode and no_grad, ``validation_step`` / ``test_step`` per batch on the
        module's device, then ``*_epoch_end``.  Returns ``[{"<stage>/<metric>": value}]`` as the
        Trainer does."""
        assert stage in ("val", "test")
        datamodule.setup("validate" if stage == "val" else "test")
        ds = datamodule.val_dataset if stage == "val" else datamodule.test_dataset
        bs = datamodule.val_batch_size if stage == "val" else datamodule.test_batch_size
        sampler = None
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            sampler = torch.utils.data.distributed.DistributedSampler(ds, shuffle=False, drop_last=False)
        loader = torch.utils.data.DataLoader(ds, batch_size=bs, sampler=sampler, shuffle=False, num_workers=0)
        step = self.validation_step if stage == "val" else self.test_step
        end = self.validation_epoch_end if stage == "val" else self.test_epoch_end
        was = self.training
        self.eval()
        try:
            dev = self.device
            outputs = [step({k: v.to(dev) for k, v in b.items()}, i) for i, b in enumerate(loader)]
            end(outputs)
        finally:
            self.train(was)
        logged = getattr(self, "logged", {})
        return [{k: float(v) for k, v in logged.items() if k.startswith(stage + "/") and k != stage + "/epoch"}]

    @torch.no_grad()
    def render_image_eval(self, intrinsics_inverse, T_wc_position, T_wc_orientation, img_height, img_width):
        """evaluation_step's render (deblur_e_nerf.py:602-652): the (H, W) image of one camera
        pose -> intensity ([3,] H, W)."""
        dev = self.train_intrinsics_inv.device
        pix = torch.stack(torch.meshgrid(torch.arange(img_width), torch.arange(img_height), indexing="xy"),
                          dim=2).to(torch.get_default_dtype()).to(dev)
        pos = T_wc_position.reshape(1, 1, 3).expand(img_height, img_width, -1).to(dev)
        rot = T_wc_orientation.reshape(1, 1, 3, 3).expand(img_height, img_width, -1, -1).to(dev)
        was = self.training
        self.eval()
        try:
            intensity, _, _, _, _ = self.render_pixels(intrinsics_inverse.to(dev), pix, pos, rot)
        finally:
            self.train(was)
        return intensity


def _affine_log_fit(pred_intensity_img, target_intensity_img, gain_exposure_prod, has_bayer_filter,
                    per_channel_log_it_scale):
    """deblur_e_nerf.py:705-811: the least-squares (f64) log-intensity scale and offset -- per
    channel, or one scale and per-channel offsets for a Bayer sensor without
    ``per_channel_log_it_scale`` -- of the predicted onto the target log intensities (normalised by
    the mean-normalised gain-exposure product).  -> corrected log predictions (B, C, H, W) f64 in the
    normalised domain, the targets (B, C, H, W), the normalised gain-exposure products (B,) f64,
    their logs (B, 1, 1, 1), gamma, scale."""
    pred, target = pred_intensity_img.detach().cpu(), target_intensity_img.detach().cpu()
    while target.dim() < 3:
        pred, target = pred[None], target[None]
    if target.dim() == 3:  # (B, H, W): grayscale -> a channel dim of 1 (:722-725)
        pred, target = pred.unsqueeze(1), target.unsqueeze(1)
    B, C, H, W = target.shape
    # the gain-exposure normalisation in the product's own dtype (deblur_e_nerf.py:707-711, 737), f64
    # only where the reference casts (OffsetGammaCorrection's const_scale, :854)
    if gain_exposure_prod is None:
        gep = torch.ones(B, dtype=torch.get_default_dtype())
    else:
        gep = torch.as_tensor(gain_exposure_prod).detach().cpu().reshape(B)
        if not gep.is_floating_point():
            gep = gep.to(torch.get_default_dtype())
    nge_in = gep / gep.mean()
    log_gep = nge_in.log().view(B, 1, 1, 1)
    nge = nge_in.to(torch.float64)
    # logs in the images' dtype, f64 only for the least squares (the reference's order, :729-792)
    plog = pred.log().to(torch.float64)
    tlog = (target.log() - log_gep).to(torch.float64)
    per_channel = (not has_bayer_filter) or per_channel_log_it_scale
    if per_channel:
        A = torch.nn.functional.pad(plog.unsqueeze(-1), (0, 1), value=1.0)  # (B, C, H, W, 2)
    else:
        A = torch.nn.functional.pad(plog.unsqueeze(-1), (0, 3), value=0.0)  # (B, 3, H, W, 4)
        for c in range(3):
            A[:, c, ..., c + 1] = 1.0
    A = A.transpose(0, 1).flatten(1, 3)                                      # (C, B H W, 2 | 4)
    y = tlog.unsqueeze(-1).transpose(0, 1).flatten(1, 3)                     # (C, B H W, 1)
    if not per_channel:
        A, y = A.flatten(0, 1), y.flatten(0, 1)
    sol = torch.linalg.lstsq(A, y).solution
    corr = (A @ sol).view(C, B, H, W).transpose(0, 1)
    if per_channel:
        gamma, scale = sol[:, 0, 0], sol[:, 1, 0].exp()
    else:
        gamma, scale = sol[0, :], sol[1:, 0].exp()
    return corr, target, nge, log_gep, gamma, scale


def affine_log_intensity_correction(pred_intensity_img, target_intensity_img, gain_exposure_prod=None,
                                    has_bayer_filter=False, per_channel_log_it_scale=False):
    """The evaluation's affine log-intensity alignment alone (deblur_e_nerf.py:705-833 with
    ``black_level_offset`` false): images ([B,] [1/3,] H, W) -> (corrected predicted intensities
    (B, 1/3, H, W), gamma, scale).  ``evaluation_correction`` adds the black-level refinement."""
    corr, _, _, log_gep, gamma, scale = _affine_log_fit(pred_intensity_img, target_intensity_img,
                                                       gain_exposure_prod, has_bayer_filter, per_channel_log_it_scale)
    # black_level_offset off: the gain-exposure normalisation undone on the prediction (:819-826)
    return (corr + log_gep).exp(), gamma, scale


def init_correction_params(has_bayer_filter, per_channel_log_it_scale=False):
    """DeblurENeRF.__init__'s initial refinement parameters (deblur_e_nerf.py:173-195): scale 1,
    offset 0 per radiance channel, gamma 1 per channel or shared (f64)."""
    rd = 3 if has_bayer_filter else 1
    per_channel = (not has_bayer_filter) or per_channel_log_it_scale
    return (torch.ones((rd, 1, 1, 1), dtype=torch.float64),
            torch.ones((rd if per_channel else 1, 1, 1, 1), dtype=torch.float64),
            torch.zeros((rd, 1, 1, 1), dtype=torch.float64))


def evaluation_correction(pred_intensity_img, target_intensity_img, gain_exposure_prod=None,
                          has_bayer_filter=False, correction=None, init=None):
    """The evaluation's intensity correction (deblur_e_nerf.py:705-935) on the CPU in f64, as the
    reference runs it: the affine log-intensity fit, then -- with ``correction.black_level_offset``
    (every shipped config) -- the joint gamma / scale / black-level refinement of an
    ``OffsetGammaCorrection`` by Gauss-Newton or Levenberg-Marquardt (``correction.optimizer``: algo
    "gn" | "lm", max_steps, lm.radius), stopped early once the error and the parameters stop moving.

    ``correction`` is the config's EasyDict (per_channel_log_it_scale, black_level_offset,
    optimizer); ``init`` the warm-start (scale, gamma, offset) the reference carries across
    evaluations (``init_correction_params`` when None).  Returns an EasyDict: ``pred`` corrected
    intensities (B, 1/3, H, W), ``target`` (B, 1/3, H, W), effective ``gamma``, ``scale``, ``offset``
    (None without the refinement), per-step ``errors`` and the ``converged`` (scale, gamma, offset)
    for the next warm start."""
    from ..external import optimizer as opt_lib
    from ..utils import modules as mod
    from .offset_gamma_correction import OffsetGammaCorrection
    cfg = correction if correction is not None else EasyDict(per_channel_log_it_scale=False,
                                                              black_level_offset=False)
    corr, target, nge, log_gep, gamma, scale = _affine_log_fit(pred_intensity_img, target_intensity_img,
                                                               gain_exposure_prod, has_bayer_filter,
                                                               cfg.per_channel_log_it_scale)
    if not cfg.black_level_offset:
        return EasyDict(pred=(corr + log_gep).exp(), target=target, gamma=gamma, scale=scale, offset=None,
                        errors=None, converged=None)
    pred = corr.exp().unsqueeze(-1)                      # (B, C, H, W, 1), f64
    tgt = target.unsqueeze(-1)                           # (B, C, H, W, 1)
    init = init_correction_params(has_bayer_filter, cfg.per_channel_log_it_scale) if init is None else init
    model = OffsetGammaCorrection(nge.view(-1, 1, 1, 1, 1), *init)
    o = cfg.optimizer
    if o.algo == "gn":
        optimizer = opt_lib.GaussNewton(model, solver=opt_lib.LSTSQ())
    elif o.algo == "lm":
        optimizer = opt_lib.LevenbergMarquardt(model, strategy=opt_lib.TrustRegion(**dict(o.lm)))
    else:
        raise NotImplementedError(o.algo)
    n = tgt.numel()
    with torch.no_grad():
        errors = [float(optimizer.model.loss(input=pred, target=tgt)) / n]
    for _ in range(1, int(o.max_steps) + 1):
        # the reference keeps the GENERATOR utils/modules.detach_clone_named_parameters returns
        # (deblur_e_nerf.py:887) and consumes it only in the check below, i.e. after the step: the
        # parameter half of its early stop compares the updated parameters with themselves, so the
        # stop rests on the errors alone.  Kept lazy here so the step count is the reference's.
        prev = mod.detach_clone_named_parameters(model)
        errors.append(float(optimizer.step(input=pred, target=tgt)) / n)
        if (torch.allclose(torch.tensor(errors[-1], dtype=torch.float64), torch.tensor(errors[-2], dtype=torch.float64))
                and mod.named_parameters_allclose(model, prev)):
            break
    conv = {k: v.detach().clone() for k, v in model.named_parameters()}
    with torch.no_grad():
        out = model(pred).squeeze(-1)
    return EasyDict(pred=out, target=target, gamma=gamma * conv["gamma"][:, 0, 0, 0],
                    scale=scale.pow(conv["gamma"][:, 0, 0, 0]) * conv["scale"][:, 0, 0, 0],
                    offset=conv["offset"][:, 0, 0, 0], errors=torch.tensor(errors, dtype=torch.float64),
                    converged=(conv["scale"], conv["gamma"], conv["offset"]))


def flat_gradient_buffers(grads):
    """The gradients grouped for the all-reduce: {dtype: (flat buffer, [gradients])} -- one f64 buffer
    for the f64 parameters (the refractory period, event_generation_params.py:196-201) and one f32
    buffer for every other floating dtype (the MLP / hash table; a half-precision gradient is
    promoted, never summed across ranks in half precision), so no f32 gradient travels as f64.  The
    groups come in a fixed order (f32, then f64), independent of the order the dtypes first appear,
    so every rank issues the same collectives."""
    groups = {torch.float32: [], torch.float64: []}
    for g in grads:
        groups[torch.float64 if g.dtype == torch.float64 else torch.float32].append(g)
    return {dt: (torch.cat([g.reshape(-1).to(dt) for g in gs]), gs) for dt, gs in groups.items() if gs}


def allreduce_gradients(module):
    """DDP gradient semantics over the ranks of the default process group: the mean of each
    gradient, as one all-reduce per dtype of one flat buffer (RCCL over xGMI on the GPU box)."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return
    grads = [p.grad for p in module.parameters() if p.grad is not None]
    if not grads:
        return
    for flat, gs in flat_gradient_buffers(grads).values():
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.div_(dist.get_world_size())
        off = 0
        for g in gs:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n
