"""Pixel-bandwidth sensor model -- MI355X-native mirror of the reference's
``deblur_e_nerf/models/pixel_bandwidth.py`` (PixelBandwidth, :7-494).

Same constructor ``(dataset_directory, min_ts, f_c_dominant_min,
target_cumprob)``, same parameters (softplus-parametrised
``tau_mil_it_eff_prod``, ``A_amp_inv``, ``A_loop_inv``, ``tau_out``,
``tau_sf``, ``tau_diff``; buffer ``tau_in_it_eff_prod``), same
``forward(normalized_interval_gen, output_ts, intensity_sampling_fn,
reset_diff=False) -> (log_intensity, auxiliary_output)`` and the same reset
state (``reset_delta_log_it``, ``reset_ts``) carried between calls.

Arithmetic: ``den_pixbw_sample_ts`` (sample timestamps) and
``den_pixbw_fwd`` / ``den_pixbw_bwd`` (linearisation, FOH discretisation,
weights, weighted log-sum, reset / decay), one thread per event in f64
(den_pixbw.hip).  The parameters' softplus parametrisation stays in PyTorch
(seven scalars).
"""
import math
import os

import numpy as np
import torch

from .. import _native
from ..utils import modules

CAMERA_CALIBRATION_FILENAME = "camera_calibration.npz"
# The reference asserts on device tensors inside forward (pixel_bandwidth.py:375, 440), which
# forces two host syncs per call.  The kernels do not need the checks; set True to run them.
CHECK_INPUTS = False


def load_camera_calibration(root_directory):
    """datasets.Event.load_camera_calibration (data/datasets.py:105-111): a plain
    .npz of arrays, read without unpickling."""
    return np.load(os.path.join(root_directory, CAMERA_CALIBRATION_FILENAME), allow_pickle=False)


class PixelBandwidth(torch.nn.Module):
    TAU_IN_IT_EFF_PROD_KEY = "input_time_const_eff_it_prod"
    TAU_MIL_IT_EFF_PROD_KEY = "miller_time_const_eff_it_prod"
    A_AMP_KEY = "amplifier_gain"
    A_CL_KEY = "closed_loop_gain"
    TAU_OUT_KEY = "output_time_const"
    F_C_SF_KEY = "sf_cutoff_freq"
    F_C_DIFF_KEY = "diff_amp_cutoff_freq"
    NS_TO_S = 1e-9
    PARAM_NAMES = ("tau_mil_it_eff_prod", "A_amp_inv", "A_loop_inv", "tau_out", "tau_sf", "tau_diff")

    def __init__(self, dataset_directory, min_ts, f_c_dominant_min, target_cumprob, calibration=None):
        """``calibration``: the camera_calibration.npz arrays as a dict, instead of
        reading them from ``dataset_directory``."""
        super().__init__()
        self.omega_c_dominant_min = 2 * math.pi * f_c_dominant_min  # rad/s
        min_ts = min_ts.detach().clone() if torch.is_tensor(min_ts) else torch.tensor(min_ts)
        self.register_buffer("min_ts", min_ts, persistent=False)
        self.register_buffer("target_cumprob_max_sample_lifetime",
                             torch.tensor(target_cumprob.max_sample_lifetime), persistent=False)

        calib = calibration if calibration is not None else load_camera_calibration(dataset_directory)
        k_in = torch.from_numpy(np.asarray(calib[self.TAU_IN_IT_EFF_PROD_KEY]))
        k_mil = torch.from_numpy(np.asarray(calib[self.TAU_MIL_IT_EFF_PROD_KEY]))
        a_amp = torch.from_numpy(np.asarray(calib[self.A_AMP_KEY]))
        a_cl = torch.from_numpy(np.asarray(calib[self.A_CL_KEY]))
        tau_out = torch.from_numpy(np.asarray(calib[self.TAU_OUT_KEY]))
        f_sf = torch.from_numpy(np.asarray(calib[self.F_C_SF_KEY]))
        f_diff = torch.from_numpy(np.asarray(calib[self.F_C_DIFF_KEY]))
        # pixel_bandwidth.py:113-144
        self.register_buffer("tau_in_it_eff_prod", k_in, persistent=False)
        self.tau_mil_it_eff_prod = torch.nn.parameter.Parameter(k_mil)
        self.A_amp_inv = torch.nn.parameter.Parameter(1 / a_amp)
        self.A_loop_inv = torch.nn.parameter.Parameter(a_cl / a_amp)
        self.tau_out = torch.nn.parameter.Parameter(tau_out)
        self.tau_sf = torch.nn.parameter.Parameter(1 / (2 * math.pi * f_sf))
        self.tau_diff = torch.nn.parameter.Parameter(1 / (2 * math.pi * f_diff))
        softplus = modules.Softplus(beta=1)
        for name in self.PARAM_NAMES:
            torch.nn.utils.parametrize.register_parametrization(self, name, softplus)
        self.register_buffer("linearized_sys_C", torch.tensor([[0, 0, 1, 0], [0, 0, 0, 1]],
                                                              dtype=torch.get_default_dtype()), persistent=False)
        self.register_buffer("linearized_sys_D", torch.zeros(2, 1), persistent=False)
        self.reset_delta_log_it = None
        self.reset_ts = None

    @property
    def A_amp(self):
        return 1 / self.A_amp_inv

    @property
    def A_loop(self):
        return 1 / self.A_loop_inv

    @property
    def omega_c_sf(self):
        return 1 / self.tau_sf

    @property
    def omega_c_diff(self):
        return 1 / self.tau_diff

    def params_vector(self):
        """The 7 model constants in den_pixbw order, post-parametrisation."""
        return torch.stack([self.tau_in_it_eff_prod.to(torch.float32), self.tau_mil_it_eff_prod,
                            self.A_amp_inv, self.A_loop_inv, self.tau_out, self.tau_sf, self.tau_diff])

    @torch.no_grad()
    def sample_intensity(self, normalized_interval_gen, output_ts, intensity_sampling_fn):
        """pixel_bandwidth.py:298-367: sample timestamps (den_pixbw_sample_ts; like the reference's
        ``output_ts - sample_lifetime`` they are differentiable in output_ts only), then the
        intensity at the timestamps clamped to min_ts (with gradients enabled)."""
        with torch.enable_grad():
            sample_ts = _native.pixbw_sample_ts(normalized_interval_gen, output_ts, self.omega_c_dominant_min,
                                                float(self.target_cumprob_max_sample_lifetime))
            sampling_output = intensity_sampling_fn(sample_ts.clamp(min=self.min_ts))
        return sampling_output[0], sample_ts, sampling_output[1:]

    def forward(self, normalized_interval_gen, output_ts, intensity_sampling_fn, reset_diff=False):
        intensity_sample, sample_ts, auxiliary_output = self.sample_intensity(
            normalized_interval_gen, output_ts, intensity_sampling_fn)
        # intensity_sample_to_weight (:375) -- a host sync, so only when CHECK_INPUTS is set
        if CHECK_INPUTS:
            assert torch.all(sample_ts.diff(dim=0).to(torch.float32) > 0)
        params = self.params_vector()
        if reset_diff:
            out, delta = _native.PixelBandwidthFunction.apply(intensity_sample, params, None, sample_ts, output_ts,
                                                              None, True)
            self.reset_delta_log_it = delta
            self.reset_ts = output_ts
        else:
            if self.reset_delta_log_it is None:
                raise RuntimeError("PixelBandwidth: a reset_diff=True call must precede (pixel_bandwidth.py:436-440)")
            if CHECK_INPUTS:  # pixel_bandwidth.py:440 (a host sync)
                assert torch.all((output_ts - self.reset_ts) >= 0)
            out, _ = _native.PixelBandwidthFunction.apply(intensity_sample, params, self.reset_delta_log_it,
                                                          sample_ts, output_ts, self.reset_ts, False)
        return out, auxiliary_output
