"""Oracle: event-generation model and event loss -- CPU PyTorch restatement
(test infrastructure, see oracle/__init__.py).

Reference semantics (deblur_e_nerf/..., file:line):
* contrast thresholds C- = 2 Cbar/(r+1), C+ = r C-   models/event_generation_params.py:86-118
* refractory delay start_ts += tau_r                models/event_generation_params.py:230-237
* diff / subdiff timestamps                         models/deblur_e_nerf.py:419-455
* Loss.compute / log_intensity_diff / _tv           loss_metric/loss.py:34-96
"""
import torch

ERROR_FNS = {
    "l1": lambda a, b: torch.nn.functional.l1_loss(a, b, reduction="none"),
    "mse": lambda a, b: torch.nn.functional.mse_loss(a, b, reduction="none"),
    "huber": lambda a, b: torch.nn.functional.huber_loss(a, b, reduction="none", delta=1.0),
    # utils/modules.py:97-122 MAPELoss: |a - b| / max(|b|, f64 eps)
    "mape": lambda a, b: torch.nn.functional.l1_loss(a, b, reduction="none") / b.abs().clamp(min=2.220446049250313e-16),
}


def contrast_log_intensity_diff(num_pos, num_neg, pos_ct, neg_ct):
    return num_pos * pos_ct - num_neg * neg_ct


def diff_timestamps(start_ts, end_ts, norm_ts_diff, norm_start):
    """(deblur_e_nerf.py:419-434) -> ts_diff, diff_start_ts, diff_end_ts (f64)."""
    ts_diff = (end_ts - start_ts) * norm_ts_diff
    s = torch.lerp(start_ts, torch.maximum(end_ts - ts_diff, start_ts), norm_start)
    e = torch.minimum(s + ts_diff, end_ts)
    return ts_diff, s, e


def event_loss(lid_meas, end_ts, start_ts, diff_lid, ts_diff, diff_valid,
               sub_lid, sub_valid, mean_ct, fn_diff="huber", fn_tv="l1",
               norm_diff=True, norm_tv=True):
    """-> (L_diff, L_tv) masked means (loss.py:34-96)."""
    grad = lid_meas / (end_ts - start_ts)
    cd = mean_ct if norm_diff else 1
    ct = mean_ct if norm_tv else 1
    err_d = ERROR_FNS[fn_diff](diff_lid / cd, (ts_diff * grad / cd).to(diff_lid.dtype))
    err_t = ERROR_FNS[fn_tv](sub_lid / ct, torch.zeros_like(sub_lid))
    return err_d[diff_valid].mean(), err_t[sub_valid].mean()
