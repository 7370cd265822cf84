"""Oracle: event preparation and pixel rays -- CPU PyTorch restatement (test
infrastructure only, see oracle/__init__.py; pinned by tests/golden/events.npz
and rays.npz, which record the reference's own modules / code run here).

Reference semantics (deblur_e_nerf/..., file:line):
* ContrastThreshold.forward  lid = num_pos*C+ - num_neg*C-   models/event_generation_params.py:106-118
* RefractoryPeriod.forward   start_ts += tau_r               models/event_generation_params.py:230-237
* diff / subdiff timestamps                                  models/deblur_e_nerf.py:418-455
* NeRF.pixel_params_to_ray                                   models/nerf.py:206-228
"""
import torch

from .loss import contrast_log_intensity_diff, diff_timestamps


def event_prep(num_pos, num_neg, end_ts, start_ts, norm, pos_ct, neg_ct, tau_r, has_diff=True, has_tv=True):
    """Raw events (i64), normalized (4,N) f64 samples, C+/C- (f32 0-d), tau_r
    (f64 0-d) -> dict(lid, start_ts, diff=(ts_diff, s, e) | None, subdiff=... | None)."""
    lid = contrast_log_intensity_diff(num_pos, num_neg, pos_ct, neg_ct)
    start = start_ts + tau_r
    out = dict(lid=lid, start_ts=start, diff=None, subdiff=None)
    tv_s, tv_e = start, end_ts
    if has_diff:
        out["diff"] = diff_timestamps(start, end_ts, norm[0], norm[1])
        tv_s, tv_e = out["diff"][1], out["diff"][2]
    if has_tv:
        out["subdiff"] = diff_timestamps(tv_s, tv_e, norm[2], norm[3])
    return out


def pixel_params_to_ray(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation):
    hom = torch.cat((pixel_position, torch.ones_like(pixel_position[..., :1])), dim=-1).unsqueeze(-1)
    d = (T_wc_orientation @ (intrinsics_inverse @ hom)).squeeze(-1)
    d = d / torch.linalg.vector_norm(d, dim=-1, keepdim=True)
    return T_wc_position, d
