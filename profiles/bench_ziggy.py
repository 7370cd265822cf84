"""Per-rank emulation of BASELINE configs[3] (configs/train/07_ziggy_and_fuzz_hdr.yaml, 4 GPUs,
2^20-ray effective batch) on one MI355X, through the drop-in operator API: DeblurENeRF.fit_step
with the yaml's model section -- ngp field (16 x 2^19 HashGrid, 64-wide MLPs), unbounded sphere
contraction, 256^3 occupancy grid, cone-angle marching, the pixel-bandwidth model on (S = 30)
with learnable sensor parameters, learnable C+/C- and refractory period, TV weight 0.1 -- with
the per-rank batch of gpus = [0, 1, 2, 3] (32,768 ray samples per render call), gradient
accumulation 8 and the dynamic event batch (update_train_batch_size).

Data is synthetic (the EDS sequence is not in this image): EDS-assumed sensor constants, a camera
circling the yaml's AABB, random events.  The field starts from random init, so the numbers are
the cost of the steps a training run starts with.  Prints one JSON line.

    python profiles/bench_ziggy.py [--opt-steps 3] [--warmup 1]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deblur-e-nerf_amd"))

import torch  # noqa: E402

# EDS-assumed DVS constants (reference scripts/eds_to_esim.py:68-79)
EDS = dict(input_time_const_eff_it_prod=(35e-12 * 25e-3) / 2000e-12,
           miller_time_const_eff_it_prod=(0.6e-12 * 25e-3) / 2000e-12, amplifier_gain=140.0,
           closed_loop_gain=1 / 0.7, output_time_const=25e-6, sf_cutoff_freq=16400.0, diff_amp_cutoff_freq=82000.0)
AABB = [0.2, -0.4, 0.0, 3.7, 3.7, 1.8]
IMG = (480, 640)


def dataset_dir(C=128):
    from scipy.spatial.transform import Rotation
    d = tempfile.mkdtemp(prefix="den_ziggy_")
    K = np.array([[560.0, 0.0, 320.0], [0.0, 560.0, 240.0], [0.0, 0.0, 1.0]], dtype=np.float32)
    cal = {k: np.array(v, dtype=np.float32) for k, v in EDS.items()}
    cal.update(pos_contrast_threshold=np.array(0.25, np.float32), neg_contrast_threshold=np.array(0.2, np.float32),
               refractory_period=np.array(1000, np.int64), intrinsics=K, bayer_pattern=np.array(""),
               img_height=np.array(IMG[0]), img_width=np.array(IMG[1]))
    ts = np.linspace(5e7, 2.05e9, C).astype(np.int64)
    c = np.array([(AABB[0] + AABB[3]) / 2, (AABB[1] + AABB[4]) / 2, (AABB[2] + AABB[5]) / 2])
    ang = np.linspace(0.0, 2.0, C)
    pos = np.stack([c[0] + 1.2 * np.cos(ang), c[1] + 1.2 * np.sin(ang), c[2] + 0.1 * np.sin(3 * ang)], -1)
    rots = []
    for p in pos:
        z = (c + np.array([0.0, 0.0, 0.3]) - p)
        z /= np.linalg.norm(z)
        x = np.cross(z, [0.0, 0.0, 1.0])
        x /= np.linalg.norm(x)
        rots.append(np.stack([x, np.cross(z, x), z], -1))
    quat = Rotation.from_matrix(np.stack(rots)).as_quat().astype(np.float32)
    np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
    np.savez(os.path.join(d, "camera_poses.npz"), T_wc_position=pos.astype(np.float32), T_wc_orientation=quat,
             T_wc_timestamp=ts)
    torch.save(torch.tensor(1_000_000), os.path.join(d, "max_refractory_period.pt"))
    return d


def event_batch(N, S, g, dev):
    """A reference-shaped batch (datamodule.py:215-247) of N events."""
    num_pos = (torch.rand(N, generator=g) < 0.5).long()
    end_ts = (torch.rand(N, generator=g, dtype=torch.float64) * 1.7e9 + 2e8).long()
    start_ts = end_ts - (-torch.log(torch.rand(N, generator=g, dtype=torch.float64)) * 2e6 + 2e4).long()
    position = torch.rand(N, 2, generator=g) * torch.tensor([IMG[1] - 1.0, IMG[0] - 1.0])
    u = torch.rand(3, N, generator=g, dtype=torch.float64)
    ev = dict(position=position[None], start_ts=start_ts[None], end_ts=end_ts[None], num_pos=num_pos[None],
              num_neg=(1 - num_pos)[None])
    nz = dict(ts_diff=torch.ones(1, N, dtype=torch.float64), diff_start_ts=u[0][None],
              ts_subdiff=(1 - torch.sqrt(1 - u[1]))[None], subdiff_start_ts=u[2][None],
              interval_gen=torch.full((1, S - 1, N), 0.5, dtype=torch.float64))
    to = lambda t: t.to(dev)  # noqa: E731
    return {"event": {k: to(v) for k, v in ev.items()}, "normalized": {k: to(v) for k, v in nz.items()}}


def build(d, gpus, acc, S):
    from deblur_e_nerf.models.deblur_e_nerf import DeblurENeRF, _TrainerStub
    from deblur_e_nerf.utils.easydict import EasyDict as ED
    ngp = ED(pos_encoding=ED(otype="HashGrid", n_levels=16, n_features_per_level=2, log2_hashmap_size=19,
                             base_resolution=16, per_level_scale=1.4472692012786865, interpolation="Linear"),
             dir_encoding=ED(degree=4),
             mlp_base=ED(hidden_activation="softplus", density_activation="shifted_trunc_exp", n_neurons=64,
                         n_hidden_layers=1, geo_feat_dim=15, weight_norm=False),
             mlp_head=ED(hidden_activation="softplus", radiance_activation="softplus", n_neurons=64,
                         n_hidden_layers=2, weight_norm=False))
    nerf = ED(aabb=AABB, contraction_type="sphere",
              occ_grid=ED(resolution=256, occ_thre=1e-2, ema_decay=0.95, warmup_steps=256, n=16),
              near_plane=0.01, far_plane=13.0, render_step_size="auto", cone_angle=0.004, early_stop_eps=1e-4,
              alpha_thre=0.0, test_chunk_size=16384, arch="ngp", ngp=ngp, load_state_dict=False, freeze=False)
    pb_free = ED(tau_mil_it_eff_prod=False, A_amp_inv=False, A_loop_inv=False, tau_out=False, tau_sf=False,
                 tau_diff=False, default=False)
    m = DeblurENeRF(
        "bench", ["event_view"], 1, gpus, 0.001, False, None,
        ED(parameterize_mean_ct=True, load_state_dict=False,
           freeze=ED(p2n_contrast_threshold_ratio=False, mean_contrast_threshold=False, default=False)),
        ED(load_state_dict=False, freeze=False),
        ED(enable=True, it_sample_size=S, f_c_dominant_min=21, target_cumprob=ED(max_sample_lifetime=0.95),
           load_state_dict=False, freeze=pb_free),
        nerf, ED(per_channel_log_it_scale=False, black_level_offset=True),
        ED(weight=ED(log_intensity_diff=1.0, log_intensity_tv=0.1, nerf_mlp_weight_decay=1e-6),
           error_fn=ED(log_intensity_diff="huber", log_intensity_tv="l1"),
           normalize=ED(log_intensity_diff=True, log_intensity_tv=True)),
        ED(lpips_net="alex"),
        # the yaml's optimizer section
        ED(algo="adam", lr=ED(default=0.01, contrast_threshold=ED(p2n_contrast_threshold_ratio=0.1,
                                                                 mean_contrast_threshold=0.1),
                              pixel_bandwidth=ED(tau_mil_it_eff_prod=0.01, A_amp_inv=0.01, A_loop_inv=0.01,
                                                 tau_out=0.01, tau_sf=0.01, tau_diff=0.01)),
           relative_lr=ED(refractory_period=50)),
        ED(algo="multi_step_lr", multi_step_lr=ED(milestones=[20, 30, 36], gamma=0.33), interval="epoch"),
        d, False, 131072)
    m.trainer = _TrainerStub(accumulate_grad_batches=acc)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt-steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--acc", type=int, default=8)
    ap.add_argument("--it-samples", type=int, default=30)
    ap.add_argument("--ranks", type=int, default=4, help="per-rank share of the yaml's effective batch")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    m = build(dataset_dir(), list(range(a.ranks)), a.acc, a.it_samples).to(dev)
    m.train()
    opt = m.configure_optimizers()["optimizer"]
    g = torch.Generator().manual_seed(1)
    N = 256 // a.ranks  # train_init_eff_batch_size // gpus (datamodule.py:75)
    rays = samples = 0
    bi = 0
    t0 = None
    for step in range(a.warmup + a.opt_steps):
        if step == a.warmup:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rays = samples = 0
        for _ in range(a.acc):
            loss = m.fit_step(event_batch(N, a.it_samples, g, dev), bi, opt)
            mspr = float(m.logged.get("train/mean_num_samples_per_ray", 0.0))
            rays += 4 * a.it_samples * N
            samples += 4 * a.it_samples * N * mspr
            bi += 1
            N = int(getattr(m, "train_batch_size", N))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({
        "what": "configs[3] per-rank emulation (07_ziggy_and_fuzz_hdr.yaml model section, gpus=4 share) via "
                "DeblurENeRF.fit_step, synthetic data, random-init field",
        "opt_steps": a.opt_steps, "micro_batches_per_opt_step": a.acc, "s_per_opt_step": round(dt / a.opt_steps, 4),
        "rays_per_s": round(rays / dt, 1), "samples_per_s": round(samples / dt, 1),
        "mean_samples_per_ray_last": round(mspr, 2), "events_per_micro_batch_last": N, "it_sample_size": a.it_samples,
        "loss_last": round(float(loss), 6)}), flush=True)


if __name__ == "__main__":
    main()
