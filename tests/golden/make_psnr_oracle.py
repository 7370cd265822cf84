"""psnr_oracle_s<k>.npz -- the reference side of bench.py's converged-PSNR leg (``psnr_long``):
the ORACLE (oracle/, the CPU PyTorch restatement of the reference path, parity-pinned by tests/)
trained exactly as the leg trains the HIP TrainStep on batch sequence k -- the same student init,
the same teacher, the same batches (bench._teacher_batch on a CPU generator seeded
PSNR_LEG["batch_seed"] + k), torch.optim.Adam with the reference's groups (L2 1e-6 on the MLP, none
on the background), the lr cut x lr_gamma at the milestones -- then rendered on the held-out views
and scored with the reference's affine log-intensity correction + PSNR (metric.py:68-72).

Test infrastructure, run in the build container (about 1 s per step on 6 threads; resumable from
a checkpoint under /tmp, which also keeps the trained parameters so the views can be re-rendered
with --render-only):

    python tests/golden/make_psnr_oracle.py --seq 0 [--threads 6]

The fixture holds the leg it was trained on (bench.py ignores a fixture of another leg), the
oracle's PSNR, its renders and the teacher's, and the loss trajectory.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "deblur-e-nerf_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import bench  # noqa: E402
from _util import unflat  # noqa: E402
from oracle import nerf as onerf  # noqa: E402
from oracle.train import step_loss  # noqa: E402

TRAIN_KEYS = ("steps", "n_events", "n_samples", "milestones", "lr_gamma", "lr0", "teacher_sigma_bias",
              "teacher_rgb_scale", "batch_seed", "teacher_seed", "student_seed")


def student_init(rd, leg):
    """TrainStep(seed=student_seed)'s initial parameters (deblur_e_nerf/train.py: the mirror's
    VanillaNeRFRadianceField under torch.manual_seed) and background raw value."""
    from deblur_e_nerf.external import mlp, ngp
    torch.manual_seed(leg["student_seed"])
    field = mlp.VanillaNeRFRadianceField([-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], radiance_dim=rd,
                                         hidden_activation=torch.nn.Softplus(beta=100),
                                         density_activation=ngp.shifted_trunc_exp,
                                         radiance_activation=torch.nn.Softplus(beta=1), mode="f32")
    return field.flat_params.detach().clone(), torch.full((rd,), math.log(math.expm1(1.0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--rd", type=int, default=1)
    ap.add_argument("--ckpt", default=None)
    ap.add_argument("--render-only", action="store_true", help="re-render the views from a finished checkpoint")
    ap.add_argument("--device", default="cpu",
                    help="where torch executes the oracle: cpu (the build container), or cuda -- torch's own GPU "
                         "kernels (rocBLAS / hipBLASLt GEMMs, elementwise ops), never libden -- for the many "
                         "sequences of the oracle's own seed study")
    ap.add_argument("--out-dir", default=None,
                    help="fixture directory (default tests/golden, tests/golden/psnr_oracle_gpu for --device cuda)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    if a.device != "cpu":
        torch.backends.cuda.matmul.allow_tf32 = False  # the oracle is f32 arithmetic
        torch.backends.cudnn.allow_tf32 = False
        torch.set_default_device(a.device)
    L = dict(bench.PSNR_LEG)
    train_cfg = json.dumps({k: L[k] for k in TRAIN_KEYS}, sort_keys=True)
    ckpt = a.ckpt or (f"/tmp/psnr_oracle_s{a.seq}.pt" if a.device == "cpu" else f"/tmp/psnr_oracle_{a.device}_s{a.seq}.pt")
    rd, n_events, n_samples, steps = a.rd, L["n_events"], L["n_samples"], L["steps"]
    with torch.device("cpu"):
        tflat = bench.teacher_field(rd, L)
        flat0, bk0 = student_init(rd, L)
    teacher = {k: v.clone().to(a.device) for k, v in unflat(tflat.to(a.device), rd).items()}
    ones = torch.ones(rd)
    flat0, bk0 = flat0.to(a.device), bk0.to(a.device)
    p = {k: v.clone().requires_grad_(True) for k, v in unflat(flat0, rd).items()}
    bk = bk0.clone().requires_grad_(True)
    names = [n for n, _, _ in onerf.layer_specs(rd)]
    leaves = [p[n + s] for n in names for s in (".weight", ".bias")]
    opt = torch.optim.Adam([{"params": leaves, "weight_decay": 1e-6}, {"params": [bk], "weight_decay": 0.0}],
                           lr=L["lr0"])
    gen = torch.Generator(device="cpu").manual_seed(L["batch_seed"] + a.seq)
    start, losses, threads = 0, [], a.threads
    if os.path.exists(ckpt):
        ck = torch.load(ckpt, weights_only=False, map_location=a.device)  # this script's own checkpoint
        if ck["train_cfg"] != train_cfg:
            raise SystemExit(f"{ckpt} was trained on another leg: {ck['train_cfg']}")
        for t, v in zip(leaves + [bk], ck["params"]):
            t.data.copy_(v)
        opt.load_state_dict(ck["opt"])
        gen.set_state(ck["gen"].cpu())
        start, losses, threads = ck["step"], ck["losses"], ck.get("threads", a.threads)
        print(f"resumed at step {start}", flush=True)
    elif a.render_only:
        raise SystemExit(f"--render-only: no checkpoint {ckpt}")
    t0 = time.time()
    for it in range(start, steps):
        for g in opt.param_groups:
            g["lr"] = bench.lr_at(L["lr0"], it, steps, L["milestones"], L["lr_gamma"])
        with torch.device("cpu"):  # the CPU generator's draws, as the HIP leg's
            b = bench._teacher_batch(gen, n_events)
        b = {k: v.to(a.device) for k, v in b.items()}
        with torch.no_grad():
            col, _, _, _ = onerf.render_rays(teacher, b["rays_o"], b["rays_d"], b["jitter"], n_samples=n_samples,
                                             bkgd=ones)
        y = torch.log(col[:, 0] + 1e-3).view(4, n_events)
        b["lid"] = (y[1] - y[0]).float().contiguous()
        opt.zero_grad()
        total, Ld, Lt = step_loss(p, torch.nn.functional.softplus(bk), b, n_samples)
        total.backward()
        opt.step()
        if it % 10 == 0 or it == steps - 1:
            losses.append((it, float(Ld), float(Lt), float(total)))
        if (it + 1) % 50 == 0 or it == steps - 1:
            torch.save({"params": [t.detach().clone() for t in leaves + [bk]], "opt": opt.state_dict(),
                        "gen": gen.get_state(), "step": it + 1, "losses": losses, "train_cfg": train_cfg,
                        "threads": a.threads}, ckpt)
            el = time.time() - t0
            print(f"seq {a.seq} step {it + 1}/{steps}  loss {float(total):.6f}  {el / (it + 1 - start):.2f} s/step",
                  flush=True)
    view = L["view"]
    with torch.device("cpu"):
        vo, vd, nv = bench.psnr_views(view, L["n_views"])
    vo, vd = vo.to(a.device), vd.to(a.device)
    vu = torch.full((vo.shape[0],), 0.5)
    with torch.no_grad():
        target, _, _, _ = onerf.render_rays(teacher, vo, vd, vu, n_samples=n_samples, bkgd=ones)
        pred, _, _, _ = onerf.render_rays(p, vo, vd, vu, n_samples=n_samples, bkgd=torch.nn.functional.softplus(bk))
    pred, target = pred.cpu(), target.cpu()
    with torch.device("cpu"):
        ps, ps_raw, gamma, scale = bench.aligned_psnr(pred, target, nv, view)
    print(f"oracle seq {a.seq}: PSNR {ps:.4f} dB (uncorrected {ps_raw:.3f}), gamma {gamma:.4f}, scale {scale:.4f}")
    out = bench.oracle_fixture_path(a.seq, a.device) if a.out_dir is None else \
        os.path.join(a.out_dir, os.path.basename(bench.oracle_fixture_path(a.seq)))
    np.savez_compressed(out, psnr_db=np.array(ps), psnr_uncorrected_db=np.array(ps_raw), gamma=np.array(gamma),
                        scale=np.array(scale), pred=pred[:, 0].reshape(nv, view, view).numpy().astype(np.float32),
                        target=target[:, 0].reshape(nv, view, view).numpy().astype(np.float32),
                        losses=np.array(losses, dtype=np.float64), rd=np.array(rd), seq=np.array(a.seq),
                        threads=np.array(threads), device=np.array(a.device),
                        leg=np.array(json.dumps(L, sort_keys=True)))
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
