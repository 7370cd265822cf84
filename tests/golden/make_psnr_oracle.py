"""psnr_oracle_converged.npz -- the converged-PSNR anchor of bench.py's ``psnr.converged`` leg:
the ORACLE (oracle/, the CPU PyTorch restatement of the reference path, parity-pinned by tests/)
trained exactly as the leg trains the HIP TrainStep -- the same student init, the same teacher,
the same batch sequence (bench._teacher_batch on a CPU generator seeded PSNR_LEG["batch_seed"]),
torch.optim.Adam with the reference's groups (L2 1e-6 on the MLP, none on the background), the
lr cut x0.3 at the milestones -- then scored on the four held-out views with the reference's
affine log-intensity correction + PSNR.  Test infrastructure (runs hours on the build container's
CPUs; resumable from a checkpoint under /tmp):

    python tests/golden/make_psnr_oracle.py [--threads 6] [--steps 2000]

The fixture holds the oracle's PSNR, its four renders and the teacher's (64 x 64 each), the
loss trajectory, and the setup; bench.py reports HIP F32 / BF16 ΔPSNR against it.
"""
import argparse
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


def student_init(rd):
    """TrainStep(seed=student_seed)'s initial parameters (deblur_e_nerf/train.py: the mirror's
    VanillaNeRFRadianceField under torch.manual_seed) and background raw value."""
    from deblur_e_nerf.external import mlp, ngp
    torch.manual_seed(bench.PSNR_LEG["student_seed"])
    field = mlp.VanillaNeRFRadianceField([-1.5, -1.5, -1.5, 1.5, 1.5, 1.5], radiance_dim=rd,
                                         hidden_activation=torch.nn.Softplus(beta=100),
                                         density_activation=ngp.shifted_trunc_exp,
                                         radiance_activation=torch.nn.Softplus(beta=1), mode="f32")
    return field.flat_params.detach().clone(), torch.full((rd,), math.log(math.expm1(1.0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--steps", type=int, default=bench.PSNR_LEG["steps"])
    ap.add_argument("--rd", type=int, default=1)
    ap.add_argument("--ckpt", default="/tmp/psnr_oracle_ckpt.pt")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    L = bench.PSNR_LEG
    rd, n_events, n_samples, view = a.rd, L["n_events"], L["n_samples"], L["view"]
    teacher = {k: v.clone() for k, v in unflat(bench.teacher_field(rd), rd).items()}
    ones = torch.ones(rd)
    flat0, bk0 = student_init(rd)
    p = {k: v.clone().requires_grad_(True) for k, v in unflat(flat0, rd).items()}
    bk = bk0.clone().requires_grad_(True)
    names = [n for n, _, _ in onerf.layer_specs(rd)]
    leaves = [p[n + s] for n in names for s in (".weight", ".bias")]
    lr0 = 0.01  # TrainStep's default
    opt = torch.optim.Adam([{"params": leaves, "weight_decay": 1e-6}, {"params": [bk], "weight_decay": 0.0}], lr=lr0)
    gen = torch.Generator().manual_seed(L["batch_seed"])
    start, losses = 0, []
    if os.path.exists(a.ckpt):
        ck = torch.load(a.ckpt, weights_only=False)  # this script's own checkpoint
        for t, v in zip(leaves + [bk], ck["params"]):
            t.data.copy_(v)
        opt.load_state_dict(ck["opt"])
        gen.set_state(ck["gen"])
        start, losses = ck["step"], ck["losses"]
        print(f"resumed at step {start}", flush=True)
    t0 = time.time()
    for it in range(start, a.steps):
        for g in opt.param_groups:
            g["lr"] = bench.lr_at(lr0, it, a.steps, L["milestones"])
        b = bench._teacher_batch(gen, n_events)
        with torch.no_grad():
            col, _, _, _ = onerf.render_rays(teacher, b["rays_o"], b["rays_d"], b["jitter"], n_samples=n_samples,
                                             bkgd=ones)
        y = torch.log(col[:, 0] + 1e-3).view(4, n_events)
        b["lid"] = (y[1] - y[0]).float().contiguous()
        opt.zero_grad()
        total, Ld, Lt = step_loss(p, torch.nn.functional.softplus(bk), b, n_samples)
        total.backward()
        opt.step()
        if it % 10 == 0 or it == a.steps - 1:
            losses.append((it, float(Ld), float(Lt), float(total)))
        if (it + 1) % 50 == 0 or it == a.steps - 1:
            torch.save({"params": [t.detach().clone() for t in leaves + [bk]], "opt": opt.state_dict(),
                        "gen": gen.get_state(), "step": it + 1, "losses": losses}, a.ckpt)
            el = time.time() - t0
            print(f"step {it + 1}/{a.steps}  loss {float(total):.6f}  {el / (it + 1 - start):.2f} s/step", flush=True)
    vo, vd, nv = bench.psnr_views(view)
    vu = torch.full((vo.shape[0],), 0.5)
    with torch.no_grad():
        target, _, _, _ = onerf.render_rays(teacher, vo, vd, vu, n_samples=n_samples, bkgd=ones)
        pred, _, _, _ = onerf.render_rays(p, vo, vd, vu, n_samples=n_samples, bkgd=torch.nn.functional.softplus(bk))
    ps, ps_raw, gamma, scale = bench.aligned_psnr(pred, target, nv, view)
    print(f"oracle converged: PSNR {ps:.3f} dB (uncorrected {ps_raw:.3f}), gamma {gamma:.4f}, scale {scale:.4f}")
    out = os.path.join(HERE, "psnr_oracle_converged.npz")
    np.savez_compressed(out, psnr_db=np.array(ps), psnr_uncorrected_db=np.array(ps_raw), gamma=np.array(gamma),
                        scale=np.array(scale), pred=pred[:, 0].reshape(nv, view, view).numpy().astype(np.float32),
                        target=target[:, 0].reshape(nv, view, view).numpy().astype(np.float32),
                        losses=np.array(losses, dtype=np.float64), steps=np.array(a.steps), rd=np.array(rd),
                        setup=np.array(repr(dict(L, steps=a.steps, lr0=lr0))))
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
