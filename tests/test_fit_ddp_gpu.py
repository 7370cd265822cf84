"""configs[3]/[4]'s composed DDP path on the product, world 2 (scripts/run.py:84-100: PL's DDP with
broadcast_buffers; deblur_e_nerf.py:465 grid update, :1269-1272 all-gathered batch size).

Two processes on the box's GPU (gloo: RCCL does not run two ranks on one device; the driver's 8-GPU
bench uses RCCL) run ``DeblurENeRF.fit_step`` with step_ziggy_rd1's model composition (ngp field,
unbounded-sphere contraction, cone-angle marching, pixel bandwidth S = 30 with learnable sensor
parameters, learnable C+/C- and tau_r, TV 0.1), each on its own event batches and its own random
draws (occupancy cell jitter, cone cameras, marching jitter):

* step 0 updates each rank's occupancy grid with its own draws; step 1 starts with rank 0's grid
  broadcast (fit_step's sync_grid), so after 3 steps every parameter and the occs / binary grid
  are bit-identical on both ranks;
* both ranks set the same next batch size from the all-gathered mean samples per ray;
* step 1's all-reduced gradient equals ONE process's training_step on the two ranks' events
  concatenated, with rank 0's grid and the step-1 parameters: the mean of per-rank means is the
  global mean (every event valid, equal shards).  Marching jitter is pinned to 0.5 in step 1 on
  both sides so the samples agree; the bound is max(1e-4, 4 x our own f32 summation-order noise,
  measured by the same single-process step with the events in two other orders; for the mean
  contrast threshold, whose gradient cancels against the loss normaliser's, 4 f32 roundoffs times
  that condition number) -- the noise floor of each quantity, as tests/test_deblur_gpu.py floors the
  reference comparisons.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
N_EV, WORLD, STEPS, S = 16, 2, 3, 30
BOUND_MAX = 0.1
EPS32 = 2.0 ** -24
MEAN_C = "contrast_threshold.parametrizations.mean_contrast_threshold.original"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(step, rank, n=N_EV):
    from test_deblur_gpu import _event_batch
    b = _event_batch(n, seed=500 + 10 * step + rank)
    b["normalized"]["interval_gen"] = torch.full((1, S - 1, n), 0.5, dtype=torch.float64)
    return b


def _to_dev(b):
    return {g: {k: v.to("cuda") for k, v in d.items()} for g, d in b.items()}


def _cat(b0, b1):
    """Two reference-shaped batches as one: events (1, N, ...) along dim 1, normalized samples along
    their last (event) dim."""
    out = {"event": {k: torch.cat([b0["event"][k], b1["event"][k]], dim=1) for k in b0["event"]},
           "normalized": {k: torch.cat([b0["normalized"][k], b1["normalized"][k]], dim=-1)
                          for k in b0["normalized"]}}
    return out


def _permute(b, seed=7):
    """The same events in another (seeded random) order: every sum over events runs differently."""
    n = b["event"]["end_ts"].shape[1]
    p = torch.randperm(n, generator=torch.Generator().manual_seed(seed))
    return {"event": {k: v[:, p] for k, v in b["event"].items()},
            "normalized": {k: v[..., p] for k, v in b["normalized"].items()}}


def _const_jitter(*size, device=None):
    return torch.full(size, 0.5, device=device)


class _RecOpt:
    """The optimizer fit_step drives, recording the (all-reduced) gradients it is handed."""

    def __init__(self, opt, m):
        self.opt, self.m, self.grads = opt, m, []

    def step(self):
        self.grads.append({k: p.grad.detach().cpu().clone() for k, p in self.m.named_parameters()
                           if p.grad is not None})
        self.opt.step()

    def zero_grad(self, set_to_none=True):
        self.opt.zero_grad(set_to_none=set_to_none)


def _state(m):
    return {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}


def _worker(rank, world, port, out, golden):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deblur_e_nerf.external import marching
    from test_deblur_gpu import build_model
    z = np.load(os.path.join(golden, "step_ziggy_rd1.npz"))
    torch.manual_seed(1000 + rank)  # per-rank draws, as each DDP process seeds its own
    m = build_model(z)
    m.train()
    opt = _RecOpt(m.configure_optimizers()["optimizer"], m)
    sizes, state1 = [], None
    for k in range(STEPS):
        if k == 1:
            marching._uniform = _const_jitter
        b = _to_dev(_batch(k, rank))
        if k == 1:
            # the step-1 parameters (identical on both ranks after step 0's averaged update); the grid
            # is broadcast inside fit_step, so record it after the step
            state1 = _state(m)
        m.fit_step(b, k, opt)
        torch.cuda.synchronize()
        sizes.append(int(m.train_batch_size))
        if k == 1:
            g = m.nerf.occupancy_grid
            state1["grid_occs"], state1["grid_binary"] = g.occs.detach().cpu().clone(), g.binary.detach().cpu().clone()
    g = m.nerf.occupancy_grid
    out[rank] = dict(state=_state(m), occs=g.occs.detach().cpu().clone(), binary=g.binary.detach().cpu().clone(),
                     sizes=sizes, grads1=opt.grads[1], state1=state1)
    dist.destroy_process_group()


def _single_step_grads(golden, state1, batch):
    """One process: the step-1 parameters, rank 0's grid, training_step on `batch` -> (gradients,
    the condition number of the mean-C gradient)."""
    from deblur_e_nerf.external import marching
    from test_deblur_gpu import _GradTap, build_model
    z = np.load(os.path.join(golden, "step_ziggy_rd1.npz"))
    m = build_model(z)
    m.train()
    sd = {k: v for k, v in state1.items() if not k.startswith("grid_")}
    m.load_state_dict(sd)
    g = m.nerf.occupancy_grid
    g.occs.copy_(state1["grid_occs"].to(g.occs.device))
    g._binary.copy_(state1["grid_binary"].to(g._binary.device))
    m._global_step = 1  # no grid update (every 16 steps)
    # the gradient of the loss's normalising constant (the mean contrast threshold handed to
    # Loss.compute): the term the mean-C gradient cancels against (its condition number)
    g_c = []
    comp = m.loss.compute

    def compute(ev, diff, sub, c):
        c = _GradTap.apply(c, lambda g: g_c.append(float(g.detach().sum())))
        return comp(ev, diff, sub, c)
    m.loss.compute = compute
    old = marching._uniform
    marching._uniform = _const_jitter
    try:
        loss = m.training_step(_to_dev(batch), 1)
        loss.backward()
    finally:
        marching._uniform = old
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters() if p.grad is not None}
    orig = m.contrast_threshold.parametrizations.mean_contrast_threshold.original
    with torch.enable_grad():
        fprime = float(torch.autograd.grad(m.contrast_threshold.mean_contrast_threshold.sum(), orig)[0])
    d_mean = abs(float(grads[MEAN_C].sum())) / abs(fprime)
    return grads, abs(sum(g_c)) / d_mean


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


@pytest.mark.timeout(600)
def test_fit_step_ddp_composed_ziggy(golden_dir):
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_worker, args=(WORLD, _free_port(), out, golden_dir), nprocs=WORLD, join=True,
                       start_method="spawn")
    r0, r1 = out[0], out[1]
    # bit-identical model state (parameters, occupancy grid, every buffer) after 3 steps
    for k in r0["state"]:
        assert torch.equal(r0["state"][k], r1["state"][k]), k
    assert torch.equal(r0["occs"], r1["occs"]) and torch.equal(r0["binary"], r1["binary"])
    assert r0["sizes"] == r1["sizes"], (r0["sizes"], r1["sizes"])
    print(f"  both ranks: next batch sizes {r0['sizes']}; state bit-identical after {STEPS} steps")
    # step 1's averaged gradient vs one process on the concatenated events
    assert torch.equal(r0["state1"]["grid_occs"], r1["state1"]["grid_occs"])
    full = _cat(_batch(1, 0), _batch(1, 1))
    g_one, cond_c = _single_step_grads(golden_dir, r0["state1"], full)
    g_perm = [_single_step_grads(golden_dir, r0["state1"], _permute(full, s))[0] for s in (7, 8)]
    # the split the ranks compute, in one process: each half's gradient (rank r's events, the same
    # state), averaged -- what the all-reduce must reproduce; its distance to the full batch is f32
    # arithmetic (a cancelling sum rounded per half, e.g. the ngp head's scalar output bias), not DDP
    g_half = [_single_step_grads(golden_dir, r0["state1"], _batch(1, r))[0] for r in (0, 1)]
    ga = r0["grads1"]
    assert set(ga) == set(g_one), (set(ga) ^ set(g_one))
    worst, bad = 0.0, []
    for k in sorted(ga):
        e = _rel(ga[k], g_one[k])
        noise = max(_rel(gp[k], g_one[k]) for gp in g_perm)
        if k == MEAN_C:  # two terms ~cond x their sum: each rank's f32 loss rounding, amplified
            noise = max(noise, EPS32 * cond_c)
        split = (g_half[0][k].double() + g_half[1][k].double()) / 2
        e_split = _rel(ga[k], split)  # the DDP composition itself: 2 ranks vs their halves in 1 process
        split_noise = _rel(split, g_one[k])
        bound = max(1e-4, 4.0 * max(noise, split_noise))
        print(f"  {k:70s} 2-rank vs 1-process {e:.2e} (order noise {noise:.1e}, split {split_noise:.1e}, "
              f"bound {bound:.1e}); vs the halves {e_split:.1e}")
        if e > bound:
            bad.append((k, e, bound))
        if e_split > max(1e-4, 4.0 * noise):
            bad.append((k + " [halves]", e_split, max(1e-4, 4.0 * noise)))
        if bound <= BOUND_MAX:
            worst = max(worst, e)
    print(f"  worst well-conditioned tensor: {worst:.2e}")
    assert not bad, bad
