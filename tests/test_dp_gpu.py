"""Data-parallel train step with the PRODUCT's per-rank gradients (libden.so on the GPU), world 2.

Two processes on the box's one GPU each run TrainStep on their shard of the events (the
sharding bench.py uses) and average the flat gradient buffer with the product's one
all-reduce (`train.allreduce_mean`; gloo here: RCCL does not run two ranks on one device, the
8-GPU driver bench uses RCCL).  The result must equal the full-batch TrainStep gradient computed in
one process -- the reference's DDP semantics (scripts/run.py:84-89: mean of per-shard means, equal to
the global mean when every event is valid, i.e. with the render background on).  F32 parity mode,
so the identity holds to f32 rounding.  Needs an MI355X (marked gpu).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from _util import norm_rel

pytestmark = pytest.mark.gpu
N_PER_RANK, WORLD, SEED = 48, 2, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deblur_e_nerf.train import TrainStep, allreduce_mean, synthetic_batch
    ts = TrainStep(N_PER_RANK, n_samples=128, radiance_dim=1, mode="f32", device="cuda", seed=SEED)
    ts.load_batch(**synthetic_batch(N_PER_RANK, seed=SEED, rank=rank, world=world))
    ts.forward()
    ts.backward()
    allreduce_mean(ts.gbuf)
    torch.cuda.synchronize()
    out[rank] = ts.gbuf.detach().cpu().clone()
    dist.destroy_process_group()


def test_two_rank_hip_gradient_equals_full_batch():
    from deblur_e_nerf.train import TrainStep, synthetic_batch
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_worker, args=(WORLD, _free_port(), out), nprocs=WORLD, join=True, start_method="spawn")
    full = TrainStep(N_PER_RANK * WORLD, n_samples=128, radiance_dim=1, mode="f32", device="cuda", seed=SEED)
    full.load_batch(**synthetic_batch(N_PER_RANK * WORLD, seed=SEED))
    full.forward()
    full.backward()
    torch.cuda.synchronize()
    g_full = full.gbuf.detach().cpu()
    assert torch.equal(out[0], out[1])  # every rank holds the same averaged buffer
    e = norm_rel(out[0].double(), g_full.double())
    print(f"2-rank all-reduced HIP gradient vs full batch: {e:.2e}")
    assert e <= 1e-5
