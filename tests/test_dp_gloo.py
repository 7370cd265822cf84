"""Data-parallel semantics of the train step, world_size 2 over gloo on CPU.

The GPU path shards the events of one step over the ranks
(`synthetic_batch(rank, world)`), computes per-rank gradients and averages them
with ONE all-reduce of the flat gradient buffer (`train.allreduce_mean`, RCCL
on the GPU box).  Here the per-rank gradient comes from the CPU oracle; the
collective and the sharding are the product's own code.  With every event valid
(render background parameter on), the mean of the per-shard means equals the
full-batch gradient (the reference's DDP semantics, scripts/run.py:84-89).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import unflat

RD, S, N_PER_RANK, WORLD = 1, 32, 6, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _params():
    from oracle import nerf as onerf
    return onerf.build_params(RD, 0, dtype=torch.float64)


def _f64(b):
    # f64 end to end, so the identity is checked to rounding (1e-12), not to f32 noise
    return {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}


def _batch(rank, world, raw):
    from deblur_e_nerf.train import synthetic_batch, synthetic_events
    from oracle.train import prepare_batch
    if raw:  # raw events sharded per rank, prepared (event prep + rays) per rank as the GPU step does
        return _f64(prepare_batch(synthetic_events(N_PER_RANK,
                                                   rank=rank, world=world), (0.27, 0.22), 1500.0))
    return _f64(synthetic_batch(N_PER_RANK, rank=rank, world=world))


def _worker(rank, world, port, out, raw=False):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deblur_e_nerf.train import allreduce_mean
    from oracle.train import flat_grad
    b = _batch(rank, world, raw)
    g, losses = flat_grad(_params(), torch.zeros(RD, dtype=torch.float64), b, S, RD)
    allreduce_mean(g)
    out[rank] = (g, torch.tensor(losses, dtype=torch.float64), b["end_ts"].clone())
    dist.destroy_process_group()


def test_sharding_partitions_the_global_batch():
    from deblur_e_nerf.train import synthetic_batch
    full = synthetic_batch(N_PER_RANK * WORLD)
    parts = [synthetic_batch(N_PER_RANK, rank=r, world=WORLD) for r in range(WORLD)]
    N = N_PER_RANK * WORLD
    for k in ("lid", "end_ts", "start_ts", "ts_diff"):
        assert torch.equal(torch.cat([p[k] for p in parts]), full[k])
    for k in ("rays_o", "rays_d", "jitter"):
        f = full[k].reshape(4, N, -1)
        cat = torch.cat([p[k].reshape(4, N_PER_RANK, -1) for p in parts], dim=1)
        assert torch.equal(cat, f), k


def test_raw_event_sharding_partitions_the_global_batch():
    """synthetic_events shards whole events (all 4 renders of an event on one rank)."""
    from deblur_e_nerf.train import synthetic_events
    full = synthetic_events(N_PER_RANK * WORLD)
    parts = [synthetic_events(N_PER_RANK, rank=r, world=WORLD) for r in range(WORLD)]
    for k in ("num_pos", "num_neg", "end_ts", "start_ts", "position"):
        assert torch.equal(torch.cat([p[k] for p in parts]), full[k]), k
    for k in ("normalized", "T_wc_position", "T_wc_orientation"):
        assert torch.equal(torch.cat([p[k] for p in parts], dim=1), full[k]), k
    j = torch.cat([p["jitter"].reshape(4, N_PER_RANK) for p in parts], dim=1)
    assert torch.equal(j, full["jitter"].reshape(4, -1))
    assert torch.equal(parts[0]["intrinsics_inverse"], full["intrinsics_inverse"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("raw", [False, True])
def test_allreduce_mean_equals_full_batch_gradient(raw):
    from oracle.train import flat_grad
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(WORLD, port, out, raw), nprocs=WORLD, join=True)
    g0, l0, e0 = out[0]
    g1, l1, e1 = out[1]
    assert not torch.equal(e0, e1)           # ranks saw different events
    assert torch.equal(g0, g1)               # identical averaged gradient on every rank
    if raw:
        from deblur_e_nerf.train import synthetic_events
        from oracle.train import prepare_batch
        full = _f64(prepare_batch(synthetic_events(N_PER_RANK * WORLD), (0.27, 0.22), 1500.0))
    else:
        from deblur_e_nerf.train import synthetic_batch
        full = _f64(synthetic_batch(N_PER_RANK * WORLD))
    g_full, losses = flat_grad(_params(), torch.zeros(RD, dtype=torch.float64), full, S, RD)
    rel = float((g0 - g_full).norm() / g_full.norm())
    assert rel < 1e-12, rel
    # per-layer check too (the small heads must not be swamped by the trunk)
    a, b = unflat(g0[:-RD], RD), unflat(g_full[:-RD], RD)
    for k in a:
        assert float((a[k] - b[k]).norm()) <= 1e-11 * float(b[k].norm()) + 1e-20, k
    assert torch.allclose(g0[-RD:], g_full[-RD:], rtol=1e-11, atol=1e-20)
    # the mean of the per-rank losses is the full-batch loss
    assert torch.allclose((l0 + l1) / 2, torch.tensor(losses, dtype=torch.float64), rtol=1e-12)


def test_pixbw_event_sharding_partitions_the_global_batch():
    """synthetic_pixbw_events shards whole events, including the interval
    generators, velocities and the 4 x S x N jitter."""
    from deblur_e_nerf.train import synthetic_pixbw_events
    S = 4
    full = synthetic_pixbw_events(N_PER_RANK * WORLD, S)
    parts = [synthetic_pixbw_events(N_PER_RANK, S, rank=r, world=WORLD) for r in range(WORLD)]
    for k in ("num_pos", "end_ts", "start_ts", "position", "T_wc_position", "velocity", "T_wc_orientation"):
        assert torch.equal(torch.cat([p[k] for p in parts]), full[k]), k
    for k in ("normalized", "interval_gen"):
        assert torch.equal(torch.cat([p[k] for p in parts], dim=1), full[k]), k
    j = torch.cat([p["jitter"].reshape(4, S, N_PER_RANK) for p in parts], dim=2)
    assert torch.equal(j, full["jitter"].reshape(4, S, -1))


def _grid_worker(rank, world, port, out):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deblur_e_nerf.external.marching import OccupancyGrid, sync_grid
    grid = OccupancyGrid([-1.5] * 3 + [1.5] * 3, resolution=16)
    g = torch.Generator().manual_seed(100 + rank)  # per-rank draws, as DataModule.setup seeds them
    history = []
    for step in range(5):
        # a rank-local update (den_occ_update runs on the GPU; here its effect: new EMA values and a
        # new threshold, different per rank), then fit_step's sync at the next step's start
        if step % 2 == 0:
            grid.occs.copy_(torch.rand(grid.num_cells, generator=g))
            grid._binary.copy_((grid.occs > 0.5).reshape(grid._binary.shape))
            grid._dirty = True
        synced = sync_grid(grid)
        history.append((synced, grid.occs.clone(), grid._binary.clone()))
    out[rank] = history
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_occupancy_grid_sync_broadcasts_rank0_after_updates():
    """DDP broadcast_buffers semantics (scripts/run.py:86-88, PyTorch default): after each
    rank-local occupancy-grid update with different per-rank draws, fit_step's sync_grid leaves
    every rank holding rank 0's occs / binary; steps without an update do not communicate."""
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_grid_worker, args=(WORLD, port, out), nprocs=WORLD, join=True)
    h0, h1 = out[0], out[1]
    for step, ((s0, o0, b0), (s1, o1, b1)) in enumerate(zip(h0, h1)):
        assert s0 == s1 == (step % 2 == 0)
        assert torch.equal(o0, o1) and torch.equal(b0, b1)
    assert not torch.equal(h0[0][1], h0[2][1])  # the grid did change between updates
