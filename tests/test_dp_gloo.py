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
    generators and the 4 x S x N jitter; every rank holds the whole camera trajectory."""
    from deblur_e_nerf.train import synthetic_pixbw_events
    S = 4
    full = synthetic_pixbw_events(N_PER_RANK * WORLD, S)
    parts = [synthetic_pixbw_events(N_PER_RANK, S, rank=r, world=WORLD) for r in range(WORLD)]
    for k in ("num_pos", "end_ts", "start_ts", "position"):
        assert torch.equal(torch.cat([p[k] for p in parts]), full[k]), k
    for k in ("T_wc_position", "T_wc_orientation", "T_wc_timestamp"):
        assert all(torch.equal(p[k], full[k]) for p in parts), k
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


class _FitStub(torch.nn.Module):
    """The attributes DeblurENeRF.fit_step reads, around the product's fit_step / sync_grid /
    allreduce_gradients: a training_step that updates the occupancy grid with per-rank draws whenever
    global_step % UPDATE_EVERY == 0 -- on EVERY micro-batch of such a group, as the reference's
    update_occ_grid(step=global_step) does (global_step only advances per optimizer step,
    deblur_e_nerf.py:465; den_occ_update's effect) -- and records the grid each micro-batch marches
    with and the global step it ran at."""
    UPDATE_EVERY = 2

    def __init__(self, rank, acc):
        super().__init__()
        from types import SimpleNamespace
        from deblur_e_nerf.external.marching import OccupancyGrid
        self.w = torch.nn.Parameter(torch.zeros(3))
        self.trainer = SimpleNamespace(accumulate_grad_batches=acc)
        self.nerf = SimpleNamespace(occupancy_grid=OccupancyGrid([-1.5] * 3 + [1.5] * 3, resolution=8))
        self._global_step = 0
        self.g = torch.Generator().manual_seed(300 + rank)
        self.seen = []

    def training_step(self, batch, batch_index):
        grid = self.nerf.occupancy_grid
        before = grid.occs.clone()
        if self._global_step % self.UPDATE_EVERY == 0:
            grid.occs.copy_(torch.rand(grid.num_cells, generator=self.g))
            grid._binary.copy_((grid.occs > 0.5).reshape(grid._binary.shape))
            grid._dirty = True
        self.seen.append((before, grid.occs.clone(), self._global_step))
        return (self.w * batch).sum()


def _fit_worker(rank, world, port, out, acc, n_micro):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deblur_e_nerf.models.deblur_e_nerf import DeblurENeRF
    m = _FitStub(rank, acc)
    opt = torch.optim.SGD(m.parameters(), lr=1.0)
    params = []
    for i in range(n_micro):
        DeblurENeRF.fit_step(m, torch.tensor([1.0, 2.0, 3.0]) * (rank + 1) * (i + 1), i, opt)
        params.append(m.w.detach().clone())
    out[rank] = (m.seen, params)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("acc", [1, 3])
def test_fit_step_grid_broadcast_per_accumulation_group(acc):
    """DDP + PL accumulation (run.py:84-100, 07_ziggy_and_fuzz_hdr.yaml accumulate_grad_batches):
    rank 0's grid is broadcast only before the first micro-batch of a group (the only forward
    after a synced one), before that micro-batch's rank-local grid update; every micro-batch of an
    updating group (global_step % n == 0) updates the grid again, so micro-batches 1..acc-1 march
    with the rank's own grid after its second, third ... update; the averaged gradient is applied
    once per group and leaves identical parameters on every rank."""
    n_micro = 4 * acc + 1
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_fit_worker, args=(WORLD, port, out, acc, n_micro), nprocs=WORLD, join=True)
    (seen0, p0), (seen1, p1) = out[0], out[1]
    repeated = 0
    for i in range(n_micro):
        (b0, a0, gs0), (b1, a1, gs1) = seen0[i], seen1[i]
        assert gs0 == gs1 == i // acc, (i, gs0, gs1)
        updating = gs0 % _FitStub.UPDATE_EVERY == 0
        if i % acc == 0:
            # the pre-update grid is rank 0's on every rank (the broadcast), then each rank updates its own
            assert torch.equal(b0, b1), i
            if i > 0:  # rank 0's grid of the previous group's last micro-batch
                assert torch.equal(b1, seen0[i - 1][1]), i
        else:  # no broadcast inside a group: each rank marches with its own grid of the last micro-batch
            assert torch.equal(b0, seen0[i - 1][1]) and torch.equal(b1, seen1[i - 1][1]), i
            repeated += updating
        if updating:  # a fresh per-rank update on every micro-batch of the group
            assert not torch.equal(a0, b0) and not torch.equal(a1, b1) and not torch.equal(a0, a1), i
        else:
            assert torch.equal(a0, b0) and torch.equal(a1, b1), i
    assert repeated == (acc - 1) * len({i // acc for i in range(n_micro) if (i // acc) % _FitStub.UPDATE_EVERY == 0
                                        and i % acc})  or acc == 1
    for i in range(n_micro):
        assert torch.equal(p0[i], p1[i]), i
        if (i + 1) % acc == 0:  # SGD lr 1 on the rank-mean of the group's summed (loss / acc) gradients
            k = i + 1 - acc
            g = sum((r + 1) * (j + 1) for r in range(WORLD) for j in range(k, i + 1)) / WORLD / acc
            prev = p0[k - 1] if k > 0 else torch.zeros(3)
            assert torch.allclose(p0[i], prev - g * torch.tensor([1.0, 2.0, 3.0])), i
        elif i > 0:
            assert torch.equal(p0[i], p0[i - 1]), i


class _MixedGrads(torch.nn.Module):
    """f32 parameters (the MLP / hash table) beside an f64 one (tau_r, event_generation_params.py:196-201)."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Parameter(torch.zeros(1000))
        self.tau = torch.nn.Parameter(torch.zeros((), dtype=torch.float64))
        self.b = torch.nn.Parameter(torch.zeros(3, 7))


def _mixed_worker(rank, world, port, out):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deblur_e_nerf.models.deblur_e_nerf import allreduce_gradients, flat_gradient_buffers
    m = _MixedGrads()
    m.a.grad = torch.full((1000,), float(rank + 1))
    m.tau.grad = torch.tensor(1e-9 * (rank + 1) + 1.0, dtype=torch.float64)
    m.b.grad = torch.full((3, 7), 3.0 * (rank + 1))
    bufs = flat_gradient_buffers([p.grad for p in m.parameters()])
    allreduce_gradients(m)
    out[rank] = ({str(dt): (b.dtype, b.numel()) for dt, (b, _) in bufs.items()}, m.a.grad.clone(), m.tau.grad.clone(),
                 m.b.grad.clone())
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_allreduce_gradients_keeps_f32_and_f64_apart():
    """allreduce_gradients (deblur_e_nerf.py's DDP step): one f32 buffer for the f32 gradients and one
    f64 buffer for tau_r's -- the f32 gradients never travel promoted to f64 -- and the result is
    each gradient's rank mean, in its own dtype (the f64 one exact to f64)."""
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_mixed_worker, args=(WORLD, port, out), nprocs=WORLD, join=True)
    for r in range(WORLD):
        bufs, ga, gt, gb = out[r]
        assert bufs == {"torch.float32": (torch.float32, 1000 + 21), "torch.float64": (torch.float64, 1)}, bufs
        assert ga.dtype == torch.float32 and torch.equal(ga, torch.full((1000,), 1.5))
        assert gb.dtype == torch.float32 and torch.equal(gb, torch.full((3, 7), 4.5))
        assert gt.dtype == torch.float64 and float(gt) == (1.0 + 1e-9 + 1.0 + 2e-9) / 2
