"""The evaluation loop at world 2 (scripts/run.py:84-118: Trainer.validate under PL's DDP, which
shards the views with a non-shuffling DistributedSampler and all-gathers the step outputs in
evaluation_epoch_end, deblur_e_nerf.py:670-691).

Two processes on the box's GPU (gloo, as tests/test_fit_ddp_gpu.py) run ``run_evaluation("val")``
twice on the eval_epoch fixtures' 3 views.  The sampler pads 3 views to 4 (rank 0 takes views 0, 2,
rank 1 views 1, 0) and the gather concatenates step by step, so rank 0's epoch end sees the views in
the order 0, 1, 2, 0 -- the duplicate included, as under Lightning.  Checked against one process
that runs validation_step on the 3 views and feeds validation_epoch_end the outputs [0, 1, 2, 0]:
the same metrics, the same correction warm start carried into the second evaluation, the same saved
predictions; rank 1 logs nothing and writes nothing."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2
FIXTURES = ["eval_epoch_rd1", "eval_epoch_rd3_gn"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(golden, name):
    """The fixture's model (the reference's field, occupancy grid from the fixture's draws) and a
    DataModule on its views, as tests/test_eval_epoch_gpu.py builds them."""
    from deblur_e_nerf.external import marching
    from test_eval_epoch_gpu import _correction, _datamodule, _ImgLogger
    from test_deblur_gpu import build_model
    from test_nerfacc_gpu import _Draws
    z = np.load(os.path.join(golden, f"{name}.npz"))
    m, d = build_model(z, correction=_correction(z), eval_save=True, return_dir=True)
    old = marching._uniform
    marching._uniform = _Draws([z["occ_u"]])
    try:
        m.nerf.update_occ_grid(step=0, T_wc_position=m.trajectory.T_wc_position)
    finally:
        marching._uniform = old
    m._logger = _ImgLogger()
    m.trainer.log_dir = tempfile.mkdtemp(prefix="den_evalddp_")
    return z, m, _datamodule(z, d)


def _saved(log_dir):
    folder = os.path.join(log_dir, "predictions")
    if not os.path.isdir(folder):
        return {}
    from deblur_e_nerf.utils import image_io
    return {f: image_io.imread_unchanged(os.path.join(folder, f)) for f in sorted(os.listdir(folder))}


def _inits(m):
    return [getattr(m, "init_correction_" + n).clone() for n in ("scale", "gamma", "offset")]


def _worker(rank, world, port, out, golden, name):
    import sys
    from conftest import PKG, ROOT
    for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z, m, dm = _setup(golden, name)
    res = []
    for ev in range(2):
        m._current_epoch = ev
        m.logged.clear()
        res.append(m.run_evaluation("val", dm)[0])
    out[rank] = dict(res=res, inits=_inits(m), saved=_saved(m.trainer.log_dir),
                     errors=os.path.isdir(os.path.join(m.trainer.log_dir, "correction-errors")))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", FIXTURES)
def test_validation_two_ranks_matches_padded_single_process(golden_dir, name):
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    mp.start_processes(_worker, args=(WORLD, _free_port(), out, golden_dir, name), nprocs=WORLD, join=True,
                       start_method="spawn")
    r0, r1 = out[0], out[1]
    # one process: the 3 views rendered, the epoch end fed them as the 2 ranks' gather orders them
    z, m, dm = _setup(golden_dir, name)
    dm.setup("validate")
    m.eval()
    with torch.no_grad():
        steps = [m.validation_step({k: v.to("cuda") for k, v in b.items()}, i)
                 for i, b in enumerate(dm.val_dataloader())]
    assert len(steps) == 3
    want = []
    for ev in range(2):
        m._current_epoch = ev
        m.logged.clear()
        m.validation_epoch_end([steps[0], steps[1], steps[2], steps[0]])
        want.append({k: float(v) for k, v in m.logged.items() if k.startswith("val/") and k != "val/epoch"})
    inits, mine = _inits(m), _saved(m.trainer.log_dir)
    for ev in range(2):
        print(f"[{name}] eval {ev}: rank 0 {r0['res'][ev]} vs one process (padded) {want[ev]}; rank 1 {r1['res'][ev]}")
        assert set(r0["res"][ev]) == set(want[ev]) and want[ev]
        for k, v in want[ev].items():
            assert abs(r0["res"][ev][k] - v) <= 1e-6 * max(1.0, abs(v)), (ev, k, r0["res"][ev][k], v)
        assert r1["res"][ev] == {}
    # the warm start carried through both evaluations, and the saved predictions (3 files: the
    # duplicate view overwrites its own)
    for a, b in zip(r0["inits"], inits):
        assert a.shape == b.shape and torch.allclose(a.double(), b.double(), rtol=1e-6, atol=1e-9), (a, b)
    assert set(r0["saved"]) == set(mine) and len(mine) == 3
    for f in mine:
        assert np.abs(r0["saved"][f].astype(np.int32) - mine[f].astype(np.int32)).max() <= 1, f
    assert r1["saved"] == {} and not r1["errors"] and r0["errors"] == bool(z["black_level_offset"])
    # the padded epoch is not the 3-view epoch: the duplicate view counts twice (as under Lightning)
    m.logged.clear()
    m.validation_epoch_end(steps)
    print(f"[{name}] 3-view psnr {float(m.logged['val/psnr'])} vs padded {want[1]['val/psnr']}")
