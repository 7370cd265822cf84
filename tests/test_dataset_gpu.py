"""The dataset build path on the GPU (den_queue_raw_events, den_max_refractory_period,
den_colorize_events, den_undistort_events through the C ABI) against the reference's own loops
(tests/golden/queue_*.npz, made by running data/datasets.py's classmethods) and, at sizes the
fixtures do not reach, against the oracle's vectorised restatement (oracle/datasets.py, itself
pinned to the fixtures by test_dataset_oracle.py).  Integer work: every comparison is exact
(torch.equal), except the OpenCV undistortion restatement (parity unpinned: OpenCV is absent),
compared with the oracle's double-precision loop at 1e-3 px."""
import os
import shutil
import tempfile

import numpy as np
import pytest
import torch

from oracle import datasets as ods

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = ["small_rggb", "unsorted_mono", "davis_grbg", "hot_pixels_bggr"]
KEYS = ("position", "start_ts", "end_ts", "num_pos", "num_neg")


def _z(golden_dir, name):
    return np.load(os.path.join(golden_dir, f"queue_{name}.npz"))


def _dev(z):
    return (torch.from_numpy(z["raw_position"].astype(np.int64)).to(DEV),
            torch.from_numpy(z["raw_timestamp"]).to(DEV), torch.from_numpy(z["raw_polarity"]).to(DEV))


@pytest.mark.parametrize("name", CASES)
def test_queue_matches_reference(golden_dir, name):
    from deblur_e_nerf import _native as nat
    z = _z(golden_dir, name)
    pos, ts, pol = _dev(z)
    H, W = int(z["img_height"]), int(z["img_width"])
    q, mx = nat.queue_raw_events(pos, ts, pol, H, W)
    for k in KEYS:
        want = torch.from_numpy(z["q_" + k])
        assert q[k].dtype == want.dtype and torch.equal(q[k].cpu(), want), k
    assert mx == int(z["max_refractory_period"])
    assert nat.max_refractory_period(pos, ts, H, W) == mx
    if str(z["bayer_pattern"]):
        ch = nat.colorize_events(q["position"], ods.bayer_channels(str(z["bayer_pattern"])))
        assert torch.equal(ch.cpu(), torch.from_numpy(z["channel_idx"]))
    und = nat.undistort_events(q["position"], None, np.eye(3), [])
    assert torch.equal(und.cpu(), torch.from_numpy(z["final_position"]))


def test_queue_no_interval_and_empty(golden_dir):
    from deblur_e_nerf import _native as nat
    z = np.load(os.path.join(golden_dir, "queue_no_interval.npz"))
    pos, ts, pol = _dev(z)
    q, mx = nat.queue_raw_events(pos, ts, pol, 4, 4)
    assert mx is None and all(len(v) == 0 for v in q.values())
    assert nat.max_refractory_period(pos, ts, 4, 4) is None
    e = torch.zeros(0, 2, dtype=torch.int64, device=DEV)
    q, mx = nat.queue_raw_events(e, torch.zeros(0, dtype=torch.int64, device=DEV),
                                 torch.zeros(0, dtype=torch.bool, device=DEV), 3, 3)
    assert mx is None and q["position"].shape == (0, 2)


def test_queue_rejects_positions_outside_the_image():
    from deblur_e_nerf import _native as nat
    pos = torch.tensor([[0, 0], [5, 1], [0, 0]], dtype=torch.int64, device=DEV)
    ts = torch.tensor([1, 2, 3], dtype=torch.int64, device=DEV)
    with pytest.raises(IndexError):
        nat.queue_raw_events(pos, ts, torch.ones(3, dtype=torch.bool, device=DEV), 2, 5)
    with pytest.raises(IndexError):
        nat.max_refractory_period(pos, ts, 2, 5)


@pytest.mark.parametrize("H,W,n,sorted_ts,seed", [(480, 640, 1 << 22, True, 1),   # 19-bit keys: 3 passes, 1024 tiles
                                                    (1, 1, 1 << 20, True, 2),      # one pixel: no sort pass
                                                    (4097, 4099, 1 << 21, False, 3),  # 25-bit keys: 4 passes
                                                    (3, 5, 100_003, True, 4)])     # ragged last tile, hot pixels
def test_queue_large_matches_oracle(H, W, n, sorted_ts, seed):
    from deblur_e_nerf import _native as nat
    g = np.random.default_rng(seed)
    pos = np.stack([g.integers(0, W, n), g.integers(0, H, n)], 1).astype(np.int64)
    steps = g.integers(0, 3, n) * g.integers(1, 1000, n)
    ts = (10 ** 6 + np.cumsum(steps)).astype(np.int64)
    if not sorted_ts:
        ts = ts[g.permutation(n)]
    pol = g.random(n) < 0.5
    want, want_mx = ods.queue_sorted(pos, ts, pol, H, W)
    q, mx = nat.queue_raw_events(torch.from_numpy(pos).to(DEV), torch.from_numpy(ts).to(DEV),
                                 torch.from_numpy(pol).to(DEV), H, W)
    for k in KEYS:
        assert torch.equal(q[k].cpu(), torch.from_numpy(want[k])), k
    assert mx == want_mx


@pytest.mark.parametrize("model,D", [("plumb_bob", [-0.12, 0.03, 1e-3, -5e-4]), ("equidistant", [0.05, -0.01, 0.002, -1e-4])])
def test_undistort_matches_oracle(model, D):
    from deblur_e_nerf import _native as nat
    g = np.random.default_rng(7)
    K = np.array([[320.0, 0, 173.0], [0, 318.0, 130.0], [0, 0, 1]], dtype=np.float32)
    pos = np.stack([g.integers(0, 346, 5000), g.integers(0, 260, 5000)], 1).astype(np.int64)
    fn = ods.undistort_plumb_bob if model == "plumb_bob" else ods.undistort_equidistant
    want = fn(pos.astype(np.float32), K, np.float32(D))
    got = nat.undistort_events(torch.from_numpy(pos).to(DEV), model, K, np.float32(D)).cpu().numpy()
    assert np.abs(got - want).max() < 1e-3
    with pytest.raises(NotImplementedError):
        nat.undistort_events(torch.from_numpy(pos).to(DEV), "fov", K, np.float32(D))


@pytest.mark.parametrize("model,D", [("plumb_bob", [-0.35, 0.12, 1.5e-3, -1e-3]),
                                     ("equidistant", [0.25, -0.08, 0.02, -0.003])])
def test_undistort_round_trip_strong_distortion_corners(model, D):
    """Strong distortion at the image corners and edges (where the iterations work hardest): the
    kernel's undistorted pixels, normalised by K and distorted again by the forward model, land back
    on the input pixels -- to 1e-3 px for the equidistant Newton solve, and for plumb_bob's fixed 5
    iterations (cv2.undistortPoints' default criteria) no worse than the oracle's own 5-iteration
    round trip; the kernel equals the oracle to 1e-3 px throughout (parity unpinned vs OpenCV)."""
    from deblur_e_nerf import _native as nat
    H, W = 260, 346
    K = np.array([[300.0, 0, 172.5], [0, 300.0, 129.5], [0, 0, 1]], dtype=np.float32)
    g = np.random.default_rng(11)
    corners = np.array([[0, 0], [W - 1, 0], [0, H - 1], [W - 1, H - 1]])
    near = (corners[:, None, :] + np.sign(np.array([W / 2, H / 2]) - corners)[:, None, :]
            * g.integers(0, 6, size=(4, 64, 2))).reshape(-1, 2)
    edges = np.concatenate([np.stack([g.integers(0, W, 128), np.zeros(128, int)], 1),
                            np.stack([np.full(128, W - 1), g.integers(0, H, 128)], 1)])
    pos = np.concatenate([near, edges]).astype(np.int64)
    got = nat.undistort_events(torch.from_numpy(pos).to(DEV), model, K, np.float32(D)).cpu().numpy().astype(np.float64)
    fn = ods.undistort_plumb_bob if model == "plumb_bob" else ods.undistort_equidistant
    want = fn(pos.astype(np.float32), K, np.float32(D)).astype(np.float64)
    ok = (got[:, 0] > -1e5) & (want[:, 0] > -1e5)
    assert np.array_equal(got[:, 0] > -1e5, want[:, 0] > -1e5)  # the same points flagged unconverged
    assert ok.mean() > 0.9 and np.abs(got[ok] - want[ok]).max() < 1e-3
    Kd = K.astype(np.float64)
    back = lambda u: (ods.distort_plumb_bob if model == "plumb_bob" else ods.distort_equidistant)(  # noqa: E731
        np.stack([(u[:, 0] - Kd[0, 2]) / Kd[0, 0], (u[:, 1] - Kd[1, 2]) / Kd[1, 1]], 1), Kd, np.float64(D))
    e_got = np.abs(back(got[ok]) - pos[ok]).max()
    e_want = np.abs(back(want[ok]) - pos[ok]).max()
    print(f"[{model}] round trip at the corners: kernel {e_got:.2e} px, oracle {e_want:.2e} px, "
          f"{(~ok).sum()} unconverged")
    assert e_got <= (1e-3 if model == "equidistant" else e_want + 1e-3)


def _raw_dir(golden_dir, name, with_poses=False):
    z = _z(golden_dir, name)
    d = tempfile.mkdtemp(prefix="den_rawds_")
    np.savez(os.path.join(d, "raw_events.npz"), position=z["raw_position"], timestamp=z["raw_timestamp"],
             polarity=z["raw_polarity"])
    H, W = int(z["img_height"]), int(z["img_width"])
    cal = dict(img_height=np.array(H, dtype=np.uint16), img_width=np.array(W, dtype=np.uint16),
               bayer_pattern=np.array(str(z["bayer_pattern"])), distortion_model=np.array("plumb_bob"),
               distortion_params=np.zeros(0, dtype=np.float32),
               intrinsics=np.array([[200.0, 0, W / 2], [0, 200.0, H / 2], [0, 0, 1]], dtype=np.float32),
               refractory_period=np.array(0), pos_contrast_threshold=np.array(0.25, dtype=np.float32),
               neg_contrast_threshold=np.array(0.25, dtype=np.float32))
    np.savez(os.path.join(d, "camera_calibration.npz"), **cal)
    return d, z


@pytest.mark.parametrize("name", ["davis_grbg", "unsorted_mono"])
def test_event_dataset_builds_and_caches_events_pt(golden_dir, name):
    """datasets.Event on a directory holding only raw_events.npz + calibration: queue -> colorize ->
    undistort on the GPU, cached as events.pt (loaded back with weights_only), equal to the
    reference's transformed events."""
    from deblur_e_nerf.data import datasets
    d, z = _raw_dir(golden_dir, name)
    try:
        ev = datasets.Event(d, None)
        assert os.path.isfile(os.path.join(d, "events.pt"))
        want = {k: torch.from_numpy(z["q_" + k]) for k in KEYS}
        want["position"] = torch.from_numpy(z["final_position"])
        if "channel_idx" in z.files:
            want["channel_idx"] = torch.from_numpy(z["channel_idx"])
        assert set(ev.events) == set(want)
        for k, v in want.items():
            assert not ev.events[k].is_cuda and ev.events[k].dtype == v.dtype and torch.equal(ev.events[k], v), k
        again = datasets.Event(d, None)  # the cache
        for k, v in want.items():
            assert torch.equal(again.events[k], v)
        perm = datasets.Event(d, 5)
        assert len(perm) == len(ev) and torch.equal(perm.events["end_ts"].sort().values, ev.events["end_ts"].sort().values)
    finally:
        shutil.rmtree(d)


def test_refractory_period_extracts_and_caches(golden_dir):
    from deblur_e_nerf.data import datasets
    from deblur_e_nerf.models.event_generation_params import RefractoryPeriod
    d, z = _raw_dir(golden_dir, "small_rggb")
    try:
        rp = RefractoryPeriod(d)
        mx = datasets.Event.load_max_refractory_period(d)
        assert mx.dtype == torch.int64 and int(mx) == int(z["max_refractory_period"])
        assert int(rp.max_refractory_period) == int(z["max_refractory_period"])
        assert 0 <= float(rp.refractory_period) < int(mx)
    finally:
        shutil.rmtree(d)


def test_datamodule_builds_from_raw_events(golden_dir):
    """DataModule (run.py:38-45's construction) on a dataset directory fresh from preprocessing:
    the training loader draws batches of the queued events."""
    from deblur_e_nerf.data.datamodule import DataModule
    from deblur_e_nerf.utils.easydict import EasyDict
    d, z = _raw_dir(golden_dir, "davis_grbg")
    try:
        dm = DataModule(0, ["novel_view"], 1, [0], EasyDict(enable=False), d, 1.0, 1.0, 1.0, None, 9, True,
                        256, 131072, 1, 1, 0)
        dm.setup("fit")
        # IterableMapDataset(TrimDataset(Event)): every queued event is in the training set (ratio 1.0)
        events = dm.train_dataset.map_dataset
        assert len(events) == len(z["q_end_ts"]) and len(events.dataset) == len(z["q_end_ts"])
        ev = next(iter(dm.train_dataloader()["event"]))
        assert ev["end_ts"].shape == (1, 256) and ev["position"].dtype == torch.float32
        assert set(ev) == {"position", "start_ts", "end_ts", "num_pos", "num_neg", "channel_idx"}
    finally:
        shutil.rmtree(d)
