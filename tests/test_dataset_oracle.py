"""The dataset build path's oracle (oracle/datasets.py) against the reference's own loops
(tests/golden/queue_*.npz: Event.queue_raw_events -> colorize_events -> undistort_events and
Event.extract_max_refractory_period, run on synthetic raw_events.npz directories by
make_golden.py), CPU only.  Integer work: every comparison is exact.  The undistortion oracle
restates OpenCV (absent here, parity unpinned): it is checked by round trips through the forward
distortion models it inverts."""
import glob
import os

import numpy as np
import pytest

from oracle import datasets as ods

CASES = ["small_rggb", "unsorted_mono", "davis_grbg", "hot_pixels_bggr"]


def _z(golden_dir, name):
    return np.load(os.path.join(golden_dir, f"queue_{name}.npz"))


@pytest.mark.parametrize("name", CASES)
def test_queue_oracle_matches_reference(golden_dir, name):
    z = _z(golden_dir, name)
    args = (z["raw_position"], z["raw_timestamp"], z["raw_polarity"], int(z["img_height"]), int(z["img_width"]))
    loop = ods.queue_loop(*args)
    vec, mx = ods.queue_sorted(*args)
    for q in (loop, vec):
        for k in ("position", "start_ts", "end_ts", "num_pos", "num_neg"):
            assert q[k].dtype == z["q_" + k].dtype and np.array_equal(q[k], z["q_" + k]), k
    assert mx == int(z["max_refractory_period"]) and str(z["max_refractory_period_dtype"]) == "torch.int64"
    assert ods.max_refractory_period_loop(z["raw_position"], z["raw_timestamp"]) == mx
    if str(z["bayer_pattern"]):
        assert np.array_equal(ods.colorize(z["q_position"], str(z["bayer_pattern"])), z["channel_idx"])
    # no distortion parameters: undistort_events is the cast to the default dtype
    assert np.array_equal(z["final_position"], z["q_position"].astype(np.float32))


def test_queue_oracle_no_interval(golden_dir):
    z = np.load(os.path.join(golden_dir, "queue_no_interval.npz"))
    q, mx = ods.queue_sorted(z["raw_position"], z["raw_timestamp"], z["raw_polarity"], 4, 4)
    assert len(q["end_ts"]) == int(z["q_count"]) == 0 and mx is None
    assert np.isinf(z["max_refractory_period"]) and str(z["max_refractory_period_dtype"]) == "torch.float64"
    assert ods.max_refractory_period_loop(z["raw_position"], z["raw_timestamp"]) is None


def test_queue_fixtures_cover_the_edge_cases(golden_dir):
    """What the fixtures exercise: repeated timestamps at a pixel (dropped events), single-event
    pixels, both polarities, unsorted input (a negative interval), multi-tile hot pixels."""
    seen_negative = False
    for name in CASES:
        z = _z(golden_dir, name)
        key = z["raw_position"][:, 1].astype(np.int64) * int(z["img_width"]) + z["raw_position"][:, 0]
        n_raw, n_q = len(key), len(z["q_end_ts"])
        assert 0 < n_q < n_raw
        _, counts = np.unique(key, return_counts=True)
        assert (counts == 1).any() or name == "hot_pixels_bggr"
        assert z["q_num_pos"].min() == 0 and z["q_num_pos"].max() == 1
        seen_negative |= int(z["max_refractory_period"]) < 0
    assert seen_negative
    assert len(glob.glob(os.path.join(golden_dir, "queue_*.npz"))) == len(CASES) + 1


def test_undistort_oracle_inverts_the_distortion_models():
    g = np.random.default_rng(0)
    K = np.array([[320.0, 0, 173.0], [0, 318.0, 130.0], [0, 0, 1]])
    xy = g.uniform(-0.45, 0.45, size=(400, 2))
    # plumb_bob: 5 fixed-point iterations converge to ~1e-3 px for this (moderate) distortion
    D = [-0.12, 0.03, 1e-3, -5e-4]
    px = ods.distort_plumb_bob(xy, K, D).astype(np.float32)
    back = ods.undistort_plumb_bob(px, K, D)
    want = np.stack([K[0, 0] * xy[:, 0] + K[0, 2], K[1, 1] * xy[:, 1] + K[1, 2]], 1)
    assert np.abs(back - want).max() < 2e-2
    # equidistant: Newton to 1e-8 in theta
    Df = [0.05, -0.01, 0.002, -1e-4]
    px = ods.distort_equidistant(xy, K, Df).astype(np.float32)
    back = ods.undistort_equidistant(px, K, Df)
    assert np.abs(back - want).max() < 1e-3
    # no distortion at all: the identity
    assert np.abs(ods.undistort_plumb_bob(want.astype(np.float32), K, [0, 0, 0, 0]) - want).max() < 1e-3
