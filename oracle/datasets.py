"""Oracle: raw-event preprocessing of the dataset loader -- numpy / pure-Python restatement (test
infrastructure only, see oracle/__init__.py; pinned by tests/golden/queue_*.npz, which record the
reference's own classmethods run on synthetic raw_events.npz directories).

Reference semantics (deblur_e_nerf/data/datasets.py, file:line):
* Event.queue_raw_events                :190-284  per pixel a maxlen-2 deque of (ts, polarity):
  an event is kept iff its pixel saw an earlier raw event (input order) and that event's
  timestamp differs; start_ts = that timestamp, num_pos = own polarity - 0 (the window's sum
  minus its first entry), num_neg = 1 - num_pos
* Event.extract_max_refractory_period   :133-187  per pixel the last appended timestamp; an
  event equal to it is skipped, else its interval to it enters the minimum (inf when none)
* Event.colorize_events                 :287-328  bayer index (x odd) + 2 (y odd)
* Event.undistort_events                :331-364  f32 cast; cv2.undistortPoints (plumb_bob) /
  cv2.fisheye.undistortPoints (equidistant), P = intrinsics -- OpenCV is absent here, so
  `undistort_*` restate OpenCV's published iterations (PARITY UNPINNED) and `distort_*` the
  forward models they invert (round trips in the tests).

`queue_loop` / `max_refractory_period_loop` follow the reference's per-event loop (the CPU
baseline bench.py times); `queue_sorted` is the vectorised restatement (stable argsort by pixel)
the tests use at larger sizes.
"""
import math

import numpy as np

BAYER_INDEX = {"R": 0, "G": 1, "B": 2}


def queue_loop(position, timestamp, polarity, img_height, img_width):
    """datasets.py:190-284 as a loop over the events with per-pixel state (the previous raw
    event's timestamp and polarity): -> dict(position, start_ts, end_ts, num_pos, num_neg)."""
    del img_height, img_width  # the reference sizes its deque grid with them; a dict needs neither
    n = len(timestamp)
    last_ts = {}
    keep = np.zeros(n, dtype=bool)
    start = np.empty(n, dtype=np.int64)
    pos = position.astype(np.int64)
    pol = polarity.astype(np.int64)
    for i in range(n):
        key = (int(pos[i, 0]), int(pos[i, 1]))
        t = int(timestamp[i])
        prev = last_ts.get(key)
        last_ts[key] = t
        if prev is not None and prev != t:
            keep[i] = True
            start[i] = prev
    return dict(position=pos[keep], start_ts=start[keep], end_ts=timestamp.astype(np.int64)[keep],
                num_pos=pol[keep], num_neg=1 - pol[keep])


def max_refractory_period_loop(position, timestamp):
    """datasets.py:133-187: the minimum interval between a pixel's consecutive distinct
    timestamps (input order, equal neighbours skipped); None for the reference's inf."""
    last = {}
    best = None
    for i in range(len(timestamp)):
        key = (int(position[i, 0]), int(position[i, 1]))
        t = int(timestamp[i])
        prev = last.get(key)
        if prev is not None and prev == t:
            continue
        last[key] = t
        if prev is not None:
            best = t - prev if best is None else min(best, t - prev)
    return best


def queue_sorted(position, timestamp, polarity, img_height, img_width):
    """The same relation vectorised: a stable sort of the pixel keys keeps input order within a
    pixel, so an event's predecessor is its left neighbour when the keys agree.
    -> (queued dict, the minimum interval or None)."""
    pos = position.astype(np.int64)
    x, y = pos[:, 0], pos[:, 1]
    if len(x) and (x.min() < 0 or y.min() < 0 or x.max() >= img_width or y.max() >= img_height):
        raise IndexError("event position outside the image")
    key = y * img_width + x
    ts = timestamp.astype(np.int64)
    order = np.argsort(key, kind="stable")
    pred = np.full(len(ts), -1, dtype=np.int64)
    same = key[order[1:]] == key[order[:-1]]
    pred[order[1:][same]] = order[:-1][same]
    has = pred >= 0
    keep = has.copy()
    keep[has] = ts[pred[has]] != ts[has]
    pol = polarity.astype(np.int64)
    start = np.where(keep, ts[np.where(has, pred, 0)], 0)
    q = dict(position=pos[keep], start_ts=start[keep], end_ts=ts[keep], num_pos=pol[keep], num_neg=1 - pol[keep])
    iv = q["end_ts"] - q["start_ts"]
    return q, (int(iv.min()) if len(iv) else None)


def bayer_channels(pattern):
    """datasets.py:289-305: the pattern string -> 4 channel indices (None: monochrome)."""
    pattern = str(pattern)
    assert len(pattern) in (0, 4)
    if pattern == "":
        return None
    assert set(pattern) == set(BAYER_INDEX)
    return [BAYER_INDEX[c] for c in pattern]


def colorize(position, pattern):
    """datasets.py:307-327: channel of the (x even/odd, y even/odd) bayer cell, u8."""
    ch = bayer_channels(pattern)
    idx = (position[:, 0] % 2) + 2 * (position[:, 1] % 2)
    return np.asarray(ch, dtype=np.uint8)[idx]


def undistort_plumb_bob(points, K, D, iters=5):
    """cv2.undistortPoints(points, K, D, P=K) for k1 k2 p1 p2 (OpenCV's fixed-point iteration,
    criteria COUNT 5), double arithmetic; points (n,2) f32 -> (n,2) f32."""
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    k1, k2, p1, p2 = (float(v) for v in np.asarray(D, dtype=np.float64))
    u, v = points[:, 0].astype(np.float64), points[:, 1].astype(np.float64)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    out = np.empty((len(u), 2), dtype=np.float32)
    for i in range(len(u)):
        x = (u[i] - cx) * (1.0 / fx)
        y = (v[i] - cy) * (1.0 / fy)
        x0, y0 = x, y
        for _ in range(iters):
            r2 = x * x + y * y
            icdist = 1.0 / (1.0 + (k2 * r2 + k1) * r2)
            if icdist < 0:
                x, y = (u[i] - cx) * (1.0 / fx), (v[i] - cy) * (1.0 / fy)
                break
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x, y = (x0 - dx) * icdist, (y0 - dy) * icdist
        w = 1.0 / (K[2, 0] * x + K[2, 1] * y + K[2, 2])
        out[i] = ((K[0, 0] * x + K[0, 1] * y + K[0, 2]) * w, (K[1, 0] * x + K[1, 1] * y + K[1, 2]) * w)
    return out


def undistort_equidistant(points, K, D, iters=10, eps=1e-8):
    """cv2.fisheye.undistortPoints(points, K, D, P=K) (Newton on theta, criteria MAX_ITER + EPS,
    10, 1e-8; unconverged or sign-flipped points -> -1e6)."""
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    k = [float(v) for v in np.asarray(D, dtype=np.float64)]
    out = np.empty((len(points), 2), dtype=np.float32)
    for i, (pu, pv) in enumerate(points.astype(np.float64)):
        pwx, pwy = (pu - K[0, 2]) / K[0, 0], (pv - K[1, 2]) / K[1, 1]
        theta_d = min(max(-math.pi / 2, math.hypot(pwx, pwy)), math.pi / 2)
        converged, theta, scale = False, theta_d, 0.0
        if abs(theta_d) > eps:
            for _ in range(iters):
                t2 = theta * theta
                t4, t6, t8 = t2 * t2, t2 * t2 * t2, t2 * t2 * t2 * t2
                a, b, c, d = k[0] * t2, k[1] * t4, k[2] * t6, k[3] * t8
                fix = (theta * (1 + a + b + c + d) - theta_d) / (1 + 3 * a + 5 * b + 7 * c + 9 * d)
                theta -= fix
                if abs(fix) < eps:
                    converged = True
                    break
            scale = math.tan(theta) / theta_d
        else:
            converged = True
        flipped = (theta_d < 0 < theta) or (theta < 0 < theta_d)
        if not converged or flipped:
            out[i] = (-1e6, -1e6)
            continue
        x, y = pwx * scale, pwy * scale
        w = 1.0 / (K[2, 0] * x + K[2, 1] * y + K[2, 2])
        out[i] = ((K[0, 0] * x + K[0, 1] * y + K[0, 2]) * w, (K[1, 0] * x + K[1, 1] * y + K[1, 2]) * w)
    return out


def distort_plumb_bob(xy_norm, K, D):
    """The Brown-Conrady model undistort_plumb_bob inverts: normalised (n,2) -> pixels (n,2) f64."""
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    k1, k2, p1, p2 = (float(v) for v in D)
    x, y = xy_norm[:, 0], xy_norm[:, 1]
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([K[0, 0] * xd + K[0, 2], K[1, 1] * yd + K[1, 2]], axis=1)


def distort_equidistant(xy_norm, K, D):
    """The Kannala-Brandt model undistort_equidistant inverts: normalised -> pixels (n,2) f64."""
    K = np.asarray(K, dtype=np.float64).reshape(3, 3)
    r = np.hypot(xy_norm[:, 0], xy_norm[:, 1])
    th = np.arctan(r)
    thd = th * (1 + D[0] * th ** 2 + D[1] * th ** 4 + D[2] * th ** 6 + D[3] * th ** 8)
    s = np.where(r > 0, thd / np.where(r > 0, r, 1), 1.0)
    return np.stack([K[0, 0] * xy_norm[:, 0] * s + K[0, 2], K[1, 1] * xy_norm[:, 1] * s + K[1, 2]], axis=1)
