"""On-disk formats the hot path reads -- mirror of the reference's data/datasets.py (Event :14-373,
CameraPose :715-758) with the same file names, keys and classmethods:

* ``camera_calibration.npz`` (intrinsics, distortion, image size, bayer_pattern, contrast
  thresholds, refractory period, pixel-bandwidth constants) -- numpy, no pickles;
* ``raw_events.npz`` -- position (n, 2) uint16, timestamp (n) i64 ns, polarity (n) bool
  (scripts/preprocess_esim.py:340-345);
* ``events.pt`` -- the queued events (position, start_ts, end_ts, num_pos, num_neg[, channel_idx]),
  built from ``raw_events.npz`` on the first construction and cached (datasets.py:43-55);
* ``max_refractory_period.pt`` -- a scalar tensor, extracted from the raw events and cached the same
  way (models/event_generation_params.py:135-149);
* ``camera_poses.npz`` -- T_wc_position (C, 3), T_wc_orientation (C, 4) XYZW, T_wc_timestamp (C) ns.

The build path's per-event work (the reference's per-pixel deque loops, colorization and
undistortion) runs on the GPU in libden.so (den_queue_raw_events, den_max_refractory_period,
den_colorize_events, den_undistort_events); there is no CPU fallback.  Cached tensors are loaded
with ``torch.load(weights_only=True)``.
"""
import os

import numpy as np
import torch

from .. import _native
from ..utils.easydict import EasyDict


def _device():
    """The GPU the build-path kernels run on (the current HIP device)."""
    if not torch.cuda.is_available():
        raise _native.DenError("building events.pt / max_refractory_period.pt from raw_events.npz needs a HIP "
                               "device (libden.so; there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


class Event(torch.utils.data.Dataset):
    RAW_EVENTS_FILENAME = "raw_events.npz"
    TF_EVENTS_FILENAME = "events.pt"
    CAMERA_CALIBRATION_FILENAME = "camera_calibration.npz"
    MAX_REFRACTORY_PERIOD_FILENAME = "max_refractory_period.pt"
    RAW_EVENT_POSITION_KEY = "position"
    RAW_EVENT_TIMESTAMP_KEY = "timestamp"
    RAW_EVENT_POLARITY_KEY = "polarity"
    IMG_HEIGHT_KEY = "img_height"
    IMG_WIDTH_KEY = "img_width"
    DISTORTION_MODEL_KEY = "distortion_model"
    DISTORTION_PARAMS_KEY = "distortion_params"
    INTRINSICS_KEY = "intrinsics"
    BAYER_PATTERN_KEY = "bayer_pattern"
    NULL_BAYER_PATTERN = ""
    BAYER_PATTERN_LEN = 4
    COLOR_CHANNEL_NAME_TO_INDEX = {"R": 0, "G": 1, "B": 2}

    def __init__(self, root_directory, permutation_seed=None):
        super().__init__()
        # datasets.py:43-55: the cached transformed events, else queue + colorize + undistort + cache
        self.events = self.load_transformed_events(root_directory)
        if self.events is None:
            camera_calibration = self.load_camera_calibration(root_directory)
            events = self.queue_raw_events(root_directory, camera_calibration)
            events = self.colorize_events(events, camera_calibration)
            events = self.undistort_events(events, camera_calibration)
            self.events = EasyDict({k: v.cpu() for k, v in events.items()})
            self.save_transformed_events(self.events, root_directory)
        if permutation_seed is not None:
            g = torch.Generator()
            g.manual_seed(permutation_seed)
            perm = torch.randperm(len(self.events.position), generator=g)
            for k, v in self.events.items():
                self.events[k] = v[perm]

    @classmethod
    def load_transformed_events(cls, root_directory):
        path = os.path.join(root_directory, cls.TF_EVENTS_FILENAME)
        if not os.path.isfile(path):
            return None
        return EasyDict(torch.load(path, weights_only=True))

    @classmethod
    def save_transformed_events(cls, transformed_events, root_directory):
        torch.save(dict(transformed_events), os.path.join(root_directory, cls.TF_EVENTS_FILENAME))

    @classmethod
    def load_raw_events(cls, root_directory):
        return np.load(os.path.join(root_directory, cls.RAW_EVENTS_FILENAME), allow_pickle=False)

    @classmethod
    def load_camera_calibration(cls, root_directory):
        return np.load(os.path.join(root_directory, cls.CAMERA_CALIBRATION_FILENAME), allow_pickle=False)

    @classmethod
    def load_max_refractory_period(cls, root_directory):
        path = os.path.join(root_directory, cls.MAX_REFRACTORY_PERIOD_FILENAME)
        return torch.load(path, weights_only=True) if os.path.isfile(path) else None

    @classmethod
    def save_max_refractory_period(cls, max_refractory_period, root_directory):
        torch.save(max_refractory_period, os.path.join(root_directory, cls.MAX_REFRACTORY_PERIOD_FILENAME))

    @classmethod
    def _raw_on_device(cls, raw_events, camera_calibration):
        pos = np.asarray(raw_events[cls.RAW_EVENT_POSITION_KEY])
        ts = np.asarray(raw_events[cls.RAW_EVENT_TIMESTAMP_KEY])
        pol = np.asarray(raw_events[cls.RAW_EVENT_POLARITY_KEY])
        assert len(pos) == len(ts) == len(pol)
        if not np.issubdtype(ts.dtype, np.integer):
            raise _native.DenError(f"raw event timestamps must be integer ns, got {ts.dtype}")
        if pol.dtype != np.bool_ and not np.isin(pol, (0, 1)).all():
            raise _native.DenError("raw event polarities must be boolean (datasets.py:208 casts them to {1, 0})")
        dev = _device()
        # datasets.py:205-208: positions cast to int64, polarities {True, False} -> {1, 0}
        pos_t = torch.from_numpy(pos.astype(np.int64)).to(dev)
        ts_t = torch.from_numpy(ts.astype(np.int64)).to(dev)
        pol_t = torch.from_numpy(pol.astype(bool)).to(dev)
        H = int(camera_calibration[cls.IMG_HEIGHT_KEY])
        W = int(camera_calibration[cls.IMG_WIDTH_KEY])
        return pos_t, ts_t, pol_t, H, W, ts.dtype

    @classmethod
    def extract_max_refractory_period(cls, raw_events, camera_calibration):
        """datasets.py:133-187 on the device (den_max_refractory_period): the minimum event interval
        over the pixels' substreams -> an int64 scalar tensor, or inf (f64) when no pixel has two
        distinct timestamps, as the reference's min over np.int64 intervals from np.array(inf)."""
        pos, ts, _, H, W, _ = cls._raw_on_device(raw_events, camera_calibration)
        mx = _native.max_refractory_period(pos, ts, H, W)
        return torch.tensor(float("inf"), dtype=torch.float64) if mx is None else torch.tensor(mx, dtype=torch.int64)

    @classmethod
    def queue_raw_events(cls, root_directory, camera_calibration):
        """datasets.py:190-284 on the device (den_queue_raw_events): -> EasyDict of position (M,2) i64,
        start_ts, end_ts, num_pos, num_neg (M) in the timestamps' dtype, in input order."""
        raw = cls.load_raw_events(root_directory)
        pos, ts, pol, H, W, ts_dtype = cls._raw_on_device(raw, camera_calibration)
        queued, _ = _native.queue_raw_events(pos, ts, pol, H, W)
        tdt = torch.from_numpy(np.zeros(0, dtype=ts_dtype)).dtype  # np.empty_like(timestamps) (:224-227)
        for k in ("start_ts", "end_ts", "num_pos", "num_neg"):
            queued[k] = queued[k].to(tdt)
        return EasyDict(queued)

    @classmethod
    def colorize_events(cls, events, camera_calibration):
        """datasets.py:287-328: channel_idx (u8) from the bayer pattern (den_colorize_events);
        a monochrome camera ("") keeps the events as they are."""
        bayer_pattern = str(camera_calibration[cls.BAYER_PATTERN_KEY])
        assert len(bayer_pattern) in (len(cls.NULL_BAYER_PATTERN), cls.BAYER_PATTERN_LEN)
        if bayer_pattern == cls.NULL_BAYER_PATTERN:
            return events
        assert set(cls.COLOR_CHANNEL_NAME_TO_INDEX.keys()) == set(bayer_pattern)
        channels = [cls.COLOR_CHANNEL_NAME_TO_INDEX[c] for c in bayer_pattern]
        events.channel_idx = _native.colorize_events(events.position, channels)
        return events

    @classmethod
    def undistort_events(cls, events, camera_calibration):
        """datasets.py:331-364 (den_undistort_events): positions to the default dtype, then the
        plumb_bob / equidistant undistortion with P = intrinsics when distortion parameters exist
        (OpenCV's iterations restated; parity unpinned, OpenCV is not in this image)."""
        params = np.asarray(camera_calibration[cls.DISTORTION_PARAMS_KEY]) \
            if cls.DISTORTION_PARAMS_KEY in camera_calibration else np.zeros(0, dtype=np.float32)
        assert len(params) in (0, 4)
        model = str(camera_calibration[cls.DISTORTION_MODEL_KEY]) if len(params) else None
        intrinsics = camera_calibration[cls.INTRINSICS_KEY] if len(params) else np.eye(3, dtype=np.float32)
        pos = events.position
        if pos.dtype != torch.int64:
            raise _native.DenError("undistort_events expects the queued int64 positions")
        out = _native.undistort_events(pos, model, intrinsics, params)
        events.position = out.to(torch.get_default_dtype())
        return events

    def __getitem__(self, index):
        return {k: v[index] for k, v in self.events.items()}

    def __len__(self):
        return len(self.events.position)


class CameraPose(torch.utils.data.Dataset):
    CAMERA_POSES_FILENAME = "camera_poses.npz"
    CAMERA_POSES_KEYS = {"T_wc_position", "T_wc_orientation", "T_wc_timestamp"}

    def __init__(self, root_directory, permutation_seed=None):
        super().__init__()
        self.camera_poses = self.load_camera_poses(root_directory)
        if permutation_seed is None:
            return
        g = torch.Generator()
        g.manual_seed(permutation_seed)
        perm = torch.randperm(len(self.camera_poses.T_wc_position), generator=g)
        for k, v in self.camera_poses.items():
            self.camera_poses[k] = v[perm]

    @classmethod
    def load_camera_poses(cls, root_directory):
        poses = EasyDict(dict(np.load(os.path.join(root_directory, cls.CAMERA_POSES_FILENAME), allow_pickle=False)))
        assert set(poses.keys()) == cls.CAMERA_POSES_KEYS
        for k, v in poses.items():
            poses[k] = torch.tensor(v)
        return poses

    @classmethod
    def from_arrays(cls, T_wc_position, T_wc_orientation, T_wc_timestamp):
        """A CameraPose from in-memory arrays (synthetic scenes, tests)."""
        obj = cls.__new__(cls)
        torch.utils.data.Dataset.__init__(obj)
        obj.camera_poses = EasyDict(T_wc_position=torch.as_tensor(T_wc_position),
                                    T_wc_orientation=torch.as_tensor(T_wc_orientation),
                                    T_wc_timestamp=torch.as_tensor(T_wc_timestamp))
        return obj

    def __getitem__(self, index):
        return {k: v[index] for k, v in self.camera_poses.items()}

    def __len__(self):
        return len(self.camera_poses.T_wc_position)
