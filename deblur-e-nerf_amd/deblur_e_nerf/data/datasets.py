"""On-disk formats the hot path reads -- mirror of the loaders of the reference's
data/datasets.py (Event :14-373, CameraPose :715-758) with the same file names and keys:

* ``camera_calibration.npz`` (intrinsics, bayer_pattern, contrast thresholds, refractory
  period, pixel-bandwidth constants) -- numpy, no pickles (``allow_pickle=False``);
* ``max_refractory_period.pt`` -- a tensor (``torch.load(weights_only=True)``);
* ``events.pt`` -- the queued events as a dict of tensors (position, start_ts, end_ts,
  num_pos, num_neg[, channel_idx]) (``torch.load(weights_only=True)``);
* ``camera_poses.npz`` -- T_wc_position (C, 3), T_wc_orientation (C, 4) XYZW,
  T_wc_timestamp (C) ns.

Building ``events.pt`` from ``raw_events.npz`` (the per-pixel queueing loop of
datasets.py:189-284) and the posed evaluation images are the reference's offline / eval data
path and are not rebuilt here (out of scope).
"""
import os

import numpy as np
import torch

from ..utils.easydict import EasyDict


class Event(torch.utils.data.Dataset):
    RAW_EVENTS_FILENAME = "raw_events.npz"
    TF_EVENTS_FILENAME = "events.pt"
    CAMERA_CALIBRATION_FILENAME = "camera_calibration.npz"
    MAX_REFRACTORY_PERIOD_FILENAME = "max_refractory_period.pt"
    INTRINSICS_KEY = "intrinsics"
    BAYER_PATTERN_KEY = "bayer_pattern"
    NULL_BAYER_PATTERN = ""
    BAYER_PATTERN_LEN = 4
    COLOR_CHANNEL_NAME_TO_INDEX = {"R": 0, "G": 1, "B": 2}

    def __init__(self, root_directory, permutation_seed=None):
        super().__init__()
        self.events = self.load_transformed_events(root_directory)
        if self.events is None:
            raise FileNotFoundError(f"{self.TF_EVENTS_FILENAME} not found in {root_directory}: queue the raw events "
                                    "with the reference's preprocessing first")
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
    def load_camera_calibration(cls, root_directory):
        return np.load(os.path.join(root_directory, cls.CAMERA_CALIBRATION_FILENAME), allow_pickle=False)

    @classmethod
    def load_max_refractory_period(cls, root_directory):
        path = os.path.join(root_directory, cls.MAX_REFRACTORY_PERIOD_FILENAME)
        return torch.load(path, weights_only=True) if os.path.isfile(path) else None

    @classmethod
    def save_max_refractory_period(cls, max_refractory_period, root_directory):
        torch.save(max_refractory_period, os.path.join(root_directory, cls.MAX_REFRACTORY_PERIOD_FILENAME))

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
