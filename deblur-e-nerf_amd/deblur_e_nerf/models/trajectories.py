"""Camera trajectory -- mirror of the reference's models/trajectories.py (LinearTrajectory,
:8-90): the pose at any timestamp by linear interpolation of the position and shortest-path
slerp of the orientation between the two bracketing pose samples.

Same constructor (a ``datasets.CameraPose``-like object holding ``camera_poses.T_wc_position``
(C, 3), ``T_wc_orientation`` (C, 4) XYZW quaternions and ``T_wc_timestamp`` (C) ns), the same
buffers (``T_wc_position``, ``T_wc_orientation_quat``, ``T_wc_timestamp``, ``bin_width``) and
the same ``forward(input_timestamp) -> (position (..., 3), orientation (..., 3, 3))``.  The
arithmetic (searchsorted, lerp, slerp with RoMa's formulas, quaternion -> matrix) is one HIP
kernel, den_trajectory; its reverse mode with respect to the query timestamps (den_trajectory_bwd)
carries the refractory period's gradient from the poses back to the render timestamps, as the
reference's autograd does through the interpolation weight.
"""
import torch

from .. import _native


class LinearTrajectory(torch.nn.Module):
    def __init__(self, camera_poses):
        super().__init__()
        cp = camera_poses.camera_poses
        self.register_buffer("T_wc_position", torch.as_tensor(cp.T_wc_position), persistent=False)
        self.register_buffer("T_wc_orientation_quat", torch.as_tensor(cp.T_wc_orientation), persistent=False)
        self.register_buffer("T_wc_timestamp", torch.as_tensor(cp.T_wc_timestamp).contiguous(), persistent=False)
        self.register_buffer("bin_width", self.T_wc_timestamp.diff(), persistent=False)
        self._status = None

    def forward(self, input_timestamp):
        dev = self.T_wc_position.device
        if self._status is None or self._status.device != dev:
            self._status = torch.zeros(1, dtype=torch.int32, device=dev)
        return _native.trajectory(self.T_wc_timestamp, self.T_wc_position, self.T_wc_orientation_quat,
                                  input_timestamp, self._status)

    def check(self):
        """The reference asserts every query lies inside the pose span (trajectories.py:55-58);
        the kernel records violations in a device flag instead of syncing per call: raise here."""
        if self._status is not None and int(self._status.item()) != 0:
            self._status.zero_()
            raise AssertionError("LinearTrajectory: a timestamp outside [T_wc_timestamp[0], T_wc_timestamp[-1]]")
