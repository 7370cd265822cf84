"""Oracle: the camera trajectory -- CPU PyTorch restatement of LinearTrajectory.forward (test
infrastructure only, see oracle/__init__.py), differentiable in the query timestamps through the
interpolation weight as the reference's autograd is.

Reference semantics (deblur_e_nerf/..., file:line):
* bins: right = searchsorted(T, t), left = right (t == T[0]) else right - 1   models/trajectories.py:44-58
* weight w = f32((t - T[left]) / bin_width[left])                               models/trajectories.py:60-63
* position lerp(p[left], p[right], w)                                           models/trajectories.py:65-71
* orientation: unitquat_slerp(q[left], q[right], w, shortest_path=True)         utils/tensor_ops.py:118-184
  (shortest-path flip, relative rotation as a full-angle rotation vector, scaled by w), then
  roma.unitquat_to_rotmat                                                       models/trajectories.py:81-88
RoMa is restated in oracle/roma.py (parity unpinned, see there); pinned end to end by
tests/golden/traj.npz, which the reference's LinearTrajectory produced.
"""
import torch

from . import roma


def _full_rotvec(q):
    """utils/tensor_ops.py:87-115 (unitquat_to_full_rotvec): angle in [0, 2 pi]."""
    angle = 2 * torch.atan2(torch.norm(q[:, :3], dim=1), q[:, 3])
    small = angle.abs() <= 1e-3
    scale = torch.where(small, 2 + angle ** 2 / 12 + 7 * angle ** 4 / 2880, angle / torch.sin(angle / 2))
    return scale[:, None] * q[:, :3]


def linear_trajectory(T_ts, T_pos, T_quat, t):
    """(C) i64 stamps, (C,3) positions, (C,4) XYZW quaternions, query t (...) f64 ->
    position (..., 3), rotation (..., 3, 3)."""
    shape = t.shape
    t = t.reshape(-1)
    right = torch.searchsorted(T_ts, t.detach())
    left = torch.where(t.detach() == T_ts[0], right, right - 1)
    bw = T_ts.diff()
    w = ((t - T_ts[left]) / bw[left]).to(T_pos.dtype)
    pos = torch.lerp(T_pos[left], T_pos[right], w[:, None])
    q0, q1 = T_quat[left], T_quat[right]
    q1 = torch.where((q0 * q1).sum(-1, keepdim=True) < 0, -q1, q1)
    rel = roma.quat_product(roma.quat_conjugation(q0), q1)
    rv = _full_rotvec(rel)
    q = roma.quat_product(q0, roma.rotvec_to_unitquat(w[:, None] * rv))
    rot = roma.unitquat_to_rotmat(q)
    return pos.reshape(*shape, 3), rot.reshape(*shape, 3, 3)
