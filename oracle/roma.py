"""Oracle: the RoMa 1.2.7 quaternion helpers the reference's trajectory uses -- CPU restatement
(test infrastructure only, see oracle/__init__.py).

RoMa (naver/roma 1.2.7, environment.yml) is not installed here (no network).  The reference
calls it from models/trajectories.py:81-88 and utils/tensor_ops.py:98-184.  Restated from RoMa's
published implementation (XYZW quaternions; the SciPy-derived small-angle series):

* ``quat_product(p, q)``      xyz = p_w q_xyz + q_w p_xyz + p_xyz x q_xyz, w = p_w q_w - p.q
* ``quat_conjugation(q)``     (-x, -y, -z, w)
* ``rotvec_to_unitquat(v)``   theta = |v|; xyz = s v with s = 1/2 - theta^2/48 + theta^4/3840
                              (theta <= 1e-3) else sin(theta/2)/theta; w = cos(theta/2)
* ``unitquat_to_rotmat(q)``   the standard (x^2 - y^2 - z^2 + w^2, 2(xy - zw), ...) matrix
* ``internal.flatten_batch_dims`` / ``unflatten_batch_dims``

Parity of this restatement against RoMa itself is UNPINNED (no RoMa output exists in the
reference tree); it stands in for RoMa when tests/golden/make_golden.py runs the reference's
LinearTrajectory / unitquat_slerp, whose own logic (searchsorted, lerp, shortest path, the
full-angle rotvec) is what the trajectory fixture pins.
"""
import types

import torch


def flatten_batch_dims(tensor, end_dim):
    batch_shape = tensor.shape[:end_dim + 1]
    flattened = tensor.flatten(end_dim=end_dim) if len(batch_shape) > 0 else tensor.unsqueeze(0)
    return flattened, batch_shape


def unflatten_batch_dims(tensor, batch_shape):
    return tensor.reshape(batch_shape + tensor.shape[1:]) if len(batch_shape) > 0 else tensor.squeeze(0)


internal = types.SimpleNamespace(flatten_batch_dims=flatten_batch_dims, unflatten_batch_dims=unflatten_batch_dims)


def quat_conjugation(quat):
    inv = quat.clone()
    inv[..., :3] *= -1
    return inv


def quat_product(p, q):
    vector = p[..., 3:4] * q[..., :3] + q[..., 3:4] * p[..., :3] + torch.cross(p[..., :3], q[..., :3], dim=-1)
    last = p[..., 3:4] * q[..., 3:4] - torch.sum(p[..., :3] * q[..., :3], dim=-1, keepdim=True)
    return torch.cat((vector, last), dim=-1)


def rotvec_to_unitquat(rotvec):
    rotvec, batch_shape = flatten_batch_dims(rotvec, end_dim=-2)
    num_rotations, D = rotvec.shape
    assert D == 3
    norms = torch.norm(rotvec, dim=-1)
    small_angle = norms <= 1e-3
    large_angle = ~small_angle
    scale = torch.empty((num_rotations,), device=rotvec.device, dtype=rotvec.dtype)
    scale[small_angle] = 0.5 - norms[small_angle] ** 2 / 48 + norms[small_angle] ** 4 / 3840
    scale[large_angle] = torch.sin(norms[large_angle] / 2) / norms[large_angle]
    quat = torch.empty((num_rotations, 4), device=rotvec.device, dtype=rotvec.dtype)
    quat[:, :3] = scale[:, None] * rotvec
    quat[:, 3] = torch.cos(norms / 2)
    return unflatten_batch_dims(quat, batch_shape)


def unitquat_to_rotmat(quat):
    quat, batch_shape = flatten_batch_dims(quat, end_dim=-2)
    num_rotations, D = quat.shape
    assert D == 4
    x, y, z, w = quat[:, 0], quat[:, 1], quat[:, 2], quat[:, 3]
    x2, y2, z2, w2 = x * x, y * y, z * z, w * w
    xy, zw, xz, yw, yz, xw = x * y, z * w, x * z, y * w, y * z, x * w
    m = torch.empty((num_rotations, 3, 3), dtype=quat.dtype, device=quat.device)
    m[:, 0, 0] = x2 - y2 - z2 + w2
    m[:, 1, 0] = 2 * (xy + zw)
    m[:, 2, 0] = 2 * (xz - yw)
    m[:, 0, 1] = 2 * (xy - zw)
    m[:, 1, 1] = -x2 + y2 - z2 + w2
    m[:, 2, 1] = 2 * (yz + xw)
    m[:, 0, 2] = 2 * (xz + yw)
    m[:, 1, 2] = 2 * (yz - xw)
    m[:, 2, 2] = -x2 - y2 + z2 + w2
    return unflatten_batch_dims(m, batch_shape)


def as_module():
    """A module object standing in for ``roma`` (test-only, tests/golden/_refload.py)."""
    m = types.ModuleType("roma")
    for name in ("quat_conjugation", "quat_product", "rotvec_to_unitquat", "unitquat_to_rotmat"):
        setattr(m, name, globals()[name])
    m.internal = internal
    return m
