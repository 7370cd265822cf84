"""Oracle: the packed rendering path the reference takes through nerfacc 0.3.1 -- CPU
restatement (test infrastructure only, see oracle/__init__.py; never imported by the product).

nerfacc 0.3.1 (pinned in the reference's environment.yml:32) is a CUDA extension that is not
vendored in /root/reference and cannot be installed here (no network), so its published
algorithm is restated:

* ``ray_aabb_intersect``  -- slab test, misses -> (1e10, 1e10)
* ``ray_marching``        -- t range (AABB / [0, 1e10], near/far clamp, stratified offset), the
  per-ray march with step clamp(t * cone_angle, step, 1e10), occupancy test at the segment
  midpoint after the scene contraction, the DDA skip (advance_to_next_voxel) for the AABB
  contraction, then the visibility filter (exclusive cumprod of 1 - alpha >= early_stop_eps,
  alpha >= alpha_thre)
* ``render_weight_from_density`` / ``accumulate_along_rays`` -- per-ray exclusive sums
* ``OccupancyGrid``       -- EMA update of nerfacc's ``_update`` (all cells below warmup_steps,
  jittered cell points, contract_inv, ``max(occ * decay, new)``, mean threshold)

Call sites in the reference: external/utils.py:106-119, external/vol_rendering.py:89-126,
models/nerf.py:98-102, 170-204.  The marching is sequential float32 arithmetic per ray (numpy
f32 scalars, no fused multiply-add), the same operation order as den_march.hip, so the packed
samples are bit-comparable.  Parity of this restatement against nerfacc itself is UNPINNED (no
nerfacc output exists in the reference tree); it is pinned through the reference's own glue
(tests/golden/make_golden.py runs vol_rendering.rendering, utils.render_image and NeRF.forward of
the reference with these functions standing in for the nerfacc module).
"""
import enum
import math

import numpy as np
import torch

f32 = np.float32
FAR = f32(1e10)
LAST = {}  # the random draws and samples of the latest ray_marching call (fixture generation)


class ContractionType(enum.Enum):
    AABB = 0
    UN_BOUNDED_TANH = 1
    UN_BOUNDED_SPHERE = 2


def _cid(ct):
    return {"AABB": 0, "UN_BOUNDED_TANH": 1, "UN_BOUNDED_SPHERE": 2}[getattr(ct, "name", str(ct)).split(".")[-1]]


# ----------------------------------------------------------------------------- marching
def ray_aabb_intersect_np(o, d, aabb):
    with np.errstate(divide="ignore", invalid="ignore"):
        tmin = (aabb[0] - o[0]) / d[0]
        tmax = (aabb[3] - o[0]) / d[0]
        if tmin > tmax:
            tmin, tmax = tmax, tmin
        tymin = (aabb[1] - o[1]) / d[1]
        tymax = (aabb[4] - o[1]) / d[1]
        if tymin > tymax:
            tymin, tymax = tymax, tymin
        if tmin > tymax or tymin > tmax:
            return FAR, FAR
        if tymin > tmin:
            tmin = tymin
        if tymax < tmax:
            tmax = tymax
        tzmin = (aabb[2] - o[2]) / d[2]
        tzmax = (aabb[5] - o[2]) / d[2]
        if tzmin > tzmax:
            tzmin, tzmax = tzmax, tzmin
        if tmin > tzmax or tzmin > tmax:
            return FAR, FAR
        if tzmin > tmin:
            tmin = tzmin
        if tzmax < tmax:
            tmax = tzmax
    return tmin, tmax


def march_prep(o, d, aabb=None, near=None, far=None, jitter=None, step=1e-3):
    """-> t_min, t_max (R) f32 (ray_marching's prologue)."""
    o, d = np.asarray(o, f32), np.asarray(d, f32)
    R = o.shape[0]
    tmin = np.zeros(R, f32)
    tmax = np.full(R, FAR, f32)
    ab = None if aabb is None else np.asarray(aabb, f32)
    for i in range(R):
        if ab is not None:
            tmin[i], tmax[i] = ray_aabb_intersect_np(o[i], d[i], ab)
        if near is not None:
            tmin[i] = max(tmin[i], f32(near))
        if far is not None:
            tmax[i] = min(tmax[i], f32(far))
        if jitter is not None:
            tmin[i] = tmin[i] + f32(jitter[i]) * f32(step)
    return tmin, tmax


def _grid_unit(xyz, roi, ctype):
    u = [(xyz[a] - roi[a]) / (roi[3 + a] - roi[a]) for a in range(3)]
    if ctype == 2:
        u = [v * f32(2) - f32(1) for v in u]
        n = np.sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2], dtype=f32)
        if n > f32(1):
            s = f32(2) - f32(1) / n
            u = [s * (v / n) for v in u]
        u = [v * f32(0.25) + f32(0.5) for v in u]
    elif ctype == 1:
        u = [f32(math.tanh(v - f32(0.5))) * f32(0.5) + f32(0.5) for v in u]
    return u


def _occupied(xyz, grid, roi, res, ctype):
    if grid is None:
        return True
    if ctype == 0 and any(xyz[a] < roi[a] or xyz[a] > roi[3 + a] for a in range(3)):
        return False
    u = _grid_unit(xyz, roi, ctype)
    ix = [min(max(int(np.trunc(u[a] * f32(res[a]))), 0), res[a] - 1) for a in range(3)]
    return bool(grid[ix[0], ix[1], ix[2]])


def _dt(t, cone, dt_min):
    return min(max(t * f32(cone), dt_min), FAR)


def _advance(t, dt_min, xyz, d, inv, roi, res, far):
    tx = []
    for a in range(3):
        span = roi[3 + a] - roi[a]
        r = f32(res[a])
        x = ((xyz[a] - roi[a]) / span) * r
        sgn = f32(math.copysign(1.0, float(d[a])))
        with np.errstate(invalid="ignore", over="ignore"):
            tx.append(((np.floor(x + f32(0.5) + f32(0.5) * sgn) - x) * inv[a]) / r * span)
    dist = np.fmax(np.fmin(np.fmin(tx[0], tx[1]), tx[2]), f32(0))
    target = t + dist
    if not (target <= far):
        target = far + dt_min
    while True:
        t = t + dt_min
        if not (t < target):
            break
    return t


def march_ray(o, d, tmin, tmax, grid=None, roi=None, res=None, ctype=0, step=1e-3, cone=0.0, max_iter=1 << 20):
    """One ray of nerfacc's ray_marching kernel -> list of (t0, t1) f32."""
    o, d = np.asarray(o, f32), np.asarray(d, f32)
    roi = None if roi is None else np.asarray(roi, f32)
    with np.errstate(divide="ignore"):
        inv = [f32(1) / d[a] for a in range(3)]
    dt_min = f32(step)
    near, far = f32(tmin), f32(tmax)
    out = []
    t0 = near
    t1 = t0 + _dt(t0, cone, dt_min)
    tm = (t0 + t1) * f32(0.5)
    it = 0
    while tm < far and it < max_iter:
        it += 1
        xyz = [o[a] + tm * d[a] for a in range(3)]
        if _occupied(xyz, grid, roi, res, ctype):
            out.append((t0, t1))
            t0 = t1
            t1 = t0 + _dt(t0, cone, dt_min)
            tm = (t0 + t1) * f32(0.5)
        elif ctype == 0:
            tm = _advance(tm, dt_min, xyz, d, inv, roi, res, far)
            dt = _dt(tm, cone, dt_min)
            t0 = tm - dt * f32(0.5)
            t1 = tm + dt * f32(0.5)
        else:
            t0 = t1
            t1 = t0 + _dt(t0, cone, dt_min)
            tm = (t0 + t1) * f32(0.5)
    return out


def march(o, d, tmin, tmax, grid=None, roi=None, res=None, ctype=0, step=1e-3, cone=0.0):
    """All rays -> ray_indices (n) i32, t_starts (n) f32, t_ends (n) f32, counts (R)."""
    ri, a0, a1, counts = [], [], [], []
    for i in range(len(tmin)):
        segs = march_ray(o[i], d[i], tmin[i], tmax[i], grid, roi, res, ctype, step, cone)
        counts.append(len(segs))
        for t0, t1 in segs:
            ri.append(i)
            a0.append(t0)
            a1.append(t1)
    return (np.asarray(ri, np.int32), np.asarray(a0, f32), np.asarray(a1, f32), np.asarray(counts, np.int32))


def visibility(ray_indices, t_starts, t_ends, sigmas=None, alphas=None, early_stop_eps=1e-4, alpha_thre=0.0):
    """render_visibility: exclusive cumprod of (1 - alpha) per ray (float64 here) -> keep mask,
    transmittance (for tolerance-aware comparisons)."""
    ri = np.asarray(ray_indices)
    if sigmas is not None:
        a = 1.0 - np.exp(-(np.asarray(sigmas, np.float64) * (np.asarray(t_ends, np.float64)
                                                            - np.asarray(t_starts, np.float64))))
    else:
        a = np.asarray(alphas, np.float64)
    T = np.empty_like(a)
    run, prev = 1.0, None
    for s in range(len(ri)):
        if ri[s] != prev:
            run, prev = 1.0, ri[s]
        T[s] = run
        run *= 1.0 - a[s]
    keep = T >= early_stop_eps
    if alpha_thre > 0:
        keep &= a >= alpha_thre
    return keep, T


def ray_marching(rays_o, rays_d, t_min=None, t_max=None, scene_aabb=None, grid=None, sigma_fn=None, alpha_fn=None,
                 early_stop_eps=1e-4, alpha_thre=0.0, near_plane=None, far_plane=None, render_step_size=1e-3,
                 stratified=False, cone_angle=0.0, jitter=None):
    """nerfacc.ray_marching with torch in / out (CPU).  ``jitter``: the U[0,1) draws of the
    stratified offset (default torch.rand_like, as nerfacc)."""
    o = rays_o.detach().float().cpu().numpy()
    d = rays_d.detach().float().cpu().numpy()
    R = o.shape[0]
    if stratified and jitter is None:
        jitter = torch.rand(R)
    LAST["jitter"] = None if not stratified else torch.as_tensor(jitter).clone()
    jit = None if not stratified else np.asarray(jitter, f32)
    if t_min is None or t_max is None:
        ab = None if scene_aabb is None else scene_aabb.detach().float().cpu().numpy()
        tmin, tmax = march_prep(o, d, ab, near_plane, far_plane, jit, render_step_size)
    else:
        raise NotImplementedError("explicit t_min / t_max are not used by the reference's call sites")
    if grid is not None:
        g = grid.binary.detach().cpu().numpy()
        roi = grid.roi_aabb.detach().float().cpu().numpy()
        res = [int(r) for r in grid.resolution]
        ctype = _cid(grid.contraction_type)
    else:
        g, roi, res, ctype = None, None, None, 0
    ri, a0, a1, _ = march(o, d, tmin, tmax, g, roi, res, ctype, f32(render_step_size), cone_angle)
    LAST.update(marched=(ri.copy(), a0.copy(), a1.copy()), t_min=tmin.copy(), t_max=tmax.copy())
    ray_indices = torch.from_numpy(ri)
    t_starts = torch.from_numpy(a0)[:, None]
    t_ends = torch.from_numpy(a1)[:, None]
    if (alpha_thre > 0.0 or early_stop_eps > 0.0) and (sigma_fn is not None or alpha_fn is not None) \
            and len(ri) > 0:
        with torch.no_grad():
            if sigma_fn is not None:
                sig = sigma_fn(t_starts, t_ends, ray_indices).reshape(-1).numpy()
                keep, _ = visibility(ri, a0, a1, sigmas=sig, early_stop_eps=early_stop_eps, alpha_thre=alpha_thre)
            else:
                alp = alpha_fn(t_starts, t_ends, ray_indices).reshape(-1).numpy()
                keep, _ = visibility(ri, a0, a1, alphas=alp, early_stop_eps=early_stop_eps, alpha_thre=alpha_thre)
        k = torch.from_numpy(keep)
        ray_indices, t_starts, t_ends = ray_indices[k], t_starts[k], t_ends[k]
        LAST["prepass_sigma"] = sig if sigma_fn is not None else None
    LAST["kept"] = (ray_indices.clone(), t_starts.clone(), t_ends.clone())
    return ray_indices, t_starts, t_ends


# ----------------------------------------------------------------------------- compositing
def _segments(ray_indices):
    ri = ray_indices.tolist()
    segs, s = [], 0
    for i in range(1, len(ri) + 1):
        if i == len(ri) or ri[i] != ri[s]:
            segs.append((s, i))
            s = i
    return segs


def render_weight_from_density(t_starts, t_ends, sigmas, *, packed_info=None, ray_indices=None, n_rays=None):
    """w_i = exp(-sum_{j<i} sigma_j dt_j) (1 - exp(-sigma_i dt_i)), per ray (torch, differentiable)."""
    sdt = (sigmas * (t_ends - t_starts))[:, 0]
    parts = []
    for s, e in _segments(ray_indices):
        c = torch.cumsum(sdt[s:e], 0)
        parts.append(torch.cat([c.new_zeros(1), c[:-1]]))
    excl = torch.cat(parts) if parts else sdt.new_zeros(0)
    return (torch.exp(-excl) * (1.0 - torch.exp(-sdt)))[:, None]


def render_weight_from_alpha(alphas, *, packed_info=None, ray_indices=None, n_rays=None):
    raise NotImplementedError("not used by the reference's call sites")


def accumulate_along_rays(weights, ray_indices, values=None, n_rays=None):
    src = weights * values if values is not None else weights
    if ray_indices.numel() == 0:
        return torch.zeros((n_rays, src.shape[-1]), dtype=src.dtype)
    if n_rays is None:
        n_rays = int(ray_indices.max()) + 1
    index = ray_indices.long()[:, None].expand(-1, src.shape[-1])
    out = torch.zeros((n_rays, src.shape[-1]), dtype=src.dtype)
    return out.scatter_add(0, index, src)


def composite_packed(t_starts, t_ends, ray_indices, n_rays, sigmas, rgbs, bkgd=None):
    """vol_rendering.rendering after rgb_sigma_fn: -> colours (R, rd), opacities (R, 1), depths (R, 1)."""
    w = render_weight_from_density(t_starts, t_ends, sigmas, ray_indices=ray_indices, n_rays=n_rays)
    col = accumulate_along_rays(w, ray_indices, values=rgbs, n_rays=n_rays)
    op = accumulate_along_rays(w, ray_indices, values=None, n_rays=n_rays)
    dp = accumulate_along_rays(w, ray_indices, values=(t_starts + t_ends) / 2.0, n_rays=n_rays)
    if bkgd is not None:
        col = col + bkgd * (1.0 - op)
    return col, op, dp


# ----------------------------------------------------------------------------- occupancy grid
class OccupancyGrid(torch.nn.Module):
    """nerfacc.OccupancyGrid (0.3.1) restated on the CPU.  ``_update`` takes the cell jitter
    ``u`` (m, 3) explicitly when given (nerfacc draws torch.rand_like) and applies nerfacc's
    gather-then-scatter EMA ``occs[idx] = max(occs[idx] * decay, occ)``."""

    def __init__(self, roi_aabb, resolution=128, contraction_type=ContractionType.AABB):
        super().__init__()
        if isinstance(resolution, int):
            resolution = [resolution] * 3
        self.register_buffer("resolution", torch.tensor(resolution, dtype=torch.int32))
        self.register_buffer("_roi_aabb", torch.as_tensor(roi_aabb, dtype=torch.float32))
        self.num_cells = int(np.prod(resolution))
        self.register_buffer("occs", torch.zeros(self.num_cells))
        self.register_buffer("_binary", torch.zeros(tuple(resolution), dtype=torch.bool))
        grid = torch.stack(torch.meshgrid(*[torch.arange(r) for r in resolution], indexing="ij"), -1)
        self.register_buffer("grid_coords", grid.reshape(-1, 3))
        self._contraction_type = contraction_type
        self.last_u = None

    roi_aabb = property(lambda self: self._roi_aabb)
    binary = property(lambda self: self._binary)
    contraction_type = property(lambda self: self._contraction_type)

    def cell_points(self, indices, u):
        """-> world points (m, 3) f32 and the unit-sphere mask (sphere contraction)."""
        res = self.resolution.float()
        x = ((self.grid_coords[indices].float() + u) / res).numpy().astype(f32)
        roi = self._roi_aabb.numpy()
        ct = _cid(self._contraction_type)
        mask = np.ones(len(x), bool)
        if ct == 2:
            y = x - f32(0.5)
            mask = np.sqrt((y * y).sum(-1, dtype=f32), dtype=f32) < f32(0.5)
            f = y * f32(4)
            n = np.sqrt((f * f).sum(-1, dtype=f32), dtype=f32)[:, None]
            with np.errstate(divide="ignore", invalid="ignore"):
                f = np.where(n > 1, f / (n * (f32(2) - n)), f)
            x = f * f32(0.5) + f32(0.5)
        elif ct == 1:
            with np.errstate(divide="ignore"):
                x = np.arctanh(x * f32(2) - f32(1)).astype(f32) + f32(0.5)
        pts = x * (roi[3:] - roi[:3]) + roi[:3]
        return torch.from_numpy(pts.astype(f32)), torch.from_numpy(mask)

    @torch.no_grad()
    def _update(self, step, occ_eval_fn, occ_thre=0.01, ema_decay=0.95, warmup_steps=256, u=None, indices=None):
        if indices is None:
            if step >= warmup_steps:
                raise NotImplementedError("pass the sampled cell indices explicitly after warm-up")
            indices = torch.arange(self.num_cells)
        if u is None:
            u = torch.rand(len(indices), 3)
        self.last_u = u
        pts, mask = self.cell_points(indices, u)
        if _cid(self._contraction_type) == 2:
            pts, indices = pts[mask], indices[mask]
        occ = occ_eval_fn(pts).squeeze(-1)
        self.occs[indices] = torch.maximum(self.occs[indices] * ema_decay, occ)
        self._binary = (self.occs > torch.clamp(self.occs.mean(), max=occ_thre)).view(self._binary.shape)

    @torch.no_grad()
    def every_n_step(self, step, occ_eval_fn, occ_thre=1e-2, ema_decay=0.95, warmup_steps=256, n=16):
        if step % n == 0 and self.training:
            self._update(step=step, occ_eval_fn=occ_eval_fn, occ_thre=occ_thre, ema_decay=ema_decay,
                         warmup_steps=warmup_steps)
