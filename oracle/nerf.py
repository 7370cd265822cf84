"""Oracle: vanilla-NeRF radiance field, fixed-count stratified sampler, nerfacc
compositing -- CPU PyTorch restatement (test infrastructure, see __init__).

Reference semantics followed (file:line under /root/reference):
* AABB contraction + selector       deblur_e_nerf/external/mlp.py:321-335
* sinusoidal encoder (scale-major)  deblur_e_nerf/external/mlp.py:227-243
* view-direction scaling by pi      deblur_e_nerf/external/mlp.py:353-355
* 8x256 skip MLP / heads            deblur_e_nerf/external/mlp.py:99-113, 193-205
* softplus(beta=100) hidden act     deblur_e_nerf/models/nerf.py:18
* shifted_trunc_exp density         deblur_e_nerf/external/ngp.py:45-65, nerf.py:22
* softplus(beta=1) radiance         deblur_e_nerf/models/nerf.py:27
* sample positions o + d*(t0+t1)/2  deblur_e_nerf/external/utils.py:83-96
* compositing (nerfacc 0.3.1)       deblur_e_nerf/external/vol_rendering.py:81-126
* NeRF.forward tail                 deblur_e_nerf/models/nerf.py:279-286
* intensity = radiance + min_int    deblur_e_nerf/models/deblur_e_nerf.py:1196-1207

The sampler is the build's fixed-count stratified scheme:
per ray [t_min, t_max] = AABB (slab test) intersected with [near, far];
N strata of width dt = (t_max - t_min)/N; sample k has midpoint
t_min + ((k + u)/N)*(t_max - t_min) with one jitter u per ray, and interval
[mid - dt/2, mid + dt/2].  A ray missing the box gets dt = 0 (zero weights).
"""
import math

import torch

AABB_CHAIR = (-1.5, -1.5, -1.5, 1.5, 1.5, 1.5)


# ----------------------------------------------------------------------------- parameters
def layer_specs(rd, width=256, depth=8, skip=4, width_cond=128, pos_deg=10, view_deg=4):
    """(name, in_features, out_features) in the reference's construction order
    (external/mlp.py:56-76 base, :155-186 heads)."""
    pos_dim = 3 * (1 + 2 * pos_deg)
    view_dim = 3 * (1 + 2 * view_deg)
    specs = []
    fin = pos_dim
    for i in range(depth):
        specs.append((f"mlp.base.hidden_layers.{i}", fin, width))
        fin = width + pos_dim if (skip is not None and i % skip == 0 and i > 0) else width
    specs.append(("mlp.sigma_layer.output_layer", fin, 1))
    specs.append(("mlp.bottleneck_layer.output_layer", fin, width))
    specs.append(("mlp.rgb_layer.hidden_layers.0", width + view_dim, width_cond))
    specs.append(("mlp.rgb_layer.output_layer", width_cond, rd))
    return specs


def build_params(rd, seed, dtype=torch.float32):
    """Weights exactly as the reference creates them: PyTorch default nn.Linear
    init (hidden_init=None, mlp.py:297-299) in construction order under
    torch.manual_seed(seed)."""
    torch.manual_seed(seed)
    params = {}
    for name, fin, fout in layer_specs(rd):
        lin = torch.nn.Linear(fin, fout)
        params[name + ".weight"] = lin.weight.detach().to(dtype).clone()
        params[name + ".bias"] = lin.bias.detach().to(dtype).clone()
    return params


# ----------------------------------------------------------------------------- field
def softplus100(z):
    return torch.nn.functional.softplus(z, beta=100, threshold=20)


class _TruncExp(torch.autograd.Function):
    """exp(x) whose backward clamps the exponent at 15 (external/ngp.py:45-61)."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.exp(torch.clamp(x, max=15))


def encode(v, n_deg):
    """[v, sin(v*2^k), sin(v*2^k + pi/2)], scale-major / dim-minor ordering."""
    scales = torch.tensor([2 ** k for k in range(n_deg)])
    xb = (v[..., None, :] * scales[:, None]).reshape(*v.shape[:-1], 3 * n_deg)
    return torch.cat([v, torch.sin(torch.cat([xb, xb + 0.5 * math.pi], dim=-1))], dim=-1)


def contract_aabb(x, aabb):
    lo = torch.tensor(aabb[:3], dtype=x.dtype)
    hi = torch.tensor(aabb[3:], dtype=x.dtype)
    xh = (x - lo) / (hi - lo)
    sel = ((xh > 0.0) & (xh < 1.0)).all(dim=-1)
    return 2 * math.pi * (xh - 0.5), sel


def contract_unbounded(x, aabb, kind):
    """The unbounded input-space contractions of VanillaNeRFRadianceField.contract_input_space
    (mlp.py:321-335): "sphere" = ngp.py:68-93 contract_to_unisphere (box at [-1, 1], outside the unit
    ball x -> (2 - 1/|x|) x/|x|, then /4 + 1/2), "tanh" = ngp.py:96-106 contract_tanh; then the same
    selector and [-pi, pi] map as the AABB case."""
    lo = torch.tensor(aabb[:3], dtype=x.dtype)
    hi = torch.tensor(aabb[3:], dtype=x.dtype)
    xh = (x - lo) / (hi - lo)
    if kind == "sphere":
        xh = xh * 2 - 1
        mag = xh.norm(dim=-1, keepdim=True)
        xh = torch.where(mag > 1, (2 - 1 / mag) * (xh / mag), xh)
        xh = xh / 4 + 0.5
    elif kind == "tanh":
        xh = (torch.tanh(xh - 0.5) + 1) / 2
    else:
        raise ValueError(kind)
    sel = ((xh > 0.0) & (xh < 1.0)).all(dim=-1)
    return 2 * math.pi * (xh - 0.5), sel


def _lin(p, name, h):
    return torch.nn.functional.linear(h, p[name + ".weight"], p[name + ".bias"])


def density_activation(raw, kind="shifted_trunc_exp"):
    """models/nerf.py:20-29: shifted_trunc_exp (external/ngp.py:45-65), softplus(beta 1), or
    shifted_softplus (softplus(x - 1))."""
    if kind == "shifted_trunc_exp":
        return _TruncExp.apply(raw - 1)
    if kind == "softplus":
        return torch.nn.functional.softplus(raw, beta=1, threshold=20)
    if kind == "shifted_softplus":
        return torch.nn.functional.softplus(raw - 1, beta=1, threshold=20)
    raise ValueError(kind)


def radiance_field(p, x, d, aabb=AABB_CHAIR, depth=8, skip=4, contraction="aabb", density="shifted_trunc_exp"):
    """VanillaNeRFRadianceField.forward(x, d) -> (rgb (n, rd), sigma (n, 1))."""
    xc, sel = contract_aabb(x, aabb) if contraction == "aabb" else contract_unbounded(x, aabb, contraction)
    pe = encode(xc, 10)
    h = pe
    for i in range(depth):
        h = softplus100(_lin(p, f"mlp.base.hidden_layers.{i}", h))
        if i % skip == 0 and i > 0:
            h = torch.cat([h, pe], dim=-1)
    sigma_raw = _lin(p, "mlp.sigma_layer.output_layer", h)
    ve = encode(d * math.pi, 4)
    bott = _lin(p, "mlp.bottleneck_layer.output_layer", h)
    g = softplus100(_lin(p, "mlp.rgb_layer.hidden_layers.0", torch.cat([bott, ve], dim=-1)))
    rgb_raw = _lin(p, "mlp.rgb_layer.output_layer", g)
    rgb = torch.nn.functional.softplus(rgb_raw, beta=1, threshold=20)
    sigma = density_activation(sigma_raw, density) * sel[..., None]
    return rgb, sigma


# ----------------------------------------------------------------------------- sampler
def ray_aabb_tmin_tmax(o, d, aabb, near, far):
    """Slab test (nerfacc ray_aabb_intersect) clipped to [near, far]."""
    lo = torch.tensor(aabb[:3], dtype=o.dtype)
    hi = torch.tensor(aabb[3:], dtype=o.dtype)
    inv = 1.0 / d
    t1 = (lo - o) * inv
    t2 = (hi - o) * inv
    tmin = torch.minimum(t1, t2).amax(dim=-1)
    tmax = torch.maximum(t1, t2).amin(dim=-1)
    if near is not None:
        tmin = torch.clamp(tmin, min=near)
    if far is not None:
        tmax = torch.clamp(tmax, max=far)
    return tmin, tmax


def stratified_samples(o, d, u, aabb, near, far, n_samples):
    """-> t0, t1 of shape (R, N) (see module docstring)."""
    tmin, tmax = ray_aabb_tmin_tmax(o, d, aabb, near, far)
    hit = tmax > tmin
    span = torch.where(hit, tmax - tmin, torch.zeros_like(tmin))
    # a missed ray: zero-length samples at its origin (nerfacc: no samples; same C, O, D, gradient)
    tmin = torch.where(hit, tmin, torch.zeros_like(tmin))
    k = torch.arange(n_samples, dtype=o.dtype)
    s = (k[None, :] + u[:, None]) / n_samples
    mid = tmin[:, None] + s * span[:, None]
    half = 0.5 * (span / n_samples)
    return mid - half[:, None], mid + half[:, None]


# ----------------------------------------------------------------------------- compositing
def composite(t0, t1, rgb, sigma, bkgd=None):
    """nerfacc 0.3.1 render_weight_from_density + accumulate_along_rays
    (vol_rendering.py:89-126), rays laid out densely as (R, N).
    rgb (R, N, rd), sigma (R, N) -> colour (R, rd), opacity (R), depth (R) (un-normalised)."""
    # zero-length samples (a missed ray's) contribute nothing (nerfacc has no such sample)
    tau = torch.where(t1 > t0, sigma * (t1 - t0), torch.zeros_like(sigma))
    alpha = 1.0 - torch.exp(-tau)
    # exclusive optical depth: a sum of the preceding terms (nerfacc's exclusive cumsum), not
    # cumsum - tau, which is inf - inf once a sigma overflows
    excl = torch.cat([torch.zeros_like(tau[..., :1]), torch.cumsum(tau, dim=-1)[..., :-1]], dim=-1)
    w = torch.exp(-excl) * alpha
    colour = (w[..., None] * rgb).sum(dim=-2)
    opacity = w.sum(dim=-1)
    depth = (w * ((t0 + t1) / 2.0)).sum(dim=-1)
    if bkgd is not None:
        colour = colour + bkgd * (1.0 - opacity[..., None])
    return colour, opacity, depth, w


def composite_bruteforce_f64(t0, t1, rgb, sigma, bkgd=None):
    """Independent per-ray float64 loop used to cross-check ``composite``."""
    t0, t1, rgb, sigma = (a.double() for a in (t0, t1, rgb, sigma))
    R, N = sigma.shape
    col = torch.zeros(R, rgb.shape[-1], dtype=torch.float64)
    op = torch.zeros(R, dtype=torch.float64)
    dep = torch.zeros(R, dtype=torch.float64)
    for r in range(R):
        T = 1.0
        for i in range(N):
            dt = float(t1[r, i] - t0[r, i])
            a = 1.0 - math.exp(-float(sigma[r, i]) * dt)
            w = T * a
            col[r] += w * rgb[r, i]
            op[r] += w
            dep[r] += w * 0.5 * float(t0[r, i] + t1[r, i])
            T *= math.exp(-float(sigma[r, i]) * dt)
    if bkgd is not None:
        col = col + bkgd.double() * (1.0 - op[:, None])
    return col, op, dep


# ----------------------------------------------------------------------------- full render
def render_rays(p, o, d, u, n_samples=128, aabb=AABB_CHAIR, near=1.43, far=6.63, bkgd=None):
    """NeRF.forward on a dense batch of rays (nerf.py:230-286 with the fixed-count
    sampler).  -> colour (R, rd), opacity (R), depth_normalised (R), extras dict."""
    t0, t1 = stratified_samples(o, d, u, aabb, near, far, n_samples)
    R, N = t0.shape
    pos = o[:, None, :] + d[:, None, :] * (t0 + t1)[..., None] / 2.0
    dirs = d[:, None, :].expand(R, N, 3)
    rgb, sigma = radiance_field(p, pos.reshape(-1, 3), dirs.reshape(-1, 3), aabb)
    rgb = rgb.reshape(R, N, -1)
    sigma = sigma.reshape(R, N)
    colour, opacity, depth, w = composite(t0, t1, rgb, sigma, bkgd)
    depth_n = depth / (opacity + 1e-10)
    return colour, opacity, depth_n, dict(t0=t0, t1=t1, rgb=rgb, sigma=sigma, depth=depth, w=w)
