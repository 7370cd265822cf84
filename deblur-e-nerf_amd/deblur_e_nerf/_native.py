"""ctypes binding of libden.so (include/den_api.h) + torch.autograd Functions.

This is the ONLY compute path of the package: there is no CPU or PyTorch
fallback.  If libden.so is missing, or no HIP device is present, every op
raises.  PyTorch provides device memory (the caching allocator), the current
HIP stream and autograd plumbing; the arithmetic happens in the HIP kernels.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DEN_LIB", os.path.join(os.path.dirname(_HERE), "libden.so"))

MODE_F32 = 0
MODE_BF16 = 1
_MODES = {"f32": MODE_F32, "fp32": MODE_F32, "float32": MODE_F32, "bf16": MODE_BF16, "bfloat16": MODE_BF16}
ERROR_FNS = {"l1": 0, "mse": 1, "huber": 2, "mape": 3}


class DenError(RuntimeError):
    pass


class RenderDesc(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("radiance_dim", ctypes.c_int32), ("n_rays", ctypes.c_int32),
                ("n_samples", ctypes.c_int32), ("aabb", ctypes.c_float * 6), ("near_plane", ctypes.c_float),
                ("far_plane", ctypes.c_float), ("train", ctypes.c_int32), ("has_bkgd", ctypes.c_int32),
                ("points", ctypes.c_int32), ("contraction", ctypes.c_int32), ("bwd_path", ctypes.c_int32),
                ("density_activation", ctypes.c_int32), ("ray_grad", ctypes.c_int32),
                ("max_workgroups", ctypes.c_int32)]


class RenderIO(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("rays_o", "rays_d", "jitter", "w_fwd", "w_bwd", "bias_pk", "bkgd",
                                               "workspace", "out_rgb", "out_opacity", "out_depth", "ray_indices",
                                               "t_starts", "t_ends")]


class NgpDesc(ctypes.Structure):
    _fields_ = [("radiance_dim", ctypes.c_int32), ("n_levels", ctypes.c_int32),
                ("n_features_per_level", ctypes.c_int32), ("log2_hashmap_size", ctypes.c_int32),
                ("base_resolution", ctypes.c_int32), ("per_level_scale", ctypes.c_float),
                ("grid_type", ctypes.c_int32), ("hidden_activation", ctypes.c_int32),
                ("radiance_activation", ctypes.c_int32), ("contraction", ctypes.c_int32),
                ("aabb", ctypes.c_float * 6), ("density_activation", ctypes.c_int32)]


class RenderGrad(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("d_rgb", "d_opacity", "d_depth", "grad_params", "grad_bkgd")]


_lib = None

_SIGS = {
    "den_version": (ctypes.c_int, []),
    "den_render_tile_samples": (ctypes.c_int32, [ctypes.c_int32]),
    "den_last_error": (ctypes.c_char_p, []),
    "den_timing_enable": (ctypes.c_int, [ctypes.c_int32]),
    "den_timing_collect": (ctypes.c_int, [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "den_param_count": (ctypes.c_int64, [ctypes.c_int32]),
    "den_param_offset": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "den_packed_fwd_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_packed_bwd_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_packed_bias_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_pack_weights": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 5),
    "den_render_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(RenderDesc)]),
    "den_render_fwd": (ctypes.c_int, [ctypes.POINTER(RenderDesc), ctypes.POINTER(RenderIO), ctypes.c_void_p]),
    "den_render_bwd": (ctypes.c_int, [ctypes.POINTER(RenderDesc), ctypes.POINTER(RenderIO),
                                      ctypes.POINTER(RenderGrad), ctypes.c_void_p]),
    "den_render_bwd_part": (ctypes.c_int, [ctypes.POINTER(RenderDesc), ctypes.POINTER(RenderIO),
                                           ctypes.POINTER(RenderGrad), ctypes.c_int32, ctypes.c_void_p]),
    "den_sum_partials": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "den_adam_step": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_float] * 5
                      + [ctypes.c_int64, ctypes.c_void_p]),
    "den_event_loss_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_event_loss_fwd": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 7),
    "den_event_loss_bwd": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 10),
    "den_event_target": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 7),
    "den_event_step_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_event_step_fwd": (ctypes.c_int, [ctypes.c_int32] * 5 + [ctypes.c_float] * 3 + [ctypes.c_void_p] * 8),
    "den_event_step_bwd": (ctypes.c_int, [ctypes.c_int32] * 5 + [ctypes.c_float] * 3 + [ctypes.c_void_p] * 8),
    "den_event_prep": (ctypes.c_int, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 15),
    "den_pixel_rays": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 7),
    "den_pixbw_sample_ts": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]),
    "den_pixbw_fwd": (ctypes.c_int, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 9),
    "den_pixbw_blocks": (ctypes.c_int, [ctypes.c_int32]),
    "den_pixbw_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]),
    "den_pixbw_bwd": (ctypes.c_int, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 13),
    # packed (ray-marching) rendering, den_march.hip
    "den_march_prep": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 3 + [ctypes.c_float] * 2
                       + [ctypes.c_void_p, ctypes.c_float] + [ctypes.c_void_p] * 3),
    "den_march_count": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 7 + [ctypes.c_int32, ctypes.c_float,
                                                                                   ctypes.c_float]
                        + [ctypes.c_void_p] * 2),
    "den_march_fill": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 7 + [ctypes.c_int32, ctypes.c_float,
                                                                                  ctypes.c_float]
                       + [ctypes.c_void_p] * 5),
    "den_scan_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "den_exclusive_scan": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "den_pack_info": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64] + [ctypes.c_void_p] * 3),
    "den_visibility": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 5 + [ctypes.c_float] * 2
                       + [ctypes.c_void_p] * 3),
    "den_compact": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 10),
    "den_composite_fwd": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 10),
    "den_composite_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32] * 2),
    "den_composite_bwd": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 14),
    "den_composite_alpha_fwd": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 10),
    "den_composite_alpha_bwd": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 14),
    "den_event_prep_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_event_prep_bwd": (ctypes.c_int, [ctypes.c_int32] * 3 + [ctypes.c_void_p] * 17),
    "den_event_target_bwd": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 12),
    "den_image_error_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_image_error": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64] + [ctypes.c_void_p] * 5),
    "den_adam_step_f64": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_double] * 5
                          + [ctypes.c_int64, ctypes.c_void_p]),
    "den_trajectory": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 8),
    "den_ngp_table_params": (ctypes.c_int64, [ctypes.POINTER(NgpDesc)]),
    "den_ngp_param_count": (ctypes.c_int64, [ctypes.POINTER(NgpDesc)]),
    "den_ngp_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(NgpDesc), ctypes.c_int64, ctypes.c_int32]),
    "den_ngp_fwd": (ctypes.c_int, [ctypes.POINTER(NgpDesc), ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 6
                    + [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 4),
    "den_ngp_bwd": (ctypes.c_int, [ctypes.POINTER(NgpDesc), ctypes.c_int64] + [ctypes.c_void_p] * 6),
    "den_hashgrid_fwd": (ctypes.c_int, [ctypes.POINTER(NgpDesc), ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "den_hashgrid_bwd": (ctypes.c_int, [ctypes.POINTER(NgpDesc), ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "den_sh_encode_fwd": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 3),
    "den_sh_encode_bwd": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 4),
    "den_render_ray_grad_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(RenderDesc)]),
    "den_render_ray_grad": (ctypes.c_int, [ctypes.POINTER(RenderDesc), ctypes.POINTER(RenderIO), ctypes.c_void_p,
                                           ctypes.c_int32, ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "den_ngp_ray_grad_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "den_ngp_ray_grad": (ctypes.c_int, [ctypes.POINTER(NgpDesc), ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
                         + [ctypes.c_void_p] * 11),
    "den_pixel_rays_bwd": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 8),
    "den_trajectory_bwd": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 8),
    "den_pixbw_sample_ts_bwd": (ctypes.c_int, [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 3),
    "den_pixbw_decay_ts_bwd": (ctypes.c_int, [ctypes.c_int32] + [ctypes.c_void_p] * 8),
    "den_occ_workspace_bytes": (ctypes.c_size_t, []),
    "den_occ_points": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int32]
                       + [ctypes.c_void_p] * 4),
    "den_occ_update": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_float] * 3
                       + [ctypes.c_int64] + [ctypes.c_void_p] * 5),
    # dataset preprocessing, den_dataset.hip
    "den_queue_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "den_queue_raw_events": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 4
                             + [ctypes.c_size_t] + [ctypes.c_void_p] * 7),
    "den_colorize_events": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_void_p] * 4),
    "den_max_refractory_period": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
                                  + [ctypes.c_void_p] * 3 + [ctypes.c_size_t] + [ctypes.c_void_p] * 2),
    "den_undistort_events": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 5),
    # evaluation views and metrics, den_eval.hip
    "den_ssim_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int32]),
    "den_ssim": (ctypes.c_int, [ctypes.c_int32] * 4 + [ctypes.c_void_p] * 3 + [ctypes.c_float] * 2
                 + [ctypes.c_void_p] * 3),
    "den_png_unfilter": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 2),
}


ABI_VERSION = 7  # include/den_api.h DEN_VERSION


def lib():
    """Load libden.so (raises DenError if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DenError(f"HIP library not found at {LIB_PATH}: build it with `python __graft_entry__.py` "
                           "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.den_version() != ABI_VERSION:  # the ctypes structs below must match the library's
            raise DenError(f"{LIB_PATH} has C-ABI version {L.den_version()}, these bindings {ABI_VERSION}: rebuild it")
        _lib = L
    return _lib


def exported_symbols():
    return sorted(_SIGS)


TIMING_CLASSES = ("render_fwd_kernel", "render_bwd_kernel", "hidden_bwd_kernel", "dw_gemm_kernel",
                  "dw_reduce_kernel", "hidden_bwd_lb_kernel")


def timing_enable(on=True):
    _check(lib().den_timing_enable(int(on)))


def timing_collect():
    """-> {kernel: (total_ms, launches)} since the last collect (den_timing_collect)."""
    n = len(TIMING_CLASSES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    _check(lib().den_timing_collect(n, ms, cnt))
    return {k: (ms[i], cnt[i]) for i, k in enumerate(TIMING_CLASSES)}


def _check(rc):
    if rc != 0:
        raise DenError(f"libden error {rc}: {lib().den_last_error().decode()}")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise DenError("libden ops need HIP device tensors (there is no CPU fallback)")


def mode_id(mode):
    if isinstance(mode, int):
        return mode
    return _MODES[str(mode).lower()]


def param_count(rd):
    return lib().den_param_count(rd)


def param_offset(rd, idx):
    return lib().den_param_offset(rd, idx)


# ----------------------------------------------------------------------------- packed weights
class PackedWeights:
    """Device buffers holding the MFMA fragment layouts of the MLP weights."""

    def __init__(self, mode, rd, device):
        L = lib()
        self.mode, self.rd = mode_id(mode), rd
        self.fwd = torch.empty(L.den_packed_fwd_bytes(self.mode), dtype=torch.uint8, device=device)
        self.bwd = torch.empty(L.den_packed_bwd_bytes(self.mode), dtype=torch.uint8, device=device)
        self.bias = torch.empty(L.den_packed_bias_bytes(self.mode) // 4, dtype=torch.float32, device=device)
        self.version = None

    def pack(self, flat_params):
        _require_device(flat_params)
        assert flat_params.dtype == torch.float32 and flat_params.is_contiguous()
        _check(lib().den_pack_weights(self.mode, self.rd, _ptr(flat_params), _ptr(self.fwd), _ptr(self.bwd),
                                      _ptr(self.bias), _stream(flat_params.device)))


# ----------------------------------------------------------------------------- render
def _desc(cfg, n_rays, n_samples, train, has_bkgd, points=0, ray_grad=False):
    d = RenderDesc()
    d.mode = cfg["mode"]
    d.radiance_dim = cfg["rd"]
    d.n_rays = n_rays
    d.n_samples = n_samples
    for i, v in enumerate(cfg["aabb"]):
        d.aabb[i] = float(v)
    d.near_plane = -1.0 if cfg.get("near") is None else float(cfg["near"])
    d.far_plane = -1.0 if cfg.get("far") is None else float(cfg["far"])
    d.train = int(train)
    d.has_bkgd = int(has_bkgd)
    d.points = int(points)
    d.contraction = int(cfg.get("contraction", 0))
    d.bwd_path = int(cfg.get("bwd_path", 0))
    d.density_activation = int(cfg.get("density", 0))
    d.ray_grad = int(bool(ray_grad))
    return d


def wg_samples(mode):
    """Samples per render workgroup tile: n_rays * n_samples must be a multiple."""
    return int(lib().den_render_tile_samples(mode_id(mode)))


def render_workspace_bytes(desc):
    n = lib().den_render_workspace_bytes(ctypes.byref(desc))
    if n == 0:
        raise DenError(lib().den_last_error().decode())
    return n


class RenderFunction(torch.autograd.Function):
    """Fused sampler + encoding + MLP + compositing (den_render_fwd/bwd).

    inputs: rays_o (R,3), rays_d (R,3), jitter (R), bkgd (rd) or None, flat
    params (P,) f32, plus non-tensor config; outputs colour (R,rd), opacity (R),
    depth (R) (un-normalised).  ``points=1`` evaluates the radiance field at
    given points instead: rays_o = positions (n,3), rays_d = directions (n,3),
    outputs rgb (n,rd), sigma (n), unused (n).  ``points=2`` evaluates it at the
    packed samples ``samples = (ray_indices (n) i32, t_starts (n), t_ends (n))`` of
    the rays rays_o / rays_d (n a multiple of the tile; the first ``n_valid`` are the
    real, ray-sorted samples): outputs rgb (n,rd), sigma (n).  When rays_o / rays_d
    require grad the backward also returns their gradients (den_render_ray_grad: the
    positions o + d t and view directions d of the samples, t detached as nerfacc's)."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, jitter, bkgd, flat, cfg, packed, n_samples, points, samples=None, n_valid=None):
        _require_device(rays_o, rays_d, jitter, bkgd, flat)
        rd = cfg["rd"]
        train = torch.is_grad_enabled() and (flat.requires_grad or (bkgd is not None and bkgd.requires_grad))
        train = (train or ctx.needs_input_grad[4] or (bkgd is not None and ctx.needs_input_grad[3])
                 or ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        R = samples[0].numel() if points == 2 else rays_o.shape[0]
        # the rays' own gradient (den_render_ray_grad) follows the backward when they require grad
        ray_grad = bool(ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        desc = _desc(cfg, R if not points else R // n_samples, n_samples, train, bkgd is not None, points, ray_grad)
        ws = torch.empty(render_workspace_bytes(desc), dtype=torch.uint8, device=rays_o.device)
        out_rgb = torch.empty(R, rd, dtype=torch.float32, device=rays_o.device)
        out_op = torch.empty(R, dtype=torch.float32, device=rays_o.device)
        out_dp = torch.empty(R, dtype=torch.float32, device=rays_o.device)
        ri, t0, t1 = samples if points == 2 else (None, None, None)
        io = RenderIO(_ptr(rays_o), _ptr(rays_d), _ptr(jitter), _ptr(packed.fwd), _ptr(packed.bwd),
                      _ptr(packed.bias), _ptr(bkgd), _ptr(ws), _ptr(out_rgb), _ptr(out_op), _ptr(out_dp),
                      _ptr(ri), _ptr(t0), _ptr(t1))
        _check(lib().den_render_fwd(ctypes.byref(desc), ctypes.byref(io), _stream(rays_o.device)))
        ctx.desc, ctx.io_keep = desc, (rays_o, rays_d, jitter, bkgd, ws, packed, ri, t0, t1, flat)
        ctx.flat_shape = flat.shape
        ctx.has_bkgd = bkgd is not None
        ctx.n_valid = R if n_valid is None else int(n_valid)
        return out_rgb, out_op, out_dp

    @staticmethod
    def backward(ctx, g_rgb, g_op, g_dp):
        rays_o, rays_d, jitter, bkgd, ws, packed, ri, t0, t1, flat = ctx.io_keep
        dev = rays_o.device
        g_rgb = torch.zeros_like(g_rgb) if g_rgb is None else g_rgb.contiguous()
        g_op = None if g_op is None else g_op.contiguous()
        g_dp = None if g_dp is None else g_dp.contiguous()
        grad_flat = torch.empty(ctx.flat_shape, dtype=torch.float32, device=dev)
        grad_bkgd = torch.empty(bkgd.shape, dtype=torch.float32, device=dev) if ctx.has_bkgd else None
        io = RenderIO(_ptr(rays_o), _ptr(rays_d), _ptr(jitter), _ptr(packed.fwd), _ptr(packed.bwd),
                      _ptr(packed.bias), _ptr(bkgd), _ptr(ws), None, None, None, _ptr(ri), _ptr(t0), _ptr(t1))
        gr = RenderGrad(_ptr(g_rgb), _ptr(g_op), _ptr(g_dp), _ptr(grad_flat), _ptr(grad_bkgd))
        _check(lib().den_render_bwd(ctypes.byref(ctx.desc), ctypes.byref(io), ctypes.byref(gr), _stream(dev)))
        d_o = d_d = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            L = lib()
            d_o, d_d = torch.empty_like(rays_o), torch.empty_like(rays_d)
            rg = torch.empty(L.den_render_ray_grad_workspace_bytes(ctypes.byref(ctx.desc)), dtype=torch.uint8,
                             device=dev)
            _check(L.den_render_ray_grad(ctypes.byref(ctx.desc), ctypes.byref(io), _ptr(flat.detach()),
                                         rays_o.shape[0], ctx.n_valid, _ptr(rg), _ptr(d_o), _ptr(d_d), _stream(dev)))
        # release the workspace (the activations kept for this backward) as soon as the
        # stream is done with it: the caching allocator orders the reuse on the same stream
        ctx.io_keep = None
        return d_o, d_d, None, grad_bkgd, grad_flat, None, None, None, None, None, None


def render(rays_o, rays_d, jitter, bkgd, flat, cfg, packed, n_samples):
    return RenderFunction.apply(rays_o.contiguous(), rays_d.contiguous(), jitter.contiguous(),
                                None if bkgd is None else bkgd.contiguous(), flat, cfg, packed, n_samples, 0)


def _point_group(cfg):
    tile = wg_samples(cfg["mode"])
    # "rays" of `group` points each (<= the per-ray sample limit)
    return tile, min(tile, 128 if mode_id(cfg["mode"]) == MODE_F32 else 256)


def field(points, dirs, flat, cfg, packed):
    """Radiance field at arbitrary points (n,3)/(n,3): -> rgb (n,rd), sigma (n)."""
    n = points.shape[0]
    tile, group = _point_group(cfg)
    pad = (-n) % tile
    if pad:
        points = torch.cat([points, points.new_zeros(pad, 3)])
        dirs = torch.cat([dirs, dirs.new_zeros(pad, 3) + torch.tensor([0.0, 0.0, 1.0], device=dirs.device)])
    rgb, sig, _ = RenderFunction.apply(points.contiguous(), dirs.contiguous(), None, None, flat, cfg, packed,
                                       group, 1)
    return rgb[:n], sig[:n]


def field_packed(rays_o, rays_d, ray_indices, t_starts, t_ends, flat, cfg, packed):
    """Radiance field at packed ray-marching samples (den_render points = 2): sample s is at
    rays_o[r] + rays_d[r] (t_starts[s] + t_ends[s]) / 2, r = ray_indices[s], viewed along
    rays_d[r] (external/utils.py:83-96) -> rgb (n, rd), sigma (n)."""
    n = ray_indices.numel()
    if n == 0:  # no sample survived the march: nothing to evaluate
        return (torch.zeros(0, cfg["rd"], device=rays_o.device), torch.zeros(0, device=rays_o.device))
    tile, group = _point_group(cfg)
    pad = (-n) % tile
    ri = ray_indices.reshape(-1).to(torch.int32)
    t0 = t_starts.reshape(-1).to(torch.float32)
    t1 = t_ends.reshape(-1).to(torch.float32)
    if pad:  # zero-length samples of ray 0 (outputs dropped, no gradient)
        ri = torch.cat([ri, ri.new_zeros(pad)])
        t0 = torch.cat([t0, t0.new_zeros(pad)])
        t1 = torch.cat([t1, t1.new_zeros(pad)])
    rgb, sig, _ = RenderFunction.apply(rays_o.float().contiguous(), rays_d.float().contiguous(), None, None, flat,
                                       cfg, packed, group, 2, (ri.contiguous(), t0.contiguous(), t1.contiguous()), n)
    return rgb[:n], sig[:n]


# ----------------------------------------------------------------------------- ngp radiance field
# models/nerf.py:20-29 density activations -> den_render_desc / den_ngp_desc.density_activation
DENSITY_ACTIVATIONS = {"shifted_trunc_exp": 0, "softplus": 1, "shifted_softplus": 2}


def density_id(fn):
    """den density_activation id of a density activation callable (models/nerf.py:20-29):
    shifted_trunc_exp, torch.nn.Softplus(beta=1) with threshold 20, or shifted_softplus."""
    name = getattr(fn, "__name__", "")
    if name in ("shifted_trunc_exp", "shifted_softplus"):
        return DENSITY_ACTIVATIONS[name]
    if isinstance(fn, torch.nn.Softplus) and fn.beta == 1 and fn.threshold == 20:
        return DENSITY_ACTIVATIONS["softplus"]
    raise DenError(f"density activation {fn!r} unsupported (shifted_trunc_exp, Softplus(beta=1), shifted_softplus)")


def ngp_desc(rd, pos_encoding, hidden_activation, radiance_activation, contraction, aabb, density=0):
    """den_ngp_desc of an NGPradianceField configuration (external/ngp.py:112-145 with the
    configs/train/*.yaml nerf.ngp entries); unsupported settings raise DenError."""
    pe = dict(pos_encoding)
    if pe.get("interpolation", "Linear") != "Linear" or pe.get("otype", "HashGrid") not in ("HashGrid", "DenseGrid"):
        raise DenError(f"ngp position encoding {pe} unsupported (Linear HashGrid / DenseGrid only)")
    d = NgpDesc()
    d.radiance_dim = int(rd)
    d.n_levels = int(pe["n_levels"])
    d.n_features_per_level = int(pe["n_features_per_level"])
    d.log2_hashmap_size = int(pe.get("log2_hashmap_size", 19))
    d.base_resolution = int(pe["base_resolution"])
    d.per_level_scale = float(pe["per_level_scale"])
    d.grid_type = 0 if pe.get("otype", "HashGrid") == "HashGrid" else 1
    d.hidden_activation = {"softplus": 0, "relu": 1}[hidden_activation]
    d.radiance_activation = {"softplus": 0, "sigmoid": 1}[radiance_activation]
    d.contraction = int(contraction)
    for i, v in enumerate(aabb):
        d.aabb[i] = float(v)
    d.density_activation = int(density)
    if lib().den_ngp_table_params(ctypes.byref(d)) < 0:
        raise DenError(f"unsupported ngp descriptor: {pe}")
    return d


def ngp_table_params(desc):
    return int(lib().den_ngp_table_params(ctypes.byref(desc)))


def ngp_param_count(desc):
    return int(lib().den_ngp_param_count(ctypes.byref(desc)))


class NgpFieldFunction(torch.autograd.Function):
    """NGPradianceField forward at points (points = 1: x, d (n,3)) or packed ray samples
    (points = 2: rays_o / rays_d (R,3) + ray_indices, t_starts, t_ends) -> rgb (n, rd), sigma (n)
    (den_ngp_fwd); backward -> the flat-parameter gradient (den_ngp_bwd)."""

    @staticmethod
    def forward(ctx, flat, desc, points, x, d, ri, t0, t1, density_only):
        _require_device(flat, x, d, ri, t0, t1)
        n = (ri.numel() if points == 2 else x.shape[0])
        dev = flat.device
        # (grad mode is off inside Function.forward: needs_input_grad says whether a backward follows)
        if density_only and (ctx.needs_input_grad[0] or ctx.needs_input_grad[3] or ctx.needs_input_grad[4]):
            # the density-only pass keeps no state for a backward (the reference's query_density
            # call sites are all no-grad: nerf.py:170-204, external/utils.py:68-81)
            raise NotImplementedError("ngp density-only query is not differentiable here: call it under "
                                      "torch.no_grad() or use the full field")
        train = bool(ctx.needs_input_grad[0] or ctx.needs_input_grad[3] or ctx.needs_input_grad[4])
        ws = (torch.empty(lib().den_ngp_workspace_bytes(ctypes.byref(desc), n, 1), dtype=torch.uint8, device=dev)
              if train and n > 0 else None)
        rgb = torch.empty(n, desc.radiance_dim, dtype=torch.float32, device=dev)
        sig = torch.empty(n, dtype=torch.float32, device=dev)
        _check(lib().den_ngp_fwd(ctypes.byref(desc), n, points, _ptr(x), _ptr(d), _ptr(ri), _ptr(t0), _ptr(t1),
                                 _ptr(flat), int(bool(density_only)), int(train), _ptr(ws), _ptr(rgb), _ptr(sig),
                                 _stream(dev)))
        ctx.keep = (desc, n, flat, ws, points, x, d, ri, t0, t1)
        return rgb, sig

    @staticmethod
    def backward(ctx, g_rgb, g_sig):
        desc, n, flat, ws, points, x, d, ri, t0, t1 = ctx.keep
        grad = torch.empty_like(flat)
        g_rgb = None if g_rgb is None else g_rgb.contiguous()
        g_sig = None if g_sig is None else g_sig.contiguous()
        d_x = d_d = None
        if ws is None:
            grad.zero_()
        else:
            st = _stream(flat.device)
            _check(lib().den_ngp_bwd(ctypes.byref(desc), n, _ptr(flat), _ptr(ws), _ptr(g_rgb), _ptr(g_sig),
                                     _ptr(grad), st))
            if ctx.needs_input_grad[3] or ctx.needs_input_grad[4]:
                L = lib()
                d_x, d_d = torch.empty_like(x), torch.empty_like(d)
                rg = torch.empty(max(1, L.den_ngp_ray_grad_workspace_bytes(n)), dtype=torch.uint8, device=x.device)
                _check(L.den_ngp_ray_grad(ctypes.byref(desc), n, points, x.shape[0] if points == 2 else 0, _ptr(x),
                                          _ptr(d), _ptr(ri), _ptr(t0), _ptr(t1), _ptr(flat), _ptr(ws), _ptr(rg),
                                          _ptr(d_x), _ptr(d_d), st))
        ctx.keep = None
        return grad, None, None, d_x, d_d, None, None, None, None


def _no_grad_if(density_only, t):
    # the density-only pass (the marching pre-pass / occupancy update) is never differentiated
    return t.detach() if density_only else t


def ngp_field(flat, desc, x, d, density_only=False):
    """-> rgb (n, rd), sigma (n) at positions x (n,3) viewed along d (n,3)."""
    x, d = _no_grad_if(density_only, x), _no_grad_if(density_only, d)
    return NgpFieldFunction.apply(flat, desc, 1, x.float().contiguous(), d.float().contiguous(), None, None, None,
                                  density_only)


def ngp_field_packed(flat, desc, rays_o, rays_d, ray_indices, t_starts, t_ends, density_only=False):
    """-> rgb (n, rd), sigma (n) at packed ray-marching samples (external/utils.py:83-96)."""
    rays_o, rays_d = _no_grad_if(density_only, rays_o), _no_grad_if(density_only, rays_d)
    return NgpFieldFunction.apply(flat, desc, 2, rays_o.float().contiguous(), rays_d.float().contiguous(),
                                  ray_indices.reshape(-1).to(torch.int32).contiguous(),
                                  t_starts.reshape(-1).float().contiguous(), t_ends.reshape(-1).float().contiguous(),
                                  density_only)


class HashGridFunction(torch.autograd.Function):
    """tcnn.Encoding (HashGrid / DenseGrid, Linear): x (n,3) in [0,1] -> (n, 2 n_levels)."""

    @staticmethod
    def forward(ctx, table, desc, x):
        _require_device(table, x)
        n = x.shape[0]
        out = torch.empty(n, 2 * desc.n_levels, dtype=torch.float32, device=x.device)
        _check(lib().den_hashgrid_fwd(ctypes.byref(desc), n, _ptr(x), _ptr(table), _ptr(out), _stream(x.device)))
        ctx.keep = (desc, x, table.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        desc, x, shape = ctx.keep
        d_table = torch.zeros(shape, dtype=torch.float32, device=x.device)
        g = g.contiguous()  # bound: a temporary's block could be reused before the kernel runs
        _check(lib().den_hashgrid_bwd(ctypes.byref(desc), x.shape[0], _ptr(x), _ptr(g), _ptr(d_table),
                                      _stream(x.device)))
        return d_table, None, None


def hashgrid(table, desc, x):
    return HashGridFunction.apply(table, desc, x.float().contiguous())


class SHEncodeFunction(torch.autograd.Function):
    """SHEncoder.forward (external/sh_encoder.py:28-193): coords (n,3) -> (n, degree^2), with the
    coords gradient of the reference's autograd graph."""

    @staticmethod
    def forward(ctx, coords, degree):
        _require_device(coords)
        n = coords.shape[0]
        out = torch.empty(n, degree * degree, dtype=torch.float32, device=coords.device)
        _check(lib().den_sh_encode_fwd(n, degree, _ptr(coords), _ptr(out), _stream(coords.device)))
        ctx.save_for_backward(coords)
        ctx.degree = degree
        return out

    @staticmethod
    def backward(ctx, g):
        (coords,) = ctx.saved_tensors
        d = torch.empty_like(coords)
        g = g.float().contiguous()
        _check(lib().den_sh_encode_bwd(coords.shape[0], ctx.degree, _ptr(coords), _ptr(g), _ptr(d),
                                       _stream(coords.device)))
        return d, None


def sh_encode(coords, degree):
    if not 1 <= int(degree) <= 8:
        raise DenError(f"SH degree {degree} outside 1..8 (external/sh_encoder.py:24)")
    return SHEncodeFunction.apply(coords.float().contiguous(), int(degree))


# ----------------------------------------------------------------------------- reductions / adam
def sum_partials(part, n, nb, out):
    _check(lib().den_sum_partials(n, nb, _ptr(part), _ptr(out), _stream(part.device)))


def adam_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step):
    _require_device(param, grad, exp_avg, exp_avg_sq)
    fn = lib().den_adam_step_f64 if param.dtype == torch.float64 else lib().den_adam_step
    _check(fn(param.numel(), _ptr(param), _ptr(grad), _ptr(exp_avg), _ptr(exp_avg_sq), lr, beta1, beta2, eps,
              weight_decay, int(step), _stream(param.device)))


# ----------------------------------------------------------------------------- event loss
class EventLossFunction(torch.autograd.Function):
    """mean_{valid} err(x / c - target)  (loss.py:62-96)."""

    @staticmethod
    def forward(ctx, x, target, c, valid, error_fn):
        _require_device(x, target, c, valid)
        N = x.numel()
        ws = torch.empty(lib().den_event_loss_workspace_bytes(N) // 4 + 1, dtype=torch.float32, device=x.device)
        out = torch.empty((), dtype=torch.float32, device=x.device)
        v = None if valid is None else valid.to(torch.uint8).contiguous()
        _check(lib().den_event_loss_fwd(N, ERROR_FNS[error_fn], _ptr(x), _ptr(target), _ptr(v), _ptr(c), _ptr(out),
                                        _ptr(ws), _stream(x.device)))
        ctx.save_for_backward(x, target, c)
        ctx.v, ctx.ws, ctx.fn = v, ws, error_fn
        return out

    @staticmethod
    def backward(ctx, g):
        x, target, c = ctx.saved_tensors
        N = x.numel()
        dx = torch.empty_like(x)
        dt = torch.empty_like(x) if target is not None and ctx.needs_input_grad[1] else None
        dc = torch.empty((), dtype=torch.float32, device=x.device)
        g = g.contiguous().to(torch.float32)
        _check(lib().den_event_loss_bwd(N, ERROR_FNS[ctx.fn], _ptr(x), _ptr(target), _ptr(ctx.v), _ptr(c), _ptr(g),
                                        _ptr(dx), _ptr(dt), _ptr(dc), _ptr(ctx.ws), _stream(x.device)))
        return dx, dt, dc.reshape(c.shape), None, None


def event_target(ts_diff, lid, end_ts, start_ts, c):
    _require_device(ts_diff, lid, end_ts, start_ts, c)
    N = lid.numel()
    out = torch.empty(N, dtype=torch.float32, device=lid.device)
    # every converted input stays bound until the launch: a freed temporary's block could be
    # handed to the next conversion (and overwritten) before the kernel reads it
    args = (ts_diff.double().contiguous(), lid.float().contiguous(), end_ts.long().contiguous(),
            start_ts.double().contiguous(), c.float().reshape(1).contiguous())
    _check(lib().den_event_target(N, *(_ptr(t) for t in args), _ptr(out), _stream(lid.device)))
    return out


# ----------------------------------------------------------------------------- pixel bandwidth
PIXBW_NPARAM = 7


class SampleTsFunction(torch.autograd.Function):
    """den_pixbw_sample_ts, differentiable in output_ts (the lifetimes are drawn under no_grad in
    the reference, pixel_bandwidth.py:298-367: d output_ts = sum over the S samples,
    den_pixbw_sample_ts_bwd)."""

    @staticmethod
    def forward(ctx, gen, output_ts, omega_c_min, max_cumprob):
        _require_device(gen, output_ts)
        S = gen.shape[0] + 1
        batch = output_ts.shape
        N = output_ts.numel()
        g = gen.reshape(S - 1, N).to(torch.float64).contiguous()
        o = output_ts.reshape(N).to(torch.float64).contiguous()
        ts = torch.empty(S, N, dtype=torch.float64, device=gen.device)
        _check(lib().den_pixbw_sample_ts(S, N, _ptr(g), _ptr(o), float(omega_c_min), float(max_cumprob), _ptr(ts),
                                         _stream(gen.device)))
        ctx.meta = (S, N, batch, output_ts.dtype)
        return ts.reshape(S, *batch)

    @staticmethod
    def backward(ctx, g_ts):
        S, N, batch, dt = ctx.meta
        d = torch.empty(N, dtype=torch.float64, device=g_ts.device)
        g = g_ts.to(torch.float64).reshape(S, N).contiguous()
        _check(lib().den_pixbw_sample_ts_bwd(S, N, _ptr(g), _ptr(d), _stream(g_ts.device)))
        return None, d.reshape(batch).to(dt), None, None


def pixbw_sample_ts(gen, output_ts, omega_c_min, max_cumprob):
    """den_pixbw_sample_ts: (S-1, ...) f64 interval generators and (...) f64 output
    timestamps (ns) -> (S, ...) f64 sample timestamps (pixel_bandwidth.py:311-360,
    before the clamp to min_ts); differentiable in output_ts."""
    return SampleTsFunction.apply(gen, output_ts, omega_c_min, max_cumprob)


class PixelBandwidthFunction(torch.autograd.Function):
    """One PixelBandwidth call after intensity sampling (pixel_bandwidth.py:369-448).

    intensity (S, ...) and params (7) = [tau_in_it_eff_prod, tau_mil_it_eff_prod, A_amp_inv,
    A_loop_inv, tau_out, tau_sf, tau_diff] (post-parametrisation) -> (out, delta_out), both (...).
    reset=True resets the differencing amplifier (delta_out = its offset, the reference's
    ``reset_delta_log_it``); otherwise delta_in / reset_ts of the preceding reset call decay the
    offset and delta_out is zeros."""

    @staticmethod
    def forward(ctx, intensity, params, delta_in, sample_ts, output_ts, reset_ts, reset):
        _require_device(intensity, params, delta_in, sample_ts, output_ts, reset_ts)
        S = intensity.shape[0]
        N = intensity[0].numel()
        dev = intensity.device
        it = intensity.reshape(S, N).to(torch.float32).contiguous()
        ts = sample_ts.reshape(S, N).to(torch.float64).contiguous()
        ots = output_ts.reshape(N).to(torch.float64).contiguous()
        prm = params.to(torch.float32).contiguous()
        din = None if reset else delta_in.reshape(N).to(torch.float32).contiguous()
        rts = None if reset else reset_ts.reshape(N).to(torch.float64).contiguous()
        out = torch.empty(N, dtype=torch.float32, device=dev)
        delta_out = torch.empty(N, dtype=torch.float32, device=dev) if reset else torch.zeros(
            N, dtype=torch.float32, device=dev)
        _check(lib().den_pixbw_fwd(S, N, int(reset), _ptr(it), _ptr(ts), _ptr(ots), _ptr(prm), _ptr(din), _ptr(rts),
                                   _ptr(out), _ptr(delta_out) if reset else None, _stream(dev)))
        ctx.save_for_backward(it, ts, ots, prm, din, rts)
        ctx.reset = bool(reset)
        ctx.in_dtype, ctx.in_shape, ctx.p_dtype = intensity.dtype, intensity.shape, params.dtype
        ctx.din_shape = None if reset else delta_in.shape
        ctx.ts_meta = (output_ts.shape, output_ts.dtype, None if reset else reset_ts.shape,
                       None if reset else reset_ts.dtype)
        if not reset:
            ctx.mark_non_differentiable(delta_out)
        batch = intensity.shape[1:]
        return out.reshape(batch), delta_out.reshape(batch)

    @staticmethod
    def backward(ctx, d_out, d_delta):
        it, ts, ots, prm, din, rts = ctx.saved_tensors
        S, N = it.shape
        dev = it.device
        L = lib()
        g = torch.zeros(N, dtype=torch.float32, device=dev) if d_out is None else \
            d_out.reshape(N).to(torch.float32).contiguous()
        dd = d_delta.reshape(N).to(torch.float32).contiguous() if (ctx.reset and d_delta is not None) else None
        ws = torch.empty(L.den_pixbw_workspace_bytes(S, N), dtype=torch.uint8, device=dev)
        nb = L.den_pixbw_blocks(N)
        d_it = torch.empty(S, N, dtype=torch.float32, device=dev)
        d_din = None if ctx.reset else torch.empty(N, dtype=torch.float32, device=dev)
        part = torch.empty(PIXBW_NPARAM * nb, dtype=torch.float32, device=dev)
        _check(L.den_pixbw_bwd(S, N, int(ctx.reset), _ptr(it), _ptr(ts), _ptr(ots), _ptr(prm), _ptr(din), _ptr(rts),
                               _ptr(g), _ptr(dd), _ptr(ws), _ptr(d_it), _ptr(d_din), _ptr(part), _stream(dev)))
        d_prm = torch.empty(PIXBW_NPARAM, dtype=torch.float32, device=dev)
        sum_partials(part, PIXBW_NPARAM, nb, d_prm)
        # the offset decay's dependence on the output / reset timestamps (non-reset calls; the
        # reset call's output_ts is the later calls' reset_ts)
        d_ots = d_rts = None
        if not ctx.reset and (ctx.needs_input_grad[4] or ctx.needs_input_grad[5]):
            d_ots = torch.empty(N, dtype=torch.float64, device=dev) if ctx.needs_input_grad[4] else None
            d_rts = torch.empty(N, dtype=torch.float64, device=dev) if ctx.needs_input_grad[5] else None
            _check(L.den_pixbw_decay_ts_bwd(N, _ptr(ots), _ptr(rts), _ptr(prm), _ptr(din), _ptr(g), _ptr(d_ots),
                                            _ptr(d_rts), _stream(dev)))
            ots_shape, ots_dt, rts_shape, rts_dt = ctx.ts_meta
            d_ots = None if d_ots is None else d_ots.reshape(ots_shape).to(ots_dt)
            d_rts = None if d_rts is None else d_rts.reshape(rts_shape).to(rts_dt)
        return (d_it.reshape(ctx.in_shape).to(ctx.in_dtype), d_prm.to(ctx.p_dtype),
                None if d_din is None else d_din.reshape(ctx.din_shape), None, d_ots, d_rts, None)


# ----------------------------------------------------------------------------- event preparation
def event_prep(num_pos, num_neg, end_ts, start_ts, normalized, ct, refractory, norm_c=None, has_diff=True,
               has_tv=True, out=None):
    """den_event_prep: ContrastThreshold + RefractoryPeriod forward and the diff /
    subdiff timestamps of DeblurENeRF.training_step (deblur_e_nerf.py:414-455).

    num_pos, num_neg, end_ts, start_ts (N) i64; normalized (4,N) f64 [ts_diff,
    diff_start_ts, ts_subdiff, subdiff_start_ts]; ct (2) f32 [C+, C-]; refractory
    (1) f64 (ns).  -> dict(lid (N) f32, start_ts (N) f64, render_ts (4,N) f64,
    ts_diff (N) f64, ts_subdiff (N) f64, target (N) f32 if norm_c is given)."""
    _require_device(num_pos, num_neg, end_ts, start_ts, normalized, ct, refractory, norm_c)
    for t, dt in ((num_pos, torch.int64), (num_neg, torch.int64), (end_ts, torch.int64), (start_ts, torch.int64),
                  (normalized, torch.float64), (ct, torch.float32), (refractory, torch.float64)):
        if t.dtype != dt or not t.is_contiguous():
            raise DenError(f"event_prep: expected contiguous {dt}, got {t.dtype}")
    N = end_ts.numel()
    if normalized.shape != (4, N) or ct.numel() != 2 or refractory.numel() != 1:
        raise DenError("event_prep: bad shapes")
    dev = end_ts.device
    if out is None:
        out = dict(lid=torch.empty(N, device=dev), start_ts=torch.empty(N, dtype=torch.float64, device=dev),
                   render_ts=torch.zeros(4, N, dtype=torch.float64, device=dev),
                   ts_diff=torch.zeros(N, dtype=torch.float64, device=dev),
                   ts_subdiff=torch.zeros(N, dtype=torch.float64, device=dev),
                   target=torch.empty(N, device=dev) if norm_c is not None else None)
    _check(lib().den_event_prep(N, int(has_diff), int(has_tv), _ptr(num_pos), _ptr(num_neg), _ptr(end_ts),
                                _ptr(start_ts), _ptr(normalized), _ptr(ct), _ptr(refractory), _ptr(norm_c),
                                _ptr(out["lid"]), _ptr(out["start_ts"]), _ptr(out["render_ts"]),
                                _ptr(out["ts_diff"]), _ptr(out["ts_subdiff"]), _ptr(out["target"]), _stream(dev)))
    return out


def _pixel_rays_shapes(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation):
    N = pixel_position.shape[0]
    lead = T_wc_position.shape[:-1]
    M = T_wc_position.numel() // (3 * N) if N else 0
    if (intrinsics_inverse.shape != (3, 3) or pixel_position.shape != (N, 2) or lead[-1:] != (N,)
            or T_wc_orientation.shape != (*lead, 3, 3) or M * N * 3 != T_wc_position.numel()):
        raise DenError("pixel_rays: bad shapes")
    return M, N


class PixelRaysFunction(torch.autograd.Function):
    """den_pixel_rays, differentiable in the poses (den_pixel_rays_bwd): the reference's autograd of
    NeRF.pixel_params_to_ray (nerf.py:206-228), the link from the rays back to the trajectory."""

    @staticmethod
    def forward(ctx, intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation):
        M, N = _pixel_rays_shapes(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation)
        o, d = torch.empty_like(T_wc_position), torch.empty_like(T_wc_position)
        _check(lib().den_pixel_rays(M, N, _ptr(intrinsics_inverse), _ptr(pixel_position), _ptr(T_wc_position),
                                    _ptr(T_wc_orientation), _ptr(o), _ptr(d), _stream(pixel_position.device)))
        ctx.save_for_backward(intrinsics_inverse, pixel_position, T_wc_orientation)
        ctx.MN = (M, N)
        return o, d

    @staticmethod
    def backward(ctx, g_o, g_d):
        k_inv, pix, rot = ctx.saved_tensors
        M, N = ctx.MN
        d_pos = torch.empty(rot.shape[:-1], dtype=torch.float32, device=rot.device) if ctx.needs_input_grad[2] else None
        d_rot = torch.empty_like(rot) if ctx.needs_input_grad[3] else None
        if d_pos is None and d_rot is None:
            return None, None, None, None
        g_o = None if g_o is None else g_o.to(torch.float32).contiguous()
        g_d = None if g_d is None else g_d.to(torch.float32).contiguous()
        _check(lib().den_pixel_rays_bwd(M, N, _ptr(k_inv), _ptr(pix), _ptr(rot), _ptr(g_o), _ptr(g_d), _ptr(d_pos),
                                        _ptr(d_rot), _stream(rot.device)))
        return None, None, d_pos, d_rot


def pixel_rays(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation, out=None):
    """den_pixel_rays (NeRF.pixel_params_to_ray, nerf.py:206-228): K^-1 (3,3),
    pixels (N,2), poses ([M,] N, 3) / ([M,] N, 3, 3) -> origins, unit directions
    ([M,] N, 3) f32.  Pixels broadcast over the leading render-group dim M.  Differentiable in
    the poses when they require grad (``out`` must then be None)."""
    _require_device(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation)
    ts = (intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation)
    if any(t.dtype != torch.float32 for t in ts):
        raise DenError("pixel_rays: expected f32 tensors")
    intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation = (t.contiguous() for t in ts)
    if torch.is_grad_enabled() and (T_wc_position.requires_grad or T_wc_orientation.requires_grad):
        if out is not None:
            raise DenError("pixel_rays: `out` buffers are for the no-grad path")
        return PixelRaysFunction.apply(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation)
    M, N = _pixel_rays_shapes(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation)
    if out is None:
        out = (torch.empty_like(T_wc_position), torch.empty_like(T_wc_position))
    _check(lib().den_pixel_rays(M, N, _ptr(intrinsics_inverse), _ptr(pixel_position), _ptr(T_wc_position),
                                _ptr(T_wc_orientation), _ptr(out[0]), _ptr(out[1]),
                                _stream(pixel_position.device)))
    return out


class TrajectoryFunction(torch.autograd.Function):
    """den_trajectory, differentiable in the query timestamps (den_trajectory_bwd): the autograd of
    LinearTrajectory.forward (trajectories.py:30-90, tensor_ops.py:118-184) through its interpolation
    weight -- the refractory period's path to the poses."""

    @staticmethod
    def forward(ctx, cam_ts, cam_pos, cam_quat, query_ts, status):
        shape = query_ts.shape
        q = query_ts.reshape(-1).to(torch.float64).contiguous()
        n = q.numel()
        C = cam_ts.numel()
        ct = cam_ts.to(torch.int64).contiguous()
        cp = cam_pos.to(torch.float32).contiguous()
        cq = cam_quat.to(torch.float32).contiguous()
        pos = torch.empty(n, 3, dtype=torch.float32, device=q.device)
        rot = torch.empty(n, 3, 3, dtype=torch.float32, device=q.device)
        _check(lib().den_trajectory(n, C, _ptr(ct), _ptr(cp), _ptr(cq), _ptr(q), _ptr(pos), _ptr(rot), _ptr(status),
                                    _stream(q.device)))
        ctx.save_for_backward(ct, cp, cq, q)
        ctx.meta = (shape, query_ts.dtype)
        return pos.reshape(*shape, 3), rot.reshape(*shape, 3, 3)

    @staticmethod
    def backward(ctx, g_pos, g_rot):
        ct, cp, cq, q = ctx.saved_tensors
        shape, dt = ctx.meta
        n = q.numel()
        d = torch.empty(n, dtype=torch.float64, device=q.device)
        gp = None if g_pos is None else g_pos.reshape(n, 3).to(torch.float32).contiguous()
        gr = None if g_rot is None else g_rot.reshape(n, 9).to(torch.float32).contiguous()
        _check(lib().den_trajectory_bwd(n, ct.numel(), _ptr(ct), _ptr(cp), _ptr(cq), _ptr(q), _ptr(gp), _ptr(gr),
                                        _ptr(d), _stream(q.device)))
        return None, None, None, d.reshape(shape).to(dt), None


def trajectory(cam_ts, cam_pos, cam_quat, query_ts, status=None):
    """den_trajectory (LinearTrajectory.forward): pose stamps (C) i64, positions (C,3) f32, XYZW
    quaternions (C,4) f32, query timestamps (...) f64 -> positions (..., 3), rotations (..., 3, 3).
    ``status`` (device i32, optional) gets bit 0 for queries outside the pose span.
    Differentiable in query_ts."""
    _require_device(cam_ts, cam_pos, cam_quat, query_ts, status)
    return TrajectoryFunction.apply(cam_ts, cam_pos, cam_quat, query_ts, status)


class EventTargetFunction(torch.autograd.Function):
    """The normalised diff-loss target f32(ts_diff * (lid / (end - start)) / c) (loss.py:72-78),
    differentiable in ts_diff, lid, start and c (den_event_target / den_event_target_bwd)."""

    @staticmethod
    def forward(ctx, ts_diff, lid, end_ts, start_ts, c):
        _require_device(ts_diff, lid, end_ts, start_ts, c)
        td = ts_diff.to(torch.float64).contiguous()
        ld = lid.to(torch.float32).contiguous()
        et = end_ts.to(torch.int64).contiguous()
        st = start_ts.to(torch.float64).contiguous()
        cc = c.to(torch.float32).reshape(1).contiguous()
        N = ld.numel()
        out = torch.empty(N, dtype=torch.float32, device=ld.device)
        _check(lib().den_event_target(N, _ptr(td), _ptr(ld), _ptr(et), _ptr(st), _ptr(cc), _ptr(out),
                                      _stream(ld.device)))
        ctx.save_for_backward(td, ld, et, st, cc)
        ctx.dtypes = (ts_diff.dtype, lid.dtype, start_ts.dtype, c.dtype, c.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        td, ld, et, st, cc = ctx.saved_tensors
        N, dev = ld.numel(), ld.device
        g = g.to(torch.float32).contiguous()
        d_td = torch.empty(N, dtype=torch.float64, device=dev) if ctx.needs_input_grad[0] else None
        d_ld = torch.empty(N, dtype=torch.float32, device=dev) if ctx.needs_input_grad[1] else None
        d_st = torch.empty(N, dtype=torch.float64, device=dev) if ctx.needs_input_grad[3] else None
        d_c = torch.empty(1, dtype=torch.float64, device=dev)
        ws = torch.empty(max(1, lib().den_event_prep_workspace_bytes(N) // 8), dtype=torch.float64, device=dev)
        _check(lib().den_event_target_bwd(N, _ptr(td), _ptr(ld), _ptr(et), _ptr(st), _ptr(cc), _ptr(g), _ptr(d_td),
                                          _ptr(d_ld), _ptr(d_st), _ptr(ws), _ptr(d_c), _stream(dev)))
        t_dt, l_dt, s_dt, c_dt, c_shape = ctx.dtypes
        return (None if d_td is None else d_td.to(t_dt), None if d_ld is None else d_ld.to(l_dt), None,
                None if d_st is None else d_st.to(s_dt), d_c.to(c_dt).reshape(c_shape))


class EventPrepFunction(torch.autograd.Function):
    """den_event_prep with its reverse mode (den_event_prep_bwd): differentiable in C+ / C- (ct,
    (2) f32), tau_r (refractory, (1) f64) and the normalising constant c (norm_c, (1) f32).
    -> lid (N) f32, start_ts (N) f64, render_ts (4,N) f64, ts_diff (N) f64, ts_subdiff (N) f64,
    target (N) f32 (zeros when norm_c is None)."""

    @staticmethod
    def forward(ctx, num_pos, num_neg, end_ts, start_ts, normalized, ct, refractory, norm_c, has_diff, has_tv):
        out = event_prep(num_pos, num_neg, end_ts, start_ts, normalized, ct.detach().float().contiguous(),
                         refractory.detach().double().reshape(1).contiguous(),
                         None if norm_c is None else norm_c.detach().float().reshape(1).contiguous(),
                         has_diff=has_diff, has_tv=has_tv)
        tgt = out["target"] if out["target"] is not None else torch.zeros_like(out["lid"])
        if not ctx.needs_input_grad[6]:
            # tau_r frozen: the timestamps are constants (no pose chain behind the renders)
            ctx.mark_non_differentiable(out["start_ts"], out["render_ts"], out["ts_diff"], out["ts_subdiff"])
        ctx.save_for_backward(num_pos, num_neg, end_ts, start_ts, normalized, ct.detach().float().contiguous(),
                              refractory.detach().double().reshape(1).contiguous(),
                              None if norm_c is None else norm_c.detach().float().reshape(1).contiguous())
        ctx.flags = (has_diff, has_tv, norm_c is not None)
        ctx.shapes = (ct.shape, ct.dtype, refractory.shape, refractory.dtype,
                      None if norm_c is None else (norm_c.shape, norm_c.dtype))
        return out["lid"], out["start_ts"], out["render_ts"], out["ts_diff"], out["ts_subdiff"], tgt

    @staticmethod
    def backward(ctx, g_lid, g_start, g_render, g_tsd, g_tss, g_tgt):
        num_pos, num_neg, end_ts, start_ts, norm, ct, tau, c = ctx.saved_tensors
        has_diff, has_tv, has_c = ctx.flags
        N, dev = end_ts.numel(), end_ts.device
        f = lambda t, dt: None if t is None else t.to(dt).contiguous()  # noqa: E731
        ws = torch.empty(max(1, lib().den_event_prep_workspace_bytes(N) // 8), dtype=torch.float64, device=dev)
        d = torch.empty(4, dtype=torch.float64, device=dev)
        _check(lib().den_event_prep_bwd(N, int(has_diff), int(has_tv), _ptr(num_pos), _ptr(num_neg), _ptr(end_ts),
                                        _ptr(start_ts), _ptr(norm), _ptr(ct), _ptr(tau), _ptr(c),
                                        _ptr(f(g_lid, torch.float32)), _ptr(f(g_start, torch.float64)),
                                        _ptr(f(g_render, torch.float64)), _ptr(f(g_tsd, torch.float64)),
                                        _ptr(f(g_tss, torch.float64)),
                                        _ptr(f(g_tgt, torch.float32)) if has_c else None, _ptr(ws), _ptr(d),
                                        _stream(dev)))
        ct_shape, ct_dtype, tau_shape, tau_dtype, c_meta = ctx.shapes
        d_c = None if c_meta is None else d[3:4].to(c_meta[1]).reshape(c_meta[0])
        return (None, None, None, None, None, d[:2].to(ct_dtype).reshape(ct_shape),
                d[2:3].to(tau_dtype).reshape(tau_shape), d_c, None, None)


def image_error(pred, target):
    """den_image_error: (B, ...) images -> (B, 2) f64 [sum of squared errors, sum of absolute errors]."""
    _require_device(pred, target)
    assert pred.shape == target.shape
    B = pred.shape[0]
    p = pred.reshape(B, -1).to(torch.float32).contiguous()
    t = target.reshape(B, -1).to(torch.float32).contiguous()
    ws = torch.empty(lib().den_image_error_workspace_bytes(B) // 8, dtype=torch.float64, device=p.device)
    out = torch.empty(B, 2, dtype=torch.float64, device=p.device)
    _check(lib().den_image_error(B, p.shape[1], _ptr(p), _ptr(t), _ptr(ws), _ptr(out), _stream(p.device)))
    return out


SSIM_WIN, SSIM_SIGMA, SSIM_K1, SSIM_K2 = 11, 1.5, 0.01, 0.03


def ssim_window():
    """torchmetrics 0.6.2's SSIM window (functional/image/ssim.py _gaussian / _gaussian_kernel): the
    normalised 1-D Gaussian over arange(-5, 6) in f32 and its outer product -> (121,) f32."""
    dist = torch.arange((1 - SSIM_WIN) / 2, (1 + SSIM_WIN) / 2, 1, dtype=torch.float32)
    g = torch.exp(-torch.pow(dist / SSIM_SIGMA, 2) / 2)
    g = (g / g.sum()).unsqueeze(0)
    return torch.matmul(g.t(), g).reshape(-1).contiguous()


def ssim(pred, target, data_range):
    """den_ssim: (B, C, H, W) image pairs -> (B,) f64 mean SSIM index per image (torchmetrics 0.6.2
    functional.ssim with data_range; H, W >= 11)."""
    _require_device(pred, target)
    assert pred.shape == target.shape and pred.dim() == 4
    B, C, H, W = pred.shape
    p = pred.to(torch.float32).contiguous()
    t = target.to(torch.float32).contiguous()
    win = ssim_window()
    c1, c2 = (SSIM_K1 * data_range) ** 2, (SSIM_K2 * data_range) ** 2
    ws = torch.empty(lib().den_ssim_workspace_bytes(B) // 8, dtype=torch.float64, device=p.device)
    out = torch.empty(B, dtype=torch.float64, device=p.device)
    wbuf = (ctypes.c_float * win.numel())(*win.tolist())
    _check(lib().den_ssim(B, C, H, W, _ptr(p), _ptr(t), wbuf, c1, c2, _ptr(ws), _ptr(out), _stream(p.device)))
    return out / (C * (H - 2 * (SSIM_WIN // 2)) * (W - 2 * (SSIM_WIN // 2)))


def png_unfilter(filtered, height, row_bytes, bpp):
    """den_png_unfilter (host): the inflated rows of a non-interlaced PNG (numpy uint8, height x
    (1 + row_bytes)) -> the reconstructed bytes (numpy uint8, height x row_bytes)."""
    import numpy as np
    src = np.ascontiguousarray(filtered, dtype=np.uint8)
    if src.size != height * (row_bytes + 1):
        raise DenError(f"png_unfilter: {src.size} bytes for {height} rows of {row_bytes}")
    out = np.empty(height * row_bytes, dtype=np.uint8)
    _check(lib().den_png_unfilter(height, row_bytes, bpp, src.ctypes.data, out.ctypes.data))
    return out


# ---------------------------------------------------------------- dataset preprocessing
INT64_MAX = (1 << 63) - 1
UNDISTORT_MODELS = {None: 0, "": 0, "plumb_bob": 1, "equidistant": 2}


def _queue_inputs(position, timestamp, img_height, img_width):
    _require_device(position, timestamp)
    if position.dtype != torch.int64 or position.dim() != 2 or position.shape[1] != 2:
        raise DenError("position must be (n, 2) int64 (datasets.py:207: raw uint16 positions cast to np.int64)")
    if timestamp.dtype != torch.int64 or timestamp.shape != (position.shape[0],):
        raise DenError("timestamp must be (n) int64 ns")
    n = position.shape[0]
    ws = torch.empty(lib().den_queue_workspace_bytes(n), dtype=torch.uint8, device=position.device)
    return n, int(img_height), int(img_width), ws, position.contiguous(), timestamp.contiguous()


def _stats(stats, img_height, img_width):
    count, min_iv, n_iv = (int(x) for x in stats.tolist())  # one device -> host read
    if count < 0:
        raise IndexError(f"an event position lies outside the {img_height} x {img_width} image")
    return count, (None if n_iv == 0 else min_iv), n_iv


def queue_raw_events(position, timestamp, polarity, img_height, img_width):
    """Event.queue_raw_events on the device (den_queue_raw_events): raw position (n,2) i64,
    timestamp (n) i64, polarity (n) bool -> (dict of the queued events' position, start_ts,
    end_ts, num_pos, num_neg device tensors, in input order; the maximum refractory period = the
    minimum queued interval, None when there is no interval)."""
    n, H, W, ws, position, timestamp = _queue_inputs(position, timestamp, img_height, img_width)
    _require_device(polarity)
    if polarity.shape != (n,):
        raise DenError("polarity must be (n)")
    pol = polarity.to(torch.uint8).contiguous()
    dev = position.device
    out = {"position": torch.empty(n, 2, dtype=torch.int64, device=dev)}
    for k in ("start_ts", "end_ts", "num_pos", "num_neg"):
        out[k] = torch.empty(n, dtype=torch.int64, device=dev)
    stats = torch.empty(3, dtype=torch.int64, device=dev)
    _check(lib().den_queue_raw_events(n, H, W, _ptr(position), _ptr(timestamp), _ptr(pol), _ptr(ws), ws.numel(),
                                      _ptr(out["position"]), _ptr(out["start_ts"]), _ptr(out["end_ts"]),
                                      _ptr(out["num_pos"]), _ptr(out["num_neg"]), _ptr(stats), _stream(dev)))
    count, min_iv, _ = _stats(stats, H, W)
    return {k: v[:count] for k, v in out.items()}, min_iv


def colorize_events(position, bayer_channel):
    """Event.colorize_events' index map on the device (den_colorize_events): (n,2) i64 positions,
    4 channel indices (top-left, top-right, bottom-left, bottom-right) -> (n) u8."""
    _require_device(position)
    position = position.contiguous()
    out = torch.empty(position.shape[0], dtype=torch.uint8, device=position.device)
    bayer = (ctypes.c_int32 * 4)(*[int(c) for c in bayer_channel])
    _check(lib().den_colorize_events(position.shape[0], _ptr(position), bayer, _ptr(out), _stream(position.device)))
    return out


def max_refractory_period(position, timestamp, img_height, img_width):
    """Event.extract_max_refractory_period on the device (den_max_refractory_period): the minimum
    interval between consecutive distinct timestamps at a pixel, as an int (ns), or None when no
    pixel has two (the reference's inf)."""
    n, H, W, ws, position, timestamp = _queue_inputs(position, timestamp, img_height, img_width)
    stats = torch.empty(3, dtype=torch.int64, device=position.device)
    _check(lib().den_max_refractory_period(n, H, W, _ptr(position), _ptr(timestamp),
                                           _ptr(ws), ws.numel(), _ptr(stats), _stream(position.device)))
    return _stats(stats, H, W)[1]


def undistort_events(position, distortion_model, intrinsics, distortion_params):
    """Event.undistort_events' arithmetic (den_undistort_events): (n,2) i64 positions -> (n,2) f32."""
    _require_device(position)
    n = position.shape[0]
    params = [float(x) for x in distortion_params]
    model = 0 if len(params) == 0 else UNDISTORT_MODELS.get(str(distortion_model))
    if model is None:
        raise NotImplementedError(f"distortion model {distortion_model!r}")  # datasets.py:360-363 (fov and others)
    if model and len(params) != 4:
        raise DenError("distortion_params must hold 4 values")
    K = (ctypes.c_float * 9)(*[float(x) for x in torch.as_tensor(intrinsics).reshape(-1).tolist()])
    D = (ctypes.c_float * 4)(*(params or [0.0] * 4))
    position = position.contiguous()
    out = torch.empty(n, 2, dtype=torch.float32, device=position.device)
    _check(lib().den_undistort_events(n, model, _ptr(position), K, D, _ptr(out), _stream(position.device)))
    return out
