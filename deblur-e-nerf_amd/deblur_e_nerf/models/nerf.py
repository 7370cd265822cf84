"""NeRF renderer -- MI355X-native mirror of the reference's
``deblur_e_nerf/models/nerf.py`` (NeRF, nerf.py:31-286).

Same constructor signature, the same ``forward(ray_origin, ray_direction) ->
(radiance, opacity, depth, mean_num_samples_per_ray)`` contract, the same
``update_occ_grid`` / ``pixel_params_to_ray`` and the same parameter / buffer
names (``radiance_field.*``, ``occupancy_grid.*``,
``parametrizations.render_bkgd.original``).

Two samplers:

* ``sampler="occupancy"`` (default; the reference's): nerfacc-style occupancy-grid
  marching with the constant ``render_step_size`` (or the cone step), the
  early-stop density pre-pass and packed compositing (external/utils.py
  render_image on den_march.hip + the fused MLP at packed samples).
* ``sampler="fixed"``: the fused fixed-count stratified sampler of
  den_render_fwd (``n_samples`` per ray, one jitter per ray while training,
  u = 0 in eval) -- BASELINE.json's "131072 rays x 128 samples" workload, which
  the benchmark and ``train.TrainStep`` run; it marches the AABB and ignores the
  occupancy grid.
"""
import torch

from .. import _native
from ..external import mlp, ngp, utils
from ..external.marching import ContractionType, OccupancyGrid, contraction_id
from ..utils import modules


def _randint(high, size, device=None):
    """torch.randint draws of the occupancy update's cone branch (a random camera per cell point,
    reference nerf.py:178-181); tests substitute the draws a reference run recorded."""
    return torch.randint(0, high, size, device=device)


def shifted_softplus(x, shift=1, beta=1, threshold=20):
    """nerf.py:20-24 (mip-NeRF's density activation): softplus(x - shift).  The fields recognise it by
    name and evaluate it inside their kernels (den density_activation 2: shift 1, beta 1,
    threshold 20); called directly it is the reference's torch expression."""
    return torch.nn.functional.softplus(x - shift, beta, threshold)


class NeRF(torch.nn.Module):
    HIDDEN_ACTIVATION_NAME_TO_FN = {
        "softplus": torch.nn.Softplus(beta=100),
        "relu": torch.nn.ReLU(),
    }
    DENSITY_ACTIVATION_NAME_TO_FN = {
        "shifted_trunc_exp": ngp.shifted_trunc_exp,
        "softplus": torch.nn.Softplus(beta=1),
        "shifted_softplus": shifted_softplus,
    }
    RADIANCE_ACTIVATION_NAME_TO_FN = {
        "softplus": torch.nn.Softplus(beta=1),
        "sigmoid": torch.nn.Sigmoid(),
    }

    def __init__(self, aabb, contraction_type, occ_grid_config, near_plane, far_plane, render_step_size,
                 render_bkgd, cone_angle, early_stop_eps, alpha_thre, test_chunk_size, arch, arch_config, num_dim,
                 radiance_dim, opacity_eps=1e-10, sampler="occupancy", n_samples=128, mode="f32"):
        super().__init__()
        if occ_grid_config is not None:
            assert torch.all(torch.tensor(occ_grid_config.resolution) > 0)
            assert 0 <= occ_grid_config.occ_thre <= 1
            assert 0 <= occ_grid_config.ema_decay <= 1
            assert occ_grid_config.warmup_steps > 0
            assert occ_grid_config.n > 0
        if (near_plane is not None) and (far_plane is not None):
            assert 0 <= near_plane <= far_plane
        assert render_step_size > 0
        assert (render_bkgd is None) or (isinstance(render_bkgd, str) and render_bkgd == "parameter") \
            or isinstance(render_bkgd, torch.Tensor)
        assert cone_angle >= 0 and 0 <= early_stop_eps <= 1 and 0 <= alpha_thre <= 1
        assert test_chunk_size > 0 and num_dim > 0 and radiance_dim > 0 and opacity_eps > 0
        assert sampler in ("occupancy", "fixed")
        if arch not in ("mlp", "ngp"):
            raise NotImplementedError(f"unknown arch {arch!r} (nerf.py:105-164: ngp or mlp)")
        if arch == "ngp" and sampler != "occupancy":
            raise NotImplementedError("the fixed-count sampler runs the fused `mlp` arch; the ngp field marches "
                                      "with the occupancy grid (the reference's sampler)")
        if sampler == "fixed" and contraction_id(contraction_type) != 0:
            raise NotImplementedError("the fixed-count sampler marches the AABB: use contraction_type AABB")
        self.register_buffer("aabb", torch.tensor(aabb), persistent=False)
        # host copies of the constants the marcher takes by value (no device -> host copy per render)
        self._aabb_host = [float(v) for v in aabb]
        self._step_host = float(render_step_size)
        self.contraction_type = contraction_type
        self.occ_grid_config = occ_grid_config
        self.near_plane = near_plane
        self.far_plane = far_plane
        self.register_buffer("render_step_size", torch.tensor(render_step_size), persistent=False)
        if render_bkgd is None:
            self.render_bkgd = None
        elif isinstance(render_bkgd, str):
            self.render_bkgd = torch.nn.parameter.Parameter(torch.ones(radiance_dim))
            torch.nn.utils.parametrize.register_parametrization(self, "render_bkgd", modules.Softplus(beta=1))
        else:
            self.register_buffer("render_bkgd", render_bkgd, persistent=False)
        self.cone_angle = cone_angle
        self.early_stop_eps = early_stop_eps
        self.alpha_thre = alpha_thre
        self.test_chunk_size = test_chunk_size
        self.opacity_eps = opacity_eps
        self.sampler = sampler
        self.n_samples = n_samples
        # the occupancy grid (nerf.py:98-102)
        resolution = occ_grid_config.resolution if occ_grid_config is not None else 128
        self.occupancy_grid = OccupancyGrid(roi_aabb=aabb, resolution=resolution, contraction_type=contraction_type)
        if arch == "ngp":
            # nerf.py:105-142: the activation names resolved, the radiance dim from the sensor
            base = dict(arch_config.mlp_base)
            base["hidden_activation"] = self.HIDDEN_ACTIVATION_NAME_TO_FN[arch_config.mlp_base.hidden_activation]
            base["density_activation"] = self.DENSITY_ACTIVATION_NAME_TO_FN[arch_config.mlp_base.density_activation]
            head = dict(arch_config.mlp_head)
            head["hidden_activation"] = self.HIDDEN_ACTIVATION_NAME_TO_FN[arch_config.mlp_head.hidden_activation]
            head["radiance_activation"] = self.RADIANCE_ACTIVATION_NAME_TO_FN[
                arch_config.mlp_head.radiance_activation]
            head["output_dim"] = radiance_dim
            self.radiance_field = ngp.NGPradianceField(
                aabb=aabb, num_dim=num_dim, use_viewdirs=True, contraction_type=contraction_type,
                pos_encoding_config=dict(arch_config.pos_encoding), dir_encoding_config=dict(arch_config.dir_encoding),
                mlp_base_config=base, mlp_head_config=head)
            return
        self.radiance_field = mlp.VanillaNeRFRadianceField(
            aabb=aabb,
            net_depth=arch_config.net_depth,
            net_width=arch_config.net_width,
            skip_layer=arch_config.skip_layer,
            net_depth_condition=arch_config.net_depth_condition,
            net_width_condition=arch_config.net_width_condition,
            num_dim=num_dim,
            contraction_type=contraction_type,
            radiance_dim=radiance_dim,
            hidden_activation=self.HIDDEN_ACTIVATION_NAME_TO_FN[arch_config.hidden_activation],
            density_activation=self.DENSITY_ACTIVATION_NAME_TO_FN[arch_config.density_activation],
            radiance_activation=self.RADIANCE_ACTIVATION_NAME_TO_FN[arch_config.radiance_activation],
            pos_encoder_max_deg=arch_config.pos_encoder_max_deg,
            view_encoder_max_deg=arch_config.view_encoder_max_deg,
            weight_norm=arch_config.weight_norm,
            mode=mode,
        )

    def update_occ_grid(self, step, T_wc_position):
        """nerf.py:170-204: every ``occ_grid.n`` steps, the EMA occupancy of the grid cells from
        the density at a random point of each sampled cell times the marching step (the cone step
        of a random camera when cone_angle > 0).  No-op for the fixed-count sampler."""
        if self.sampler != "occupancy" or self.occ_grid_config is None:
            return None
        step_size = self.render_step_size

        def occ_eval_fn(x):
            if self.cone_angle > 0.0:
                camera_ids = _randint(len(T_wc_position), (x.shape[0],), device=T_wc_position.device)
                origins = T_wc_position[camera_ids, :]
                t = (origins - x).norm(dim=-1, keepdim=True)
                s = torch.clamp(t * self.cone_angle, min=self.render_step_size)
                if (self.near_plane is not None) and (self.far_plane is not None):
                    s = torch.where((t > self.near_plane) & (t < self.far_plane), s, torch.zeros_like(s))
            else:
                s = step_size
            with torch.no_grad():
                density = self.radiance_field.query_density(x)
            return density * s

        cfg = self.occ_grid_config
        self.occupancy_grid.every_n_step(step, occ_eval_fn, cfg.occ_thre, cfg.ema_decay, cfg.warmup_steps, cfg.n)

    @staticmethod
    def pixel_params_to_ray(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation):
        """nerf.py:206-228 on the device (den_pixel_rays): (3,3), (N,2), ([M,] N, 3),
        ([M,] N, 3, 3) -> ray origins, unit directions ([M,] N, 3); differentiable in the poses
        (den_pixel_rays_bwd) when they require grad."""
        pix = pixel_position.float()
        lead = T_wc_position.shape[:-1]
        if pix.dim() > 2:
            # an image grid of pixels (H, W, 2) with poses (..., H, W, 3) (evaluation_step,
            # deblur_e_nerf.py:620-634): flatten the grid, render groups stay in front
            n = pix.shape[:-1]
            if tuple(lead[len(lead) - len(n):]) != tuple(n):
                raise _native.DenError("pixel_params_to_ray: pixel grid and pose grid differ")
            N = pix[..., 0].numel()
            o, d = _native.pixel_rays(intrinsics_inverse.float().contiguous(), pix.reshape(N, 2).contiguous(),
                                      T_wc_position.float().reshape(-1, N, 3).contiguous(),
                                      T_wc_orientation.float().reshape(-1, N, 3, 3).contiguous())
            return o.reshape(*lead, 3), d.reshape(*lead, 3)
        return _native.pixel_rays(intrinsics_inverse.float().contiguous(), pix.contiguous(),
                                  T_wc_position.float().contiguous(), T_wc_orientation.float().contiguous())

    def _forward_fixed(self, ray_origin, ray_direction):
        shape = ray_origin.shape[:-1]
        o = ray_origin.reshape(-1, 3).float().contiguous()
        d = ray_direction.reshape(-1, 3).float().contiguous()
        R = o.shape[0]
        rf = self.radiance_field
        jitter = torch.rand(R, device=o.device) if self.training else torch.zeros(R, device=o.device)
        # the kernel renders whole workgroup tiles: pad the ray batch
        tile_rays = _native.wg_samples(rf.mode) // self.n_samples
        pad = (-R) % tile_rays
        if pad:
            o = torch.cat([o, o[:1].expand(pad, 3)])
            d = torch.cat([d, d[:1].expand(pad, 3)])
            jitter = torch.cat([jitter, jitter.new_zeros(pad)])
        bkgd = self.render_bkgd
        radiance, opacity, depth = _native.render(
            o, d, jitter, None if bkgd is None else bkgd.float(), rf.flat_leaf(),
            rf.render_cfg(self.near_plane, self.far_plane), rf.packed(), self.n_samples)
        radiance, opacity, depth = radiance[:R], opacity[:R], depth[:R]
        return radiance.reshape(*shape, -1), opacity.reshape(*shape, 1), depth.reshape(*shape, 1), \
            float(self.n_samples) * R

    def forward(self, ray_origin, ray_direction):
        if self.sampler == "fixed":
            radiance, opacity, depth, num_samples_across_rays = self._forward_fixed(ray_origin, ray_direction)
        else:
            rays = utils.Rays(origins=ray_origin, viewdirs=ray_direction)
            ray_marching_aabb = self._aabb_host if contraction_id(self.contraction_type) == 0 else None
            radiance, opacity, depth, num_samples_across_rays = utils.render_image(
                self.radiance_field, self.occupancy_grid, rays, ray_marching_aabb, self.near_plane, self.far_plane,
                self._step_host, self.render_bkgd, self.cone_angle, self.early_stop_eps, self.alpha_thre,
                self.test_chunk_size)
        # nerf.py:279-286
        radiance = radiance.squeeze(dim=-1)
        opacity = opacity.squeeze(dim=-1)
        depth = depth.squeeze(dim=-1)
        depth = depth / (opacity + self.opacity_eps)
        num_rays = ray_origin.numel() // ray_origin.shape[-1]
        mean_num_samples_per_ray = num_samples_across_rays / num_rays
        return radiance, opacity, depth, mean_num_samples_per_ray


__all__ = ["NeRF", "ContractionType", "shifted_softplus"]
