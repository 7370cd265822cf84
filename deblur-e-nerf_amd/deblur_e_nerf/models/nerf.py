"""NeRF renderer -- MI355X-native mirror of the reference's
``deblur_e_nerf/models/nerf.py`` (NeRF, nerf.py:31-286).

Same constructor signature (plus ``n_samples`` and ``mode``), same
``forward(ray_origin, ray_direction) -> (radiance, opacity, depth,
mean_num_samples_per_ray)`` contract and the same parameter names
(``radiance_field.*``, ``parametrizations.render_bkgd.original``).

Ray marching: nerfacc's occupancy-grid marching with a constant
``render_step_size`` and early stopping (external/utils.py:106-119) is replaced
by the fused fixed-count stratified sampler of den_render_fwd (n_samples per
ray, one jitter per ray while training, u = 0 in eval as nerfacc's
``stratified=radiance_field.training``).  The packed occupancy-grid path is the
next row of SURVEY.md 8(f) (#1); ``update_occ_grid`` is accepted and ignored.
"""
import torch

from .. import _native
from ..external import mlp, ngp
from ..utils import modules


def shifted_softplus(x, shift=1, beta=1, threshold=20):
    raise NotImplementedError("only the shifted_trunc_exp density activation is fused (nerf.py:22)")


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
                 radiance_dim, opacity_eps=1e-10, n_samples=128, mode="f32"):
        super().__init__()
        if (near_plane is not None) and (far_plane is not None):
            assert 0 <= near_plane <= far_plane
        assert render_step_size > 0
        assert (render_bkgd is None) or (isinstance(render_bkgd, str) and render_bkgd == "parameter") \
            or isinstance(render_bkgd, torch.Tensor)
        assert cone_angle >= 0 and 0 <= early_stop_eps <= 1 and 0 <= alpha_thre <= 1
        assert test_chunk_size > 0 and num_dim > 0 and radiance_dim > 0 and opacity_eps > 0
        if arch != "mlp":
            raise NotImplementedError("the ngp arch (tcnn HashGrid) is out of scope; use arch: mlp")
        self.register_buffer("aabb", torch.tensor(aabb), persistent=False)
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
        self.n_samples = n_samples
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
        """Occupancy-grid update (nerf.py:170-204): not needed by the fixed-count
        sampler; kept so the reference's training_step runs unchanged."""
        return None

    @staticmethod
    def pixel_params_to_ray(intrinsics_inverse, pixel_position, T_wc_position, T_wc_orientation):
        """nerf.py:206-228 on the device (den_pixel_rays): (3,3), (N,2), ([M,] N, 3),
        ([M,] N, 3, 3) -> ray origins, unit directions ([M,] N, 3).  Forward only:
        pose refinement (gradients into the trajectory) is out of scope."""
        return _native.pixel_rays(intrinsics_inverse.float().contiguous(), pixel_position.float().contiguous(),
                                  T_wc_position.float().contiguous(), T_wc_orientation.float().contiguous())

    def forward(self, ray_origin, ray_direction):
        shape = ray_origin.shape[:-1]
        o = ray_origin.reshape(-1, 3).float().contiguous()
        d = ray_direction.reshape(-1, 3).float().contiguous()
        R = o.shape[0]
        rf = self.radiance_field
        if self.training:
            jitter = torch.rand(R, device=o.device)
        else:
            jitter = torch.zeros(R, device=o.device)
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
        radiance = radiance.reshape(*shape, -1).squeeze(-1)
        opacity = opacity.reshape(shape)
        depth = depth.reshape(shape) / (opacity + self.opacity_eps)
        return radiance, opacity, depth, float(self.n_samples)
