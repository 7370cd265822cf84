/*
 * den_api.h -- C ABI of libden.so, the MI355X-native (gfx950) hot path of
 * Deblur e-NeRF: fused stratified sampling + positional encoding + 8x256 NeRF
 * MLP (MFMA) + alpha compositing, its backward, the pixel-bandwidth sensor
 * model and the event loss.
 *
 * Plain C: pointers, sizes and an opaque stream handle (hipStream_t passed as
 * void*).  No torch types.  Every device pointer is caller-owned device memory
 * (the PyTorch caching allocator on the Python side); the library allocates
 * nothing and keeps no state except a thread-local last-error string.
 * All calls are stream-ordered and capturable into a hipGraph.
 *
 * Return value of every int function: 0 on success, otherwise a DEN_E* code;
 * den_last_error() gives text.  Nothing in the library aborts or exits.
 *
 * The reference interface each entry point replaces (paths relative to the
 * reference repo wengflow/deblur-e-nerf @ 2024-10-22):
 *   den_render_fwd   <- deblur_e_nerf/models/nerf.py:230-286 NeRF.forward ->
 *                       external/utils.py:38-140 render_image (nerfacc
 *                       ray_marching + rendering) -> external/mlp.py:350-358
 *                       VanillaNeRFRadianceField.forward ->
 *                       external/vol_rendering.py:16-128 rendering
 *   den_render_bwd   <- torch autograd through the same chain (nerfacc's
 *                       custom transmittance backward + nn.Linear backward)
 *   den_dw_reduce /  <- the weight-gradient half of nn.Linear backward
 *   den_dw_gemm         (cuBLAS split-K in the reference)
 *   den_pack_weights <- (no reference counterpart: MFMA fragment layout)
 *   den_pixbw_*      <- deblur_e_nerf/models/pixel_bandwidth.py:298-494
 *                       PixelBandwidth.sample_intensity / forward and
 *                       utils/control.py:29-123 foh_cont2discrete
 *   den_event_prep   <- deblur_e_nerf/models/event_generation_params.py:106-118
 *                       ContrastThreshold.forward, :230-237 RefractoryPeriod.forward
 *                       and the timestamp derivation of
 *                       deblur_e_nerf/models/deblur_e_nerf.py:418-455 training_step
 *   den_pixel_rays   <- deblur_e_nerf/models/nerf.py:206-228 NeRF.pixel_params_to_ray
 *   den_trajectory   <- deblur_e_nerf/models/trajectories.py:30-90 LinearTrajectory.forward
 *   den_*_ray_grad / den_pixel_rays_bwd / den_trajectory_bwd / den_pixbw_*_ts_bwd
 *                    <- torch autograd from the renders back to the render timestamps (the
 *                       refractory-period gradient through the camera pose, deblur_e_nerf.py:419-455)
 *   den_event_loss_* <- deblur_e_nerf/loss_metric/loss.py:34-96 Loss.compute
 *   den_event_target
 *   den_image_error  <- deblur_e_nerf/loss_metric/metric.py:28-92 (L1, PSNR)
 *   den_ssim         <- deblur_e_nerf/loss_metric/metric.py:74-81 (torchmetrics 0.6.2 ssim)
 *   den_png_unfilter <- the PNG decode inside cv2.imread, deblur_e_nerf/data/datasets.py:504-509
 *                       (PosedImage.load_posed_imgs; host code)
 *   den_adam_step    <- torch.optim.Adam as configured by
 *                       deblur_e_nerf/models/deblur_e_nerf.py:1055-1112
 *   den_march_* / den_visibility / den_compact / den_pack_info / den_exclusive_scan
 *                    <- nerfacc 0.3.1 ray_marching (+ render_visibility), called at
 *                       deblur_e_nerf/external/utils.py:106-119
 *   den_composite_*  <- deblur_e_nerf/external/vol_rendering.py:81-126 (nerfacc
 *                       render_weight_from_density + accumulate_along_rays)
 *   den_occ_*        <- nerfacc OccupancyGrid.every_n_step, called at
 *                       deblur_e_nerf/models/nerf.py:170-204
 *   den_ngp_* / den_hashgrid_*
 *                    <- deblur_e_nerf/external/ngp.py:109-280 NGPradianceField (tcnn.Encoding
 *                       HashGrid + MLP + SHEncoder) forward / backward
 *   den_queue_raw_events / den_max_refractory_period / den_colorize_events / den_undistort_events
 *                    <- deblur_e_nerf/data/datasets.py:133-187, 190-328, 331-364 (Event's
 *                       raw_events.npz -> events.pt / max_refractory_period.pt build path)
 */
#ifndef DEN_API_H
#define DEN_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DEN_VERSION 7  /* 7: den_render_desc.max_workgroups (two render calls sharing the chip);
                          6: den_ssim / den_png_unfilter (the evaluation views and metrics);
                          5: den_queue_raw_events / den_max_refractory_period / den_colorize_events /
                          den_undistort_events; den_render_desc.ray_grad;
                          4: density_activation in den_render_desc / den_ngp_desc; den_sh_encode_* */

enum den_status {
  DEN_OK = 0,
  DEN_EINVAL = 1,      /* bad argument / null pointer / inconsistent sizes */
  DEN_EUNSUPPORTED = 2,/* shape or configuration outside what the kernels implement */
  DEN_EHIP = 3         /* a HIP runtime call failed */
};

/* Arithmetic mode of the fused MLP. */
enum den_mode {
  DEN_MODE_F32 = 0,  /* parity mode: f32 operands, f32 MFMA (16x16x4), exact f32 FMA chains */
  DEN_MODE_BF16 = 1  /* perf mode: bf16 operands, f32 accumulate (32x32x16 MFMA) */
};

/* Radiance-field / renderer configuration.  The MLP shape is the reference's
 * `mlp` arch (configs/train/synthetic.yaml:104-114): depth 8, width 256, skip
 * after layer 4, condition depth 1 width 128, pos-enc degree 10, view-enc
 * degree 4, softplus(beta=100) hidden activation, shifted_trunc_exp density,
 * softplus radiance.  radiance_dim in {1, 3}. */
typedef struct den_render_desc {
  int32_t mode;            /* den_mode */
  int32_t radiance_dim;    /* 1 or 3 */
  int32_t n_rays;          /* rays in this call */
  int32_t n_samples;       /* samples per ray, fixed count, 64..(128 F32 / 256 BF16),
                              dividing it; n_rays * n_samples a multiple of
                              den_render_tile_samples(mode) */
  float aabb[6];           /* min xyz, max xyz (nerf.py:212, AABB contraction) */
  float near_plane;        /* < 0 => none */
  float far_plane;         /* < 0 => none */
  int32_t train;           /* 1: keep activations in the workspace for den_render_bwd */
  int32_t has_bkgd;        /* 1: composite over bkgd (render_bkgd, nerf.py:219-230) */
  int32_t points;          /* 0: render rays with the fused fixed-count sampler + compositing.
                              1: evaluate the radiance field at given points instead
                              (VanillaNeRFRadianceField.forward, mlp.py:350-358):
                              rays_o/rays_d = per-point positions/directions (n,3),
                              n = n_rays*n_samples; out_rgb = rgb (n,rd), out_opacity =
                              sigma (n); in den_render_bwd d_rgb/d_opacity are dL/drgb,
                              dL/dsigma per point.
                              2: the same for packed ray-marching samples (the rgb_sigma_fn
                              closure of external/utils.py:83-96): sample s is at
                              rays_o[r] + rays_d[r] * (t_starts[s] + t_ends[s]) / 2 with
                              r = ray_indices[s], viewed along rays_d[r]; n = n_rays*n_samples
                              samples (pad with zero-length samples of any valid ray). */
  int32_t contraction;     /* input-space contraction (mlp.py:321-335): 0 AABB, 1 tanh
                              (ngp.py:96-106), 2 unbounded sphere (ngp.py:68-93); the
                              fixed-count sampler (points = 0) needs 0 */
  int32_t bwd_path;        /* BF16 backward: 0 layer-major hidden layers + streamed weight
                              gradients (in place: dz_l overwrites the forward activation S_{l+1},
                              l = 0..6, so one train forward feeds ONE den_render_bwd);
                              1 the F32 mode's sample-major chain + split-K GEMMs on the same bf16
                              operands (an A/B reference path).  F32 mode ignores it. */
  int32_t density_activation; /* models/nerf.py:20-29: 0 shifted_trunc_exp (exp(x - 1), gradient
                              clamped at exp(15), external/ngp.py:45-61), 1 softplus(beta 1,
                              threshold 20), 2 shifted_softplus (softplus(x - 1)) */
  int32_t ray_grad;        /* 1: den_render_ray_grad follows the backward (the gradient into the rays,
                              the refractory period's pose path): the BF16 layer-major backward then
                              keeps dz_g in the workspace for it (otherwise dz_g never leaves the chip) */
  int32_t max_workgroups;  /* 0: the persistent launches (BF16 forward, head backward, layer-major hidden
                              layers, streamed weight gradients) run one workgroup per CU; > 0: at most
                              this many, so that two render calls on two streams can share the chip
                              (profiles/split_probe.py: one half's forward beside the other half's
                              backward -- slower than the two in sequence).  No reference
                              counterpart (a launch-shape knob). */
} den_render_desc;

/* Device buffers of one render call. */
typedef struct den_render_io {
  const float* rays_o;     /* (R,3) */
  const float* rays_d;     /* (R,3) unit directions */
  const float* jitter;     /* (R)   stratified offset u in [0,1) */
  const void* w_fwd;       /* packed forward fragments   (den_pack_weights) */
  const void* w_bwd;       /* packed transposed fragments (den_pack_weights) */
  const float* bias_pk;    /* packed biases               (den_pack_weights) */
  const float* bkgd;       /* (rd) post-activation background, or NULL */
  void* workspace;         /* den_render_workspace_bytes() bytes */
  float* out_rgb;          /* (R,rd) composited radiance */
  float* out_opacity;      /* (R) */
  float* out_depth;        /* (R) sum_i w_i t_mid_i (not yet divided by opacity) */
  const int32_t* ray_indices; /* points = 2: (n) ray of each packed sample */
  const float* t_starts;   /* points = 2: (n) */
  const float* t_ends;     /* points = 2: (n) */
} den_render_io;

/* Upstream gradients / outputs of den_render_bwd. */
typedef struct den_render_grad {
  const float* d_rgb;      /* (R,rd) dL/d out_rgb */
  const float* d_opacity;  /* (R) or NULL */
  const float* d_depth;    /* (R) or NULL */
  float* grad_params;      /* flat f32 gradient buffer, reference state-dict order
                              of nerf.radiance_field.mlp.* (den_param_count) --
                              OVERWRITTEN (not accumulated) */
  float* grad_bkgd;        /* (rd) dL/d bkgd (post-activation), or NULL -- overwritten */
} den_render_grad;

int den_version(void);
/* Samples per render workgroup tile: n_rays * n_samples must be a multiple of it
 * (128 in F32 mode, 512 in BF16 mode). */
int32_t den_render_tile_samples(int32_t mode);
const char* den_last_error(void);

/* Kernel timing, for measurement only (bench.py's roofline).  While enabled,
 * every render-path launch is bracketed by two hipEvents recorded on its own
 * stream.  den_timing_collect waits for them and returns, per kernel class
 * (0 render_fwd_kernel, 1 render_bwd_kernel, 2 hidden_bwd_kernel,
 * 3 dw_gemm_kernel, 4 dw_reduce_kernel), the summed duration in ms and the
 * launch count since the last collect.  No reference counterpart. */
int den_timing_enable(int32_t on);
int den_timing_collect(int32_t n_classes, double* total_ms, int64_t* launches);

/* Number of f32 parameters of the MLP (595,844 for rd=3) and the offset of the
 * tensor `idx` in the flat buffer, in the reference's named_parameters() order:
 * base.hidden_layers.{0..7}.{weight,bias}, sigma_layer.output_layer.{w,b},
 * bottleneck_layer.output_layer.{w,b}, rgb_layer.hidden_layers.0.{w,b},
 * rgb_layer.output_layer.{w,b}  (24 tensors). */
int64_t den_param_count(int32_t radiance_dim);
int64_t den_param_offset(int32_t radiance_dim, int32_t idx);

/* Sizes of the packed weight buffers for a mode. */
size_t den_packed_fwd_bytes(int32_t mode);
size_t den_packed_bwd_bytes(int32_t mode);
size_t den_packed_bias_bytes(int32_t mode);

/* flat f32 params (den_param_count) -> MFMA fragment layouts. */
int den_pack_weights(int32_t mode, int32_t radiance_dim, const float* params,
                     void* w_fwd, void* w_bwd, float* bias_pk, void* stream);

size_t den_render_workspace_bytes(const den_render_desc* desc);

int den_render_fwd(const den_render_desc* desc, const den_render_io* io, void* stream);

/* Requires the workspace of a preceding den_render_fwd with train=1 and the
 * same desc/io.  Writes grad_params (overwrite) and grad_bkgd. */
int den_render_bwd(const den_render_desc* desc, const den_render_io* io,
                   const den_render_grad* grad, void* stream);
/* den_render_bwd in two stream-ordered halves (for profiling / overlap):
 * part 1 = compositing adjoint + MLP dz chain (one kernel), part 2 = weight /
 * bias / background gradients from the dz written by part 1.  On the BF16
 * layer-major path part 1 also writes the hidden layers' gradients, and (unless
 * desc.ray_grad) the L0 / L5-pe weight-gradient partials that part 2 reduces: call
 * part 2 after part 1 on the same desc / io / workspace. */
int den_render_bwd_part(const den_render_desc* desc, const den_render_io* io,
                        const den_render_grad* grad, int32_t part, void* stream);

/* Gradient of the render with respect to its rays (the rays' part of the reference's autograd:
 * positions o + d (t0 + t1) / 2 and view direction d, external/utils.py:83-96, with the marching
 * intervals detached as nerfacc returns them).  After den_render_bwd on the same desc / io
 * (train = 1): reads the layer gradients it left in the workspace and the flat parameters
 * (reference order, den_param_offset).  points 0: d_rays_o / d_rays_d (n_rays, 3) of the fixed-count
 * rays; points 2: (n_rays_out, 3) of the rays the packed samples index, whose first n_valid samples
 * have sorted ray_indices (the rest is padding without gradient); points 1: (n, 3) per point /
 * direction.  Overwritten.  rg_workspace: den_render_ray_grad_workspace_bytes(desc) bytes.
 * Replaces: the autograd of origins[ray_indices] + viewdirs * t and of the encoders / MLP inputs. */
size_t den_render_ray_grad_workspace_bytes(const den_render_desc* desc);
int den_render_ray_grad(const den_render_desc* desc, const den_render_io* io, const float* params,
                        int32_t n_rays_out, int64_t n_valid, void* rg_workspace, float* d_rays_o, float* d_rays_d,
                        void* stream);
/* Reverse mode of den_pixel_rays with respect to the poses (nerf.py:206-228 autograd):
 * g_ray_o / g_ray_d (M,N,3) (either may be NULL = 0) -> d_t_pos (M,N,3), d_t_rot (M,N,3,3)
 * (either may be NULL; overwritten). */
int den_pixel_rays_bwd(int32_t M, int32_t N, const float* k_inv, const float* pixel, const float* t_rot,
                       const float* g_ray_o, const float* g_ray_d, float* d_t_pos, float* d_t_rot, void* stream);
/* Reverse mode of den_trajectory with respect to the query timestamps (trajectories.py:30-90 +
 * tensor_ops.py:118-184 autograd; the pose samples are buffers): g_position (n,3), g_rotation
 * (n,3,3) (either may be NULL) -> d_query_ts (n) f64, overwritten. */
int den_trajectory_bwd(int64_t n, int32_t C, const int64_t* cam_ts, const float* cam_pos, const float* cam_quat,
                       const double* query_ts, const float* g_position, const float* g_rotation, double* d_query_ts,
                       void* stream);

/* ---------------------------------------------------------------- pixel bandwidth
 * Per-event pixel-bandwidth model (pixel_bandwidth.py).  Parameters are the
 * post-softplus values (the module's parametrised attributes) in this order:
 *   [0] tau_in_it_eff_prod (buffer) [1] tau_mil_it_eff_prod [2] A_amp_inv
 *   [3] A_loop_inv [4] tau_out [5] tau_sf [6] tau_diff                        */
#define DEN_PIXBW_NPARAM 7

/* sample_ts (S,N) f64 from gen (S-1,N) f64 and output_ts (N) f64
 * (pixel_bandwidth.py:311-360; un-clamped). */
int den_pixbw_sample_ts(int32_t S, int32_t N, const double* gen, const double* output_ts,
                        double omega_c_min, double max_cumprob, double* sample_ts, void* stream);

/* Reverse mode of den_pixbw_sample_ts with respect to output_ts (the lifetimes are out of autograd,
 * pixel_bandwidth.py:298-367): d_output_ts (N) f64 = sum_k g_sample_ts (k, n), overwritten. */
int den_pixbw_sample_ts_bwd(int32_t S, int32_t N, const double* g_sample_ts, double* d_output_ts, void* stream);

/* Forward.  intensity (S,N) f32, sample_ts (S,N) f64.  reset != 0: writes
 * delta_out (N) and returns out = sf log-intensity; otherwise reads delta_in
 * (N) and reset_ts (N) f64 and applies the decay.  weights_out (S,N,o) f32
 * optional (may be NULL). */
int den_pixbw_fwd(int32_t S, int32_t N, int32_t reset, const float* intensity,
                  const double* sample_ts, const double* output_ts, const float* params,
                  const float* delta_in, const double* reset_ts, float* out,
                  float* delta_out, void* stream);

/* Backward.  d_out (N), d_delta_out (N, reset only, may be NULL) ->
 * d_intensity (S,N) (overwrite), d_delta_in (N, non-reset only; overwrite),
 * d_params_partial (DEN_PIXBW_NPARAM x n_blocks f32 partial sums; the caller
 * sums them with den_sum_partials).  n_blocks = den_pixbw_blocks(N).
 * workspace: den_pixbw_workspace_bytes(S, N) bytes (f64 Phi / Bd / Btd of every
 * segment and the running row vectors of the weight recurrence). */
int den_pixbw_blocks(int32_t N);
size_t den_pixbw_workspace_bytes(int32_t S, int32_t N);
int den_pixbw_bwd(int32_t S, int32_t N, int32_t reset, const float* intensity,
                  const double* sample_ts, const double* output_ts, const float* params,
                  const float* delta_in, const double* reset_ts, const float* d_out,
                  const float* d_delta_out, void* workspace, float* d_intensity, float* d_delta_in,
                  float* d_params_partial, void* stream);

/* Timestamp gradients of a non-reset call's offset decay (pixel_bandwidth.py:435-446):
 * out = y - delta_in exp(-1e-9 f32(output_ts - reset_ts) / tau_diff) -> d_output_ts = -d_reset_ts =
 * d_out delta_in e 1e-9 / tau_diff (N) f64, either may be NULL. */
int den_pixbw_decay_ts_bwd(int32_t N, const double* output_ts, const double* reset_ts, const float* params,
                           const float* delta_in, const float* d_out, double* d_output_ts, double* d_reset_ts,
                           void* stream);

/* ---------------------------------------------------------------- event loss
 * One term of Loss.compute (loss.py:62-96) over N events:
 *   err_i = f(x_i / c - t_i),  L = mean_{i valid} err_i
 * x = rendered log-intensity difference (f32), c = normalising constant (the
 * mean contrast threshold, or 1), t = normalised target (NULL => 0, the TV
 * term).  error_fn: 0 = l1, 1 = mse, 2 = huber(delta = 1), 3 = mape.  valid: u8 mask or
 * NULL (all valid).  No valid event => L = NaN (torch's empty mean).
 * workspace: den_event_loss_workspace_bytes(N), shared by fwd and bwd (bwd
 * reads the valid count left by fwd). */
size_t den_event_loss_workspace_bytes(int32_t N);
int den_event_loss_fwd(int32_t N, int32_t error_fn, const float* x, const float* target, const uint8_t* valid,
                       const float* norm_c, float* loss, void* workspace, void* stream);
/* g_loss = dTotal/dL (device scalar).  Writes d_x (N), d_target (N, may be NULL)
 * and d_c (1) = dTotal/dc through the x/c input (target's c-dependence is the
 * caller's chain rule through d_target). */
int den_event_loss_bwd(int32_t N, int32_t error_fn, const float* x, const float* target, const uint8_t* valid,
                       const float* norm_c, const float* g_loss, float* d_x, float* d_target, float* d_c,
                       void* workspace, void* stream);
/* Normalised diff-term target (loss.py:74-77), f64 arithmetic rounded to f32:
 *   t_i = f32( ts_diff_i * (lid_i / (end_ts_i - start_ts_i)) / c ) */
int den_event_target(int32_t N, const double* ts_diff, const float* lid, const int64_t* end_ts,
                     const double* start_ts, const float* norm_c, float* target, void* stream);

/* Fused measurement step for pixel_bandwidth.enable = false
 * (DeblurENeRF.training_step, deblur_e_nerf.py:472-549): radiance of the 4
 * render groups [diff start, diff end, tv start, tv end] x N events (rd
 * channels, bayer channel per event when rd = 3) -> I = radiance + min_int,
 * y = log I, L_diff = mean_valid f_d((y1-y0)/c - target),
 * L_tv = mean_valid f_t((y3-y2)/c), total = w_d L_diff + w_t L_tv.
 * valid = opacity > 0 at start or end unless has_bkgd (deblur_e_nerf.py:1204-1207).
 * out[0..2] = L_diff, L_tv, total.  The bwd writes d total / d radiance
 * (4,N,rd) and must follow the fwd on the same workspace. */
size_t den_event_step_workspace_bytes(int32_t N);
int den_event_step_fwd(int32_t N, int32_t rd, int32_t fn_d, int32_t fn_t, int32_t has_bkgd, float min_int,
                       float w_d, float w_t, const float* radiance, const float* opacity, const int64_t* channel,
                       const float* target, const float* norm_c, void* workspace, float* out, void* stream);
int den_event_step_bwd(int32_t N, int32_t rd, int32_t fn_d, int32_t fn_t, int32_t has_bkgd, float min_int,
                       float w_d, float w_t, const float* radiance, const float* opacity, const int64_t* channel,
                       const float* target, const float* norm_c, void* workspace, float* d_radiance, void* stream);

/* ---------------------------------------------------------------- event preparation
 * The event corrections and supervision timestamps of DeblurENeRF.training_step,
 * one thread per event:
 *   lid       = f32(num_pos) * C+ - f32(num_neg) * C-         (ContrastThreshold.forward)
 *   start_out = f64(start_ts) + tau_r                          (RefractoryPeriod.forward)
 *   has_diff: dt = (end - start_out) * norm[0]; s = lerp(start_out, max(end - dt, start_out), norm[1]);
 *             e = min(s + dt, end); render_ts[0] = s, render_ts[1] = e, ts_diff = dt,
 *             target = f32(dt * (lid / (end - start_out)) / norm_c)  (loss.py:74-77; needs norm_c)
 *   has_tv:   the same on [s, e] (or [start_out, end] without has_diff) with norm[2], norm[3]
 *             -> render_ts[2], render_ts[3], ts_subdiff
 * norm (4,N) f64 = the datamodule's normalized ts_diff, diff_start_ts, ts_subdiff,
 * subdiff_start_ts samples; ct (2) f32 = C+, C- and refractory (1) f64 = tau_r ns are
 * the modules' post-parametrisation values (device scalars).  render_ts (4,N) f64 is
 * the [diff start, diff end, tv start, tv end] timestamp grid the renders consume.
 * ts_diff, ts_subdiff, target may be NULL.  Its reverse mode is den_event_prep_bwd (C+/C-/tau_r
 * are learnable in configs/train/07_*.yaml: ct_freeze / refr_freeze false). */
int den_event_prep(int32_t N, int32_t has_diff, int32_t has_tv, const int64_t* num_pos, const int64_t* num_neg,
                   const int64_t* end_ts, const int64_t* start_ts, const double* norm, const float* ct,
                   const double* refractory, const float* norm_c, float* lid, double* start_out, double* render_ts,
                   double* ts_diff, double* ts_subdiff, float* target, void* stream);

/* Reverse mode of den_event_prep (gradients of ContrastThreshold / RefractoryPeriod / the
 * timestamp derivation / the loss target, with torch's lerp / maximum / minimum derivative
 * conventions): upstream gradients g_lid (N) f32, g_start (N) f64, g_render_ts (4,N) f64,
 * g_ts_diff, g_ts_subdiff (N) f64, g_target (N) f32 -- each may be NULL -- give
 * d_params (4) f64 = [dL/dC+, dL/dC-, dL/dtau_r, dL/dnorm_c].  workspace:
 * den_event_prep_workspace_bytes(N). */
size_t den_event_prep_workspace_bytes(int32_t N);
int den_event_prep_bwd(int32_t N, int32_t has_diff, int32_t has_tv, const int64_t* num_pos, const int64_t* num_neg,
                       const int64_t* end_ts, const int64_t* start_ts, const double* norm, const float* ct,
                       const double* refractory, const float* norm_c, const float* g_lid, const double* g_start,
                       const double* g_render_ts, const double* g_ts_diff, const double* g_ts_subdiff,
                       const float* g_target, void* workspace, double* d_params, void* stream);
/* Reverse mode of den_event_target: d_ts_diff (N) f64, d_lid (N) f32, d_start (N) f64 (each may be
 * NULL, overwritten) and d_c (1) f64 = dL/dnorm_c.  workspace: den_event_prep_workspace_bytes(N). */
int den_event_target_bwd(int32_t N, const double* ts_diff, const float* lid, const int64_t* end_ts,
                         const double* start_ts, const float* norm_c, const float* g_target, double* d_ts_diff,
                         float* d_lid, double* d_start, void* workspace, double* d_c, void* stream);

/* Rays of M render groups x N pixels (NeRF.pixel_params_to_ray):
 *   ray_d[m,n] = normalize(t_rot[m,n] @ (k_inv @ [pixel[n], 1])),  ray_o[m,n] = t_pos[m,n]
 * k_inv (3,3) row-major, pixel (N,2), t_pos (M,N,3), t_rot (M,N,3,3) row-major, f32.
 * ray_o, ray_d (M,N,3): exactly the (R,3) ray layout den_render_fwd reads, R = M*N. */
int den_pixel_rays(int32_t M, int32_t N, const float* k_inv, const float* pixel, const float* t_pos,
                   const float* t_rot, float* ray_o, float* ray_d, void* stream);

/* ---------------------------------------------------------------- packed rendering (nerfacc path)
 * The reference's occupancy-grid marching + volume rendering (models/nerf.py:98-102,170-204,
 * 230-286 -> external/utils.py:38-140 -> external/vol_rendering.py:16-128), i.e. nerfacc 0.3.1's
 * ray_marching / render_visibility / render_weight_from_density / accumulate_along_rays /
 * OccupancyGrid (environment.yml:32; restated, not vendored).  Packed samples are sorted by
 * ray; offsets (n_rays + 1) i64 = exclusive scan of the per-ray counts (packed_info).
 * Grids are (res0, res1, res2) u8 in meshgrid "ij" order, 1 = occupied. */

/* t_min / t_max per ray: AABB slab test (aabb NULL: 0 / 1e10; a miss: 1e10 / 1e10), clamped by
 * near / far (< 0: none), then t_min += jitter * step when jitter != NULL (stratified)
 * (nerfacc ray_marching prologue, called at external/utils.py:106-119). */
int den_march_prep(int32_t n_rays, const float* rays_o, const float* rays_d, const float* aabb, float near_plane,
                   float far_plane, const float* jitter, float step, float* t_min, float* t_max, void* stream);
/* Per-ray sample counts of the constant / cone step march with occupancy skipping (DDA skip for
 * the AABB contraction).  grid NULL: no skipping (roi/res unused). */
int den_march_count(int32_t n_rays, const float* rays_o, const float* rays_d, const float* t_min, const float* t_max,
                    const float* roi, const int32_t* res, const uint8_t* grid, int32_t contraction, float step,
                    float cone, int32_t* counts, void* stream);
/* The same march writing the packed samples at offsets (from den_exclusive_scan of the counts). */
int den_march_fill(int32_t n_rays, const float* rays_o, const float* rays_d, const float* t_min, const float* t_max,
                   const float* roi, const int32_t* res, const uint8_t* grid, int32_t contraction, float step,
                   float cone, const int64_t* offsets, int32_t* ray_indices, float* t_starts, float* t_ends,
                   void* stream);
/* offsets[0..n] = exclusive scan of counts[0..n) (offsets[n] = total). */
size_t den_scan_workspace_bytes(int64_t n);
int den_exclusive_scan(int64_t n, const int32_t* counts, int64_t* offsets, void* workspace, void* stream);
/* offsets (n_rays + 1) of n samples with sorted ray_indices (nerfacc pack_info). */
int den_pack_info(int32_t n_rays, int64_t n, const int32_t* ray_indices, int64_t* offsets, void* stream);
/* render_visibility: alpha = 1 - exp(-sigma (t1 - t0)) (or given alphas), T = exclusive cumprod
 * (1 - alpha); keep = T >= early_stop_eps [and alpha >= alpha_thre when alpha_thre > 0];
 * counts = kept samples per ray. */
int den_visibility(int32_t n_rays, const int64_t* offsets, const float* t_starts, const float* t_ends,
                   const float* sigmas, const float* alphas, float early_stop_eps, float alpha_thre, uint8_t* keep,
                   int32_t* counts, void* stream);
/* Keep the samples with keep != 0, at out_offsets (exclusive scan of den_visibility's counts). */
int den_compact(int32_t n_rays, const int64_t* offsets, const uint8_t* keep, const int64_t* out_offsets,
                const int32_t* ray_indices, const float* t_starts, const float* t_ends, int32_t* out_ray_indices,
                float* out_t_starts, float* out_t_ends, void* stream);
/* vol_rendering.rendering after rgb_sigma_fn: weights from density, colours (n_rays, rd),
 * opacities (n_rays), depths (n_rays) = sum w (t0 + t1)/2, colours += bkgd (1 - opacity). */
int den_composite_fwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts, const float* t_ends,
                      const float* sigmas, const float* rgbs, const float* bkgd, float* colors, float* opacities,
                      float* depths, void* stream);
/* Its adjoint: d_sigmas (n), d_rgbs (n, rd) overwritten; d_bkgd (rd, may be NULL) overwritten,
 * using workspace of den_composite_workspace_bytes. d_opacities / d_depths may be NULL. */
size_t den_composite_workspace_bytes(int32_t n_rays, int32_t rd);
int den_composite_bwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts, const float* t_ends,
                      const float* sigmas, const float* rgbs, const float* bkgd, const float* d_colors,
                      const float* d_opacities, const float* d_depths, float* d_sigmas, float* d_rgbs, float* d_bkgd,
                      void* workspace, void* stream);
/* The same from alphas (nerfacc render_weight_from_alpha: w_i = alpha_i prod_{j<i} (1 - alpha_j); the
 * rgb_alpha_fn branch of vol_rendering.py:16-27,96-106): `alphas` in place of the sigmas, d_alphas out. */
int den_composite_alpha_fwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts,
                            const float* t_ends, const float* alphas, const float* rgbs, const float* bkgd,
                            float* colors, float* opacities, float* depths, void* stream);
int den_composite_alpha_bwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts,
                            const float* t_ends, const float* alphas, const float* rgbs, const float* bkgd,
                            const float* d_colors, const float* d_opacities, const float* d_depths, float* d_alphas,
                            float* d_rgbs, float* d_bkgd, void* workspace, void* stream);
/* OccupancyGrid._update, part 1: world positions of the sampled cells (cell index + jitter in
 * [0,1)^3, / res, inverse contraction); mask = 0 for cells outside the unit sphere (sphere
 * contraction); marks the sampled cells in `sampled` (cells bytes, zero on entry). */
int den_occ_points(int64_t m, const int64_t* cell_indices, const float* jitter, const int32_t* res, const float* roi,
                   int32_t contraction, float* points, uint8_t* mask, uint8_t* sampled, void* stream);
/* part 2, after the density at the points: occs[c] *= ema_decay on the sampled cells, then
 * occs[idx] = max(occs[idx], sigma * step) (step_sizes (m) or the constant step_size), then
 * binary = occs > min(mean(occs), occ_thre).  Clears `sampled`.  workspace: den_occ_workspace_bytes. */
size_t den_occ_workspace_bytes(void);
int den_occ_update(int64_t m, const int64_t* cell_indices, const uint8_t* mask, const float* sigmas,
                   const float* step_sizes, float step_size, float ema_decay, float occ_thre, int64_t cells,
                   float* occs, uint8_t* sampled, uint8_t* binary, void* workspace, void* stream);

/* Camera poses at n timestamps (LinearTrajectory.forward, models/trajectories.py:30-90):
 * searchsorted over the C sorted pose stamps cam_ts (i64 ns), lerp of the positions (C,3) and
 * shortest-path slerp of the XYZW orientations (C,4) (utils/tensor_ops.py:118-184), then
 * quaternion -> row-major rotation matrix; query_ts (n) f64 ns -> position (n,3), rotation (n,3,3)
 * f32.  status (optional, device i32): bit 0 is OR-ed in when a query lies outside
 * [cam_ts[0], cam_ts[C-1]] (the reference asserts; the pose is clamped to the end bins). */
int den_trajectory(int64_t n, int32_t C, const int64_t* cam_ts, const float* cam_pos, const float* cam_quat,
                   const double* query_ts, float* position, float* rotation, int32_t* status, void* stream);

/* Evaluation image errors (Metric.compute, loss_metric/metric.py:28-92): for n_img images of
 * `pixels` f32 values each, sse_sae (n_img, 2) f64 = [sum (pred - target)^2, sum |pred - target|]
 * (PSNR = 10 log10(range^2 / (sse / pixels)), L1 = sae / pixels).  workspace:
 * den_image_error_workspace_bytes(n_img). */
size_t den_image_error_workspace_bytes(int32_t n_img);
int den_image_error(int32_t n_img, int64_t pixels, const float* pred, const float* target, void* workspace,
                    double* sse_sae, void* stream);

/* ---------------------------------------------------------------- ngp radiance field
 * The `ngp` arch (external/ngp.py:109-280 NGPradianceField, the default of configs/train/*.yaml):
 * tiny-cuda-nn multiresolution grid encoding (tcnn.Encoding, otype HashGrid / DenseGrid, Linear
 * interpolation, 2 features per level, <= 16 levels), mlp_base 32 -> 64 -> 1 + 15, SH degree 4,
 * mlp_head 31 -> 64 -> 64 -> rd (n_neurons 64, 1 / 2 hidden layers, geo_feat_dim 15: the
 * shipped configs; others are DEN_EUNSUPPORTED), shifted_trunc_exp density.
 * Flat parameters (f32): the grid table (den_ngp_table_params floats, tcnn's level-major layout),
 * then mlp_base.1.hidden_layers.0.{weight,bias}, mlp_base.1.output_layer.{weight,bias},
 * mlp_head.hidden_layers.{0,1}.{weight,bias}, mlp_head.output_layer.{weight,bias} (torch (out, in)).
 * Replaces: tcnn.Encoding forward / backward (CUDA) and the torch nn.Linear / SHEncoder /
 * activation kernels of NGPradianceField.forward and its autograd backward. */
typedef struct den_ngp_desc {
  int32_t radiance_dim;          /* 1 or 3 */
  int32_t n_levels;              /* 1..16 */
  int32_t n_features_per_level;  /* 2 */
  int32_t log2_hashmap_size;
  int32_t base_resolution;
  float per_level_scale;
  int32_t grid_type;             /* 0 HashGrid, 1 DenseGrid */
  int32_t hidden_activation;     /* 0 softplus(beta=100), 1 relu (models/nerf.py:17-20) */
  int32_t radiance_activation;   /* 0 softplus(beta=1), 1 sigmoid (models/nerf.py:26-29) */
  int32_t contraction;           /* 0 AABB, 1 UN_BOUNDED_TANH, 2 UN_BOUNDED_SPHERE */
  float aabb[6];
  int32_t density_activation;    /* as den_render_desc.density_activation */
} den_ngp_desc;

/* Grid-table floats (tcnn sizing: per level min(next_multiple(res^3, 8), 2^log2_hashmap_size)
 * entries x 2) and all flat parameters; -1 for an unsupported descriptor. */
int64_t den_ngp_table_params(const den_ngp_desc* desc);
int64_t den_ngp_param_count(const den_ngp_desc* desc);
/* Workspace of a training forward + backward over n samples (saved activations, per-layer
 * gradients, weight-gradient partials); 0 for inference. */
size_t den_ngp_workspace_bytes(const den_ngp_desc* desc, int64_t n, int32_t train);
/* Field at n samples.  points = 1: x (n,3) positions and d (n,3) directions; points = 2: packed
 * ray-marching samples, x / d = ray origins / unit directions (R,3), ray_idx (n) i32, t0 / t1 (n)
 * (position o + d (t0 + t1) / 2, external/utils.py:83-96).  density_only skips the head (the
 * marching pre-pass sigma_fn; out_rgb may be null).  train = 1 keeps what den_ngp_bwd needs in
 * the workspace.  Outputs: rgb (n, rd), sigma (n). */
int den_ngp_fwd(const den_ngp_desc* desc, int64_t n, int32_t points, const float* x, const float* d,
                const int32_t* ray_idx, const float* t0, const float* t1, const float* params, int32_t density_only,
                int32_t train, void* workspace, float* out_rgb, float* out_sigma, void* stream);
/* Gradient of sum(d_rgb * rgb) + sum(d_sigma * sigma) w.r.t. the flat parameters of the last
 * training forward over the same workspace.  grad_params is overwritten (the table part is
 * cleared on the stream, then scattered with f32 atomics as tcnn does). */
int den_ngp_bwd(const den_ngp_desc* desc, int64_t n, const float* params, void* workspace, const float* d_rgb,
                const float* d_sigma, float* grad_params, void* stream);
/* Gradient of the same field with respect to its inputs, after den_ngp_bwd on the same workspace:
 * tcnn's input gradient of the Linear grid encoding + the SH encoder and the contraction.  points 1:
 * d_x, d_d (n,3) per point; points 2: (n_rays, 3) per ray (sorted ray_idx), position o + d (t0+t1)/2
 * and view direction d as in den_ngp_fwd.  rg_workspace: den_ngp_ray_grad_workspace_bytes(n). */
size_t den_ngp_ray_grad_workspace_bytes(int64_t n);
int den_ngp_ray_grad(const den_ngp_desc* desc, int64_t n, int32_t points, int32_t n_rays, const float* x,
                     const float* d, const int32_t* ray_idx, const float* t0, const float* t1, const float* params,
                     void* workspace, void* rg_workspace, float* d_x, float* d_d, void* stream);
/* tcnn.Encoding alone: x (n,3) in [0,1] -> out (n, 2 n_levels); backward accumulates
 * (atomic adds, caller zeroes) d_table += dL/dtable. */
int den_hashgrid_fwd(const den_ngp_desc* desc, int64_t n, const float* x, const float* table, float* out,
                     void* stream);
int den_hashgrid_bwd(const den_ngp_desc* desc, int64_t n, const float* x, const float* d_out, float* d_table,
                     void* stream);
/* SHEncoder alone (external/sh_encoder.py:15-193): real spherical harmonics of degree 1..8 of
 * coords (n,3) -> out (n, degree^2), the tcnn basis and sign convention, f32; the polynomials are
 * evaluated as written (unit length is not assumed).  The backward writes d_coords (n,3) =
 * sum_k d_out[:,k] dY_k/d(x,y,z), the autograd gradient of the reference module. */
int den_sh_encode_fwd(int64_t n, int32_t degree, const float* coords, float* out, void* stream);
int den_sh_encode_bwd(int64_t n, int32_t degree, const float* coords, const float* d_out, float* d_coords,
                      void* stream);

/* ---------------------------------------------------------------- reductions / optimizer */
/* out[j] = sum_b partial[j*n_blocks + b] for j < n (deterministic order). */
int den_sum_partials(int32_t n, int32_t n_blocks, const float* partial, float* out, void* stream);

/* torch.optim.Adam (amsgrad=False, L2 weight decay added to the gradient) on a
 * flat f32 buffer; per-element lr / weight decay via group ids. */
int den_adam_step(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  float lr, float beta1, float beta2, float eps, float weight_decay,
                  int64_t step, void* stream);
/* The same for f64 parameters (the refractory period, event_generation_params.py:196-201). */
int den_adam_step_f64(int64_t n, double* param, const double* grad, double* exp_avg, double* exp_avg_sq, double lr,
                      double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream);

/* ---------------------------------------------------------------- dataset preprocessing */
/* Raw events (raw_events.npz: position (n,2) cast to i64, timestamp (n) i64 ns, polarity (n) bool
 * as u8 0/1) -> queued events, replacing the per-event Python loops of
 *   data/datasets.py:190-284 Event.queue_raw_events and
 *   data/datasets.py:133-187 Event.extract_max_refractory_period
 *   (called from models/event_generation_params.py:136-149 RefractoryPeriod.__init__).
 * An event is queued iff an earlier raw event (input order) lies at its pixel with a different
 * timestamp t_prev (the immediately preceding one at that pixel); it becomes [start_ts = t_prev,
 * end_ts = t], num_pos = its polarity, num_neg = 1 - num_pos, in input order.  The maximum
 * refractory period is the minimum of t - t_prev over the queued events (the reference's
 * per-pixel deduplicated sliding window gives the same intervals).
 * Outputs (device, caller-allocated with room for n events): out_position (n,2) i64, out_start_ts,
 * out_end_ts, out_num_pos, out_num_neg (n) i64.  out_stats (device, 3 i64): [queued count M (-1 if
 * any position lies outside the img_height x img_width image: the reference raises IndexError),
 * minimum interval (INT64_MAX when none: the reference's inf), number of intervals].  The first M
 * entries of each output are the queued events.  Bit-exact integer work: a stable LSD radix sort
 * of the pixel keys (values = event indices), then neighbours. */
size_t den_queue_workspace_bytes(int64_t n);
int den_queue_raw_events(int64_t n, int32_t img_height, int32_t img_width, const int64_t* position,
                         const int64_t* timestamp, const uint8_t* polarity, void* workspace, size_t workspace_bytes,
                         int64_t* out_position, int64_t* out_start_ts, int64_t* out_end_ts, int64_t* out_num_pos,
                         int64_t* out_num_neg, int64_t* out_stats, void* stream);
/* data/datasets.py:287-328 Event.colorize_events: out_channel_idx (n) u8 = bayer_channel[(x odd) +
 * 2 (y odd)] for positions (n,2) i64; bayer_channel is a HOST pointer to the 4 channel indices
 * (0..2) of the pattern's letters (R 0, G 1, B 2) in top-left, top-right, bottom-left,
 * bottom-right order.  (A monochrome camera, pattern "", has no channel: the caller skips it.) */
int den_colorize_events(int64_t n, const int64_t* position, const int32_t* bayer_channel, uint8_t* out_channel_idx,
                        void* stream);
/* Only out_stats of den_queue_raw_events (Event.extract_max_refractory_period); the same workspace. */
int den_max_refractory_period(int64_t n, int32_t img_height, int32_t img_width, const int64_t* position,
                              const int64_t* timestamp, void* workspace, size_t workspace_bytes, int64_t* out_stats,
                              void* stream);
/* data/datasets.py:331-364 Event.undistort_events: positions (n,2) i64 cast to f32 (the default
 * dtype), then model 0 = none (the cast only), 1 = plumb_bob (cv2.undistortPoints, k1 k2 p1 p2,
 * 5 fixed-point iterations), 2 = equidistant (cv2.fisheye.undistortPoints, k1..k4, Newton on
 * theta, 10 iterations / 1e-8; unconverged or flipped points -> -1e6), re-projected with
 * P = intrinsics; double arithmetic, f32 out (n,2).  intrinsics (row-major 3x3 f32) and distortion
 * (4 f32) are HOST pointers.  OpenCV is absent from this image: parity unpinned. */
int den_undistort_events(int64_t n, int32_t model, const int64_t* position, const float* intrinsics,
                         const float* distortion, float* out, void* stream);

/* ---------------------------------------------------------------- evaluation (PosedImage, Metric) */
/* SSIM of n_img (channels, height, width) f32 image pairs (loss_metric/metric.py:74-81 ->
 * torchmetrics 0.6.2 functional.ssim: 11 x 11 Gaussian window, sigma 1.5; c1 = (0.01 range)^2,
 * c2 = (0.03 range)^2 with range = the metric's max_target_val).  torchmetrics crops 5 pixels on
 * every side after its reflect-padded convolution, so only windows inside the image count:
 * ssim_sum (n_img) f64 = the sum of the SSIM index over channels x (height - 10) x (width - 10)
 * (the caller divides).  window: HOST pointer to the 121 f32 weights (torchmetrics' outer product
 * of the normalised 1-D Gaussian).  height, width >= 11.  workspace: den_ssim_workspace_bytes(n_img). */
size_t den_ssim_workspace_bytes(int32_t n_img);
int den_ssim(int32_t n_img, int32_t channels, int32_t height, int32_t width, const float* pred, const float* target,
             const float* window, float c1, float c2, void* workspace, double* ssim_sum, void* stream);
/* HOST function: PNG scanline unfiltering (filter types 0-4 per row, bytewise, the left neighbour
 * bpp bytes back): filtered = height rows of [filter type byte | row_bytes bytes] (the inflated IDAT
 * stream of a non-interlaced PNG), out = height x row_bytes reconstructed bytes.  Used for the 16-bit
 * colour views (data/datasets.py:508 reads them with cv2.imread); DEN_EINVAL on an unknown type. */
int den_png_unfilter(int64_t height, int64_t row_bytes, int32_t bpp, const uint8_t* filtered, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* DEN_API_H */
