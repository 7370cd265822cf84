// den_events.hip -- event preparation and pixel rays: the steps of
// DeblurENeRF.training_step in front of the render.
//
//   event_prep_kernel   (one thread per event; i64 / f64 / f32 elementwise, HBM-bound)
//     a1  ContrastThreshold.forward     event_generation_params.py:106-118
//           dlogI = f32(n+) * C+  -  f32(n-) * C-        (i64 counts x f32 0-d tensors -> f32)
//     a2  RefractoryPeriod.forward      event_generation_params.py:230-237
//           start = f64(start_ts) + tau_r                (i64 + f64 0-d tensor -> f64)
//     a3  diff / subdiff timestamps     deblur_e_nerf.py:418-455
//           dt = (end - start) * u_dt ; s = lerp(start, max(end - dt, start), u_s) ; e = min(s + dt, end)
//         and the normalised diff target of Loss.log_intensity_diff (loss.py:74-77), fused.
//   pixel_rays_kernel   (one thread per (render group, event))
//     a5  NeRF.pixel_params_to_ray      nerf.py:206-228
//           d = normalize(R_wc (K^-1 [u, v, 1]^T)) ; o = p_wc
//
// Rounding follows the reference's CPU arithmetic: products and sums are kept
// separate (no contraction) where torch evaluates them as separate tensor ops,
// and lerp is torch's two-sided fused form (ATen lerp_vec: fma(w, end - start, start)
// for |w| < 0.5, fma(w - 1, end - start, end) otherwise).
#include "den_device.h"

namespace den {

struct EventPrepArgs {
  int N, has_diff, has_tv;
  const int64_t* num_pos;      // (N)
  const int64_t* num_neg;      // (N)
  const int64_t* end_ts;       // (N) ns
  const int64_t* start_ts;     // (N) ns, before the refractory shift
  const double* norm;          // (4,N): ts_diff, diff_start_ts, ts_subdiff, subdiff_start_ts
  const float* ct;             // (2): C+, C- (post-parametrisation)
  const double* refractory;    // (1): tau_r ns (post-parametrisation)
  const float* norm_c;         // (1) mean contrast threshold for the target, or null
  float* lid;                  // (N)
  double* start_out;           // (N) refractory-shifted start
  double* render_ts;           // (4,N): diff start, diff end, subdiff start, subdiff end
  double* ts_diff;             // (N) diff interval, or null
  double* ts_subdiff;          // (N) subdiff interval, or null
  float* target;               // (N) normalised diff target, or null
};

__device__ __forceinline__ double torch_lerp(double a, double b, double w) {
  const double d = b - a;
  return fabs(w) < 0.5 ? fma(w, d, a) : fma(w - 1.0, d, b);
}

#pragma clang fp contract(off)
__global__ void event_prep_kernel(EventPrepArgs E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E.N) return;
  const int N = E.N;
  // a1
  const float lid = (float)E.num_pos[i] * E.ct[0] - (float)E.num_neg[i] * E.ct[1];
  E.lid[i] = lid;
  // a2
  const double end = (double)E.end_ts[i];
  const double start = (double)E.start_ts[i] + E.refractory[0];
  E.start_out[i] = start;
  // a3
  double tv_s = start, tv_e = end;
  if (E.has_diff) {
    const double dt = (end - start) * E.norm[i];
    const double s = torch_lerp(start, fmax(end - dt, start), E.norm[N + i]);
    const double e = fmin(s + dt, end);
    E.render_ts[i] = s;
    E.render_ts[N + i] = e;
    if (E.ts_diff) E.ts_diff[i] = dt;
    if (E.target) E.target[i] = (float)(dt * ((double)lid / (end - start)) / (double)E.norm_c[0]);
    tv_s = s;
    tv_e = e;
  }
  if (E.has_tv) {
    const double dt = (tv_e - tv_s) * E.norm[2 * N + i];
    const double s = torch_lerp(tv_s, fmax(tv_e - dt, tv_s), E.norm[3 * N + i]);
    const double e = fmin(s + dt, tv_e);
    E.render_ts[2 * N + i] = s;
    E.render_ts[3 * N + i] = e;
    if (E.ts_subdiff) E.ts_subdiff[i] = dt;
  }
}

// (M,N) rays from N pixels (broadcast over the M render groups) and (M,N) poses.
__global__ void pixel_rays_kernel(int M, int N, const float* __restrict__ k_inv, const float* __restrict__ pixel,
                                  const float* __restrict__ t_pos, const float* __restrict__ t_rot,
                                  float* __restrict__ ray_o, float* __restrict__ ray_d) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= (int64_t)M * N) return;
  const int n = (int)(r % N);
  const float u = pixel[2 * n], v = pixel[2 * n + 1];
  float kp[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) kp[a] = (k_inv[3 * a] * u + k_inv[3 * a + 1] * v) + k_inv[3 * a + 2];
  const float* R = t_rot + 9 * r;
  float dd[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) dd[a] = (R[3 * a] * kp[0] + R[3 * a + 1] * kp[1]) + R[3 * a + 2] * kp[2];
  const float nrm = sqrtf((dd[0] * dd[0] + dd[1] * dd[1]) + dd[2] * dd[2]);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    ray_d[3 * r + a] = dd[a] / nrm;
    ray_o[3 * r + a] = t_pos[3 * r + a];
  }
}
#pragma clang fp contract(on)

}  // namespace den
