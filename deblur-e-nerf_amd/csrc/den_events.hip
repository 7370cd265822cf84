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
// Reverse mode of pixel_rays_kernel (NeRF.pixel_params_to_ray autograd): with y = R (K^-1 [u v 1]),
// d = y / |y|:  dL/dy = (g_d - d (d . g_d)) / |y|,  dL/dR = dL/dy (K^-1 [u v 1])^T,  dL/dp = g_o.
// Overwrites d_t_pos (M,N,3) / d_t_rot (M,N,3,3); either may be null.
__global__ void pixel_rays_bwd_kernel(int M, int N, const float* __restrict__ k_inv, const float* __restrict__ pixel,
                                      const float* __restrict__ t_rot, const float* __restrict__ g_o,
                                      const float* __restrict__ g_d, float* __restrict__ d_t_pos,
                                      float* __restrict__ d_t_rot) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= (int64_t)M * N) return;
  const int n = (int)(r % N);
  const float u = pixel[2 * n], v = pixel[2 * n + 1];
  float kp[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) kp[a] = (k_inv[3 * a] * u + k_inv[3 * a + 1] * v) + k_inv[3 * a + 2];
  const float* R = t_rot + 9 * r;
  float y[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) y[a] = (R[3 * a] * kp[0] + R[3 * a + 1] * kp[1]) + R[3 * a + 2] * kp[2];
  const float nrm = sqrtf((y[0] * y[0] + y[1] * y[1]) + y[2] * y[2]);
  float gd[3], dd[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    gd[a] = g_d ? g_d[3 * r + a] : 0.0f;
    dd[a] = y[a] / nrm;
  }
  const float dot = (dd[0] * gd[0] + dd[1] * gd[1]) + dd[2] * gd[2];
  if (d_t_rot)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float gy = (gd[a] - dd[a] * dot) / nrm;
#pragma unroll
      for (int b = 0; b < 3; ++b) d_t_rot[9 * r + 3 * a + b] = gy * kp[b];
    }
  if (d_t_pos)
#pragma unroll
    for (int a = 0; a < 3; ++a) d_t_pos[3 * r + a] = g_o ? g_o[3 * r + a] : 0.0f;
}

// ------------------------------------------------------------------ event preparation: backward
// Reverse mode of event_prep_kernel (and of the loss target), per event in f64, with torch's
// derivative conventions: lerp(a, b, w) -> (1 - w, w); maximum / minimum -> the larger / smaller
// argument, split in half on a tie.  Upstream gradients (each optional): lid (N) f32, start (N)
// f64, render_ts (4,N) f64, ts_diff / ts_subdiff (N) f64, target (N) f32.  Per block partial sums
// of dL/dC+, dL/dC-, dL/dtau_r, dL/dc -> part[4][nb] (f64).
struct EventPrepBwdArgs {
  EventPrepArgs F;             // the forward's inputs (outputs unused)
  const float* g_lid;
  const double* g_start;
  const double* g_render;
  const double* g_ts_diff;
  const double* g_ts_subdiff;
  const float* g_target;
  double* part;                // [4][gridDim.x]
};

__device__ __forceinline__ void max_bwd(double a, double b, double g, double* ga, double* gb) {
  if (a > b) *ga += g;
  else if (b > a) *gb += g;
  else { *ga += 0.5 * g; *gb += 0.5 * g; }
}
__device__ __forceinline__ void min_bwd(double a, double b, double g, double* ga, double* gb) {
  if (a < b) *ga += g;
  else if (b < a) *gb += g;
  else { *ga += 0.5 * g; *gb += 0.5 * g; }
}

constexpr int PREP_BWD_BLOCK = 256;

__global__ void event_prep_bwd_kernel(EventPrepBwdArgs B) {
  const EventPrepArgs& E = B.F;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};  // dC+, dC-, dtau, dc
  if (i < E.N) {
    const int N = E.N;
    const double npos = (double)(float)E.num_pos[i], nneg = (double)(float)E.num_neg[i];
    const float lid = (float)E.num_pos[i] * E.ct[0] - (float)E.num_neg[i] * E.ct[1];
    const double end = (double)E.end_ts[i];
    const double start = (double)E.start_ts[i] + E.refractory[0];
    // forward recompute
    double dt = 0, m = 0, s = start, e = end;
    if (E.has_diff) {
      dt = (end - start) * E.norm[i];
      m = fmax(end - dt, start);
      s = torch_lerp(start, m, E.norm[N + i]);
      e = fmin(s + dt, end);
    }
    const double tvs = s, tve = e;
    double a_start = B.g_start ? B.g_start[i] : 0.0, a_end = 0.0, a_lid = B.g_lid ? (double)B.g_lid[i] : 0.0;
    double a_s = B.g_render ? B.g_render[i] : 0.0, a_e = B.g_render ? B.g_render[N + i] : 0.0;
    double a_dt = B.g_ts_diff ? B.g_ts_diff[i] : 0.0;
    if (E.has_tv) {
      const double u2 = E.norm[2 * N + i], u3 = E.norm[3 * N + i];
      const double dt2 = (tve - tvs) * u2;
      const double m2 = fmax(tve - dt2, tvs);
      const double s2 = torch_lerp(tvs, m2, u3);
      double a_s2 = B.g_render ? B.g_render[2 * N + i] : 0.0, a_e2 = B.g_render ? B.g_render[3 * N + i] : 0.0;
      double a_dt2 = B.g_ts_subdiff ? B.g_ts_subdiff[i] : 0.0, a_tvs = 0.0, a_tve = 0.0, a_m2 = 0.0, a_sum = 0.0;
      // e2 = min(s2 + dt2, tve)
      {
        double ga = 0.0, gb = 0.0;
        min_bwd(s2 + dt2, tve, a_e2, &ga, &gb);
        a_sum += ga;
        a_tve += gb;
      }
      a_s2 += a_sum;
      a_dt2 += a_sum;
      // s2 = lerp(tvs, m2, u3)
      a_tvs += a_s2 * (1.0 - u3);
      a_m2 += a_s2 * u3;
      // m2 = max(tve - dt2, tvs)
      {
        double ga = 0.0, gb = 0.0;
        max_bwd(tve - dt2, tvs, a_m2, &ga, &gb);
        a_tve += ga;
        a_dt2 -= ga;
        a_tvs += gb;
      }
      // dt2 = (tve - tvs) * u2
      a_tve += a_dt2 * u2;
      a_tvs -= a_dt2 * u2;
      if (E.has_diff) { a_s += a_tvs; a_e += a_tve; }
      else { a_start += a_tvs; a_end += a_tve; }
    }
    if (E.has_diff) {
      const double u0 = E.norm[i], u1 = E.norm[N + i];
      // target = f32(dt * (lid / (end - start)) / c)
      if (B.g_target && E.norm_c) {
        const double gt = (double)B.g_target[i], c = (double)E.norm_c[0], D = end - start;
        const double G = (double)lid / D, T = dt * G / c;
        a_dt += gt * G / c;
        a_lid += gt * dt / (D * c);
        a_start += gt * dt * (double)lid / (D * D * c);
        acc[3] += -gt * T / c;
      }
      // e = min(s + dt, end)
      double a_sum = 0.0;
      {
        double ga = 0.0, gb = 0.0;
        min_bwd(s + dt, end, a_e, &ga, &gb);
        a_sum += ga;
        a_end += gb;
      }
      a_s += a_sum;
      a_dt += a_sum;
      // s = lerp(start, m, u1)
      a_start += a_s * (1.0 - u1);
      const double a_m = a_s * u1;
      // m = max(end - dt, start)
      {
        double ga = 0.0, gb = 0.0;
        max_bwd(end - dt, start, a_m, &ga, &gb);
        a_end += ga;
        a_dt -= ga;
        a_start += gb;
      }
      // dt = (end - start) * u0
      a_start -= a_dt * u0;
      a_end += a_dt * u0;
    }
    acc[0] = a_lid * npos;
    acc[1] = -a_lid * nneg;
    acc[2] = a_start;
  }
  __shared__ double sh[4][PREP_BWD_BLOCK];
  for (int q = 0; q < 4; ++q) sh[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int w = PREP_BWD_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int q = 0; q < 4; ++q) sh[q][threadIdx.x] += sh[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int q = 0; q < 4; ++q) B.part[q * gridDim.x + blockIdx.x] = sh[q][0];
}

// the loss target alone (Loss.log_intensity_diff, loss.py:72-78):
//   t = f32(ts_diff * (lid / (end - start)) / c): gradients to ts_diff, lid, start and c (partials)
__global__ void event_target_bwd_kernel(int N, const double* ts_diff, const float* lid, const int64_t* end_ts,
                                        const double* start_ts, const float* c, const float* g_target,
                                        double* d_ts_diff, float* d_lid, double* d_start, double* dc_part) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double dc = 0.0;
  if (i < N) {
    const double gt = (double)g_target[i], cc = (double)c[0], D = (double)end_ts[i] - start_ts[i];
    const double G = (double)lid[i] / D, T = ts_diff[i] * G / cc;
    if (d_ts_diff) d_ts_diff[i] = gt * G / cc;
    if (d_lid) d_lid[i] = (float)(gt * ts_diff[i] / (D * cc));
    if (d_start) d_start[i] = gt * ts_diff[i] * (double)lid[i] / (D * D * cc);
    dc = -gt * T / cc;
  }
  __shared__ double sh[PREP_BWD_BLOCK];
  sh[threadIdx.x] = dc;
  __syncthreads();
  for (int w = PREP_BWD_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) dc_part[blockIdx.x] = sh[0];
}

// out[j] = sum_b part[j * nb + b] (f64, fixed order)
__global__ void sum_partials_f64_kernel(int n, int nb, const double* part, double* out) {
  const int j = blockIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += part[(int64_t)j * nb + b];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = red[0];
}

// ------------------------------------------------------------------ camera trajectory
// LinearTrajectory.forward (models/trajectories.py:30-90), one thread per query timestamp:
//   right = searchsorted(T_wc_timestamp, t) ; left = (t == ts[0]) ? right : right - 1
//   w = f32((t - ts[left]) / (ts[left+1] - ts[left]))          (f64, bin_width = diff of the i64 stamps)
//   position = lerp(p[left], p[right], w)                         (torch's two-sided form)
//   orientation = unitquat_to_rotmat(slerp(q[left], q[right], w))  (utils/tensor_ops.py:118-184: shortest
//     path, relative rotation as a full-angle rotation vector, scaled by w, back to a quaternion)
// in f32 with RoMa 1.2.7's formulas (XYZW quaternions; small-angle series below 1e-3 rad).
struct TrajArgs {
  int64_t n;
  int C;
  const int64_t* cam_ts;  // (C) sorted ns
  const float* cam_pos;   // (C, 3)
  const float* cam_q;     // (C, 4) XYZW unit quaternions
  const double* query;    // (n) ns
  float* pos;             // (n, 3)
  float* rot;             // (n, 3, 3) row-major
  int* status;            // bit 0: a query outside [ts[0], ts[C-1]] (the reference asserts), or null
};

__device__ __forceinline__ float lerp_f(float a, float b, float w) {
  const float d = b - a;
  return fabsf(w) < 0.5f ? fmaf(w, d, a) : fmaf(w - 1.0f, d, b);
}

__device__ __forceinline__ void quat_mul(const float* p, const float* q, float* o) {
  // roma.quat_product: xyz = p_w q_xyz + q_w p_xyz + p_xyz x q_xyz ; w = p_w q_w - p_xyz . q_xyz
  const float c0 = p[1] * q[2] - p[2] * q[1], c1 = p[2] * q[0] - p[0] * q[2], c2 = p[0] * q[1] - p[1] * q[0];
  o[0] = (p[3] * q[0] + q[3] * p[0]) + c0;
  o[1] = (p[3] * q[1] + q[3] * p[1]) + c1;
  o[2] = (p[3] * q[2] + q[3] * p[2]) + c2;
  o[3] = p[3] * q[3] - ((p[0] * q[0] + p[1] * q[1]) + p[2] * q[2]);
}

__global__ void trajectory_kernel(TrajArgs T) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T.n) return;
  const double t = T.query[i];
  int lo = 0, hi = T.C;
  while (lo < hi) {  // torch.searchsorted (left): first stamp >= t
    const int mid = (lo + hi) >> 1;
    if ((double)T.cam_ts[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  int right = lo;
  int left = (t == (double)T.cam_ts[0]) ? right : right - 1;
  if (left < 0 || right >= T.C || left > T.C - 2) {
    if (T.status) atomicOr(T.status, 1);
    left = left < 0 ? 0 : (left > T.C - 2 ? T.C - 2 : left);
    right = right >= T.C ? T.C - 1 : (right < left ? left : right);
  }
  const double bw = (double)(T.cam_ts[left + 1] - T.cam_ts[left]);
  const float w = (float)((t - (double)T.cam_ts[left]) / bw);
  for (int a = 0; a < 3; ++a) T.pos[i * 3 + a] = lerp_f(T.cam_pos[left * 3 + a], T.cam_pos[right * 3 + a], w);
  float q0[4], q1[4];
  for (int a = 0; a < 4; ++a) {
    q0[a] = T.cam_q[left * 4 + a];
    q1[a] = T.cam_q[right * 4 + a];
  }
  // shortest path: flip q1 when q0 . q1 < 0
  if (((q0[0] * q1[0] + q0[1] * q1[1]) + q0[2] * q1[2]) + q0[3] * q1[3] < 0.0f)
    for (int a = 0; a < 4; ++a) q1[a] = -q1[a];
  const float q0c[4] = {-q0[0], -q0[1], -q0[2], q0[3]};
  float rel[4];
  quat_mul(q0c, q1, rel);
  // unitquat_to_full_rotvec: angle in [0, 2 pi]
  const float vn = sqrtf((rel[0] * rel[0] + rel[1] * rel[1]) + rel[2] * rel[2]);
  const float ang = 2.0f * atan2f(vn, rel[3]);
  float sc;
  if (fabsf(ang) <= 1e-3f) {
    const float a2 = ang * ang;
    sc = (2.0f + a2 / 12.0f) + 7.0f * (a2 * a2) / 2880.0f;
  } else {
    sc = ang / sinf(ang / 2.0f);
  }
  float v[3];
  for (int a = 0; a < 3; ++a) v[a] = w * (sc * rel[a]);
  // rotvec_to_unitquat
  const float n = sqrtf((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
  float s2;
  if (n <= 1e-3f) {
    const float n2 = n * n;
    s2 = (0.5f - n2 / 48.0f) + (n2 * n2) / 3840.0f;
  } else {
    s2 = sinf(n / 2.0f) / n;
  }
  const float r[4] = {s2 * v[0], s2 * v[1], s2 * v[2], cosf(n / 2.0f)};
  float q[4];
  quat_mul(q0, r, q);
  // unitquat_to_rotmat
  const float x = q[0], y = q[1], z = q[2], ww = q[3];
  const float x2 = x * x, y2 = y * y, z2 = z * z, w2 = ww * ww;
  const float xy = x * y, zw = z * ww, xz = x * z, yw = y * ww, yz = y * z, xw = x * ww;
  float* m = T.rot + i * 9;
  m[0] = ((x2 - y2) - z2) + w2;
  m[3] = 2.0f * (xy + zw);
  m[6] = 2.0f * (xz - yw);
  m[1] = 2.0f * (xy - zw);
  m[4] = ((-x2 + y2) - z2) + w2;
  m[7] = 2.0f * (yz + xw);
  m[2] = 2.0f * (xz + yw);
  m[5] = 2.0f * (yz - xw);
  m[8] = ((-x2 - y2) + z2) + w2;
}

// Reverse mode of trajectory_kernel with respect to the query timestamp (the camera samples are
// buffers): w = (t - ts[l]) / bw, so dL/dt = dL/dw / bw with
//   dL/dw = g_pos . (p[r] - p[l])                                  (torch.lerp: d/dweight = end - start)
//         + g_R : dR/dq . (q0 (x) dr/dw)                           (q = q0 (x) r(w), r = rotvec_to_unitquat(w v0))
// r(w) = [sin(w |v0| / 2) v0 / |v0|, cos(w |v0| / 2)] so dr/dw = [cos(h) v0 / 2, -|v0| sin(h) / 2],
// h = w |v0| / 2 (the limit of RoMa's small-angle series as well).  dq/dw is tangent to the unit
// sphere, so any quaternion -> matrix form with the right values on it gives the same dR/dw.
// Out-of-span queries (clamped to the end bins by the forward) get the clamped bin's derivative.
__global__ void trajectory_bwd_kernel(TrajArgs T, const float* g_pos, const float* g_rot, double* d_query) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T.n) return;
  const double t = T.query[i];
  int lo = 0, hi = T.C;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((double)T.cam_ts[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  int right = lo;
  int left = (t == (double)T.cam_ts[0]) ? right : right - 1;
  if (left < 0 || right >= T.C || left > T.C - 2) {
    left = left < 0 ? 0 : (left > T.C - 2 ? T.C - 2 : left);
    right = right >= T.C ? T.C - 1 : (right < left ? left : right);
  }
  const double bw = (double)(T.cam_ts[left + 1] - T.cam_ts[left]);
  const float w = (float)((t - (double)T.cam_ts[left]) / bw);
  float gw = 0.0f;
  if (g_pos)
    for (int a = 0; a < 3; ++a) gw += g_pos[i * 3 + a] * (T.cam_pos[right * 3 + a] - T.cam_pos[left * 3 + a]);
  if (g_rot) {
    float q0[4], q1[4];
    for (int a = 0; a < 4; ++a) {
      q0[a] = T.cam_q[left * 4 + a];
      q1[a] = T.cam_q[right * 4 + a];
    }
    if (((q0[0] * q1[0] + q0[1] * q1[1]) + q0[2] * q1[2]) + q0[3] * q1[3] < 0.0f)
      for (int a = 0; a < 4; ++a) q1[a] = -q1[a];
    const float q0c[4] = {-q0[0], -q0[1], -q0[2], q0[3]};
    float rel[4];
    quat_mul(q0c, q1, rel);
    const float vn = sqrtf((rel[0] * rel[0] + rel[1] * rel[1]) + rel[2] * rel[2]);
    const float ang = 2.0f * atan2f(vn, rel[3]);
    float sc;
    if (fabsf(ang) <= 1e-3f) {
      const float a2 = ang * ang;
      sc = (2.0f + a2 / 12.0f) + 7.0f * (a2 * a2) / 2880.0f;
    } else {
      sc = ang / sinf(ang / 2.0f);
    }
    float v0[3];
    for (int a = 0; a < 3; ++a) v0[a] = sc * rel[a];
    const float th = sqrtf((v0[0] * v0[0] + v0[1] * v0[1]) + v0[2] * v0[2]);
    // the forward rotation r(w) and dr/dw
    const float n = fabsf(w) * th;
    float s2;
    if (n <= 1e-3f) {
      const float n2 = n * n;
      s2 = (0.5f - n2 / 48.0f) + (n2 * n2) / 3840.0f;
    } else {
      s2 = sinf(n / 2.0f) / n;
    }
    const float r[4] = {s2 * w * v0[0], s2 * w * v0[1], s2 * w * v0[2], cosf(n / 2.0f)};
    const float h = 0.5f * w * th;
    const float dr[4] = {0.5f * cosf(h) * v0[0], 0.5f * cosf(h) * v0[1], 0.5f * cosf(h) * v0[2],
                         -0.5f * th * sinf(h)};
    float q[4], dq[4];
    quat_mul(q0, r, q);
    quat_mul(q0, dr, dq);
    const float x = q[0], y = q[1], z = q[2], ww = q[3];
    const float* G = g_rot + i * 9;
    // dR/dq of the forward's matrix (rows of 4: d/dx, d/dy, d/dz, d/dw), contracted with g_R
    const float gq0 = 2.0f * (G[0] * x + G[3] * y + G[6] * z + G[1] * y - G[4] * x + G[7] * ww + G[2] * z -
                              G[5] * ww - G[8] * x);
    const float gq1 = 2.0f * (-G[0] * y + G[3] * x - G[6] * ww + G[1] * x + G[4] * y + G[7] * z + G[2] * ww +
                              G[5] * z - G[8] * y);
    const float gq2 = 2.0f * (-G[0] * z + G[3] * ww + G[6] * x - G[1] * ww - G[4] * z + G[7] * y + G[2] * x +
                              G[5] * y + G[8] * z);
    const float gq3 = 2.0f * (G[0] * ww + G[3] * z - G[6] * y - G[1] * z + G[4] * ww + G[7] * x + G[2] * y -
                              G[5] * x + G[8] * ww);
    gw += ((gq0 * dq[0] + gq1 * dq[1]) + gq2 * dq[2]) + gq3 * dq[3];
  }
  d_query[i] = (double)gw / bw;
}
#pragma clang fp contract(on)

}  // namespace den
