// den_march.hip -- the packed (variable samples per ray) rendering path of the reference:
// nerfacc 0.3.1 (pinned in the reference's environment.yml:32; not vendored) occupancy-grid ray
// marching, sample visibility (early stop / alpha threshold), packed compositing forward and
// backward, and the occupancy-grid EMA update, restated from nerfacc's published algorithm for the
// reference's call sites:
//   ray_marching                       external/utils.py:106-119
//   render_weight_from_density +
//   accumulate_along_rays + background external/vol_rendering.py:81-126
//   OccupancyGrid.every_n_step         models/nerf.py:98-102, 170-204
// The radiance field at the packed samples is the fused MLP of den_render.hip (points = 2).
//
// Layout: packed samples sorted by ray; `offsets` (n_rays + 1) i64 = exclusive scan of the
// per-ray counts (nerfacc's packed_info as [start, start + count)).  One thread per ray marches;
// one wave per ray scans (64 samples per step, a carry across steps).
#include "den_device.h"

namespace den {

constexpr float MARCH_FAR = 1e10f;  // nerfacc's "no intersection" / unbounded t

// ------------------------------------------------------------------ ray / AABB + near / far + jitter
struct MarchPrepArgs {
  int n_rays;
  const float* rays_o;
  const float* rays_d;
  int has_aabb;
  float aabb[6];
  float near_p, far_p;  // < 0: none
  const float* jitter;  // (R) U[0,1): stratified sampling (training), or null
  float step;
  float* t_min;
  float* t_max;
};

// nerfacc _ray_aabb_intersect: slab test, a miss gives near = far = 1e10
__device__ __forceinline__ void ray_aabb_nerfacc(const float* o, const float* d, const float* aabb, float* tn,
                                                 float* tf) {
#pragma clang fp contract(off)
  float tmin = __fdiv_rn(aabb[0] - o[0], d[0]);
  float tmax = __fdiv_rn(aabb[3] - o[0], d[0]);
  if (tmin > tmax) { float t = tmin; tmin = tmax; tmax = t; }
  float tymin = __fdiv_rn(aabb[1] - o[1], d[1]);
  float tymax = __fdiv_rn(aabb[4] - o[1], d[1]);
  if (tymin > tymax) { float t = tymin; tymin = tymax; tymax = t; }
  if (tmin > tymax || tymin > tmax) { *tn = MARCH_FAR; *tf = MARCH_FAR; return; }
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  float tzmin = __fdiv_rn(aabb[2] - o[2], d[2]);
  float tzmax = __fdiv_rn(aabb[5] - o[2], d[2]);
  if (tzmin > tzmax) { float t = tzmin; tzmin = tzmax; tzmax = t; }
  if (tmin > tzmax || tzmin > tmax) { *tn = MARCH_FAR; *tf = MARCH_FAR; return; }
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  *tn = tmin;
  *tf = tmax;
}

__global__ void march_prep_kernel(MarchPrepArgs P) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n_rays) return;
  float o[3], d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o[a] = P.rays_o[(int64_t)i * 3 + a];
    d[a] = P.rays_d[(int64_t)i * 3 + a];
  }
  float tn = 0.0f, tf = MARCH_FAR;
  if (P.has_aabb) ray_aabb_nerfacc(o, d, P.aabb, &tn, &tf);
  if (P.near_p >= 0.0f) tn = fmaxf(tn, P.near_p);  // torch.clamp(t_min, min=near_plane)
  if (P.far_p >= 0.0f) tf = fminf(tf, P.far_p);
  if (P.jitter) tn = tn + P.jitter[i] * P.step;   // stratified: t_min += rand * render_step_size
  P.t_min[i] = tn;
  P.t_max[i] = tf;
}

// ------------------------------------------------------------------ marching
struct MarchArgs {
  int n_rays;
  const float* rays_o;
  const float* rays_d;
  const float* t_min;
  const float* t_max;
  float roi[6];
  int res[3];
  const uint8_t* grid;      // binary occupancy, res0*res1*res2 (ij order), or null (everything occupied)
  int contraction;          // CONTRACT_* of the grid
  float step, cone;
  int max_iter;             // per-ray loop guard (every wave drains)
  const int64_t* offsets;   // fill pass: (n_rays + 1)
  int* counts;              // count pass: (n_rays)
  int* ray_idx;
  float* t0;
  float* t1;
};

__device__ __forceinline__ float march_dt(float t, float cone, float dt_min) {
  return fminf(fmaxf(t * cone, dt_min), MARCH_FAR);  // calc_dt: clamp(t * cone_angle, dt_min, dt_max)
}

__device__ __forceinline__ void grid_unit(const float* xyz, const float* roi, int type, float* u) {
#pragma clang fp contract(off)
#pragma unroll
  for (int a = 0; a < 3; ++a) u[a] = __fdiv_rn(xyz[a] - roi[a], roi[3 + a] - roi[a]);  // roi_to_unit
  if (type == CONTRACT_SPHERE) {  // unbounded_to_unit_sphere
#pragma unroll
    for (int a = 0; a < 3; ++a) u[a] = u[a] * 2.0f - 1.0f;
    const float nrm = __fsqrt_rn(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    if (nrm > 1.0f) {
      const float s = 2.0f - __fdiv_rn(1.0f, nrm);
#pragma unroll
      for (int a = 0; a < 3; ++a) u[a] = s * __fdiv_rn(u[a], nrm);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) u[a] = u[a] * 0.25f + 0.5f;
  } else if (type == CONTRACT_TANH) {  // unbounded_to_unit_tanh
#pragma unroll
    for (int a = 0; a < 3; ++a) u[a] = tanhf(u[a] - 0.5f) * 0.5f + 0.5f;
  }
}

__device__ __forceinline__ bool grid_occupied(const MarchArgs& P, const float* xyz) {
  if (!P.grid) return true;
  if (P.contraction == CONTRACT_AABB)
    for (int a = 0; a < 3; ++a)
      if (xyz[a] < P.roi[a] || xyz[a] > P.roi[3 + a]) return false;
  float u[3];
  grid_unit(xyz, P.roi, P.contraction, u);
  int ix[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    int v = (int)(u[a] * (float)P.res[a]);  // make_int3: truncation
    ix[a] = v < 0 ? 0 : (v > P.res[a] - 1 ? P.res[a] - 1 : v);
  }
  return P.grid[((int64_t)ix[0] * P.res[1] + ix[1]) * P.res[2] + ix[2]] != 0;
}

// distance_to_next_voxel + advance_to_next_voxel (AABB only: the DDA skip)
__device__ __forceinline__ float advance_to_next_voxel(const MarchArgs& P, float t, float dt_min, const float* xyz,
                                                       const float* dir, const float* inv, float far) {
#pragma clang fp contract(off)
  float tx[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float span = P.roi[3 + a] - P.roi[a];
    const float res = (float)P.res[a];
    const float x = __fdiv_rn(xyz[a] - P.roi[a], span) * res;
    const float sgn = copysignf(1.0f, dir[a]);
    tx[a] = __fdiv_rn((floorf(x + 0.5f + 0.5f * sgn) - x) * inv[a], res) * span;
  }
  const float dist = fmaxf(fminf(fminf(tx[0], tx[1]), tx[2]), 0.0f);
  float target = t + dist;
  // once past `far` the march ends whatever the target: clip it so an axis-parallel ray
  // (inv = inf) cannot spin here
  if (!(target <= far)) target = far + dt_min;
  do {
    t += dt_min;
  } while (t < target);
  return t;
}

template <bool FILL>
__global__ void march_kernel(MarchArgs P) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.n_rays) return;
  float o[3], d[3], inv[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o[a] = P.rays_o[(int64_t)i * 3 + a];
    d[a] = P.rays_d[(int64_t)i * 3 + a];
    inv[a] = __fdiv_rn(1.0f, d[a]);
  }
  const float near = P.t_min[i], far = P.t_max[i];
  const float dt_min = P.step;
  int64_t base = FILL ? P.offsets[i] : 0;
  int j = 0;
  float t0 = near;
  float t1 = t0 + march_dt(t0, P.cone, dt_min);
  float tm = (t0 + t1) * 0.5f;
  for (int it = 0; tm < far && it < P.max_iter; ++it) {
    float xyz[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) xyz[a] = o[a] + tm * d[a];
    if (grid_occupied(P, xyz)) {
      if (FILL) {
        P.t0[base + j] = t0;
        P.t1[base + j] = t1;
        P.ray_idx[base + j] = i;
      }
      ++j;
      t0 = t1;
      t1 = t0 + march_dt(t0, P.cone, dt_min);
      tm = (t0 + t1) * 0.5f;
    } else if (P.contraction == CONTRACT_AABB) {
      tm = advance_to_next_voxel(P, tm, dt_min, xyz, d, inv, far);
      const float dt = march_dt(tm, P.cone, dt_min);
      t0 = tm - dt * 0.5f;
      t1 = tm + dt * 0.5f;
    } else {
      t0 = t1;
      t1 = t0 + march_dt(t0, P.cone, dt_min);
      tm = (t0 + t1) * 0.5f;
    }
  }
  if (!FILL) P.counts[i] = j;
}

// Unbounded contractions (sphere / tanh: configs[3]/[4]) have no DDA skip, so the step sequence
// t_{k+1} = t_k + calc_dt(t_k) does not depend on occupancy and the march is a filter over it.  One
// wave per ray: every lane runs the same f32 chain (identical values, so the samples are bit-equal to
// march_kernel's), lane l keeps step 64 b + l of block b, tests its occupancy, and the wave compacts
// the occupied steps in order with a ballot prefix count.  One dependent occupancy load per 64 steps
// instead of per step, and 64x the threads (march_kernel runs one thread per ray: a 2,040-ray call
// is 32 waves on a 256-CU chip, latency-bound at ~0.6 ms).
template <bool FILL>
__global__ __launch_bounds__(256) void march_wave_kernel(MarchArgs P) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= P.n_rays) return;  // whole waves
  float o[3], d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o[a] = P.rays_o[(int64_t)i * 3 + a];
    d[a] = P.rays_d[(int64_t)i * 3 + a];
  }
  const float far = P.t_max[i];
  const float dt_min = P.step;
  const int64_t base = FILL ? P.offsets[i] : 0;
  int64_t j = 0;
  float t = P.t_min[i];  // t0 of the next block's first step (the same in every lane)
  for (int k0 = 0; k0 < P.max_iter; k0 += 64) {
    float my0 = 0.0f, my1 = 0.0f;
#pragma unroll 8
    for (int u = 0; u < 64; ++u) {
      const float t1 = t + march_dt(t, P.cone, dt_min);
      if (u == lane) {
        my0 = t;
        my1 = t1;
      }
      t = t1;
    }
    const float tm = (my0 + my1) * 0.5f;
    const bool live = tm < far && k0 + lane < P.max_iter;
    bool occ = false;
    if (live) {
      float xyz[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) xyz[a] = o[a] + tm * d[a];
      occ = grid_occupied(P, xyz);
    }
    const uint64_t m = __ballot(occ);
    if (FILL && occ) {
      const int64_t at = base + j + __popcll(m & ((1ull << lane) - 1));
      P.t0[at] = my0;
      P.t1[at] = my1;
      P.ray_idx[at] = i;
    }
    j += __popcll(m);
    if (__ballot(live) != ~0ull) break;  // tm grows with k: the first dead step ends the ray
  }
  if (!FILL && lane == 0) P.counts[i] = (int)j;
}

// ------------------------------------------------------------------ exclusive scan (i32 counts -> i64 offsets)
constexpr int SCAN_BLOCK = 256, SCAN_PER = 8, SCAN_TILE = SCAN_BLOCK * SCAN_PER;

__device__ __forceinline__ int64_t block_excl_scan_i64(int64_t v, int64_t* total) {
  __shared__ int64_t s[SCAN_BLOCK];
  const int t = threadIdx.x;
  s[t] = v;
  __syncthreads();
  for (int off = 1; off < SCAN_BLOCK; off <<= 1) {
    int64_t add = t >= off ? s[t - off] : 0;
    __syncthreads();
    s[t] += add;
    __syncthreads();
  }
  const int64_t incl = s[t];
  *total = s[SCAN_BLOCK - 1];
  __syncthreads();
  return incl - v;
}

// per tile: local exclusive scan into out, tile total into sums[tile]
__global__ void scan_tile_kernel(int64_t n, const int* in, int64_t* out, int64_t* sums) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER;
  int64_t v[SCAN_PER], run = 0;
#pragma unroll
  for (int q = 0; q < SCAN_PER; ++q) {
    v[q] = base + q < n ? in[base + q] : 0;
    run += v[q];
  }
  int64_t total;
  int64_t ex = block_excl_scan_i64(run, &total);
#pragma unroll
  for (int q = 0; q < SCAN_PER; ++q) {
    if (base + q < n) out[base + q] = ex;
    ex += v[q];
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}
// one block: exclusive scan of the tile sums in place (sequential over chunks of SCAN_BLOCK);
// out[n] = grand total
__global__ void scan_sums_kernel(int64_t ntiles, int64_t* sums, int64_t* out, int64_t n) {
  int64_t carry = 0;
  for (int64_t b = 0; b < ntiles; b += SCAN_BLOCK) {
    const int64_t k = b + threadIdx.x;
    const int64_t v = k < ntiles ? sums[k] : 0;
    int64_t total;
    const int64_t ex = block_excl_scan_i64(v, &total);
    if (k < ntiles) sums[k] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) out[n] = carry;
}
__global__ void scan_add_kernel(int64_t n, const int64_t* sums, int64_t* out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] += sums[k / SCAN_TILE];
}

// offsets of sorted ray indices: offsets[r] = lower_bound(ray_idx, r), offsets[R] = n
__global__ void pack_info_kernel(int n_rays, int64_t n, const int* ray_idx, int64_t* offsets) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n_rays) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ray_idx[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  offsets[r] = r == n_rays ? n : lo;
}

// ------------------------------------------------------------------ wave-level scans of one ray
__device__ __forceinline__ float wave_incl_prod(float v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    float o = __shfl_up(v, off, 64);
    if (lane >= off) v *= o;
  }
  return v;
}

// ------------------------------------------------------------------ visibility + compaction
struct VisArgs {
  int n_rays;
  const int64_t* offsets;
  const float* t0;
  const float* t1;
  const float* sigma;     // sigma_fn output (n), or null when alpha is given
  const float* alpha;     // alpha_fn output (n)
  float early_stop_eps, alpha_thre;
  uint8_t* keep;          // (n)
  int* counts;            // (n_rays) kept per ray
  // compaction
  const int64_t* out_offsets;
  const int* in_ray;
  int* out_ray;
  float* out_t0;
  float* out_t1;
};

// render_visibility: T_i = prod_{j<i} (1 - alpha_j) >= early_stop_eps [and alpha_i >= alpha_thre]
__global__ void visibility_kernel(VisArgs V) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= V.n_rays) return;
  const int64_t s0 = V.offsets[r], s1 = V.offsets[r + 1];
  float carry = 1.0f;
  int kept = 0;
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t s = b + lane;
    const bool in = s < s1;
    float a = 0.0f;
    if (in) a = V.sigma ? 1.0f - expf(-(V.sigma[s] * (V.t1[s] - V.t0[s]))) : V.alpha[s];
    const float incl = wave_incl_prod(in ? 1.0f - a : 1.0f);
    const float up = __shfl_up(incl, 1, 64);
    const float T = carry * (lane == 0 ? 1.0f : up);
    bool k = in && (T >= V.early_stop_eps);
    if (V.alpha_thre > 0.0f) k = k && (a >= V.alpha_thre);
    if (in) V.keep[s] = k ? 1 : 0;
    kept += __popcll(__ballot(k));
    carry *= __shfl(incl, 63, 64);
  }
  if (lane == 0) V.counts[r] = kept;
}

__global__ void compact_kernel(VisArgs V) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= V.n_rays) return;
  const int64_t s0 = V.offsets[r], s1 = V.offsets[r + 1];
  int64_t o = V.out_offsets[r];
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t s = b + lane;
    const bool k = s < s1 && V.keep[s];
    const uint64_t m = __ballot(k);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (k) {
      V.out_ray[o + before] = V.in_ray[s];
      V.out_t0[o + before] = V.t0[s];
      V.out_t1[o + before] = V.t1[s];
    }
    o += __popcll(m);
  }
}

// ------------------------------------------------------------------ packed compositing
struct CompArgs {
  int n_rays, rd;
  const int64_t* offsets;
  const float* t0;
  const float* t1;
  const float* sigma;     // (n)
  const float* rgb;       // (n, rd)
  const float* bkgd;      // (rd) or null
  float* color;           // (R, rd)
  float* opacity;         // (R)
  float* depth;           // (R) sum w t_mid
  // backward
  const float* d_color;
  const float* d_opacity;
  const float* d_depth;
  float* d_sigma;         // (n)
  float* d_rgb;           // (n, rd)
  float* bkgd_partial;    // (rd, R)
  int alpha;              // 1: `sigma` holds alphas (render_weight_from_alpha)
};

// per sample: tau (0 for zero-length samples), t_mid.  Alpha mode (render_weight_from_alpha,
// vol_rendering.py:96-106's rgb_alpha_fn branch): the input is alpha, tau = -log(1 - alpha), and dlt
// = 1 so that d/d(input) below is d/dtau * dtau/dalpha with the 1 / (1 - alpha) applied separately.
__device__ __forceinline__ void comp_sample(const CompArgs& C, int64_t s, bool in, float* tau, float* dlt,
                                            float* tmid) {
#pragma clang fp contract(off)
  if (!in) { *tau = 0.0f; *dlt = 0.0f; *tmid = 0.0f; return; }
  const float a0 = C.t0[s], a1 = C.t1[s];
  *tmid = (a0 + a1) / 2.0f;
  if (C.alpha) {
    *dlt = 1.0f;
    *tau = -log1pf(-fminf(C.sigma[s], 1.0f));
    return;
  }
  *dlt = a1 - a0;
  *tau = (a1 > a0) ? C.sigma[s] * *dlt : 0.0f;
}
// 1 - exp(-tau): alpha itself in alpha mode (exact, also at alpha = 1)
__device__ __forceinline__ float comp_alpha(const CompArgs& C, int64_t s, float tau) {
  return C.alpha ? fminf(C.sigma[s], 1.0f) : 1.0f - expf(-tau);
}

// nerfacc render_weight_from_density (w_i = exp(-sum_{j<i} tau_j)(1 - exp(-tau_i))) +
// accumulate_along_rays x3 + background (vol_rendering.py:89-126); one wave per ray
__global__ void composite_fwd_kernel(CompArgs C) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= C.n_rays) return;
  const int64_t s0 = C.offsets[r], s1 = C.offsets[r + 1];
  float carry = 0.0f, cs[3] = {0.f, 0.f, 0.f}, op = 0.f, dp = 0.f;
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t s = b + lane;
    const bool in = s < s1;
    float tau, dlt, tmid;
    comp_sample(C, s, in, &tau, &dlt, &tmid);
    const float excl = carry + wave_excl_scan(tau);
    const float w = in ? expf(-excl) * comp_alpha(C, s, tau) : 0.0f;
    if (in)
      for (int ch = 0; ch < C.rd; ++ch) cs[ch] += w * C.rgb[s * C.rd + ch];
    op += w;
    dp += w * tmid;
    carry += wave_sum(tau);
  }
  op = wave_sum(op);
  dp = wave_sum(dp);
  for (int ch = 0; ch < 3; ++ch) cs[ch] = wave_sum(cs[ch]);
  if (lane == 0) {
    for (int ch = 0; ch < C.rd; ++ch) {
      float v = cs[ch];
      if (C.bkgd) v = v + C.bkgd[ch] * (1.0f - op);
      C.color[(int64_t)r * C.rd + ch] = v;
    }
    C.opacity[r] = op;
    C.depth[r] = dp;
  }
}

// adjoint: with g_i = dC.rgb_i + (dO - dC.bkgd) + dD t_mid_i,
//   dL/dsigma_i = delta_i (T_{i+1} g_i - sum_{k>i} w_k g_k),  dL/drgb_i = w_i dC,  dL/dbkgd = dC (1 - O)
// The suffix sums run back to front (the reverse cumulative sum torch's autograd of the reference's
// cumsum takes): total - prefix cancels to eps * total for the late samples of a saturated ray, whose
// dL/dsigma then carries that error times their large delta sigma into the density gradients.
// Pass 1 (front to back) keeps each sample's exclusive optical depth in d_sigma and w_i g_i in
// d_rgb[.][0] (scratch); pass 2 (back to front) reads them and overwrites both with the gradients.

__global__ void composite_bwd_kernel(CompArgs C) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= C.n_rays) return;
  const int64_t s0 = C.offsets[r], s1 = C.offsets[r + 1];
  float dC[3] = {0.f, 0.f, 0.f};
  for (int ch = 0; ch < C.rd; ++ch) dC[ch] = C.d_color[(int64_t)r * C.rd + ch];
  const float dO = C.d_opacity ? C.d_opacity[r] : 0.0f;
  const float dD = C.d_depth ? C.d_depth[r] : 0.0f;
  float bk_dot = 0.0f;
  if (C.bkgd)
    for (int ch = 0; ch < C.rd; ++ch) bk_dot += dC[ch] * C.bkgd[ch];
  const float dO_eff = dO - bk_dot;
  auto g_of = [&](int64_t s, float tmid) {
    float g = dO_eff + dD * tmid;
    for (int ch = 0; ch < C.rd; ++ch) g += dC[ch] * C.rgb[s * C.rd + ch];
    return g;
  };
  // pass 1: exclusive optical depth and w g per sample, the opacity
  float carry = 0.0f, op = 0.0f;
  for (int64_t b = s0; b < s1; b += 64) {
    const int64_t s = b + lane;
    const bool in = s < s1;
    float tau, dlt, tmid;
    comp_sample(C, s, in, &tau, &dlt, &tmid);
    const float excl = carry + wave_excl_scan(tau);
    if (in) {
      const float w = expf(-excl) * comp_alpha(C, s, tau);
      op += w;
      C.d_sigma[s] = excl;
      C.d_rgb[s * C.rd] = w * g_of(s, tmid);
    }
    carry += wave_sum(tau);
  }
  const float opacity = wave_sum(op);
  // pass 2: back to front, suffix_i = sum_{k > i} w_k g_k accumulated directly.  Alpha mode
  // instead needs S_i = sum_{k > i} alpha_k g_k prod_{i<j<k} (1 - alpha_j) (dL/dalpha_i =
  // T_i (g_i - S_i), exact also at alpha_i = 1 where the later weights vanish but their
  // derivatives do not): the back-to-front affine recurrence U_i = alpha_i g_i + (1 - alpha_i)
  // U_{i+1}, S_i = U_{i+1}, as a wave suffix scan of the maps u -> b + c u.
  float later = 0.0f;  // sum of w g over the blocks after this one
  float u_carry = 0.0f;  // alpha mode: U at the first sample of the blocks after this one
  const int64_t nb = (s1 - s0 + 63) / 64;
  for (int64_t q = nb - 1; q >= 0; --q) {
    const int64_t s = s0 + q * 64 + lane;
    const bool in = s < s1;
    float tau, dlt, tmid;
    comp_sample(C, s, in, &tau, &dlt, &tmid);
    const float excl = in ? C.d_sigma[s] : 0.0f;
    const float wg = in ? C.d_rgb[s * C.rd] : 0.0f;
    const float incl = wave_incl_suffix(wg);     // sum over lanes >= this one
    const float nxt = __shfl_down(incl, 1, 64);  // sum over lanes > this one (adds only)
    const float suffix = later + (lane < 63 ? nxt : 0.0f);
    const float g = in ? g_of(s, tmid) : 0.0f;
    float s_alpha = 0.0f;
    if (C.alpha) {  // wave-uniform branch
      const float a = in ? fminf(C.sigma[s], 1.0f) : 0.0f;
      float b = a * g, c = 1.0f - a;  // identity map on lanes past the ray
      for (int d = 1; d < 64; d <<= 1) {
        const float bd = __shfl_down(b, d, 64), cd = __shfl_down(c, d, 64);
        if (lane + d < 64) {
          b = b + c * bd;
          c = c * cd;
        }
      }
      const float u = b + c * u_carry;
      const float u_next = __shfl_down(u, 1, 64);
      s_alpha = lane < 63 ? u_next : u_carry;
      u_carry = __shfl(u, 0, 64);
    }
    if (in) {
      const float w = expf(-excl) * comp_alpha(C, s, tau);
      if (C.alpha) {
        // the clamp min(alpha, 1) passes the gradient up to alpha = 1 inclusive (torch.clamp)
        C.d_sigma[s] = C.sigma[s] > 1.0f ? 0.0f : expf(-excl) * (g - s_alpha);
      } else {
        const float Tnext = expf(-(excl + tau));
        const float dtau = Tnext * g - suffix;
        C.d_sigma[s] = (dlt > 0.0f) ? dtau * dlt : 0.0f;
      }
      for (int ch = 0; ch < C.rd; ++ch) C.d_rgb[s * C.rd + ch] = w * dC[ch];
    }
    later += __shfl(incl, 0, 64);
  }
  if (lane == 0 && C.bkgd_partial)
    for (int ch = 0; ch < C.rd; ++ch)
      C.bkgd_partial[(int64_t)ch * C.n_rays + r] = C.bkgd ? dC[ch] * (1.0f - opacity) : 0.0f;
}

// ------------------------------------------------------------------ occupancy grid
struct OccArgs {
  int64_t m;               // sampled cells
  const int64_t* idx;      // (m) cell indices (ij order)
  const float* u;          // (m, 3) U[0,1) jitter inside the cell
  int res[3];
  float roi[6];
  int contraction;
  float* pts;              // (m, 3) world positions
  uint8_t* mask;           // (m) 0: outside the unit sphere (sphere contraction), skipped
  const float* sigma;      // (m) density at pts
  const float* step;       // (m) step size per point, or null (use step_c)
  float step_c, decay;
  float* occs;             // (cells)
  uint8_t* sampled;        // (cells) scratch flags
  int64_t cells;
  float occ_thre;
  float* part;             // reduction partials
  uint8_t* binary;         // (cells)
};

// x = (grid_coords + u) / res in [0,1]^3 -> contract_inv -> world (nerfacc OccupancyGrid._update)
__global__ void occ_points_kernel(OccArgs A) {
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.m) return;
  const int64_t c = A.idx[j];
  const int64_t cz = c % A.res[2], cy = (c / A.res[2]) % A.res[1], cx = c / ((int64_t)A.res[1] * A.res[2]);
  const int64_t cc[3] = {cx, cy, cz};
  float x[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) x[a] = __fdiv_rn((float)cc[a] + A.u[j * 3 + a], (float)A.res[a]);
  uint8_t ok = 1;
  if (A.contraction == CONTRACT_SPHERE) {
    float y[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) y[a] = x[a] - 0.5f;
    ok = __fsqrt_rn(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]) < 0.5f;
    // unit_sphere_to_unbounded: f = (x - 0.5) * 4, |f| > 1 -> f / (|f| (2 - |f|)), then [-1,1] -> [0,1]
    float f[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) f[a] = y[a] * 4.0f;
    const float n = __fsqrt_rn(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    if (n > 1.0f)
#pragma unroll
      for (int a = 0; a < 3; ++a) f[a] = __fdiv_rn(f[a], n * (2.0f - n));
#pragma unroll
    for (int a = 0; a < 3; ++a) x[a] = f[a] * 0.5f + 0.5f;
  } else if (A.contraction == CONTRACT_TANH) {
#pragma unroll
    for (int a = 0; a < 3; ++a) x[a] = atanhf(x[a] * 2.0f - 1.0f) + 0.5f;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) A.pts[j * 3 + a] = x[a] * (A.roi[3 + a] - A.roi[a]) + A.roi[a];
  A.mask[j] = ok;
  if (ok) A.sampled[c] = 1;
}

// the sampled cells decay once: occs *= ema_decay
__global__ void occ_decay_kernel(OccArgs A) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= A.cells) return;
  if (A.sampled[c]) {
    A.occs[c] = A.occs[c] * A.decay;
    A.sampled[c] = 0;
  }
}

// occs[idx] = max(occs[idx], sigma * step): scatter-max (nerfacc's comment: "suppose to use
// scatter max"); occupancies are >= 0, so their bit patterns order as integers
__global__ void occ_max_kernel(OccArgs A) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.m || !A.mask[j]) return;
  const float occ = A.sigma[j] * (A.step ? A.step[j] : A.step_c);
  if (!(occ >= 0.0f)) return;  // NaN (inf * 0) leaves the cell as it is
  atomicMax((int*)(A.occs + A.idx[j]), __float_as_int(occ));
}

constexpr int OCC_BLOCK = 256;
__global__ void occ_mean_partial_kernel(OccArgs A) {
  __shared__ float s[OCC_BLOCK];
  float v = 0.0f;
  for (int64_t c = (int64_t)blockIdx.x * OCC_BLOCK + threadIdx.x; c < A.cells; c += (int64_t)gridDim.x * OCC_BLOCK)
    v += A.occs[c];
  s[threadIdx.x] = v;
  __syncthreads();
  for (int w = OCC_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) A.part[blockIdx.x] = s[0];
}
// binary = occs > min(mean(occs), occ_thre); part[0..nb) -> the mean in part[nb]
__global__ void occ_binary_kernel(OccArgs A, int nb) {
  __shared__ float thr;
  if (threadIdx.x == 0) {
    float t = 0.0f;
    for (int b = 0; b < nb; ++b) t += A.part[b];
    const float mean = (float)((double)t / (double)A.cells);
    thr = fminf(mean, A.occ_thre);
  }
  __syncthreads();
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < A.cells; c += (int64_t)gridDim.x * blockDim.x)
    A.binary[c] = A.occs[c] > thr ? 1 : 0;
}

}  // namespace den
