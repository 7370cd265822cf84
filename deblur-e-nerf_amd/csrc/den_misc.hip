// den_misc.hip -- weight packing, Adam, deterministic partial sums, event loss.
#include "den_device.h"

namespace den {

// ------------------------------------------------------------------ weight packing
// One thread per packed element.  Forward chunk (layer l, row tile i):
//   BF16: [kappa][lane][8]   lane -> row 32i+(lane&31), group lane>>5, element j
//   F32 : [kappa/4][lane][4] lane -> row 16i+(lane&15), group lane>>4
// element = W_l[row][chain_feature(kappa, group, j)].
// Backward chunk (transposed layer j, row tile i): rows = chain inputs of
// layer bwd_layer(j), k = its (padded) outputs: element = W_l[out][in].
struct PackArgs {
  int mode, rd;
  const float* params;
  void* w_fwd;
  void* w_bwd;
  float* bias;
};

__device__ __forceinline__ float param_w(const PackArgs& P, int l, int o, int f) {
  int t, r, c;
  if (!ref_coord(l, o, f, P.rd, &t, &r, &c)) return 0.0f;
  const float w = P.params[param_offset(P.rd, 2 * t) + (int64_t)r * ref_in(t) + c];
  return P.mode == 0 ? w : (float)((double)w * col_scale(P.mode, l, f));
}

__device__ __forceinline__ void decode_elem(int mode, int64_t e, int* kappa, int* lane, int* j) {
  if (mode == 1) {
    *kappa = (int)(e / 512);
    *lane = (int)((e / 8) % 64);
    *j = (int)(e % 8);
  } else {
    *kappa = (int)((e / 256) * 4 + (e % 4));
    *lane = (int)((e / 4) % 64);
    *j = 0;
  }
}

__global__ void pack_kernel(PackArgs P) {
  const int mode = P.mode, TM = tm_of(mode), ES = es_of(mode);
  const int64_t nf = fwd_bytes(mode) / ES, nb = bwd_bytes(mode) / ES, nbias = bias_floats(mode);
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nf) {
    int l = 0;
    while (l + 1 < NL && fwd_layer_offset(mode, l + 1) / ES <= e) ++l;
    const int64_t in_layer = e - fwd_layer_offset(mode, l) / ES;
    const int64_t per_chunk = chunk_bytes_K(fwd_K(mode, l)) / ES;
    const int i = (int)(in_layer / per_chunk);
    int kappa, lane, j;
    decode_elem(mode, in_layer % per_chunk, &kappa, &lane, &j);
    const int grp = lane / TM;
    const int o = TM * i + lane % TM;
    const float v = param_w(P, l, o, chain_feature(mode, kappa, grp, j));
    if (mode == 1) ((__bf16*)P.w_fwd)[e] = (__bf16)v;
    else ((float*)P.w_fwd)[e] = v;
    return;
  }
  e -= nf;
  if (e < nb) {
    int jb = 0;
    while (jb + 1 < NBL && bwd_layer_offset(mode, jb + 1) / ES <= e) ++jb;
    const int l = bwd_layer(jb);
    const int64_t in_layer = e - bwd_layer_offset(mode, jb) / ES;
    const int64_t per_chunk = chunk_bytes_K(bwd_K(mode, jb)) / ES;
    const int i = (int)(in_layer / per_chunk);
    int kappa, lane, j;
    decode_elem(mode, in_layer % per_chunk, &kappa, &lane, &j);
    const int grp = lane / TM;
    const int in_f = TM * i + lane % TM;
    const int out_f = chain_feature(mode, kappa, grp, j);
    const float v = param_w(P, l, out_f, in_f);
    if (mode == 1) ((__bf16*)P.w_bwd)[e] = (__bf16)v;
    else ((float*)P.w_bwd)[e] = v;
    return;
  }
  e -= nb;
  if (e < nbias) {
    const int chunk = (int)(e / TM), q = (int)(e % TM);
    int l = 0;
    while (l + 1 < NL && fwd_chunk_index(mode, l + 1) <= chunk) ++l;
    const int i = chunk - fwd_chunk_index(mode, l);
    const int o = TM * i + stored_to_row(mode, q);
    int t, r;
    P.bias[e] = ref_bias_coord(l, o, P.rd, &t, &r)
                    ? (float)((double)P.params[param_offset(P.rd, 2 * t + 1) + r] * bias_scale(mode, l))
                    : 0.0f;
  }
}

// ------------------------------------------------------------------ Adam (torch.optim.Adam, single-tensor path)
//   g += wd * p ; m.lerp_(g, 1-b1) ; v = v*b2 + (1-b2)*g*g
//   p += -(lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
// Scalars are formed in double on the host and rounded to f32 exactly as torch
// rounds its Python-float scalars.
template <typename T>
__global__ void adam_kernel(int64_t n, T* p, const T* g, T* m, T* v, T step_size, T w1, T b2, T w2, T eps, T wd,
                            T bc2_sqrt) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  T gi = g[i];
  const T pi = p[i];
  if (wd != T(0)) gi = gi + wd * pi;
  const T mo = m[i];
  const T mi = w1 < T(0.5) ? mo + w1 * (gi - mo) : gi - (gi - mo) * (T(1) - w1);
  const T vi = v[i] * b2 + w2 * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const T denom = sqrt(vi) / bc2_sqrt + eps;
  p[i] = pi + (-step_size) * (mi / denom);
}

// ------------------------------------------------------------------ partial sums
// out[j] = sum_b part[j * nb + b], one workgroup per j (any blockDim.x <= 1024, a multiple of 64):
// 8 loads in flight per lane, then a fixed-order tree -- deterministic for a given launch shape.
__global__ __launch_bounds__(1024) void sum_partials_kernel(int n, int nb, const float* part, float* out) {
  const int j = blockIdx.x;
  if (j >= n) return;
  const float* p = part + (int64_t)j * nb;
  const int T = blockDim.x;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = threadIdx.x;
  for (; b + 7 * T < nb; b += 8 * T) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += p[b + u * T];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (b + u * T < nb) a[u] += p[b + u * T];
  float s = ((a[0] + a[4]) + (a[1] + a[5])) + ((a[2] + a[6]) + (a[3] + a[7]));
  __shared__ float red[1024];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = T / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = red[0];
}

// ------------------------------------------------------------------ event loss (loss.py:34-96)
// error functions of (input a, target t): 0 l1, 1 mse, 2 huber (delta 1), 3 mape (utils/modules.py:97-122:
// |a - t| / max(|t|, eps), eps = the f64 machine epsilon)
constexpr float MAPE_EPS = 2.220446049250313e-16f;
__device__ __forceinline__ float sgnf(float d) { return d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f); }
__device__ __forceinline__ float err_fn(int fn, float a, float t) {
  const float d = a - t, ad = fabsf(d);
  if (fn == 0) return ad;                                   // l1
  if (fn == 1) return d * d;                                // mse
  if (fn == 3) return ad / fmaxf(fabsf(t), MAPE_EPS);       // mape
  return ad < 1.0f ? 0.5f * d * d : (ad - 0.5f);            // huber, delta = 1
}
// d err / d a
__device__ __forceinline__ float derr_fn(int fn, float a, float t) {
  const float d = a - t;
  if (fn == 0) return sgnf(d);
  if (fn == 1) return 2.0f * d;
  if (fn == 3) return sgnf(d) / fmaxf(fabsf(t), MAPE_EPS);
  return d < -1.0f ? -1.0f : (d > 1.0f ? 1.0f : d);
}
// d err / d t (torch's autograd: abs' gradient sign(x), clamp's passes where |t| >= eps)
__device__ __forceinline__ float derr_dt_fn(int fn, float a, float t) {
  if (fn != 3) return -derr_fn(fn, a, t);
  const float m = fmaxf(fabsf(t), MAPE_EPS);
  const float g = -sgnf(a - t) / m;
  return fabsf(t) >= MAPE_EPS ? g - fabsf(a - t) * sgnf(t) / (m * m) : g;
}

constexpr int LOSS_BLOCK = 256;

// pass 1: per-block (sum err, count)
__global__ void loss_partial_kernel(int N, int fn, const float* x, const float* target, const uint8_t* valid,
                                    const float* c, float* part) {
  __shared__ float se[LOSS_BLOCK], sc[LOSS_BLOCK];
  int i = blockIdx.x * LOSS_BLOCK + threadIdx.x;
  float e = 0.0f, k = 0.0f;
  if (i < N && (!valid || valid[i])) {
    float a = x[i] / c[0];
    float t = target ? target[i] : 0.0f;
    e = err_fn(fn, a, t);
    k = 1.0f;
  }
  se[threadIdx.x] = e;
  sc[threadIdx.x] = k;
  __syncthreads();
  for (int w = LOSS_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      se[threadIdx.x] += se[threadIdx.x + w];
      sc[threadIdx.x] += sc[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x] = se[0];
    part[gridDim.x + blockIdx.x] = sc[0];
  }
}
// pass 2: fixed-order final sum -> loss, count
__global__ void loss_final_kernel(int nb, const float* part, float* loss, float* count) {
  __shared__ float se[LOSS_BLOCK], sc[LOSS_BLOCK];
  float e = 0.0f, k = 0.0f;
  for (int b = threadIdx.x; b < nb; b += LOSS_BLOCK) {
    e += part[b];
    k += part[nb + b];
  }
  se[threadIdx.x] = e;
  sc[threadIdx.x] = k;
  __syncthreads();
  for (int w = LOSS_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      se[threadIdx.x] += se[threadIdx.x + w];
      sc[threadIdx.x] += sc[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = se[0] / sc[0];  // NaN on zero valid events, as torch's empty mean
    count[0] = sc[0];
  }
}
// backward: dL/dx, dL/dtarget per event, per-block partials of dL/dc
__global__ void loss_bwd_kernel(int N, int fn, const float* x, const float* target, const uint8_t* valid,
                                const float* c, const float* gout, const float* count, float* dx, float* dtarget,
                                float* dc_part) {
  __shared__ float sd[LOSS_BLOCK];
  int i = blockIdx.x * LOSS_BLOCK + threadIdx.x;
  float dcv = 0.0f;
  if (i < N) {
    float gx = 0.0f, gt = 0.0f;
    if (!valid || valid[i]) {
      const float cc = c[0];
      float a = x[i] / cc;
      float t = target ? target[i] : 0.0f;
      float gerr = gout[0] / count[0];
      float de = derr_fn(fn, a, t) * gerr;
      gx = de / cc;
      gt = derr_dt_fn(fn, a, t) * gerr;
      dcv = de * (-x[i] / (cc * cc));
    }
    dx[i] = gx;
    if (dtarget) dtarget[i] = gt;
  }
  sd[threadIdx.x] = dcv;
  __syncthreads();
  for (int w = LOSS_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sd[threadIdx.x] += sd[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) dc_part[blockIdx.x] = sd[0];
}

// target (loss.py:74-77): f32( ts_diff * (lid / (end - start)) / c ), f64 arithmetic
__global__ void event_target_kernel(int N, const double* ts_diff, const float* lid, const int64_t* end_ts,
                                    const double* start_ts, const float* c, float* target) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  double grad = (double)lid[i] / ((double)end_ts[i] - start_ts[i]);
  target[i] = (float)(ts_diff[i] * grad / (double)c[0]);
}

}  // namespace den

namespace den {
// ------------------------------------------------------------------ fused event step (pixel bandwidth off)
// The measurement path of DeblurENeRF.training_step (deblur_e_nerf.py:472-549)
// for pixel_bandwidth.enable = false, fused over the 4 render groups
// [diff start, diff end, tv start, tv end] x N events:
//   I = radiance(+bayer channel) + min_int ; y = log I (deblur_e_nerf.py:1153-1157, 1203)
//   L_diff = mean_valid f_d((y1 - y0)/c - t) ; L_tv = mean_valid f_t((y3 - y2)/c)   (loss.py:62-96)
//   valid = is_valid(start) | is_valid(end), is_valid = opacity > 0 unless has_bkgd (1204-1207)
// total = w_d L_diff + w_t L_tv.
struct EventStepArgs {
  int N, rd, fn_d, fn_t, has_bkgd;
  float min_int, w_d, w_t;
  const float* radiance;   // [4][N][rd]
  const float* opacity;    // [4][N]
  const int64_t* channel;  // [N] or null
  const float* target;     // [N] normalised diff target
  const float* c;          // [1]
  float* part;             // [4][nb] partial sums: err_d, cnt_d, err_t, cnt_t
  float* out;              // [4]: L_diff, L_tv, total, (scratch)
  float* d_radiance;       // [4][N][rd]
};

__device__ __forceinline__ float ev_logI(const EventStepArgs& E, int g, int i) {
  const int ch = (E.rd > 1 && E.channel) ? (int)E.channel[i] : 0;
  return logf(E.radiance[((int64_t)g * E.N + i) * E.rd + ch] + E.min_int);
}
__device__ __forceinline__ bool ev_valid(const EventStepArgs& E, int g0, int i) {
  if (E.has_bkgd) return true;
  return E.opacity[(int64_t)g0 * E.N + i] > 0.0f || E.opacity[(int64_t)(g0 + 1) * E.N + i] > 0.0f;
}

__global__ void event_step_partial_kernel(EventStepArgs E) {
  __shared__ float s[4][LOSS_BLOCK];
  const int i = blockIdx.x * LOSS_BLOCK + threadIdx.x;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (i < E.N) {
    const float c = E.c[0];
    if (ev_valid(E, 0, i)) {
      float x = ev_logI(E, 1, i) - ev_logI(E, 0, i);
      v[0] = err_fn(E.fn_d, x / c, E.target[i]);
      v[1] = 1.0f;
    }
    if (ev_valid(E, 2, i)) {
      float x = ev_logI(E, 3, i) - ev_logI(E, 2, i);
      v[2] = err_fn(E.fn_t, x / c, 0.0f);
      v[3] = 1.0f;
    }
  }
  for (int q = 0; q < 4; ++q) s[q][threadIdx.x] = v[q];
  __syncthreads();
  for (int w = LOSS_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int q = 0; q < 4; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int q = 0; q < 4; ++q) E.part[q * gridDim.x + blockIdx.x] = s[q][0];
}

__global__ void event_step_final_kernel(EventStepArgs E, int nb) {
  __shared__ float s[4][LOSS_BLOCK];
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nb; b += LOSS_BLOCK)
    for (int q = 0; q < 4; ++q) v[q] += E.part[q * nb + b];
  for (int q = 0; q < 4; ++q) s[q][threadIdx.x] = v[q];
  __syncthreads();
  for (int w = LOSS_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int q = 0; q < 4; ++q) s[q][threadIdx.x] += s[q][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float Ld = s[0][0] / s[1][0], Lt = s[2][0] / s[3][0];
    E.out[0] = Ld;
    E.out[1] = Lt;
    E.out[2] = E.w_d * Ld + E.w_t * Lt;
    E.out[3] = 0.0f;
    E.part[0] = s[1][0];  // keep the valid counts for the backward
    E.part[1] = s[3][0];
  }
}

// d total / d radiance for the 4 groups (zeros on the channels not selected)
__global__ void event_step_bwd_kernel(EventStepArgs E) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E.N) return;
  const float c = E.c[0];
  const float cnt_d = E.part[0], cnt_t = E.part[1];
  const int ch = (E.rd > 1 && E.channel) ? (int)E.channel[i] : 0;
  float dy[4] = {0.f, 0.f, 0.f, 0.f};
  if (ev_valid(E, 0, i)) {
    float x = ev_logI(E, 1, i) - ev_logI(E, 0, i);
    float g = derr_fn(E.fn_d, x / c, E.target[i]) * (E.w_d / cnt_d) / c;
    dy[1] = g;
    dy[0] = -g;
  }
  if (ev_valid(E, 2, i)) {
    float x = ev_logI(E, 3, i) - ev_logI(E, 2, i);
    float g = derr_fn(E.fn_t, x / c, 0.0f) * (E.w_t / cnt_t) / c;
    dy[3] = g;
    dy[2] = -g;
  }
  for (int g = 0; g < 4; ++g) {
    const int64_t base = ((int64_t)g * E.N + i) * E.rd;
    const float I = E.radiance[base + ch] + E.min_int;
    for (int k = 0; k < E.rd; ++k) E.d_radiance[base + k] = (k == ch) ? dy[g] / I : 0.0f;
  }
}

// ------------------------------------------------------------------ image errors (Metric.compute, metric.py:28-92)
// per image b: sum of squared and of absolute pixel errors (f64 accumulation), one block per
// (image, slice); partials [img][2][slices] reduced in a fixed order by sum_partials_f64_kernel.
constexpr int IMG_BLOCK = 256, IMG_SLICES = 64;
__global__ void image_error_kernel(int64_t pix, const float* pred, const float* target, double* part) {
  const int b = blockIdx.y, sl = blockIdx.x;
  const float* p = pred + (int64_t)b * pix;
  const float* t = target + (int64_t)b * pix;
  double se = 0.0, ae = 0.0;
  for (int64_t k = (int64_t)sl * IMG_BLOCK + threadIdx.x; k < pix; k += (int64_t)IMG_SLICES * IMG_BLOCK) {
    const double d = (double)p[k] - (double)t[k];
    se += d * d;
    ae += fabs(d);
  }
  __shared__ double s0[IMG_BLOCK], s1[IMG_BLOCK];
  s0[threadIdx.x] = se;
  s1[threadIdx.x] = ae;
  __syncthreads();
  for (int w = IMG_BLOCK / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s0[threadIdx.x] += s0[threadIdx.x + w];
      s1[threadIdx.x] += s1[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((int64_t)b * 2 + 0) * IMG_SLICES + sl] = s0[0];
    part[((int64_t)b * 2 + 1) * IMG_SLICES + sl] = s1[0];
  }
}
}  // namespace den
