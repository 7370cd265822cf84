// den_ngp_mfma.hip -- the `ngp` field's MLPs on the matrix cores: v_mfma_f32_32x32x2_f32 (f32
// operands, f32 accumulation, exact f32 products), forward and backward.
//
// Why: a per-lane formulation (measured in r02 and removed: 13.1 vs 3.5 ms fwd + bwd per 2^19
// samples) runs the 9.3 K MACs per sample as v_fmac_f32 with scalar weight
// operands -- one FMA per lane per instruction behind a stream of scalar loads -- and measured
// ~4 TF/s on the head MLP.  Here a wave owns 32 samples; features are the M (row) dimension, the 32
// samples the N (column) dimension, and the weights the A operand:
//   * lane (h = lane >> 5, j = lane & 31) supplies B[k = h][n = j]: for step s the activation of
//     input feature col(s, h) of sample j, and A[m = j][k = h] = W[row m][col(s, h)];
//   * accumulator register r of a 32-row tile t holds row 32 t + ngp_row(r, h) of sample j, so a
//     layer's output registers ARE the next layer's B operands (step 16 t + r <-> feature
//     32 t + ngp_row(r, h)): no cross-lane traffic between layers, only a permutation of W's columns;
//   * the permuted weights ("images", ~50 KB forward / ~39 KB backward) are built once per
//     workgroup in LDS from the flat parameters and read as one ds_read_b128 per 4 MFMAs;
//   * each half of the wave runs the grid encoding of half of the levels of its 32 samples (the
//     layer-0 B operand), and in the backward scatters the table gradient of the levels whose
//     feature rows its accumulators hold.
// Per 32 samples: 192 MFMAs forward (layers 64xE, 16x64, 64x31, 64x64, rdx64), 148 backward
// (W^T products down to the encoding gradient).
#include "den_device.h"

namespace den {

// Measured (r02): 8-wave workgroups (32-sample tiles in flight), compiled for 4 waves per
// SIMD (128 VGPRs; 2 / 3 were slower), at most 512 workgroups looping over tiles (2 resident per CU;
// 1024 / 2048 / 4096 were slower); the table gradient aggregated by ngp_scatter_kernel.
constexpr int NM_WAVES = 8, NM_THREADS = 64 * NM_WAVES;
constexpr int NM_OCC = 4;      // waves per SIMD the field kernels are compiled for
constexpr int NM_GRID = 512;   // workgroups at most

// Activations of the MFMA kernels: softplus(beta = 100) with torch's threshold as
// max(bx, 0) + log1p(exp(-|bx|)) from the hardware exp2 / log2 with log1p(t) = log(1 + t) t / ((1 + t) - 1)
// (Goldberg) and a multiply by 0.01; its derivative from the output y as -expm1(-100 y) with
// expm1(z) = (e^z - 1) z / log(e^z) (Kahan).  A few ulps from the libm forms (which cost ~50 VALU
// instructions per element with the IEEE division).
__device__ __forceinline__ float ngp_sp100_fast(float x) {
  const float bx = x * 100.0f;
  const float t = __expf(-fabsf(bx));
  const float u = 1.0f + t;
  const float l1p = u == 1.0f ? t : __logf(u) * (t * __builtin_amdgcn_rcpf(u - 1.0f));
  const float v = (fmaxf(bx, 0.0f) + l1p) * 0.01f;
  return bx > 20.0f ? x : v;
}
__device__ __forceinline__ float ngp_dsp100_out_fast(float y) {
  const float by = y * 100.0f;
  const float z = -by, u = __expf(z);
  const float em1 = u == 1.0f ? z : (u - 1.0f) * (z * __builtin_amdgcn_rcpf(__logf(u)));
  return by > 20.0f ? 1.0f : -em1;
}
template <bool RELU>
__device__ __forceinline__ float ngp_act_t(float x) {
  if constexpr (RELU) return fmaxf(x, 0.0f);
  else return ngp_sp100_fast(x);
}

// accumulator register r of half h holds row ngp_row(r, h) of its 32-row tile
__device__ __forceinline__ int ngp_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
// input feature of step s, half h, when the input is a 64-wide layer output (two tiles)
__device__ __forceinline__ int ngp_col64(int s, int h) { return 32 * (s >> 4) + ngp_row(s & 15, h); }

// Image sections: A operands [tile][step / 4][lane][4] (a lane's 4 consecutive steps are one b128),
// then (forward) the biases in accumulator order [slot][half][16].
constexpr int FI_A0 = 0, FI_A1 = FI_A0 + 2 * 16 * 64, FI_A2 = FI_A1 + 32 * 64, FI_A3 = FI_A2 + 2 * 16 * 64,
              FI_A4 = FI_A3 + 2 * 32 * 64, FI_B = FI_A4 + 32 * 64, FI_FLOATS = FI_B + 8 * 32;
constexpr int BI_A4 = 0, BI_A3 = BI_A4 + 2 * 4 * 64, BI_A2 = BI_A3 + 2 * 32 * 64, BI_A1 = BI_A2 + 32 * 64,
              BI_A0 = BI_A1 + 2 * 8 * 64, BI_FLOATS = BI_A0 + 32 * 64;

struct NgpSlot {
  int t, s, j, h;
};
// q-th float of a section of S steps per tile
__device__ __forceinline__ NgpSlot ngp_slot(int q, int S) {
  const int t = q / (S * 64), rem = q - t * S * 64, w = rem & 255, lane = w >> 2;
  return NgpSlot{t, (rem >> 8) * 4 + (w & 3), lane & 31, lane >> 5};
}

// Forward image.  Layer 0 (64 x E): half h holds the encoding of levels [h L0, ..); layer 1 (16 x 64):
// one tile, rows >= 16 zero; layer 2 (64 x 31): steps 0..7 the SH values 8 h + s, steps 8..15 the base
// output registers 0..7 (row ngp_row(s - 8, h); row 0, the density, has zero weight, geo row g is
// head input 15 + g); layer 3 (64 x 64); layer 4 (rd x 64): rows >= rd zero.
__device__ float ngp_fi(const float* __restrict__ mlp, const NgpOff& o, int E, int L0, int rd, int q) {
  if (q < FI_A1) {
    const NgpSlot z = ngp_slot(q - FI_A0, 16);
    const int c = z.h ? 2 * L0 + z.s : z.s;
    const bool v = z.h ? c < E : z.s < 2 * L0;
    return v ? mlp[o.w[0] + (32 * z.t + z.j) * E + c] : 0.0f;
  }
  if (q < FI_A2) {
    const NgpSlot z = ngp_slot(q - FI_A1, 32);
    return z.j < 1 + NGP_GEO ? mlp[o.w[1] + z.j * NGP_W + ngp_col64(z.s, z.h)] : 0.0f;
  }
  if (q < FI_A3) {
    const NgpSlot z = ngp_slot(q - FI_A2, 16);
    int c;
    if (z.s < 8) {
      c = 8 * z.h + z.s;
    } else {
      const int g = ngp_row(z.s - 8, z.h);
      c = g >= 1 ? NGP_SH - 1 + g : -1;
    }
    return c >= 0 ? mlp[o.w[2] + (32 * z.t + z.j) * NGP_HIN + c] : 0.0f;
  }
  if (q < FI_A4) {
    const NgpSlot z = ngp_slot(q - FI_A3, 32);
    return mlp[o.w[3] + (32 * z.t + z.j) * NGP_W + ngp_col64(z.s, z.h)];
  }
  if (q < FI_B) {
    const NgpSlot z = ngp_slot(q - FI_A4, 32);
    return z.j < rd ? mlp[o.w[4] + z.j * NGP_W + ngp_col64(z.s, z.h)] : 0.0f;
  }
  // bias slots: layer 0 tiles 0, 1 | layer 1 | layer 2 tiles 0, 1 | layer 3 tiles 0, 1 | layer 4
  const int b = q - FI_B, k = b >> 5, h = (b >> 4) & 1, r = b & 15;
  const int layer = k == 0 || k == 1 ? 0 : k == 2 ? 1 : k <= 4 ? 2 : k <= 6 ? 3 : 4;
  const int t = k == 1 || k == 4 || k == 6 ? 1 : 0;
  const int out = layer == 1 ? 1 + NGP_GEO : layer == 4 ? rd : NGP_W;
  const int boff = layer == 0 ? o.b[0] : layer == 1 ? o.b[1] : layer == 2 ? o.b[2] : layer == 3 ? o.b[3] : o.b[4];
  const int row = 32 * t + ngp_row(r, h);
  return row < out ? mlp[boff + row] : 0.0f;
}

// Backward image: A[m][k] = W[k][m] (W^T).  W4^T: 2 tiles, steps s < 2 carry output 2 s + h (< rd);
// W3^T: 2 tiles x 32 steps; W2^T: one tile whose row m in 1..15 is head input 15 + m (the geo
// gradient lands on base-output row m; row 0 is the density's); W1^T: 2 tiles x 8 steps (the 16
// base-output rows); W0^T: one tile of E rows.
__device__ float ngp_bi(const float* __restrict__ mlp, const NgpOff& o, int E, int rd, int q) {
  if (q < BI_A3) {
    const NgpSlot z = ngp_slot(q - BI_A4, 4);
    const int c = 2 * z.s + z.h;
    return z.s < 2 && c < rd ? mlp[o.w[4] + c * NGP_W + 32 * z.t + z.j] : 0.0f;
  }
  if (q < BI_A2) {
    const NgpSlot z = ngp_slot(q - BI_A3, 32);
    return mlp[o.w[3] + ngp_col64(z.s, z.h) * NGP_W + 32 * z.t + z.j];
  }
  if (q < BI_A1) {
    const NgpSlot z = ngp_slot(q - BI_A2, 32);
    return z.j >= 1 && z.j <= NGP_GEO ? mlp[o.w[2] + ngp_col64(z.s, z.h) * NGP_HIN + NGP_SH - 1 + z.j] : 0.0f;
  }
  if (q < BI_A0) {
    const NgpSlot z = ngp_slot(q - BI_A1, 8);
    return mlp[o.w[1] + ngp_row(z.s, z.h) * NGP_W + 32 * z.t + z.j];
  }
  const NgpSlot z = ngp_slot(q - BI_A0, 32);
  return z.j < E ? mlp[o.w[0] + ngp_col64(z.s, z.h) * E + z.j] : 0.0f;
}

__device__ __forceinline__ f32x16 ngp_mfma(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// acc[t] += A(section, tile t) B over the first `steps` steps (rounded up to 4; the weights of the
// padding steps are zero), b[s] = this lane's B operand of step s
template <int T, int S>
__device__ __forceinline__ void ngp_mm(const float* sec, const float* b, f32x16* acc, int lane, int steps = S) {
#pragma unroll
  for (int g = 0; g < S / 4; ++g) {
    if (4 * g >= steps) break;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const f32x4 a = *(const f32x4*)(sec + (t * S + 4 * g) * 64 + lane * 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[t] = ngp_mfma(a[u], b[4 * g + u], acc[t]);
    }
  }
}
__device__ __forceinline__ f32x16 ngp_bias(const float* img, int slot, int h) {
  const float* p = img + FI_B + slot * 32 + h * 16;
  f32x16 v;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 q = *(const f32x4*)(p + 4 * u);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * u + e] = q[e];
  }
  return v;
}
__device__ __forceinline__ f32x16 ngp_zero16() {
  f32x16 v;
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = 0.0f;
  return v;
}
// level l0 + q of half 1, q of half 0 (both indices wave-uniform: scalar loads, then a select)
__device__ __forceinline__ NgpLevel ngp_level_h(const NgpGrid& G, int q, int l1, int h) {
  const NgpLevel a = ngp_level(G, q);
  const NgpLevel b = ngp_level(G, l1 < NGP_MAX_LEVELS ? l1 : 0);
  return h ? b : a;
}

// ------------------------------------------------------------------ forward
template <bool RELU>
__global__ __launch_bounds__(NM_THREADS, NM_OCC) void ngp_fwd_mfma_kernel(NgpArgs A) {
  __shared__ __attribute__((aligned(16))) float img[FI_FLOATS];
  const int E = A.enc, L = A.grid.n_levels, L0 = (L + 1) / 2;
  for (int q = threadIdx.x; q < FI_FLOATS; q += NM_THREADS) img[q] = ngp_fi(A.mlp, A.off, E, L0, A.rd, q);
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int64_t n = A.n;
  float* S = A.save;
  const int64_t ntiles = (n + 31) / 32;
  const int nl = h ? L - L0 : L0;         // levels encoded by this half
  const int fbase = h ? 2 * L0 : 0;       // their first feature
  for (int64_t tile = (int64_t)blockIdx.x * NM_WAVES + (threadIdx.x >> 6); tile < ntiles;
       tile += (int64_t)gridDim.x * NM_WAVES) {
    const int64_t i = tile * 32 + j;
    const bool ok = i < n;
    const int64_t ic = ok ? i : n - 1;
    // save rows: uniform row offsets (row * nn; nn is opaque per tile so they are not hoisted out of
    // the loop as per-row registers) from a per-lane base; Sh adds this half's 4-row shift
    int64_t nn = A.ld;
    asm volatile("" : "+s"(nn));
    float* S0 = S ? S + i : nullptr;
    float* Sh = S ? S + i + 4 * h * nn : nullptr;
    float xn[3], sel, dir[3];
    ngp_point(A, ic, xn, &sel, dir);
    float feat[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float f0 = 0.0f, f1 = 0.0f;
      if (q < nl) {
        NgpCorner C;
        ngp_corners(ngp_level_h(A.grid, q, L0 + q, h), A.grid.hashed, xn, C);
        float2 v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
          v[c] = *(const float2*)(A.table + 2 * (int64_t)C.idx[c]);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          f0 = fmaf(C.w[c], v[c].x, f0);
          f1 = fmaf(C.w[c], v[c].y, f1);
        }
      }
      feat[2 * q] = f0;
      feat[2 * q + 1] = f1;
    }
    if (S && ok) {
#pragma unroll
      for (int s = 0; s < 16; ++s)
        if (s < 2 * nl) S0[(NS_FEAT + fbase + s) * nn] = feat[s];
    }
    // layer 0 (64 x E) + activation
    float hb[32];
    {
      f32x16 acc[2] = {ngp_bias(img, 0, h), ngp_bias(img, 1, h)};
      ngp_mm<2, 16>(img + FI_A0, feat, acc, lane, 2 * L0);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pre = acc[t][r], a = ngp_act_t<RELU>(pre);
          hb[16 * t + r] = a;
          if (S && ok) {
            const int row = 32 * t + ngp_row(r, 0);
            Sh[(NS_H0 + row) * nn] = a;
          }
        }
    }
    // layer 1 (16 x 64): density (row 0) and geo features
    f32x16 ob[1] = {ngp_bias(img, 2, h)};
    ngp_mm<1, 32>(img + FI_A1, hb, ob, lane);
    if (h == 0 && ok) {
      const float o0 = ob[0][0];
      A.out_sigma[i] = sel != 0.0f ? density_act(o0, A.density_act) : 0.0f;
      if (S) {
        S0[NS_O0 * nn] = o0;
        S0[NS_SEL * nn] = sel;
#pragma unroll
        for (int a = 0; a < 3; ++a) S0[(NS_X + a) * nn] = xn[a];
      }
    }
    if (A.density_only) continue;
    // head input: SH values 8 h .. 8 h + 7, base-output registers 0..7
    float hin[16];
    {
      float sh[NGP_SH];
      ngp_sh4(dir, sh);
#pragma unroll
      for (int s = 0; s < 8; ++s) hin[s] = h ? sh[8 + s] : sh[s];
#pragma unroll
      for (int q = 0; q < 8; ++q) hin[8 + q] = ob[0][q];
      if (S && ok) {
#pragma unroll
        for (int s = 0; s < 8; ++s) Sh[(NS_HIN + 4 * h + s) * nn] = hin[s];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (q > 0 || h > 0) Sh[(NS_HIN + NGP_SH - 1 + ngp_row(q, 0)) * nn] = hin[8 + q];
        }
      }
    }
    // head layers 2 (64 x 31) and 3 (64 x 64)
    {
      f32x16 acc[2] = {ngp_bias(img, 3, h), ngp_bias(img, 4, h)};
      ngp_mm<2, 16>(img + FI_A2, hin, acc, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pre = acc[t][r], a = ngp_act_t<RELU>(pre);
          hb[16 * t + r] = a;
          if (S && ok) {
            const int row = 32 * t + ngp_row(r, 0);
            Sh[(NS_H1 + row) * nn] = a;
          }
        }
    }
    {
      f32x16 acc[2] = {ngp_bias(img, 5, h), ngp_bias(img, 6, h)};
      ngp_mm<2, 32>(img + FI_A3, hb, acc, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pre = acc[t][r], a = ngp_act_t<RELU>(pre);
          hb[16 * t + r] = a;
          if (S && ok) {
            const int row = 32 * t + ngp_row(r, 0);
            Sh[(NS_H2 + row) * nn] = a;
          }
        }
    }
    // output layer (rd x 64): rows 0..2 are registers 0..2 of half 0
    f32x16 ro[1] = {ngp_bias(img, 7, h)};
    ngp_mm<1, 32>(img + FI_A4, hb, ro, lane);
    if (h == 0 && ok) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float r = ro[0][c];
        if (c < A.rd)
          A.out_rgb[i * A.rd + c] = A.rad_sigmoid ? __fdiv_rn(1.0f, 1.0f + expf(-r)) : (r > 20.0f ? r : log1pf(expf(r)));
        if (S) S0[(NS_R + c) * nn] = r;
      }
    }
  }
}

// this lane's activation derivative of saved layer rows (outputs at rows Q; the pre-activation rows
// P of the save layout stay unwritten): the softplus derivative from the saved OUTPUT y alone,
// exp(100 x) / (exp(100 x) + 1) = 1 - exp(-100 y) = -expm1(-100 y), and 100 y > 20 exactly where
// 100 x > 20 (torch's threshold; at the boundary both round to 1) -- 192 rows (768 B) per sample
// less to save and re-read than the pre-activations.
template <bool RELU>
__device__ __forceinline__ float ngp_dact_row(const float* S, int P, int Q, int row, int64_t n) {
  if constexpr (RELU) return S[(Q + row) * n] > 0.0f ? 1.0f : 0.0f;
  return ngp_dsp100_out_fast(S[(Q + row) * n]);
}

template <bool RELU>
__global__ __launch_bounds__(NM_THREADS, NM_OCC) void ngp_bwd_mfma_kernel(NgpArgs A) {
  __shared__ __attribute__((aligned(16))) float img[BI_FLOATS];
  const int E = A.enc, L = A.grid.n_levels, rd = A.rd;
  for (int q = threadIdx.x; q < BI_FLOATS; q += NM_THREADS) img[q] = ngp_bi(A.mlp, A.off, E, rd, q);
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int64_t n = A.n;
  const float* S = A.save;
  float* D = A.dz;
  const int64_t ntiles = (n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * NM_WAVES + (threadIdx.x >> 6); tile < ntiles;
       tile += (int64_t)gridDim.x * NM_WAVES) {
    const int64_t i = tile * 32 + j;
    const bool ok = i < n;
    const int64_t ic = ok ? i : n - 1;
    // per-lane bases + uniform row offsets, as in the forward
    int64_t nn = A.ld;
    asm volatile("" : "+s"(nn));
    const float* S0 = S + ic;
    const float* Sh = S + ic + 4 * h * nn;
    float* D0 = D + i;
    float* Dh = D + i + 4 * h * nn;
    // radiance activation: this lane's K index carries outputs h (step 0) and 2 + h (step 1)
    float dr[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = 2 * u + h;
      if (c < rd) {
        const float g = A.d_rgb && ok ? A.d_rgb[ic * rd + c] : 0.0f;
        const float rv = S0[(NS_R + c) * nn];
        if (A.rad_sigmoid) {
          const float s = __fdiv_rn(1.0f, 1.0f + expf(-rv));
          dr[u] = g * (s * (1.0f - s));
        } else {
          const float z = expf(rv);
          dr[u] = rv > 20.0f ? g : g * __fdiv_rn(z, z + 1.0f);
        }
      }
      if (ok && c < 3) D0[(ND_R + c) * nn] = dr[u];
    }
    float dz[32];
    {
      f32x16 acc[2] = {ngp_zero16(), ngp_zero16()};
      ngp_mm<2, 4>(img + BI_A4, dr, acc, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * t + ngp_row(r, 0);
          dz[16 * t + r] = acc[t][r] * ngp_dact_row<RELU>(Sh, NS_H2P, NS_H2, row, nn);
          if (ok) Dh[(ND_Z3 + row) * nn] = dz[16 * t + r];
        }
    }
    {
      f32x16 acc[2] = {ngp_zero16(), ngp_zero16()};
      ngp_mm<2, 32>(img + BI_A3, dz, acc, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * t + ngp_row(r, 0);
          dz[16 * t + r] = acc[t][r] * ngp_dact_row<RELU>(Sh, NS_H1P, NS_H1, row, nn);
          if (ok) Dh[(ND_Z2 + row) * nn] = dz[16 * t + r];
        }
    }
    // base output: geo rows 1..15 from the head input gradient, row 0 the density's
    float dob[8];
    {
      f32x16 dg[1] = {ngp_zero16()};
      ngp_mm<1, 32>(img + BI_A2, dz, dg, lane);
      const float gs = A.d_sigma && ok ? A.d_sigma[ic] : 0.0f;
      const float sel = S0[NS_SEL * nn];
      const float o0 = S0[NS_O0 * nn];
      const float d0 = sel != 0.0f ? gs * density_dact_from_raw(o0, A.density_act) : 0.0f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        dob[q] = q == 0 && h == 0 ? d0 : dg[0][q];
        if (ok) Dh[(ND_O + ngp_row(q, 0)) * nn] = dob[q];
      }
    }
    {
      f32x16 acc[2] = {ngp_zero16(), ngp_zero16()};
      ngp_mm<2, 8>(img + BI_A1, dob, acc, lane);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 32 * t + ngp_row(r, 0);
          dz[16 * t + r] = acc[t][r] * ngp_dact_row<RELU>(Sh, NS_H0P, NS_H0, row, nn);
          if (ok) Dh[(ND_Z0 + row) * nn] = dz[16 * t + r];
        }
    }
    f32x16 df[1] = {ngp_zero16()};
    ngp_mm<1, 32>(img + BI_A0, dz, df, lane);
    // the encoding gradient goes to ND_F rows; ngp_scatter_kernel aggregates and adds it
    if (ok) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (ngp_row(r, h) < E) Dh[(ND_F + ngp_row(r, 0)) * nn] = df[0][r];
    }
  }
}

}  // namespace den

namespace den {

// ------------------------------------------------------------------ workgroup-aggregated table scatter
// The memory-side atomic requests (one per distinct 64-B segment per instruction) bound the table
// gradient: 32 per sample in the configs[3] emulation with the in-kernel fold + quad scatter.  Here a
// workgroup takes 256 consecutive samples (ray-ordered: one or two rays) and, level by level, inserts
// their 8 corner contributions into an LDS hash table keyed by the entry index (open addressing, slot
// = index mod 4096, at most 2,048 records so never full; LDS float atomics merge equal entries), then
// walks the table in slot order with lane pairs on the two features of one entry: entries that are
// neighbours in memory (x-neighbour cells: dense rows, or the aligned 8-entry groups of a hashed level)
// sit in neighbouring slots, so one 64-B request carries up to 8 entries' adds.
constexpr int NSC_SLOTS = 4096, NSC_THREADS = 256;
constexpr uint32_t NSC_EMPTY = 0xFFFFFFFFu;

// Same-cell lanes fold first (ngp_fold: coarse levels put whole runs of a ray in one cell, which would
// serialise on the LDS atomics); the emission pass leaves the table empty for the next level.
__global__ __launch_bounds__(NSC_THREADS) void ngp_scatter_kernel(NgpArgs A) {
  __shared__ uint32_t key[NSC_SLOTS];
  __shared__ float val[2][NSC_SLOTS];
  const int tid = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * NSC_THREADS + tid;
  const bool ok = i < A.n;
  const int64_t ic = ok ? i : A.n - 1;
  float xn[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xn[a] = A.save[(int64_t)(NS_X + a) * A.ld + ic];
  for (int q = tid; q < NSC_SLOTS; q += NSC_THREADS) {
    key[q] = NSC_EMPTY;
    val[0][q] = 0.0f;
    val[1][q] = 0.0f;
  }
  __syncthreads();
  for (int l = 0; l < A.grid.n_levels; ++l) {
    const float g0 = ok ? A.dz[(int64_t)(ND_F + 2 * l) * A.ld + ic] : 0.0f;
    const float g1 = ok ? A.dz[(int64_t)(ND_F + 2 * l + 1) * A.ld + ic] : 0.0f;
    NgpCorner C;
    uint32_t cell[3];
    ngp_corners(A.grid, l, xn, C, cell);
    float v[16];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      v[2 * c] = C.w[c] * g0;
      v[2 * c + 1] = C.w[c] * g1;
    }
    // the zero test goes into the fold: a lane with nothing to add neither absorbs its same-cell
    // partners (which would drop their values) nor is absorbed
    const bool emit = ngp_fold(cell, v, ok && (g0 != 0.0f || g1 != 0.0f));
    if (emit) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t e = C.idx[c];
        uint32_t s = e & (NSC_SLOTS - 1);
        while (true) {
          const uint32_t k = key[s];
          if (k == e) break;
          if (k == NSC_EMPTY) {
            const uint32_t old = atomicCAS(&key[s], NSC_EMPTY, e);
            if (old == NSC_EMPTY || old == e) break;
          }
          s = (s + 1) & (NSC_SLOTS - 1);
        }
        atomicAdd(&val[0][s], v[2 * c]);
        atomicAdd(&val[1][s], v[2 * c + 1]);
      }
    }
    __syncthreads();
    for (int q = tid; q < 2 * NSC_SLOTS; q += NSC_THREADS) {
      const int s = q >> 1, f = q & 1;
      const uint32_t k = key[s];
      if (k != NSC_EMPTY) {
        unsafeAtomicAdd(A.d_table + 2 * (int64_t)k + f, val[f][s]);
        val[f][s] = 0.0f;
        if (f == 0) key[s] = NSC_EMPTY;  // the f = 1 lane of the pair read it in the same instruction
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ weight gradients on MFMA
// dW[o][k] = sum_s dZ[o][s] X[k][s], db[o] = sum_s dZ[o][s] with the samples as the K dimension of
// v_mfma_f32_32x32x2_f32: A[m][k] = dZ row m, B[k][n] = X row n.  Six tasks of two 32 x 32 tiles
// each: layer 0 (2 row tiles x E columns), layer 1 (16 rows x 2 column tiles), layer 2 (2 x 31),
// layer 3 rows 0..31 and 32..63 (x 2 column tiles each), layer 4 (rd x 2).  Lane (j, h) loads row j
// of a 32-row block at samples 8 u + 4 h .. + 3 (one 16-B load per operand row block and 4 steps;
// any sample-to-k assignment works as long as A and B agree), so the feature-major rows stream in
// without LDS.  The bias is the row sum of the A operand, accumulated (in f64) from the same registers.
// Workgroup = (split, task), 4 waves over interleaved 32-sample chunks, reduced through LDS into
// partials [task][split][2][32][32] + [64]; a second kernel sums the splits in a fixed order.
constexpr int NDW_TASKS = 6, NDW_PART = 2 * 32 * 32 + 64;
constexpr int NDW_CHUNK = 64;  // the samples of a split: a multiple of this (the padded save stride)

struct NgpDwTask {
  int a_row, a_rows, mt;  // dZ rows (first, valid count), row tiles (1 or 2; column tiles = 3 - mt)
  int b_row, b_rows;      // X rows
  int k_in, m_off;        // weight row length, first weight row of the task
  int64_t w_off, b_off;
};
struct NgpDwMfArgs {
  const float* dz;
  const float* save;
  int64_t n, ld, per_split;
  int splits;
  NgpDwTask T[NDW_TASKS];
  float* partial;  // [task][split][NDW_PART]
  float* grad;
};

// 4 samples of row `row` (valid if row < rows) starting at q (zero past s1)
__device__ __forceinline__ f32x4 ngp_dw_load(const float* base, int row, int rows, int64_t ld, int64_t q, int64_t s1) {
  f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
  if (row < rows && q < s1) {
    v = *(const f32x4*)(base + (int64_t)row * ld + q);
    if (q + 4 > s1) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (q + e >= s1) v[e] = 0.0f;
    }
  }
  return v;
}

// MT: row tiles of the launch's tasks (2: layers 0 and 2; 1: the others) -- a compile-time operand
// shape keeps the double-buffered operands at 3 x 4 x 4 registers per buffer
template <int MT>
__global__ __launch_bounds__(256) void ngp_dw_mfma_kernel(NgpDwMfArgs P, int task0, int task_stride) {
  __shared__ __attribute__((aligned(16))) float red[2][NDW_PART];
  const int task = task0 + (int)blockIdx.y * task_stride;
  const NgpDwTask T = P.T[task];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  constexpr int mt = MT, nt = 3 - MT;
  const float* Ab = P.dz + (int64_t)T.a_row * P.ld;
  const float* Bb = P.save + (int64_t)T.b_row * P.ld;
  const int64_t s0 = (int64_t)blockIdx.x * P.per_split;
  const int64_t s1 = s0 + P.per_split < P.n ? s0 + P.per_split : P.n;
  f32x16 acc[2] = {ngp_zero16(), ngp_zero16()};
  double bsum[2] = {0.0, 0.0};  // f64: the bias is a long sum of cancelling terms
  // the operands of chunk c + 128 load while chunk c's MFMAs run (two register sets, unrolled by 2)
  auto load = [&](int64_t c, f32x4 (&a)[mt][4], f32x4 (&b)[nt][4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = c + 8 * u + 4 * h;
#pragma unroll
      for (int t = 0; t < mt; ++t) a[t][u] = ngp_dw_load(Ab, 32 * t + j, T.a_rows, P.ld, q, s1);
#pragma unroll
      for (int t = 0; t < nt; ++t) b[t][u] = ngp_dw_load(Bb, 32 * t + j, T.b_rows, P.ld, q, s1);
    }
  };
  auto compute = [&](const f32x4 (&a)[mt][4], const f32x4 (&b)[nt][4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (mt == 2) {
          acc[0] = ngp_mfma(a[0][u][e], b[0][u][e], acc[0]);
          acc[1] = ngp_mfma(a[1][u][e], b[0][u][e], acc[1]);
          bsum[1] += (double)a[1][u][e];
        } else {
          acc[0] = ngp_mfma(a[0][u][e], b[0][u][e], acc[0]);
          acc[1] = ngp_mfma(a[0][u][e], b[1][u][e], acc[1]);
        }
        bsum[0] += (double)a[0][u][e];
      }
  };
  f32x4 a0[mt][4], b0[nt][4], a1[mt][4], b1[nt][4];
  const int64_t c0 = s0 + 32 * wave;
  if (c0 < s1) load(c0, a0, b0);
  for (int64_t c = c0; c < s1; c += 256) {
    if (c + 128 < s1) load(c + 128, a1, b1);
    compute(a0, b0);
    if (c + 256 < s1) load(c + 256, a0, b0);
    if (c + 128 < s1) compute(a1, b1);
  }
  // tile tt: rows ngp_row(r, h), column j; bias of rows 32 t + j from both halves.  Waves 2, 3 store,
  // waves 0, 1 add theirs: the split's partial is (w0 + w2) + (w1 + w3), a fixed order.
  float bias[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) bias[t] = (float)(bsum[t] + __shfl_xor(bsum[t], 32));
  float* R = red[wave & 1];
  if (wave >= 2) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 16; ++r) R[tt * 1024 + ngp_row(r, h) * 32 + j] = acc[tt][r];
    if (h == 0) {
      R[2048 + j] = bias[0];
      R[2048 + 32 + j] = bias[1];
    }
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float& d = R[tt * 1024 + ngp_row(r, h) * 32 + j];
        d = acc[tt][r] + d;
      }
    if (h == 0) {
      R[2048 + j] = bias[0] + R[2048 + j];
      R[2048 + 32 + j] = bias[1] + R[2048 + 32 + j];
    }
  }
  __syncthreads();
  float* out = P.partial + ((int64_t)task * P.splits + blockIdx.x) * NDW_PART;
  for (int e = threadIdx.x; e < NDW_PART; e += 256) out[e] = red[0][e] + red[1][e];
}

// 64 partial elements per workgroup, the splits in 4 interleaved groups (8 loads in flight per
// lane), the groups combined in a fixed order
__global__ __launch_bounds__(256) void ngp_dw_mfma_reduce_kernel(NgpDwMfArgs P) {
  __shared__ float part[4][64];
  const NgpDwTask T = P.T[blockIdx.y];
  const int el = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el;
  float s = 0.0f;
  if (e < NDW_PART) {
    const float* src = P.partial + (int64_t)blockIdx.y * P.splits * NDW_PART + e;
    int sp = g;
    for (; sp + 28 < P.splits; sp += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(sp + 4 * u) * NDW_PART];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; sp < P.splits; sp += 4) s += src[(int64_t)sp * NDW_PART];
  }
  part[g][el] = s;
  __syncthreads();
  if (g != 0 || e >= NDW_PART) return;
  s = (part[0][el] + part[1][el]) + (part[2][el] + part[3][el]);
  if (e < 2048) {
    const int tt = e >> 10, row = (e >> 5) & 31, col = e & 31;
    const int mrow = (T.mt == 2 ? 32 * tt : 0) + row, ncol = (T.mt == 2 ? 0 : 32 * tt) + col;
    if (mrow < T.a_rows && ncol < T.b_rows) P.grad[T.w_off + (int64_t)(T.m_off + mrow) * T.k_in + ncol] = s;
  } else {
    const int m = e - 2048;
    if (m < T.a_rows) P.grad[T.b_off + T.m_off + m] = s;
  }
}

}  // namespace den
