// den_ngp.hip -- the `ngp` radiance field (reference external/ngp.py NGPradianceField, the shipped
// default arch of configs/train/*.yaml): tiny-cuda-nn's multiresolution hash-grid encoding, the
// mlp_base / mlp_head MLPs (external/mlp.py MLP with the configured activations), the degree-4
// SH view encoding (external/sh_encoder.py) and shifted_trunc_exp density -- forward, backward
// (hash-table scatter + per-sample layer gradients) and the weight-gradient GEMMs.
//
// One sample per lane.  The work per sample is latency-bound gathers (16 levels x 8 corners of
// float2 from a <= 50 MB table, resident in the 256 MB MALL) plus 9.3 K f32 MACs of tiny MLPs,
// so the field is laid out for occupancy, not for MFMA: the MLP weights are wave-uniform
// (kernel-argument pointer + compile-time offsets), so they come through the scalar cache into
// SGPR operands of v_fmac_f32 and cost no VGPRs or LDS; activations stay in VGPRs.  f32
// throughout, in torch's operation order where it matters (softplus threshold, SH products),
// so parity is at the f32-rounding level against the reference.
//
// Saved state (train) and per-layer gradients are FEATURE-major ([row][n]): a wave's stores and
// loads of one feature are 256 contiguous bytes, and the weight-gradient GEMM dW = dZ^T X reads
// rows that are contiguous over samples (k = samples).
#include "den_device.h"

namespace den {

constexpr int NGP_MAX_LEVELS = 16;
constexpr int NGP_F = 2;                         // features per level
constexpr int NGP_ENC = NGP_MAX_LEVELS * NGP_F;  // encoding width (32)
constexpr int NGP_W = 64;                        // n_neurons (base and head)
constexpr int NGP_GEO = 15;                      // geo_feat_dim
constexpr int NGP_SH = 16;                       // SH degree 4
constexpr int NGP_HIN = NGP_SH + NGP_GEO;        // head input (31)

// MLP parameter offsets (floats) after the hash table, reference named_parameters() order:
// mlp_base.1.hidden_layers.0 (64 x E, E = 2 n_levels), mlp_base.1.output_layer (16 x 64),
// mlp_head.hidden_layers.0 (64 x 31), .1 (64 x 64), mlp_head.output_layer (rd x 64); weight then
// bias, torch (out, in) layout.
struct NgpOff {
  int w[5], b[5];
};
DEN_HD inline NgpOff ngp_offsets(int enc, int rd) {
  NgpOff o{};
  const int in[5] = {enc, NGP_W, NGP_HIN, NGP_W, NGP_W};
  const int out[5] = {NGP_W, 1 + NGP_GEO, NGP_W, NGP_W, rd};
  int off = 0;
  for (int l = 0; l < 5; ++l) {
    o.w[l] = off;
    off += in[l] * out[l];
    o.b[l] = off;
    off += out[l];
  }
  return o;
}
DEN_HD inline int ngp_mlp_params(int enc, int rd) {
  const NgpOff o = ngp_offsets(enc, rd);
  return o.b[4] + rd;
}

// saved rows (train): encoding, pre-activation and output of each hidden layer, head input,
// radiance pre-activation, density pre-activation, selector, contracted position
enum {
  NS_FEAT = 0,
  NS_H0P = NS_FEAT + NGP_ENC,
  NS_H0 = NS_H0P + NGP_W,
  NS_HIN = NS_H0 + NGP_W,
  NS_H1P = NS_HIN + 32,
  NS_H1 = NS_H1P + NGP_W,
  NS_H2P = NS_H1 + NGP_W,
  NS_H2 = NS_H2P + NGP_W,
  NS_R = NS_H2 + NGP_W,
  NS_O0 = NS_R + 4,
  NS_SEL = NS_O0 + 1,
  NS_X = NS_SEL + 1,
  NS_ROWS = NS_X + 3
};
// per-layer pre-activation gradients (rows): layer 0 (64), base output (16), head 0 (64), head 1 (64), rgb (rd)
// and (MFMA backward with the workgroup-aggregated scatter) the encoding gradient (E rows)
enum { ND_Z0 = 0, ND_O = ND_Z0 + NGP_W, ND_Z2 = ND_O + 1 + NGP_GEO, ND_Z3 = ND_Z2 + NGP_W, ND_R = ND_Z3 + NGP_W,
       ND_F = ND_R + 4, ND_ROWS = ND_F + NGP_ENC };

struct NgpGrid {
  int n_levels;
  int hashed;                      // HashGrid (tcnn GridType::Hash) vs DenseGrid
  float scale[NGP_MAX_LEVELS];     // exp2f(l * log2f(per_level_scale)) * base_resolution - 1
  uint32_t res[NGP_MAX_LEVELS];    // ceilf(scale) + 1
  uint32_t entries[NGP_MAX_LEVELS];
  uint32_t offset[NGP_MAX_LEVELS];  // entry offset of the level
};

struct NgpArgs {
  int64_t n;
  int rd;
  int points;        // 1: positions x (n,3) + directions (n,3); 2: packed samples of rays
  int contraction;   // CONTRACT_*
  int hidden_relu;   // hidden activation: 0 softplus(beta = 100), 1 relu
  int rad_sigmoid;   // radiance activation: 0 softplus(beta = 1), 1 sigmoid
  int density_act;   // density activation (den_device.h density_act)
  int density_only;  // sigma_fn of the marching pre-pass: skip the head
  float aabb[6];
  const float* x;    // points 1: positions; points 2: ray origins (R,3)
  const float* d;    // points 1: directions; points 2: ray directions (R,3)
  const int* ray_idx;
  const float* t0;
  const float* t1;
  const float* table;  // hash-grid parameters
  const float* mlp;    // MLP parameters (offsets: off)
  NgpOff off;
  int enc;             // encoding width 2 n_levels (<= NGP_ENC)
  NgpGrid grid;
  float* out_rgb;      // (n, rd)
  float* out_sigma;    // (n)
  int64_t ld;          // row stride of save / dz: n rounded up to 64 (16-B aligned sample quads)
  float* save;         // train: [NS_ROWS][ld]
  // backward
  const float* d_rgb;
  const float* d_sigma;
  float* d_table;
  float* dz;           // [ND_ROWS][ld]
};

// ------------------------------------------------------------------ elementwise pieces

// SHEncoder (external/sh_encoder.py:27-80), degree 4, the reference's f32 operation order
__device__ __forceinline__ void ngp_sh4(const float* dv, float* out) {
#pragma clang fp contract(off)
  const float x = dv[0], y = dv[1], z = dv[2];
  const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
  out[0] = 0.28209479177387814f;
  out[1] = -0.48860251190291987f * y;
  out[2] = 0.48860251190291987f * z;
  out[3] = -0.48860251190291987f * x;
  out[4] = 1.0925484305920792f * xy;
  out[5] = -1.0925484305920792f * yz;
  out[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
  out[7] = -1.0925484305920792f * xz;
  out[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
  out[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
  out[10] = 2.8906114426405538f * xy * z;
  out[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
  out[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
  out[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
  out[14] = 1.4453057213202769f * z * (x2 - y2);
  out[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

// ------------------------------------------------------------------ grid encoding (tcnn grid.h)
// cell / fractional position of one coordinate: pos = fmaf(scale, x, 0.5) (pos_fract)
struct NgpCorner {
  uint32_t idx[8];
  float w[8];
};

// the grid constants of one level
struct NgpLevel {
  float scale;
  uint32_t res, entries, offset;
};
__device__ __forceinline__ NgpLevel ngp_level(const NgpGrid& G, int l) {
  return NgpLevel{G.scale[l], G.res[l], G.entries[l], G.offset[l]};
}

__device__ __forceinline__ uint32_t ngp_index(const NgpLevel& V, int hashed, uint32_t cx, uint32_t cy, uint32_t cz) {
  // grid_index: dense strides while the stride stays <= the level size, else the prime hash
  const uint32_t size = V.entries, res = V.res;
  uint32_t stride = 1, index = 0;
  const uint32_t c[3] = {cx, cy, cz};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    if (stride <= size) {
      index += c[d] * stride;
      stride *= res;
    } else {
      stride = 0xFFFFFFFFu;  // the loop has ended (stride > size stays true)
    }
  }
  // index % size without the ~40-instruction runtime division where it is not needed: a hashed
  // level has size = 2^log2_hashmap_size (entries were capped there); a dense index of in-range cells
  // is below 2 size (cell <= res - 1, +1 for the upper corner: < res^3 + res^2 + res < 2 size)
  if (hashed && size < stride) return (cx ^ (cy * 2654435761u) ^ (cz * 805459861u)) & (size - 1);
  if (index < size) return index;
  return index - size < size ? index - size : index % size;
}

__device__ __forceinline__ void ngp_corners(const NgpLevel& V, int hashed, const float* x, NgpCorner& C,
                                            uint32_t* cell_out = nullptr) {
  float frac[3];
  uint32_t cell[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float pos = fmaf(V.scale, x[d], 0.5f);
    const float fl = floorf(pos);
    cell[d] = (uint32_t)(int)fl;
    frac[d] = pos - fl;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float w = 1.0f;
    uint32_t p[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      if ((c >> d) & 1) {
        w *= frac[d];
        p[d] = cell[d] + 1;
      } else {
        w *= 1.0f - frac[d];
        p[d] = cell[d];
      }
    }
    C.w[c] = w;
    C.idx[c] = V.offset + ngp_index(V, hashed, p[0], p[1], p[2]);
  }
  if (cell_out) {
#pragma unroll
    for (int d = 0; d < 3; ++d) cell_out[d] = cell[d];
  }
}
__device__ __forceinline__ void ngp_corners(const NgpGrid& G, int l, const float* x, NgpCorner& C,
                                            uint32_t* cell_out = nullptr) {
  ngp_corners(ngp_level(G, l), G.hashed, x, C, cell_out);
}

// Pre-aggregation of the table-gradient scatter: the samples of a wave are consecutive samples of
// the packed rays, so at the coarse levels neighbouring lanes sit in the same cell and add to the
// same 8 entries.  In steps k = 0 .. NGP_AGG_STEPS - 1, the lane with the k + 1 low bits clear
// folds in the 16 values of lane + 2^k when both hold the same base cell (lane ^ 1, ^ 2 by DPP
// quad_perm, ^ 4, ^ 8, ^ 16 by ds_swizzle bit mode); only lanes that were not folded issue atomics.
// Equal cells give identical corner indices, so the fold is exact (another summation order of the
// same terms, like the atomics themselves).  Measured on the configs[3] emulation (ray-ordered
// samples): 1.19 -> 0.88 s per optimizer step with quads at every level, 0.84 with 16-lane groups; no
// cost on unordered points (profiles/ngp_bench.py).
constexpr int NGP_AGG_STEPS = 4;  // configs[3] emulation: 0.88 (2 steps) / 0.86 (3) / 0.84 (4) / 0.84 (5) s per step
// value of lane ^ 2^K (K < 5: within 32 lanes); an inactive source yields `old`
template <int K>
__device__ __forceinline__ int ngp_xlane(int v, int old) {
  if constexpr (K == 0) return __builtin_amdgcn_update_dpp(old, v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
  else if constexpr (K == 1) return __builtin_amdgcn_update_dpp(old, v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
  else return __builtin_amdgcn_ds_swizzle(v, ((1 << K) << 10) | 0x1F);  // bit mode: xor_mask = 2^K
}
template <int K>
__device__ __forceinline__ void ngp_fold_step(const uint32_t* cell, float* v, bool& alive, uint64_t active) {
  const int lane = threadIdx.x & 63;
  constexpr int M = (2 << K) - 1;
  // a partner past n (returned, or not `ok`) has stale registers: it never matches
  bool same = (active >> (lane ^ (1 << K))) & 1;
#pragma unroll
  for (int d = 0; d < 3; ++d) same = same && (uint32_t)ngp_xlane<K>((int)cell[d], 0) == cell[d];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float pv = __builtin_bit_cast(float, ngp_xlane<K>(__builtin_bit_cast(int, v[q]), 0));
    if ((lane & M) == 0 && same) v[q] += pv;
  }
  if ((lane & M) == (1 << K) && same) alive = false;
}
// -> whether this lane still issues its (folded) values; `ok` false: a lane past n (it issues nothing
// and is nobody's partner)
__device__ __forceinline__ bool ngp_fold(const uint32_t* cell, float* v, bool ok = true) {
  bool alive = ok;
  const uint64_t active = __ballot(ok);
  ngp_fold_step<0>(cell, v, alive, active);
  if constexpr (NGP_AGG_STEPS > 1) ngp_fold_step<1>(cell, v, alive, active);
  if constexpr (NGP_AGG_STEPS > 2) ngp_fold_step<2>(cell, v, alive, active);
  if constexpr (NGP_AGG_STEPS > 3) ngp_fold_step<3>(cell, v, alive, active);
  if constexpr (NGP_AGG_STEPS > 4) ngp_fold_step<4>(cell, v, alive, active);
  return alive;
}

__device__ __forceinline__ void ngp_encode(const NgpGrid& G, const float* __restrict__ table, const float* x,
                                           float* feat) {
#pragma unroll
  for (int l = 0; l < NGP_MAX_LEVELS; ++l) {
    float f0 = 0.0f, f1 = 0.0f;
    if (l < G.n_levels) {
      NgpCorner C;
      ngp_corners(G, l, x, C);
      float2 v[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = *(const float2*)(table + 2 * (int64_t)C.idx[c]);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        f0 = fmaf(C.w[c], v[c].x, f0);
        f1 = fmaf(C.w[c], v[c].y, f1);
      }
    }
    feat[2 * l] = f0;
    feat[2 * l + 1] = f1;
  }
}

// position (points 1: given; points 2: o + d (t0 + t1)/2 of the sample's ray) -> contracted x in
// [0,1]^3 + selector (ngp.py:230-238), and the view direction
__device__ __forceinline__ void ngp_point(const NgpArgs& A, int64_t i, float* xn, float* sel, float* dir) {
  float pos[3];
  if (A.points == 2) {
    const int64_t r = A.ray_idx[i];
    float o[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.x[r * 3 + a];
      dir[a] = A.d[r * 3 + a];
    }
    {
#pragma clang fp contract(off)
      const float tt = A.t0[i] + A.t1[i];
#pragma unroll
      for (int a = 0; a < 3; ++a) pos[a] = o[a] + __fdiv_rn(dir[a] * tt, 2.0f);
    }
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      pos[a] = A.x[i * 3 + a];
      dir[a] = A.d[i * 3 + a];
    }
  }
  contract_unit(pos, A.aabb, xn, sel, A.contraction);
}

// ------------------------------------------------------------------ standalone encoding (tcnn.Encoding)
struct NgpEncArgs {
  int64_t n;
  NgpGrid grid;
  const float* x;      // (n, 3) in [0,1]
  const float* table;
  float* out;          // (n, 2 L)
  const float* d_out;  // backward
  float* d_table;
};

__global__ __launch_bounds__(256) void ngp_encode_kernel(NgpEncArgs E) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E.n) return;
  float x[3] = {E.x[i * 3], E.x[i * 3 + 1], E.x[i * 3 + 2]};
  float feat[NGP_ENC];
  ngp_encode(E.grid, E.table, x, feat);
  const int w = 2 * E.grid.n_levels;
  for (int f = 0; f < w; ++f) E.out[i * w + f] = feat[f];
}

__global__ __launch_bounds__(256) void ngp_encode_bwd_kernel(NgpEncArgs E) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E.n) return;
  float x[3] = {E.x[i * 3], E.x[i * 3 + 1], E.x[i * 3 + 2]};
  const int w = 2 * E.grid.n_levels;
  for (int l = 0; l < E.grid.n_levels; ++l) {
    NgpCorner C;
    ngp_corners(E.grid, l, x, C);
    const float g0 = E.d_out[i * w + 2 * l], g1 = E.d_out[i * w + 2 * l + 1];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float* t = E.d_table + 2 * (int64_t)C.idx[c];
      unsafeAtomicAdd(t, C.w[c] * g0);
      unsafeAtomicAdd(t + 1, C.w[c] * g1);
    }
  }
}

}  // namespace den
