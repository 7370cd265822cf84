// den_device.h -- device-side helpers: MFMA traits, exact-f32 sampler math,
// activations, wave scans, weight-chunk staging.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "den_geom.h"

// Every hot kernel's code starts on a 4 KiB boundary (r04y A/B); -DDEN_NO_CODE_ALIGN
// builds the default placement for the instruction-fetch comparison (profiles/gpu_r05pl.sh)
#ifdef DEN_NO_CODE_ALIGN
#define DEN_CODE_ALIGN
#else
#define DEN_CODE_ALIGN __attribute__((aligned(4096)))
#endif

// Diagnostic build only (-DDEN_CLOCK, MI355X_MICROARCH.md 'DVFS give-back' item 6): each hot kernel
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz) once at its start and once at its end,
// workgroup by workgroup, into a buffer of its own that no kernel reads (den_debug_clock copies it
// out); in-kernel clock = delta memtime / delta realtime x 100 MHz.  Kernel slots: 0 render_fwd,
// 1 render_head_bwd, 2 hidden_bwd (L7..L1, the last launch wins), 3 hidden_bwd Lb, 4 dwstream.
#ifdef DEN_CLOCK
constexpr int DEN_CLOCK_KERNELS = 5, DEN_CLOCK_WGS = 512;
__device__ uint64_t den_clock[DEN_CLOCK_KERNELS * DEN_CLOCK_WGS * 4];
#define DEN_CLOCK_BEGIN()                                            \
  const uint64_t den_clk_t0_ = __builtin_amdgcn_s_memtime();         \
  const uint64_t den_clk_r0_ = __builtin_amdgcn_s_memrealtime()
#define DEN_CLOCK_END(k)                                                                       \
  do {                                                                                         \
    const uint64_t t1_ = __builtin_amdgcn_s_memtime(), r1_ = __builtin_amdgcn_s_memrealtime(); \
    if (threadIdx.x == 0 && blockIdx.x < DEN_CLOCK_WGS) {                                      \
      uint64_t* o_ = den_clock + ((int64_t)(k) * DEN_CLOCK_WGS + blockIdx.x) * 4;              \
      __builtin_nontemporal_store(den_clk_t0_, o_);                                            \
      __builtin_nontemporal_store(den_clk_r0_, o_ + 1);                                        \
      __builtin_nontemporal_store(t1_, o_ + 2);                                                \
      __builtin_nontemporal_store(r1_, o_ + 3);                                                \
    }                                                                                          \
  } while (0)
#else
#define DEN_CLOCK_BEGIN() \
  do {                    \
  } while (0)
#define DEN_CLOCK_END(k) \
  do {                   \
  } while (0)
#endif

namespace den {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE> struct Tr;

// BF16 perf mode: v_mfma_f32_32x32x16_bf16. Lane l: col = l&31, group h = l>>5.
template <> struct Tr<1> {
  static constexpr int TM = 32, KI = 16, NG = 2, REGS = 16, FPT = 2 /* frags per tile */;
  using Acc = f32x16;
  using Frag = bf16x8;
  static __device__ __forceinline__ Acc mfma(const Frag& a, const Frag& b, const Acc& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ Frag zero_frag() {
    Frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (__bf16)0.0f;
    return f;
  }
};

// F32 parity mode: v_mfma_f32_16x16x4_f32 (exact f32 FMA chain). Lane l: col = l&15, group g = l>>4.
template <> struct Tr<0> {
  static constexpr int TM = 16, KI = 4, NG = 4, REGS = 4, FPT = 4;
  using Acc = f32x4;
  using Frag = float;
  static __device__ __forceinline__ Acc mfma(float a, float b, const Acc& c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ Frag zero_frag() { return 0.0f; }
};

template <int MODE>
__device__ __forceinline__ void acc_to_frags(const typename Tr<MODE>::Acc& a, typename Tr<MODE>::Frag* f) {
  if constexpr (MODE == 1) {
    // one v_cvt_pk_bf16_f32 per register pair (element-wise casts let the compiler pair them
    // across the SLP-packed adds of the epilogue, at the cost of v_alignbit / v_perm fix-ups)
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x2 p = {a[8 * s + 2 * q], a[8 * s + 2 * q + 1]};
        w[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(p, bf16x2));
      }
      const uint4 u = make_uint4(w[0], w[1], w[2], w[3]);
      f[s] = __builtin_bit_cast(bf16x8, u);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) f[r] = a[r];
  }
}

template <int MODE>
__device__ __forceinline__ typename Tr<MODE>::Acc acc_zero() {
  typename Tr<MODE>::Acc a;
#pragma unroll
  for (int r = 0; r < Tr<MODE>::REGS; ++r) a[r] = 0.0f;
  return a;
}

// Activation tensors in HBM are wave-block major (den_geom.h): the TM x TN tile of one wave is
// one contiguous block -- [frag f][lane][16 B] in BF16 (2 KiB), [lane][16 B] in F32 (1 KiB) --
// so every store / load instruction of a wave moves 1 KiB of consecutive bytes.
// `tile` is the (wave-uniform) base of the tile; each lane adds its own offset.

// Activation / dz tiles are written once and read once, by a later kernel, after far more data
// than the caches hold: BF16 stores and loads of them go non-temporal.
typedef unsigned int den_u32x4 __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ void st_stream(V* p, V v) {
  static_assert(sizeof(V) == 16, "16-byte streams");
  __builtin_nontemporal_store(__builtin_bit_cast(den_u32x4, v), (den_u32x4*)p);
}
// A wave-uniform read of kernel-constant data (ray inputs, the background colour) as a SCALAR load
// (constant address space): it waits on lgkmcnt, not behind every older vector-memory op of the wave
// (vmcnt is in-order: a vector load here would wait out the wave's stores and LDS-DMAs in flight).
// The address must be wave-uniform.
template <typename T>
__device__ __forceinline__ T ld_uniform(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}
template <typename V>
__device__ __forceinline__ V ld_stream(const V* p) {
  static_assert(sizeof(V) == 16, "16-byte streams");
  return __builtin_bit_cast(V, __builtin_nontemporal_load((const den_u32x4*)p));
}

// Store a lane's operand fragments of one tile (stored order: regs 0..REGS-1).
template <int MODE>
__device__ __forceinline__ void store_tile_frags(void* tile, const typename Tr<MODE>::Frag* f) {
  char* p = (char*)tile + (threadIdx.x & 63) * 16;
  if constexpr (MODE == 1) {
    st_stream((bf16x8*)p, f[0]);
    st_stream((bf16x8*)(p + 1024), f[1]);
  } else {
    f32x4 v = {f[0], f[1], f[2], f[3]};
    *(f32x4*)p = v;
  }
}

// Store a lane's REGS accumulator values (stored order) as operand dtype.
template <int MODE>
__device__ __forceinline__ void store_tile_vals(void* tile, const typename Tr<MODE>::Acc& a) {
  char* p = (char*)tile + (threadIdx.x & 63) * 16;
  if constexpr (MODE == 1) {
    uint32_t w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      __bf16 lo = (__bf16)a[2 * q], hi = (__bf16)a[2 * q + 1];
      w[q] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
    st_stream((uint4*)p, make_uint4(w[0], w[1], w[2], w[3]));
    st_stream((uint4*)(p + 1024), make_uint4(w[4], w[5], w[6], w[7]));
  } else {
    *(f32x4*)p = a;
  }
}

template <int MODE>
__device__ __forceinline__ typename Tr<MODE>::Acc load_tile_vals(const void* tile) {
  typename Tr<MODE>::Acc a;
  const char* p = (const char*)tile + (threadIdx.x & 63) * 16;
  if constexpr (MODE == 1) {
    uint4 u0 = ld_stream((const uint4*)p), u1 = ld_stream((const uint4*)(p + 1024));
    uint32_t w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      a[2 * q] = __uint_as_float(w[q] << 16);
      a[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
    a = *(const f32x4*)p;
  }
  return a;
}

// ------------------------------------------------------------------ activations
// torch.nn.functional.softplus(x, beta, threshold=20) and its derivative.
template <bool EXACT>
__device__ __forceinline__ float softplus_b100(float z) {
  float bz = z * 100.0f;
  if (bz > 20.0f) return z;
  if constexpr (EXACT) return log1pf(expf(bz)) / 100.0f;
  else return __logf(1.0f + __expf(bz)) * 0.01f;
}
// derivative from the activation's own output s = softplus(z): sigmoid(100 z) = 1 - exp(-100 s)
template <bool EXACT>
__device__ __forceinline__ float dsoftplus_b100_from_out(float s) {
  if constexpr (EXACT) return -expm1f(-100.0f * s);
  else return 1.0f - __expf(-100.0f * s);
}
// BF16 path, base-2 scaled units (den_geom.h KAPPA): s' = max(t,0) + log2(1 + 2^-|t|)
// (for t > 20*log2(e) the log term is 0 in f32: torch's threshold branch).
// max(t, 0) as v_med3_f32(t, 0, FLT_MAX): fmaxf lowers to maxnum, which makes the compiler
// canonicalize an MFMA result first (a second v_max_f32 per element in the forward epilogue).
__device__ __forceinline__ float softplus2_scaled(float t) {
  return __builtin_amdgcn_fmed3f(t, 0.0f, 3.4028235e38f) +
         __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(-fabsf(t)));
}
// its derivative from the output: sigmoid(100 z) = 1 - 2^-s'
__device__ __forceinline__ float dsoftplus2_scaled_from_out(float s) { return 1.0f - __builtin_amdgcn_exp2f(-s); }

template <int MODE>
__device__ __forceinline__ float hidden_act(float z) {
  if constexpr (MODE == 0) return softplus_b100<true>(z);
  else return softplus2_scaled(z);
}
template <int MODE>
__device__ __forceinline__ float hidden_dact(float s) {
  if constexpr (MODE == 0) return dsoftplus_b100_from_out<true>(s);
  else return dsoftplus2_scaled_from_out(s);
}

__device__ __forceinline__ float softplus_b1(float x) { return x > 20.0f ? x : log1pf(expf(x)); }

// density activations (models/nerf.py:20-29): 0 shifted_trunc_exp exp(x - 1) whose backward clamps
// the exponent at 15 (external/ngp.py:45-61), 1 softplus(beta 1, threshold 20), 2 shifted_softplus
// softplus(x - 1)
__device__ __forceinline__ float density_act(float raw, int act) {
  if (act == 0) return expf(raw - 1.0f);
  return softplus_b1(act == 2 ? raw - 1.0f : raw);
}
// d sigma / d raw from the output sigma: the clamped exponential, or sigmoid(u) = 1 - exp(-softplus(u))
// (1 past the threshold, where softplus(u) = u > 20)
__device__ __forceinline__ float density_dact_from_out(float sigma, int act) {
  return act == 0 ? fminf(sigma, 3269017.5f /* expf(15) */) : -expm1f(-sigma);
}
// the same from the raw value
__device__ __forceinline__ float density_dact_from_raw(float raw, int act) {
  if (act == 0) return expf(fminf(raw - 1.0f, 15.0f));
  const float u = act == 2 ? raw - 1.0f : raw;
  if (u > 20.0f) return 1.0f;
  const float z = expf(u);
  return __fdiv_rn(z, z + 1.0f);
}

// ------------------------------------------------------------------ exact f32 sampler math
// Mirrors oracle/nerf.py op-for-op (no FMA contraction), so that positions and
// hence encodings are bit-identical to the PyTorch CPU restatement.
struct RayGeom {
  float tmin, span;  // span = 0 for a ray that misses the box
};

__device__ __forceinline__ RayGeom ray_geom(const float* o, const float* d, const float* aabb, float near_p,
                                            float far_p) {
#pragma clang fp contract(off)
  float tmn = -INFINITY, tmx = INFINITY;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float inv = __fdiv_rn(1.0f, d[a]);
    float t1 = (aabb[a] - o[a]) * inv;
    float t2 = (aabb[3 + a] - o[a]) * inv;
    tmn = fmaxf(tmn, fminf(t1, t2));
    tmx = fminf(tmx, fmaxf(t1, t2));
  }
  if (near_p >= 0.0f) tmn = fmaxf(tmn, near_p);
  if (far_p >= 0.0f) tmx = fminf(tmx, far_p);
  // A ray that misses AABB n [near, far] gets zero-length samples at its origin:
  // nerfacc would return no samples at all (C = bkgd, O = D = 0, no gradient),
  // which zero-length samples reproduce, and the MLP never sees the far-away
  // points of a clipped slab intersection (whose raw coordinates enter the
  // positional encoding unbounded).
  RayGeom g;
  const bool hit = tmx > tmn;
  g.tmin = hit ? tmn : 0.0f;
  g.span = hit ? (tmx - tmn) : 0.0f;
  return g;
}

__device__ __forceinline__ void sample_interval(const RayGeom& g, int k, float u, int n, float* t0, float* t1) {
#pragma clang fp contract(off)
  float s = __fdiv_rn((float)k + u, (float)n);
  float mid = g.tmin + s * g.span;
  float half = 0.5f * __fdiv_rn(g.span, (float)n);
  *t0 = mid - half;
  *t1 = mid + half;
}

// Input-space contraction of VanillaNeRFRadianceField.contract_input_space (mlp.py:321-335):
//   type 0 AABB   : x = (p - lo)/(hi - lo)
//   type 1 tanh   : x = (tanh((p - lo)/(hi - lo) - 0.5) + 1)/2          (ngp.py:96-106)
//   type 2 sphere : y = 2(p - lo)/(hi - lo) - 1, |y| > 1 -> (2 - 1/|y|) y/|y|, x = y/4 + 0.5 (ngp.py:68-93)
// then selector = all(0 < x < 1) and x' = 2*pi*(x - 0.5).
enum { CONTRACT_AABB = 0, CONTRACT_TANH = 1, CONTRACT_SPHERE = 2 };

// the contracted position x in [0,1]^3 (for the interior) and the selector; the ngp field
// (ngp.py:230-238) encodes x itself, the mlp field x' = 2 pi (x - 0.5) (contract_point)
__device__ __forceinline__ void contract_unit(const float* pos, const float* aabb, float* x, float* sel,
                                              int type = CONTRACT_AABB) {
#pragma clang fp contract(off)
#pragma unroll
  for (int a = 0; a < 3; ++a) x[a] = __fdiv_rn(pos[a] - aabb[a], aabb[3 + a] - aabb[a]);
  if (type == CONTRACT_SPHERE) {
#pragma unroll
    for (int a = 0; a < 3; ++a) x[a] = x[a] * 2.0f - 1.0f;
    const float mag = __fsqrt_rn(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    if (mag > 1.0f) {
      const float s = 2.0f - __fdiv_rn(1.0f, mag);
#pragma unroll
      for (int a = 0; a < 3; ++a) x[a] = s * __fdiv_rn(x[a], mag);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) x[a] = __fdiv_rn(x[a], 4.0f) + 0.5f;
  } else if (type == CONTRACT_TANH) {
#pragma unroll
    for (int a = 0; a < 3; ++a) x[a] = __fdiv_rn(tanhf(x[a] - 0.5f) + 1.0f, 2.0f);
  }
  bool in = true;
#pragma unroll
  for (int a = 0; a < 3; ++a) in = in && (x[a] > 0.0f) && (x[a] < 1.0f);
  *sel = in ? 1.0f : 0.0f;
}

__device__ __forceinline__ void contract_point(const float* pos, const float* aabb, float* xc, float* sel,
                                               int type = CONTRACT_AABB) {
#pragma clang fp contract(off)
  float x[3];
  contract_unit(pos, aabb, x, sel, type);
#pragma unroll
  for (int a = 0; a < 3; ++a) xc[a] = 6.2831855f * (x[a] - 0.5f);
}

// sample position o + d*(t0 + t1)/2 (external/utils.py:83-87), then the contraction
__device__ __forceinline__ void contract(const float* o, const float* d, float t0, float t1, const float* aabb,
                                         float* xc, float* sel, int type = CONTRACT_AABB) {
#pragma clang fp contract(off)
  const float tt = t0 + t1;
  float pos[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) pos[a] = o[a] + __fdiv_rn(d[a] * tt, 2.0f);
  contract_point(pos, aabb, xc, sel, type);
}

// encoding feature f of [v, sin(v*2^k), sin(v*2^k + pi/2)] (scale-major, dim-minor)
template <bool EXACT>
__device__ __forceinline__ float enc_feature(const float* v, int f, int n_deg) {
#pragma clang fp contract(off)
  const int nd = 3 * n_deg;
  if (f < 3) return v[f];
  if (f < 3 + 2 * nd) {
    int q = f - 3;
    bool cosine = q >= nd;
    if (cosine) q -= nd;
    float xb = v[q % 3] * (float)(1 << (q / 3));
    if (cosine) xb = xb + 1.5707964f;
    if constexpr (EXACT) return sinf(xb);
    else return __sinf(xb);
  }
  return 0.0f;
}

// The render samples' field inputs, shared by the forward and the kernels that recompute the
// encodings instead of reading stored ones (BF16: den_dwstream.hip, den_render.hip's backward).
// Sample s of a render call (den_render_desc.points): 0 the fixed-count stratified sampler (ray
// s / n_samples), 1 a given point, 2 a packed ray-marching sample -> contracted position xc, view
// direction, selector.  AT: any argument struct with the RenderArgs sampler fields.
template <typename AT>
__device__ __forceinline__ void sample_point(const AT& A, const float* aabb, int64_t s, float* xc, float* dir,
                                             float* sel) {
  float o[3];
  if (A.points == 1) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.rays_o[s * 3 + a];
      dir[a] = A.rays_d[s * 3 + a];
    }
    contract_point(o, aabb, xc, sel, A.contraction);
  } else if (A.points == 2) {
    // packed ray-marching samples: position o + d (t0 + t1)/2 of the sample's ray (utils.py:83-87)
    const int64_t r = A.ray_idx[s];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.rays_o[r * 3 + a];
      dir[a] = A.rays_d[r * 3 + a];
    }
    contract(o, dir, A.t_start[s], A.t_end[s], aabb, xc, sel, A.contraction);
  } else {
    const int64_t ray = s / A.n_samples;
    const int k = (int)(s - ray * A.n_samples);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.rays_o[ray * 3 + a];
      dir[a] = A.rays_d[ray * 3 + a];
    }
    const float u = A.jitter[ray];
    RayGeom g = ray_geom(o, dir, aabb, A.near_p, A.far_p);
    float t0, t1;
    sample_interval(g, k, u, A.n_samples, &t0, &t1);
    contract(o, dir, t0, t1, aabb, xc, sel);
  }
}

// the view-encoding input d * pi (mlp.py:353-355)
__device__ __forceinline__ void view_input(const float* dir, float* dv) {
#pragma clang fp contract(off)
#pragma unroll
  for (int a = 0; a < 3; ++a) dv[a] = dir[a] * 3.1415927f;
}

// the sine argument of encoding feature f (f in the sine range), exactly as enc_feature forms it
__device__ __forceinline__ float enc_arg(const float* v, int f, int n_deg) {
#pragma clang fp contract(off)
  const int nd = 3 * n_deg;
  int q = f - 3;
  const bool cosine = q >= nd;
  if (cosine) q -= nd;
  float xb = v[q % 3] * (float)(1 << (q / 3));
  if (cosine) xb = xb + 1.5707964f;
  return xb;
}

// accumulator tile p of the encoding of v (n_deg 10: pe of the position, 4: ve of the view input):
// register r of lane group grp = feature p * TM + acc_row(grp, r), as the forward's fake tiles.
// BF16 (two lane groups): the two groups' features of a register differ by 4 and are compile-time
// constants, so the argument is one select between two constant-index products and ONE sine --
// not a per-lane choice of the coordinate (v[q % 3] with a lane-dependent q), whose lane masks
// filled the forward's scalar registers.  The same values as enc_feature, bit for bit.
// BF16: registers [R0, R0 + R) of enc_tile<1>(v, p, grp, n_deg) into out[0 .. R)
template <int R0, int R>
__device__ __forceinline__ void enc_tile_regs(const float* v, int p, int grp, int n_deg, float* out) {
  const int nd = 3 * n_deg;
  const bool hi = grp != 0;
#pragma unroll
  for (int r = R0; r < R0 + R; ++r) {
    const int f0 = p * 32 + acc_row(1, 0, r), f1 = f0 + 4;
    const bool sin0 = f0 >= 3 && f0 < 3 + 2 * nd, sin1 = f1 >= 3 && f1 < 3 + 2 * nd;
    if (sin0 && sin1) {
      const float x = hi ? enc_arg(v, f1, n_deg) : enc_arg(v, f0, n_deg);
      out[r - R0] = __sinf(x);
    } else {
      out[r - R0] = hi ? enc_feature<false>(v, f1, n_deg) : enc_feature<false>(v, f0, n_deg);
    }
  }
}

template <int MODE>
__device__ __forceinline__ typename Tr<MODE>::Acc enc_tile(const float* v, int p, int grp, int n_deg) {
  typename Tr<MODE>::Acc a;
  if constexpr (MODE == 1) {
    float o[16];
    enc_tile_regs<0, 16>(v, p, grp, n_deg, o);
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = o[r];
  } else {
#pragma unroll
    for (int r = 0; r < Tr<MODE>::REGS; ++r) a[r] = enc_feature<true>(v, p * Tr<MODE>::TM + acc_row(MODE, grp, r), n_deg);
  }
  return a;
}

// ------------------------------------------------------------------ wave primitives
// DPP forms (no LDS round trip): a ds_bpermute shuffle costs an LDS latency per step, and the
// compositing scans chain 20 of them (r05: 39 ds_bpermute in the head backward, all on its adjoint's
// critical path).  dpp_shift: lane l gets v of the source lane the control names, 0 where there is
// none (row_shr / row_shl / wave_shr / wave_shl) or where the row is masked off (row_bcast).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_shift(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
}
__device__ __forceinline__ float wave_readlane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// inclusive prefix sum over the wave: within rows of 16 (row_shr 1, 2, 4, 8), then row 15's total into
// rows 1 and 3 (row_bcast:15) and lane 31's into rows 2 and 3 (row_bcast:31)
__device__ __forceinline__ float wave_incl_scan(float v) {
  v += dpp_shift<0x111>(v);
  v += dpp_shift<0x112>(v);
  v += dpp_shift<0x114>(v);
  v += dpp_shift<0x118>(v);
  v += dpp_shift<0x142, 0xa>(v);
  v += dpp_shift<0x143, 0xc>(v);
  return v;
}
// inclusive suffix sum over the wave (lane l gets the sum over lanes >= l): within rows (row_shl 1, 2,
// 4, 8), then the later rows' totals (lanes 16, 32, 48 after the row pass) added per row -- adds only
__device__ __forceinline__ float wave_incl_suffix(float v) {
  v += dpp_shift<0x101>(v);
  v += dpp_shift<0x102>(v);
  v += dpp_shift<0x104>(v);
  v += dpp_shift<0x108>(v);
  const float t3 = wave_readlane(v, 48), t2 = wave_readlane(v, 32) + t3, t1 = wave_readlane(v, 16) + t2;
  const int row = (threadIdx.x & 63) >> 4;
  return row == 0 ? v + t1 : row == 1 ? v + t2 : row == 2 ? v + t3 : v;
}
// exclusive prefix sum over the wave (lane 0 gets 0); adds only, no incl - v subtraction
__device__ __forceinline__ float wave_excl_scan(float v) { return dpp_shift<0x138>(wave_incl_scan(v)); }  // wave_shr:1
// v of lane l + 1 (lane 63: 0)
__device__ __forceinline__ float wave_next_lane(float v) { return dpp_shift<0x130>(v); }  // wave_shl:1
__device__ __forceinline__ float wave_sum(float v) { return wave_readlane(wave_incl_scan(v), 63); }

// ------------------------------------------------------------------ weight chunk staging
// A chunk (one packed TM-row tile of a layer, <= 20 KiB, a multiple of 1 KiB)
// is copied global -> LDS by LDS-DMA (global_load_lds_dwordx4: each wave moves
// 1 KiB per instruction, lane-linear), issued before the MFMA block of the
// current chunk into the other slot of a 2-slot ring; the barrier that ends
// the chunk also drains the DMA (vmcnt(0)), one barrier per chunk.
constexpr int WG_THREADS = 512;
constexpr int CHUNK_MAX = 64 * 320;  // 20 KiB

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void dma_chunk(const char* g, char* lds_slot, int bytes) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < (CHUNK_MAX + WG_THREADS * 16 - 1) / (WG_THREADS * 16); ++q) {
    const int off = q * WG_THREADS * 16 + wave * 1024;  // wave-uniform
    if (off < bytes)
      __builtin_amdgcn_global_load_lds((const void*)(g + off + lane * 16), (lds_ptr_t)(lds_slot + off), 16, 0, 0);
  }
}

// MFMA block over one LDS chunk: acc += A(chunk) * B(x[0..KS)).
template <int MODE, int KS>
__device__ __forceinline__ void mfma_chunk(const char* lds_chunk, const typename Tr<MODE>::Frag* x,
                                           typename Tr<MODE>::Acc& acc) {
  const int lane = threadIdx.x & 63;
  if constexpr (MODE == 1) {
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      bf16x8 a = *(const bf16x8*)(lds_chunk + k * 1024 + lane * 16);
      acc = Tr<1>::mfma(a, x[k], acc);
    }
  } else {
    static_assert(KS % 4 == 0, "f32 k-steps come in groups of 4");
#pragma unroll
    for (int k4 = 0; k4 < KS / 4; ++k4) {
      f32x4 a = *(const f32x4*)(lds_chunk + k4 * 1024 + lane * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = Tr<0>::mfma(a[q], x[4 * k4 + q], acc);
    }
  }
}

}  // namespace den
