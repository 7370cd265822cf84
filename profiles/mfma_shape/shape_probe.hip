// shape_probe.hip -- diagnostic (guide rule 28): the BF16 forward's layer body in
// the two bf16 MFMA shapes, same output tile per wave, random data, for an A/B by wall and clock.
//
// Body (both shapes): a persistent workgroup of 8 waves per CU (two per SIMD, <= 256 VGPRs), one
// 256 x 256 bf16 weight layer resident in LDS (128 KiB, read as A fragments by ds_read_b128 exactly as
// render_fwd_kernel reads its weight ring), a wave's 32 samples as B fragments in registers, and per
// layer: 8 x 32 output rows = MFMA chain over K = 256, then the scaled softplus epilogue
// (med3 + exp2 + add + log2 + add per element, den_device.h softplus2_scaled) and bf16 packing straight
// into the next layer's B fragments (the accumulators ARE the next B operand, as in the product).
//   SHAPE 32: v_mfma_f32_32x32x16_bf16 -- per 32-row tile 16 MFMAs (k-steps of 16); lane l holds sample
//             l & 31, rows acc_row(1, l >> 5, r) (den_geom.h); chain: k-step 2t + s <- acc regs 8s..8s+7.
//   SHAPE 16: v_mfma_f32_16x16x32_bf16 -- per 32-row block 2 row tiles x 2 sample blocks x 8 k-blocks of
//             32 = 32 MFMAs; lane l holds sample 16 cb + (l & 15), rows 4 (l >> 4) + [0, 4) of each row
//             tile; chain: k-block p of sample block cb <- {row tile 0's 4 values, row tile 1's 4 values}
//             -- a different k-order of the next layer's packed weights, no cross-lane moves.
// The same FLOP, LDS bytes, VALU and registers in both; only the MFMA shape differs.  Each workgroup
// stamps s_memtime / s_memrealtime at its start and end (lane 0 of wave 0, vector stores to a buffer of
// their own) for the clock it held.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

#ifndef SHAPE16_PF
#define SHAPE16_PF 0
#endif

namespace {

constexpr int WAVES = 8;
constexpr int W_BYTES = 256 * 256 * 2;

__device__ __forceinline__ float sp2(float t) {
  return __builtin_amdgcn_fmed3f(t, 0.0f, 3.4028235e38f) +
         __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(-fabsf(t)));
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2 p = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(p, bf16x2));
}

__device__ __forceinline__ bf16x8 pack8(float v0, float v1, float v2, float v3, float v4, float v5, float v6,
                                        float v7) {
  const uint4 u = make_uint4(pack2(v0, v1), pack2(v2, v3), pack2(v4, v5), pack2(v6, v7));
  return __builtin_bit_cast(bf16x8, u);
}

// Both layer bodies are software-pipelined as render_fwd_kernel's: the epilogue of tile (block) t - 1
// sits in the same scheduling region as the MFMA chain of tile t (a sched_barrier closes each region, so
// the compiler interleaves the two but does not hoist later tiles' LDS reads into it).

// one layer, SHAPE 32: 8 row tiles x 16 k-steps; A fragment (tile t, k-step k) at LDS (t * 16 + k) KiB
__device__ __forceinline__ void epi32(const f32x16& acc, bf16x8 (&bout)[16], int t) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
    bout[2 * t + s] = pack8(sp2(acc[8 * s]), sp2(acc[8 * s + 1]), sp2(acc[8 * s + 2]), sp2(acc[8 * s + 3]),
                            sp2(acc[8 * s + 4]), sp2(acc[8 * s + 5]), sp2(acc[8 * s + 6]), sp2(acc[8 * s + 7]));
}
__device__ __forceinline__ void layer32(const char* lds, const bf16x8 (&bin)[16], bf16x8 (&bout)[16], float bias,
                                        int lane) {
  f32x16 prev;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = bias;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const bf16x8 a = *(const bf16x8*)(lds + (t * 16 + k) * 1024 + lane * 16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bin[k], acc, 0, 0, 0);
    }
    if (t > 0) epi32(prev, bout, t - 1);
    __builtin_amdgcn_sched_barrier(0);
    prev = acc;
  }
  epi32(prev, bout, 7);
  __builtin_amdgcn_sched_barrier(0);
}

// one layer, SHAPE 16: 8 blocks of 32 rows x 8 k-blocks; A fragment (row tile 2p + h, k-block kb) at LDS
// ((2p + h) * 8 + kb) KiB; B fragments bin[cb * 8 + kb]
__device__ __forceinline__ void epi16(const f32x4 (&acc)[2][2], bf16x8 (&bout)[16], int p) {
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
    bout[cb * 8 + p] = pack8(sp2(acc[0][cb][0]), sp2(acc[0][cb][1]), sp2(acc[0][cb][2]), sp2(acc[0][cb][3]),
                             sp2(acc[1][cb][0]), sp2(acc[1][cb][1]), sp2(acc[1][cb][2]), sp2(acc[1][cb][3]));
}
__device__ __forceinline__ void layer16(const char* lds, const bf16x8 (&bin)[16], bf16x8 (&bout)[16], float bias,
                                        int lane) {
  f32x4 prev[2][2];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    f32x4 acc[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[h][cb][r] = bias;
#if SHAPE16_PF
    // A fragments one k-block ahead in a second register set (no write to a register an in-flight
    // MFMA still reads: the hazard s_nops of the plain loop)
    bf16x8 a[2][2];
    a[0][0] = *(const bf16x8*)(lds + ((2 * p) * 8) * 1024 + lane * 16);
    a[0][1] = *(const bf16x8*)(lds + ((2 * p + 1) * 8) * 1024 + lane * 16);
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const int c = kb & 1;
      if (kb + 1 < 8) {
        a[c ^ 1][0] = *(const bf16x8*)(lds + ((2 * p) * 8 + kb + 1) * 1024 + lane * 16);
        a[c ^ 1][1] = *(const bf16x8*)(lds + ((2 * p + 1) * 8 + kb + 1) * 1024 + lane * 16);
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[0][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c][0], bin[cb * 8 + kb], acc[0][cb], 0, 0, 0);
        acc[1][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c][1], bin[cb * 8 + kb], acc[1][cb], 0, 0, 0);
      }
    }
#else
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const bf16x8 a0 = *(const bf16x8*)(lds + ((2 * p) * 8 + kb) * 1024 + lane * 16);
      const bf16x8 a1 = *(const bf16x8*)(lds + ((2 * p + 1) * 8 + kb) * 1024 + lane * 16);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[0][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bin[cb * 8 + kb], acc[0][cb], 0, 0, 0);
        acc[1][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bin[cb * 8 + kb], acc[1][cb], 0, 0, 0);
      }
    }
#endif
    if (p > 0) epi16(prev, bout, p - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) prev[h][cb] = acc[h][cb];
  }
  epi16(prev, bout, 7);
  __builtin_amdgcn_sched_barrier(0);
}

template <int SHAPE>
__global__ __launch_bounds__(64 * WAVES, 1) void shape_probe_kernel(const char* w, const bf16x8* b0, float bias_scale,
                                                                    int layers, bf16x8* out, uint64_t* clk) {
  __shared__ __attribute__((aligned(16))) char lds[W_BYTES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int i = threadIdx.x; i < W_BYTES / 16; i += 64 * WAVES) ((uint4*)lds)[i] = ((const uint4*)w)[i];
  __syncthreads();
  bf16x8 x[16], y[16];
  const int64_t gw = (int64_t)blockIdx.x * WAVES + wave;
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = b0[(gw * 16 + k) * 64 + lane];
  const float bias = bias_scale * (float)((lane * 37 + wave * 11) % 17 - 8);
  for (int l = 0; l < layers; l += 2) {
    if constexpr (SHAPE == 32) {
      layer32(lds, x, y, bias, lane);
      layer32(lds, y, x, bias, lane);
    } else {
      layer16(lds, x, y, bias, lane);
      layer16(lds, y, x, bias, lane);
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) out[(gw * 16 + k) * 64 + lane] = x[k];
  if (threadIdx.x == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t* c = clk + (int64_t)blockIdx.x * 4;
    c[0] = t0;
    c[1] = r0;
    c[2] = t1;
    c[3] = r1;
  }
}

}  // namespace

extern "C" int shape_probe_launch(int shape, int grid, const void* w, const void* b0, float bias_scale, int layers,
                                  void* out, void* clk, void* stream) {
  if ((shape != 16 && shape != 32) || grid <= 0 || layers <= 0 || (layers & 1)) return 1;
  hipStream_t s = (hipStream_t)stream;
  if (shape == 32)
    hipLaunchKernelGGL(shape_probe_kernel<32>, dim3(grid), dim3(64 * WAVES), 0, s, (const char*)w,
                       (const bf16x8*)b0, bias_scale, layers, (bf16x8*)out, (uint64_t*)clk);
  else
    hipLaunchKernelGGL(shape_probe_kernel<16>, dim3(grid), dim3(64 * WAVES), 0, s, (const char*)w,
                       (const bf16x8*)b0, bias_scale, layers, (bf16x8*)out, (uint64_t*)clk);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
