// den_render.hip -- fused render forward / backward-chain kernels for gfx950.
//
// One workgroup = 8 waves = 8 x TN consecutive samples = whole rays
// (TN = 32 samples/wave in BF16 mode, 16 in F32 mode).  Each wave keeps its
// samples' activations in registers as MFMA B-fragments; the packed weights of
// one TM-row tile ("chunk") at a time are streamed through a double-buffered
// LDS ring shared by the 8 waves.
//
// Forward (reference: models/nerf.py:230-286 -> external/utils.py:38-140 ->
// external/mlp.py:321-358 -> external/vol_rendering.py:81-126):
//   sampler -> contraction + positional/view encoding -> L0..L7 (softplus
//   beta=100, skip after L4) -> [bottleneck | sigma] -> rgb hidden -> rgb ->
//   transmittance scan + accumulation + background.
// Backward chain: compositing adjoint (reverse scan) -> dz of every layer
// (written to the workspace for the weight-gradient GEMMs, den_dw.hip) via
// the transposed packed weights.
#include "den_device.h"

namespace den {

constexpr int LDS_BUF = CHUNK_MAX;  // bytes per ring slot

template <int MODE>
struct RenderArgs {
  int n_samples;    // per ray
  int n_rays;
  int rd;
  int train;
  int has_bkgd;
  int points;             // 0 fixed-count sampler, 1 given points, 2 packed samples (ray_idx, t_start, t_end)
  int contraction;        // CONTRACT_* (den_device.h)
  float aabb[6];
  float near_p, far_p;
  const float* rays_o;
  const float* rays_d;
  const float* jitter;
  const int* ray_idx;     // points == 2: per-sample ray index, t_start, t_end (nerfacc packed layout)
  const float* t_start;
  const float* t_end;
  const char* w;          // packed fwd (or bwd) chunks
  const float* bias;      // packed biases (fwd)
  const float* bkgd;
  char* act[NACT];        // activation / dz tensors [n_total][width]
  float* rec;             // per-sample {sigma, rgb0, rgb1, rgb2}
  float* out_rgb;
  float* out_opacity;
  float* out_depth;
  // backward
  const float* d_rgb;
  const float* d_opacity;
  const float* d_depth;
  float* bkgd_partial;    // [4][n_rays]
};

// ------------------------------------------------------------------ helpers

// Base of tile `tile` of activation tensor `a` for the wave that owns `sample` (wave-block major
// layout, den_geom.h); the per-lane offset is added by store_tile_* / load_tile_vals.
template <int MODE>
__device__ __forceinline__ char* act_ptr(const RenderArgs<MODE>& A, int a, int64_t sample, int tile) {
  constexpr int TM = Tr<MODE>::TM, ES = es_of(MODE);
  const int64_t wb = __builtin_amdgcn_readfirstlane((int)(sample / TM));  // uniform across the wave
  return A.act[a] + (wb * (act_width(MODE, a) / TM) + tile) * (int64_t)(TM * TM * ES);
}

// One chunk step of the pipeline: prefetch chunk (t+1), run `body` on chunk t,
// publish chunk t+1 into the other ring slot, barrier.
template <typename Body>
__device__ __forceinline__ void chunk_step(char* lds, const char* wbase, int t, int64_t next_off, int next_bytes,
                                           Body&& body) {
  if (next_bytes > 0) dma_chunk(wbase + next_off, lds + ((t + 1) & 1) * LDS_BUF, next_bytes);
  body(lds + (t & 1) * LDS_BUF);
  __syncthreads();
}

// ---- forward weight ring: FWD_RING slots, chunk t+2 in flight while chunk t is computed.
// The LDS-DMA is issued through inline asm, so the compiler does not track it (tracked, it makes
// the first LDS read of every chunk wait vmcnt(0) -- i.e. for the deeper prefetch and for the
// activation stores too); each step instead waits explicitly for chunk t+1 only:
// vmcnt(<DMA ops of chunk t+2> + <stores of this step>), both issued after chunk t+1's DMA.
#ifndef DEN_FWD_RING
#define DEN_FWD_RING 3
#endif
#ifndef DEN_FWD_STAGGER
#define DEN_FWD_STAGGER 0
#endif
#ifndef DEN_FWD_SETPRIO
#define DEN_FWD_SETPRIO 0
#endif
constexpr int FWD_RING = DEN_FWD_RING;
static_assert(FWD_RING == 2 || FWD_RING == 3, "forward weight ring: 2 or 3 slots");

// BF16 forward workgroup: DEN_FWD_WAVES_BF16 waves (32 samples each) share one weight stream.
// Every workgroup streams the whole packed MLP (1.2 MB) through LDS, so samples per workgroup set
// the L2 -> LDS weight traffic (78 GB per 2^24-sample step at 256 per workgroup).  Measured: 16
// waves (half the weight traffic) take 38.4 ms against 28.0 ms for 8 waves: the 8-wave kernel holds
// 202 VGPRs per wave (one workgroup per CU), and 16 waves per workgroup cap a wave at 128.
#ifndef DEN_FWD_WAVES_BF16
#define DEN_FWD_WAVES_BF16 8
#endif
DEN_HD constexpr int fwd_waves(int mode) { return mode == 1 ? DEN_FWD_WAVES_BF16 : 8; }
DEN_HD constexpr int fwd_threads(int mode) { return 64 * fwd_waves(mode); }
DEN_HD constexpr int fwd_wg_samples(int mode) { return fwd_waves(mode) * tm_of(mode); }
static_assert(FWD_RING == 3 || DEN_FWD_WAVES_BF16 == 8, "the 2-slot ring's tracked DMA assumes 512 threads");

// per-wave count of DMA instructions dma_chunk_untracked<NTH> issues for `bytes` (wave-uniform)
template <int NTH>
__device__ __forceinline__ int dma_ops(int bytes) {
  const int wave = threadIdx.x >> 6;
  int n = 0;
#pragma unroll
  for (int q = 0; q < (CHUNK_MAX + NTH * 16 - 1) / (NTH * 16); ++q) n += (q * NTH * 16 + wave * 1024 < bytes) ? 1 : 0;
  return n;
}

template <int NTH>
__device__ __forceinline__ void dma_chunk_untracked(const char* g, char* lds_slot, int bytes) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < (CHUNK_MAX + NTH * 16 - 1) / (NTH * 16); ++q) {
    // wave-uniform offset (readfirstlane is 32-bit: never pass it a 64-bit pointer)
    const int off = __builtin_amdgcn_readfirstlane(q * NTH * 16 + wave * 1024);
    if (off < bytes) {
      const char* base = g + off;
      const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(lds_slot + off));
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"((uint32_t)lane * 16),
                   "s"(base), "s"(m0) : "memory", "m0");
    }
  }
}

// s_waitcnt vmcnt(VM) lgkmcnt(0) (gfx9 encoding; expcnt left at its maximum)
template <int VM>
__device__ __forceinline__ void wait_vm_lgkm0() {
  static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | ((VM >> 4) << 14));
}
__device__ __forceinline__ void wait_vm_lgkm0_rt(int n) {  // n wave-uniform, 0..7
  switch (n) {
    case 0: wait_vm_lgkm0<0>(); break;
    case 1: wait_vm_lgkm0<1>(); break;
    case 2: wait_vm_lgkm0<2>(); break;
    case 3: wait_vm_lgkm0<3>(); break;
    case 4: wait_vm_lgkm0<4>(); break;
    case 5: wait_vm_lgkm0<5>(); break;
    case 6: wait_vm_lgkm0<6>(); break;
    default: wait_vm_lgkm0<7>(); break;
  }
}

// One forward step: issue chunk t+2 into the slot chunk t-1 used (free since the last barrier),
// run `body` on chunk t (it issues n_st stores), wait for chunk t+1, barrier.
template <int NTH, typename Body>
__device__ __forceinline__ void chunk_step3(char* lds, const char* wbase, int t, int64_t off2, int bytes2, int n_st,
                                            Body&& body) {
  if (bytes2 > 0) dma_chunk_untracked<NTH>(wbase + off2, lds + ((t + 2) % 3) * LDS_BUF, bytes2);
  body(lds + (t % 3) * LDS_BUF);
  wait_vm_lgkm0_rt(dma_ops<NTH>(bytes2) + n_st);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// chunk geometry helpers (forward / backward)
template <int MODE>
__device__ __forceinline__ void fwd_next(int l, int i, int64_t* off, int* bytes) {
  int nl = l, ni = i + 1;
  if (ni >= fwd_tiles(MODE, l)) { nl = l + 1; ni = 0; }
  if (nl >= NL) { *off = 0; *bytes = 0; return; }
  *bytes = chunk_bytes_K(fwd_K(MODE, nl));
  *off = fwd_layer_offset(MODE, nl) + (int64_t)ni * *bytes;
}
// geometry of the chunk two after (l, i)
template <int MODE>
__device__ __forceinline__ void fwd_next2(int l, int i, int64_t* off, int* bytes) {
  int nl = l, ni = i + 1;
  if (ni >= fwd_tiles(MODE, l)) { nl = l + 1; ni = 0; }
  if (nl >= NL) { *off = 0; *bytes = 0; return; }
  fwd_next<MODE>(nl, ni, off, bytes);
}
template <int MODE, int LAST_J>
__device__ __forceinline__ void bwd_next(int j, int i, int64_t* off, int* bytes) {
  int nj = j, ni = i + 1;
  if (ni >= bwd_tiles(MODE, j)) { nj = j + 1; ni = 0; }
  if (nj > LAST_J) { *off = 0; *bytes = 0; return; }
  *bytes = chunk_bytes_K(bwd_K(MODE, nj));
  *off = bwd_layer_offset(MODE, nj) + (int64_t)ni * *bytes;
}

// ------------------------------------------------------------------ forward layer
// Runs all row tiles of forward layer L with input fragments x1[0..KS1) ++ x2[0..KS2).
// EPI: 0 = hidden softplus(100) -> xo (+store act outA), 1 = bottleneck/sigma, 2 = rgb.
// Software pipeline: the VALU epilogue of tile i-1 is issued in the same
// basic block as the MFMA chain of tile i, so the two interleave.
template <int MODE, int L, int EPI, typename Frag, typename Acc>
__device__ __forceinline__ void fwd_epilogue(const RenderArgs<MODE>& A, int64_t sample, Acc& acc, int i, Frag* xo,
                                             int outA, Acc* special) {
  using T = Tr<MODE>;
  constexpr int TM = T::TM, FPT = T::FPT;
  if constexpr (EPI == 0) {
#pragma unroll
    for (int r = 0; r < T::REGS; ++r) acc[r] = hidden_act<MODE>(acc[r]);
    acc_to_frags<MODE>(acc, xo + i * FPT);
  } else if constexpr (EPI == 1) {
    if (i < WIDTH / TM) {
      acc_to_frags<MODE>(acc, xo + i * FPT);
    } else if (i == WIDTH / TM) {
      *special = acc;  // row 0 = sigma_raw (lane group 0, reg 0)
    }
  } else {
    *special = acc;  // rows 0..rd-1 = rgb_raw (lane group 0, regs 0..rd-1)
  }
}

// HBM store of forward tile i (train mode), issued at the START of the chunk interval after
// the one that computed it: the barrier closing an interval drains vmcnt(0) (it must wait for
// the weight DMA), so a store issued there has a whole interval to complete instead of
// stalling that barrier.
template <int MODE, int EPI, typename Frag>
__device__ __forceinline__ void fwd_store(const RenderArgs<MODE>& A, int64_t sample, int i, const Frag* xo,
                                          int outA) {
  constexpr int TM = Tr<MODE>::TM, FPT = Tr<MODE>::FPT;
  if (!A.train) return;
  if constexpr (EPI == 0) {
    store_tile_frags<MODE>(act_ptr(A, outA, sample, i), xo + i * FPT);
  } else if constexpr (EPI == 1) {
    if (i < WIDTH / TM) store_tile_frags<MODE>(act_ptr(A, A_BT, sample, i), xo + i * FPT);
  }
}

template <int MODE, int L, int KS1, int KS2, int EPI, typename Frag, typename Acc>
__device__ __forceinline__ void fwd_layer(const RenderArgs<MODE>& A, char* lds, int64_t sample, const Frag* x1,
                                          const Frag* x2, Frag* xo, int outA, Acc* special) {
  using T = Tr<MODE>;
  constexpr int TM = T::TM;
  constexpr int NT = fwd_tiles(MODE, L);
  constexpr int CB = fwd_chunk_index(MODE, L);
  const int lane = threadIdx.x & 63, grp = lane / TM;
  Acc prev;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    auto body = [&](const char* chunk) {
      if (i >= 2) fwd_store<MODE, EPI>(A, sample, i - 2, xo, outA);
      Acc acc;
      const float* bias = (const float*)(lds + FWD_RING * LDS_BUF) + (CB + i) * TM + grp * T::REGS;
#if DEN_FWD_STAGGER
      // waves 4-7 (each SIMD's second wave) run the epilogue of tile i-1 BEFORE the MFMA chain of
      // tile i, waves 0-3 after it: within a barrier interval the two waves of a SIMD then offer
      // the matrix pipe and the VALU complementary work instead of the same work at once
      const bool late = (threadIdx.x >> 6) >= 4;
      if (late) {
        if (i > 0) fwd_epilogue<MODE, L, EPI>(A, sample, prev, i - 1, xo, outA, special);
        __builtin_amdgcn_sched_barrier(0);
      }
#endif
#pragma unroll
      for (int r = 0; r < T::REGS; ++r) acc[r] = bias[r];
      mfma_chunk<MODE, KS1>(chunk, x1, acc);
      if constexpr (KS2 > 0) mfma_chunk<MODE, KS2>(chunk + KS1 * TM * T::KI * es_of(MODE), x2, acc);
#if DEN_FWD_STAGGER
      if (!late) {
        __builtin_amdgcn_sched_barrier(0);
        if (i > 0) fwd_epilogue<MODE, L, EPI>(A, sample, prev, i - 1, xo, outA, special);
      }
#else
      if (i > 0) fwd_epilogue<MODE, L, EPI>(A, sample, prev, i - 1, xo, outA, special);
#endif
      prev = acc;
    };
    int64_t noff;
    int nbytes;
    if constexpr (FWD_RING == 3) {
      fwd_next2<MODE>(L, i, &noff, &nbytes);
      // stores the body issues: fwd_store of tile i-2 (2 bf16 / 1 f32 instructions per tile)
      const bool st = A.train && i >= 2 && (EPI == 0 || (EPI == 1 && i - 2 < WIDTH / TM));
      chunk_step3<fwd_threads(MODE)>(lds, A.w, CB + i, noff, nbytes, st ? (MODE == 1 ? 2 : 1) : 0, body);
    } else {
      fwd_next<MODE>(L, i, &noff, &nbytes);
      chunk_step(lds, A.w, CB + i, noff, nbytes, body);
    }
  }
  fwd_epilogue<MODE, L, EPI>(A, sample, prev, NT - 1, xo, outA, special);
  if constexpr (NT >= 2) fwd_store<MODE, EPI>(A, sample, NT - 2, xo, outA);
  fwd_store<MODE, EPI>(A, sample, NT - 1, xo, outA);
}

// ------------------------------------------------------------------ forward kernel
template <int MODE>
__global__ __launch_bounds__(fwd_threads(MODE), 1024 / fwd_threads(MODE)) void render_fwd_kernel(RenderArgs<MODE> A) {
  using T = Tr<MODE>;
  using Frag = typename T::Frag;
  using Acc = typename T::Acc;
  constexpr int TM = T::TM, FPT = T::FPT, REGS = T::REGS;
  constexpr bool EXACT = MODE == 0;
  constexpr int WGS = fwd_wg_samples(MODE);
  constexpr int NTH = fwd_threads(MODE);
  constexpr int NBIAS = (int)bias_floats(MODE);
  __shared__ __attribute__((aligned(16))) char lds[FWD_RING * LDS_BUF + NBIAS * 4 + WGS * 16];
  float* bias_lds = (float*)(lds + FWD_RING * LDS_BUF);
  float* rec_lds = bias_lds + NBIAS;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane % TM, grp = lane / TM;
  const int64_t sample = (int64_t)blockIdx.x * WGS + wave * TM + c;
  const int64_t ray = sample / A.n_samples;
#if DEN_FWD_SETPRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half: static priority
#endif
  const int k = (int)(sample - ray * A.n_samples);

  // prologue: whole bias table -> LDS, chunk 0 -> slot 0 (and chunk 1 -> slot 1 with the 3-slot ring)
  for (int q = threadIdx.x; q < NBIAS; q += NTH) bias_lds[q] = A.bias[q];
  if constexpr (FWD_RING == 3) {
    dma_chunk_untracked<NTH>(A.w, lds, chunk_bytes_K(fwd_K(MODE, 0)));
    int64_t off1;
    int bytes1;
    fwd_next<MODE>(0, 0, &off1, &bytes1);
    dma_chunk_untracked<NTH>(A.w + off1, lds + LDS_BUF, bytes1);
  } else {
    dma_chunk(A.w, lds, chunk_bytes_K(fwd_K(MODE, 0)));
  }

  float o[3], d[3], xc[3], sel;
  if (A.points == 1) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.rays_o[sample * 3 + a];
      d[a] = A.rays_d[sample * 3 + a];
    }
    contract_point(o, A.aabb, xc, &sel, A.contraction);
  } else if (A.points == 2) {
    // packed ray-marching samples: position o + d (t0 + t1)/2 of the sample's ray (utils.py:83-87)
    const int64_t r = A.ray_idx[sample];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.rays_o[r * 3 + a];
      d[a] = A.rays_d[r * 3 + a];
    }
    contract(o, d, A.t_start[sample], A.t_end[sample], A.aabb, xc, &sel, A.contraction);
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = A.rays_o[ray * 3 + a];
      d[a] = A.rays_d[ray * 3 + a];
    }
    const float u = A.jitter[ray];
    RayGeom g = ray_geom(o, d, A.aabb, A.near_p, A.far_p);
    float t0, t1;
    sample_interval(g, k, u, A.n_samples, &t0, &t1);
    contract(o, d, t0, t1, A.aabb, xc, &sel);
  }

  // positional encoding as PE_PAD/TM fake accumulator tiles -> fragments
  constexpr int PE_T = PE_PAD / TM;
  Frag pe[PE_T * FPT];
#pragma unroll
  for (int p = 0; p < PE_T; ++p) {
    Acc a;
#pragma unroll
    for (int r = 0; r < REGS; ++r) a[r] = enc_feature<EXACT>(xc, p * TM + acc_row(MODE, grp, r), 10);
    if (A.train) store_tile_vals<MODE>(act_ptr(A, A_PE, sample, p), a);
    acc_to_frags<MODE>(a, pe + p * FPT);
  }
  if constexpr (FWD_RING == 3) wait_vm_lgkm0<0>();  // the untracked prologue DMAs landed
  __syncthreads();

  constexpr int KS = WIDTH / T::KI;  // k-steps of a 256-wide input
  Frag xa[KS], xb[KS];
  Acc sig_acc, rgb_acc;
  fwd_layer<MODE, 0, PE_T * FPT, 0, 0>(A, lds, sample, pe, pe, xa, A_S0 + 0, &sig_acc);
  fwd_layer<MODE, 1, KS, 0, 0>(A, lds, sample, xa, xa, xb, A_S0 + 1, &sig_acc);
  fwd_layer<MODE, 2, KS, 0, 0>(A, lds, sample, xb, xb, xa, A_S0 + 2, &sig_acc);
  fwd_layer<MODE, 3, KS, 0, 0>(A, lds, sample, xa, xa, xb, A_S0 + 3, &sig_acc);
  fwd_layer<MODE, 4, KS, 0, 0>(A, lds, sample, xb, xb, xa, A_S0 + 4, &sig_acc);
  fwd_layer<MODE, 5, KS, PE_T * FPT, 0>(A, lds, sample, xa, pe, xb, A_S0 + 5, &sig_acc);
  fwd_layer<MODE, 6, KS, 0, 0>(A, lds, sample, xb, xb, xa, A_S0 + 6, &sig_acc);
  fwd_layer<MODE, 7, KS, 0, 0>(A, lds, sample, xa, xa, xb, A_S0 + 7, &sig_acc);
  fwd_layer<MODE, L_B, KS, 0, 1>(A, lds, sample, xb, xb, xa, 0, &sig_acc);  // xa <- bottleneck

  // view-direction encoding (mlp.py:353-355): condition * pi, degree 4
  constexpr int VE_T = VE_PAD / TM;
  Frag ve[VE_T * FPT];
  {
#pragma clang fp contract(off)
    float dv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) dv[a] = d[a] * 3.1415927f;
#pragma unroll
    for (int p = 0; p < VE_T; ++p) {
      Acc a;
#pragma unroll
      for (int r = 0; r < REGS; ++r) a[r] = enc_feature<EXACT>(dv, p * TM + acc_row(MODE, grp, r), 4);
      if (A.train) store_tile_vals<MODE>(act_ptr(A, A_VE, sample, p), a);
      acc_to_frags<MODE>(a, ve + p * FPT);
    }
  }
  fwd_layer<MODE, L_G, KS, VE_T * FPT, 0>(A, lds, sample, xa, ve, xb, A_G, &sig_acc);
  fwd_layer<MODE, L_R, WIDTH_COND / T::KI, 0, 2>(A, lds, sample, xb, xb, xa, 0, &rgb_acc);

  // per-sample sigma / rgb (lane group 0 holds rows 0..)
  const int wl = wave * TM + c;  // WG-local sample
  if (grp == 0) {
    // select, not multiply: a sample outside the box (only zero-length samples of missed rays; nerfacc
    // never produces one) must get sigma = 0 even where exp overflows (inf * 0 = NaN)
    float sigma = sel != 0.0f ? expf(sig_acc[0] - 1.0f) : 0.0f;
    float r0 = softplus_b1(rgb_acc[0]);
    float r1 = A.rd > 1 ? softplus_b1(rgb_acc[1]) : 0.0f;
    float r2 = A.rd > 2 ? softplus_b1(rgb_acc[2]) : 0.0f;
    f32x4 v = {sigma, r0, r1, r2};
    *(f32x4*)(rec_lds + wl * 4) = v;
    if (A.train) *(f32x4*)(A.rec + sample * 4) = v;
    if (A.points) {
      A.out_opacity[sample] = sigma;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        if (ch < A.rd) A.out_rgb[sample * A.rd + ch] = v[1 + ch];
    }
  }
  if (A.points) return;
  __syncthreads();

  // compositing: one wave per ray (nerfacc render_weight_from_density +
  // accumulate_along_rays, vol_rendering.py:89-126)
  const int rays_per_wg = WGS / A.n_samples;
  if (wave < rays_per_wg) {
    const int64_t r = (int64_t)blockIdx.x * rays_per_wg + wave;
    float ro[3], rdv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      ro[a] = A.rays_o[r * 3 + a];
      rdv[a] = A.rays_d[r * 3 + a];
    }
    RayGeom rg = ray_geom(ro, rdv, A.aabb, A.near_p, A.far_p);
    const float ru = A.jitter[r];
    const int spl = A.n_samples / 64;  // samples per lane (1, 2 or 4)
    float tau[4], tmid[4], locx[4];
    float run = 0.0f;
    
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      int kk = lane * spl + q;
      float a0, a1;
      sample_interval(rg, kk, ru, A.n_samples, &a0, &a1);
      float sg = rec_lds[(wave * A.n_samples + kk) * 4];
      // zero-length samples (missed rays) contribute nothing, also where sigma overflowed
      tau[q] = (a1 > a0) ? sg * (a1 - a0) : 0.0f;
      tmid[q] = (a0 + a1) / 2.0f;
      locx[q] = run;
      run += tau[q];
    }
    // exclusive optical depth as a sum of the preceding terms only (nerfacc's sequential
    // exclusive cumsum): never incl - tau, which is inf - inf once a sigma overflows
    float base = wave_excl_scan(run);
    float cs[3] = {0.f, 0.f, 0.f}, op = 0.f, dp = 0.f;
    
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      int kk = lane * spl + q;
      float excl = base + locx[q];
      float w = expf(-excl) * (1.0f - expf(-tau[q]));
      const float* rc = rec_lds + (wave * A.n_samples + kk) * 4;
      cs[0] += w * rc[1];
      cs[1] += w * rc[2];
      cs[2] += w * rc[3];
      op += w;
      dp += w * tmid[q];
    }
    op = wave_sum(op);
    dp = wave_sum(dp);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) cs[ch] = wave_sum(cs[ch]);
    if (lane == 0) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        if (ch >= A.rd) break;
        float v = cs[ch];
        if (A.has_bkgd) v = v + A.bkgd[ch] * (1.0f - op);
        A.out_rgb[r * A.rd + ch] = v;
      }
      A.out_opacity[r] = op;
      A.out_depth[r] = dp;
    }
  }
}

// ------------------------------------------------------------------ backward kernel
// Transposed layer j: input dz fragments x[0..KS), output row tiles -> dS of the
// layer's chain inputs; epilogue multiplies by the activation derivative read
// from the stored forward activation (act index SA) and stores dz (index DZ).
// DER: 0 = softplus(100) derivative from stored output, 1 = identity.
// The stored activation of tile i is loaded before tile i's MFMA chain and
// consumed by its epilogue one tile later (software pipeline, as forward).
template <int MODE, int LAST_J, int J, int KS, int DER, typename Frag>
__device__ __forceinline__ void bwd_layer_run(const RenderArgs<MODE>& A, char* lds, int64_t sample, const Frag* x,
                                              Frag* xo, int SA, int DZ) {
  using T = Tr<MODE>;
  using Acc = typename T::Acc;
  constexpr int NT = bwd_tiles(MODE, J);
  constexpr int FPT = T::FPT;
  int cb = 0;
  for (int jj = 0; jj < J; ++jj) cb += bwd_tiles(MODE, jj);
  Acc prev, s_prev, s_cur;
  auto epilogue = [&](Acc& acc, const Acc& sv, int i) {
    if constexpr (DER == 0) {
#pragma unroll
      for (int r = 0; r < T::REGS; ++r) acc[r] = acc[r] * hidden_dact<MODE>(sv[r]);
    }
    acc_to_frags<MODE>(acc, xo + i * FPT);
  };
  // dz stores deferred to the start of the next chunk interval (see fwd_store)
  auto store = [&](int i) { store_tile_frags<MODE>(act_ptr(A, DZ, sample, i), xo + i * FPT); };
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    int64_t noff;
    int nbytes;
    bwd_next<MODE, LAST_J>(J, i, &noff, &nbytes);
    if constexpr (DER == 0) s_cur = load_tile_vals<MODE>(act_ptr(A, SA, sample, i));
    chunk_step(lds, A.w, cb + i, noff, nbytes, [&](const char* chunk) {
      if (i >= 2) store(i - 2);
      Acc acc = acc_zero<MODE>();
      mfma_chunk<MODE, KS>(chunk, x, acc);
      if (i > 0) epilogue(prev, s_prev, i - 1);
      prev = acc;
    });
    s_prev = s_cur;
  }
  epilogue(prev, s_prev, NT - 1);
  if constexpr (NT >= 2) store(NT - 2);
  store(NT - 1);
}

// LAST_J = NBL - 1: the whole chain (F32 parity mode).  LAST_J = 2: stop after Lb^T (writes
// dz_7); the hidden layers then run layer-major in den_hidden.hip (BF16 mode).
template <int MODE, int LAST_J>
__global__ __launch_bounds__(512, 2) void render_bwd_kernel(RenderArgs<MODE> A) {
  using T = Tr<MODE>;
  using Frag = typename T::Frag;
  using Acc = typename T::Acc;
  constexpr int TM = T::TM, FPT = T::FPT, REGS = T::REGS;
  constexpr int WGS = wg_samples(MODE);
  __shared__ __attribute__((aligned(16))) char lds[2 * LDS_BUF + WGS * 16];
  float* rec_lds = (float*)(lds + 2 * LDS_BUF);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane % TM, grp = lane / TM;
  const int64_t sample = (int64_t)blockIdx.x * WGS + wave * TM + c;

  dma_chunk(A.w, lds, chunk_bytes_K(bwd_K(MODE, 0)));

  // ---- compositing adjoint, one wave per ray
  const int rays_per_wg = WGS / A.n_samples;
  if (A.points) {
    // per-point upstream gradients (VanillaNeRFRadianceField.forward outputs)
    if (grp == 0) {
      f32x4 rv = *(const f32x4*)(A.rec + sample * 4);
      float dsig = A.d_opacity ? A.d_opacity[sample] : 0.0f;
      float g3[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        if (ch < A.rd) g3[ch] = A.d_rgb[sample * A.rd + ch];
      f32x4 o4 = {dsig * fminf(rv[0], 3269017.5f), g3[0] * (-expm1f(-rv[1])), g3[1] * (-expm1f(-rv[2])),
                  g3[2] * (-expm1f(-rv[3]))};
      *(f32x4*)(rec_lds + (wave * TM + c) * 4) = o4;
    }
  } else if (wave < rays_per_wg) {
    const int64_t r = (int64_t)blockIdx.x * rays_per_wg + wave;
    float ro[3], rdv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      ro[a] = A.rays_o[r * 3 + a];
      rdv[a] = A.rays_d[r * 3 + a];
    }
    RayGeom rg = ray_geom(ro, rdv, A.aabb, A.near_p, A.far_p);
    const float ru = A.jitter[r];
    const int spl = A.n_samples / 64;
    float dC[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
      if (ch < A.rd) dC[ch] = A.d_rgb[r * A.rd + ch];
    float dO = A.d_opacity ? A.d_opacity[r] : 0.0f;
    const float dD = A.d_depth ? A.d_depth[r] : 0.0f;
    float bk_dot = 0.0f;
    if (A.has_bkgd)
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        if (ch < A.rd) bk_dot += dC[ch] * A.bkgd[ch];
    float tau[4], tmid[4], dlt[4], loc[4], locx[4], sg4[4], rc4[4][3];
    float run = 0.0f;
    
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      int kk = lane * spl + q;
      float a0, a1;
      sample_interval(rg, kk, ru, A.n_samples, &a0, &a1);
      f32x4 rv = *(const f32x4*)(A.rec + (r * A.n_samples + kk) * 4);
      sg4[q] = rv[0];
      rc4[q][0] = rv[1];
      rc4[q][1] = rv[2];
      rc4[q][2] = rv[3];
      dlt[q] = a1 - a0;
      tau[q] = (a1 > a0) ? rv[0] * dlt[q] : 0.0f;
      tmid[q] = (a0 + a1) / 2.0f;
      locx[q] = run;
      run += tau[q];
      loc[q] = run;
    }
    float base = wave_excl_scan(run);
    float w[4], gv[4], op_part = 0.0f;
    float wg_run = 0.0f, wgl[4];
    
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      float excl = base + locx[q];
      w[q] = expf(-excl) * (1.0f - expf(-tau[q]));
      op_part += w[q];
    }
    const float opacity = wave_sum(op_part);
    const float dO_eff = dO - bk_dot;
    
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      gv[q] = dC[0] * rc4[q][0] + dC[1] * rc4[q][1] + dC[2] * rc4[q][2] + dO_eff + dD * tmid[q];
      wg_run += w[q] * gv[q];
      wgl[q] = wg_run;
    }
    // suffix sums of w*g: total - inclusive prefix
    float wg_incl_lane = wave_incl_scan(wg_run);
    float wg_total = __shfl(wg_incl_lane, 63, 64);
    float wg_base = wg_incl_lane - wg_run;
    
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      int kk = lane * spl + q;
      float suffix = wg_total - (wg_base + wgl[q]);  // sum_{j>k} w_j g_j
      float incl = base + loc[q];
      float Tnext = expf(-incl);
      float dtau = Tnext * gv[q] - suffix;
      float dsig = dtau * dlt[q];
      // raw-output gradients: trunc_exp backward clamps at 15 (ngp.py:57-61);
      // softplus(beta=1) derivative sigmoid(x) = 1 - exp(-softplus(x))
      float dsig_raw = dsig * fminf(sg4[q], 3269017.5f /* expf(15) */);
      float v0 = w[q] * dC[0] * (-expm1f(-rc4[q][0]));
      float v1 = w[q] * dC[1] * (-expm1f(-rc4[q][1]));
      float v2 = w[q] * dC[2] * (-expm1f(-rc4[q][2]));
      f32x4 o4 = {dsig_raw, v0, v1, v2};
      *(f32x4*)(rec_lds + (wave * A.n_samples + kk) * 4) = o4;
    }
    if (lane == 0 && A.bkgd_partial) {
      for (int ch = 0; ch < 3; ++ch)
        A.bkgd_partial[(int64_t)ch * A.n_rays + r] = (ch < A.rd && A.has_bkgd) ? dC[ch] * (1.0f - opacity) : 0.0f;
    }
  }
  __syncthreads();

  // ---- fake dz tiles from the per-sample raw gradients
  const int wl = wave * TM + c;
  f32x4 g4 = *(const f32x4*)(rec_lds + wl * 4);
  Acc dzr = acc_zero<MODE>(), dzs = acc_zero<MODE>();
  if (grp == 0) {
    dzr[0] = g4[1];
    if (A.rd > 1) dzr[1] = g4[2];
    if (A.rd > 2) dzr[2] = g4[3];
    dzs[0] = g4[0];
  }
  store_tile_vals<MODE>(act_ptr(A, D_ZR, sample, 0), dzr);
  if constexpr (DZR_W / TM > 1) store_tile_vals<MODE>(act_ptr(A, D_ZR, sample, 1), acc_zero<MODE>());

  constexpr int KS = WIDTH / T::KI;
  Frag fr[FPT];
  acc_to_frags<MODE>(dzr, fr);
  Frag xa[KS + 2 * FPT], xb[KS + 2 * FPT];
  // j=0 Lr^T: dz_r -> dG * softplus'(G) -> DZG (128 rows)
  bwd_layer_run<MODE, LAST_J, 0, FPT, 0>(A, lds, sample, fr, xa, A_G, D_ZG);
  // j=1 Lg^T: dz_g (K=128) -> dBott (identity) -> DZB tiles 0..
  bwd_layer_run<MODE, LAST_J, 1, WIDTH_COND / T::KI, 1>(A, lds, sample, xa, xb, 0, D_ZB);
  // sigma head row(s) of Lb as extra fake tile(s) appended to the DZB fragments
  {
    constexpr int EXTRA_T = (DZB_W - WIDTH) / TM;  // sigma tile + zero padding
#pragma unroll
    for (int e = 0; e < EXTRA_T; ++e) {
      Acc t = e == 0 ? dzs : acc_zero<MODE>();
      store_tile_vals<MODE>(act_ptr(A, D_ZB, sample, WIDTH / TM + e), t);
      if (WIDTH + e * TM < fwd_M(MODE, L_B)) acc_to_frags<MODE>(t, xb + KS + e * FPT);
    }
  }
  // j=2 Lb^T: dz_b (K = fwd_M(Lb)) -> dS7 * softplus'(S7) -> DZ7
  bwd_layer_run<MODE, LAST_J, 2, fwd_M(MODE, L_B) / T::KI, 0>(A, lds, sample, xb, xa, A_S0 + 7, D_Z0 + 7);
  if constexpr (LAST_J > 2) {
    // j=3.. L7^T..L1^T
    bwd_layer_run<MODE, LAST_J, 3, KS, 0>(A, lds, sample, xa, xb, A_S0 + 6, D_Z0 + 6);
    bwd_layer_run<MODE, LAST_J, 4, KS, 0>(A, lds, sample, xb, xa, A_S0 + 5, D_Z0 + 5);
    bwd_layer_run<MODE, LAST_J, 5, KS, 0>(A, lds, sample, xa, xb, A_S0 + 4, D_Z0 + 4);
    bwd_layer_run<MODE, LAST_J, 6, KS, 0>(A, lds, sample, xb, xa, A_S0 + 3, D_Z0 + 3);
    bwd_layer_run<MODE, LAST_J, 7, KS, 0>(A, lds, sample, xa, xb, A_S0 + 2, D_Z0 + 2);
    bwd_layer_run<MODE, LAST_J, 8, KS, 0>(A, lds, sample, xb, xa, A_S0 + 1, D_Z0 + 1);
    bwd_layer_run<MODE, LAST_J, 9, KS, 0>(A, lds, sample, xa, xb, A_S0 + 0, D_Z0 + 0);
  }
}

template __global__ void render_fwd_kernel<0>(RenderArgs<0>);
template __global__ void render_fwd_kernel<1>(RenderArgs<1>);
template __global__ void render_bwd_kernel<0, NBL - 1>(RenderArgs<0>);
template __global__ void render_bwd_kernel<1, NBL - 1>(RenderArgs<1>);
template __global__ void render_bwd_kernel<1, 2>(RenderArgs<1>);

}  // namespace den
