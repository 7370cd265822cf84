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
  float* lr_partial;      // [workgroup][LR_PART]: the fused Lr weight gradient (render_bwd_kernel, LAST_J = 1)
  int64_t n_items;        // forward: 256-sample (BF16) / 128-sample (F32) blocks, walked by a persistent grid
  int density_act;        // den_render_desc.density_activation
  int keep_dzg;           // den_render_desc.ray_grad: the BF16 head backward also stores dz_g (D_ZG)
  int64_t bstride[NACT + 1];  // bytes from one wave block of each activation (and D_ZB8) to the next
  char* sigma_dz;         // layer-major BF16: sigma's dz, one bf16 per sample (den_geom.h D_ZB8)
};

// ------------------------------------------------------------------ helpers

// Base of tile `tile` of activation tensor `a` for the wave that owns `sample` (wave-block major
// layout, den_geom.h); the per-lane offset is added by store_tile_* / load_tile_vals.
template <int MODE, typename AT>
__device__ __forceinline__ char* act_ptr(const AT& A, int a, int64_t sample, int tile) {
  constexpr int TM = Tr<MODE>::TM, ES = es_of(MODE);
  const int64_t wb = __builtin_amdgcn_readfirstlane((int)(sample / TM));  // uniform across the wave
  return A.act[a == D_ZB8 ? D_ZB : a] + wb * A.bstride[a] + tile * (int64_t)(TM * TM * ES);
}

// The backward ring's LDS-DMA through inline asm (untracked: the compiler then does not make the
// chunk's first LDS read wait vmcnt(0) -- i.e. for the DMA of the NEXT chunk, issued just before, and
// every store in flight).  Returns the DMA instructions this wave issued (wave-uniform).
__device__ __forceinline__ int dma_chunk_ut(const char* g, char* lds_slot, int bytes) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < WG_THREADS / 64);
  const uint32_t loff = (uint32_t)(threadIdx.x & 63) * 16;
  int n = 0;
#pragma unroll
  for (int q = 0; q < (CHUNK_MAX + WG_THREADS * 16 - 1) / (WG_THREADS * 16); ++q) {
    const int off = q * WG_THREADS * 16 + wave * 1024;  // wave-uniform
    if (off < bytes) {
      const uint64_t a64 = (uint64_t)(uintptr_t)(g + off);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a64);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a64 >> 32));
      const char* base = (const char*)(uintptr_t)(((uint64_t)hi << 32) | lo);
      const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(lds_slot + off));
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(loff), "s"(base), "s"(m0)
                   : "memory", "m0");
      ++n;
    }
  }
  return n;
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
// The same with the untracked DMA: chunk t+1 is waited for by count -- all but the n_after
// vector-memory ops the body issues after it (vmcnt is in-order) -- so the DMA overlaps the body and
// the stores stay in flight.  n_after must never exceed what the body issues (an under-count only
// waits longer).
// (body returns the vector-memory ops it issued; at most 5 are left in flight.)
template <typename Body>
__device__ __forceinline__ void chunk_step_ut(char* lds, const char* wbase, int t, int64_t next_off, int next_bytes,
                                              Body&& body) {
  if (next_bytes > 0) dma_chunk_ut(wbase + next_off, lds + ((t + 1) & 1) * LDS_BUF, next_bytes);
  const int n_after = body(lds + (t & 1) * LDS_BUF);
  asm volatile("" ::: "memory");
  switch (n_after) {
    case 0: __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (0 << 8)); break;
    case 1: __builtin_amdgcn_s_waitcnt(1 | (7 << 4) | (0 << 8)); break;
    case 2: __builtin_amdgcn_s_waitcnt(2 | (7 << 4) | (0 << 8)); break;
    case 3: __builtin_amdgcn_s_waitcnt(3 | (7 << 4) | (0 << 8)); break;
    case 4: __builtin_amdgcn_s_waitcnt(4 | (7 << 4) | (0 << 8)); break;
    default: __builtin_amdgcn_s_waitcnt(5 | (7 << 4) | (0 << 8)); break;
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- forward weight ring: FWD_RING slots of FWD_G row tiles each; chunks t+1 .. t+FWD_RING-1 are in
// flight while chunk t is computed.  The LDS-DMA is issued through inline asm, so the compiler does
// not track it (tracked, it makes the first LDS read of every chunk wait vmcnt(0) -- i.e. for the
// deeper prefetch and for the activation stores too).  Each step instead waits for chunk t+1 only,
// by count: vmcnt is in-order, so "chunk t+1 landed" = at most <vector-memory ops issued after its
// DMA> outstanding (FwdVm keeps that count).  The activation stores of a step then have FWD_RING - 2
// further chunk intervals to drain before a wait covers them.
//
// The kernel is persistent: one workgroup per CU walks 256-sample blocks ("items", whole rays),
// and the weight stream runs on across items -- the weights are the same for every item, so the
// chunks of the next item's first layer are loaded during the current item's last layers and the
// next item starts on a full ring, with no launch or refill bubble.  The ring slot of a chunk is
// therefore a run-time value (the item's chunk count is not a multiple of FWD_RING).
// Measured (r02/r03 A/B): two row tiles per chunk on a 3-slot ring (one barrier per
// 32 MFMAs), 8 waves of 32 samples (two 32-sample blocks per wave with 4 waves was slower), the
// compiler's instruction order (pinned interleaves were slower), weight fragments read 4 k-steps
// ahead.
constexpr int FWD_G = 2;     // row tiles per forward chunk (one barrier per chunk)
constexpr int FWD_RING = 3;  // ring slots
constexpr int FWD_PF = 4;    // weight fragments read ahead (BF16)
constexpr int FWD_SLOT = FWD_G * CHUNK_MAX;  // bytes per forward ring slot
static_assert(FWD_RING * FWD_SLOT <= 128 * 1024, "forward ring exceeds the LDS budget");
DEN_HD constexpr int fwd_nchunks_l(int mode, int l) { return (fwd_tiles(mode, l) + FWD_G - 1) / FWD_G; }
DEN_HD constexpr int fwd_gchunk_index(int mode, int l) {
  int c = 0;
  for (int i = 0; i < l; ++i) c += fwd_nchunks_l(mode, i);
  return c;
}
DEN_HD constexpr int fwd_item_chunks(int mode) { return fwd_gchunk_index(mode, NL); }

// Forward workgroup: 8 waves x TM samples (BF16: 256 samples) share one weight stream -- every item
// streams the whole packed MLP (1.2 MB) through LDS, so samples per item set the L2 -> LDS weight
// traffic (78 GB per 2^24-sample step at 256 per item).
DEN_HD constexpr int fwd_nb(int mode) { return 1; }
DEN_HD constexpr int fwd_waves(int mode) { return 8; }
DEN_HD constexpr int fwd_threads(int mode) { return 64 * fwd_waves(mode); }
DEN_HD constexpr int fwd_wg_samples(int mode) { return fwd_waves(mode) * fwd_nb(mode) * tm_of(mode); }
DEN_HD constexpr int fwd_min_waves(int mode) { return 2; }  // 256 registers per wave
// LDS layout of the forward: [bias table | per-sample records | weight ring].  With the bias table
// first, a tile's bias reads address it by the 16-bit immediate offset of ds_read (behind the ring,
// at 120 KiB, every tile computed its bias addresses by VALU; r04 ISA budget: -2.7 % issue cycles
// together with the scalar DMA offsets below).
DEN_HD constexpr int fwd_ring_off(int mode) {
  return (int)((bias_floats(mode) * 4 + fwd_wg_samples(mode) * 16 + 1023) / 1024 * 1024);
}
DEN_HD constexpr int fwd_bias_off(int mode) { return 0; }

// wofs: this wave's 1 KiB piece offset, wave * 1024, as a wave-uniform (SGPR) value
template <int NTH>
__device__ __forceinline__ void dma_chunk_untracked(const char* g, char* lds_slot, int bytes, int wofs) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < (FWD_SLOT + NTH * 16 - 1) / (NTH * 16); ++q) {
    // scalar piece offset and LDS address: no per-piece readfirstlane (nor its SGPR hazard)
    const int off = q * NTH * 16 + wofs;
    if (off < bytes) {
      const char* base = g + off;
      const uint32_t m0 = (uint32_t)(uintptr_t)(lds_ptr_t)lds_slot + (uint32_t)off;
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
// n wave-uniform; counts above 15 wait for 15 (stricter than needed, never looser)
__device__ __forceinline__ void wait_vm_lgkm0_rt(int n) {
  switch (n) {
    case 0: wait_vm_lgkm0<0>(); break;
    case 1: wait_vm_lgkm0<1>(); break;
    case 2: wait_vm_lgkm0<2>(); break;
    case 3: wait_vm_lgkm0<3>(); break;
    case 4: wait_vm_lgkm0<4>(); break;
    case 5: wait_vm_lgkm0<5>(); break;
    case 6: wait_vm_lgkm0<6>(); break;
    case 7: wait_vm_lgkm0<7>(); break;
    case 8: wait_vm_lgkm0<8>(); break;
    case 9: wait_vm_lgkm0<9>(); break;
    case 10: wait_vm_lgkm0<10>(); break;
    case 11: wait_vm_lgkm0<11>(); break;
    case 12: wait_vm_lgkm0<12>(); break;
    case 13: wait_vm_lgkm0<13>(); break;
    case 14: wait_vm_lgkm0<14>(); break;
    default: wait_vm_lgkm0<15>(); break;
  }
}

// Vector-memory ops this wave issued in the current item (DMA pieces + global stores), and the
// count right after each of the last FWD_RING - 1 chunk DMAs (hist[0] oldest).  Every value is a
// compile-time constant of the unrolled item body.  A store must be counted here or not at all: an
// uncounted op only makes a wait stricter, an over-count would let the barrier pass before a chunk
// landed.  At an item's start everything issued before it has landed (the item prologue waits),
// so the counts restart at 0.
struct FwdVm {
  int issued;
  int wofs;  // this wave's DMA piece offset (wave * 1024), wave-uniform
  int hist[FWD_RING - 1];
#ifdef DEN_FWD_PROF
  // experiment builds only: cycles in body / vmcnt wait / barrier, kernel start, item prologues,
  // item tails, kernel end, (unused)
  uint64_t prof[8];
#endif
};
#ifdef DEN_FWD_PROF
__device__ uint64_t den_fwd_prof[512 * 8 * 8];
#endif

// One forward step on chunk t (in ring slot `slot`, run-time 0..FWD_RING-1): issue chunk
// t+FWD_RING-1 into the slot chunk t-1 used (free since the last barrier), run `body` on chunk t
// (it issues n_st stores), wait for chunk t+1, barrier.
template <int NTH, int RING_OFF, typename Body>
__device__ __forceinline__ void fwd_step(char* lds, const char* wbase, int slot, int64_t off_n, int bytes_n,
                                         int n_st, FwdVm& vm, Body&& body) {
  constexpr int R = FWD_RING;
#ifdef DEN_FWD_PROF
  const uint64_t p0 = __builtin_amdgcn_s_memtime();
#endif
  const int dst = slot == 0 ? R - 1 : slot - 1;  // (slot + R - 1) % R
  dma_chunk_untracked<NTH>(wbase + off_n, lds + RING_OFF + dst * FWD_SLOT, bytes_n, vm.wofs);
  // the DMA ops EVERY wave issues (some issue one more): an under-count, so the count stays a
  // compile-time constant and each wait an immediate
  vm.issued += bytes_n / (NTH * 16);
#pragma unroll
  for (int k = 0; k + 1 < R - 1; ++k) vm.hist[k] = vm.hist[k + 1];
  vm.hist[R - 2] = vm.issued;
  body(lds + RING_OFF + slot * FWD_SLOT);
#ifdef DEN_FWD_PROF
  const uint64_t p1 = __builtin_amdgcn_s_memtime();
#endif
  vm.issued += n_st;
  // chunk t+1's DMA was issued R-2 steps ago: hist[0]
  wait_vm_lgkm0_rt(vm.issued - vm.hist[0]);
#ifdef DEN_FWD_PROF
  const uint64_t p2 = __builtin_amdgcn_s_memtime();
#endif
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#ifdef DEN_FWD_PROF
  const uint64_t p3 = __builtin_amdgcn_s_memtime();
  vm.prof[0] += p1 - p0;
  vm.prof[1] += p2 - p1;
  vm.prof[2] += p3 - p2;
#endif
}

// geometry of the forward chunk k after chunk c of layer l: FWD_G consecutive row tiles of one
// layer (fewer at a layer's end), contiguous in the packed layout; past the last layer the stream
// wraps to layer 0 (the next item's first chunks)
template <int MODE>
__device__ __forceinline__ void fwd_ahead(int l, int c, int k, int64_t* off, int* bytes) {
#pragma unroll
  for (int s = 0; s < k; ++s) {
    if (++c >= fwd_nchunks_l(MODE, l)) {
      c = 0;
      if (++l == NL) l = 0;
    }
  }
  const int tile = chunk_bytes_K(fwd_K(MODE, l));
  const int left = fwd_tiles(MODE, l) - c * FWD_G;
  *bytes = (left < FWD_G ? left : FWD_G) * tile;
  *off = fwd_layer_offset(MODE, l) + (int64_t)c * FWD_G * tile;
}

// ring slot of the item's chunk `gc` (compile-time) given the slot of its chunk 0 (run-time)
__device__ __forceinline__ int fwd_slot(int slot0, int gc) {
  const int s = slot0 + gc % FWD_RING;
  return s >= FWD_RING ? s - FWD_RING : s;
}

// WRAP (persistent kernels): past the last chunk the stream wraps to chunk 0, the next item's
// W0: layer 0's tiles travel as ONE chunk (the head backward's Lr^T, 4 x 2 KiB)
template <int MODE, int LAST_J, bool WRAP = false, bool W0 = false>
__device__ __forceinline__ void bwd_next(int j, int i, int64_t* off, int* bytes) {
  int nj = j, ni = i + 1;
  if (ni >= bwd_tiles(MODE, j)) { nj = j + 1; ni = 0; }
  if (nj > LAST_J) {
    if (!WRAP) { *off = 0; *bytes = 0; return; }
    nj = 0;
  }
  *bytes = chunk_bytes_K(bwd_K(MODE, nj));
  *off = bwd_layer_offset(MODE, nj) + (int64_t)ni * *bytes;
  if (W0 && nj == 0) *bytes *= bwd_tiles(MODE, 0);
}

// ------------------------------------------------------------------ forward layer
// Fragment arrays are block-major: block b's k-th fragment of an input of stride S is x[b * S + k].
// Runs all row tiles of forward layer L with input fragments x1[0..KS1) ++ x2[0..KS2).
// EPI: 0 = hidden softplus(100) -> xo (+store act outA), 1 = bottleneck/sigma, 2 = rgb.
// The VALU epilogue of tile i-1 is issued in the same basic block as the MFMA chain of tile i
// (TRAIN is a template parameter: no branch splits it), so the two interleave.
struct FwdOut {
  float sigma_raw;   // sigma layer output (lane group 0)
  float rgb_raw[3];  // rgb layer outputs 0..rd-1 (lane group 0)
};

template <int MODE, int L, int EPI, int NB, typename Frag, typename Acc>
__device__ __forceinline__ void fwd_epilogue(Acc* acc, int i, Frag* xo, FwdOut* out) {
  using T = Tr<MODE>;
  constexpr int TM = T::TM, FPT = T::FPT, KS = WIDTH / T::KI;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if constexpr (EPI == 0) {
#pragma unroll
      for (int r = 0; r < T::REGS; ++r) acc[b][r] = hidden_act<MODE>(acc[b][r]);
      acc_to_frags<MODE>(acc[b], xo + b * KS + i * FPT);
    } else if constexpr (EPI == 1) {
      if (i < WIDTH / TM) {
        acc_to_frags<MODE>(acc[b], xo + b * KS + i * FPT);
      } else if (i == WIDTH / TM) {
        out[b].sigma_raw = acc[b][0];  // row 256 = sigma_raw (lane group 0, reg 0)
      }
    } else {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) out[b].rgb_raw[ch] = acc[b][ch];  // rows 0..rd-1 (lane group 0)
    }
  }
}

// HBM store of forward tile i (train mode), issued in the chunk interval after the one that
// computed it, so that the barrier closing an interval does not wait for it.
template <int MODE, bool TRAIN, int EPI, int NB, typename Frag, typename AT>
__device__ __forceinline__ void fwd_store(const AT& A, const int64_t* sample, int i, const Frag* xo, int outA) {
  constexpr int TM = Tr<MODE>::TM, FPT = Tr<MODE>::FPT, KS = WIDTH / Tr<MODE>::KI;
  if constexpr (!TRAIN) return;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if constexpr (EPI == 0) {
      store_tile_frags<MODE>(act_ptr<MODE>(A, outA, sample[b], i), xo + b * KS + i * FPT);
    } else if constexpr (EPI == 1) {
      if (i < WIDTH / TM) store_tile_frags<MODE>(act_ptr<MODE>(A, A_BT, sample[b], i), xo + b * KS + i * FPT);
    }
  }
}

// global store instructions fwd_store issues for tile i (store_tile_frags: 2 in BF16, 1 in F32)
template <int MODE, bool TRAIN, int EPI, int NB>
__device__ __forceinline__ constexpr int fwd_store_ops(int i) {
  if (!TRAIN) return 0;
  const int per = NB * (MODE == 1 ? 2 : 1);
  if (EPI == 0) return per;
  if (EPI == 1) return i < WIDTH / tm_of(MODE) ? per : 0;
  return 0;
}

// The last row tile's epilogue of layer L and the stores of its last two tiles.
template <int MODE, bool TRAIN, int L, int EPI, int NB, typename Frag, typename Acc, typename AT>
__device__ __forceinline__ void fwd_layer_tail(const AT& A, const int64_t* sample, Acc* last, Frag* xo, int outA,
                                               FwdOut* out) {
  constexpr int NT = fwd_tiles(MODE, L);
  fwd_epilogue<MODE, L, EPI, NB>(last, NT - 1, xo, out);
  if constexpr (NT >= 2) fwd_store<MODE, TRAIN, EPI, NB>(A, sample, NT - 2, xo, outA);
  fwd_store<MODE, TRAIN, EPI, NB>(A, sample, NT - 1, xo, outA);
}
template <int MODE, bool TRAIN, int L, int EPI, int NB>
__device__ __forceinline__ constexpr int fwd_tail_store_ops() {
  constexpr int NT = fwd_tiles(MODE, L);
  return (NT >= 2 ? fwd_store_ops<MODE, TRAIN, EPI, NB>(NT - 2) : 0) + fwd_store_ops<MODE, TRAIN, EPI, NB>(NT - 1);
}

// acc[b] += W_chunk x[b * S + 0 .. KS), b < NB: one LDS read of each weight fragment per NB MFMAs.
// BF16: the weight fragments are read FWD_PF k-steps ahead into a register ring (left alone, the
// compiler issues each read right before its MFMAs and waits out the LDS latency every k-step).
template <int MODE, int K0, int K1, int NB, int S>
__device__ __forceinline__ void mfma_chunk_nb(const char* lds_chunk, const typename Tr<MODE>::Frag* x,
                                              typename Tr<MODE>::Acc* acc) {
  const int lane = threadIdx.x & 63;
  constexpr int KS = K1 - K0;
  if constexpr (KS <= 0) {
    return;
  } else if constexpr (MODE == 1) {
    constexpr int PF = FWD_PF < KS ? FWD_PF : KS;
    // the chunk's LDS address as a run-time VGPR: unrolled, a compile-time slot would be folded into
    // every read's 16-bit offset field, which the third ring slot overflows (r03 A/B: -0.4 ms)
    typedef __attribute__((address_space(3))) const bf16x8 lds_frag_t;
    uint32_t lb = (uint32_t)(uintptr_t)(lds_ptr_t)lds_chunk + (uint32_t)lane * 16u;
    asm volatile("" : "+v"(lb));
    const lds_frag_t* lq = (const lds_frag_t*)(uintptr_t)lb;
    auto rd = [&](int k) -> bf16x8 { return lq[k * 64]; };
    bf16x8 a[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) a[p] = rd(K0 + p);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const bf16x8 cur = a[k % PF];
      if (k + PF < KS) a[k % PF] = rd(K0 + k + PF);
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[b] = Tr<1>::mfma(cur, x[b * S + K0 + k], acc[b]);
    }
  } else {
    static_assert(K0 % 4 == 0 && K1 % 4 == 0, "f32 k-steps come in groups of 4");
#pragma unroll
    for (int k4 = K0 / 4; k4 < K1 / 4; ++k4) {
      const f32x4 a = *(const f32x4*)(lds_chunk + k4 * 1024 + lane * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = Tr<0>::mfma(a[q], x[b * S + 4 * k4 + q], acc[b]);
    }
  }
}

// Layer transitions: the epilogue of a layer's last row tile (and its last two tile stores) does not
// run on its own between two layers -- every wave would then be in VALU at once, the MFMAs idle.
// With DEFER the layer leaves its last accumulators in `tail`; the next layer runs them (`pend`,
// PEND_ST stores) inside the body of its first tile, between the MFMAs that do not read the last
// input tile (k-steps [0, KS1 - FPT)) and the FPT that do.
struct NoPend {
  __device__ __forceinline__ void operator()() const {}
};

template <int MODE, bool TRAIN, int L, int KS1, int S1, int KS2, int S2, int EPI, int NB, bool DEFER, int PEND_ST,
          typename Frag, typename Acc, typename Pend, typename AT>
__device__ __forceinline__ void fwd_layer(const AT& A, char* lds, int slot0, int grp, const int64_t* sample,
                                          const Frag* x1, const Frag* x2, Frag* xo, int outA, FwdOut* out,
                                          FwdVm& vm, Pend&& pend, Acc* tail) {
  using T = Tr<MODE>;
  constexpr int TM = T::TM, FPT = T::FPT;
  constexpr int NT = fwd_tiles(MODE, L);
  constexpr int CB = fwd_chunk_index(MODE, L);
  constexpr int NC = fwd_nchunks_l(MODE, L);
  constexpr int GB = fwd_gchunk_index(MODE, L);
  constexpr int TILE_BYTES = chunk_bytes_K(fwd_K(MODE, L));
  constexpr int KSPLIT = PEND_ST >= 0 ? KS1 - FPT : KS1;  // PEND_ST < 0: no pending epilogue
  static_assert(KSPLIT >= 0, "pending epilogue split");
  Acc prev[NB];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    auto body = [&](const char* chunk) {
#pragma unroll
      for (int j = 0; j < FWD_G; ++j) {
        const int i = c * FWD_G + j;
        if (i < NT) {
          const char* tile = chunk + j * TILE_BYTES;
          Acc acc[NB];
          const float* bias = (const float*)(lds + fwd_bias_off(MODE)) + (CB + i) * TM + grp * T::REGS;
#pragma unroll
          for (int r = 0; r < T::REGS; ++r) acc[0][r] = bias[r];
#pragma unroll
          for (int b = 1; b < NB; ++b) acc[b] = acc[0];
          if (i == 0 && PEND_ST >= 0) {
            mfma_chunk_nb<MODE, 0, KSPLIT, NB, S1>(tile, x1, acc);
            pend();
            mfma_chunk_nb<MODE, KSPLIT, KS1, NB, S1>(tile, x1, acc);
          } else {
            mfma_chunk_nb<MODE, 0, KS1, NB, S1>(tile, x1, acc);
          }
          if constexpr (KS2 > 0)
            mfma_chunk_nb<MODE, 0, KS2, NB, S2>(tile + KS1 * TM * T::KI * es_of(MODE), x2, acc);
          if (i > 0) fwd_epilogue<MODE, L, EPI, NB>(prev, i - 1, xo, out);
          if (i >= 2) fwd_store<MODE, TRAIN, EPI, NB>(A, sample, i - 2, xo, outA);
#pragma unroll
          for (int b = 0; b < NB; ++b) prev[b] = acc[b];
        }
      }
    };
    int64_t noff;
    int nbytes;
    fwd_ahead<MODE>(L, c, FWD_RING - 1, &noff, &nbytes);
    int n_st = (c == 0 && PEND_ST > 0) ? PEND_ST : 0;
#pragma unroll
    for (int j = 0; j < FWD_G; ++j) {
      const int i = c * FWD_G + j;
      if (i < NT && i >= 2) n_st += fwd_store_ops<MODE, TRAIN, EPI, NB>(i - 2);
    }
    fwd_step<fwd_threads(MODE), fwd_ring_off(MODE)>(lds, A.w, fwd_slot(slot0, GB + c), noff, nbytes, n_st, vm, body);
  }
  if constexpr (DEFER) {
#pragma unroll
    for (int b = 0; b < NB; ++b) tail[b] = prev[b];
  } else {
    fwd_layer_tail<MODE, TRAIN, L, EPI, NB>(A, sample, prev, xo, outA, out);
    vm.issued += fwd_tail_store_ops<MODE, TRAIN, L, EPI, NB>();
  }
}

// ------------------------------------------------------------------ forward kernel
// Compositing of item `item` (fixed-count sampler): one wave per ray, nerfacc
// render_weight_from_density + accumulate_along_rays (vol_rendering.py:89-126), from the item's
// per-sample records in rec_lds.  r05bb: run by waves 0 .. rays_per_wg - 1 in the MIDDLE of the next
// item (between its L_B and L_G layers; rec_lds is rewritten only at that item's end), where the
// older waves of each SIMD pair wait at the chunk barriers for their partners anyway -- at the item
// boundary it sat on the critical path (every wave waited for it at the next item's first barrier).
// The ray data and background by scalar loads: a vector load here would wait out every store and
// ring DMA in flight.
template <int MODE, typename AT>
__device__ __forceinline__ void fwd_composite(const AT& A, const float* rec_lds, int64_t item, int wave, int lane,
                                              const float* aabb) {
  constexpr int WGS = fwd_wg_samples(MODE);
  const int rays_per_wg = WGS / A.n_samples;
  const int64_t r = item * rays_per_wg + __builtin_amdgcn_readfirstlane(wave);
  float ro[3], rdv[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    ro[a] = ld_uniform(A.rays_o + r * 3 + a);
    rdv[a] = ld_uniform(A.rays_d + r * 3 + a);
  }
  RayGeom rg = ray_geom(ro, rdv, aabb, A.near_p, A.far_p);
  const float ru = ld_uniform(A.jitter + r);
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
  // exclusive optical depth as a sum of the preceding terms only (nerfacc's sequential exclusive
  // cumsum): never incl - tau, which is inf - inf once a sigma overflows
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
      if (A.has_bkgd) v = v + ld_uniform(A.bkgd + ch) * (1.0f - op);
      A.out_rgb[r * A.rd + ch] = v;
    }
    A.out_opacity[r] = op;
    A.out_depth[r] = dp;
  }
}

template <int MODE, bool TRAIN>
DEN_CODE_ALIGN  // page-aligned code (r04y A/B)
__global__ __launch_bounds__(fwd_threads(MODE), fwd_min_waves(MODE)) void render_fwd_kernel(RenderArgs<MODE> A0) {
  using T = Tr<MODE>;
  using Frag = typename T::Frag;
  using Acc = typename T::Acc;
  constexpr int TM = T::TM, FPT = T::FPT, REGS = T::REGS;
  constexpr bool EXACT = MODE == 0;
  constexpr int NB = fwd_nb(MODE);
  constexpr int WGS = fwd_wg_samples(MODE);
  constexpr int NTH = fwd_threads(MODE);
  constexpr int NBIAS = (int)bias_floats(MODE);
  constexpr int NCH = fwd_item_chunks(MODE);
  __shared__ __attribute__((aligned(1024))) char lds[fwd_ring_off(MODE) + FWD_RING * FWD_SLOT];
  float* bias_lds = (float*)(lds + fwd_bias_off(MODE));
  float* rec_lds = bias_lds + NBIAS;

  const int wave = threadIdx.x >> 6;
  DEN_CLOCK_BEGIN();
#ifdef DEN_FWD_PROF
  uint64_t prof[8] = {0, 0, 0, __builtin_amdgcn_s_memtime(), 0, 0, 0, 0};
#endif

  // once per workgroup: the bias table -> LDS, the first item's chunks 0 .. FWD_RING-2 -> slots
  // 0 .. FWD_RING-2 (later items find theirs loaded by the previous item's last steps)
  for (int q = threadIdx.x; q < NBIAS; q += NTH) bias_lds[q] = A0.bias[q];
#pragma unroll
  for (int ch = 0; ch < FWD_RING - 1; ++ch) {
    int64_t off_c;
    int bytes_c;
    fwd_ahead<MODE>(0, 0, ch, &off_c, &bytes_c);
    dma_chunk_untracked<NTH>(A0.w + off_c, lds + fwd_ring_off(MODE) + ch * FWD_SLOT, bytes_c, __builtin_amdgcn_readfirstlane(wave * 1024));
  }
  int slot0 = 0;  // ring slot of the current item's chunk 0

  for (int64_t item = blockIdx.x; item < A0.n_items; item += gridDim.x) {
    // the arguments re-read from the kernarg segment in every item: through a pointer the compiler
    // cannot prove loop-invariant, so it does not hoist ~30 argument words out of the loop and keep
    // them live (in SGPRs, then spilled into VGPRs) across the whole item
    typedef __attribute__((address_space(4))) const RenderArgs<MODE> KArgs;
    KArgs* Ap = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();  // A0 is the kernel's only argument
    asm volatile("" : "+s"(Ap));
    KArgs& A = *Ap;
    // lane-derived values recomputed per item from an opaque copy of the thread index: hoisted out
    // of the loop, the per-lane LDS addresses of every bias read and encoding row stay live across
    // the item and spill
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, c = lane % TM, grp = lane / TM;
    float aabb[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) aabb[q] = A.aabb[q];
#ifdef DEN_FWD_PROF
    const uint64_t q0 = __builtin_amdgcn_s_memtime();
#endif
    int64_t sample[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) sample[b] = item * WGS + (wave * NB + b) * TM + c;
    FwdVm vm;
    vm.issued = 0;
    vm.wofs = __builtin_amdgcn_readfirstlane((tid >> 6) * 1024);
#pragma unroll
    for (int k = 0; k < FWD_RING - 1; ++k) vm.hist[k] = 0;
#ifdef DEN_FWD_PROF
#pragma unroll
    for (int q = 0; q < 8; ++q) vm.prof[q] = 0;
#endif

    // sample positions -> positional encoding as PE_PAD/TM fake accumulator tiles -> fragments.
    // pe is kept for the backward (the streamed L0 / L5-pe weight gradient reads it: den_dwstream.hip
    // on recomputing it instead); ve only in F32 mode (the BF16 head backward recomputes its tile)
    constexpr bool STORE_PE = TRAIN, STORE_VE = TRAIN && MODE == 0;
    constexpr int PE_T = PE_PAD / TM, PE_S = PE_T * FPT;
    float dir[NB][3], sel[NB];
    Frag pe[NB * PE_S];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float o[3], xc[3];
      if (A.points == 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          o[a] = A.rays_o[sample[b] * 3 + a];
          dir[b][a] = A.rays_d[sample[b] * 3 + a];
        }
        contract_point(o, aabb, xc, &sel[b], A.contraction);
      } else if (A.points == 2) {
        const int64_t r = A.ray_idx[sample[b]];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          o[a] = A.rays_o[r * 3 + a];
          dir[b][a] = A.rays_d[r * 3 + a];
        }
        contract(o, dir[b], A.t_start[sample[b]], A.t_end[sample[b]], aabb, xc, &sel[b], A.contraction);
      } else {
        const int64_t ray = sample[b] / A.n_samples;
        const int k = (int)(sample[b] - ray * A.n_samples);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          o[a] = A.rays_o[ray * 3 + a];
          dir[b][a] = A.rays_d[ray * 3 + a];
        }
        const float u = A.jitter[ray];
        RayGeom g = ray_geom(o, dir[b], aabb, A.near_p, A.far_p);
        float t0, t1;
        sample_interval(g, k, u, A.n_samples, &t0, &t1);
        contract(o, dir[b], t0, t1, aabb, xc, &sel[b]);
      }
#pragma unroll
      for (int p = 0; p < PE_T; ++p) {
        const Acc a = enc_tile<MODE>(xc, p, grp, 10);
        if (STORE_PE) store_tile_vals<MODE>(act_ptr<MODE>(A, A_PE, sample[b], p), a);
        acc_to_frags<MODE>(a, pe + b * PE_S + p * FPT);
      }
    }
    // the item's first chunks landed (their DMAs: the prologue, or the previous item's last steps);
    // the pe stores (the youngest vector-memory ops) may stay in flight -- vmcnt is in-order, so
    // waiting for all but them covers the DMAs (older ops left in flight only make the later counted
    // waits stricter)
    // the pe fragments are complete here: without this (or the stores of the F32 forward) the
    // compiler sinks the encoding into layer 0's schedule, whose lane masks then spill (the BF16
    // inference forward did, 52 SGPRs + 27 VGPRs, before r05)
#pragma unroll
    for (int q = 0; q < NB * PE_S; ++q) asm volatile("" : "+v"(pe[q]));
    constexpr int PE_ST = STORE_PE ? NB * PE_T * (MODE == 1 ? 2 : 1) : 0;
    static_assert(PE_ST < 64, "vmcnt is 6 bits");
    wait_vm_lgkm0<PE_ST>();
    __syncthreads();
#ifdef DEN_FWD_PROF
    prof[4] += __builtin_amdgcn_s_memtime() - q0;
#endif

    constexpr int KS = WIDTH / T::KI;  // k-steps of a 256-wide input
    Frag xa[NB * KS], xb[NB * KS];
    FwdOut out[NB];
    Acc tl[NB];  // last row tile of the previous layer, finished inside the next one (fwd_layer DEFER)
    // the previous layer's tail, run by the next layer inside its first tile (xo: where it writes)
#define DEN_PEND(LP, EPIP, XO, OUTA) \
  [&]() { fwd_layer_tail<MODE, TRAIN, LP, EPIP, NB>(A, sample, tl, XO, OUTA, out); }
#define DEN_PST(LP, EPIP) fwd_tail_store_ops<MODE, TRAIN, LP, EPIP, NB>()
    fwd_layer<MODE, TRAIN, 0, PE_S, PE_S, 0, 0, 0, NB, true, -1>(A, lds, slot0, grp, sample, pe, pe, xa, A_S0 + 0, out,
                                                                 vm, NoPend{}, tl);
    fwd_layer<MODE, TRAIN, 1, KS, KS, 0, 0, 0, NB, true, DEN_PST(0, 0)>(A, lds, slot0, grp, sample, xa, xa, xb, A_S0 + 1,
                                                                        out, vm, DEN_PEND(0, 0, xa, A_S0 + 0), tl);
    fwd_layer<MODE, TRAIN, 2, KS, KS, 0, 0, 0, NB, true, DEN_PST(1, 0)>(A, lds, slot0, grp, sample, xb, xb, xa, A_S0 + 2,
                                                                        out, vm, DEN_PEND(1, 0, xb, A_S0 + 1), tl);
    fwd_layer<MODE, TRAIN, 3, KS, KS, 0, 0, 0, NB, true, DEN_PST(2, 0)>(A, lds, slot0, grp, sample, xa, xa, xb, A_S0 + 3,
                                                                        out, vm, DEN_PEND(2, 0, xa, A_S0 + 2), tl);
    fwd_layer<MODE, TRAIN, 4, KS, KS, 0, 0, 0, NB, true, DEN_PST(3, 0)>(A, lds, slot0, grp, sample, xb, xb, xa, A_S0 + 4,
                                                                        out, vm, DEN_PEND(3, 0, xb, A_S0 + 3), tl);
    fwd_layer<MODE, TRAIN, 5, KS, KS, PE_S, PE_S, 0, NB, true, DEN_PST(4, 0)>(
        A, lds, slot0, grp, sample, xa, pe, xb, A_S0 + 5, out, vm, DEN_PEND(4, 0, xa, A_S0 + 4), tl);
    fwd_layer<MODE, TRAIN, 6, KS, KS, 0, 0, 0, NB, true, DEN_PST(5, 0)>(A, lds, slot0, grp, sample, xb, xb, xa, A_S0 + 6,
                                                                        out, vm, DEN_PEND(5, 0, xb, A_S0 + 5), tl);
    fwd_layer<MODE, TRAIN, 7, KS, KS, 0, 0, 0, NB, true, DEN_PST(6, 0)>(A, lds, slot0, grp, sample, xa, xa, xb, A_S0 + 7,
                                                                        out, vm, DEN_PEND(6, 0, xa, A_S0 + 6), tl);
    // xa <- bottleneck; its tail (the sigma row tile) runs inside L_G
    fwd_layer<MODE, TRAIN, L_B, KS, KS, 0, 0, 1, NB, true, DEN_PST(7, 0)>(A, lds, slot0, grp, sample, xb, xb, xa, 0, out,
                                                                          vm, DEN_PEND(7, 0, xb, A_S0 + 7), tl);

    // view-direction encoding (mlp.py:353-355): condition * pi, degree 4
    constexpr int VE_T = VE_PAD / TM, VE_S = VE_T * FPT;
    Frag ve[NB * VE_S];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float dv[3];
      view_input(dir[b], dv);
#pragma unroll
      for (int p = 0; p < VE_T; ++p) {
        const Acc a = enc_tile<MODE>(dv, p, grp, 4);
        if (STORE_VE) {
          store_tile_vals<MODE>(act_ptr<MODE>(A, A_VE, sample[b], p), a);
          vm.issued += MODE == 1 ? 2 : 1;
        }
        acc_to_frags<MODE>(a, ve + b * VE_S + p * FPT);
      }
    }
    // the previous item's compositing (fwd_composite)
    if (!A.points && item >= (int64_t)gridDim.x && wave < WGS / A.n_samples)
      fwd_composite<MODE>(A, rec_lds, item - gridDim.x, wave, lane, aabb);
    fwd_layer<MODE, TRAIN, L_G, KS, KS, VE_S, VE_S, 0, NB, true, DEN_PST(L_B, 1)>(
        A, lds, slot0, grp, sample, xa, ve, xb, A_G, out, vm, DEN_PEND(L_B, 1, xa, 0), tl);
    fwd_layer<MODE, TRAIN, L_R, WIDTH_COND / T::KI, KS, 0, 0, 2, NB, false, DEN_PST(L_G, 0)>(
        A, lds, slot0, grp, sample, xb, xb, xa, 0, out, vm, DEN_PEND(L_G, 0, xb, A_G), tl);
#undef DEN_PEND
#undef DEN_PST
#ifdef DEN_FWD_PROF
#pragma unroll
    for (int q = 0; q < 3; ++q) prof[q] += vm.prof[q];
    const uint64_t q1 = __builtin_amdgcn_s_memtime();
#endif
    slot0 = fwd_slot(slot0, NCH);  // the next item's chunk 0 follows this item's last chunk

    // per-sample sigma / rgb (lane group 0 holds rows 0..)
    if (grp == 0) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int wl = (wave * NB + b) * TM + c;  // WG-local sample
        // select, not multiply: a sample outside the box (only zero-length samples of missed rays;
        // nerfacc never produces one) must get sigma = 0 even where exp overflows (inf * 0 = NaN)
        float sigma = sel[b] != 0.0f ? density_act(out[b].sigma_raw, A.density_act) : 0.0f;
        float r0 = softplus_b1(out[b].rgb_raw[0]);
        float r1 = A.rd > 1 ? softplus_b1(out[b].rgb_raw[1]) : 0.0f;
        float r2 = A.rd > 2 ? softplus_b1(out[b].rgb_raw[2]) : 0.0f;
        f32x4 v = {sigma, r0, r1, r2};
        *(f32x4*)(rec_lds + wl * 4) = v;
        if (TRAIN) *(f32x4*)(A.rec + sample[b] * 4) = v;
        if (A.points) {
          A.out_opacity[sample[b]] = sigma;
#pragma unroll
          for (int ch = 0; ch < 3; ++ch)
            if (ch < A.rd) A.out_rgb[sample[b] * A.rd + ch] = v[1 + ch];
        }
      }
    }
#ifdef DEN_FWD_PROF
    prof[7] += __builtin_amdgcn_s_memtime() - q1;  // the per-sample outputs of the tail
#endif
    // (points = 0: this item is composited by waves 0 .. rays_per_wg - 1 in the middle of the next
    // item, or after the loop for the last one -- fwd_composite)
#ifdef DEN_FWD_PROF
    prof[5] += __builtin_amdgcn_s_memtime() - q1;
#endif
  }
  // the last item's compositing (its records: every wave's, published by this barrier)
  if (!A0.points && (int64_t)blockIdx.x < A0.n_items) {
    __syncthreads();
    if (wave < WGS / A0.n_samples) {
      const int64_t last = blockIdx.x + (A0.n_items - 1 - blockIdx.x) / gridDim.x * gridDim.x;
      int tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      float aabb[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) aabb[q] = A0.aabb[q];
      fwd_composite<MODE>(A0, rec_lds, last, wave, tid & 63, aabb);
    }
  }
  // the last item's steps prefetched chunks of an item that does not exist: let those DMAs land
  // before the workgroup (and its LDS) goes away
  wait_vm_lgkm0<0>();
  if constexpr (MODE == 1 && TRAIN) DEN_CLOCK_END(0);
#ifdef DEN_FWD_PROF
  prof[6] = __builtin_amdgcn_s_memtime();
  if (blockIdx.x < 512 && (threadIdx.x & 63) == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) den_fwd_prof[(blockIdx.x * 8 + wave) * 8 + q] = prof[q];
  }
#endif
}

// ------------------------------------------------------------------ backward kernel
// Transposed layer j: input dz fragments x[0..KS), output row tiles -> dS of the
// layer's chain inputs; epilogue multiplies by the activation derivative read
// from the stored forward activation (act index SA) and stores dz (index DZ).
// DER: 0 = softplus(100) derivative from stored output, 1 = identity.
// The stored activation of tile i is loaded before tile i's MFMA chain and
// consumed by its epilogue one tile later (software pipeline, as forward).
struct NoTileHook {
  template <typename Acc>
  __device__ __forceinline__ void operator()(int, const Acc&) const {}
};
// UT steps: work of step i run after its MFMAs (returns the vector-memory ops it issued)
struct NoStepHook {
  __device__ __forceinline__ int operator()(int) const { return 0; }
};
// DZ < 0: the dz tiles stay in registers only (xo), nothing is stored.
// UT (BF16): the untracked-DMA chunk step, with `shook` run in each step after its MFMAs (DER = 0:
// the activations preloaded, PRE below).
// W0 (with UT): layer 0 travels as one chunk -- J = 0 reads all its tiles from one ring slot with
// no step in between (one wait + barrier after the last tile, for the next layer's first chunk,
// issued at tile 0); J > 0 wraps to the whole layer 0.  t0: the ring index of the layer's first
// chunk (default: its index in a per-item stream of one chunk per tile).
template <int MODE, int LAST_J, int J, int KS, int DER, bool WRAP = false, bool UT = false, bool W0 = false,
          typename AT, typename Frag, typename Hook = NoTileHook, typename StepHook = NoStepHook>
__device__ __forceinline__ void bwd_layer_run(const AT& A, char* lds, int64_t sample, const Frag* x, Frag* xo, int SA,
                                              int DZ, Hook&& hook = Hook{}, StepHook&& shook = StepHook{}, int t0 = -1,
                                              const uint4 (*pre_in)[2] = nullptr) {
  using T = Tr<MODE>;
  using Acc = typename T::Acc;
  constexpr int NT = bwd_tiles(MODE, J);
  constexpr int FPT = T::FPT;
  static_assert(!W0 || UT, "the whole-layer-0 chunk runs on the untracked step");
  int cb = 0;
  for (int jj = 0; jj < J; ++jj) cb += bwd_tiles(MODE, jj);
  if (t0 >= 0) cb = t0;
  Acc prev, s_prev, s_cur;
  // hook(i, stored activation of tile i): run in tile i's epilogue, when the load has landed
  auto epilogue = [&](Acc& acc, const Acc& sv, int i) {
    if constexpr (DER == 0) hook(i, sv);
    if constexpr (DER == 0) {
#pragma unroll
      for (int r = 0; r < T::REGS; ++r) acc[r] = acc[r] * hidden_dact<MODE>(sv[r]);
    }
    acc_to_frags<MODE>(acc, xo + i * FPT);
  };
  // dz stores deferred to the start of the next chunk interval (see fwd_store)
  auto store = [&](int i) {
    if (DZ >= 0) store_tile_frags<MODE>(act_ptr<MODE>(A, DZ, sample, i), xo + i * FPT);
  };
  // UT with DER = 0 (the head's Lr^T chain, 4 tiles): every tile's stored activation is loaded up
  // front, packed (8 dwords per tile, unpacked at its epilogue), so no activation load sits inside the
  // untracked steps (their counted waits would not know it) and the four HBM round trips overlap
  constexpr bool PRE = UT && DER == 0;
  static_assert(!PRE || (MODE == 1 && NT <= 4), "the preloaded activations: BF16, at most 4 tiles");
  // (pre_in: the caller issued these loads itself, earlier)
  uint4 sraw[PRE ? NT : 1][2];
  // (unpacked where its epilogue reads it: the compiler's wait for the load then sits there)
  auto sval = [&](int i) -> Acc {
    Acc a;
    if constexpr (PRE) {
      const uint32_t w[8] = {sraw[i][0].x, sraw[i][0].y, sraw[i][0].z, sraw[i][0].w,
                             sraw[i][1].x, sraw[i][1].y, sraw[i][1].z, sraw[i][1].w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a[2 * q] = __uint_as_float(w[q] << 16);
        a[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
      }
    }
    return a;
  };
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      if (pre_in) {
        sraw[i][0] = pre_in[i][0];
        sraw[i][1] = pre_in[i][1];
      } else {
        const char* p = act_ptr<MODE>(A, SA, sample, i) + (threadIdx.x & 63) * 16;
        sraw[i][0] = ld_stream((const uint4*)p);
        sraw[i][1] = ld_stream((const uint4*)(p + 1024));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    int64_t noff;
    int nbytes;
    if constexpr (W0 && J == 0) {
      // the next layer's first chunk, issued with tile 0
      bwd_next<MODE, LAST_J, WRAP, W0>(J, NT - 1, &noff, &nbytes);
      if (i != 0) nbytes = 0;
    } else {
      bwd_next<MODE, LAST_J, WRAP, W0>(J, i, &noff, &nbytes);
    }
    if constexpr (DER == 0 && !PRE) s_cur = load_tile_vals<MODE>(act_ptr<MODE>(A, SA, sample, i));
    auto body = [&](const char* chunk) {
      if (i >= 2) store(i - 2);
      Acc acc = acc_zero<MODE>();
      mfma_chunk<MODE, KS>(chunk, x, acc);
      if (i > 0) {
        if constexpr (PRE) epilogue(prev, sval(i - 1), i - 1);
        else epilogue(prev, s_prev, i - 1);
      }
      prev = acc;
    };
    if constexpr (UT && W0 && J == 0) {
      if (nbytes > 0) dma_chunk_ut(A.w + noff, lds + ((cb + 1) & 1) * LDS_BUF, nbytes);
      body(lds + (cb & 1) * LDS_BUF + i * chunk_bytes_K(bwd_K(MODE, J)));
      (void)shook(i);
      if (i == NT - 1) {
        // the next layer's first chunk landed (every older op too); the barrier publishes it
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (0 << 8));
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    } else if constexpr (UT) {
      static_assert(MODE == 1, "the untracked step counts the body's stores only (no loads: PRE)");
      // the body's ops after the DMA: store(i - 2), two 1 KiB stores (store_tile_frags), and the
      // step hook's
      chunk_step_ut(lds, A.w, cb + i, noff, nbytes, [&](const char* chunk) -> int {
        body(chunk);
        return ((i >= 2 && DZ >= 0) ? 2 : 0) + shook(i);
      });
    } else {
      chunk_step(lds, A.w, cb + i, noff, nbytes, body);
    }
    if constexpr (!PRE) s_prev = s_cur;
  }
  if constexpr (PRE) epilogue(prev, sval(NT - 1), NT - 1);
  else epilogue(prev, s_prev, NT - 1);
  if constexpr (NT >= 2) store(NT - 2);
  store(NT - 1);
}

// LAST_J = NBL - 1: the whole chain (F32 parity mode).  LAST_J = 2: stop after Lb^T (writes
// dz_7); the hidden layers then run layer-major in den_hidden.hip (BF16 mode).  LAST_J = 1: stop
// after Lg^T (writes dz_b with the sigma tile; Lb^T runs layer-major, den_hidden.hip).
// Fused Lr weight gradient (BF16, LAST_J = 1): dW_r = dz_r^T G over the workgroup's samples by MFMA
// (k = samples, both operands by transposed LDS reads as in den_hidden.hip), instead of a streamed
// launch that re-reads G and dz_r.  Per wave an LDS scratch holds a dz_r tile replicated at stored
// positions 8t + ch (ch < rd) and the current G tile; the A operand of G tile t keeps rows 8t.. only,
// so the four tiles share one accumulator (row 8t + ch, column = G feature of tile t).  The eight
// waves' accumulators are summed in LDS into one partial per workgroup, [tile t][ch][32] + bias[ch]
// (lr_reduce*_kernel, den_dw.hip, reduce them in a fixed order).
constexpr int LRW_SCR = 4096;  // bytes of LDS scratch per wave
constexpr int LR_PART = 388;   // floats per workgroup partial: 4 x 3 x 32 + 3 bias + 1 pad

// ---- compositing adjoint of one item (WGS samples = whole rays), one wave per ray -> the per-sample
// raw-output gradients {d sigma_raw, d rgb_raw} in rec_lds (points: the per-point upstream gradients)
template <int MODE, typename AT>
__device__ __forceinline__ void head_adjoint(const AT& A, float* rec_lds, int64_t item, int64_t sample, int wave,
                                             int lane, int c, int grp) {
  constexpr int TM = Tr<MODE>::TM;
  constexpr int WGS = wg_samples(MODE);
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
      f32x4 o4 = {dsig * density_dact_from_out(rv[0], A.density_act), g3[0] * (-expm1f(-rv[1])), g3[1] * (-expm1f(-rv[2])),
                  g3[2] * (-expm1f(-rv[3]))};
      *(f32x4*)(rec_lds + (wave * TM + c) * 4) = o4;
    }
  } else if (wave < rays_per_wg) {
    const int64_t r = item * rays_per_wg + wave;
    float ro[3], rdv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      ro[a] = A.rays_o[r * 3 + a];
      rdv[a] = A.rays_d[r * 3 + a];
    }
    float aabb[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) aabb[q] = A.aabb[q];
    RayGeom rg = ray_geom(ro, rdv, aabb, A.near_p, A.far_p);
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
    float wg_run = 0.0f, wgq[4];

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
      wgq[q] = w[q] * gv[q];
      wg_run += wgq[q];
    }
    // suffix sums of w*g accumulated back to front (the reverse cumulative sum of torch's autograd of
    // the reference's cumsum): total - prefix cancels to eps * total on the late samples of a
    // saturated ray (den_march.hip composite_bwd_kernel)
    const float wg_suf_incl = wave_incl_suffix(wg_run);            // lanes >= this one
    const float wg_after = wave_next_lane(wg_suf_incl);       // lanes > this one
    float sfx[4] = {0.f, 0.f, 0.f, 0.f}, later = lane < 63 ? wg_after : 0.0f;
#pragma unroll
    for (int q = 3; q >= 0; --q) {
      if (q >= spl) continue;
      sfx[q] = later;
      later += wgq[q];
    }

#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= spl) break;
      int kk = lane * spl + q;
      float suffix = sfx[q];  // sum_{j>k} w_j g_j
      float incl = base + loc[q];
      float Tnext = expf(-incl);
      float dtau = Tnext * gv[q] - suffix;
      float dsig = dtau * dlt[q];
      // raw-output gradients from the outputs: the density activation's (trunc_exp's backward clamps at
      // 15, ngp.py:57-61); softplus(beta=1) derivative sigmoid(x) = 1 - exp(-softplus(x))
      float dsig_raw = dsig * density_dact_from_out(sg4[q], A.density_act);
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
}

template <int MODE, int LAST_J>
// Page-aligned code, as every hot kernel here: the same render_bwd instructions ran 0.1-0.3 ms
// apart at different code addresses (r04u / r04w / r04y same-box A/B, profiles/r04{w,y}_ab.json)
DEN_CODE_ALIGN
__global__ __launch_bounds__(512, 2) void render_bwd_kernel(RenderArgs<MODE> A) {
  using T = Tr<MODE>;
  using Frag = typename T::Frag;
  using Acc = typename T::Acc;
  constexpr int TM = T::TM, FPT = T::FPT, REGS = T::REGS;
  constexpr int WGS = wg_samples(MODE);
  constexpr bool FUSE_LR = MODE == 1 && LAST_J == 1;
  __shared__ __attribute__((aligned(16))) char lds[2 * LDS_BUF + WGS * 16 + (FUSE_LR ? 8 * LRW_SCR : 0)];
  float* rec_lds = (float*)(lds + 2 * LDS_BUF);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane % TM, grp = lane / TM;
  const int64_t sample = (int64_t)blockIdx.x * WGS + wave * TM + c;

  dma_chunk(A.w, lds, chunk_bytes_K(bwd_K(MODE, 0)));

  // ---- compositing adjoint, one wave per ray
  head_adjoint<MODE>(A, rec_lds, blockIdx.x, sample, wave, lane, c, grp);
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
  if constexpr (!FUSE_LR) {
    store_tile_vals<MODE>(act_ptr<MODE>(A, D_ZR, sample, 0), dzr);
    if constexpr (DZR_W / TM > 1) store_tile_vals<MODE>(act_ptr<MODE>(A, D_ZR, sample, 1), acc_zero<MODE>());
  }
  f32x16 lacc;  // FUSE_LR: the shared dW_r accumulator
#pragma unroll
  for (int r = 0; r < 16; ++r) lacc[r] = 0.0f;
  float ldb[3] = {0.f, 0.f, 0.f};
  char* lscr = lds + 2 * LDS_BUF + WGS * 16 + wave * LRW_SCR;
  if constexpr (FUSE_LR) {
    // dz_r (bf16, as the stored D_ZR tile) of sample c at stored positions 8t + ch of every fragment
    const __bf16 z0 = (__bf16)g4[1], z1 = A.rd > 1 ? (__bf16)g4[2] : (__bf16)0.0f,
                 z2 = A.rd > 2 ? (__bf16)g4[3] : (__bf16)0.0f, zz = (__bf16)0.0f;
    const bf16x8 v = {z0, z1, z2, zz, zz, zz, zz, zz};
    *(bf16x8*)(lscr + hb_slot(lane, 0) * 16) = v;
    *(bf16x8*)(lscr + 1024 + hb_slot(lane, 1) * 16) = v;
    if (grp == 0) {
      ldb[0] = (float)z0;
      ldb[1] = (float)z1;
      ldb[2] = (float)z2;
    }
  }
  auto lr_hook = [&](int i, const Acc& sv) {
    if constexpr (FUSE_LR) {
      // G tile i (exactly its stored bf16: sv came from it) into the scratch, then
      // lacc += [dz_r rows 8i..] x G_i over the wave's 32 samples (two k-steps of 16)
      Frag gf[FPT];
      acc_to_frags<MODE>(sv, gf);
      char* gs = lscr + 2048;
      *(bf16x8*)(gs + hb_slot(lane, 0) * 16) = gf[0];
      *(bf16x8*)(gs + 1024 + hb_slot(lane, 1) * 16) = gf[1];
      const bool keep = ((lane & 31) >> 3) == i;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 a = hb_tr_frag(lscr, kk);
        const bf16x8 zero = {};
        a = keep ? a : zero;
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, hb_tr_frag(gs, kk), lacc, 0, 0, 0);
      }
    }
  };

  constexpr int KS = WIDTH / T::KI;
  Frag fr[FPT];
  acc_to_frags<MODE>(dzr, fr);
  Frag xa[KS + 2 * FPT], xb[KS + 2 * FPT];
  // j=0 Lr^T: dz_r -> dG * softplus'(G) -> DZG (128 rows) [+ the fused Lr weight gradient]
  bwd_layer_run<MODE, LAST_J, 0, FPT, 0>(A, lds, sample, fr, xa, A_G, D_ZG, lr_hook);
  // j=1 Lg^T: dz_g (K=128) -> dBott (identity) -> DZB tiles 0..
  bwd_layer_run<MODE, LAST_J, 1, WIDTH_COND / T::KI, 1>(A, lds, sample, xa, xb, 0,
                                                       (MODE == 1 && LAST_J == 1) ? D_ZB8 : D_ZB);
  // sigma head row(s) of Lb as extra fake tile(s) appended to the DZB fragments
  if constexpr (MODE == 1 && LAST_J == 1) {
    // Lb runs layer-major (hidden_bwd_kernel<true>): dz_b as 8-tile blocks, then sigma's dz as one
    // bf16 per sample (D_ZB8 / sigma_dz, den_geom.h)
    if (grp == 0) {
      const int64_t wb = __builtin_amdgcn_readfirstlane((int)(sample / TM));
      *(__bf16*)(A.sigma_dz + wb * 64 + c * 2) = (__bf16)dzs[0];
    }
  } else {
    constexpr int EXTRA_T = (DZB_W - WIDTH) / TM;  // sigma tile + zero padding
#pragma unroll
    for (int e = 0; e < EXTRA_T; ++e) {
      Acc t = e == 0 ? dzs : acc_zero<MODE>();
      store_tile_vals<MODE>(act_ptr<MODE>(A, D_ZB, sample, WIDTH / TM + e), t);
      if (WIDTH + e * TM < fwd_M(MODE, L_B)) acc_to_frags<MODE>(t, xb + KS + e * FPT);
    }
  }
  if constexpr (FUSE_LR) {
    // the eight waves' dW_r (rows 8t + ch = register 4t + ch of lanes 0..31) and bias into one
    // partial, through the weight ring (idle: the last chunk_step issued no DMA and ended in a barrier)
    float* red = (float*)lds;
    if (lane < 32) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) red[wave * LR_PART + (t * 3 + ch) * 32 + lane] = lacc[4 * t + ch];
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float b = wave_sum(ldb[ch]);
      if (lane == 0) red[wave * LR_PART + 384 + ch] = b;
    }
    if (lane == 0) red[wave * LR_PART + 387] = 0.0f;
    __syncthreads();
    for (int e = threadIdx.x; e < LR_PART; e += blockDim.x) {
      float v = red[e];
#pragma unroll
      for (int w = 1; w < 8; ++w) v += red[w * LR_PART + e];
      A.lr_partial[(int64_t)blockIdx.x * LR_PART + e] = v;
    }
  }
  // j=2 Lb^T: dz_b (K = fwd_M(Lb)) -> dS7 * softplus'(S7) -> DZ7
  if constexpr (LAST_J >= 2)
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

// BF16 sample-major backward (bwd_path = 1, the A/B reference path): the pe / ve tiles its split-K
// GEMMs read, written from the samples (the BF16 forward keeps neither); one wave per wave block
__global__ __launch_bounds__(256) void enc_store_kernel(RenderArgs<1> A, int64_t n_blocks) {
  const int64_t wb = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wb >= n_blocks) return;
  const int lane = threadIdx.x & 63;
  const int64_t s = wb * 32 + (lane & 31);
  float aabb[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) aabb[q] = A.aabb[q];
  float xc[3], dir[3], sel, dv[3];
  sample_point(A, aabb, s, xc, dir, &sel);
  view_input(dir, dv);
#pragma unroll
  for (int p = 0; p < PE_PAD / 32; ++p) store_tile_vals<1>(act_ptr<1>(A, A_PE, s, p), enc_tile<1>(xc, p, lane >> 5, 10));
#pragma unroll
  for (int p = 0; p < VE_PAD / 32; ++p) store_tile_vals<1>(act_ptr<1>(A, A_VE, s, p), enc_tile<1>(dv, p, lane >> 5, 4));
}

template __global__ void render_fwd_kernel<0, false>(RenderArgs<0>);
template __global__ void render_fwd_kernel<0, true>(RenderArgs<0>);
template __global__ void render_fwd_kernel<1, false>(RenderArgs<1>);
template __global__ void render_fwd_kernel<1, true>(RenderArgs<1>);
template __global__ void render_bwd_kernel<0, NBL - 1>(RenderArgs<0>);
template __global__ void render_bwd_kernel<1, NBL - 1>(RenderArgs<1>);

}  // namespace den
