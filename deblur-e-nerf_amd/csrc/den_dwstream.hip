// den_dwstream.hip -- weight / bias gradients of the non-hidden layers (BF16 mode), streamed:
//   dW[o][i] = sum_n dz[n][o] x[n][i],  db[o] = sum_n dz[n][o]
// over all ray samples, for the GEMMs the layer-major hidden backward (den_hidden.hip) does not
// cover, fused by shared operand so that every operand byte is read from HBM once:
//   {L0, L5's pe columns}  A = [dz_0 | dz_5] (16 row tiles), B = pe (2 column tiles)
//   Lg                     A = dz_g (4 row tiles), B = [bottleneck | ve] (9 column tiles)
// Layout and machinery as den_hidden.hip: one persistent workgroup per CU sweeps a contiguous
// range of 32-sample wave blocks; the (MT + NT) 2 KiB tiles of a block arrive by untracked LDS-DMA
// DEPTH blocks ahead into an XOR-permuted ring slot (hb_slot: conflict-free transposed reads);
// both MFMA operands have k = samples and are read with ds_read_tr16_b64 (hb_tr_frag).  Each of
// the NW waves owns the output tiles t = w, w + NW, ... of the MT x NT grid in AGPRs for the whole
// launch; bias sums come from the dz operand by VALU.  Each workgroup writes one split-K partial
// [wg][MT][NT + 1][64][16] (dw_reduce_kernel layout) reduced in a fixed order.
//
// Reference: the nn.Linear backward of base.hidden_layers.{0,5} (pe columns), sigma_layer,
// bottleneck_layer, rgb_layer.* (external/mlp.py:99-113, 193-205).
// Included by den_api.hip after den_hidden.hip (hb_slot, hb_tr_frag, hb_wait_vm_lgkm0, HB_TILE).

namespace den {

// waves per workgroup of the streamed weight-gradient launches {L0 + L5 pe} and Lg, and the ring
// shape of the Lg launch (Lb's and Lr's weight gradients come from den_hidden.hip and
// render_bwd_kernel<1, 1>) (r02 / r03 A/B, profiles/r0{2,3}_*experiments.txt: 4 -> 16
// waves took the {L0 + L5 pe} / Lg launches from 13.0 to 10.8 ms per step; U = 4 wave blocks per Lr
// ring step with 3 steps in flight and U = 2 with 2 for Lg, 7.6 -> 6.6 ms)
constexpr int DWS_NW1 = 16, DWS_NW3 = 16;
constexpr int DWS_D3 = 2, DWS_U3 = 2;  // Lg: ring steps in flight, wave blocks per step (26 KiB each)

struct DwStreamArgs {
  const char* a[2];     // dz tensors (wave-block major), row tiles [0, MA) from a[0], [MA, MT) from a[1]
  int a_tiles[2];       // tiles per wave block of each dz tensor
  const char* b[2];     // x tensors, column tiles [0, NB) from b[0], [NB, NT) from b[1] (unused when computed)
  int b_tiles[2];
  float* partial;       // [gridDim.x][MT][NT + 1][64][16]
  int64_t n_blocks;
  int64_t per_wg;
  // the render samples (RenderArgs' sampler fields, sample_point): the encodings recomputed (ENC)
  int points, n_samples, contraction;
  float aabb[6];
  float near_p, far_p;
  const float* rays_o;
  const float* rays_d;
  const float* jitter;
  const int* ray_idx;
  const float* t_start;
  const float* t_end;
};

// A BF16 accumulator tile into LDS where the LDS-DMA of its stored copy would put it (the
// XOR-permuted slots of hb_slot, piece f = registers 8f .. 8f + 7)
__device__ __forceinline__ void lds_tile_store(char* tile, const f32x16& a) {
  bf16x8 f[2];
  acc_to_frags<1>(a, f);
  const int lane = threadIdx.x & 63;
  *(bf16x8*)(tile + hb_slot(lane, 0) * 16) = f[0];
  *(bf16x8*)(tile + 1024 + hb_slot(lane, 1) * 16) = f[1];
}

// ENC bits: 1 = column tiles [0, NB) are the positional encoding (PE_PAD = 2 tiles), 2 = column
// tiles [NB, NT) are the view encoding (VE_PAD = 1 tile) -- computed from the samples' rays into
// the ring slot instead of stored by the forward and read back (192 B per sample each way)
constexpr int ENC_PE = 1, ENC_VE = 2;

// DMA of one 1 KiB piece of tile `t` (fragment f) of a wave block into its ring-slot position
__device__ __forceinline__ void dws_dma_piece(const char* tile_src, char* dst, int f) {
  const int lane = threadIdx.x & 63;
  const uint32_t off = (uint32_t)hb_slot(lane, f) * 16;
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)dst);
  // the 64-bit source as scalars (two readfirstlanes, each through uint32_t: the low word must not
  // sign-extend into the high one): the "s" operand then never lands in VGPRs, whatever the
  // compiler concludes about the uniformity of the address arithmetic around it
  const uint64_t a64 = (uint64_t)(uintptr_t)(tile_src + f * 1024);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a64);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a64 >> 32));
  const char* base = (const char*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"(off), "s"(base), "s"(m0)
               : "memory", "m0");
}

// The fixed-count sampler's encodings (points == 0) are pipelined: the block's ray (o, d, jitter;
// one ray per 32-sample block) arrives by one untracked dword LDS-DMA of wave 0 a ring step ahead of
// the block's tiles, and waves [0, T_ENC) compute the block's encoding tiles from it one iteration
// before its MFMAs -- no global-memory latency on the critical path (r05: computed synchronously
// from global memory inside the fetch, the {L0 + L5 pe} launch took 5.5 ms against 2.9 ms with pe
// stored).  Given points / packed samples (points 1 / 2) keep the synchronous fetch-time path.
__device__ __forceinline__ void dws_dma_ray(const float* src, char* dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" : : "v"(src), "s"(m0) : "memory", "m0");
}
constexpr int DWS_RAY_BYTES = 256;
#ifndef DEN_DWS_EXP
#define DEN_DWS_EXP 0  // experiment builds only (profiles/exp_variants.sh): 1 no encoding, 2 no sampler
#endif  // per ring slot: 64 lanes x 4 B of the ray DMA (lanes 0..6 used)

// U: wave blocks per ring slot (one barrier per U blocks); P.n_blocks / P.per_wg count U-block steps
template <int MA, int MT, int NB, int NT, int NW, int DEPTH, int U = 1, int ENC = 0>
__attribute__((aligned(4096)))  // page-aligned code (r04y A/B)
__global__ __launch_bounds__(64 * NW, 1) void dwstream_kernel(DwStreamArgs P) {
  constexpr int TILES = MT + NT;
  constexpr int BLK = TILES * HB_TILE;              // one wave block's tiles
  constexpr int SLOT = U * BLK;
  constexpr int RING = DEPTH + 1;
  constexpr int T_PE = (ENC & ENC_PE) ? NB : 0;     // computed column tiles: [MT, MT + T_PE) pe,
  constexpr int T_VE = (ENC & ENC_VE) ? NT - NB : 0;  // [MT + NB, MT + NT) ve
  static_assert(!(ENC & ENC_PE) || NB == PE_PAD / 32, "pe is PE_PAD / 32 column tiles");
  static_assert(!(ENC & ENC_VE) || NT - NB == VE_PAD / 32, "ve is VE_PAD / 32 column tiles");
  static_assert(!(ENC & ENC_VE) || !(ENC & ENC_PE), "one encoding per launch");
  constexpr int T_DMA = TILES - T_PE - T_VE;        // stored tiles, fetched by LDS-DMA
  constexpr int T_ENC = T_PE + T_VE;
  static_assert(T_ENC == 0 || U == 1, "the encoding launches step one wave block at a time");
  static_assert(T_ENC <= NW, "one wave per encoding tile");
  constexpr int PIECES = 2 * T_DMA * U;             // 1 KiB DMA pieces per step
  constexpr int TPW = (MT * NT + NW - 1) / NW;      // output tiles per wave
  constexpr int RAY_LDS = T_ENC > 0 ? RING * DWS_RAY_BYTES : 0;
  static_assert(RING * SLOT + RAY_LDS <= 160 * 1024, "ring exceeds the LDS");
  __shared__ __attribute__((aligned(16))) char lds[RING * SLOT + RAY_LDS];
  char* ray_lds = lds + RING * SLOT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR) for the DMA operands
  // readfirstlane hides the range of threadIdx.x >> 6: without it the compiler cannot prove the
  // output-tile guards (t < MT * NT) true, branches around every MFMA and copies the accumulators
  // through each branch (r05: 5.7 ms -> measured below with the range restored)
  __builtin_assume(wave >= 0 && wave < NW);
  const int64_t b0 = (int64_t)blockIdx.x * P.per_wg;
  const int64_t b1 = b0 + P.per_wg < P.n_blocks ? b0 + P.per_wg : P.n_blocks;
  const bool pipe = T_ENC > 0 && P.points == 0 && DEN_DWS_EXP != 3 && DEN_DWS_EXP != 5;  // kernel argument: uniform

  // the encoding tiles of wave block `blk` into ring slot `dst` (waves [0, T_ENC): tile = wave), lane
  // = sample (l & 31), lane group l >> 5, the forward's sampler and enc_tile -- bit-identical to the
  // tiles it would store.  `ray`: the pipelined path's ray in LDS (o, d, jitter), else null (the
  // sampler reads global memory).
  auto encode = [&](int64_t blk, char* dst, const float* ray) __attribute__((always_inline)) {
    if constexpr (T_ENC > 0 && DEN_DWS_EXP != 1 && DEN_DWS_EXP != 5) {
      const int te = wave;
      if (te < T_ENC) {
        // lane-derived values from an opaque copy of the thread index: loop-invariant, the
        // encoding's per-lane-group constants were hoisted out of the block loop and spilled
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int ln = tid & 63;
        const int64_t s = blk * 32 + (ln & 31);
        // the sampler's arguments read here, from the kernarg segment through an opaque pointer:
        // preloaded, the dozen extra argument words stay live in scalar registers across the loop
        typedef __attribute__((address_space(4))) const DwStreamArgs KArgs;
        KArgs* Pp = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();  // P is the kernel's only argument
        asm volatile("" : "+s"(Pp));
        float aabb[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) aabb[q] = Pp->aabb[q];
        float xc[3], dir[3], sel;
        if (ray) {
          // the fixed-count sampler of sample_point with the block's one ray (n_samples is 64, 128
          // or 256: a 32-sample wave block lies within one ray)
          const int64_t s0 = blk * 32;
          const int64_t r = s0 / Pp->n_samples;
          const int k = (int)(s0 - r * Pp->n_samples) + (ln & 31);
          float o[3];
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            o[a] = ray[a];
            dir[a] = ray[3 + a];
          }
#if DEN_DWS_EXP == 2
          for (int a = 0; a < 3; ++a) xc[a] = o[a] + dir[a] * (float)k;
#else
          const RayGeom g = ray_geom(o, dir, aabb, Pp->near_p, Pp->far_p);
          float t0, t1;
          sample_interval(g, k, ray[6], Pp->n_samples, &t0, &t1);
          contract(o, dir, t0, t1, aabb, xc, &sel);
#endif
        } else {
          sample_point(*Pp, aabb, s, xc, dir, &sel);
        }
        f32x16 v;
        float dv[3];
        view_input(dir, dv);
        // the tile index as a compile-time constant (wave-uniform branches): enc_tile's feature
        // indices then fold, with no per-lane coordinate choice
#pragma unroll
        for (int tt = 0; tt < T_ENC; ++tt)
          if (te == tt) v = T_PE ? enc_tile<1>(xc, tt, ln >> 5, 10) : enc_tile<1>(dv, tt, ln >> 5, 4);
        lds_tile_store(dst + (MT + (T_PE ? 0 : NB) + te) * HB_TILE, v);
      }
    }
  };

  // wave 0 (pipelined path): block blk's ray into its ray slot; issued every iteration (the address
  // clamped to the range) so that wave 0's DMA count per iteration stays uniform
  auto ray_dma = [&](int64_t blk) __attribute__((always_inline)) {
    const int64_t bc = blk < b1 ? blk : b1 - 1;
    const int64_t r = bc * 32 / P.n_samples;
    const float* src = lane < 3 ? P.rays_o + r * 3 + lane
                     : lane < 6 ? P.rays_d + r * 3 + (lane - 3)
                     : lane == 6 ? P.jitter + r : P.rays_o + r * 3;
    dws_dma_ray(src, ray_lds + (int)((blk - b0) % RING) * DWS_RAY_BYTES);
  };

  auto fetch = [&](int64_t blk, char* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < (PIECES + NW - 1) / NW; ++q) {
      const int pc = __builtin_amdgcn_readfirstlane(q * NW + wave);
      if (pc < PIECES) {
        const int ub = pc / (2 * T_DMA), tp = pc % (2 * T_DMA);
        const int td = tp >> 1, f = tp & 1;
        const int t = (td >= MT && T_PE) ? td + T_PE : td;  // the stored tiles skip the computed pe range
        const int64_t wb = blk * U + ub;
        const char* src;
        if (t < MA) src = P.a[0] + (wb * P.a_tiles[0] + t) * HB_TILE;
        else if (t < MT) src = P.a[1] + (wb * P.a_tiles[1] + (t - MA)) * HB_TILE;
        else if (t < MT + NB) src = P.b[0] + (wb * P.b_tiles[0] + (t - MT)) * HB_TILE;
        else src = P.b[1] + (wb * P.b_tiles[1] + (t - MT - NB)) * HB_TILE;
        dws_dma_piece(src, dst + ub * BLK + t * 2048 + f * 1024, f);
      }
    }
    if (!pipe) encode(blk, dst, nullptr);  // synchronous (given points / packed samples)
  };
  // DMA instructions this wave issues per block (pieces pc = q * NW + wave < PIECES)
  const bool extra = wave < PIECES % NW;
  constexpr int OPS_LO = PIECES / NW, OPS_HI = OPS_LO + 1;
  // ... plus wave 0's ray DMA on the pipelined path
  const bool ray_wave = pipe && wave == 0;

#pragma unroll
  for (int u = 0; u < DEPTH; ++u)
    if (b0 + u < b1) fetch(b0 + u, lds + u * SLOT);
  if (ray_wave)
#pragma unroll
    for (int u = 0; u <= DEPTH; ++u) ray_dma(b0 + u);

  f32x16 acc[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  float db[(MT + NW - 1) / NW];  // bias partials of the row tiles mt = w, w + NW, ... (column 0 owners)
#pragma unroll
  for (int j = 0; j < (MT + NW - 1) / NW; ++j) db[j] = 0.0f;
  hb_wait_vm_lgkm0<0>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (pipe && b0 < b1) {
    // the first block's encodings (the loop computes block blk + 1's during block blk)
    encode(b0, lds, (const float*)ray_lds);
    hb_wait_vm_lgkm0<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  for (int64_t blk = b0; blk < b1; ++blk) {
    const int u = (int)((blk - b0) % RING);
    if (blk + DEPTH < b1) fetch(blk + DEPTH, lds + ((u + DEPTH) % RING) * SLOT);
    if (ray_wave) ray_dma(blk + DEPTH + 1);
    if (pipe && blk + 1 < b1) {
      const int u1 = (u + 1) % RING;
      encode(blk + 1, lds + u1 * SLOT, (const float*)(ray_lds + u1 * DWS_RAY_BYTES));
    }
#pragma unroll
    for (int ub = 0; ub < U; ++ub) {
    const char* cur = lds + u * SLOT + ub * BLK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int t = wave + j * NW;
        if (t < MT * NT) {
          const int mt = t / NT, nt = t % NT;
          const bf16x8 a = hb_tr_frag(cur + mt * HB_TILE, kk);
          const bf16x8 bb = hb_tr_frag(cur + (MT + nt) * HB_TILE, kk);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc[j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < (MT + NW - 1) / NW; ++j) {
        const int mt = wave + j * NW;
        if (mt < MT) {
          const bf16x8 a = hb_tr_frag(cur + mt * HB_TILE, kk);
#pragma unroll
          for (int e = 0; e < 8; ++e) db[j] += (float)a[e];
        }
      }
    }
    }
    if (blk + DEPTH < b1) {
      if (ray_wave) {
        if (extra) hb_wait_vm_lgkm0<(DEPTH - 1) * (OPS_HI + 1)>();
        else hb_wait_vm_lgkm0<(DEPTH - 1) * (OPS_LO + 1)>();
      } else {
        if (extra) hb_wait_vm_lgkm0<(DEPTH - 1) * OPS_HI>();
        else hb_wait_vm_lgkm0<(DEPTH - 1) * OPS_LO>();
      }
    } else {
      hb_wait_vm_lgkm0<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  // partial of this workgroup: [mt][nt][lane][16], the bias in the ones-tile slot nt = NT
  float* base = P.partial + (int64_t)blockIdx.x * MT * (NT + 1) * 1024;
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + j * NW;
    if (t < MT * NT) {
      float* o = base + ((int64_t)(t / NT) * (NT + 1) + t % NT) * 1024 + lane * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 v = {acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]};
        *(f32x4*)(o + 4 * q) = v;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < (MT + NW - 1) / NW; ++j) {
    const int mt = wave + j * NW;
    if (mt < MT) {
      // lane l holds feature (l & 31) of this row tile (two lane halves: samples 8(l >> 5)..)
      const float bsum = db[j] + __shfl_xor(db[j], 32, 64);
      float* o = base + ((int64_t)mt * (NT + 1) + NT) * 1024;
      // ones-tile slot of row m (column 0; dw_reduce_kernel reads nothing else of this tile):
      // lane 32 ((m >> 2) & 1), register (m & 3) + 4 (m >> 3)
      if (lane < 32) {
        const int m = lane;
        o[(32 * ((m >> 2) & 1)) * 16 + (m & 3) + 4 * (m >> 3)] = bsum;
      }
    }
  }
}

// the launches of a BF16 backward
template __global__ void dwstream_kernel<8, 16, 2, 2, DWS_NW1, 3, 1, ENC_PE>(DwStreamArgs);  // L0 + L5 pe
// (the Lg launch, dwstream_kernel<4, 4, 8, 9, DWS_NW3, DWS_D3, DWS_U3, ENC_VE>, was replaced in r05 by the
// weight gradient fused into render_head_bwd_kernel)

}  // namespace den
