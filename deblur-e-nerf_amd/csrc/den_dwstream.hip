// den_dwstream.hip -- weight / bias gradients of the non-hidden layers (BF16 mode), streamed:
//   dW[o][i] = sum_n dz[n][o] x[n][i],  db[o] = sum_n dz[n][o]
// over all ray samples, for the GEMM the layer-major hidden backward (den_hidden.hip) and the
// head backward (den_head_bwd.hip: Lr, Lg) do not cover, fused by shared operand so that every
// operand byte is read from HBM once:
//   {L0, L5's pe columns}  A = [dz_0 | dz_5] (16 row tiles), B = pe (2 column tiles)
// Layout and machinery as den_hidden.hip: one persistent workgroup per CU sweeps a contiguous
// range of 32-sample wave blocks; the (MT + NT) 2 KiB tiles of a block arrive by untracked LDS-DMA
// DEPTH blocks ahead into an XOR-permuted ring slot (hb_slot: conflict-free transposed reads);
// both MFMA operands have k = samples and are read with ds_read_tr16_b64 (hb_tr_frag).  Each of
// the NW waves owns the output tiles t = w, w + NW, ... of the MT x NT grid in AGPRs for the whole
// launch; bias sums come from the dz operand by VALU.  Each workgroup writes one split-K partial
// [wg][MT][NT + 1][64][16] (dw_reduce_kernel layout) reduced in a fixed order.
//
// pe is the forward's stored copy (128 B per sample written, read once here).  r05 measured the
// alternative -- recomputing the two pe tiles per block from the block's ray (sampler + encoding,
// the ray LDS-DMA'd a ring step ahead, the tiles computed an iteration ahead of their MFMAs):
// 3.8 ms against 2.9 ms for the stored copy, whose extra forward store did not move the forward's
// time (23.75 vs 23.65 ms, profiles/gpu_r05r.sh); the encoding waves' VALU work (the sampler's
// divisions, 16 sines per lane) lands on the block step's critical path, and spreading it over more
// waves was slower still (the sampler then runs on every one: 4.8 / 5.1 / 6.6 ms for 2 / 4 / 8
// waves per tile, profiles/r05q).
//
// Reference: the nn.Linear backward of base.hidden_layers.{0,5} (pe columns) (external/mlp.py:99-113).
// Included by den_api.hip after den_hidden.hip (hb_slot, hb_tr_frag, hb_wait_vm_lgkm0, HB_TILE).

namespace den {

// waves per workgroup (r02 / r03 A/B, profiles/r0{2,3}_*experiments.txt: 4 -> 16 waves took the
// streamed launches from 13.0 to 10.8 ms per step)
constexpr int DWS_NW1 = 16;

struct DwStreamArgs {
  const char* a[2];     // dz tensors (wave-block major), row tiles [0, MA) from a[0], [MA, MT) from a[1]
  int64_t a_bs[2];      // bytes from one wave block of each dz tensor to the next
  const char* b[2];     // x tensors, column tiles [0, NB) from b[0], [NB, NT) from b[1]
  int64_t b_bs[2];
  float* partial;       // [gridDim.x][MT][NT + 1][64][16]
  int64_t n_blocks;
  int64_t per_wg;
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

// U: wave blocks per ring slot (one barrier per U blocks); P.n_blocks / P.per_wg count U-block steps
template <int MA, int MT, int NB, int NT, int NW, int DEPTH, int U = 1>
DEN_CODE_ALIGN  // page-aligned code (r04y A/B)
__global__ __launch_bounds__(64 * NW, 1) void dwstream_kernel(DwStreamArgs P) {
  constexpr int TILES = MT + NT;
  constexpr int BLK = TILES * HB_TILE;              // one wave block's tiles
  constexpr int SLOT = U * BLK;
  constexpr int RING = DEPTH + 1;
  constexpr int PIECES = 2 * TILES * U;             // 1 KiB DMA pieces per step
  constexpr int TPW = (MT * NT + NW - 1) / NW;      // output tiles per wave
  static_assert(RING * SLOT <= 160 * 1024, "ring exceeds the LDS");
  __shared__ __attribute__((aligned(16))) char lds[RING * SLOT];
  DEN_CLOCK_BEGIN();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR) for the DMA operands
  // readfirstlane hides the range of threadIdx.x >> 6: without it the compiler cannot prove the
  // output-tile guards (t < MT * NT) true, branches around every MFMA and copies the accumulators
  // through each branch (r05: 4.4 ms, 2.9 ms with the range restored)
  __builtin_assume(wave >= 0 && wave < NW);
  const int64_t b0 = (int64_t)blockIdx.x * P.per_wg;
  const int64_t b1 = b0 + P.per_wg < P.n_blocks ? b0 + P.per_wg : P.n_blocks;

  auto fetch = [&](int64_t blk, char* dst) __attribute__((always_inline)) {
    // (force-inlined: outlined as a call, as the compiler once chose, the launch faulted)
#pragma unroll
    for (int q = 0; q < (PIECES + NW - 1) / NW; ++q) {
      const int pc = __builtin_amdgcn_readfirstlane(q * NW + wave);
      if (pc < PIECES) {
        const int ub = pc / (2 * TILES), tp = pc % (2 * TILES);
        const int t = tp >> 1, f = tp & 1;
        const int64_t wb = blk * U + ub;
        const char* src;
        if (t < MA) src = P.a[0] + wb * P.a_bs[0] + t * HB_TILE;
        else if (t < MT) src = P.a[1] + wb * P.a_bs[1] + (t - MA) * HB_TILE;
        else if (t < MT + NB) src = P.b[0] + wb * P.b_bs[0] + (t - MT) * HB_TILE;
        else src = P.b[1] + wb * P.b_bs[1] + (t - MT - NB) * HB_TILE;
        dws_dma_piece(src, dst + pc * 1024, f);
      }
    }
  };
  // DMA instructions this wave issues per block (pieces pc = q * NW + wave < PIECES)
  const bool extra = wave < PIECES % NW;
  constexpr int OPS_LO = PIECES / NW, OPS_HI = OPS_LO + 1;

#pragma unroll
  for (int u = 0; u < DEPTH; ++u)
    if (b0 + u < b1) fetch(b0 + u, lds + u * SLOT);

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

  for (int64_t blk = b0; blk < b1; ++blk) {
    const int u = (int)((blk - b0) % RING);
    if (blk + DEPTH < b1) fetch(blk + DEPTH, lds + ((u + DEPTH) % RING) * SLOT);
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
      if (extra) hb_wait_vm_lgkm0<(DEPTH - 1) * OPS_HI>();
      else hb_wait_vm_lgkm0<(DEPTH - 1) * OPS_LO>();
    } else {
      hb_wait_vm_lgkm0<0>();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  DEN_CLOCK_END(4);
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
template __global__ void dwstream_kernel<8, 16, 2, 2, DWS_NW1, 3, 1>(DwStreamArgs);  // L0 + L5 pe
// (the Lg launch, dwstream_kernel<4, 4, 8, 9, 16, 2, 2> on [bottleneck | ve], was replaced in r05 by
// the weight gradient fused into render_head_bwd_kernel)

}  // namespace den
