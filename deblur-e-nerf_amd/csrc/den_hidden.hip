// den_hidden.hip -- layer-major backward of the [bottleneck | sigma] layer Lb and the hidden layers
// L7..L1 (BF16 mode).
//
// One launch per layer l (transposed layer j = 10 - l; Lb = l 8, j 2), one persistent workgroup per CU
// sweeping a contiguous range of 32-sample wave blocks of the wave-block-major activation tensors
// (den_geom.h).  Per block, wave w of 8 (two per SIMD at 256 registers) owns W^T row tile w:
//   chain : dS_{l-1} = W_l^T dz_l                (A = the wave's W_l^T row tiles held in registers for
//           dz_{l-1} = dS_{l-1} * (1 - 2^-S'_{l-1})   the whole launch, B = dz_l fragments from LDS)
//   dW    : dW_l[the wave's rows][all 256] += dz_l (x) S'_{l-1},  db_l += dz_l
//           (k = samples: both operands by ds_read_b64_tr_b16 from the same LDS blocks; the bias from
//           VALU sums of the dz operand), accumulated in registers over the whole range, written once as a
//           split-K partial for dw_reduce_kernel (den_dw.hip layout, MT = NT = 8).
// dz_l and S'_{l-1} (16 KiB per block each) arrive by LDS-DMA 3 blocks ahead (96 KiB in flight per CU).  Per sample and layer
// this moves 1.5 KiB of HBM (read dz_l and S'_{l-1}, write dz_{l-1}) where the sample-major chain
// plus the split-K GEMM (den_render.hip + den_dw.hip; kept for the F32 parity mode) move 3 KiB.
//
// Reference: the nn.Linear backward of base.hidden_layers.{1..7}, bottleneck_layer and sigma_layer
// with softplus(beta=100) on their input (external/mlp.py:99-113, :155-186, models/nerf.py:18), in the
// scaled base-2 units of den_geom.h.
#include "den_device.h"

namespace den {

// Waves per workgroup: 8 (two per SIMD at 256 registers, one W^T row tile each).  L7..L1: 4.559 ->
// 4.327 ms per launch against 4 waves at 512 registers (ABBA order, profiles/r06ar_ab.jsonl); Lb: 5.211
// -> 4.934 ms per launch with its sigma k-step W^T fragment in LDS, the S' fragments read in the
// epilogue and dz fragments read one k-step ahead (profiles/r06at_ab.jsonl; held in registers, these
// spill at 256; 2 ahead measured 4.960).
template <bool LB>
struct HbCfg {
  static constexpr int WAVES = 8;
  static constexpr int RT = 8 / WAVES;         // W^T row tiles per wave
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int STORE_OPS = 2 * RT;     // dz_{l-1} stores per wave per block
  // Lb: the sigma k-step's W^T fragment lives in LDS (its registers would spill)
  static constexpr bool WT16_LDS = LB;
};
constexpr int HB_TILE = 2048;          // one 32 x 32 BF16 tile of a wave block
constexpr int HB_BLOCK = 8 * HB_TILE;  // the 256 features of one 32-sample wave block
constexpr int HB_SIG = 256;            // LB: LDS bytes for sigma's bf16[32] dz of a block (aligned)
// The pe weight-gradient fold (PEM; possible once a wave holds one W^T row tile):
// L5 (PEM 1) also forms dW_5's pe columns from its dz_5 operand; L1 (PEM 2) forms dW_0 = dz_0 (x) pe and
// db_0 from the dz_0 it computes, which then never leaves the chip (each wave stages its tile in LDS
// for the transposed read).  pe (the forward's stored copy, 2 tiles per wave block) arrives as a third
// part of each ring slot, one 1 KiB piece from each of waves 0..3.  The partials take
// den_dwstream.hip's [wg][16][3] layout (L1 row tiles 0..7 with the bias, L5 8..15), so the streamed
// launch's two reductions read them unchanged.  Both variants trade the chain's dz read-ahead and the
// early derivative factors (L7..L1's) for the 32 registers of the two pe accumulator tiles.
constexpr int HB_PE = 2 * HB_TILE;     // PEM: pe bytes per wave block
// PEM: the ring runs fewer blocks ahead (L5 two: 3 slots of 36 KiB; L1 one: 2 slots, beside its dz_0
// stages), and the last hb_wtl_k k-steps of the waves' W^T fragments live in the LDS this frees (8 KiB
// each, 4 registers per lane each; L1 at 4 of them and two ahead still spilled 12)
#ifndef DEN_HB_DEPTH_PE2
#define DEN_HB_DEPTH_PE2 1
#endif
template <int PEM> constexpr int hb_depth_pe() { return PEM == 1 ? 2 : DEN_HB_DEPTH_PE2; }
template <int PEM> constexpr int hb_wtl_k() {  // (LDS: L5 156 KiB, L1 152 KiB)
  return PEM == 1 ? 6 : PEM == 2 ? (DEN_HB_DEPTH_PE2 == 1 ? 8 : 4) : 0;
}
// Measured (r02/r03): one persistent workgroup per CU; non-temporal dz_l / S'_{l-1}
// loads and dz_{l-1} stores (streamed once; cached stores were slower); 3 blocks in flight (4 did not
// help); dz_l fragments read 4 k-steps ahead; the epilogue and the dW MFMAs kept in separate phases
// (overlapping them, in compiler order or a pinned interleave, was 1-2 ms per step slower).
constexpr int HB_GRID_MAX = 256;  // persistent workgroups (one per CU)
constexpr int HB_PF_L = 4;        // dz_l fragments read ahead of the chain MFMAs
constexpr int HB_PF_LB = 1;       // (Lb: registers, see HbCfg)
#ifndef DEN_HB_DEPTH_L
#define DEN_HB_DEPTH_L 3
#endif
constexpr int HB_DEPTH_LB = 3;    // blocks in flight ahead of the computed one (Lb: 33 KiB slots, <= 4 fit)
constexpr int HB_DEPTH_L = DEN_HB_DEPTH_L;  // L7..L1 (32 KiB slots: up to 4 ahead in 160 KiB; 4 measured
                                            // no faster with the block-major rows, profiles/r06y_ab.jsonl)

typedef short hb_v4i16 __attribute__((ext_vector_type(4)));

// Experiment builds only (-DDEN_HIDDEN_PROF, profiles/hidden_prof.py): per-wave cycle split of a launch
// by s_memtime marks -- 0 DMA issue, 1 chain (dz fragments + W^T MFMAs, Lb's sigma k-step), 2 epilogue
// (activation derivative + dz stores), 3 dW / db, 4 Lb's sigma weight-gradient row, 5 vmcnt wait for the
// next block, 6 barrier, 7 the whole launch; slot 0 = the last L7..L1 launch, slot 1 = Lb.
struct HbProf {
#ifdef DEN_HIDDEN_PROF
  uint64_t p[8];
  uint64_t t;
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int q = 0; q < 8; ++q) p[q] = 0;
    t = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void mark(int q) {
    const uint64_t n = __builtin_amdgcn_s_memtime();
    p[q] += n - t;
    t = n;
  }
#else
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void mark(int) {}
#endif
};
#ifdef DEN_HIDDEN_PROF
__device__ uint64_t den_hidden_prof[2 * 256 * 8 * 8];
#endif

struct HiddenArgs {
  const char* w;      // packed transposed weights of the layer (bwd chunk 0 of layer j, 16 KiB per row tile)
  const char* dz_in;  // dz_l
  const char* s_in;   // S'_{l-1}
  char* dz_out;       // dz_{l-1}
  float* partial;     // [gridDim.x][8][9][64][16]
  int64_t n_blocks;   // 32-sample wave blocks
  int64_t per_wg;     // blocks per workgroup
  int64_t bs_dz_in, bs_s, bs_dz_out;  // bytes from one wave block to the next (den_geom.h SROW_BYTES rows)
  const char* sigma_dz;               // LB: sigma's dz, one bf16 per sample
  const char* pe;                     // PEM: the stored pe (2 tiles per wave block)
  int64_t bs_pe;
  float* pe_partial;                  // PEM: [gridDim.x][16][3][64][16] (den_dwstream.hip layout)
  int pe_mt0;                         // PEM: first row tile (L1 0, L5 8)
};

// 16-byte LDS slot that holds tile lane `lane`'s fragment f inside a 1 KiB piece:
// lane c + 32h -> 32h + (c ^ 4(2h + f)).  An involution for each (h, f); it spreads the
// 4-sample x 16-feature blocks of the transposed reads over all 64 banks, while the plain
// per-lane fragment reads stay a permutation of one 1 KiB piece (conflict-free either way).
__device__ __forceinline__ int hb_slot(int lane, int f) {
  const int h = lane >> 5;
  return 32 * h + ((lane & 31) ^ (4 * (2 * h + f)));
}

// LDS-DMA of one 16 KiB block (pieces pc = 2t + f of 1 KiB): the destination of an LDS-DMA
// instruction is linear, so lane p fetches the tile lane whose fragment belongs in slot p.
template <int WAVES>
__device__ __forceinline__ void hb_dma(const char* src, char* dst) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 16 / WAVES; ++q) {
    const int pc = q * WAVES + wave;  // wave-uniform
    __builtin_amdgcn_global_load_lds((const void*)(src + pc * 1024 + hb_slot(lane, pc & 1) * 16),
                                     (lds_ptr_t)(dst + pc * 1024), 16, 0, 0);
  }
}

// The same DMA issued through inline asm: the compiler then does not track it, so it does not make
// every LDS read wait vmcnt(0) for the prefetches in flight (it cannot tell the ring slots apart);
// hidden_bwd_kernel waits for them explicitly (hb_wait_vm_lgkm0 + barrier).  The "memory" clobber
// keeps LDS reads and global stores in program order around it.
template <int WAVES>
__device__ __forceinline__ void hb_dma_untracked(const char* src, char* dst) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // per-lane 32-bit offsets (two: the slot permutation depends on the fragment parity); the 64-bit
  // base stays in SGPRs (saddr form), so the ring needs no per-instruction VGPR address pairs
  const uint32_t off0 = (uint32_t)hb_slot(lane, 0) * 16, off1 = (uint32_t)hb_slot(lane, 1) * 16;
#pragma unroll
  for (int q = 0; q < 16 / WAVES; ++q) {
    // wave-uniform piece index (readfirstlane is 32-bit: never pass it a 64-bit pointer)
    const int pc = __builtin_amdgcn_readfirstlane(q * WAVES + wave);
    const char* base = src + pc * 1024;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(dst + pc * 1024));
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"((pc & 1) ? off1 : off0),
                 "s"(base), "s"(m0) : "memory", "m0");
  }
}

// LB: sigma's 32 bf16 dz of a wave block (64 B of HiddenArgs.sigma_dz) into LDS, by lanes 0..3;
// every wave issues it (the same bytes), so each wave's DMA count per block stays uniform (issued by one
// wave only, with its own vmcnt budget: Lb 5.162 -> 5.195 ms, no gain, profiles/r06aw_ab.jsonl)
__device__ __forceinline__ void hb_dma_sigma(const char* src, char* dst) {
  const int lane = threadIdx.x & 63;
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)dst);
  if (lane < 4)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"((uint32_t)lane * 16),
                 "s"(src), "s"(m0) : "memory", "m0");
}

// PEM: the pe block of a wave block (4 x 1 KiB pieces, the slot permutation of hb_dma) by waves 0..3
__device__ __forceinline__ void hb_dma_pe(const char* src, char* dst) {
  const int lane = threadIdx.x & 63;
  const int pc = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (pc < 4) {
    const uint32_t off = (uint32_t)hb_slot(lane, pc & 1) * 16;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(dst + pc * 1024));
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"(off), "s"(src + pc * 1024),
                 "s"(m0) : "memory", "m0");
  }
}

// This lane's own fragment f of a tile in LDS (the chain's B operand / the stored activation).
__device__ __forceinline__ bf16x8 hb_frag(const char* tile, int f) {
  return *(const bf16x8*)(tile + f * 1024 + hb_slot(threadIdx.x & 63, f) * 16);
}

// Operand with k = samples: row (A) / column (B) index = feature (stored position) l & 31 of the
// tile, k-slot 8(l >> 5) + j = sample 16 kk + 8(l >> 5) + j of the block; two transposed reads of
// 4 samples x 16 features per 16-lane group.
__device__ __forceinline__ bf16x8 hb_tr_frag(const char* tile, int kk) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int hq = g & 1, p = i & 3, f = p >> 1;
  bf16x8 out;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int c = 16 * kk + 8 * (g >> 1) + 4 * r + (i >> 2);
    const char* a = tile + f * 1024 + hb_slot(c + 32 * hq, f) * 16 + (p & 1) * 8;
    const hb_v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) hb_v4i16*)a);
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * r + e] = __builtin_bit_cast(__bf16, (short)v[e]);
  }
  return out;
}

// s_waitcnt vmcnt(VM) lgkmcnt(0) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14;
// expcnt left at its maximum).
template <int VM>
__device__ __forceinline__ void hb_wait_vm_lgkm0() {
  static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | ((VM >> 4) << 14));
}

// One 32-sample block from its LDS slot: the chain (dz_{l-1} stored), then the dW / db accumulation.
// Sigma's weight-gradient row of one block (LB, see hb_block): dW_sigma[q] = sum_n dz_sigma[n] S7[n][q]
// for the wave's S7 tile w by VALU dot products: the transposed fragment of an S7 tile
// (hb_tr_frag: lane l holds stored position l & 31 of the tile at samples 16 kk + 8 (l >> 5) + j) times
// the same eight samples' sigma dz, four v_dot2c_f32_bf16 per fragment, into one f32 per lane
// (the two lane halves hold the two sample halves; added at the end).  r06: this replaced four
// dependent 32x32x16 MFMAs into one accumulator per block (at 4 waves: tile 2w in column 0, 2w + 1 in
// column 16 of a 16-register tile) -- 703 cycles per block of the Lb launch's 5.5 k (DEN_HIDDEN_PROF,
// profiles/r06c_hidden_prof.json), the MFMA chain's latency exposed -- and frees 14 registers.
__device__ __forceinline__ void hb_sigma_dw(const char* sig, const char* sb, float (&sd)[HbCfg<true>::RT]) {
  constexpr int HB_RT = HbCfg<true>::RT;
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // (no scheduling fence: with the dot2 row its LDS reads may start under the dW MFMAs' tail, no
  // spills; Lb 5.398 -> 5.337 ms in ABBA order, profiles/r06ah_ab.jsonl)
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const bf16x8 sv = *(const bf16x8*)(sig + 32 * kk + 16 * (lane >> 5));
#pragma unroll
    for (int t = 0; t < HB_RT; ++t) {
      const bf16x8 a = hb_tr_frag(sb + (HB_RT * wave + t) * HB_TILE, kk);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bf16x2_t x = {a[2 * q], a[2 * q + 1]}, y = {sv[2 * q], sv[2 * q + 1]};
        sd[t] = __builtin_amdgcn_fdot2_f32_bf16(x, y, sd[t], false);
      }
    }
  }
}

// LB: the [bottleneck | sigma] layer (Lb, den_render.hip's transposed layer j = 2): besides the 8
// bottleneck tiles, sigma's dz arrives as 32 bf16 per block (staged after them); the chain takes it as
// a 17th k-step whose B fragment holds sigma at stored position 0 (W_b^T's sigma column; the rest of
// that k-step and the 18th are zero padding).  Sigma's weight-gradient row would be a ninth row tile
// of 8 more accumulator tiles; instead wave w forms the row for its S7 tile w by VALU dot products
// (hb_sigma_dw).
template <bool LB, int PEM>
__device__ __forceinline__ void hb_block(const HiddenArgs& P, const char* cur, const bf16x8* wt16,
                                         const bf16x8* wtl, char* stage,
                                         int64_t b, const bf16x8 (&wt)[HbCfg<LB>::RT][LB ? 17 : 16],
                                         f32x16 (&dw)[HbCfg<LB>::RT][8], float (&db)[HbCfg<LB>::RT],
                                         float (&sd)[HbCfg<LB>::RT], float& sdb, f32x16 (&dwp)[2], float& db0,
                                         HbProf& hp) {
  constexpr int HB_RT = HbCfg<LB>::RT;
  static_assert(PEM == 0 || (!LB && HB_RT == 1), "the pe fold is for L1 / L5 at one row tile per wave");
  constexpr bool EARLY = !LB && PEM == 0;  // S' prefetch + derivative factors in the chain's shadow
  constexpr int HB_PF = EARLY ? HB_PF_L : HB_PF_LB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int DZ_BYTES = LB ? HB_BLOCK + HB_SIG : HB_BLOCK;
  const char* dzb = cur;
  const char* sig = cur + HB_BLOCK;  // LB: sigma's dz, bf16[32]
  const char* sb = cur + DZ_BYTES;
  const char* peb = sb + HB_BLOCK;   // PEM: the block's pe tiles
  // chain: both row tiles of this wave share each dz_l fragment (K = 256, 16 k-steps): one LDS read
  // feeds two independent MFMAs, and the reads run HB_PF k-steps ahead of their use (issued
  // one per k-step, the compiler waited out the LDS latency before every MFMA)
  f32x16 accs[HB_RT];
#pragma unroll
  for (int t = 0; t < HB_RT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) accs[t][r] = 0.0f;
  // the epilogue's S'_{l-1} fragments (the activation derivative's input), read before the chain so
  // that their LDS latency hides under its 32 MFMAs instead of opening each tile's epilogue
  bf16x8 sf[HB_RT][2];
#pragma unroll
  for (int t = 0; t < HB_RT; ++t)
#pragma unroll
    for (int f = 0; f < 2; ++f)
      if constexpr (EARLY) sf[t][f] = hb_frag(sb + (HB_RT * wave + t) * HB_TILE, f);
  __builtin_amdgcn_sched_barrier(0);  // (left alone, the compiler sinks these reads back to their use)
  // L7..L1: the epilogue's 32 activation-derivative factors 1 - 2^-S', computed in the chain MFMAs'
  // shadow (r06, profiles/r06v_ab.jsonl: 4.639 -> 4.607 ms per launch in ABBA order).  Lb has no
  // registers for them: there it is 16 exp2 in the epilogue (+260 cycles per block against L1, phase
  // split profiles/r06aw_hidden_prof.json), but the same factors in its chain spill 12 registers and
  // computed right after its sigma k-step still 8
  float dv[HB_RT][16];
  {
    bf16x8 bq[HB_PF];
#pragma unroll
    for (int p = 0; p < HB_PF; ++p) bq[p] = hb_frag(dzb + (p >> 1) * HB_TILE, p & 1);
    // PEM: k-steps [KL, 16) of the wave's W^T from LDS (wtl), each read one k-step ahead; the
    // scheduling fence per k-step keeps the compiler from hoisting them all (their registers are the
    // point)
    constexpr int KL = 16 - hb_wtl_k<PEM>();
    bf16x8 wn;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const bf16x8 cur = bq[k % HB_PF];
      if (k + HB_PF < 16) bq[k % HB_PF] = hb_frag(dzb + ((k + HB_PF) >> 1) * HB_TILE, (k + HB_PF) & 1);
      static_assert(PEM == 0 || HB_RT == 1, "");
      const bf16x8 wa = k >= KL ? wn : wt[0][k < KL ? k : 0];
      if (PEM && k + 1 >= KL && k + 1 < 16) wn = wtl[((k + 1 - KL) * 8 + wave) * 64 + lane];
#pragma unroll
      for (int t = 0; t < HB_RT; ++t)
        accs[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(PEM ? wa : wt[t][k], cur, accs[t], 0, 0, 0);
      if constexpr (PEM) __builtin_amdgcn_sched_barrier(0);
      if constexpr (EARLY) {  // HB_RT of the derivative factors per k-step
#pragma unroll
        for (int e = 0; e < HB_RT; ++e) {
          const int q = k * HB_RT + e, t = q >> 4, r = q & 15;
          dv[t][r] = dsoftplus2_scaled_from_out((float)sf[t][r >> 3][r & 7]);
        }
      }
    }
  }
  if constexpr (LB) {
    // B fragment of the sigma k-step: sample c = lane (lanes 0..31) has sigma at stored position 0
    const __bf16 z = *(const __bf16*)(sig + 2 * (lane & 31)), zz = (__bf16)0.0f;
    const bf16x8 bs = {lane < 32 ? z : zz, zz, zz, zz, zz, zz, zz, zz};
#pragma unroll
    for (int t = 0; t < HB_RT; ++t)
      accs[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(HbCfg<LB>::WT16_LDS ? wt16[(HB_RT * wave + t) * 64 + lane]
                                                                                    : wt[t][16],
                                                        bs, accs[t], 0, 0, 0);
    sdb += (float)bs[0];

  }
  hp.mark(1);
  // then the activation derivative
#pragma unroll
  for (int t = 0; t < HB_RT; ++t) {
    f32x16 acc = accs[t];
    // (Lb reads them here: held across its chain they would spill)
    const bf16x8 s0 = !EARLY ? hb_frag(sb + (HB_RT * wave + t) * HB_TILE, 0) : sf[t][0];
    const bf16x8 s1 = !EARLY ? hb_frag(sb + (HB_RT * wave + t) * HB_TILE, 1) : sf[t][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (EARLY) {
        acc[r] = acc[r] * dv[t][r];
      } else {
        const float sv = (float)(r < 8 ? s0[r] : s1[r - 8]);
        acc[r] = acc[r] * dsoftplus2_scaled_from_out(sv);
      }
    }
    // dz_{l-1} tile: stored now, the weight-gradient MFMAs below cover its write latency
    bf16x8 of[2];
    acc_to_frags<1>(acc, of);
    if constexpr (PEM == 2) {
      // dz_0 stays on chip: the wave's tile into its LDS stage (hb_slot order, read back transposed by
      // the pe phase below; LDS operations of one wave complete in order)
      *(bf16x8*)(stage + hb_slot(lane, 0) * 16) = of[0];
      *(bf16x8*)(stage + 1024 + hb_slot(lane, 1) * 16) = of[1];
    } else {
      char* d = P.dz_out + b * P.bs_dz_out + (HB_RT * wave + t) * HB_TILE + lane * 16;  // dz_{l-1}: 8 tiles per block
      __builtin_nontemporal_store(of[0], (bf16x8*)d);
      __builtin_nontemporal_store(of[1], (bf16x8*)(d + 1024));
    }
    // keep the scheduler from hoisting the next phase's LDS reads here (register pressure: W^T lives
    // in 128 VGPRs and dW in all 256 AGPRs for the whole launch)
    __builtin_amdgcn_sched_barrier(0);
  }
  hp.mark(2);
  // weight / bias gradients over the block's 32 samples (two k-steps of 16)
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 a[HB_RT];
#pragma unroll
    for (int t = 0; t < HB_RT; ++t) a[t] = hb_tr_frag(dzb + (HB_RT * wave + t) * HB_TILE, kk);
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const bf16x8 bb = hb_tr_frag(sb + n * HB_TILE, kk);
#pragma unroll
      for (int t = 0; t < HB_RT; ++t) dw[t][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t], bb, dw[t][n], 0, 0, 0);
      if constexpr (PEM == 2) {  // (registers: at most four S' fragments in flight)
        if (n % 4 == 3) __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < HB_RT; ++t) db[t] += (float)a[t][j];
    if constexpr (PEM == 1) {  // dW_5's pe columns: the same dz_5 operand against the pe tiles
#pragma unroll
      for (int n = 0; n < 2; ++n) dwp[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], hb_tr_frag(peb + n * HB_TILE, kk),
                                                                                    dwp[n], 0, 0, 0);
    }
  }
  if constexpr (PEM == 2) {  // dW_0 = dz_0 (x) pe and db_0 from the staged dz_0 tile
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 a0 = hb_tr_frag(stage, kk);
#pragma unroll
      for (int n = 0; n < 2; ++n)
        dwp[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, hb_tr_frag(peb + n * HB_TILE, kk), dwp[n], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) db0 += (float)a0[j];
    }
  }
  hp.mark(3);
  // sigma's weight-gradient row last (placed between the chain and the epilogue or before the dW
  // MFMAs its operands spill registers or it measured slower: r03)
  if constexpr (LB) {
    hb_sigma_dw(sig, sb, sd);
    hp.mark(4);
  }
}

template <bool LB, int PEM>
DEN_CODE_ALIGN  // page-aligned code (r04y A/B)
__global__ __launch_bounds__(HbCfg<LB>::THREADS, 1) void hidden_bwd_kernel(HiddenArgs P) {
  constexpr int HB_WAVES = HbCfg<LB>::WAVES, HB_RT = HbCfg<LB>::RT;
  constexpr int HB_STORE_OPS = PEM == 2 ? 0 : HbCfg<LB>::STORE_OPS;  // (PEM 2: dz_0 is not stored)
  // HB_RING LDS slots of [dz_l block | S'_{l-1} block]; HB_DEPTH blocks in flight ahead of the one
  // being computed.  Each wave waits for its own part of block b+1 at the end of block b (vmcnt; the
  // younger prefetches and stores stay in flight), then the workgroup barrier publishes every part.
  constexpr int DZ_STAGED = LB ? HB_BLOCK + HB_SIG : HB_BLOCK;  // bytes of them staged
  constexpr int SLOT = DZ_STAGED + HB_BLOCK + (PEM ? HB_PE : 0);
  constexpr int KST = LB ? 17 : 16;              // chain k-steps
  constexpr int ROW_BYTES = (LB ? 288 : 256) * 64;  // packed W^T row tile (chunk_bytes_K(bwd_K))
  constexpr int MTA = LB ? 9 : 8;                // partial row tiles
  constexpr int DMA_OPS = 2 * (HB_BLOCK / 1024 / HB_WAVES) + (LB ? 1 : 0);  // per wave per block
  // vector-memory ops a wave issues after its DMA of block b+1 by the end of block b (issue order:
  // stores(b-2), DMA(b+2), stores(b-1), DMA(b+3), stores(b)); the asm DMAs clobber "memory", so the
  // stores keep their program order around them
  constexpr int HB_DEPTH = LB ? HB_DEPTH_LB : PEM ? hb_depth_pe<PEM>() : HB_DEPTH_L;
  constexpr int HB_RING = HB_DEPTH + 1;
  constexpr int YOUNGER = HB_STORE_OPS + (HB_DEPTH - 1) * (DMA_OPS + HB_STORE_OPS);
  constexpr int YOUNGER_PE = YOUNGER + (PEM ? HB_DEPTH - 1 : 0);  // PEM, waves 0..3: + their pe pieces
  // LDS: the ring, then LB's sigma k-step W^T fragments (8 KiB), PEM's last HB_WTL_K W^T k-steps
  // (8 KiB each) and PEM 2's dz_0 stages (2 KiB per wave)
  constexpr int WT16_BYTES = HbCfg<LB>::WT16_LDS ? 8 * 64 * 16 : 0;
  constexpr int WTL_K = hb_wtl_k<PEM>();
  constexpr int WTL_BYTES = WTL_K * 8 * 64 * 16;
  constexpr int STAGE_BYTES = PEM == 2 ? HB_WAVES * HB_TILE : 0;
  constexpr int LDS_TOTAL = HB_RING * SLOT + WT16_BYTES + WTL_BYTES + STAGE_BYTES;
  static_assert(LDS_TOTAL <= 160 * 1024, "hidden ring exceeds the LDS");
  __shared__ __attribute__((aligned(16))) char lds[LDS_TOTAL];
  const bf16x8* wt16 = (const bf16x8*)(lds + HB_RING * SLOT);
  const bf16x8* wtl = (const bf16x8*)(lds + HB_RING * SLOT + WT16_BYTES);
  DEN_CLOCK_BEGIN();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* stage = lds + HB_RING * SLOT + WT16_BYTES + WTL_BYTES + wave * HB_TILE;  // PEM 2
  const bool pe_wave = PEM && __builtin_amdgcn_readfirstlane(wave) < 4;
  // a contiguous range of P.per_wg blocks per workgroup (r03: strided by the grid, so that all
  // workgroups sweep one address window, measured the same)
  const int64_t b0 = (int64_t)blockIdx.x * P.per_wg;
  const int64_t n_it = b0 < P.n_blocks ? (b0 + P.per_wg < P.n_blocks ? P.per_wg : P.n_blocks - b0) : 0;
  auto blk = [&](int64_t it) { return b0 + it; };
  auto fetch = [&](int64_t b, char* dst) {
    hb_dma_untracked<HB_WAVES>(P.dz_in + b * P.bs_dz_in, dst);
    if constexpr (LB) hb_dma_sigma(P.sigma_dz + b * 64, dst + HB_BLOCK);
    hb_dma_untracked<HB_WAVES>(P.s_in + b * P.bs_s, dst + DZ_STAGED);
    if constexpr (PEM) hb_dma_pe(P.pe + b * P.bs_pe, dst + DZ_STAGED + HB_BLOCK);
  };
#pragma unroll
  for (int u = 0; u < HB_DEPTH; ++u)
    if (u < n_it) fetch(blk(u), lds + u * SLOT);

  // W_l^T row tile w: packed [row tile][kappa][lane][8] = the chain's A fragments
  bf16x8 wt[HB_RT][KST];
#pragma unroll
  for (int t = 0; t < HB_RT; ++t)
#pragma unroll
    for (int k = 0; k < KST; ++k)
      wt[t][k] = *(const bf16x8*)(P.w + (int64_t)(HB_RT * wave + t) * ROW_BYTES + k * 1024 + lane * 16);
  if constexpr (HbCfg<LB>::WT16_LDS) {
#pragma unroll
    for (int t = 0; t < HB_RT; ++t) ((bf16x8*)wt16)[(HB_RT * wave + t) * 64 + lane] = wt[t][16];
  }
  if constexpr (PEM) {
#pragma unroll
    for (int q = 0; q < WTL_K; ++q)
#pragma unroll
      for (int t = 0; t < HB_RT; ++t) ((bf16x8*)wtl)[(q * 8 + HB_RT * wave + t) * 64 + lane] = wt[t][16 - WTL_K + q];
  }
  f32x16 dw[HB_RT][8];
#pragma unroll
  for (int t = 0; t < HB_RT; ++t)
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) dw[t][n][r] = 0.0f;
  float db[HB_RT], sd[HB_RT];  // bias partial: feature (lane & 31) of row tile HB_RT w + t, this lane's
                               // samples; LB: sigma's weight-gradient row, stored position lane & 31 of S7
                               // tile HB_RT w + t
#pragma unroll
  for (int t = 0; t < HB_RT; ++t) db[t] = sd[t] = 0.0f;
  float sdb = 0.0f;  // LB: sigma's bias gradient (lanes 0..31)
  f32x16 dwp[2];     // PEM: the pe weight-gradient tiles of the wave's row tile (pe columns 0..31, 32..63)
  float db0 = 0.0f;  // PEM 2: db_0 partial, feature (lane & 31) of row tile w, this lane's samples
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) dwp[n][r] = 0.0f;
  HbProf hp;
  hp.init();
#ifdef DEN_HIDDEN_PROF
  const uint64_t hp_start = hp.t;
#endif
  hb_wait_vm_lgkm0<0>();       // block b0 (and the prologue prefetches) landed
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int64_t it = 0; it < n_it; ++it) {
    const int u = (int)(it % HB_RING);
    hp.mark(6);
    // prefetch block it + HB_DEPTH into the slot block it - 1 used (free since the last barrier)
    if (it + HB_DEPTH < n_it) fetch(blk(it + HB_DEPTH), lds + ((u + HB_DEPTH) % HB_RING) * SLOT);
    hp.mark(0);
    hb_block<LB, PEM>(P, lds + u * SLOT, wt16, wtl, stage, blk(it), wt, dw, db, sd, sdb, dwp, db0, hp);
    if (it + HB_DEPTH < n_it) {
      if (pe_wave) hb_wait_vm_lgkm0<YOUNGER_PE>();
      else hb_wait_vm_lgkm0<YOUNGER>();
    } else {
      hb_wait_vm_lgkm0<0>();
    }
    hp.mark(5);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  hp.mark(6);
  DEN_CLOCK_END(LB ? 3 : 2);
#ifdef DEN_HIDDEN_PROF
  hp.p[7] = hp.t - hp_start;
  if (blockIdx.x < 256 && lane == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) den_hidden_prof[((LB ? 256 : 0) + blockIdx.x) * 64 + wave * 8 + q] = hp.p[q];
  }
#endif
  // split-K partial of this workgroup (dw_gemm_kernel layout: [wg][mt][nt][lane][16]); the bias
  // goes where that layout's ones tile (nt = 8) keeps it: column 0 = lanes 0 and 32, row m in
  // register (m & 3) + 4 (m >> 3) of lane 32 ((m >> 2) & 1)
#pragma unroll
  for (int t = 0; t < HB_RT; ++t) {
    const float bsum = db[t] + __shfl_xor(db[t], 32, 64);
    if (lane < 32) {
      const int m = lane;
      float* o = P.partial + (((int64_t)blockIdx.x * MTA + HB_RT * wave + t) * 9 + 8) * 1024;
      o[(32 * ((m >> 2) & 1)) * 16 + (m & 3) + 4 * (m >> 3)] = bsum;
    }
  }
  if constexpr (LB) {
    // row tile 8 = [sigma, 31 padding rows]: sigma is accumulator row 0 (lanes 0..31, register 0),
    // column 32 n + lane; every other element of the tiles written as zero.  Stored position q of S7
    // tile w: sd[0] of lanes q and q + 32 (the two sample halves)
#pragma unroll
    for (int nn = 0; nn < HB_RT; ++nn) {
      const float v = sd[nn] + __shfl_xor(sd[nn], 32, 64);
      float* o = P.partial + (((int64_t)blockIdx.x * MTA + 8) * 9 + HB_RT * wave + nn) * 1024 + lane * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 z = {q == 0 && lane < 32 ? v : 0.0f, 0.0f, 0.0f, 0.0f};
        *(f32x4*)(o + 4 * q) = z;
      }
    }
    const float bs = wave_sum(sdb);
    if (wave == 0) {
      float* o = P.partial + (((int64_t)blockIdx.x * MTA + 8) * 9 + 8) * 1024 + lane * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 z = {q == 0 && lane == 0 ? bs : 0.0f, 0.0f, 0.0f, 0.0f};
        *(f32x4*)(o + 4 * q) = z;
      }
    }
  }
  if constexpr (PEM) {
    // pe partial ([wg][16][3] tiles): row tile pe_mt0 + w, pe column tiles 0, 1; L1's db_0 in the ones
    // tile (nt 2) where the hidden bias goes (above); L5's ones tile is never read (bias 0)
    float* o = P.pe_partial + (((int64_t)blockIdx.x * 16 + P.pe_mt0 + wave) * 3) * 1024;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 v = {dwp[n][4 * q], dwp[n][4 * q + 1], dwp[n][4 * q + 2], dwp[n][4 * q + 3]};
        *(f32x4*)(o + n * 1024 + lane * 16 + 4 * q) = v;
      }
    if constexpr (PEM == 2) {
      const float bsum = db0 + __shfl_xor(db0, 32, 64);
      if (lane < 32) o[2 * 1024 + (32 * ((lane >> 2) & 1)) * 16 + (lane & 3) + 4 * (lane >> 3)] = bsum;
    }
  }
#pragma unroll
  for (int t = 0; t < HB_RT; ++t)
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      float* o = P.partial + (((int64_t)blockIdx.x * MTA + HB_RT * wave + t) * 9 + n) * 1024 + lane * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 v = {dw[t][n][4 * q], dw[t][n][4 * q + 1], dw[t][n][4 * q + 2], dw[t][n][4 * q + 3]};
        *(f32x4*)(o + 4 * q) = v;
      }
    }
}

template __global__ void hidden_bwd_kernel<false, 0>(HiddenArgs);
template __global__ void hidden_bwd_kernel<false, 1>(HiddenArgs);
template __global__ void hidden_bwd_kernel<false, 2>(HiddenArgs);
template __global__ void hidden_bwd_kernel<true, 0>(HiddenArgs);

}  // namespace den
