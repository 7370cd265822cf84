// den_head_bwd.hip -- the BF16 head backward as a persistent kernel with the Lg weight gradient fused.
//
// Per 256-sample item (whole rays), as render_bwd_kernel<1, 1>: the compositing adjoint, Lr^T (with
// the fused Lr weight gradient) -> dz_g, Lg^T -> dz_b (+ sigma's dz) for the layer-major hidden
// backward.  In addition the Lg weight gradient
//   dW_g[o][i] = sum_n dz_g[n][o] x[n][i],  x = [bottleneck (256) | ve (27, padded 32)],  db_g = sum_n dz_g
// is accumulated here, where dz_g is born: dz_g is no longer written to HBM and read back by a
// streamed launch (den_dwstream.hip's Lg launch is gone: -512 B per sample of traffic and a launch).
//   * one workgroup (8 waves) per CU walks items blockIdx.x, + gridDim.x, ...; the weight chunks
//     of the chain wrap to the next item's first chunk (bwd_layer_run WRAP);
//   * after Lr^T each wave stages its dz_g tiles (4 x 2 KiB, the XOR-permuted slot layout of
//     den_hidden.hip) in LDS; a barrier; wave w then owns output column tile w of the bottleneck part
//     (all 4 row tiles, k = the item's 256 samples): the bottleneck tile (block b, column w) of each
//     of the item's 8 wave blocks arrives by untracked LDS-DMA in a private double buffer, both
//     MFMA operands by transposed LDS reads;
//   * the item's eight view-encoding tiles (enc_tile, as the forward) go to LDS -- with the
//     fixed-count sampler computed from the staged ray data by the waves the adjoint leaves idle,
//     during it (r05ar); waves 0..3 own the four (row tile w, ve) output tiles plus row tile w's bias;
//   * the adjoint's inputs (records, ray data) are staged in LDS one item ahead (r05ag), the Lr^T G
//     tiles loaded at the item top (r05ah), and every chain step waits by count for its weight chunk
//     only (untracked DMA, r05aa-ad), so the dz_b stores stay in flight;
//   * the accumulators live in registers for the whole launch; each workgroup writes one split-K
//     partial in den_dwstream.hip's layout [wg][4][10][64][16] (column 9: the bias), reduced in a
//     fixed order by dw_reduce_kernel -- deterministic.
// Reference: the nn.Linear backward of rgb_layer.hidden_layers.0 (external/mlp.py:193-205), fed by
// the view encoding of mlp.py:353-355.

namespace den {

#ifdef DEN_HEAD_PROF
// experiment builds only: per-wave cycles of the head backward's phases (den_debug_head_prof,
// profiles/head_prof.py)
__device__ uint64_t den_head_prof[256 * 8 * 8];
#define HD_T(q) prof[q] += __builtin_amdgcn_s_memtime() - t_; t_ = __builtin_amdgcn_s_memtime()
#else
#define HD_T(q)
#endif

#ifndef DEN_HEAD_UT
#define DEN_HEAD_UT 1  // the Lg^T chain's weight DMA untracked (chunk_step_ut)
#endif

constexpr int HD_STAGE = 8 * 4 * HB_TILE;  // dz_g of the item: 8 waves x 4 tiles (also each wave's Lr scratch)
constexpr int HD_XBUF = 2 * HB_TILE;       // per wave: a double buffer of one bottleneck tile
constexpr int HD_VE = 8 * HB_TILE;         // the item's view-encoding tiles, one per wave block

// One bottleneck tile (2 KiB, two 1 KiB pieces) into this wave's private LDS buffer, untracked (the
// waits are explicit); lane p fetches the tile lane whose fragment belongs in LDS slot p (hb_dma)
__device__ __forceinline__ void hd_dma_piece(const char* src, char* dst, int f) {
  const int lane = threadIdx.x & 63;
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)dst);
  const uint64_t a64 = (uint64_t)(uintptr_t)src;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a64);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a64 >> 32));
  const char* base = (const char*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  const uint32_t off = (uint32_t)hb_slot(lane, f) * 16;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"(off), "s"(base), "s"(m0)
               : "memory", "m0");
}
__device__ __forceinline__ void hd_dma_tile(const char* src, char* dst) {
  hd_dma_piece(src, dst, 0);
  hd_dma_piece(src + 1024, dst + 1024, 1);
}

// The compositing adjoint's inputs one item ahead (fixed-count sampler).  Its first global load
// waited for every older memory op of the wave -- vmcnt is in-order -- i.e. for the previous item's
// dz_b stores to drain: 7.6 k cycles per item while six of the eight waves waited (r05 head
// profile).  The next item's per-sample records (4 KiB, waves 0..3, one 1 KiB LDS-DMA each, into
// rec_lds where the adjoint writes its results in place) and its rays' data (wave 4, one dword per
// lane: per ray o, d, jitter, d_rgb, d_opacity, d_depth = 12 floats, then bkgd) are DMA'd during
// the current item's first Lg^T step; that step's successors' counted waits cover them.
constexpr int HD_NRAY = 256;
template <typename AT>
__device__ __forceinline__ int hd_stage_adjoint(const AT& A, int64_t nx, int wave, char* rec_lds, float* nray) {
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  constexpr int WGS = wg_samples(1);
  if (wave < 4) {
    // linear: lane l's 16 B (sample nx WGS + 64 wave + l) at rec_lds + 1024 wave + 16 l
    const uint64_t a64 = (uint64_t)(uintptr_t)((const char*)A.rec + (nx * WGS + wave * 64) * 16);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a64);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a64 >> 32));
    const char* base = (const char*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(rec_lds + wave * 1024));
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"((uint32_t)lane * 16),
                 "s"(base), "s"(m0) : "memory", "m0");
    return 1;
  }
  if (wave != 4) return 0;
  const int rpw = WGS / A.n_samples;
  const float* dummy = A.rays_o;
  const float* src = dummy;
  if (lane < 12 * rpw) {
    const int q = lane / 12, e = lane - 12 * q;
    const int64_t r = nx * rpw + q;
    if (e < 3) src = A.rays_o + r * 3 + e;
    else if (e < 6) src = A.rays_d + r * 3 + (e - 3);
    else if (e == 6) src = A.jitter + r;
    else if (e < 10) src = (e - 7 < A.rd) ? A.d_rgb + r * A.rd + (e - 7) : dummy;
    else if (e == 10) src = A.d_opacity ? A.d_opacity + r : dummy;
    else src = A.d_depth ? A.d_depth + r : dummy;
  } else if (lane >= 48 && lane < 51) {
    src = (A.has_bkgd && lane - 48 < A.rd) ? A.bkgd + (lane - 48) : dummy;
  }
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)nray);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" : : "v"(src), "s"(m0) : "memory", "m0");
  return 1;
}

// head_adjoint (den_render.hip, points = 0) on the staged inputs: the records from rec_lds (each
// lane reads its own samples before it overwrites them with the results), the ray data from nray
template <typename AT>
__device__ __forceinline__ void head_adjoint_staged(const AT& A, float* rec_lds, const float* nray, const float* bk,
                                                    int64_t item, int wave, int lane) {
  constexpr int WGS = wg_samples(1);
  const int rays_per_wg = WGS / A.n_samples;
  if (wave >= rays_per_wg) return;
  const int64_t r = item * rays_per_wg + wave;
  const float* nr = nray + wave * 12;
  float ro[3], rdv[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    ro[a] = nr[a];
    rdv[a] = nr[3 + a];
  }
  float aabb[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) aabb[q] = A.aabb[q];
  RayGeom rg = ray_geom(ro, rdv, aabb, A.near_p, A.far_p);
  const float ru = nr[6];
  const int spl = A.n_samples / 64;
  float dC[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch)
    if (ch < A.rd) dC[ch] = nr[7 + ch];
  const float dO = A.d_opacity ? nr[10] : 0.0f;
  const float dD = A.d_depth ? nr[11] : 0.0f;
  float bk_dot = 0.0f;
  if (A.has_bkgd)
#pragma unroll
    for (int ch = 0; ch < 3; ++ch)
      if (ch < A.rd) bk_dot += dC[ch] * bk[ch];
  float tau[4], tmid[4], dlt[4], loc[4], locx[4], sg4[4], rc4[4][3];
  float run = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q >= spl) break;
    const int kk = lane * spl + q;
    float a0, a1;
    sample_interval(rg, kk, ru, A.n_samples, &a0, &a1);
    const f32x4 rv = *(const f32x4*)(rec_lds + (wave * A.n_samples + kk) * 4);
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
  const float base = wave_excl_scan(run);
  float w[4], gv[4], op_part = 0.0f, wg_run = 0.0f, wgq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q >= spl) break;
    w[q] = expf(-(base + locx[q])) * (1.0f - expf(-tau[q]));
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
  const float wg_suf_incl = wave_incl_suffix(wg_run);
  const float wg_after = wave_next_lane(wg_suf_incl);
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
    const int kk = lane * spl + q;
    const float Tnext = expf(-(base + loc[q]));
    const float dtau = Tnext * gv[q] - sfx[q];
    const float dsig = dtau * dlt[q];
    const float dsig_raw = dsig * density_dact_from_out(sg4[q], A.density_act);
    const f32x4 o4 = {dsig_raw, w[q] * dC[0] * (-expm1f(-rc4[q][0])), w[q] * dC[1] * (-expm1f(-rc4[q][1])),
                      w[q] * dC[2] * (-expm1f(-rc4[q][2]))};
    *(f32x4*)(rec_lds + (wave * A.n_samples + kk) * 4) = o4;
  }
  if (lane == 0 && A.bkgd_partial) {
    for (int ch = 0; ch < 3; ++ch)
      A.bkgd_partial[(int64_t)ch * A.n_rays + r] = (ch < A.rd && A.has_bkgd) ? dC[ch] * (1.0f - opacity) : 0.0f;
  }
}

DEN_CODE_ALIGN  // page-aligned code (r04y A/B)
__global__ __launch_bounds__(512, 1) void render_head_bwd_kernel(RenderArgs<1> A0, float* lg_partial) {
  constexpr int MODE = 1;
  using T = Tr<MODE>;
  using Frag = typename T::Frag;
  using Acc = typename T::Acc;
  constexpr int TM = T::TM, FPT = T::FPT;
  constexpr int WGS = wg_samples(MODE);
  constexpr int LDS_BYTES = 2 * LDS_BUF + WGS * 16 + HD_STAGE + 8 * HD_XBUF + HD_VE + HD_NRAY;
  static_assert(LDS_BYTES <= 160 * 1024, "the head kernel's LDS exceeds the CU's");
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  float* rec_lds = (float*)(lds + 2 * LDS_BUF);
  char* stage = lds + 2 * LDS_BUF + WGS * 16;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < 8);  // the range readfirstlane hides (see dwstream_kernel)
  char* xbuf = stage + HD_STAGE + wave * HD_XBUF;
  char* lscr = stage + wave * (4 * HB_TILE);  // this wave's Lr scratch = its own dz_g staging area
  char* vet = stage + HD_STAGE + 8 * HD_XBUF;  // ve tiles of the item's 8 wave blocks
  float* nray = (float*)(vet + HD_VE);         // the next item's ray data (hd_stage_adjoint)

  // first item's weight chunk 0 (later items: wrapped in by the previous item's last chain step)
  dma_chunk(A0.w, lds, bwd_tiles(MODE, 0) * chunk_bytes_K(bwd_K(MODE, 0)));  // all of Lr^T: one chunk
  int gc = 0;  // ring index of the item's Lr^T chunk (then Lg^T's 8)
  if (A0.points == 0 && (int64_t)blockIdx.x < (int64_t)A0.n_rays * A0.n_samples / WGS) {
    // the first item's adjoint inputs (later items': staged by the previous item)
    hd_stage_adjoint(A0, blockIdx.x, wave, (char*)rec_lds, nray);
    __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (0 << 8));  // vmcnt(0) lgkmcnt(0)
    __syncthreads();
  }

  f32x16 lacc;  // dW_r (the fused Lr weight gradient), as render_bwd_kernel<1, 1>
  f32x16 gacc[5];  // dW_g: [0..3] = (row tile mt, column tile wave); [4] = (row tile wave, ve) for waves < 4
#pragma unroll
  for (int r = 0; r < 16; ++r) lacc[r] = 0.0f;
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) gacc[q][r] = 0.0f;
  float ldb[3] = {0.f, 0.f, 0.f}, gdb = 0.0f;
  const int64_t n_items = (int64_t)A0.n_rays * A0.n_samples / WGS;
  DEN_CLOCK_BEGIN();
#ifdef DEN_HEAD_PROF
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  uint64_t t_ = t_start;
#endif

  for (int64_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    // the arguments re-read from the kernarg segment per item through an opaque pointer (as the
    // forward): hoisted out of the loop, every chunk's per-lane DMA address stayed live and spilled
    typedef __attribute__((address_space(4))) const RenderArgs<1> KArgs;
    KArgs* Ap = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();  // A0 is the kernel's first argument
    asm volatile("" : "+s"(Ap));
    KArgs& A = *Ap;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // lane-derived values per item (not hoisted across the loop)
    const int lane = tid & 63, c = lane % TM, grp = lane / TM;
    const int64_t sample = item * WGS + wave * TM + c;

    // the Lr^T chain's stored G tiles, issued before the adjoint (which reads only LDS now, so
    // nothing waits behind them): their HBM round trip overlaps it
    // (the background colour read first: the compiler puts a full vmcnt(0) before that LDS read)
    float bk[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) bk[ch] = nray[48 + ch];
    uint4 graw[WIDTH_COND / TM][2];
#pragma unroll
    for (int t = 0; t < WIDTH_COND / TM; ++t) {
      const char* p = act_ptr<MODE>(A, A_G, sample, t) + lane * 16;
      graw[t][0] = ld_stream((const uint4*)p);
      graw[t][1] = ld_stream((const uint4*)(p + 1024));
    }
    // the item's view-encoding tiles (the Lg weight gradient's B operand for the ve columns; lane =
    // sample c, lane group grp (enc_tile), the DMA'd-tile layout), as the forward computes them.
    // Fixed-count sampler: the directions from the staged ray data, all eight tiles by the waves the
    // adjoint leaves idle (one wave per ray), during it -- wave rpw + b also computes tile b of the
    // adjoint's wave b.  Tiles 0..6 are free here (the previous item's dw_block(b <= 6) ran before its
    // last chain step's barrier); tile 7 is stored after the barrier below (dw_block(7) follows the
    // chain).  Otherwise each wave computes its own after the Lr^T chain.
    bf16x8 vef[2];
    auto ve_frags = [&](const float* d) {
      float dv[3];
      view_input(d, dv);
      acc_to_frags<MODE>(enc_tile<MODE>(dv, 0, grp, 4), vef);
    };
    auto ve_store = [&](int b) {
      *(bf16x8*)(vet + b * HB_TILE + hb_slot(lane, 0) * 16) = vef[0];
      *(bf16x8*)(vet + b * HB_TILE + 1024 + hb_slot(lane, 1) * 16) = vef[1];
    };
    const int rpw = WGS / A.n_samples;  // (points == 0) rays per item = the adjoint's waves
    const bool ve_pre = A.points == 0 && rpw <= 4;
    if (ve_pre && wave >= rpw) {
      if (wave - rpw < rpw) {
        ve_frags(nray + ((wave - rpw) * TM) / A.n_samples * 12 + 3);
        ve_store(wave - rpw);
      }
      ve_frags(nray + (wave * TM) / A.n_samples * 12 + 3);
      if (wave != 7) ve_store(wave);
    }
    if (A.points == 0) head_adjoint_staged(A, rec_lds, nray, bk, item, wave, lane);
    else head_adjoint<MODE>(A, rec_lds, item, sample, wave, lane, c, grp);
    HD_T(0);
    // also: every wave is done with the previous item's staged dz_g.  LDS only (__syncthreads'
    // release fence would wait out the G loads above too)
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ve_pre && wave == 7) ve_store(7);
    HD_T(1);

    // fake dz tiles from the per-sample raw gradients (render_bwd_kernel<1, 1>)
    const f32x4 g4 = *(const f32x4*)(rec_lds + (wave * TM + c) * 4);
    Acc dzr = acc_zero<MODE>();
    if (grp == 0) {
      dzr[0] = g4[1];
      if (A.rd > 1) dzr[1] = g4[2];
      if (A.rd > 2) dzr[2] = g4[3];
    }
    {
      const __bf16 z0 = (__bf16)g4[1], z1 = A.rd > 1 ? (__bf16)g4[2] : (__bf16)0.0f,
                   z2 = A.rd > 2 ? (__bf16)g4[3] : (__bf16)0.0f, zz = (__bf16)0.0f;
      const bf16x8 v = {z0, z1, z2, zz, zz, zz, zz, zz};
      *(bf16x8*)(lscr + hb_slot(lane, 0) * 16) = v;
      *(bf16x8*)(lscr + 1024 + hb_slot(lane, 1) * 16) = v;
      if (grp == 0) {
        ldb[0] += (float)z0;
        ldb[1] += (float)z1;
        ldb[2] += (float)z2;
      }
    }
    // the dz_r tile's transposed fragments: the same A operand (masked per G tile) for all four tiles
    const bf16x8 dzr_tr[2] = {hb_tr_frag(lscr, 0), hb_tr_frag(lscr, 1)};
    auto lr_hook = [&](int i, const Acc& sv) {
      Frag gf[FPT];
      acc_to_frags<MODE>(sv, gf);
      char* gs = lscr + 2048;
      *(bf16x8*)(gs + hb_slot(lane, 0) * 16) = gf[0];
      *(bf16x8*)(gs + 1024 + hb_slot(lane, 1) * 16) = gf[1];
      const bool keep = ((lane & 31) >> 3) == i;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 zero = {};
        const bf16x8 a = keep ? dzr_tr[kk] : zero;
        lacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, hb_tr_frag(gs, kk), lacc, 0, 0, 0);
      }
    };

    constexpr int KS = WIDTH / T::KI;
    Frag fr[FPT];
    acc_to_frags<MODE>(dzr, fr);
    Frag xa[KS + 2 * FPT], xb[KS + 2 * FPT];
    // j=0 Lr^T: dz_r -> dz_g in registers (xa, 4 tiles; stored only for den_render_ray_grad) + the
    // fused Lr weight gradient
    bwd_layer_run<MODE, 1, 0, FPT, 0, true, true, true>(A, lds, sample, fr, xa, A_G, A.keep_dzg ? D_ZG : -1, lr_hook,
                                                         NoStepHook{}, gc, graw);
    HD_T(2);
    // dz_g into this wave's staging area (its Lr scratch, done with): 4 tiles, the DMA'd-tile layout
#pragma unroll
    for (int t = 0; t < WIDTH_COND / TM; ++t) {
      *(bf16x8*)(lscr + t * HB_TILE + hb_slot(lane, 0) * 16) = xa[t * FPT];
      *(bf16x8*)(lscr + t * HB_TILE + 1024 + hb_slot(lane, 1) * 16) = xa[t * FPT + 1];
    }
    // the view-encoding tile when it was not computed during the adjoint (read by waves 0..3 after the
    // chain's barriers)
    if (!ve_pre) {
      if (A.points == 0) {
        ve_frags(nray + (wave * TM) / A.n_samples * 12 + 3);  // nray: restaged only in Lg^T's step 0
      } else {
        const int64_t ray = A.points == 2 ? (int64_t)A.ray_idx[sample] : sample;
        float d[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) d[a] = A.rays_d[ray * 3 + a];
        ve_frags(d);
      }
      ve_store(wave);
    }
    HD_T(3);
    // j=1 Lg^T: dz_g (K=128) -> dBott (identity) -> DZB tiles, its last step wrapping in the next
    // item's chunk 0 -- with the Lg weight gradient's blocks interleaved: step i (i >= 1) runs block
    // i - 1 (every wave's dz_g and ve tile are published by step 0's barrier) and issues the
    // bottleneck tile of block i + 1 into the slot block i - 1 used; blocks 0 and 1 are issued here,
    // block 7 runs after the chain.  A block's tile is issued two steps before its use, and each
    // step's counted wait (the next weight chunk, issued after it) covers it: vmcnt is in-order.
    // Wave w = bottleneck column tile w (x 4 row tiles), and for w < 4 the (row tile w, ve) tile +
    // row tile w's bias.
    const int64_t wb0 = item * (WGS / TM);  // the item's first wave block
    auto bt_src = [&](int b) { return A.act[A_BT] + (wb0 + b) * A.bstride[A_BT] + wave * (int64_t)HB_TILE; };
    hd_dma_tile(bt_src(0), xbuf);
    hd_dma_tile(bt_src(1), xbuf + HB_TILE);
    auto dw_block = [&](int b) {
      const char* xt = xbuf + (b & 1) * HB_TILE;
      const char* zt = stage + b * (4 * HB_TILE);  // wave b's dz_g tiles = wave block b of the item
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 bx = hb_tr_frag(xt, kk);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          gacc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hb_tr_frag(zt + mt * HB_TILE, kk), bx, gacc[mt], 0, 0, 0);
        if (wave < 4) {
          const bf16x8 a = hb_tr_frag(zt + wave * HB_TILE, kk);
          gacc[4] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, hb_tr_frag(vet + b * HB_TILE, kk), gacc[4], 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 8; ++e) gdb += (float)a[e];
        }
      }
    };
    auto lg_step = [&](int i) -> int {
      if (i < 1) {
        // the next item's adjoint inputs (rec_lds and nray are free: read before the Lr^T chain)
        const int64_t nx = item + gridDim.x;
        return (A.points == 0 && nx < n_items) ? hd_stage_adjoint(A, nx, wave, (char*)rec_lds, nray) : 0;
      }
      dw_block(i - 1);
      int n = 0;
      if (i + 1 >= 8) return n;
      // the slot's previous tile (block i - 1) is consumed: its reads fed the MFMAs above
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0), vmcnt / expcnt untouched
      asm volatile("" ::: "memory");
      hd_dma_tile(bt_src(i + 1), xbuf + ((i + 1) & 1) * HB_TILE);
      return n + 2;
    };
    bwd_layer_run<MODE, 1, 1, WIDTH_COND / T::KI, 1, true, true, true>(A, lds, sample, xa, xb, 0, D_ZB8, NoTileHook{},
                                                                       lg_step, gc + 1);
    gc += 1 + bwd_tiles(MODE, 1);
    // sigma's dz: one bf16 per sample in its own array (A.sigma_dz, den_geom.h D_ZB8)
    if (grp == 0) {
      const int64_t wb = __builtin_amdgcn_readfirstlane((int)(sample / TM));
      *(__bf16*)(A.sigma_dz + wb * 64 + c * 2) = (__bf16)g4[0];
    }
    HD_T(4);
    // block 7 (its tile was issued in step 5; step 7's wait covered it)
    dw_block(7);
    HD_T(5);
  }
  // drain (nothing of ours in flight past here but the wrapped chunk DMA of a non-existent item)
  __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (0 << 8));
  __syncthreads();
  DEN_CLOCK_END(1);
#ifdef DEN_HEAD_PROF
  prof[6] = __builtin_amdgcn_s_memtime() - t_start;
  prof[7] = (n_items - blockIdx.x + gridDim.x - 1) / gridDim.x;
  if (blockIdx.x < 256 && (threadIdx.x & 63) == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) den_head_prof[(blockIdx.x * 8 + wave) * 8 + q] = prof[q];
  }
#endif

  const int lane = threadIdx.x & 63;
  // ---- Lr partial (as render_bwd_kernel<1, 1>), through the weight ring
  {
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
      A0.lr_partial[(int64_t)blockIdx.x * LR_PART + e] = v;
    }
  }
  // ---- Lg partial [wg][mt][nt][lane][16], nt = 9 the bias (den_dwstream.hip's layout)
  constexpr int NT = 9;
  float* base = lg_partial + (int64_t)blockIdx.x * 4 * (NT + 1) * 1024;
  auto put = [&](int mt, int nt, const f32x16& acc) {
    float* o = base + ((int64_t)mt * (NT + 1) + nt) * 1024 + lane * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
      *(f32x4*)(o + 4 * q) = v;
    }
  };
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) put(mt, wave, gacc[mt]);
  if (wave < 4) {
    put(wave, 8, gacc[4]);
    // lane l holds feature (l & 31) of row tile `wave` (two lane halves: samples 8 (l >> 5) ..)
    const float bsum = gdb + __shfl_xor(gdb, 32, 64);
    float* o = base + ((int64_t)wave * (NT + 1) + NT) * 1024;
    if (lane < 32) {
      const int m = lane;
      o[(32 * ((m >> 2) & 1)) * 16 + (m & 3) + 4 * (m >> 3)] = bsum;
    }
  }
}

}  // namespace den
