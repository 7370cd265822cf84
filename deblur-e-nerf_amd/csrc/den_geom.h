// den_geom.h -- MLP geometry, MFMA fragment maps and packed-weight layout,
// shared by host code (packing offsets, workspace sizing) and kernels.
//
// The network is the reference's `mlp` arch (external/mlp.py:126-205,
// 246-358; configs/train/synthetic.yaml:104-114):
//   L0..L7  : 8 hidden Linear(256) + softplus(beta=100), skip concat of the
//             positional encoding after L4 (L5 input = [h4, pe])
//   Lb      : bottleneck Linear(256, no act) fused with the sigma head
//             (row 256 of Lb = sigma_layer)
//   Lg      : rgb hidden Linear([bott, ve] -> 128) + softplus(beta=100)
//   Lr      : rgb output Linear(128 -> rd) + softplus(beta=1)
//
// Layout conventions (both arithmetic modes):
// * activations are "feature tiles" of TM rows; a wave holds TN samples.
// * an MFMA accumulator tile (rows = features, cols = samples) becomes the B
//   operand of the next layer without data movement; the resulting k-order
//   permutation is baked into the packed weights (chain_feature()).
// * activations stored to HBM keep each lane group's accumulator registers
//   contiguous: stored position q within a tile <-> tile row stored_to_row(q).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define DEN_HD __host__ __device__ __forceinline__
#else
#define DEN_HD inline
#endif

namespace den {

constexpr int NL = 11;          // forward layers L0..L7, Lb, Lg, Lr
constexpr int L_B = 8, L_G = 9, L_R = 10;
constexpr int WIDTH = 256, WIDTH_COND = 128;
constexpr int PE_DIM = 63, VE_DIM = 27;  // 3*(1+2*10), 3*(1+2*4)
constexpr int PE_PAD = 64, VE_PAD = 32;

// ---------------------------------------------------------------- modes
// mode 0 = F32  : v_mfma_f32_16x16x4_f32, TM = TN = 16, KI = 4, 4 lane groups
// mode 1 = BF16 : v_mfma_f32_32x32x16_bf16, TM = TN = 32, KI = 16, 2 lane groups
DEN_HD constexpr int tm_of(int mode) { return mode == 0 ? 16 : 32; }
DEN_HD constexpr int ki_of(int mode) { return mode == 0 ? 4 : 16; }
DEN_HD constexpr int es_of(int mode) { return mode == 0 ? 4 : 2; }   // operand element bytes
DEN_HD constexpr int wave_samples(int mode) { return tm_of(mode); }
DEN_HD constexpr int waves_per_wg() { return 8; }
DEN_HD constexpr int wg_samples(int mode) { return 8 * tm_of(mode); }  // 128 (F32) / 256 (BF16)

DEN_HD constexpr int round_up(int x, int m) { return (x + m - 1) / m * m; }

// forward layer input width (padded, chain order) and output rows (padded)
DEN_HD constexpr int fwd_K(int mode, int l) {
  return l == 0 ? PE_PAD : l == 5 ? WIDTH + PE_PAD : l == L_G ? WIDTH + VE_PAD : l == L_R ? WIDTH_COND : WIDTH;
}
DEN_HD constexpr int fwd_M(int mode, int l) {
  return l < 8 ? WIDTH : l == L_B ? round_up(WIDTH + 1, tm_of(mode)) : l == L_G ? WIDTH_COND : tm_of(mode);
}
DEN_HD constexpr int fwd_tiles(int mode, int l) { return fwd_M(mode, l) / tm_of(mode); }
DEN_HD constexpr int fwd_ksteps(int mode, int l) { return fwd_K(mode, l) / ki_of(mode); }
// bytes of one packed row tile (TM rows x K) -- identical formula for both modes
DEN_HD constexpr int chunk_bytes_K(int K) { return 64 * K; }

DEN_HD constexpr int fwd_chunk_index(int mode, int l) {
  int c = 0;
  for (int i = 0; i < l; ++i) c += fwd_tiles(mode, i);
  return c;
}
DEN_HD constexpr int fwd_nchunks(int mode) { return fwd_chunk_index(mode, NL); }
DEN_HD constexpr int64_t fwd_layer_offset(int mode, int l) {
  int64_t o = 0;
  for (int i = 0; i < l; ++i) o += (int64_t)fwd_tiles(mode, i) * chunk_bytes_K(fwd_K(mode, i));
  return o;
}
DEN_HD constexpr int64_t fwd_bytes(int mode) { return fwd_layer_offset(mode, NL); }

// backward (transposed) layers, in execution order j = 0..9:
//   j=0 Lr^T, 1 Lg^T, 2 Lb^T, 3 L7^T, 4 L6^T, 5 L5^T, 6 L4^T, 7 L3^T, 8 L2^T, 9 L1^T
constexpr int NBL = 10;
DEN_HD constexpr int bwd_layer(int j) { return j == 0 ? L_R : j == 1 ? L_G : j == 2 ? L_B : 10 - j; }
DEN_HD constexpr int bwd_rows(int mode, int j) { return j == 0 ? WIDTH_COND : WIDTH; }
DEN_HD constexpr int bwd_K(int mode, int j) { return fwd_M(mode, bwd_layer(j)); }
DEN_HD constexpr int bwd_tiles(int mode, int j) { return bwd_rows(mode, j) / tm_of(mode); }
DEN_HD constexpr int64_t bwd_layer_offset(int mode, int j) {
  int64_t o = 0;
  for (int i = 0; i < j; ++i) o += (int64_t)bwd_tiles(mode, i) * chunk_bytes_K(bwd_K(mode, i));
  return o;
}
DEN_HD constexpr int64_t bwd_bytes(int mode) { return bwd_layer_offset(mode, NBL); }

// packed biases: TM floats per forward row tile, in stored order
DEN_HD constexpr int64_t bias_floats(int mode) { return (int64_t)fwd_nchunks(mode) * tm_of(mode); }

// ---------------------------------------------------------------- fragment maps
// Accumulator row held by lane group `grp`, register `r` (within a TM tile).
DEN_HD constexpr int acc_row(int mode, int grp, int r) {
  return mode == 0 ? 4 * grp + r : (r & 3) + 8 * (r >> 2) + 4 * grp;
}
// Stored position q within a tile: lane group grp writes its REGS registers contiguously.
DEN_HD constexpr int stored_to_row(int mode, int q) {
  return mode == 0 ? q : acc_row(1, q >> 4, q & 15);
}
DEN_HD constexpr int row_to_stored(int mode, int row) {
  // inverse of stored_to_row
  return mode == 0 ? row : (16 * ((row >> 2) & 1) + ((row & 3) + 4 * (row >> 3)));
}
// Input feature (chain order) consumed at k-step kappa, k-slot (lane group grp, element j).
// BF16: element j of lane half h in k-step 2p+s <- acc reg 8s+j of tile p.
// F32 : lane group g in k-step 4p+r <- acc reg r of tile p.
DEN_HD constexpr int chain_feature(int mode, int kappa, int grp, int j) {
  return mode == 0 ? 16 * (kappa >> 2) + acc_row(0, grp, kappa & 3)
                   : 32 * (kappa >> 1) + acc_row(1, grp, 8 * (kappa & 1) + j);
}

// ---------------------------------------------------------------- flat parameter buffer
// Reference named_parameters() order under nerf.radiance_field (mlp.py):
//  0..15 base.hidden_layers.{0..7}.{weight,bias}, 16/17 sigma_layer.output_layer,
//  18/19 bottleneck_layer.output_layer, 20/21 rgb_layer.hidden_layers.0,
//  22/23 rgb_layer.output_layer
DEN_HD constexpr int ref_out(int t, int rd) {  // t = tensor pair index 0..11
  return t < 8 ? WIDTH : t == 8 ? 1 : t == 9 ? WIDTH : t == 10 ? WIDTH_COND : rd;
}
DEN_HD constexpr int ref_in(int t) {
  return t == 0 ? PE_DIM : t == 5 ? WIDTH + PE_DIM : t < 8 ? WIDTH : t == 8 || t == 9 ? WIDTH
         : t == 10 ? WIDTH + VE_DIM : WIDTH_COND;
}
DEN_HD constexpr int64_t param_offset(int rd, int idx) {
  int64_t o = 0;
  for (int i = 0; i < idx; ++i) {
    int t = i >> 1;
    o += (i & 1) ? ref_out(t, rd) : (int64_t)ref_out(t, rd) * ref_in(t);
  }
  return o;
}
DEN_HD constexpr int64_t param_count(int rd) { return param_offset(rd, 24); }

// Map a padded forward (layer l, out row o, chain input feature f) to the
// reference tensor pair t and (row, col); returns false for padding.
DEN_HD bool ref_coord(int l, int o, int f, int rd, int* t, int* row, int* col) {
  int tt, rr, cc;
  if (l < 8) {
    tt = l; rr = o;
    if (l == 0) { if (f >= PE_DIM) return false; cc = f; }
    else if (l == 5) { if (f >= WIDTH + PE_DIM) return false; cc = f; }
    else cc = f;
  } else if (l == L_B) {
    if (o < WIDTH) { tt = 9; rr = o; }
    else if (o == WIDTH) { tt = 8; rr = 0; }
    else return false;
    cc = f;
  } else if (l == L_G) {
    tt = 10; rr = o;
    if (f >= WIDTH + VE_DIM) return false;
    cc = f;
  } else {
    tt = 11; rr = o;
    if (o >= rd) return false;
    cc = f;
  }
  *t = tt; *row = rr; *col = cc;
  return true;
}
DEN_HD bool ref_bias_coord(int l, int o, int rd, int* t, int* row) {
  int dummy_col;
  return ref_coord(l, o, 0, rd, t, row, &dummy_col);
}

// ---------------------------------------------------------------- BF16 activation scaling
// In BF16 mode softplus(beta=100) is evaluated in base 2 on t = K*z with
// K = 100*log2(e):  s' = log2(1 + 2^t) = K * softplus_100(z).  K is folded into
// the packed weights/biases (W' = col_scale * W, b' = bias_scale * b), so the
// epilogue is v_exp + v_log + 3 VALU.  Activations kept for the backward are
// in these scaled units; the weight-gradient reduction multiplies by the same
// factors (dL/dW = col_scale * dL/dW').  F32 mode uses scale 1 (exact path).
constexpr double KAPPA = 144.26950408889634;  // 100 / ln 2
DEN_HD double col_scale(int mode, int l, int f) {
  if (mode == 0) return 1.0;
  if (l == 0) return KAPPA;                       // pe input
  if (l < 8) return (l == 5 && f >= WIDTH) ? KAPPA : 1.0;
  if (l == L_B || l == L_R) return 1.0 / KAPPA;   // consume K-scaled activations, identity / softplus(1) out
  return KAPPA;                                   // L_G: [bottleneck, ve] raw inputs, softplus(100) out
}
DEN_HD double bias_scale(int mode, int l) {
  if (mode == 0) return 1.0;
  return (l == L_B || l == L_R) ? 1.0 : KAPPA;
}

// ---------------------------------------------------------------- workspace (render)
// Activation tensors kept for the backward, each [n_samples][width] in the
// operand dtype, stored order within tiles.
// dz of [bottleneck | sigma] and of the rgb head are padded to whole 32-wide
// tiles in both modes (the weight-gradient GEMM works on 32x32 tiles).
constexpr int DZB_W = 288, DZR_W = 32;
enum ActId { A_PE = 0, A_S0 = 1, /* S0..S7 = 1..8 */ A_BT = 9, A_VE = 10, A_G = 11,
             D_Z0 = 12, /* DZ0..DZ7 = 12..19 */ D_ZB = 20, D_ZG = 21, D_ZR = 22, NACT = 23 };
// The layer-major BF16 path (render_head_bwd_kernel -> hidden_bwd_kernel<true>) keeps dz_b as 8 tiles
// per wave block (the bottleneck's 256; act_ptr's pseudo id D_ZB8) and sigma's dz as one bf16 per sample
// in an array of its own: the Lb launch then streams dz_b exactly as the other hidden launches stream
// dz -- with the 288-wide layout its dz read skipped a 2 KiB sigma tile per block and read 64 B of it.
constexpr int D_ZB8 = NACT;
// Block-major rows (r06; ws_layout in den_api.hip): in the layer-major BF16 training layout the
// activations the hidden launches stream live in one row per wave block -- S_l in 16 KiB slot l
// (l = 0..7), dz_l over S_{l+1} (l = 0..6; dz_7 in slot 8) and dz_b's 8 tiles (D_ZB8) in slot 9 -- so
// each of those launches reads and writes within one SROW_BYTES row (profiles/stream_probe: 6.23 TB/s
// for a hidden launch's pattern there, 5.1-5.8 TB/s for three tensors 8 GiB apart).  The bottleneck
// and G, which only the head backward reads, stay contiguous (in the rows too: the same step time, the
// head 0.17 ms slower and the hidden launches 0.025 ms faster, profiles/r06ac_ab.jsonl).  Every other
// layout keeps contiguous tensors; kernels address a wave block through the per-activation block
// stride of their arguments.
constexpr int64_t SROW_BYTES = 10 * 16384;
DEN_HD constexpr int64_t srow_offset(int a) {
  return (a >= A_S0 && a <= A_S0 + 7) ? (int64_t)(a - A_S0) * 16384
       : (a >= D_Z0 && a <= D_Z0 + 7) ? (int64_t)(a - D_Z0 + 1) * 16384 : a == D_ZB8 ? 9 * 16384 : -1;
}
DEN_HD constexpr int act_width(int mode, int a) {
  return a == A_PE ? PE_PAD : a <= 8 ? WIDTH : a == A_BT ? WIDTH : a == A_VE ? VE_PAD : a == A_G ? WIDTH_COND
       : a <= 19 ? WIDTH : a == D_ZB ? DZB_W : a == D_ZG ? WIDTH_COND : DZR_W;
}

}  // namespace den
