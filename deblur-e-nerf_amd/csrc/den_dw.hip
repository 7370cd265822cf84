// den_dw.hip -- weight/bias gradients of the fused MLP:
//   dW_l[o][i] = sum_n dz_l[n][o] * x_l[n][i],   db_l[o] = sum_n dz_l[n][o]
// a GEMM whose contraction runs over all ray samples (16.8M at the benchmark
// size).  Split-K over samples: workgroup s owns a contiguous sample range
// and the WHOLE (M x N) output of the layer, so every byte of dz and x is read
// from HBM exactly once.  One wave per 32-row tile of dz; each wave keeps all
// N/32 column tiles (+ one all-ones tile that yields db) in accumulators.
// Partials are reduced deterministically by dw_reduce_kernel, which also undoes
// the stored-order permutation and scatters into the reference's flat
// parameter layout (den_geom.h param_offset).
//
// BF16: v_mfma_f32_32x32x16_bf16, operands with samples as k read from a
//       row-major [sample][feature] LDS image by ds_read_b64_tr_b16.
// F32 : v_mfma_f32_32x32x2_f32, plain ds_read_b32 fragments.
#include "den_device.h"

namespace den {

typedef short v4i16 __attribute__((ext_vector_type(4)));

// Operands are wave-block-major activation tensors (den_geom.h): [n / TN][tiles][TM x TN tile],
// BF16 tile = [frag f][lane c + 32h][8] (stored positions 16h + 8f + j), F32 tile = [lane c + 16g][4].
struct DwArgs {
  const char* A;       // dz tensor; the GEMM uses its tiles [a_t0, a_t0 + M / TM)
  int a_tiles;         // tiles per wave block of the dz tensor
  int a_t0;
  const char* B1;      // x  (N1 / TM tiles per wave block)
  const char* B2;      // x' (N2 / TM tiles, second input segment; null when N2 = 0)
  int64_t n;           // samples
  int64_t per_split;   // samples per split (multiple of 32)
  float* partial;      // [splits][MT][NT+1][64 lanes][16]
};

// 16-byte unit v (memory order) of the DW_BK-sample chunk starting at sample k0 of a tensor with
// `tiles` tiles per wave block, restricted to tiles [t0, t0 + nt): source byte offset and the
// (row = sample in chunk, column = stored feature) it lands at in the row-major LDS image.
template <int MODE, int DW_BK>
__device__ __forceinline__ int64_t dw_unit(int v, int nt, int tiles, int t0, int64_t k0, int* row, int* col) {
  if constexpr (MODE == 1) {
    const int t = v / (4 * DW_BK), r = v % (4 * DW_BK);
    const int f = r / (2 * DW_BK), r2 = r % (2 * DW_BK);
    const int h = r2 / DW_BK, cl = r2 % DW_BK;
    *row = cl;
    *col = 32 * t + 16 * h + 8 * f;
    return ((k0 / 32) * tiles + t0 + t) * 2048 + f * 1024 + ((int)(k0 % 32) + cl + 32 * h) * 16;
  } else {
    const int jb = v / (nt * 64), r = v % (nt * 64);
    const int t = r / 64, ln = r % 64;
    *row = 16 * jb + (ln & 15);
    *col = 16 * t + 4 * (ln >> 4);
    return ((k0 / 16 + jb) * tiles + t0 + t) * 1024 + ln * 16;
  }
}

constexpr int DW_BK_MAX = 32;  // samples per LDS stage (16 for register-heavy shapes)

template <int MODE>
DEN_HD constexpr int dw_pad_bytes(int W) {
  // BF16: choose the row pitch so that 4 consecutive rows start 16 banks apart
  // (conflict-free transposed reads); F32 reads are conflict-free for any pitch.
  return MODE == 1 ? 4 * (((16 - (W / 2)) % 64 + 64) % 64) : 16;
}

// WN waves per 32-row tile of dz split its N/32 column tiles (narrow layers: rgb output, M = 32).
template <int MODE, int MT, int N1, int N2, int WN>
__global__ __launch_bounds__(64 * MT * WN) void dw_gemm_kernel(DwArgs P) {
  constexpr int M = 32 * MT, N = N1 + N2, NT = N / 32;
  static_assert(NT % WN == 0, "column tiles split evenly over the waves of a row tile");
  constexpr int NTG = NT / WN;  // column tiles per wave
  constexpr int DW_BK = (NT + 1) * 16 > 160 ? 16 : 32;
  constexpr int ES = es_of(MODE);
  constexpr int PA = M * ES + dw_pad_bytes<MODE>(M), PB = N * ES + dw_pad_bytes<MODE>(N);
  constexpr int IMG = DW_BK * (PA + PB);
  constexpr int THREADS = 64 * MT * WN;
  constexpr int TMm = tm_of(MODE);
  constexpr int NTA = M / TMm, NT1 = N1 / TMm, NT2 = N2 / TMm;  // tiles per segment
  // 16-B units of a chunk per segment (4 per sample and tile in both modes), in memory order
  constexpr int SA = DW_BK * NTA * 4, SB1 = DW_BK * NT1 * 4, SB2 = DW_BK * NT2 * 4;
  constexpr int UNITS = SA + SB1 + SB2;
  constexpr int UPT = (UNITS + THREADS - 1) / THREADS;
  __shared__ __attribute__((aligned(16))) char lds[2 * IMG];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int mt = wave % MT, cg = wave / MT;  // row tile, column group
  const int64_t k_begin = (int64_t)blockIdx.x * P.per_split;
  const int64_t k_end = min(P.n, k_begin + P.per_split);
  const int nchunks = (int)((k_end - k_begin + DW_BK - 1) / DW_BK);

  f32x16 acc[NTG + 1];
#pragma unroll
  for (int t = 0; t <= NTG; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;

  // unit u of a chunk -> global source and LDS destination (consecutive threads read consecutive
  // 16 B of the wave-block-major tensors; the LDS image stays row-major [sample][stored feature])
  auto unit = [&](int u, int64_t k0, const char** src, char** dst, char* img) {
    int row, col;
    if (u < SA) {
      *src = P.A + dw_unit<MODE, DW_BK>(u, NTA, P.a_tiles, P.a_t0, k0, &row, &col);
      *dst = img + row * PA + col * ES;
    } else if (u < SA + SB1) {
      *src = P.B1 + dw_unit<MODE, DW_BK>(u - SA, NT1, NT1, 0, k0, &row, &col);
      *dst = img + DW_BK * PA + row * PB + col * ES;
    } else {
      *src = P.B2 + dw_unit<MODE, DW_BK>(u - SA - SB1, NT2, NT2, 0, k0, &row, &col);
      *dst = img + DW_BK * PA + row * PB + (N1 + col) * ES;
    }
    return row;
  };
  uint4 st[UPT];
  auto load = [&](int ch) {
    const int64_t k0 = k_begin + (int64_t)ch * DW_BK;
#pragma unroll
    for (int q = 0; q < UPT; ++q) {
      int u = q * THREADS + threadIdx.x;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (u < UNITS) {
        const char* src;
        char* dst;
        const int row = unit(u, k0, &src, &dst, lds);
        if (k0 + row < k_end) v = MODE == 1 ? ld_stream((const uint4*)src) : *(const uint4*)src;
      }
      st[q] = v;
    }
  };
  auto store = [&](int slot) {
    char* img = lds + slot * IMG;
#pragma unroll
    for (int q = 0; q < UPT; ++q) {
      int u = q * THREADS + threadIdx.x;
      if (u < UNITS) {
        const char* src;
        char* dst;
        unit(u, 0, &src, &dst, img);
        *(uint4*)dst = st[q];
      }
    }
  };

  if (nchunks > 0) {
    load(0);
    store(0);
  }
  __syncthreads();

  for (int ch = 0; ch < nchunks; ++ch) {
    const bool more = ch + 1 < nchunks;
    if (more) load(ch + 1);
    const char* imgA = lds + (ch & 1) * IMG;
    const char* imgB = imgA + DW_BK * PA;
    if constexpr (MODE == 1) {
      // ones fragment (bf16 1.0 = 0x3f80)
      bf16x8 ones;
#pragma unroll
      for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
      const int q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1, h = lane >> 5;
#pragma unroll
      for (int kk = 0; kk < DW_BK / 16; ++kk) {
        const int row0 = kk * 16 + 8 * h + q;
        auto tr_frag = [&](const char* img, int pitch, int col0) {
          const char* a0 = img + row0 * pitch + (col0 + 16 * g1 + 4 * p) * 2;
          v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a0);
          v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(a0 + 4 * pitch));
          bf16x8 f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f[j] = __builtin_bit_cast(__bf16, (short)lo[j]);
            f[4 + j] = __builtin_bit_cast(__bf16, (short)hi[j]);
          }
          return f;
        };
        bf16x8 a = tr_frag(imgA, PA, 32 * mt);
#pragma unroll
        for (int t = 0; t < NTG; ++t) {
          bf16x8 b = tr_frag(imgB, PB, 32 * (cg * NTG + t));
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t], 0, 0, 0);
        }
        acc[NTG] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, ones, acc[NTG], 0, 0, 0);
      }
    } else {
      const int c = lane & 31, h = lane >> 5;
#pragma unroll 4
      for (int kk = 0; kk < DW_BK / 2; ++kk) {
        const int row = 2 * kk + h;
        float a = *(const float*)(imgA + row * PA + (32 * mt + c) * 4);
#pragma unroll
        for (int t = 0; t < NTG; ++t) {
          float b = *(const float*)(imgB + row * PB + (32 * (cg * NTG + t) + c) * 4);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
        }
        acc[NTG] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, 1.0f, acc[NTG], 0, 0, 0);
      }
    }
    if (more) store((ch + 1) & 1);
    __syncthreads();
  }

  float* out = P.partial + (((int64_t)blockIdx.x * MT + mt) * (NT + 1)) * 1024;
#pragma unroll
  for (int t = 0; t <= NTG; ++t) {
    if (t == NTG && cg != 0) break;  // the ones (bias) tile is column group 0's
    f32x4* o4 = (f32x4*)(out + (t == NTG ? NT : cg * NTG + t) * 1024 + lane * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
      o4[q] = v;
    }
  }
}

// Reduce over splits + scatter into the flat parameter gradient.
// Element e of the [MT][NT+1][64][16] block: tile (mt, nt), lane, reg.
struct DwReduceArgs {
  const float* partial;
  int splits, MT, NT;
  int m_off;       // chain-feature offset of A's first column (stored order)
  int layer;       // forward layer id (den_geom.h)
  int mode;        // chain mode (stored-order permutation)
  int rd;
  int n1;          // width of the first input segment (features of x before the second segment)
  int n1_feat;     // chain-feature offset of the second segment (e.g. 256 for [h4, pe])
  int bias;        // 0: skip the ones tile (the bias gradient is written by another launch)
  float* grad;     // flat params layout
  int64_t split_stride;  // floats between consecutive splits' partials (0: MT * (NT + 1) * 1024)
  int64_t first;         // float offset of this reduction's first tile inside a split's partial
};

// One workgroup = DWR_EL consecutive partial elements x DWR_SG split groups (one wave each: every
// load instruction reads 256 consecutive bytes).  Wave g sums splits g, g + DWR_SG, ... through
// DWR_UNROLL independent accumulators (that many loads in flight per lane), the groups are combined
// in a fixed order: deterministic.  (One thread per element walking all splits serially ran at
// ~1 TB/s: 69 us per hidden layer of 256 x 288 KB partials.)
constexpr int DWR_EL = 64, DWR_SG = 4, DWR_UNROLL = 16;
// partial element e ([MT][NT + 1][64][16]: tile, lane, register) of sum s -> the flat gradient
__device__ void dw_scatter(const DwReduceArgs& R, int64_t e, float s);
constexpr int DWR_THREADS = DWR_EL * DWR_SG;

__global__ __launch_bounds__(DWR_THREADS) void dw_reduce_kernel(DwReduceArgs R) {
  const int64_t per = (int64_t)R.MT * (R.NT + 1) * 1024;
  const int64_t stride = R.split_stride > 0 ? R.split_stride : per;
  const int el = threadIdx.x % DWR_EL, g = threadIdx.x / DWR_EL;
  const int64_t e = (int64_t)blockIdx.x * DWR_EL + el;
  const bool live = e < per;
  const float* src = R.partial + R.first + (live ? e : 0);
  float acc[DWR_UNROLL];
#pragma unroll
  for (int u = 0; u < DWR_UNROLL; ++u) acc[u] = 0.0f;
  int sp = g;
  for (; sp + (DWR_UNROLL - 1) * DWR_SG < R.splits; sp += DWR_UNROLL * DWR_SG) {
#pragma unroll
    for (int u = 0; u < DWR_UNROLL; ++u) acc[u] += src[(int64_t)(sp + u * DWR_SG) * stride];
  }
#pragma unroll
  for (int u = 0; u < DWR_UNROLL; ++u)
    if (sp + u * DWR_SG < R.splits) acc[u] += src[(int64_t)(sp + u * DWR_SG) * stride];
#pragma unroll
  for (int w = DWR_UNROLL / 2; w > 0; w /= 2)
#pragma unroll
    for (int u = 0; u < w; ++u) acc[u] += acc[u + w];
  __shared__ float red[DWR_SG][DWR_EL];
  red[g][el] = acc[0];
  __syncthreads();
  if (g != 0 || !live) return;
  float s = red[0][el];
#pragma unroll
  for (int q = 1; q < DWR_SG; ++q) s += red[q][el];
  dw_scatter(R, e, s);
}

// Fused Lr weight gradient (render_bwd_kernel<1, 1>, den_render.hip): one LR_PART-float partial per
// render workgroup, [tile t][ch][32 columns] + bias[ch] + pad.  Stage 1: workgroup y sums partials
// y, y + G1, ... (one thread per element, eight loads in flight, fixed order); stage 2 sums the G1
// stage-1 rows in order and scatters like dw_reduce_kernel (MT 1, NT 4: element (t, ch, col) is
// register ch of lane col in column tile t; bias ch is register ch of lane 0 in the ones tile).
constexpr int LRP = 388;  // = LR_PART
__global__ __launch_bounds__(448) void lr_reduce1_kernel(const float* part, int64_t n_wg, int G1, float* st1) {
  const int e = threadIdx.x;
  if (e >= LRP) return;
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.0f;
  int64_t sp = blockIdx.x;
  for (; sp + 7LL * G1 < n_wg; sp += 8LL * G1) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += part[(sp + (int64_t)u * G1) * LRP + e];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (sp + (int64_t)u * G1 < n_wg) acc[u] += part[(sp + (int64_t)u * G1) * LRP + e];
  float v = acc[0];
#pragma unroll
  for (int u = 1; u < 8; ++u) v += acc[u];
  st1[(int64_t)blockIdx.x * LRP + e] = v;
}

// stage 2: workgroup e (one per element): thread t sums rows t, t + 256, ... then a fixed-order tree
__global__ __launch_bounds__(256) void lr_reduce2_kernel(const float* st1, int G1, DwReduceArgs R) {
  const int e = blockIdx.x, t = threadIdx.x;
  float v = 0.0f;
  for (int y = t; y < G1; y += 256) v += st1[(int64_t)y * LRP + e];
  __shared__ float red[256];
  red[t] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t != 0) return;
  v = red[0];
  int nt, lane, reg;
  if (e < 384) {
    nt = e / 96;
    reg = (e % 96) / 32;
    lane = e % 32;
  } else {
    nt = 4;
    reg = e - 384;
    lane = 0;
  }
  dw_scatter(R, ((int64_t)nt << 10) + lane * 16 + reg, v);
}

__device__ void dw_scatter(const DwReduceArgs& R, int64_t e, float s) {
  const int reg = (int)(e & 15), lane = (int)((e >> 4) & 63);
  const int64_t tile = e >> 10;
  const int nt = (int)(tile % (R.NT + 1)), mt = (int)(tile / (R.NT + 1));
  const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5), col = lane & 31;
  // stored position -> chain feature (per TM-wide tile of the chain mode)
  const int TMc = tm_of(R.mode);
  const int m = R.m_off + 32 * mt + row;
  const int o = (m / TMc) * TMc + stored_to_row(R.mode, m % TMc);
  int t, rr, cc;
  if (nt == R.NT) {  // ones tile -> bias gradient (column 0 only)
    if (col != 0 || !R.bias) return;
    if (!ref_bias_coord(R.layer, o, R.rd, &t, &rr)) return;
    R.grad[param_offset(R.rd, 2 * t + 1) + rr] = R.mode == 0 ? s : (float)((double)s * bias_scale(R.mode, R.layer));
    return;
  }
  const int n = 32 * nt + col;
  int f;
  if (n < R.n1) f = (n / TMc) * TMc + stored_to_row(R.mode, n % TMc);
  else {
    int n2 = n - R.n1;
    f = R.n1_feat + (n2 / TMc) * TMc + stored_to_row(R.mode, n2 % TMc);
  }
  if (!ref_coord(R.layer, o, f, R.rd, &t, &rr, &cc)) return;
  R.grad[param_offset(R.rd, 2 * t) + (int64_t)rr * ref_in(t) + cc] =
      R.mode == 0 ? s : (float)((double)s * col_scale(R.mode, R.layer, f));
}

template __global__ void dw_gemm_kernel<1, 8, 64, 0, 1>(DwArgs);
template __global__ void dw_gemm_kernel<1, 8, 256, 0, 1>(DwArgs);
template __global__ void dw_gemm_kernel<1, 8, 256, 64, 1>(DwArgs);
template __global__ void dw_gemm_kernel<1, 1, 256, 0, 4>(DwArgs);
template __global__ void dw_gemm_kernel<1, 4, 256, 32, 1>(DwArgs);
template __global__ void dw_gemm_kernel<1, 1, 128, 0, 4>(DwArgs);
template __global__ void dw_gemm_kernel<0, 8, 64, 0, 1>(DwArgs);
template __global__ void dw_gemm_kernel<0, 8, 256, 0, 1>(DwArgs);
template __global__ void dw_gemm_kernel<0, 8, 256, 64, 1>(DwArgs);
template __global__ void dw_gemm_kernel<0, 1, 256, 0, 4>(DwArgs);
template __global__ void dw_gemm_kernel<0, 4, 256, 32, 1>(DwArgs);
template __global__ void dw_gemm_kernel<0, 1, 128, 0, 4>(DwArgs);

}  // namespace den
