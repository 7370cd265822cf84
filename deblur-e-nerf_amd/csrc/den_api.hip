// den_api.hip -- C ABI of libden.so (declared in include/den_api.h).
// Single translation unit: includes every kernel file.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/den_api.h"
#include "den_dw.hip"
#include "den_events.hip"
#include "den_hidden.hip"
#include "den_dwstream.hip"
#include "den_march.hip"
#include "den_misc.hip"
#include "den_ngp.hip"
#include "den_ngp_mfma.hip"
#include "den_pixbw.hip"
#include "den_render.hip"
#include "den_head_bwd.hip"
#include "den_raygrad.hip"
#include "den_sh.hip"
#include "den_dataset.hip"
#include "den_eval.hip"

using namespace den;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define DEN_HIP(call)                                                                               \
  do {                                                                                              \
    hipError_t e_ = (call);                                                                         \
    if (e_ != hipSuccess) return fail(DEN_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)
// DEN_SYNC_CHECK=1 (debugging only; breaks stream capture): every launch is followed by a device
// synchronisation, so an asynchronous fault is reported at the launch that caused it (source line)
inline bool sync_check() {
  static const bool on = [] {
    const char* e = std::getenv("DEN_SYNC_CHECK");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
#define DEN_LAUNCHED()                                                                                  \
  do {                                                                                                  \
    hipError_t e_ = hipGetLastError();                                                                  \
    if (e_ == hipSuccess && sync_check()) e_ = hipDeviceSynchronize();                                  \
    if (e_ != hipSuccess)                                                                               \
      return fail(DEN_EHIP, std::string("launch (den_api.hip:") + std::to_string(__LINE__) + "): " +   \
                                hipGetErrorString(e_));                                                 \
  } while (0)

// ---- kernel timing (measurement only; bench.py).  When enabled, each render-path launch is
// bracketed by a pair of hipEvents recorded on the launch stream itself.
enum { T_RENDER_FWD = 0, T_RENDER_BWD = 1, T_HIDDEN_BWD = 2, T_DW_GEMM = 3, T_DW_REDUCE = 4, T_HIDDEN_LB = 5, T_NCLASS = 6 };
struct TimingRec {
  int cls;
  hipEvent_t a, b;
};
bool g_timing = false;
std::mutex g_timing_mu;
std::vector<TimingRec> g_timing_recs;

struct TimedLaunch {
  TimingRec r{};
  hipStream_t s;
  bool on;
  TimedLaunch(int cls, hipStream_t st) : s(st), on(g_timing) {
    if (!on) return;
    r.cls = cls;
    on = hipEventCreate(&r.a) == hipSuccess && hipEventCreate(&r.b) == hipSuccess &&
         hipEventRecord(r.a, s) == hipSuccess;
  }
  ~TimedLaunch() {
    if (!on) return;
    (void)hipEventRecord(r.b, s);
    std::lock_guard<std::mutex> g(g_timing_mu);
    g_timing_recs.push_back(r);
  }
};
#define DEN_TIMED(cls, s) TimedLaunch timed_##cls##_(cls, s)

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }



struct WsLayout {
  size_t act[NACT];
  int64_t bstride[NACT + 1];  // bytes from one wave block of each activation (and D_ZB8) to the next
  size_t sigma_dz;            // layer-major BF16: sigma's dz, one bf16 per sample (den_geom.h D_ZB8)
  size_t rec, bkgd_partial, dw_partial, lr_partial, lr_stage1, pe_partial, total;
  int splits;
  int64_t per_split;
};

constexpr int64_t DW_BLOCK_MAX = 9LL * 11 * 1024;  // floats per split, bound over the shapes (L5: MT 8, NT+1 11; Lb: MT 9, NT+1 9)

// persistent workgroups of the layer-major hidden backward: one per CU, at most one per wave block
constexpr int LR_G1 = 1024;  // stage-1 rows of the fused Lr weight-gradient reduction (at most)
inline int64_t hidden_grid(int64_t n_samples) { return std::min<int64_t>(HB_GRID_MAX, std::max<int64_t>(1, n_samples / 32)); }
// the grid of a persistent launch of this render call: at most desc.max_workgroups when it is set
inline int64_t cap_grid(const den_render_desc* d, int64_t g) {
  return d->max_workgroups > 0 ? std::max<int64_t>(1, std::min<int64_t>(g, d->max_workgroups)) : g;
}
inline int64_t hidden_grid(const den_render_desc* d) { return cap_grid(d, hidden_grid((int64_t)d->n_rays * d->n_samples)); }

// BF16 backward: layer-major hidden layers (den_hidden.hip) unless the descriptor selects the
// sample-major chain + split-K GEMMs of the F32 mode (bwd_path = 1, A/B comparisons).
inline bool use_hidden_path(const den_render_desc* d) { return d->mode == DEN_MODE_BF16 && d->bwd_path == 0; }
// ... with the pe weight gradients folded into the L1 / L5 launches (den_hidden.hip PEM) unless
// den_render_ray_grad will read dz_0, which the folded L1 launch keeps on chip
inline bool use_pe_fold(const den_render_desc* d) {
#ifdef DEN_NO_PE_FOLD
  return false;
#else
  return use_hidden_path(d) && d->train && !d->ray_grad;
#endif
}

WsLayout ws_layout(const den_render_desc* d) {
  WsLayout L{};
  const int64_t n = (int64_t)d->n_rays * d->n_samples;
  size_t off = 0;
  const int tm = tm_of(d->mode), es = es_of(d->mode);
  const int64_t n_blocks = n / tm;
  for (int a = 0; a <= NACT; ++a)
    L.bstride[a] = (int64_t)((a == D_ZB8 ? WIDTH : act_width(d->mode, a)) / tm) * tm * tm * es;
  // layer-major BF16 training: the activations the hidden launches stream as block-major rows
  // (den_geom.h SROW_BYTES): S_0..S_7, dz_l over S_{l+1} (l = 0..6) -- read for the last time by the
  // launch before the one writing it, never by that one -- dz_7 and dz_b's 8 tiles, one row per wave
  // block: 6.4 KB of workspace per sample for S / dz instead of 10 KB.  r06
  // (profiles/stream_probe, profiles/r06u_ab.jsonl): a hidden launch's pattern (two 16 KiB reads +
  // one 16 KiB write per block) streams at 5.5 TB/s when the write lands on the block just read (the
  // earlier dz_l-over-S_l aliasing), at 5.1-5.8 TB/s for three tensors 8 GiB apart -- varying with
  // how each process's pages map to channels -- and at 6.2 TB/s within one row; the hidden launches
  // ran 4.88 / 4.73-4.98 / 4.64-4.73 ms for the three layouts.
  const bool rows = use_hidden_path(d) && d->train;
  if (rows) {
    for (int a = 0; a <= NACT; ++a) {
      const int64_t o = srow_offset(a);
      if (o < 0) continue;
      L.act[a == D_ZB8 ? D_ZB : a] = off + (size_t)o;  // D_ZB's base is the dz_b slot (the 288-wide D_ZB unused)
      L.bstride[a] = SROW_BYTES;
    }
    off += align256((size_t)n_blocks * (size_t)SROW_BYTES);
    L.sigma_dz = off;
    off += align256((size_t)n * 2);
  }
  for (int a = 0; a < NACT; ++a) {
    if (rows && (srow_offset(a) >= 0 || a == D_ZB)) continue;
    L.act[a] = off;
    // pe: kept by the forward (read once by the streamed L0 / L5-pe weight gradient); ve: kept by the
    // F32 forward only (the BF16 head backward recomputes its tile in LDS; the sample-major BF16 path
    // writes it itself, enc_store_kernel)
    // dz_g: kept on chip by the BF16 head backward (render_head_bwd_kernel, the fused Lg weight
    // gradient) unless den_render_ray_grad will read it
    const bool enc = a == A_VE || (a == D_ZG && !d->ray_grad);
    if (d->train && !(enc && use_hidden_path(d))) off += align256((size_t)n * act_width(d->mode, a) * es);
  }
  L.rec = off;
  if (d->train) off += align256((size_t)n * 16);
  L.bkgd_partial = off;
  off += align256((size_t)4 * d->n_rays * 4);
  // weight-gradient split-K: >= 2048 samples per split, <= 256 splits
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(256, n / 2048));
  int64_t per = (n + splits - 1) / splits;
  per = (per + DW_BK_MAX - 1) / DW_BK_MAX * DW_BK_MAX;
  splits = (n + per - 1) / per;
  L.splits = (int)splits;
  L.per_split = per;
  L.dw_partial = off;
  // shared by the split-K GEMMs, the layer-major hidden backward (den_hidden.hip) and the streamed
  // weight gradients (den_dwstream.hip, at most 9 x 9 tiles per workgroup)
  const size_t hidden = (size_t)hidden_grid(n) * 9 * 9 * 1024;
  if (d->train) off += align256(std::max((size_t)splits * DW_BLOCK_MAX, hidden) * 4);
  // fused Lr weight gradient (render_bwd_kernel<1, 1>): one LR_PART-float partial per render
  // workgroup + the stage-1 rows of its reduction
  L.lr_partial = off;
  L.lr_stage1 = off;
  if (d->train && use_hidden_path(d)) {
    off += align256((size_t)(n / wg_samples(d->mode)) * LR_PART * 4);
    L.lr_stage1 = off;
    off += align256((size_t)LR_G1 * LR_PART * 4);
  }
  // the folded pe weight gradients' split-K partials (den_dwstream.hip's [wg][16][3] layout), written
  // by the L5 and L1 launches, reduced after both
  L.pe_partial = off;
  if (use_pe_fold(d)) off += align256((size_t)hidden_grid(n) * 16 * 3 * 1024 * 4);
  L.total = off;
  return L;
}

// bytes from one wave block of activation `a` to the next
inline int64_t block_bytes(const WsLayout& L, int mode, int a) { return L.bstride[a]; }

int check_desc(const den_render_desc* d) {
  if (!d) return fail(DEN_EINVAL, "null desc");
  if (d->mode != DEN_MODE_F32 && d->mode != DEN_MODE_BF16) return fail(DEN_EINVAL, "mode must be 0 (F32) or 1 (BF16)");
  if (d->radiance_dim != 1 && d->radiance_dim != 3) return fail(DEN_EUNSUPPORTED, "radiance_dim must be 1 or 3");
  if (d->n_rays <= 0) return fail(DEN_EINVAL, "n_rays must be > 0");
  const int wgs = wg_samples(d->mode);
  if (d->n_samples < 64 || d->n_samples > wgs || wgs % d->n_samples != 0)
    return fail(DEN_EUNSUPPORTED, "n_samples must be 64..128 (F32) / 64..256 (BF16) and divide it");
  if (((int64_t)d->n_rays * d->n_samples) % std::max(wgs, fwd_wg_samples(d->mode)) != 0)
    return fail(DEN_EUNSUPPORTED, "n_rays * n_samples must be a multiple of the workgroup tile "
                                  "(den_render_tile_samples)");
  if (d->points < 0 || d->points > 2) return fail(DEN_EINVAL, "points must be 0, 1 or 2");
  if (d->points == 0 && fwd_wg_samples(d->mode) % d->n_samples != 0)
    return fail(DEN_EUNSUPPORTED, "the fused compositing needs whole rays per forward workgroup");
  if (d->contraction < 0 || d->contraction > 2) return fail(DEN_EINVAL, "contraction must be 0 (AABB), 1 (tanh) or 2 (sphere)");
  if (d->points == 0 && d->contraction != 0)
    return fail(DEN_EUNSUPPORTED, "the fixed-count sampler (points = 0) marches the AABB: contraction must be 0");
  if (d->density_activation < 0 || d->density_activation > 2)
    return fail(DEN_EINVAL, "density_activation must be 0 (shifted_trunc_exp), 1 (softplus) or 2 (shifted_softplus)");
  if (d->max_workgroups < 0) return fail(DEN_EINVAL, "max_workgroups must be >= 0 (0: one workgroup per CU)");
  return DEN_OK;
}

template <int MODE>
RenderArgs<MODE> make_args(const den_render_desc* d, const den_render_io* io, const WsLayout& L) {
  RenderArgs<MODE> A{};
  A.n_samples = d->n_samples;
  A.n_rays = d->n_rays;
  A.rd = d->radiance_dim;
  A.train = d->train;
  A.has_bkgd = d->has_bkgd;
  A.points = d->points;
  A.contraction = d->contraction;
  for (int i = 0; i < 6; ++i) A.aabb[i] = d->aabb[i];
  A.near_p = d->near_plane;
  A.far_p = d->far_plane;
  A.rays_o = io->rays_o;
  A.rays_d = io->rays_d;
  A.jitter = io->jitter;
  A.ray_idx = io->ray_indices;
  A.t_start = io->t_starts;
  A.t_end = io->t_ends;
  A.bias = io->bias_pk;
  A.bkgd = io->bkgd;
  char* ws = (char*)io->workspace;
  for (int a = 0; a < NACT; ++a) A.act[a] = ws ? ws + L.act[a] : nullptr;
  A.rec = ws ? (float*)(ws + L.rec) : nullptr;
  A.bkgd_partial = ws ? (float*)(ws + L.bkgd_partial) : nullptr;
  A.lr_partial = ws ? (float*)(ws + L.lr_partial) : nullptr;
  A.out_rgb = io->out_rgb;
  A.out_opacity = io->out_opacity;
  A.out_depth = io->out_depth;
  A.density_act = d->density_activation;
  A.keep_dzg = d->ray_grad;
  for (int a = 0; a <= NACT; ++a) A.bstride[a] = L.bstride[a];
  A.sigma_dz = ws ? ws + L.sigma_dz : nullptr;
  return A;
}

// Split-K weight-gradient GEMM of one layer + its reduction into the flat gradient.
// red_n1 < 0: columns [0, N1) are the first input segment; red_n1 = 0 maps every column to the
// second segment at chain feature n1_feat (the pe columns of L5).  bias = 0 skips the bias.
template <int MODE, int MT, int N1, int N2, int WN = 1>
int launch_dw(const den_render_desc* d, const WsLayout& L, char* ws, int layer, int a_dz, int a_x1, int a_x2,
              int n1_feat, float* grad, hipStream_t s, int m_off = 0, int red_n1 = -1, int bias = 1) {
  DwArgs P{};
  P.A = ws + L.act[a_dz];
  P.a_tiles = act_width(MODE, a_dz) / tm_of(MODE);
  P.a_t0 = m_off / tm_of(MODE);
  P.B1 = ws + L.act[a_x1];
  P.B2 = a_x2 >= 0 ? ws + L.act[a_x2] : nullptr;
  P.n = (int64_t)d->n_rays * d->n_samples;
  P.per_split = L.per_split;
  P.partial = (float*)(ws + L.dw_partial);
  {
    DEN_TIMED(T_DW_GEMM, s);
    hipLaunchKernelGGL((dw_gemm_kernel<MODE, MT, N1, N2, WN>), dim3(L.splits), dim3(64 * MT * WN), 0, s, P);
  }
  DEN_LAUNCHED();
  DwReduceArgs R{};
  R.partial = P.partial;
  R.splits = L.splits;
  R.MT = MT;
  R.NT = (N1 + N2) / 32;
  R.m_off = m_off;
  R.layer = layer;
  R.mode = MODE;
  R.rd = d->radiance_dim;
  R.n1 = red_n1 < 0 ? N1 : red_n1;
  R.n1_feat = n1_feat;
  R.bias = bias;
  R.grad = grad;
  const int64_t per = (int64_t)MT * (R.NT + 1) * 1024;
  {
    DEN_TIMED(T_DW_REDUCE, s);
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((per + DWR_EL - 1) / DWR_EL)), dim3(DWR_THREADS), 0, s, R);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

// One streamed weight-gradient launch (den_dwstream.hip) over the whole sample range.
template <int MA, int MT, int NB, int NT, int NW, int DEPTH, int U = 1>
int launch_dwstream(const den_render_desc* d, const WsLayout& L, char* ws, int a0, int a1, int b0, int b1,
                    hipStream_t s) {
  const int64_t n = (int64_t)d->n_rays * d->n_samples;
  DwStreamArgs P{};
  P.a[0] = ws + L.act[a0];
  P.a_bs[0] = block_bytes(L, DEN_MODE_BF16, a0);
  P.a[1] = a1 >= 0 ? ws + L.act[a1] : nullptr;
  P.a_bs[1] = a1 >= 0 ? block_bytes(L, DEN_MODE_BF16, a1) : 0;
  P.b[0] = b0 >= 0 ? ws + L.act[b0] : nullptr;
  P.b_bs[0] = b0 >= 0 ? block_bytes(L, DEN_MODE_BF16, b0) : 0;
  P.b[1] = b1 >= 0 ? ws + L.act[b1] : nullptr;
  P.b_bs[1] = b1 >= 0 ? block_bytes(L, DEN_MODE_BF16, b1) : 0;
  P.partial = (float*)(ws + L.dw_partial);
  static_assert(U == 1 || U == 2 || U == 4 || U == 8, "U divides the wave blocks (n is a multiple of 256)");
  P.n_blocks = n / 32 / U;
  const int64_t grid = hidden_grid(d);
  P.per_wg = (P.n_blocks + grid - 1) / grid;
  {
    DEN_TIMED(T_DW_GEMM, s);
    hipLaunchKernelGGL((dwstream_kernel<MA, MT, NB, NT, NW, DEPTH, U>), dim3((unsigned)grid), dim3(64 * NW), 0, s, P);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

// Reduction of row tiles [mt0, mt0 + MT) of a streamed partial with NT_ALL column tiles into layer
// `layer`'s gradient (red_n1 / n1_feat / bias as in launch_dw).
int launch_dwstream_reduce(const den_render_desc* d, const WsLayout& L, char* ws, int MT_ALL, int NT_ALL, int mt0,
                           int MT, int layer, int red_n1, int n1_feat, int bias, float* grad, hipStream_t s,
                           int splits = -1, size_t region = (size_t)-1) {
  DwReduceArgs R{};
  R.partial = (float*)(ws + (region == (size_t)-1 ? L.dw_partial : region));
  R.splits = splits > 0 ? splits : (int)hidden_grid(d);
  R.MT = MT;
  R.NT = NT_ALL;
  R.m_off = 0;
  R.layer = layer;
  R.mode = DEN_MODE_BF16;
  R.rd = d->radiance_dim;
  R.n1 = red_n1;
  R.n1_feat = n1_feat;
  R.bias = bias;
  R.grad = grad;
  R.split_stride = (int64_t)MT_ALL * (NT_ALL + 1) * 1024;
  R.first = (int64_t)mt0 * (NT_ALL + 1) * 1024;
  const int64_t per = (int64_t)MT * (NT_ALL + 1) * 1024;
  {
    DEN_TIMED(T_DW_REDUCE, s);
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((per + DWR_EL - 1) / DWR_EL)), dim3(DWR_THREADS), 0, s, R);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

// Reduction of the fused Lr weight-gradient partials (render_bwd_kernel<1, 1>) into the gradient.
int launch_lr_reduce(const den_render_desc* d, const WsLayout& L, char* ws, float* grad, hipStream_t s, int64_t n_wg) {
  const int G1 = (int)std::min<int64_t>(LR_G1, n_wg);
  DwReduceArgs R{};
  R.MT = 1;
  R.NT = 4;
  R.m_off = 0;
  R.layer = L_R;
  R.mode = DEN_MODE_BF16;
  R.rd = d->radiance_dim;
  R.n1 = 128;
  R.n1_feat = 0;
  R.bias = 1;
  R.grad = grad;
  float* st1 = (float*)(ws + L.lr_stage1);
  {
    DEN_TIMED(T_DW_REDUCE, s);
    hipLaunchKernelGGL(lr_reduce1_kernel, dim3((unsigned)G1), dim3(448), 0, s, (const float*)(ws + L.lr_partial), n_wg,
                       G1, st1);
  }
  DEN_LAUNCHED();
  {
    DEN_TIMED(T_DW_REDUCE, s);
    hipLaunchKernelGGL(lr_reduce2_kernel, dim3(LR_PART - 1), dim3(256), 0, s, (const float*)st1, G1, R);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

// Layer-major backward of hidden layer l (den_hidden.hip) + reduction of its weight/bias gradient;
// l = 8 is the [bottleneck | sigma] layer Lb (input S7, dz_b with the sigma tile, 9 row tiles).
int launch_hidden(const den_render_desc* d, const den_render_io* io, const WsLayout& L, char* ws, int l, float* grad,
                  hipStream_t s) {
  const int64_t n = (int64_t)d->n_rays * d->n_samples;
  const bool lb = l == 8;
  HiddenArgs H{};
  H.w = (const char*)io->w_bwd + bwd_layer_offset(DEN_MODE_BF16, 10 - l);
  H.dz_in = ws + L.act[lb ? D_ZB : D_Z0 + l];
  H.s_in = ws + L.act[A_S0 + l - 1];
  H.dz_out = ws + L.act[D_Z0 + l - 1];
  H.partial = (float*)(ws + L.dw_partial);
  H.n_blocks = n / 32;
  H.bs_dz_in = L.bstride[lb ? D_ZB8 : D_Z0 + l];
  H.bs_s = L.bstride[A_S0 + l - 1];
  H.bs_dz_out = L.bstride[D_Z0 + l - 1];
  H.sigma_dz = ws + L.sigma_dz;
  // the pe fold: L5 adds dW_5's pe columns, L1 dW_0 (dz_0 then stays on chip)
  const int pem = use_pe_fold(d) ? (l == 5 ? 1 : l == 1 ? 2 : 0) : 0;
  H.pe = ws + L.act[A_PE];
  H.bs_pe = L.bstride[A_PE];
  H.pe_partial = (float*)(ws + L.pe_partial);
  H.pe_mt0 = l == 5 ? 8 : 0;
  const int64_t grid = hidden_grid(d);
  H.per_wg = (H.n_blocks + grid - 1) / grid;
  {
    TimedLaunch timed_(lb ? T_HIDDEN_LB : T_HIDDEN_BWD, s);
    const dim3 g((unsigned)grid), t(HbCfg<false>::THREADS);
    if (lb)
      hipLaunchKernelGGL((hidden_bwd_kernel<true, 0>), g, dim3(HbCfg<true>::THREADS), 0, s, H);
    else if (pem == 1)
      hipLaunchKernelGGL((hidden_bwd_kernel<false, 1>), g, t, 0, s, H);
    else if (pem == 2)
      hipLaunchKernelGGL((hidden_bwd_kernel<false, 2>), g, t, 0, s, H);
    else
      hipLaunchKernelGGL((hidden_bwd_kernel<false, 0>), g, t, 0, s, H);
  }
  DEN_LAUNCHED();
  if (lb) return launch_dwstream_reduce(d, L, ws, 9, 8, 0, 9, L_B, WIDTH, 0, 1, grad, s);
  DwReduceArgs R{};
  R.partial = H.partial;
  R.splits = (int)grid;
  R.MT = 8;
  R.NT = 8;
  R.m_off = 0;
  R.layer = l;
  R.mode = DEN_MODE_BF16;
  R.rd = d->radiance_dim;
  R.n1 = WIDTH;
  R.n1_feat = 0;
  R.bias = 1;
  R.grad = grad;
  const int64_t per = 8LL * 9 * 1024;
  {
    DEN_TIMED(T_DW_REDUCE, s);
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((per + DWR_EL - 1) / DWR_EL)), dim3(DWR_THREADS), 0, s, R);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

// compute units of the device that owns stream `s` (the persistent kernels run one workgroup per
// CU); cached per device, thread-safe (several host threads may drive several devices)
int device_cu_count(hipStream_t s) {
  static std::atomic<int> cached[64];
  int dev = -1;
  if (hipStreamGetDevice(s, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev < 0 || dev >= 64) return 256;
  int n = cached[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

template <int MODE>
int render_fwd_impl(const den_render_desc* d, const den_render_io* io, hipStream_t s) {
  WsLayout L = ws_layout(d);
  RenderArgs<MODE> A = make_args<MODE>(d, io, L);
  A.w = (const char*)io->w_fwd;
  const int64_t n = (int64_t)d->n_rays * d->n_samples;
  A.n_items = n / fwd_wg_samples(MODE);
  // persistent: one workgroup per CU (the 143 KB weight ring + records admit one), each walking
  // items blockIdx.x, blockIdx.x + grid, ...
  const unsigned grid = (unsigned)cap_grid(d, std::min<int64_t>(A.n_items, device_cu_count(s)));
  {
    DEN_TIMED(T_RENDER_FWD, s);
    if (d->train)
      hipLaunchKernelGGL((render_fwd_kernel<MODE, true>), dim3(grid), dim3(fwd_threads(MODE)), 0, s, A);
    else
      hipLaunchKernelGGL((render_fwd_kernel<MODE, false>), dim3(grid), dim3(fwd_threads(MODE)), 0, s, A);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

template <int MODE>
int render_bwd_impl(const den_render_desc* d, const den_render_io* io, const den_render_grad* g, hipStream_t s,
                    int parts) {
  WsLayout L = ws_layout(d);
  RenderArgs<MODE> A = make_args<MODE>(d, io, L);
  A.w = (const char*)io->w_bwd;
  A.d_rgb = g->d_rgb;
  A.d_opacity = g->d_opacity;
  A.d_depth = g->d_depth;
  const int64_t n = (int64_t)d->n_rays * d->n_samples;
  char* ws = (char*)io->workspace;
  float* G = g->grad_params;
  const bool hidden = use_hidden_path(d);
  int rc;
  if (parts & 1) {
    if constexpr (MODE == DEN_MODE_BF16) {
      if (hidden) {
        // head (compositing adjoint, Lr^T + dW_r, Lg^T + dW_g) sample-major and persistent, then Lb,
        // L7..L1 layer-major.  The Lg partial shares dw_partial with the hidden launches: reduced first.
        const int64_t items = n / wg_samples(MODE);
        // one persistent workgroup per CU, as the forward; at most what the split-K partial region
        // holds (4 x 10 tiles per workgroup; ws_layout sizes it for the hidden launches' 256 x 9 x 9,
        // i.e. >= 518 head workgroups) and the Lr partials (one per item)
        const int64_t dw_cap = (int64_t)(L.lr_partial - L.dw_partial) / (4 * 10 * 1024 * 4);
        const int head_grid = (int)cap_grid(d, std::max<int64_t>(
            1, std::min<int64_t>({items, (int64_t)device_cu_count(s), dw_cap})));
        {
          DEN_TIMED(T_RENDER_BWD, s);
          hipLaunchKernelGGL(render_head_bwd_kernel, dim3((unsigned)head_grid), dim3(512), 0, s, A,
                             (float*)(ws + L.dw_partial));
        }
        DEN_LAUNCHED();
        if ((rc = launch_lr_reduce(d, L, ws, G, s, head_grid)) != DEN_OK) return rc;
        if ((rc = launch_dwstream_reduce(d, L, ws, 4, 9, 0, 4, L_G, 256, WIDTH, 1, G, s, head_grid)) != DEN_OK)
          return rc;
        for (int l = 8; l >= 1; --l)
          if ((rc = launch_hidden(d, io, L, ws, l, G, s)) != DEN_OK) return rc;
      }
    }
    if (!hidden) {
      DEN_TIMED(T_RENDER_BWD, s);
      hipLaunchKernelGGL((render_bwd_kernel<MODE, NBL - 1>), dim3((unsigned)(n / wg_samples(MODE))), dim3(512), 0, s,
                         A);
      DEN_LAUNCHED();
    }
  }
  if (!(parts & 2)) return DEN_OK;
  if (hidden) {
    // L0's and L5's pe-column weight gradients: folded into the L1 / L5 launches (part 1 wrote their
    // partials), else streamed by one operand-sharing launch (den_dwstream.hip) over dz_0, dz_5 and pe
    const bool fold = use_pe_fold(d);
    const size_t region = fold ? L.pe_partial : L.dw_partial;
    if (!fold && (rc = launch_dwstream<8, 16, 2, 2, DWS_NW1, 3, 1>(d, L, ws, D_Z0 + 0, D_Z0 + 5, A_PE, -1, s)) != DEN_OK)
      return rc;
    if ((rc = launch_dwstream_reduce(d, L, ws, 16, 2, 0, 8, 0, 64, 0, 1, G, s, -1, region)) != DEN_OK) return rc;
    if ((rc = launch_dwstream_reduce(d, L, ws, 16, 2, 8, 8, 5, 0, WIDTH, 0, G, s, -1, region)) != DEN_OK) return rc;
    // (Lb's weight gradient comes from its hidden launch, Lr's and Lg's from render_head_bwd_kernel)
    if (g->grad_bkgd) {
      hipLaunchKernelGGL(sum_partials_kernel, dim3(d->radiance_dim), dim3(1024), 0, s, d->radiance_dim, d->n_rays,
                         (const float*)(ws + L.bkgd_partial), g->grad_bkgd);
      DEN_LAUNCHED();
    }
    return DEN_OK;
  }
  if constexpr (MODE == DEN_MODE_BF16) {
    const int64_t nb = n / 32;
    hipLaunchKernelGGL(enc_store_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, make_args<MODE>(d, io, L), nb);
    DEN_LAUNCHED();
  }
  if ((rc = launch_dw<MODE, 8, 64, 0>(d, L, ws, 0, D_Z0 + 0, A_PE, -1, 0, G, s)) != DEN_OK) return rc;
  if (hidden) {
    // pe columns of L5 (the S4 columns and the bias come from the hidden launch of layer 5)
    if ((rc = launch_dw<MODE, 8, 64, 0>(d, L, ws, 5, D_Z0 + 5, A_PE, -1, WIDTH, G, s, 0, 0, 0)) != DEN_OK) return rc;
  } else {
    if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, 1, D_Z0 + 1, A_S0 + 0, -1, 0, G, s)) != DEN_OK) return rc;
    if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, 2, D_Z0 + 2, A_S0 + 1, -1, 0, G, s)) != DEN_OK) return rc;
    if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, 3, D_Z0 + 3, A_S0 + 2, -1, 0, G, s)) != DEN_OK) return rc;
    if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, 4, D_Z0 + 4, A_S0 + 3, -1, 0, G, s)) != DEN_OK) return rc;
    if ((rc = launch_dw<MODE, 8, 256, 64>(d, L, ws, 5, D_Z0 + 5, A_S0 + 4, A_PE, WIDTH, G, s)) != DEN_OK) return rc;
    if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, 6, D_Z0 + 6, A_S0 + 5, -1, 0, G, s)) != DEN_OK) return rc;
    if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, 7, D_Z0 + 7, A_S0 + 6, -1, 0, G, s)) != DEN_OK) return rc;
  }
  // [bottleneck | sigma]: the 256 bottleneck rows, then the sigma tile (row 256) with 4 waves splitting
  // its 8 column tiles (one 9-wave launch would spill: 9 accumulator tiles at 3 waves per SIMD)
  if ((rc = launch_dw<MODE, 8, 256, 0>(d, L, ws, L_B, D_ZB, A_S0 + 7, -1, 0, G, s)) != DEN_OK) return rc;
  if ((rc = launch_dw<MODE, 1, 256, 0, 4>(d, L, ws, L_B, D_ZB, A_S0 + 7, -1, 0, G, s, WIDTH)) != DEN_OK) return rc;
  if ((rc = launch_dw<MODE, 4, 256, 32>(d, L, ws, L_G, D_ZG, A_BT, A_VE, WIDTH, G, s)) != DEN_OK) return rc;
  // rgb output (M = 32): 4 waves split the 4 column tiles
  if ((rc = launch_dw<MODE, 1, 128, 0, 4>(d, L, ws, L_R, D_ZR, A_G, -1, 0, G, s)) != DEN_OK) return rc;
  if (g->grad_bkgd) {
    hipLaunchKernelGGL(sum_partials_kernel, dim3(d->radiance_dim), dim3(1024), 0, s, d->radiance_dim, d->n_rays,
                       (const float*)(ws + L.bkgd_partial), g->grad_bkgd);
    DEN_LAUNCHED();
  }
  return DEN_OK;
}

}  // namespace

extern "C" {

int den_version(void) { return DEN_VERSION; }

#ifdef DEN_FWD_PROF
// experiment builds only: per-wave cycle split of the last render_fwd launch (512 WGs x 8 waves x 4)
int den_debug_fwd_prof(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(den_fwd_prof), sizeof(uint64_t) * 512 * 8 * 8) == hipSuccess ? DEN_OK
                                                                                                        : DEN_EHIP;
}
#endif

#ifdef DEN_CLOCK
// diagnostic builds only: the start / end stamps of every hot kernel's last launch (den_device.h)
int den_debug_clock(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(den_clock), sizeof(uint64_t) * DEN_CLOCK_KERNELS * DEN_CLOCK_WGS * 4) ==
                 hipSuccess
             ? DEN_OK
             : DEN_EHIP;
}
#endif

#ifdef DEN_HIDDEN_PROF
// experiment builds only: per-wave phase cycles of the last L7..L1 and Lb launches (2 x 256 WGs x 8 waves x 8)
int den_debug_hidden_prof(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(den_hidden_prof), sizeof(uint64_t) * 2 * 256 * 8 * 8) == hipSuccess
             ? DEN_OK
             : DEN_EHIP;
}
#endif

#ifdef DEN_HEAD_PROF
// experiment builds only: per-wave phase cycles of the last render_head_bwd launch (256 WGs x 8 waves x 8)
int den_debug_head_prof(uint64_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(den_head_prof), sizeof(uint64_t) * 256 * 8 * 8) == hipSuccess ? DEN_OK
                                                                                                          : DEN_EHIP;
}
#endif

int32_t den_render_tile_samples(int32_t mode) {
  return (mode == 0 || mode == 1) ? std::max(wg_samples(mode), fwd_wg_samples(mode)) : -1;
}

int den_timing_enable(int32_t on) {
  std::lock_guard<std::mutex> g(g_timing_mu);
  g_timing = on != 0;
  return DEN_OK;
}

int den_timing_collect(int32_t n_classes, double* total_ms, int64_t* launches) {
  if (n_classes < 0 || (n_classes > 0 && (!total_ms || !launches))) return fail(DEN_EINVAL, "bad timing buffers");
  std::vector<TimingRec> recs;
  {
    std::lock_guard<std::mutex> g(g_timing_mu);
    recs.swap(g_timing_recs);
  }
  for (int c = 0; c < n_classes; ++c) total_ms[c] = 0.0, launches[c] = 0;
  int rc = DEN_OK;
  for (auto& r : recs) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess)
      rc = fail(DEN_EHIP, "timing event failed");
    else if (r.cls < n_classes)
      total_ms[r.cls] += ms, launches[r.cls] += 1;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  return rc;
}
const char* den_last_error(void) { return g_err.c_str(); }

int64_t den_param_count(int32_t rd) { return (rd == 1 || rd == 3) ? param_count(rd) : -1; }
int64_t den_param_offset(int32_t rd, int32_t idx) {
  if ((rd != 1 && rd != 3) || idx < 0 || idx > 24) return -1;
  return param_offset(rd, idx);
}

size_t den_packed_fwd_bytes(int32_t mode) { return (mode == 0 || mode == 1) ? (size_t)fwd_bytes(mode) : 0; }
size_t den_packed_bwd_bytes(int32_t mode) { return (mode == 0 || mode == 1) ? (size_t)bwd_bytes(mode) : 0; }
size_t den_packed_bias_bytes(int32_t mode) { return (mode == 0 || mode == 1) ? (size_t)bias_floats(mode) * 4 : 0; }

int den_pack_weights(int32_t mode, int32_t rd, const float* params, void* w_fwd, void* w_bwd, float* bias_pk,
                     void* stream) {
  if (mode != 0 && mode != 1) return fail(DEN_EINVAL, "bad mode");
  if (rd != 1 && rd != 3) return fail(DEN_EUNSUPPORTED, "radiance_dim must be 1 or 3");
  if (!params || !w_fwd || !w_bwd || !bias_pk) return fail(DEN_EINVAL, "null pointer");
  PackArgs P{mode, rd, params, w_fwd, w_bwd, bias_pk};
  const int es = es_of(mode);
  const int64_t total = fwd_bytes(mode) / es + bwd_bytes(mode) / es + bias_floats(mode);
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, P);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_render_workspace_bytes(const den_render_desc* d) {
  if (check_desc(d) != DEN_OK) return 0;
  return ws_layout(d).total;
}

int den_render_fwd(const den_render_desc* d, const den_render_io* io, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!io || !io->rays_o || !io->rays_d || !io->w_fwd || !io->bias_pk || !io->out_rgb || !io->out_opacity ||
      !io->out_depth || (d->points == 0 && !io->jitter))
    return fail(DEN_EINVAL, "null pointer in den_render_io");
  if (d->points == 2 && (!io->ray_indices || !io->t_starts || !io->t_ends))
    return fail(DEN_EINVAL, "points = 2 needs ray_indices, t_starts and t_ends");
  if (d->has_bkgd && !io->bkgd) return fail(DEN_EINVAL, "has_bkgd but bkgd == NULL");
  if (d->points && d->has_bkgd) return fail(DEN_EINVAL, "points mode has no background");
  if (!io->workspace) return fail(DEN_EINVAL, "workspace is required (den_render_workspace_bytes)");
  return d->mode == 0 ? render_fwd_impl<0>(d, io, (hipStream_t)stream) : render_fwd_impl<1>(d, io, (hipStream_t)stream);
}

int den_render_bwd(const den_render_desc* d, const den_render_io* io, const den_render_grad* g, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!d->train) return fail(DEN_EINVAL, "den_render_bwd needs a train=1 forward");
  if (!io || !io->workspace || !io->w_bwd || !io->rays_o || !io->rays_d || (d->points == 0 && !io->jitter))
    return fail(DEN_EINVAL, "null pointer in den_render_io");
  if (!g || !g->d_rgb || !g->grad_params) return fail(DEN_EINVAL, "null pointer in den_render_grad");
  if (d->has_bkgd && !io->bkgd) return fail(DEN_EINVAL, "has_bkgd but bkgd == NULL");
  return d->mode == 0 ? render_bwd_impl<0>(d, io, g, (hipStream_t)stream, 3)
                      : render_bwd_impl<1>(d, io, g, (hipStream_t)stream, 3);
}

int den_render_bwd_part(const den_render_desc* d, const den_render_io* io, const den_render_grad* g, int32_t part,
                        void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (part != 1 && part != 2) return fail(DEN_EINVAL, "part must be 1 (dz chain) or 2 (weight gradients)");
  if (!d->train || !io || !io->workspace || !io->w_bwd || !g || !g->d_rgb || !g->grad_params)
    return fail(DEN_EINVAL, "null pointer / train=0");
  return d->mode == 0 ? render_bwd_impl<0>(d, io, g, (hipStream_t)stream, part)
                      : render_bwd_impl<1>(d, io, g, (hipStream_t)stream, part);
}

size_t den_render_ray_grad_workspace_bytes(const den_render_desc* d) {
  if (check_desc(d) != DEN_OK) return 0;
  return (size_t)d->n_rays * d->n_samples * 6 * sizeof(float);
}

int den_render_ray_grad(const den_render_desc* d, const den_render_io* io, const float* params, int32_t n_rays_out,
                        int64_t n_valid, void* rg_workspace, float* d_rays_o, float* d_rays_d, void* stream) {
  int rc = check_desc(d);
  if (rc) return rc;
  if (!d->train) return fail(DEN_EINVAL, "den_render_ray_grad needs a train=1 forward and its den_render_bwd");
  if (use_hidden_path(d) && !d->ray_grad)
    return fail(DEN_EINVAL, "den_render_ray_grad needs desc.ray_grad = 1 on the forward and backward (BF16 keeps "
                            "dz_g only then)");
  if (!io || !io->workspace || !io->rays_o || !io->rays_d || !params || !rg_workspace || !d_rays_o || !d_rays_d ||
      (d->points == 0 && !io->jitter) || (d->points == 2 && (!io->ray_indices || !io->t_starts || !io->t_ends)))
    return fail(DEN_EINVAL, "null pointer");
  const int64_t n = (int64_t)d->n_rays * d->n_samples;
  if (d->points == 2 && (n_rays_out <= 0 || n_valid < 0 || n_valid > n))
    return fail(DEN_EINVAL, "points = 2 needs n_rays_out > 0 and 0 <= n_valid <= samples");
  const WsLayout L = ws_layout(d);
  const char* ws = (const char*)io->workspace;
  RayGradArgs G{};
  G.points = d->points;
  G.contraction = d->contraction;
  G.rd = d->radiance_dim;
  G.n_samples = d->n_samples;
  G.n = n;
  for (int i = 0; i < 6; ++i) G.aabb[i] = d->aabb[i];
  G.near_p = d->near_plane;
  G.far_p = d->far_plane;
  G.rays_o = io->rays_o;
  G.rays_d = io->rays_d;
  G.jitter = io->jitter;
  G.ray_idx = io->ray_indices;
  G.t0 = io->t_starts;
  G.t1 = io->t_ends;
  G.per_sample = (float*)rg_workspace;
  RayGradMlp M{params, ws + L.act[D_Z0 + 0], ws + L.act[D_Z0 + 5], ws + L.act[D_ZG],
               block_bytes(L, d->mode, D_Z0 + 0), block_bytes(L, d->mode, D_Z0 + 5), block_bytes(L, d->mode, D_ZG),
               d->mode == DEN_MODE_F32 ? 1.0f : (float)KAPPA};
  hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)((n + RG_THREADS - 1) / RG_THREADS);
  if (d->mode == DEN_MODE_F32) hipLaunchKernelGGL(raygrad_mlp_kernel<0>, dim3(grid), dim3(RG_THREADS), 0, st, G, M);
  else hipLaunchKernelGGL(raygrad_mlp_kernel<1>, dim3(grid), dim3(RG_THREADS), 0, st, G, M);
  DEN_LAUNCHED();
  if (d->points == 1) {
    hipLaunchKernelGGL(raygrad_split_kernel, dim3(grid), dim3(RG_THREADS), 0, st, n, G.per_sample, d_rays_o,
                       d_rays_d);
  } else {
    const int R = d->points == 0 ? d->n_rays : n_rays_out;
    hipLaunchKernelGGL(raygrad_reduce_kernel, dim3((R + 3) / 4), dim3(256), 0, st, R, d->points, d->n_samples,
                       io->ray_indices, n_valid, G.per_sample, d_rays_o, d_rays_d);
  }
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_sum_partials(int32_t n, int32_t nb, const float* part, float* out, void* stream) {
  if (n <= 0 || nb <= 0 || !part || !out) return fail(DEN_EINVAL, "bad arguments");
  hipLaunchKernelGGL(sum_partials_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, n, nb, part, out);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_adam_step(int64_t n, float* p, const float* g, float* m, float* v, float lr, float beta1, float beta2,
                  float eps, float wd, int64_t step, void* stream) {
  if (n <= 0 || !p || !g || !m || !v || step < 1) return fail(DEN_EINVAL, "bad arguments");
  // torch forms these in Python double and rounds them to f32 when applied
  const double b1 = (double)beta1, b2 = (double)beta2;
  const double bc1 = 1.0 - std::pow(b1, (double)step);
  const double bc2 = 1.0 - std::pow(b2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2s = (float)std::sqrt(bc2);
  hipLaunchKernelGGL(adam_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, p, g,
                     m, v, step_size, (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), eps, wd, bc2s);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_adam_step_f64(int64_t n, double* p, const double* g, double* m, double* v, double lr, double beta1,
                      double beta2, double eps, double wd, int64_t step, void* stream) {
  if (n <= 0 || !p || !g || !m || !v || step < 1) return fail(DEN_EINVAL, "bad arguments");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel<double>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, p,
                     g, m, v, lr / bc1, 1.0 - beta1, beta2, 1.0 - beta2, eps, wd, std::sqrt(bc2));
  DEN_LAUNCHED();
  return DEN_OK;
}

// ------------------------------------------------------------------ pixel bandwidth
int den_pixbw_blocks(int32_t N) { return N > 0 ? (N + PIXBW_BLOCK - 1) / PIXBW_BLOCK : 0; }

size_t den_pixbw_workspace_bytes(int32_t S, int32_t N) {
  if (S < 2 || N <= 0) return 0;
  return ((size_t)(S - 1) * PIXBW_SEG_F + (size_t)S * 8) * (size_t)N * sizeof(double);
}

int den_pixbw_sample_ts(int32_t S, int32_t N, const double* gen, const double* out_ts, double omega_c_min,
                        double max_cumprob, double* ts, void* stream) {
  if (S < 2 || N <= 0 || !out_ts || !ts || (S > 2 && !gen)) return fail(DEN_EINVAL, "bad arguments");
  if (!(omega_c_min > 0.0) || !(max_cumprob > 0.0 && max_cumprob < 1.0))
    return fail(DEN_EINVAL, "omega_c_min must be > 0 and max_cumprob in (0, 1)");
  // torch.distributions.Exponential keeps the Python-float rate as an f32 tensor and the target
  // cumulative probability is an f32 buffer (pixel_bandwidth.py:81-83, 344-350)
  const float rate = (float)(1e-9 * omega_c_min), cum = (float)max_cumprob;
  const int64_t tot = (int64_t)S * N;
  hipLaunchKernelGGL(pixbw_sample_ts_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     S, N, gen, out_ts, rate, cum, ts);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_pixbw_sample_ts_bwd(int32_t S, int32_t N, const double* g_sample_ts, double* d_output_ts, void* stream) {
  if (S < 2 || N <= 0 || !g_sample_ts || !d_output_ts) return fail(DEN_EINVAL, "bad arguments");
  hipLaunchKernelGGL(pixbw_sample_ts_bwd_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     S, N, g_sample_ts, d_output_ts);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_pixbw_decay_ts_bwd(int32_t N, const double* output_ts, const double* reset_ts, const float* params,
                           const float* delta_in, const float* d_out, double* d_output_ts, double* d_reset_ts,
                           void* stream) {
  if (N <= 0 || !output_ts || !reset_ts || !params || !delta_in || !d_out) return fail(DEN_EINVAL, "bad arguments");
  if (!d_output_ts && !d_reset_ts) return DEN_OK;
  hipLaunchKernelGGL(pixbw_decay_ts_bwd_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     N, output_ts, reset_ts, params, delta_in, d_out, d_output_ts, d_reset_ts);
  DEN_LAUNCHED();
  return DEN_OK;
}

static int pixbw_args(int32_t S, int32_t N, int32_t reset, const float* it, const double* ts, const double* out_ts,
                      const float* prm, const float* delta_in, const double* reset_ts, PixArgs* A) {
  if (S < 2 || N <= 0 || !it || !ts || !out_ts || !prm) return fail(DEN_EINVAL, "bad arguments");
  if (!reset && (!delta_in || !reset_ts))
    return fail(DEN_EINVAL, "a non-reset call needs delta_in and reset_ts of a preceding reset call");
  *A = PixArgs{};
  A->S = S;
  A->N = N;
  A->reset = reset ? 1 : 0;
  A->it = it;
  A->ts = ts;
  A->out_ts = out_ts;
  A->prm = prm;
  A->delta_in = delta_in;
  A->reset_ts = reset_ts;
  return DEN_OK;
}

int den_pixbw_fwd(int32_t S, int32_t N, int32_t reset, const float* it, const double* ts, const double* out_ts,
                  const float* prm, const float* delta_in, const double* reset_ts, float* out, float* delta_out,
                  void* stream) {
  PixArgs A;
  int rc = pixbw_args(S, N, reset, it, ts, out_ts, prm, delta_in, reset_ts, &A);
  if (rc) return rc;
  if (!out || (reset && !delta_out)) return fail(DEN_EINVAL, "out (and delta_out for a reset call) are required");
  A.out = out;
  A.delta_out = delta_out;
  if (S - 1 <= PIXBW_WAVE_SEGS)
    hipLaunchKernelGGL(pixbw_fwd_wave_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, A);
  else
    hipLaunchKernelGGL(pixbw_fwd_kernel, dim3((unsigned)den_pixbw_blocks(N)), dim3(PIXBW_BLOCK), 0, (hipStream_t)stream, A);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_pixbw_bwd(int32_t S, int32_t N, int32_t reset, const float* it, const double* ts, const double* out_ts,
                  const float* prm, const float* delta_in, const double* reset_ts, const float* d_out,
                  const float* d_delta_out, void* workspace, float* d_it, float* d_delta_in, float* d_prm,
                  void* stream) {
  PixArgs A;
  int rc = pixbw_args(S, N, reset, it, ts, out_ts, prm, delta_in, reset_ts, &A);
  if (rc) return rc;
  if (!d_out || !workspace || !d_it || !d_prm || (!reset && !d_delta_in))
    return fail(DEN_EINVAL, "d_out, workspace, d_intensity, d_params_partial (and d_delta_in) are required");
  A.d_out = d_out;
  A.d_delta_out = reset ? d_delta_out : nullptr;
  A.ws = (double*)workspace;
  A.d_it = d_it;
  A.d_delta_in = d_delta_in;
  A.d_prm = d_prm;
  const int64_t seg_threads = 4 * (int64_t)(S - 1) * N;
  hipLaunchKernelGGL(pixbw_seg_kernel, dim3((unsigned)((seg_threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(pixbw_bwd_kernel, dim3((unsigned)den_pixbw_blocks(N)), dim3(PIXBW_BLOCK), 0, (hipStream_t)stream, A);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_event_loss_workspace_bytes(int32_t N) {
  const int nb = (N + LOSS_BLOCK - 1) / LOSS_BLOCK;
  return (size_t)(2 * nb + 2 + nb) * 4;
}

int den_event_loss_fwd(int32_t N, int32_t fn, const float* x, const float* target, const uint8_t* valid,
                       const float* c, float* loss, void* ws, void* stream) {
  if (N <= 0 || fn < 0 || fn > 3 || !x || !c || !loss || !ws) return fail(DEN_EINVAL, "bad arguments");
  const int nb = (N + LOSS_BLOCK - 1) / LOSS_BLOCK;
  float* part = (float*)ws;
  float* count = part + 2 * nb;
  hipLaunchKernelGGL(loss_partial_kernel, dim3(nb), dim3(LOSS_BLOCK), 0, (hipStream_t)stream, N, fn, x, target, valid,
                     c, part);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(LOSS_BLOCK), 0, (hipStream_t)stream, nb, part, loss, count);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_event_loss_bwd(int32_t N, int32_t fn, const float* x, const float* target, const uint8_t* valid,
                       const float* c, const float* gout, float* d_x, float* d_target, float* d_c, void* ws,
                       void* stream) {
  if (N <= 0 || fn < 0 || fn > 3 || !x || !c || !gout || !d_x || !d_c || !ws) return fail(DEN_EINVAL, "bad arguments");
  const int nb = (N + LOSS_BLOCK - 1) / LOSS_BLOCK;
  float* part = (float*)ws;
  float* count = part + 2 * nb;
  float* dcp = count + 2;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(nb), dim3(LOSS_BLOCK), 0, (hipStream_t)stream, N, fn, x, target, valid, c,
                     gout, count, d_x, d_target, dcp);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, 1, nb, (const float*)dcp, d_c);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_event_target(int32_t N, const double* ts_diff, const float* lid, const int64_t* end_ts,
                     const double* start_ts, const float* c, float* target, void* stream) {
  if (N <= 0 || !ts_diff || !lid || !end_ts || !start_ts || !c || !target) return fail(DEN_EINVAL, "bad arguments");
  hipLaunchKernelGGL(event_target_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, N, ts_diff, lid,
                     end_ts, start_ts, c, target);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_event_step_workspace_bytes(int32_t N) {
  const int nb = (N + LOSS_BLOCK - 1) / LOSS_BLOCK;
  return (size_t)(4 * nb + 8) * 4;
}

static EventStepArgs make_event_args(int32_t N, int32_t rd, int32_t fn_d, int32_t fn_t, int32_t has_bkgd,
                                     float min_int, float w_d, float w_t, const float* radiance, const float* opacity,
                                     const int64_t* channel, const float* target, const float* c, void* ws,
                                     float* out, float* d_radiance) {
  EventStepArgs E{};
  E.N = N; E.rd = rd; E.fn_d = fn_d; E.fn_t = fn_t; E.has_bkgd = has_bkgd;
  E.min_int = min_int; E.w_d = w_d; E.w_t = w_t;
  E.radiance = radiance; E.opacity = opacity; E.channel = channel; E.target = target; E.c = c;
  E.part = (float*)ws; E.out = out; E.d_radiance = d_radiance;
  return E;
}

int den_event_step_fwd(int32_t N, int32_t rd, int32_t fn_d, int32_t fn_t, int32_t has_bkgd, float min_int, float w_d,
                       float w_t, const float* radiance, const float* opacity, const int64_t* channel,
                       const float* target, const float* c, void* ws, float* out, void* stream) {
  if (N <= 0 || (rd != 1 && rd != 3) || fn_d < 0 || fn_d > 3 || fn_t < 0 || fn_t > 3 || !radiance || !target || !c ||
      !ws || !out || (!has_bkgd && !opacity) || (rd > 1 && !channel))
    return fail(DEN_EINVAL, "bad arguments");
  EventStepArgs E = make_event_args(N, rd, fn_d, fn_t, has_bkgd, min_int, w_d, w_t, radiance, opacity, channel,
                                    target, c, ws, out, nullptr);
  const int nb = (N + LOSS_BLOCK - 1) / LOSS_BLOCK;
  hipLaunchKernelGGL(event_step_partial_kernel, dim3(nb), dim3(LOSS_BLOCK), 0, (hipStream_t)stream, E);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(event_step_final_kernel, dim3(1), dim3(LOSS_BLOCK), 0, (hipStream_t)stream, E, nb);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_event_step_bwd(int32_t N, int32_t rd, int32_t fn_d, int32_t fn_t, int32_t has_bkgd, float min_int, float w_d,
                       float w_t, const float* radiance, const float* opacity, const int64_t* channel,
                       const float* target, const float* c, void* ws, float* d_radiance, void* stream) {
  if (N <= 0 || !radiance || !target || !c || !ws || !d_radiance || (!has_bkgd && !opacity) || (rd > 1 && !channel))
    return fail(DEN_EINVAL, "bad arguments");
  EventStepArgs E = make_event_args(N, rd, fn_d, fn_t, has_bkgd, min_int, w_d, w_t, radiance, opacity, channel,
                                    target, c, ws, nullptr, d_radiance);
  hipLaunchKernelGGL(event_step_bwd_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, E);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_event_prep(int32_t N, int32_t has_diff, int32_t has_tv, const int64_t* num_pos, const int64_t* num_neg,
                   const int64_t* end_ts, const int64_t* start_ts, const double* norm, const float* ct,
                   const double* refractory, const float* norm_c, float* lid, double* start_out, double* render_ts,
                   double* ts_diff, double* ts_subdiff, float* target, void* stream) {
  if (N <= 0 || !num_pos || !num_neg || !end_ts || !start_ts || !norm || !ct || !refractory || !lid || !start_out ||
      !render_ts || (target && (!norm_c || !has_diff)))
    return fail(DEN_EINVAL, "bad arguments");
  EventPrepArgs E{N, has_diff ? 1 : 0, has_tv ? 1 : 0, num_pos, num_neg, end_ts, start_ts, norm, ct, refractory,
                  norm_c, lid, start_out, render_ts, ts_diff, ts_subdiff, target};
  hipLaunchKernelGGL(event_prep_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, E);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_pixel_rays(int32_t M, int32_t N, const float* k_inv, const float* pixel, const float* t_pos,
                   const float* t_rot, float* ray_o, float* ray_d, void* stream) {
  if (M <= 0 || N <= 0 || (int64_t)M * N > (int64_t)INT32_MAX * 64 || !k_inv || !pixel || !t_pos || !t_rot ||
      !ray_o || !ray_d)
    return fail(DEN_EINVAL, "bad arguments");
  const int64_t n = (int64_t)M * N;
  hipLaunchKernelGGL(pixel_rays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, M, N,
                     k_inv, pixel, t_pos, t_rot, ray_o, ray_d);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_pixel_rays_bwd(int32_t M, int32_t N, const float* k_inv, const float* pixel, const float* t_rot,
                       const float* g_ray_o, const float* g_ray_d, float* d_t_pos, float* d_t_rot, void* stream) {
  if (M <= 0 || N <= 0 || (int64_t)M * N > (int64_t)INT32_MAX * 64 || !k_inv || !pixel || !t_rot ||
      (!d_t_pos && !d_t_rot))
    return fail(DEN_EINVAL, "bad arguments");
  const int64_t n = (int64_t)M * N;
  hipLaunchKernelGGL(pixel_rays_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, M,
                     N, k_inv, pixel, t_rot, g_ray_o, g_ray_d, d_t_pos, d_t_rot);
  DEN_LAUNCHED();
  return DEN_OK;
}

// ------------------------------------------------------------------ packed rendering (den_march.hip)
static int march_args(int32_t n_rays, const float* o, const float* d, const float* t_min, const float* t_max,
                      const float* roi, const int32_t* res, const uint8_t* grid, int32_t contraction, float step,
                      float cone, MarchArgs* M) {
  if (n_rays <= 0 || !o || !d || !t_min || !t_max || !(step > 0.0f) || !(cone >= 0.0f))
    return fail(DEN_EINVAL, "bad arguments");
  if (contraction < 0 || contraction > 2) return fail(DEN_EINVAL, "contraction must be 0, 1 or 2");
  if (grid && (!roi || !res || res[0] <= 0 || res[1] <= 0 || res[2] <= 0))
    return fail(DEN_EINVAL, "an occupancy grid needs roi and a positive resolution");
  *M = MarchArgs{};
  M->n_rays = n_rays;
  M->rays_o = o;
  M->rays_d = d;
  M->t_min = t_min;
  M->t_max = t_max;
  if (grid) {
    for (int a = 0; a < 6; ++a) M->roi[a] = roi[a];
    for (int a = 0; a < 3; ++a) M->res[a] = res[a];
  }
  M->grid = grid;
  M->contraction = grid ? contraction : CONTRACT_AABB;
  M->step = step;
  M->cone = cone;
  M->max_iter = 1 << 20;
  return DEN_OK;
}

int den_march_prep(int32_t n_rays, const float* rays_o, const float* rays_d, const float* aabb, float near_plane,
                   float far_plane, const float* jitter, float step, float* t_min, float* t_max, void* stream) {
  if (n_rays <= 0 || !rays_o || !rays_d || !t_min || !t_max || !(step > 0.0f)) return fail(DEN_EINVAL, "bad arguments");
  MarchPrepArgs P{};
  P.n_rays = n_rays;
  P.rays_o = rays_o;
  P.rays_d = rays_d;
  P.has_aabb = aabb ? 1 : 0;
  if (aabb)
    for (int a = 0; a < 6; ++a) P.aabb[a] = aabb[a];
  P.near_p = near_plane;
  P.far_p = far_plane;
  P.jitter = jitter;
  P.step = step;
  P.t_min = t_min;
  P.t_max = t_max;
  hipLaunchKernelGGL(march_prep_kernel, dim3((n_rays + 255) / 256), dim3(256), 0, (hipStream_t)stream, P);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_march_count(int32_t n_rays, const float* rays_o, const float* rays_d, const float* t_min, const float* t_max,
                    const float* roi, const int32_t* res, const uint8_t* grid, int32_t contraction, float step,
                    float cone, int32_t* counts, void* stream) {
  MarchArgs M;
  int rc = march_args(n_rays, rays_o, rays_d, t_min, t_max, roi, res, grid, contraction, step, cone, &M);
  if (rc) return rc;
  if (!counts) return fail(DEN_EINVAL, "counts is required");
  M.counts = counts;
  if (M.contraction != CONTRACT_AABB)
    hipLaunchKernelGGL(march_wave_kernel<false>, dim3((n_rays + 3) / 4), dim3(256), 0, (hipStream_t)stream, M);
  else
    hipLaunchKernelGGL(march_kernel<false>, dim3((n_rays + 127) / 128), dim3(128), 0, (hipStream_t)stream, M);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_march_fill(int32_t n_rays, const float* rays_o, const float* rays_d, const float* t_min, const float* t_max,
                   const float* roi, const int32_t* res, const uint8_t* grid, int32_t contraction, float step,
                   float cone, const int64_t* offsets, int32_t* ray_indices, float* t_starts, float* t_ends,
                   void* stream) {
  MarchArgs M;
  int rc = march_args(n_rays, rays_o, rays_d, t_min, t_max, roi, res, grid, contraction, step, cone, &M);
  if (rc) return rc;
  if (!offsets || !ray_indices || !t_starts || !t_ends) return fail(DEN_EINVAL, "null output");
  M.offsets = offsets;
  M.ray_idx = ray_indices;
  M.t0 = t_starts;
  M.t1 = t_ends;
  if (M.contraction != CONTRACT_AABB)
    hipLaunchKernelGGL(march_wave_kernel<true>, dim3((n_rays + 3) / 4), dim3(256), 0, (hipStream_t)stream, M);
  else
    hipLaunchKernelGGL(march_kernel<true>, dim3((n_rays + 127) / 128), dim3(128), 0, (hipStream_t)stream, M);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_scan_workspace_bytes(int64_t n) {
  return n <= 0 ? 8 : (size_t)((n + SCAN_TILE - 1) / SCAN_TILE) * sizeof(int64_t);
}

int den_exclusive_scan(int64_t n, const int32_t* counts, int64_t* offsets, void* workspace, void* stream) {
  if (n < 0 || !offsets || (n > 0 && (!counts || !workspace))) return fail(DEN_EINVAL, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    DEN_HIP(hipMemsetAsync(offsets, 0, sizeof(int64_t), st));
    return DEN_OK;
  }
  const int64_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  int64_t* sums = (int64_t*)workspace;
  hipLaunchKernelGGL(scan_tile_kernel, dim3((unsigned)tiles), dim3(SCAN_BLOCK), 0, st, n, counts, offsets, sums);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(SCAN_BLOCK), 0, st, tiles, sums, offsets, n);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, (const int64_t*)sums,
                     offsets);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_pack_info(int32_t n_rays, int64_t n, const int32_t* ray_indices, int64_t* offsets, void* stream) {
  if (n_rays <= 0 || n < 0 || !offsets || (n > 0 && !ray_indices)) return fail(DEN_EINVAL, "bad arguments");
  hipLaunchKernelGGL(pack_info_kernel, dim3((n_rays + 256) / 256), dim3(256), 0, (hipStream_t)stream, n_rays, n,
                     ray_indices, offsets);
  DEN_LAUNCHED();
  return DEN_OK;
}

constexpr int RAYS_PER_WG = 4;  // one wave per ray

int den_visibility(int32_t n_rays, const int64_t* offsets, const float* t_starts, const float* t_ends,
                   const float* sigmas, const float* alphas, float early_stop_eps, float alpha_thre, uint8_t* keep,
                   int32_t* counts, void* stream) {
  if (n_rays <= 0 || !offsets || !t_starts || !t_ends || (!sigmas && !alphas) || !keep || !counts)
    return fail(DEN_EINVAL, "bad arguments");
  VisArgs V{};
  V.n_rays = n_rays;
  V.offsets = offsets;
  V.t0 = t_starts;
  V.t1 = t_ends;
  V.sigma = sigmas;
  V.alpha = sigmas ? nullptr : alphas;
  V.early_stop_eps = early_stop_eps;
  V.alpha_thre = alpha_thre;
  V.keep = keep;
  V.counts = counts;
  hipLaunchKernelGGL(visibility_kernel, dim3((n_rays + RAYS_PER_WG - 1) / RAYS_PER_WG), dim3(64 * RAYS_PER_WG), 0,
                     (hipStream_t)stream, V);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_compact(int32_t n_rays, const int64_t* offsets, const uint8_t* keep, const int64_t* out_offsets,
                const int32_t* ray_indices, const float* t_starts, const float* t_ends, int32_t* out_ray_indices,
                float* out_t_starts, float* out_t_ends, void* stream) {
  if (n_rays <= 0 || !offsets || !keep || !out_offsets || !ray_indices || !t_starts || !t_ends || !out_ray_indices ||
      !out_t_starts || !out_t_ends)
    return fail(DEN_EINVAL, "bad arguments");
  VisArgs V{};
  V.n_rays = n_rays;
  V.offsets = offsets;
  V.t0 = t_starts;
  V.t1 = t_ends;
  V.keep = (uint8_t*)keep;
  V.out_offsets = out_offsets;
  V.in_ray = ray_indices;
  V.out_ray = out_ray_indices;
  V.out_t0 = out_t_starts;
  V.out_t1 = out_t_ends;
  hipLaunchKernelGGL(compact_kernel, dim3((n_rays + RAYS_PER_WG - 1) / RAYS_PER_WG), dim3(64 * RAYS_PER_WG), 0,
                     (hipStream_t)stream, V);
  DEN_LAUNCHED();
  return DEN_OK;
}

static int composite_fwd_impl(int alpha, int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts,
                              const float* t_ends, const float* sigmas, const float* rgbs, const float* bkgd,
                              float* colors, float* opacities, float* depths, void* stream) {
  if (n_rays <= 0 || rd < 1 || rd > 3 || !offsets || !t_starts || !t_ends || !sigmas || !rgbs || !colors ||
      !opacities || !depths)
    return fail(DEN_EINVAL, "bad arguments");
  CompArgs C{};
  C.n_rays = n_rays;
  C.rd = rd;
  C.offsets = offsets;
  C.t0 = t_starts;
  C.t1 = t_ends;
  C.sigma = sigmas;
  C.rgb = rgbs;
  C.bkgd = bkgd;
  C.color = colors;
  C.opacity = opacities;
  C.depth = depths;
  C.alpha = alpha;
  hipLaunchKernelGGL(composite_fwd_kernel, dim3((n_rays + RAYS_PER_WG - 1) / RAYS_PER_WG), dim3(64 * RAYS_PER_WG), 0,
                     (hipStream_t)stream, C);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_composite_workspace_bytes(int32_t n_rays, int32_t rd) {
  return n_rays > 0 && rd > 0 ? (size_t)n_rays * rd * sizeof(float) : 0;
}

static int composite_bwd_impl(int alpha, int32_t n_rays, int32_t rd, const int64_t* offsets,
                              const float* t_starts, const float* t_ends, const float* sigmas, const float* rgbs,
                              const float* bkgd, const float* d_colors, const float* d_opacities,
                              const float* d_depths, float* d_sigmas, float* d_rgbs, float* d_bkgd, void* workspace,
                              void* stream) {
  if (n_rays <= 0 || rd < 1 || rd > 3 || !offsets || !t_starts || !t_ends || !sigmas || !rgbs || !d_colors ||
      !d_sigmas || !d_rgbs || (d_bkgd && (!bkgd || !workspace)))
    return fail(DEN_EINVAL, "bad arguments");
  CompArgs C{};
  C.n_rays = n_rays;
  C.rd = rd;
  C.offsets = offsets;
  C.t0 = t_starts;
  C.t1 = t_ends;
  C.sigma = sigmas;
  C.rgb = rgbs;
  C.bkgd = bkgd;
  C.d_color = d_colors;
  C.d_opacity = d_opacities;
  C.d_depth = d_depths;
  C.d_sigma = d_sigmas;
  C.d_rgb = d_rgbs;
  C.bkgd_partial = d_bkgd ? (float*)workspace : nullptr;
  C.alpha = alpha;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(composite_bwd_kernel, dim3((n_rays + RAYS_PER_WG - 1) / RAYS_PER_WG), dim3(64 * RAYS_PER_WG), 0,
                     st, C);
  DEN_LAUNCHED();
  if (d_bkgd) {
    hipLaunchKernelGGL(sum_partials_kernel, dim3(rd), dim3(256), 0, st, rd, n_rays, (const float*)workspace, d_bkgd);
    DEN_LAUNCHED();
  }
  return DEN_OK;
}

int den_composite_fwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts, const float* t_ends,
                      const float* sigmas, const float* rgbs, const float* bkgd, float* colors, float* opacities,
                      float* depths, void* stream) {
  return composite_fwd_impl(0, n_rays, rd, offsets, t_starts, t_ends, sigmas, rgbs, bkgd, colors, opacities, depths,
                            stream);
}
int den_composite_alpha_fwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts,
                            const float* t_ends, const float* alphas, const float* rgbs, const float* bkgd,
                            float* colors, float* opacities, float* depths, void* stream) {
  return composite_fwd_impl(1, n_rays, rd, offsets, t_starts, t_ends, alphas, rgbs, bkgd, colors, opacities, depths,
                            stream);
}
int den_composite_bwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts, const float* t_ends,
                      const float* sigmas, const float* rgbs, const float* bkgd, const float* d_colors,
                      const float* d_opacities, const float* d_depths, float* d_sigmas, float* d_rgbs, float* d_bkgd,
                      void* workspace, void* stream) {
  return composite_bwd_impl(0, n_rays, rd, offsets, t_starts, t_ends, sigmas, rgbs, bkgd, d_colors, d_opacities,
                            d_depths, d_sigmas, d_rgbs, d_bkgd, workspace, stream);
}
int den_composite_alpha_bwd(int32_t n_rays, int32_t rd, const int64_t* offsets, const float* t_starts,
                            const float* t_ends, const float* alphas, const float* rgbs, const float* bkgd,
                            const float* d_colors, const float* d_opacities, const float* d_depths, float* d_alphas,
                            float* d_rgbs, float* d_bkgd, void* workspace, void* stream) {
  return composite_bwd_impl(1, n_rays, rd, offsets, t_starts, t_ends, alphas, rgbs, bkgd, d_colors, d_opacities,
                            d_depths, d_alphas, d_rgbs, d_bkgd, workspace, stream);
}

constexpr int OCC_NB = 1024;  // fixed reduction width (deterministic mean)

size_t den_occ_workspace_bytes(void) { return OCC_NB * sizeof(float); }

int den_occ_points(int64_t m, const int64_t* cell_indices, const float* jitter, const int32_t* res, const float* roi,
                   int32_t contraction, float* points, uint8_t* mask, uint8_t* sampled, void* stream) {
  if (m <= 0 || !cell_indices || !jitter || !res || !roi || !points || !mask || !sampled || contraction < 0 ||
      contraction > 2)
    return fail(DEN_EINVAL, "bad arguments");
  OccArgs A{};
  A.m = m;
  A.idx = cell_indices;
  A.u = jitter;
  for (int a = 0; a < 3; ++a) A.res[a] = res[a];
  for (int a = 0; a < 6; ++a) A.roi[a] = roi[a];
  A.contraction = contraction;
  A.pts = points;
  A.mask = mask;
  A.sampled = sampled;
  hipLaunchKernelGGL(occ_points_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_occ_update(int64_t m, const int64_t* cell_indices, const uint8_t* mask, const float* sigmas,
                   const float* step_sizes, float step_size, float ema_decay, float occ_thre, int64_t cells,
                   float* occs, uint8_t* sampled, uint8_t* binary, void* workspace, void* stream) {
  if (m <= 0 || cells <= 0 || !cell_indices || !mask || !sigmas || !occs || !sampled || !binary || !workspace)
    return fail(DEN_EINVAL, "bad arguments");
  OccArgs A{};
  A.m = m;
  A.idx = cell_indices;
  A.mask = (uint8_t*)mask;
  A.sigma = sigmas;
  A.step = step_sizes;
  A.step_c = step_size;
  A.decay = ema_decay;
  A.occ_thre = occ_thre;
  A.cells = cells;
  A.occs = occs;
  A.sampled = sampled;
  A.binary = binary;
  A.part = (float*)workspace;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(occ_decay_kernel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, st, A);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(occ_max_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, A);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(occ_mean_partial_kernel, dim3(OCC_NB), dim3(OCC_BLOCK), 0, st, A);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(occ_binary_kernel, dim3(1024), dim3(256), 0, st, A, OCC_NB);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_trajectory(int64_t n, int32_t C, const int64_t* cam_ts, const float* cam_pos, const float* cam_quat,
                   const double* query_ts, float* position, float* rotation, int32_t* status, void* stream) {
  if (n < 0 || C < 2 || !cam_ts || !cam_pos || !cam_quat || (n > 0 && (!query_ts || !position || !rotation)))
    return fail(DEN_EINVAL, "bad arguments (a trajectory needs >= 2 poses)");
  if (n == 0) return DEN_OK;
  TrajArgs T{n, C, cam_ts, cam_pos, cam_quat, query_ts, position, rotation, status};
  hipLaunchKernelGGL(trajectory_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_trajectory_bwd(int64_t n, int32_t C, const int64_t* cam_ts, const float* cam_pos, const float* cam_quat,
                       const double* query_ts, const float* g_position, const float* g_rotation, double* d_query_ts,
                       void* stream) {
  if (n < 0 || C < 2 || !cam_ts || !cam_pos || !cam_quat || (n > 0 && (!query_ts || !d_query_ts)))
    return fail(DEN_EINVAL, "bad arguments (a trajectory needs >= 2 poses)");
  if (n == 0) return DEN_OK;
  TrajArgs T{n, C, cam_ts, cam_pos, cam_quat, query_ts, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(trajectory_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T,
                     g_position, g_rotation, d_query_ts);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_event_prep_workspace_bytes(int32_t N) {
  return N > 0 ? (size_t)(4 * ((N + PREP_BWD_BLOCK - 1) / PREP_BWD_BLOCK)) * sizeof(double) : 0;
}

int den_event_prep_bwd(int32_t N, int32_t has_diff, int32_t has_tv, const int64_t* num_pos, const int64_t* num_neg,
                       const int64_t* end_ts, const int64_t* start_ts, const double* norm, const float* ct,
                       const double* refractory, const float* norm_c, const float* g_lid, const double* g_start,
                       const double* g_render_ts, const double* g_ts_diff, const double* g_ts_subdiff,
                       const float* g_target, void* workspace, double* d_params, void* stream) {
  if (N <= 0 || !num_pos || !num_neg || !end_ts || !start_ts || !norm || !ct || !refractory || !workspace ||
      !d_params || (g_target && (!norm_c || !has_diff)))
    return fail(DEN_EINVAL, "bad arguments");
  EventPrepBwdArgs B{};
  B.F = EventPrepArgs{N, has_diff ? 1 : 0, has_tv ? 1 : 0, num_pos, num_neg, end_ts, start_ts, norm, ct, refractory,
                      norm_c, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  B.g_lid = g_lid;
  B.g_start = g_start;
  B.g_render = g_render_ts;
  B.g_ts_diff = g_ts_diff;
  B.g_ts_subdiff = g_ts_subdiff;
  B.g_target = g_target;
  B.part = (double*)workspace;
  const int nb = (N + PREP_BWD_BLOCK - 1) / PREP_BWD_BLOCK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(event_prep_bwd_kernel, dim3(nb), dim3(PREP_BWD_BLOCK), 0, st, B);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(sum_partials_f64_kernel, dim3(4), dim3(256), 0, st, 4, nb, (const double*)B.part, d_params);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_event_target_bwd(int32_t N, const double* ts_diff, const float* lid, const int64_t* end_ts,
                         const double* start_ts, const float* norm_c, const float* g_target, double* d_ts_diff,
                         float* d_lid, double* d_start, void* workspace, double* d_c, void* stream) {
  if (N <= 0 || !ts_diff || !lid || !end_ts || !start_ts || !norm_c || !g_target || !workspace || !d_c)
    return fail(DEN_EINVAL, "bad arguments");
  const int nb = (N + PREP_BWD_BLOCK - 1) / PREP_BWD_BLOCK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(event_target_bwd_kernel, dim3(nb), dim3(PREP_BWD_BLOCK), 0, st, N, ts_diff, lid, end_ts, start_ts,
                     norm_c, g_target, d_ts_diff, d_lid, d_start, (double*)workspace);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(sum_partials_f64_kernel, dim3(1), dim3(256), 0, st, 1, nb, (const double*)workspace, d_c);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_image_error_workspace_bytes(int32_t n_img) {
  return n_img > 0 ? (size_t)n_img * 2 * IMG_SLICES * sizeof(double) : 0;
}

int den_image_error(int32_t n_img, int64_t pixels, const float* pred, const float* target, void* workspace,
                    double* sse_sae, void* stream) {
  if (n_img <= 0 || pixels <= 0 || !pred || !target || !workspace || !sse_sae) return fail(DEN_EINVAL, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(image_error_kernel, dim3(IMG_SLICES, n_img), dim3(IMG_BLOCK), 0, st, pixels, pred, target,
                     (double*)workspace);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(sum_partials_f64_kernel, dim3(2 * n_img), dim3(256), 0, st, 2 * n_img, IMG_SLICES,
                     (const double*)workspace, sse_sae);
  DEN_LAUNCHED();
  return DEN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- ngp radiance field
namespace {
// tcnn's GridEncodingTemplated sizing, float32 host arithmetic (oracle/tcnn.py grid_levels)
bool ngp_grid(const den_ngp_desc* d, NgpGrid* G, int64_t* table_floats) {
  if (!d || d->n_levels < 1 || d->n_levels > NGP_MAX_LEVELS || d->n_features_per_level != NGP_F ||
      d->log2_hashmap_size < 1 || d->log2_hashmap_size > 30 || d->base_resolution < 1 || !(d->per_level_scale >= 1.0f) ||
      (d->grid_type != 0 && d->grid_type != 1) || (d->radiance_dim != 1 && d->radiance_dim != 3) ||
      d->hidden_activation < 0 || d->hidden_activation > 1 || d->radiance_activation < 0 ||
      d->radiance_activation > 1 || d->contraction < 0 || d->contraction > 2 || d->density_activation < 0 ||
      d->density_activation > 2)
    return false;
  NgpGrid g{};
  g.n_levels = d->n_levels;
  g.hashed = d->grid_type == 0;
  // f32 steps as tcnn's grid_scale, exp2 / log2 evaluated in double and rounded once (the oracle,
  // oracle/tcnn.py grid_levels, does the same)
  const float log2_pls = (float)std::log2((double)d->per_level_scale);
  uint64_t off = 0;
  for (int l = 0; l < d->n_levels; ++l) {
    const float e = (float)l * log2_pls;
    const float scale = (float)std::exp2((double)e) * (float)d->base_resolution - 1.0f;
    const uint32_t res = (uint32_t)std::ceil(scale) + 1;
    const uint32_t max_params = 0xFFFFFFFFu / 2;
    uint64_t entries = std::pow((float)res, 3.0f) > (float)max_params ? max_params : (uint64_t)res * res * res;
    entries = (entries + 7) / 8 * 8;
    if (g.hashed) entries = std::min<uint64_t>(entries, 1ull << d->log2_hashmap_size);
    if (off + entries > 0x7FFFFFFFull) return false;
    g.scale[l] = scale;
    g.res[l] = res;
    g.entries[l] = (uint32_t)entries;
    g.offset[l] = (uint32_t)off;
    off += entries;
  }
  *G = g;
  *table_floats = (int64_t)off * NGP_F;
  return true;
}

// workgroups of the MFMA field kernels: one 32-sample tile per wave, capped (they loop)
unsigned ngp_mf_grid(int64_t n) {
  const int64_t wg = ((n + 31) / 32 + NM_WAVES - 1) / NM_WAVES;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(wg, NM_GRID));
}

struct NgpWs {
  size_t save, dz, partial, total;
  int splits;
  int64_t per_split;
};
int64_t ngp_ld(int64_t n) { return (n + 63) / 64 * 64; }
NgpWs ngp_ws(int64_t n) {
  NgpWs w{};
  size_t off = 0;
  w.save = off;
  off += align256((size_t)NS_ROWS * ngp_ld(n) * 4);
  w.dz = off;
  off += align256((size_t)ND_ROWS * ngp_ld(n) * 4);
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>(256, (n + 4095) / 4096));
  int64_t per = (n + splits - 1) / splits;
  per = (per + NDW_CHUNK - 1) / NDW_CHUNK * NDW_CHUNK;
  w.splits = (int)((n + per - 1) / per);
  w.per_split = per;
  w.partial = off;
  off += align256((size_t)NDW_TASKS * w.splits * NDW_PART * 4);
  w.total = off;
  return w;
}
}  // namespace

extern "C" {

int64_t den_ngp_table_params(const den_ngp_desc* desc) {
  NgpGrid g;
  int64_t t;
  return ngp_grid(desc, &g, &t) ? t : -1;
}

int64_t den_ngp_param_count(const den_ngp_desc* desc) {
  const int64_t t = den_ngp_table_params(desc);
  return t < 0 ? -1 : t + ngp_mlp_params(2 * desc->n_levels, desc->radiance_dim);
}

size_t den_ngp_workspace_bytes(const den_ngp_desc* desc, int64_t n, int32_t train) {
  if (!train || n <= 0 || den_ngp_table_params(desc) < 0) return 0;
  return ngp_ws(n).total;
}

int den_ngp_fwd(const den_ngp_desc* desc, int64_t n, int32_t points, const float* x, const float* d,
                const int32_t* ray_idx, const float* t0, const float* t1, const float* params, int32_t density_only,
                int32_t train, void* workspace, float* out_rgb, float* out_sigma, void* stream) {
  NgpGrid g;
  int64_t tfl;
  if (!ngp_grid(desc, &g, &tfl)) return fail(DEN_EUNSUPPORTED, "unsupported ngp descriptor");
  if (n < 0 || (points != 1 && points != 2) || !params || !out_sigma || (!density_only && !out_rgb) ||
      (train && (!workspace || density_only)) || (n > 0 && (!x || !d)) ||
      (points == 2 && n > 0 && (!ray_idx || !t0 || !t1)))
    return fail(DEN_EINVAL, "bad arguments");
  if (n == 0) return DEN_OK;
  NgpArgs A{};
  A.n = n;
  A.rd = desc->radiance_dim;
  A.points = points;
  A.contraction = desc->contraction;
  A.hidden_relu = desc->hidden_activation;
  A.density_act = desc->density_activation;
  A.rad_sigmoid = desc->radiance_activation;
  A.density_only = density_only ? 1 : 0;
  for (int i = 0; i < 6; ++i) A.aabb[i] = desc->aabb[i];
  A.x = x;
  A.d = d;
  A.ray_idx = ray_idx;
  A.t0 = t0;
  A.t1 = t1;
  A.table = params;
  A.mlp = params + tfl;
  A.off = ngp_offsets(2 * g.n_levels, desc->radiance_dim);
  A.enc = 2 * g.n_levels;
  A.grid = g;
  A.out_rgb = out_rgb;
  A.out_sigma = out_sigma;
  A.ld = ngp_ld(n);
  A.save = train ? (float*)((char*)workspace + ngp_ws(n).save) : nullptr;
  if (A.hidden_relu)
    hipLaunchKernelGGL(ngp_fwd_mfma_kernel<true>, dim3(ngp_mf_grid(n)), dim3(NM_THREADS), 0, (hipStream_t)stream, A);
  else
    hipLaunchKernelGGL(ngp_fwd_mfma_kernel<false>, dim3(ngp_mf_grid(n)), dim3(NM_THREADS), 0, (hipStream_t)stream, A);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_ngp_bwd(const den_ngp_desc* desc, int64_t n, const float* params, void* workspace, const float* d_rgb,
                const float* d_sigma, float* grad_params, void* stream) {
  NgpGrid g;
  int64_t tfl;
  if (!ngp_grid(desc, &g, &tfl)) return fail(DEN_EUNSUPPORTED, "unsupported ngp descriptor");
  if (n < 0 || !params || !workspace || !grad_params) return fail(DEN_EINVAL, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  DEN_HIP(hipMemsetAsync(grad_params, 0, (size_t)tfl * 4, st));
  if (n == 0) {
    DEN_HIP(hipMemsetAsync(grad_params + tfl, 0, (size_t)ngp_mlp_params(2 * g.n_levels, desc->radiance_dim) * 4, st));
    return DEN_OK;
  }
  const NgpWs W = ngp_ws(n);
  char* ws = (char*)workspace;
  NgpArgs A{};
  A.n = n;
  A.rd = desc->radiance_dim;
  A.hidden_relu = desc->hidden_activation;
  A.density_act = desc->density_activation;
  A.rad_sigmoid = desc->radiance_activation;
  A.mlp = params + tfl;
  A.off = ngp_offsets(2 * g.n_levels, desc->radiance_dim);
  A.enc = 2 * g.n_levels;
  A.grid = g;
  A.ld = ngp_ld(n);
  A.save = (float*)(ws + W.save);
  A.d_rgb = d_rgb;
  A.d_sigma = d_sigma;
  A.d_table = grad_params;
  A.dz = (float*)(ws + W.dz);
  if (A.hidden_relu)
    hipLaunchKernelGGL(ngp_bwd_mfma_kernel<true>, dim3(ngp_mf_grid(n)), dim3(NM_THREADS), 0, st, A);
  else
    hipLaunchKernelGGL(ngp_bwd_mfma_kernel<false>, dim3(ngp_mf_grid(n)), dim3(NM_THREADS), 0, st, A);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(ngp_scatter_kernel, dim3((unsigned)((n + NSC_THREADS - 1) / NSC_THREADS)), dim3(NSC_THREADS), 0, st,
                     A);
  DEN_LAUNCHED();
  const int rd = desc->radiance_dim;
  const NgpOff& O = A.off;
  NgpDwMfArgs Q{};
  Q.dz = A.dz;
  Q.save = A.save;
  Q.n = n;
  Q.ld = A.ld;
  Q.per_split = W.per_split;
  Q.splits = W.splits;
  Q.partial = (float*)(ws + W.partial);
  Q.grad = grad_params + tfl;
  Q.T[0] = NgpDwTask{ND_Z0, NGP_W, 2, NS_FEAT, A.enc, A.enc, 0, O.w[0], O.b[0]};
  Q.T[1] = NgpDwTask{ND_O, 1 + NGP_GEO, 1, NS_H0, NGP_W, NGP_W, 0, O.w[1], O.b[1]};
  Q.T[2] = NgpDwTask{ND_Z2, NGP_W, 2, NS_HIN, NGP_HIN, NGP_HIN, 0, O.w[2], O.b[2]};
  Q.T[3] = NgpDwTask{ND_Z3, 32, 1, NS_H1, NGP_W, NGP_W, 0, O.w[3], O.b[3]};
  Q.T[4] = NgpDwTask{ND_Z3 + 32, 32, 1, NS_H1, NGP_W, NGP_W, 32, O.w[3], O.b[3]};
  Q.T[5] = NgpDwTask{ND_R, rd, 1, NS_H2, NGP_W, NGP_W, 0, O.w[4], O.b[4]};
  // tasks 0, 2: two row tiles; 1, 3, 4, 5: one
  hipLaunchKernelGGL(ngp_dw_mfma_kernel<2>, dim3((unsigned)W.splits, 2), dim3(256), 0, st, Q, 0, 2);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(ngp_dw_mfma_kernel<1>, dim3((unsigned)W.splits, 1), dim3(256), 0, st, Q, 1, 0);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(ngp_dw_mfma_kernel<1>, dim3((unsigned)W.splits, 3), dim3(256), 0, st, Q, 3, 1);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(ngp_dw_mfma_reduce_kernel, dim3((NDW_PART + 63) / 64, NDW_TASKS), dim3(256), 0, st, Q);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_ngp_ray_grad_workspace_bytes(int64_t n) { return n > 0 ? (size_t)n * 6 * sizeof(float) : 0; }

int den_ngp_ray_grad(const den_ngp_desc* desc, int64_t n, int32_t points, int32_t n_rays, const float* x,
                     const float* d, const int32_t* ray_idx, const float* t0, const float* t1, const float* params,
                     void* workspace, void* rg_workspace, float* d_x, float* d_d, void* stream) {
  NgpGrid g;
  int64_t tfl;
  if (!ngp_grid(desc, &g, &tfl)) return fail(DEN_EUNSUPPORTED, "unsupported ngp descriptor");
  if (n < 0 || (points != 1 && points != 2) || !params || !workspace || !d_x || !d_d || (n > 0 && !rg_workspace) ||
      (n > 0 && (!x || !d)) || (points == 2 && (n_rays <= 0 || (n > 0 && (!ray_idx || !t0 || !t1)))))
    return fail(DEN_EINVAL, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    if (points == 2) {
      DEN_HIP(hipMemsetAsync(d_x, 0, (size_t)n_rays * 3 * 4, st));
      DEN_HIP(hipMemsetAsync(d_d, 0, (size_t)n_rays * 3 * 4, st));
    }
    return DEN_OK;
  }
  const NgpWs W = ngp_ws(n);
  char* ws = (char*)workspace;
  RayGradArgs G{};
  G.points = points;
  G.contraction = desc->contraction;
  G.rd = desc->radiance_dim;
  G.n = n;
  for (int i = 0; i < 6; ++i) G.aabb[i] = desc->aabb[i];
  G.rays_o = x;
  G.rays_d = d;
  G.ray_idx = ray_idx;
  G.t0 = t0;
  G.t1 = t1;
  G.per_sample = (float*)rg_workspace;
  RayGradNgp Q{};
  Q.table = params;
  Q.mlp = params + tfl;
  Q.off = ngp_offsets(2 * g.n_levels, desc->radiance_dim);
  Q.grid = g;
  Q.ld = ngp_ld(n);
  Q.save = (const float*)(ws + W.save);
  Q.dz = (const float*)(ws + W.dz);
  const unsigned grid = (unsigned)((n + RG_THREADS - 1) / RG_THREADS);
  hipLaunchKernelGGL(raygrad_ngp_kernel, dim3(grid), dim3(RG_THREADS), 0, st, G, Q);
  DEN_LAUNCHED();
  if (points == 1)
    hipLaunchKernelGGL(raygrad_split_kernel, dim3(grid), dim3(RG_THREADS), 0, st, n, G.per_sample, d_x, d_d);
  else
    hipLaunchKernelGGL(raygrad_reduce_kernel, dim3((n_rays + 3) / 4), dim3(256), 0, st, n_rays, 2, 0, ray_idx, n,
                       G.per_sample, d_x, d_d);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_hashgrid_fwd(const den_ngp_desc* desc, int64_t n, const float* x, const float* table, float* out,
                     void* stream) {
  NgpGrid g;
  int64_t tfl;
  if (!ngp_grid(desc, &g, &tfl)) return fail(DEN_EUNSUPPORTED, "unsupported grid descriptor");
  if (n < 0 || (n > 0 && (!x || !table || !out))) return fail(DEN_EINVAL, "bad arguments");
  if (n == 0) return DEN_OK;
  NgpEncArgs E{n, g, x, table, out, nullptr, nullptr};
  hipLaunchKernelGGL(ngp_encode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, E);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_hashgrid_bwd(const den_ngp_desc* desc, int64_t n, const float* x, const float* d_out, float* d_table,
                     void* stream) {
  NgpGrid g;
  int64_t tfl;
  if (!ngp_grid(desc, &g, &tfl)) return fail(DEN_EUNSUPPORTED, "unsupported grid descriptor");
  if (n < 0 || (n > 0 && (!x || !d_out || !d_table))) return fail(DEN_EINVAL, "bad arguments");
  if (n == 0) return DEN_OK;
  NgpEncArgs E{n, g, x, nullptr, nullptr, d_out, d_table};
  hipLaunchKernelGGL(ngp_encode_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     E);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_sh_encode_fwd(int64_t n, int32_t degree, const float* coords, float* out, void* stream) {
  if (degree < 1 || degree > SH_MAX_DEG) return fail(DEN_EINVAL, "SH degree must be in 1..8");
  if (n < 0 || (n > 0 && (!coords || !out))) return fail(DEN_EINVAL, "bad arguments");
  if (n == 0) return DEN_OK;
  sh_dispatch(degree, false, n, coords, nullptr, out, (hipStream_t)stream);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_sh_encode_bwd(int64_t n, int32_t degree, const float* coords, const float* d_out, float* d_coords,
                      void* stream) {
  if (degree < 1 || degree > SH_MAX_DEG) return fail(DEN_EINVAL, "SH degree must be in 1..8");
  if (n < 0 || (n > 0 && (!coords || !d_out || !d_coords))) return fail(DEN_EINVAL, "bad arguments");
  if (n == 0) return DEN_OK;
  sh_dispatch(degree, true, n, coords, d_out, d_coords, (hipStream_t)stream);
  DEN_LAUNCHED();
  return DEN_OK;
}

}  // extern "C"

// ---- raw-event preprocessing (den_dataset.hip)
namespace {
struct QueueWs {
  size_t keys[2], vals[2], counts, totals, scal, valid, start, offsets, scan, total;
  int64_t n_tiles;
};
QueueWs queue_ws(int64_t n) {
  QueueWs W{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += align256(bytes); return o; };
  W.n_tiles = (n + QS_TILE - 1) / QS_TILE;
  for (int b = 0; b < 2; ++b) W.keys[b] = take((size_t)n * 4);
  for (int b = 0; b < 2; ++b) W.vals[b] = take((size_t)n * 4);
  W.counts = take((size_t)QS_RADIX * W.n_tiles * 4);
  W.totals = take(QS_RADIX * 4);
  W.scal = take(64);  // status i32 | min interval (biased u64) | interval count u64
  W.valid = take((size_t)n * 4);
  W.start = take((size_t)n * 8);
  W.offsets = take((size_t)(n + 1) * 8);
  W.scan = take(den_scan_workspace_bytes(n));
  W.total = off;
  return W;
}
__global__ void queue_init_kernel(int32_t* status, unsigned long long* min_biased, unsigned long long* n_int) {
  *status = 0;
  *min_biased = ~0ull;  // INT64_MAX biased
  *n_int = 0;
}
__global__ void queue_empty_kernel(int64_t* stats) {
  stats[0] = 0;
  stats[1] = INT64_MAX;
  stats[2] = 0;
}

// shared body of den_queue_raw_events / den_max_refractory_period (out_position == null: stats only)
int queue_impl(int64_t n, int32_t H, int32_t W_, const int64_t* position, const int64_t* ts, const uint8_t* polarity,
               void* workspace, size_t ws_bytes, int64_t* out_position, int64_t* out_start, int64_t* out_end,
               int64_t* out_pos, int64_t* out_neg, int64_t* stats, hipStream_t st) {
  if (n < 0 || H <= 0 || W_ <= 0 || !stats || (n > 0 && (!position || !ts || !workspace)))
    return fail(DEN_EINVAL, "bad arguments");
  if (out_position && (!polarity || !out_start || !out_end || !out_pos || !out_neg))
    return fail(DEN_EINVAL, "bad arguments: queued-event outputs");
  if (n > (int64_t)UINT32_MAX - 1 || (int64_t)H * W_ > (int64_t)UINT32_MAX)
    return fail(DEN_EUNSUPPORTED, "more than 2^32 - 1 events or pixels");
  if (n == 0) {
    hipLaunchKernelGGL(queue_empty_kernel, dim3(1), dim3(1), 0, st, stats);
    DEN_LAUNCHED();
    return DEN_OK;
  }
  const QueueWs L = queue_ws(n);
  if (ws_bytes < L.total) return fail(DEN_EINVAL, "workspace too small (den_queue_workspace_bytes)");
  char* ws = (char*)workspace;
  uint32_t* keys[2] = {(uint32_t*)(ws + L.keys[0]), (uint32_t*)(ws + L.keys[1])};
  uint32_t* vals[2] = {(uint32_t*)(ws + L.vals[0]), (uint32_t*)(ws + L.vals[1])};
  uint32_t* counts = (uint32_t*)(ws + L.counts);
  uint32_t* totals = (uint32_t*)(ws + L.totals);
  int32_t* status = (int32_t*)(ws + L.scal);
  unsigned long long* min_biased = (unsigned long long*)(ws + L.scal + 8);
  unsigned long long* n_int = (unsigned long long*)(ws + L.scal + 16);
  int32_t* valid = (int32_t*)(ws + L.valid);
  int64_t* start = (int64_t*)(ws + L.start);
  int64_t* offsets = (int64_t*)(ws + L.offsets);
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(queue_init_kernel, dim3(1), dim3(1), 0, st, status, min_biased, n_int);
  hipLaunchKernelGGL(queue_keys_kernel, dim3(blocks), dim3(256), 0, st, n, H, W_, position, keys[0], vals[0], status);
  DEN_LAUNCHED();
  // pixel keys need ceil(log2(H * W)) bits: 8-bit digits, LSD, stable
  int bits = 0;
  while (bits < 32 && (((int64_t)1) << bits) < (int64_t)H * W_) ++bits;
  int cur = 0;
  for (int shift = 0; shift < bits; shift += 8) {
    hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)L.n_tiles), dim3(QS_THREADS), 0, st, n, shift, keys[cur],
                       counts, L.n_tiles);
    hipLaunchKernelGGL(radix_scan_kernel, dim3(QS_RADIX), dim3(QS_THREADS), 0, st, L.n_tiles, counts, totals);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)L.n_tiles), dim3(QS_THREADS), 0, st, n, shift, keys[cur],
                       vals[cur], counts, totals, L.n_tiles, keys[cur ^ 1], vals[cur ^ 1]);
    DEN_LAUNCHED();
    cur ^= 1;
  }
  hipLaunchKernelGGL(queue_mark_kernel, dim3(blocks), dim3(256), 0, st, n, keys[cur], vals[cur], ts, valid, start,
                     min_biased, n_int);
  DEN_LAUNCHED();
  if (out_position) {
    int rc = den_exclusive_scan(n, valid, offsets, ws + L.scan, st);
    if (rc != DEN_OK) return rc;
  }
  QueueEmitArgs E{};
  E.n = n;
  E.position = position;
  E.ts = ts;
  E.polarity = polarity;
  E.valid = valid;
  E.offsets = offsets;
  E.start_tmp = start;
  E.out_position = out_position;
  E.out_start_ts = out_start;
  E.out_end_ts = out_end;
  E.out_num_pos = out_pos;
  E.out_num_neg = out_neg;
  E.status = status;
  E.min_biased = min_biased;
  E.n_intervals = n_int;
  E.out_count = stats;
  E.out_min_interval = stats + 1;
  E.out_n_intervals = stats + 2;
  if (!out_position) E.offsets = nullptr;
  hipLaunchKernelGGL(queue_emit_kernel, dim3(out_position ? blocks : 1), dim3(256), 0, st, E);
  DEN_LAUNCHED();
  return DEN_OK;
}
}  // namespace

extern "C" {

size_t den_queue_workspace_bytes(int64_t n) { return n <= 0 ? 256 : queue_ws(n).total; }

int den_queue_raw_events(int64_t n, int32_t img_height, int32_t img_width, const int64_t* position,
                         const int64_t* timestamp, const uint8_t* polarity, void* workspace, size_t workspace_bytes,
                         int64_t* out_position, int64_t* out_start_ts, int64_t* out_end_ts, int64_t* out_num_pos,
                         int64_t* out_num_neg, int64_t* out_stats, void* stream) {
  if (!out_position && n > 0) return fail(DEN_EINVAL, "bad arguments: out_position");
  return queue_impl(n, img_height, img_width, position, timestamp, polarity, workspace, workspace_bytes, out_position,
                    out_start_ts, out_end_ts, out_num_pos, out_num_neg, out_stats, (hipStream_t)stream);
}

int den_colorize_events(int64_t n, const int64_t* position, const int32_t* bayer_channel, uint8_t* out_channel_idx,
                        void* stream) {
  if (n < 0 || !bayer_channel || (n > 0 && (!position || !out_channel_idx))) return fail(DEN_EINVAL, "bad arguments");
  Bayer B{};
  for (int q = 0; q < 4; ++q) {
    if (bayer_channel[q] < 0 || bayer_channel[q] > 2) return fail(DEN_EINVAL, "bayer channel indices must be 0..2");
    B.ch[q] = bayer_channel[q];
  }
  if (n == 0) return DEN_OK;
  hipLaunchKernelGGL(colorize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     position, B, out_channel_idx);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_max_refractory_period(int64_t n, int32_t img_height, int32_t img_width, const int64_t* position,
                              const int64_t* timestamp, void* workspace, size_t workspace_bytes, int64_t* out_stats,
                              void* stream) {
  return queue_impl(n, img_height, img_width, position, timestamp, nullptr, workspace, workspace_bytes, nullptr,
                    nullptr, nullptr, nullptr, nullptr, out_stats, (hipStream_t)stream);
}

int den_undistort_events(int64_t n, int32_t model, const int64_t* position, const float* intrinsics,
                         const float* distortion, float* out, void* stream) {
  if (n < 0 || model < 0 || model > 2 || (n > 0 && (!position || !out)) || (model > 0 && (!intrinsics || !distortion)))
    return fail(DEN_EINVAL, "bad arguments");
  if (n == 0) return DEN_OK;
  UndistortArgs A{};
  A.n = n;
  A.model = model;
  for (int q = 0; q < 9; ++q) A.K[q] = intrinsics ? (double)intrinsics[q] : 0.0;
  for (int q = 0; q < 4; ++q) A.D[q] = distortion ? (double)distortion[q] : 0.0;
  A.position = position;
  A.out = out;
  hipLaunchKernelGGL(undistort_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A);
  DEN_LAUNCHED();
  return DEN_OK;
}

size_t den_ssim_workspace_bytes(int32_t n_img) { return n_img > 0 ? (size_t)n_img * SSIM_SLICES * sizeof(double) : 0; }

int den_ssim(int32_t n_img, int32_t channels, int32_t height, int32_t width, const float* pred, const float* target,
             const float* window, float c1, float c2, void* workspace, double* ssim_sum, void* stream) {
  if (n_img <= 0 || channels <= 0 || height < 2 * SSIM_HALF + 1 || width < 2 * SSIM_HALF + 1 || !pred || !target ||
      !window || !workspace || !ssim_sum)
    return fail(DEN_EINVAL, "bad arguments (images must be at least 11 x 11)");
  SsimArgs A{};
  A.C = channels;
  A.H = height;
  A.W = width;
  A.c1 = c1;
  A.c2 = c2;
  for (int q = 0; q < SSIM_WIN * SSIM_WIN; ++q) A.win[q] = window[q];
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ssim_kernel, dim3(SSIM_SLICES, n_img), dim3(SSIM_BLOCK), 0, st, A, pred, target,
                     (double*)workspace);
  DEN_LAUNCHED();
  hipLaunchKernelGGL(sum_partials_f64_kernel, dim3(n_img), dim3(256), 0, st, n_img, SSIM_SLICES,
                     (const double*)workspace, ssim_sum);
  DEN_LAUNCHED();
  return DEN_OK;
}

int den_png_unfilter(int64_t height, int64_t row_bytes, int32_t bpp, const uint8_t* filtered, uint8_t* out) {
  if (height < 0 || row_bytes < 0 || bpp < 1 || bpp > 8 || (height > 0 && row_bytes > 0 && (!filtered || !out)))
    return fail(DEN_EINVAL, "bad arguments");
  if (!png_unfilter_host(height, row_bytes, bpp, filtered, out)) return fail(DEN_EINVAL, "unknown PNG filter type");
  return DEN_OK;
}

}  // extern "C"
