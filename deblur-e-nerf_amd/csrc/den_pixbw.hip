// den_pixbw.hip -- pixel-bandwidth sensor model on gfx950: one thread per event, f64 inside.
//
// Reference (deblur_e_nerf/..., file:line):
//   sample timestamps   models/pixel_bandwidth.py:298-367 (sample_intensity)
//   linearised system   models/pixel_bandwidth.py:181-228
//   FOH discretisation  utils/control.py:29-123 (state preserved, "efficient" form)
//   weights             models/pixel_bandwidth.py:260-296
//   output, reset       models/pixel_bandwidth.py:398-448 (glue :450-494)
//
// The reference materialises (S-1, N, 4, 4) systems in f32, runs batched matrix_exp and
// linalg.solve, and a Python loop of S-2 batched matmuls.  Here one thread owns one event and
// folds its S-1 segments -- descending, as the weight recurrence runs -- straight into the two
// weighted sums, in f64 (inputs and outputs stay f32 as the reference's; the reference's own f32
// result is ~1e-6 away from its f64 one).
//
// Backward: the thread re-runs the forward sweep keeping Phi / Bd / Btd of every segment and the
// running row vectors c_i in the workspace, runs the adjoint of the weight recurrence in ascending
// order, and pulls each segment's adjoint back through the discretisation: closed-form adjoints of
// the substitution solves, and the Frechet derivative of expm, dL/dX = L(X^T, dL/dPhi), computed
// as ONE matrix exponential in dual arithmetic (value X^T, tangent dL/dPhi).  The 7 parameter
// gradients are reduced per block (deterministic) and summed by den_sum_partials.
#include "den_device.h"

namespace den {

constexpr int PIXBW_BLOCK = 64;    // one wave per block
constexpr int PIXBW_NPARAM = 7;
// workspace doubles per segment: Phi (16), Bd (4), Btd (4), then (segment-parallel backward) the four
// Frechet derivatives L(X, E_m) (4 x 16)
constexpr int PIXBW_SEG_F = 24 + 64;  // per segment: Phi, B_d, B~_d, then the four L(X, E_m)
constexpr double PIXBW_NS = 1e-9;  // PixelBandwidth.NS_TO_S

// ------------------------------------------------------------------ dual numbers
struct Dual {
  double v, d;
};
__device__ __forceinline__ Dual operator+(Dual a, Dual b) { return {a.v + b.v, a.d + b.d}; }
__device__ __forceinline__ Dual operator-(Dual a, Dual b) { return {a.v - b.v, a.d - b.d}; }
__device__ __forceinline__ Dual operator*(Dual a, Dual b) { return {a.v * b.v, a.v * b.d + a.d * b.v}; }
__device__ __forceinline__ Dual operator*(double s, Dual b) { return {s * b.v, s * b.d}; }
__device__ __forceinline__ Dual operator+(Dual a, double s) { return {a.v + s, a.d}; }
__device__ __forceinline__ Dual operator/(Dual a, Dual b) {
  const double q = a.v / b.v;
  return {q, (a.d - q * b.d) / b.v};
}
__device__ __forceinline__ double vpart(double x) { return x; }
__device__ __forceinline__ double vpart(const Dual& x) { return x.v; }
template <class T>
__device__ __forceinline__ T pb_one();
template <>
__device__ __forceinline__ double pb_one<double>() { return 1.0; }
template <>
__device__ __forceinline__ Dual pb_one<Dual>() { return {1.0, 0.0}; }

// ------------------------------------------------------------------ 4x4 matrices (row-major)
template <class T>
struct Mat4 {
  T e[16];
};

template <class T>
__device__ __forceinline__ void mat_mul(const Mat4<T>& a, const Mat4<T>& b, Mat4<T>& c) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T s = a.e[4 * i] * b.e[j];
#pragma unroll
      for (int k = 1; k < 4; ++k) s = s + a.e[4 * i + k] * b.e[4 * k + j];
      c.e[4 * i + j] = s;
    }
}

// Q <- P^-1 Q: Gauss-Jordan elimination with partial pivoting on the value part; rows are swapped
// through compile-time-indexed code (no dynamic register indexing).
template <class T>
__device__ __forceinline__ void mat_solve(Mat4<T>& P, Mat4<T>& Q) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      if (fabs(vpart(P.e[4 * r + c])) > fabs(vpart(P.e[5 * c]))) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const T t = P.e[4 * c + j];
          P.e[4 * c + j] = P.e[4 * r + j];
          P.e[4 * r + j] = t;
          const T u = Q.e[4 * c + j];
          Q.e[4 * c + j] = Q.e[4 * r + j];
          Q.e[4 * r + j] = u;
        }
      }
    }
    const T inv = pb_one<T>() / P.e[5 * c];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r == c) continue;
      const T f = P.e[4 * r + c] * inv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        P.e[4 * r + j] = P.e[4 * r + j] - f * P.e[4 * c + j];
        Q.e[4 * r + j] = Q.e[4 * r + j] - f * Q.e[4 * c + j];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const T inv = pb_one<T>() / P.e[5 * r];
#pragma unroll
    for (int j = 0; j < 4; ++j) Q.e[4 * r + j] = Q.e[4 * r + j] * inv;
  }
}

// R = e^A by scaling and squaring with the [13/13] Pade approximant (Higham 2005).  The number of
// squarings comes from the 1-norm of the value part, so a Dual input yields the exact derivative
// of the approximant in the direction of its tangent part.
template <class T>
__device__ void mat_exp(const Mat4<T>& A, Mat4<T>& R) {
  double nrm = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += fabs(vpart(A.e[4 * i + j]));
    nrm = fmax(nrm, s);
  }
  constexpr double THETA13 = 5.371920351148152;
  int sq = 0;
  if (nrm > THETA13) sq = (int)ceil(log2(nrm / THETA13));
  const double sc = ldexp(1.0, -sq);
  const double b[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0, 1187353796428800.0,
                        129060195264000.0,   10559470521600.0,    670442572800.0,    33522128640.0,
                        1323241920.0,        40840800.0,          960960.0,          16380.0,
                        182.0,               1.0};
  Mat4<T> X, X2, X4, X6, U, V, W;
#pragma unroll
  for (int i = 0; i < 16; ++i) X.e[i] = sc * A.e[i];
  mat_mul(X, X, X2);
  mat_mul(X2, X2, X4);
  mat_mul(X4, X2, X6);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    U.e[i] = b[13] * X6.e[i] + b[11] * X4.e[i] + b[9] * X2.e[i];
    V.e[i] = b[12] * X6.e[i] + b[10] * X4.e[i] + b[8] * X2.e[i];
  }
  mat_mul(X6, U, W);
#pragma unroll
  for (int i = 0; i < 16; ++i) U.e[i] = W.e[i] + b[7] * X6.e[i] + b[5] * X4.e[i] + b[3] * X2.e[i];
  mat_mul(X6, V, W);
#pragma unroll
  for (int i = 0; i < 16; ++i) V.e[i] = W.e[i] + b[6] * X6.e[i] + b[4] * X4.e[i] + b[2] * X2.e[i];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    U.e[5 * d] = U.e[5 * d] + b[1];
    V.e[5 * d] = V.e[5 * d] + b[0];
  }
  mat_mul(X, U, W);  // odd part
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    R.e[i] = V.e[i] + W.e[i];
    V.e[i] = V.e[i] - W.e[i];
  }
  mat_solve(V, R);  // (V - U)^-1 (V + U)
  for (int s = 0; s < sq; ++s) {
    mat_mul(R, R, W);
    R = W;
  }
}

// ------------------------------------------------------------------ one segment
struct PixPrm {
  double kin, kmil, ainv, linv, tout, tsf, tdf;
};
__device__ __forceinline__ PixPrm pb_params(const float* p) {
  return {(double)p[0], (double)p[1], (double)p[2], (double)p[3], (double)p[4], (double)p[5], (double)p[6]};
}
// linearized_sys_params (pixel_bandwidth.py:181-194): 2 zeta w_n and w_n^2 at intensity I
__device__ __forceinline__ void pb_lin(const PixPrm& P, double I, double* a, double* b) {
  const double tin = P.kin / I, tmil = P.kmil / I;
  const double pp = (tin + tmil) * P.tout;
  *a = (tin + P.tout + (1.0 / P.ainv + 1.0) * tmil) / pp;
  *b = (1.0 / P.linv + 1.0) / pp;
}
// X = A dt (linearize_sys, :218-226): A = [[-a, -b, 0, 0], [1, 0, 0, 0], [0, ws, -ws, 0], [0, 0, wd, -wd]]
__device__ __forceinline__ void pb_X(double a, double b, double ws, double wd, double dt, Mat4<double>& X) {
#pragma unroll
  for (int i = 0; i < 16; ++i) X.e[i] = 0.0;
  X.e[0] = -dt * a;
  X.e[1] = -dt * b;
  X.e[4] = dt;
  X.e[9] = dt * ws;
  X.e[10] = -dt * ws;
  X.e[14] = dt * wd;
  X.e[15] = -dt * wd;
}
// FOH terms (control.py:87-93, 109-114) from Phi = e^{A dt}:  M = A^-1 B = (0, -1, -1, -1) exactly
// (row 1 of A M = B gives M0 = 0, row 0 M1 = -1, rows 2 and 3 M3 = M2 = M1);  G1 = (Phi - I) M;
// y = (A dt)^-1 G1 by substitution in the same rows;  G2 = y - M;  Bd = G1 - G2, Btd = G2.
__device__ __forceinline__ void pb_foh(const Mat4<double>& phi, double a, double b, double ws, double wd, double dt,
                                       double* g1, double* y) {
#pragma unroll
  for (int i = 0; i < 4; ++i) g1[i] = (i ? 1.0 : 0.0) - (phi.e[4 * i + 1] + phi.e[4 * i + 2] + phi.e[4 * i + 3]);
  y[0] = g1[1] / dt;
  y[1] = -(g1[0] / dt + a * y[0]) / b;
  y[2] = y[1] - g1[2] / (dt * ws);
  y[3] = y[2] - g1[3] / (dt * wd);
}

struct PixArgs {
  int S, N, reset;
  const float* it;       // (S, N) intensity samples
  const double* ts;      // (S, N) sample timestamps, ns
  const double* out_ts;  // (N)
  const float* prm;      // (7)
  const float* delta_in; // (N) non-reset
  const double* reset_ts;// (N) non-reset
  float* out;            // (N)
  float* delta_out;      // (N) reset
  const float* d_out;
  const float* d_delta_out;
  double* ws;
  float* d_it;
  float* d_delta_in;
  float* d_prm;          // (7, gridDim.x)
};

// sample_ts.diff(dim=0).to(f32) (pixel_bandwidth.py:486), in seconds (:385)
__device__ __forceinline__ double pb_dt(const PixArgs& A, int n, int k) {
  const float d = (float)(A.ts[(int64_t)(k + 1) * A.N + n] - A.ts[(int64_t)k * A.N + n]);
  return (double)d * PIXBW_NS;
}
__device__ __forceinline__ double* pb_seg(const PixArgs& A, int n, int k, int f) {
  return A.ws + ((int64_t)k * PIXBW_SEG_F + f) * A.N + n;
}
__device__ __forceinline__ double* pb_row(const PixArgs& A, int n, int i, int f) {  // c_i, f = 4 o + q
  return A.ws + ((int64_t)(A.S - 1) * PIXBW_SEG_F + (int64_t)i * 8 + f) * A.N + n;
}

// Phi = e^{A dt}, Bd, Btd of segment k of event n (linearisation at I[k+1], FOH discretisation)
__device__ __forceinline__ void pb_seg_sys(const PixArgs& A, int n, const PixPrm& P, int k, Mat4<double>& phi,
                                           double* bd, double* btd) {
  const double I1 = (double)A.it[(int64_t)(k + 1) * A.N + n];
  const double dt = pb_dt(A, n, k);
  const double ws = 1.0 / P.tsf, wd = 1.0 / P.tdf;
  double a, b;
  pb_lin(P, I1, &a, &b);
  Mat4<double> X;
  pb_X(a, b, ws, wd, dt, X);
  mat_exp(X, phi);
  double g1[4], yv[4];
  pb_foh(phi, a, b, ws, wd, dt, g1, yv);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    btd[q] = yv[q] + (q ? 1.0 : 0.0);
    bd[q] = g1[q] - btd[q];
  }
}

// Forward sweep of event n (discretized_sys_to_weight, :283-294, fused with the weighted log-sum of
// :406-415): segments k = S-2 .. 0 with c = c_{k+1} = C Phi[S-2] ... Phi[k+1]:
//   w[k+1] += c Btd_k,   w[k] = c Bd_k (completed by the next step),   c <- c Phi_k.
// PRE: Phi / Bd / Btd from the workspace (pixbw_seg_kernel); lds != null: from an LDS image [k][24]
template <bool KEEP, bool PRE = false>
__device__ void pb_sweep(const PixArgs& A, int n, const PixPrm& P, double* y, double* den,
                         const double* lds = nullptr) {
  const int S = A.S, N = A.N, no = A.reset ? 2 : 1;
  const double ws = 1.0 / P.tsf, wd = 1.0 / P.tdf;
  double c[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  if (A.reset) {  // rows (sf, diff) of C (:156-160)
    c[0][2] = 1.0;
    c[1][3] = 1.0;
  } else {        // the diff row only (:208-210)
    c[0][3] = 1.0;
  }
  double num[2] = {0.0, 0.0}, dsum[2] = {0.0, 0.0}, wpend[2] = {0.0, 0.0};
  for (int k = S - 2; k >= 0; --k) {
    const double I1 = (double)A.it[(int64_t)(k + 1) * N + n];
    Mat4<double> phi;
    double bd[4], btd[4];
    if constexpr (PRE) {  // from pixbw_seg_kernel
#pragma unroll
      for (int e = 0; e < 16; ++e) phi.e[e] = *pb_seg(A, n, k, e);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bd[q] = *pb_seg(A, n, k, 16 + q);
        btd[q] = *pb_seg(A, n, k, 20 + q);
      }
    } else if (lds) {
#pragma unroll
      for (int e = 0; e < 16; ++e) phi.e[e] = lds[k * 24 + e];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bd[q] = lds[k * 24 + 16 + q];
        btd[q] = lds[k * 24 + 20 + q];
      }
    } else {
      pb_seg_sys(A, n, P, k, phi, bd, btd);
    }
    if constexpr (KEEP && !PRE) {
#pragma unroll
      for (int e = 0; e < 16; ++e) *pb_seg(A, n, k, e) = phi.e[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        *pb_seg(A, n, k, 16 + q) = bd[q];
        *pb_seg(A, n, k, 20 + q) = btd[q];
      }
    }
    if constexpr (KEEP) {
#pragma unroll
      for (int o = 0; o < 2; ++o)
#pragma unroll
        for (int q = 0; q < 4; ++q) *pb_row(A, n, k + 1, 4 * o + q) = c[o][q];
    }
    const double L1 = log(I1);
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      if (o >= no) break;
      double w = wpend[o], pw = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w += c[o][q] * btd[q];
        pw += c[o][q] * bd[q];
      }
      num[o] += w * L1;
      dsum[o] += w;
      wpend[o] = pw;
      if (k >= 1) {
        double cn[4];
#pragma unroll
        for (int q2 = 0; q2 < 4; ++q2) {
          double s = 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) s += c[o][q] * phi.e[4 * q + q2];
          cn[q2] = s;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) c[o][q] = cn[q];
      }
    }
  }
  const double L0 = log((double)A.it[n]);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    if (o >= no) break;
    num[o] += wpend[o] * L0;
    dsum[o] += wpend[o];
    y[o] = num[o] / dsum[o];
    den[o] = dsum[o];
  }
}

__global__ __launch_bounds__(PIXBW_BLOCK) void pixbw_fwd_kernel(PixArgs A) {
  const int n = blockIdx.x * PIXBW_BLOCK + threadIdx.x;
  if (n >= A.N) return;
  const PixPrm P = pb_params(A.prm);
  double y[2] = {0.0, 0.0}, den[2] = {1.0, 1.0};
  pb_sweep<false>(A, n, P, y, den);
  if (A.reset) {
    // reset the differencing amplifier (:419-434): out = source-follower output, delta = diff - sf
    A.out[n] = (float)y[0];
    A.delta_out[n] = (float)(y[1] - y[0]);
  } else {
    // decay of the reset offset (:435-446); reset_dt is cast to f32 as the reference does
    const double rdt = (double)(float)(A.out_ts[n] - A.reset_ts[n]) * PIXBW_NS;
    A.out[n] = (float)(y[0] - (double)A.delta_in[n] * exp(-rdt / P.tdf));
  }
}

// Forward with one wave per event: lane k computes segment k's Phi / Bd / Btd (the matrix
// exponentials run in parallel) into LDS, lane 0 runs the weight recurrence over them.  A 68-event
// micro-batch was 68 threads each running S - 1 exponentials in sequence.  S - 1 <= PIXBW_WAVE_SEGS.
constexpr int PIXBW_WAVE_SEGS = 63;
__global__ __launch_bounds__(256) void pixbw_fwd_wave_kernel(PixArgs A) {
  __shared__ double seg[4][PIXBW_WAVE_SEGS * 24];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + w;
  const PixPrm P = pb_params(A.prm);
  if (n < A.N && lane < A.S - 1) {
    Mat4<double> phi;
    double bd[4], btd[4];
    pb_seg_sys(A, n, P, lane, phi, bd, btd);
    double* d = seg[w] + lane * 24;
#pragma unroll
    for (int e = 0; e < 16; ++e) d[e] = phi.e[e];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[16 + q] = bd[q];
      d[20 + q] = btd[q];
    }
  }
  __syncthreads();
  if (n >= A.N || lane != 0) return;
  double y[2] = {0.0, 0.0}, den[2] = {1.0, 1.0};
  pb_sweep<false>(A, n, P, y, den, seg[w]);
  if (A.reset) {
    A.out[n] = (float)y[0];
    A.delta_out[n] = (float)(y[1] - y[0]);
  } else {
    const double rdt = (double)(float)(A.out_ts[n] - A.reset_ts[n]) * PIXBW_NS;
    A.out[n] = (float)(y[0] - (double)A.delta_in[n] * exp(-rdt / P.tdf));
  }
}

// Adjoint of segment k's discretisation: (phib, bdb, btdb) = dL/d(Phi, Bd, Btd) -> parameter
// gradients (accumulated in gp) and dL/dI[k+1] through the linearisation (returned).
__device__ double pb_seg_bwd(const PixArgs& A, int n, const PixPrm& P, int k, const double* phib_in,
                             const double* bdb, const double* btdb, double* gp) {
  const double I1 = (double)A.it[(int64_t)(k + 1) * A.N + n];
  const double dt = pb_dt(A, n, k);
  const double ws = 1.0 / P.tsf, wd = 1.0 / P.tdf;
  double a, b;
  pb_lin(P, I1, &a, &b);
  Mat4<double> X, phi;
  pb_X(a, b, ws, wd, dt, X);
#pragma unroll
  for (int e = 0; e < 16; ++e) phi.e[e] = *pb_seg(A, n, k, e);
  double g1[4], y[4];
  pb_foh(phi, a, b, ws, wd, dt, g1, y);
  double phib[16], g1b[4], yb[4];
#pragma unroll
  for (int e = 0; e < 16; ++e) phib[e] = phib_in[e];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    yb[q] = btdb[q] - bdb[q];  // Btd = G2 = y - M, Bd = G1 - G2
    g1b[q] = bdb[q];
  }
  double ab = 0.0, bb = 0.0, wsb = 0.0, wdb = 0.0;
  // y3 = y2 - g1_3 / (dt wd)
  yb[2] += yb[3];
  g1b[3] -= yb[3] / (dt * wd);
  wdb += yb[3] * g1[3] / (dt * wd * wd);
  // y2 = y1 - g1_2 / (dt ws)
  yb[1] += yb[2];
  g1b[2] -= yb[2] / (dt * ws);
  wsb += yb[2] * g1[2] / (dt * ws * ws);
  // y1 = -q / b,  q = g1_0 / dt + a y0
  const double q = g1[0] / dt + a * y[0];
  const double qb = -yb[1] / b;
  bb += yb[1] * q / (b * b);
  g1b[0] += qb / dt;
  ab += qb * y[0];
  yb[0] += qb * a;
  // y0 = g1_1 / dt
  g1b[1] += yb[0] / dt;
  // g1_i = [i >= 1] - (Phi_i1 + Phi_i2 + Phi_i3)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 1; j < 4; ++j) phib[4 * i + j] -= g1b[i];
  // Phi = e^X: the four entries of dL/dX = L(X^T, dL/dPhi) the parameters reach, as
  // <E_m, L(X^T, G)> = <L(X, E_m), G> with the L(X, E_m) of pixbw_seg_kernel
  double fr[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < 16; ++e) s += *pb_seg(A, n, k, 24 + 16 * m + e) * phib[e];
    fr[m] = s;
  }
  ab -= dt * fr[0];
  bb -= dt * fr[1];
  wsb += dt * fr[2];
  wdb += dt * fr[3];
  // linearized_sys_params (:183-191) chain rule
  const double tin = P.kin / I1, tmil = P.kmil / I1, pp = (tin + tmil) * P.tout;
  const double aamp = 1.0 / P.ainv, aloop = 1.0 / P.linv;
  const double numb = ab / pp;
  const double ppb = -(ab * a + bb * b) / pp;
  const double tinb = numb + ppb * P.tout;
  const double tmilb = numb * (aamp + 1.0) + ppb * P.tout;
  gp[0] += tinb / I1;                          // tau_in_it_eff_prod
  gp[1] += tmilb / I1;                         // tau_mil_it_eff_prod
  gp[2] -= numb * tmil * aamp * aamp;          // A_amp_inv  (A_amp = 1 / A_amp_inv)
  gp[3] -= (bb / pp) * aloop * aloop;          // A_loop_inv
  gp[4] += numb + ppb * (tin + tmil);          // tau_out
  gp[5] -= wsb * ws * ws;                      // tau_sf     (w_sf = 1 / tau_sf)
  gp[6] -= wdb * wd * wd;                      // tau_diff
  return -(tinb * tin + tmilb * tmil) / I1;
}

// Segment-parallel part of the backward: one thread per (event, segment, m).  The per-segment work
// -- Phi = e^X and the Frechet derivatives the adjoint needs -- does not depend on the recurrences,
// so it leaves the per-event serial loop (a 68-event micro-batch was 68 threads running 29 segments
// x 2 matrix exponentials each).  Thread m computes e^(X + eps E_m) in dual arithmetic, E_m the
// directions whose entries of dL/dX the parameters reach: E_0 = e_00 (a), E_1 = e_01 (b),
// E_2 = e_21 - e_22 (w_sf), E_3 = e_32 - e_33 (w_diff); m = 0 also stores Phi, Bd, Btd.
__global__ __launch_bounds__(256) void pixbw_seg_kernel(PixArgs A) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)(A.S - 1) * A.N;
  if (t >= 4 * per) return;
  const int m = (int)(t / per);
  const int64_t r = t - m * per;
  const int k = (int)(r / A.N), n = (int)(r - (int64_t)k * A.N);
  const PixPrm P = pb_params(A.prm);
  const double I1 = (double)A.it[(int64_t)(k + 1) * A.N + n];
  const double dt = pb_dt(A, n, k);
  const double ws = 1.0 / P.tsf, wd = 1.0 / P.tdf;
  double a, b;
  pb_lin(P, I1, &a, &b);
  Mat4<double> X;
  pb_X(a, b, ws, wd, dt, X);
  Mat4<Dual> XE, R;
#pragma unroll
  for (int e = 0; e < 16; ++e) XE.e[e] = Dual{X.e[e], 0.0};
  if (m == 0) XE.e[0].d = 1.0;
  else if (m == 1) XE.e[1].d = 1.0;
  else if (m == 2) { XE.e[9].d = 1.0; XE.e[10].d = -1.0; }
  else { XE.e[14].d = 1.0; XE.e[15].d = -1.0; }
  mat_exp(XE, R);
#pragma unroll
  for (int e = 0; e < 16; ++e) *pb_seg(A, n, k, 24 + 16 * m + e) = R.e[e].d;
  if (m == 0) {
    Mat4<double> phi;
    double bd[4], btd[4];
    pb_seg_sys(A, n, P, k, phi, bd, btd);
#pragma unroll
    for (int e = 0; e < 16; ++e) *pb_seg(A, n, k, e) = phi.e[e];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *pb_seg(A, n, k, 16 + q) = bd[q];
      *pb_seg(A, n, k, 20 + q) = btd[q];
    }
  }
}

__global__ __launch_bounds__(PIXBW_BLOCK) void pixbw_bwd_kernel(PixArgs A) {
  const int n = blockIdx.x * PIXBW_BLOCK + threadIdx.x;
  double gp[PIXBW_NPARAM] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (n < A.N) {
    const int S = A.S, N = A.N, no = A.reset ? 2 : 1;
    const PixPrm P = pb_params(A.prm);
    double y[2] = {0.0, 0.0}, den[2] = {1.0, 1.0};
    pb_sweep<true, true>(A, n, P, y, den);
    // adjoints of the weighted outputs
    double yb[2] = {0.0, 0.0};
    const double g = (double)A.d_out[n];
    if (A.reset) {
      const double gd = A.d_delta_out ? (double)A.d_delta_out[n] : 0.0;
      yb[0] = g - gd;
      yb[1] = gd;
    } else {
      const double rdt = (double)(float)(A.out_ts[n] - A.reset_ts[n]) * PIXBW_NS;
      const double e = exp(-rdt / P.tdf);
      yb[0] = g;
      A.d_delta_in[n] = (float)(-g * e);
      gp[6] -= g * (double)A.delta_in[n] * e * rdt / (P.tdf * P.tdf);
    }
    // ascending adjoint sweep of the weight recurrence; segment k's adjoint is complete at step k + 1
    double cbc[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};  // dL/dc_i
    double cbn[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};  // dL/dc_{i+1} (partial)
    double pphi[16], pbd[4];
#pragma unroll
    for (int e = 0; e < 16; ++e) pphi[e] = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) pbd[q] = 0.0;
    for (int i = 0; i < S; ++i) {
      const double Ii = (double)A.it[(int64_t)i * N + n];
      const bool has_bd = i <= S - 2, has_btd = i >= 1;
      double cn[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
      double ci[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
      double bd[4] = {0.0, 0.0, 0.0, 0.0}, btd[4] = {0.0, 0.0, 0.0, 0.0};
      if (has_bd) {
#pragma unroll
        for (int q = 0; q < 4; ++q) bd[q] = *pb_seg(A, n, i, 16 + q);
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
          for (int q = 0; q < 4; ++q) cn[o][q] = *pb_row(A, n, i + 1, 4 * o + q);
      }
      if (has_btd) {
#pragma unroll
        for (int q = 0; q < 4; ++q) btd[q] = *pb_seg(A, n, i - 1, 20 + q);
#pragma unroll
        for (int o = 0; o < 2; ++o)
#pragma unroll
          for (int q = 0; q < 4; ++q) ci[o][q] = *pb_row(A, n, i, 4 * o + q);
      }
      // w[i] = c_{i+1} Bd_i + c_i Btd_{i-1};  y_o = sum w L / sum w
      const double Li = log(Ii);
      double wb[2] = {0.0, 0.0}, ib = 0.0;
#pragma unroll
      for (int o = 0; o < 2; ++o) {
        if (o >= no) break;
        double w = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) w += cn[o][q] * bd[q] + ci[o][q] * btd[q];
        wb[o] = yb[o] * (Li - y[o]) / den[o];
        ib += yb[o] * w / den[o];
      }
      ib /= Ii;
      double bdb[4] = {0.0, 0.0, 0.0, 0.0};
      if (has_bd) {
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          if (o >= no) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            cbn[o][q] += wb[o] * bd[q];
            bdb[q] += wb[o] * cn[o][q];
          }
        }
      }
      if (has_btd) {
        double btdb[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          if (o >= no) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            cbc[o][q] += wb[o] * btd[q];
            btdb[q] += wb[o] * ci[o][q];
          }
        }
        ib += pb_seg_bwd(A, n, P, i - 1, pphi, pbd, btdb, gp);
      }
      double phib[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) phib[e] = 0.0;
      if (has_bd && has_btd) {  // c_i = c_{i+1} Phi_i for 1 <= i <= S-2
        double ph[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) ph[e] = *pb_seg(A, n, i, e);
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          if (o >= no) break;
#pragma unroll
          for (int a4 = 0; a4 < 4; ++a4) {
            double s = 0.0;
#pragma unroll
            for (int b4 = 0; b4 < 4; ++b4) {
              phib[4 * a4 + b4] += cn[o][a4] * cbc[o][b4];
              s += cbc[o][b4] * ph[4 * a4 + b4];
            }
            cbn[o][a4] += s;
          }
        }
      }
      A.d_it[(int64_t)i * N + n] = (float)ib;
#pragma unroll
      for (int e = 0; e < 16; ++e) pphi[e] = phib[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) pbd[q] = bdb[q];
#pragma unroll
      for (int o = 0; o < 2; ++o)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          cbc[o][q] = cbn[o][q];
          cbn[o][q] = 0.0;
        }
    }
  }
  // deterministic per-block parameter partials (one wave per block)
#pragma unroll
  for (int j = 0; j < PIXBW_NPARAM; ++j) {
    double v = gp[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (threadIdx.x == 0) A.d_prm[(int64_t)j * gridDim.x + blockIdx.x] = (float)v;
  }
}

// ------------------------------------------------------------------ sample timestamps
// torch.linspace(1, 0, steps) in f64 (ATen's symmetric formula) and at::lerp (fused form)
__device__ __forceinline__ double pb_linspace(int i, int steps) {
#pragma clang fp contract(off)
  const double step = (0.0 - 1.0) / (double)(steps - 1);
  return i < steps / 2 ? 1.0 + step * (double)i : 0.0 - step * (double)(steps - i - 1);
}
__device__ __forceinline__ double pb_lerp(double a, double b, double w) {
  return fabs(w) < 0.5 ? fma(w, b - a, a) : fma(w - 1.0, b - a, b);
}

// sample_intensity (:311-360): boundaries b = linspace(1, 0, S); v_j = lerp(b_j, b_{j+1}, gen_j);
// normalised lifetimes n = [1, lerp(v_{k-1}, v_k, 0.5) ..., 0]; lifetime = -log1p(-p n) / rate with
// the f32 rate 1e-9 omega and the f32 cumulative probability p; ts = out_ts - lifetime (un-clamped).
__global__ void pixbw_sample_ts_kernel(int S, int N, const double* gen, const double* out_ts, float rate, float cum,
                                       double* ts) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)S * N) return;
  const int k = (int)(e / N), n = (int)(e - (int64_t)k * N);
  double nl;
  if (k == 0) {
    nl = 1.0;
  } else if (k == S - 1) {
    nl = 0.0;
  } else {
    const double v0 = pb_lerp(pb_linspace(k - 1, S), pb_linspace(k, S), gen[(int64_t)(k - 1) * N + n]);
    const double v1 = pb_lerp(pb_linspace(k, S), pb_linspace(k + 1, S), gen[(int64_t)k * N + n]);
    nl = pb_lerp(v0, v1, 0.5);
  }
  const double p = (double)cum * nl;
  ts[e] = out_ts[n] - (-log1p(-p) / (double)rate);
}

// Reverse mode of the sample timestamps with respect to output_ts: ts_k = out_ts - lifetime_k with the
// lifetimes out of autograd (sample_intensity runs under no_grad; only output_ts - lifetime is
// recorded, pixel_bandwidth.py:359-363), so d out_ts = sum_k d ts_k.  Overwrites d_out_ts (N).
__global__ void pixbw_sample_ts_bwd_kernel(int S, int N, const double* g_ts, double* d_out_ts) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double acc = 0.0;
  for (int k = 0; k < S; ++k) acc += g_ts[(int64_t)k * N + n];
  d_out_ts[n] = acc;
}

// Reverse mode of the offset decay of a non-reset call (:435-446) with respect to its timestamps:
// out = y - delta exp(-w_diff 1e-9 f32(out_ts - reset_ts)), so d out / d out_ts = delta e w_diff 1e-9 =
// -d out / d reset_ts.  d_out_ts / d_reset_ts (N) overwritten; either may be null.
__global__ void pixbw_decay_ts_bwd_kernel(int N, const double* out_ts, const double* reset_ts, const float* prm,
                                          const float* delta_in, const float* d_out, double* d_out_ts,
                                          double* d_reset_ts) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const double tdf = (double)prm[6];
  const double rdt = (double)(float)(out_ts[n] - reset_ts[n]) * PIXBW_NS;
  const double e = exp(-rdt / tdf);
  const double g = (double)d_out[n] * (double)delta_in[n] * e * PIXBW_NS / tdf;
  if (d_out_ts) d_out_ts[n] = g;
  if (d_reset_ts) d_reset_ts[n] = -g;
}

}  // namespace den
