// SHEncoder (external/sh_encoder.py:15-193): the real spherical-harmonics direction encoding of
// degree 1..8 as a standalone op (the ngp field fuses degree 4, den_ngp.hip ngp_sh4).
//
// Instead of the 64 written-out polynomials, one recurrence.  Band l, order m:
//   Y_l^0 = K_l^0 Q_l^0(z),   Y_l^{+m} = c_l^m Q_l^m(z) C_m(x,y),   Y_l^{-m} = c_l^m Q_l^m(z) S_m(x,y)
// with C_m + i S_m = (x + i y)^m, c_l^m = sqrt(2) (-1)^m K_l^m, K_l^m = sqrt((2l+1)/(4 pi) (l-m)!/(l+m)!),
// and Q_l^m = P_l^m / (1 - z^2)^{m/2} the associated Legendre polynomial without its sin^m factor:
//   Q_m^m = (2m-1)!!,  Q_{m+1}^m = (2m+1) z Q_m^m,  (l-m) Q_l^m = (2l-1) z Q_{l-1}^m - (l+m-1) Q_{l-2}^m.
// These are exactly the polynomials in (x, y, z) the reference writes out (tcnn's
// spherical_harmonics.h basis, Condon-Shortley phase), so non-unit input evaluates as it does there;
// output column l^2 + l + m.  The backward runs the same recurrence on dual numbers (value and the
// three partials), which is the reference's autograd gradient of the same polynomials.
//
// HBM-bound elementwise op: 12 B in, 4 deg^2 B out per direction.  Each 256-thread block stages
// its (256, deg^2) output slab in LDS (row pitch deg^2 + 1 against bank conflicts) and streams it
// out coalesced; the backward stages d_out the same way.
#pragma once

namespace den {

constexpr int SH_THREADS = 256;
constexpr int SH_MAX_DEG = 8;

struct ShCoef {
  float c[SH_MAX_DEG * (SH_MAX_DEG + 1) / 2];  // c_l^m at l (l+1) / 2 + m
};

struct ShDual {
  float v, dx, dy, dz;
};
__device__ __forceinline__ ShDual operator+(ShDual a, ShDual b) { return {a.v + b.v, a.dx + b.dx, a.dy + b.dy, a.dz + b.dz}; }
__device__ __forceinline__ ShDual operator-(ShDual a, ShDual b) { return {a.v - b.v, a.dx - b.dx, a.dy - b.dy, a.dz - b.dz}; }
__device__ __forceinline__ ShDual operator*(ShDual a, ShDual b) {
  return {a.v * b.v, a.dx * b.v + a.v * b.dx, a.dy * b.v + a.v * b.dy, a.dz * b.v + a.v * b.dz};
}
__device__ __forceinline__ ShDual operator*(float s, ShDual a) { return {s * a.v, s * a.dx, s * a.dy, s * a.dz}; }
__device__ __forceinline__ ShDual sh_const(float v, ShDual) { return {v, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ float sh_const(float v, float) { return v; }

// emit(k, Y_k) for every column k < DEG^2
template <int DEG, typename T, typename Emit>
__device__ __forceinline__ void sh_eval(T x, T y, T z, const ShCoef& cf, Emit emit) {
  T cm = sh_const(1.f, x), sm = sh_const(0.f, x);  // (x + i y)^m
  float qmm = 1.f;                                // (2m-1)!!
#pragma unroll
  for (int m = 0; m < DEG; ++m) {
    T q2 = sh_const(0.f, x), q1 = sh_const(0.f, x);
#pragma unroll
    for (int l = m; l < DEG; ++l) {
      T q;
      if (l == m)
        q = sh_const(qmm, x);
      else if (l == m + 1)
        q = float(2 * m + 1) * qmm * z;
      else
        q = (1.f / float(l - m)) * (float(2 * l - 1) * (z * q1) - float(l + m - 1) * q2);
      const float c = cf.c[l * (l + 1) / 2 + m];
      if (m == 0) {
        emit(l * l + l, c * q);
      } else {
        const T cq = c * q;
        emit(l * l + l + m, cq * cm);
        emit(l * l + l - m, cq * sm);
      }
      q2 = q1;
      q1 = q;
    }
    const T cn = x * cm - y * sm, sn = x * sm + y * cm;
    cm = cn;
    sm = sn;
    qmm *= float(2 * m + 1);
  }
}

template <int DEG>
__global__ __launch_bounds__(SH_THREADS) void sh_fwd_kernel(int64_t n, const float* __restrict__ coords,
                                                          float* __restrict__ out, ShCoef cf) {
  constexpr int K = DEG * DEG, P = K + 1;
  static_assert(SH_THREADS * P * 4 <= 160 * 1024, "the staging tile exceeds gfx950's 160 KiB of LDS per workgroup "
                                                 "(degree 8 needs 65 KiB: gfx950 only, over gfx90a / gfx942's 64 KiB)");
  __shared__ float tile[SH_THREADS * P];
  const int64_t base = int64_t(blockIdx.x) * SH_THREADS;
  const int t = threadIdx.x;
  const int64_t i = base + t;
  if (i < n) {
    const float x = coords[3 * i], y = coords[3 * i + 1], z = coords[3 * i + 2];
    float* row = tile + t * P;
    sh_eval<DEG>(x, y, z, cf, [&](int k, float v) { row[k] = v; });
  }
  __syncthreads();
  const int64_t cnt = (n - base < SH_THREADS ? n - base : SH_THREADS) * K;
  float* dst = out + base * K;
  for (int64_t g = t; g < cnt; g += SH_THREADS) dst[g] = tile[g + g / K];
}

template <int DEG>
__global__ __launch_bounds__(SH_THREADS) void sh_bwd_kernel(int64_t n, const float* __restrict__ coords,
                                                          const float* __restrict__ d_out,
                                                          float* __restrict__ d_coords, ShCoef cf) {
  constexpr int K = DEG * DEG, P = K + 1;
  static_assert(SH_THREADS * P * 4 <= 160 * 1024, "the staging tile exceeds gfx950's 160 KiB of LDS per workgroup "
                                                 "(degree 8 needs 65 KiB: gfx950 only, over gfx90a / gfx942's 64 KiB)");
  __shared__ float tile[SH_THREADS * P];
  const int64_t base = int64_t(blockIdx.x) * SH_THREADS;
  const int t = threadIdx.x;
  const int64_t cnt = (n - base < SH_THREADS ? n - base : SH_THREADS) * K;
  const float* src = d_out + base * K;
  for (int64_t g = t; g < cnt; g += SH_THREADS) tile[g + g / K] = src[g];
  __syncthreads();
  const int64_t i = base + t;
  if (i >= n) return;
  const ShDual x{coords[3 * i], 1.f, 0.f, 0.f}, y{coords[3 * i + 1], 0.f, 1.f, 0.f}, z{coords[3 * i + 2], 0.f, 0.f, 1.f};
  const float* row = tile + t * P;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  sh_eval<DEG>(x, y, z, cf, [&](int k, ShDual v) {
    const float g = row[k];
    gx += g * v.dx;
    gy += g * v.dy;
    gz += g * v.dz;
  });
  d_coords[3 * i] = gx;
  d_coords[3 * i + 1] = gy;
  d_coords[3 * i + 2] = gz;
}

// c_l^m on the host, in double, rounded once
inline ShCoef sh_coefs() {
  ShCoef cf{};
  const double pi = 3.14159265358979323846;
  for (int l = 0; l < SH_MAX_DEG; ++l)
    for (int m = 0; m <= l; ++m) {
      double ratio = 1.0;  // (l-m)! / (l+m)!
      for (int j = l - m + 1; j <= l + m; ++j) ratio /= double(j);
      double k = std::sqrt((2 * l + 1) / (4.0 * pi) * ratio);
      if (m > 0) k *= std::sqrt(2.0) * ((m & 1) ? -1.0 : 1.0);
      cf.c[l * (l + 1) / 2 + m] = float(k);
    }
  return cf;
}

template <int DEG>
inline void sh_launch(bool bwd, int64_t n, const float* coords, const float* d_out, float* out, hipStream_t st) {
  const ShCoef cf = sh_coefs();
  const dim3 grid((unsigned)((n + SH_THREADS - 1) / SH_THREADS));
  if (bwd)
    hipLaunchKernelGGL(sh_bwd_kernel<DEG>, grid, dim3(SH_THREADS), 0, st, n, coords, d_out, out, cf);
  else
    hipLaunchKernelGGL(sh_fwd_kernel<DEG>, grid, dim3(SH_THREADS), 0, st, n, coords, out, cf);
}

inline void sh_dispatch(int degree, bool bwd, int64_t n, const float* coords, const float* d_out, float* out,
                        hipStream_t st) {
  switch (degree) {
    case 1: sh_launch<1>(bwd, n, coords, d_out, out, st); break;
    case 2: sh_launch<2>(bwd, n, coords, d_out, out, st); break;
    case 3: sh_launch<3>(bwd, n, coords, d_out, out, st); break;
    case 4: sh_launch<4>(bwd, n, coords, d_out, out, st); break;
    case 5: sh_launch<5>(bwd, n, coords, d_out, out, st); break;
    case 6: sh_launch<6>(bwd, n, coords, d_out, out, st); break;
    case 7: sh_launch<7>(bwd, n, coords, d_out, out, st); break;
    default: sh_launch<8>(bwd, n, coords, d_out, out, st); break;
  }
}

}  // namespace den
