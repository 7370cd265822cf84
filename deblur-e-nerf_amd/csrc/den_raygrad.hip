// den_raygrad.hip -- gradients of a render with respect to its RAYS (origins and directions).
//
// In the reference every sample position is o + d (t0 + t1) / 2 and the view condition is d itself
// (external/utils.py:83-96), with the marching intervals t0 / t1 out of autograd (nerfacc returns
// them detached).  Autograd therefore carries dL/d(position) and dL/d(view direction) back into the
// rays, and from there through NeRF.pixel_params_to_ray and LinearTrajectory into the render
// timestamps -- the path by which the refractory period tau_r (which shifts the start timestamps,
// event_generation_params.py:230-237) gets its gradient (deblur_e_nerf.py:419-455).
//
// Per sample (after the field's backward has left its per-layer gradients in the workspace):
//   mlp field (den_render workspace, either mode):
//     dL/d pe  = W0^T dz0 + W5[:, 256:319]^T dz5      (pe = positional encoding of the contraction)
//     dL/d ve  = Wg[:, 256:283]^T dzg                  (ve = view encoding of pi d)
//     then the sinusoidal-encoding derivative (d sin(v 2^k) / dv = 2^k cos(v 2^k), the cos half as
//     sin(v 2^k + pi/2)), the 2 pi (x - 1/2) map, the contraction Jacobian (AABB / tanh / sphere).
//   ngp field (den_ngp workspace, MFMA backward):
//     dL/d x   = sum_levels scale_l sum_corners (d w_c / d frac) (g0 T[c].0 + g1 T[c].1)  (tcnn's
//                input gradient of the Linear grid encoding), then the contraction Jacobian;
//     dL/d sh  = Wh0[:, 0:16]^T dz_h0, through the degree-4 SH polynomials of d.
//   -> per sample (d position, d view dir); a ray's d origin = sum d position, d direction =
//      sum (d position (t0 + t1)/2 + d view dir), reduced per ray by one wave in a fixed order
//      (deterministic; the reference's index backward of origins[ray_indices] uses atomics).
#include "den_device.h"

namespace den {

// d(contract_unit(pos)) / d pos (den_device.h contract_unit; ngp.py:68-106, mlp.py:321-335):
// J[a][b] = d xhat_a / d pos_b
__device__ __forceinline__ void contract_unit_jac(const float* pos, const float* aabb, int type, float (&J)[3][3]) {
  float inv[3], u[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    inv[a] = 1.0f / (aabb[3 + a] - aabb[a]);
    u[a] = (pos[a] - aabb[a]) * inv[a];
#pragma unroll
    for (int b = 0; b < 3; ++b) J[a][b] = 0.0f;
  }
  if (type == CONTRACT_TANH) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float t = tanhf(u[a] - 0.5f);
      J[a][a] = 0.5f * (1.0f - t * t) * inv[a];
    }
  } else if (type == CONTRACT_SPHERE) {
    float y[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) y[a] = u[a] * 2.0f - 1.0f;
    const float m = sqrtf(y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
    if (m > 1.0f) {
      // z = (2 - 1/m) y / m = f(m) y, f = 2/m - 1/m^2; dz/dy = f I + f'(m) y y^T / m
      const float f = 2.0f / m - 1.0f / (m * m);
      const float fp = -2.0f / (m * m) + 2.0f / (m * m * m);
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const float dz = (a == b ? f : 0.0f) + fp * y[a] * y[b] / m;
          J[a][b] = dz * 0.25f * 2.0f * inv[b];
        }
    } else {
#pragma unroll
      for (int a = 0; a < 3; ++a) J[a][a] = 0.5f * inv[a];
    }
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) J[a][a] = inv[a];
  }
}

// d(enc_feature(v, ., n_deg)) / dv contracted with the feature gradients g[0 .. 3 + 6 n_deg)
template <int NDEG>
__device__ __forceinline__ void enc_backward(const float* v, const float* g, float* dv) {
#pragma clang fp contract(off)
  constexpr int ND = 3 * NDEG;
#pragma unroll
  for (int a = 0; a < 3; ++a) dv[a] = g[a];
#pragma unroll
  for (int q = 0; q < ND; ++q) {
    const int a = q % 3;
    const float sc = (float)(1 << (q / 3));
    const float xb = v[a] * sc;
    dv[a] += g[3 + q] * sc * cosf(xb);
    dv[a] += g[3 + ND + q] * sc * cosf(xb + 1.5707964f);
  }
}

// 4 consecutive features f .. f+3 (f % 4 == 0) of sample s from an activation / dz tensor of
// `width` features in the wave-block-major layout (den_geom.h, den_render.hip act_ptr)
template <int MODE>
__device__ __forceinline__ void act_load4(const char* act, int64_t block_bytes, int64_t s, int f, float* out) {
  constexpr int TM = tm_of(MODE), ES = es_of(MODE);
  const char* tile = act + (s / TM) * block_bytes + (f / TM) * (int64_t)(TM * TM * ES);
  const int c = (int)(s % TM), row = f % TM;
  if constexpr (MODE == 0) {
    // lane c + 16 (row / 4), registers row % 4
    const f32x4 v = *(const f32x4*)(tile + (c + 16 * (row >> 2)) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = v[q];
  } else {
    // row = (r & 3) + 8 (r >> 2) + 4 grp: rows 4k .. 4k+3 are registers 4 (row >> 3) + 0..3 of lane
    // group (row >> 2) & 1, i.e. bf16 words q, q + 1 with q = 2 (row >> 3) (fragment q >> 2)
    const int grp = (row >> 2) & 1, r0 = 4 * (row >> 3);
    const int lane = c + 32 * grp;
    const char* p = tile + lane * 16 + (r0 >> 3) * 1024 + (r0 & 7) * 2;
    const uint2 w = *(const uint2*)p;
    out[0] = __uint_as_float(w.x << 16);
    out[1] = __uint_as_float(w.x & 0xffff0000u);
    out[2] = __uint_as_float(w.y << 16);
    out[3] = __uint_as_float(w.y & 0xffff0000u);
  }
}

struct RayGradArgs {
  int points;        // 0 fixed-count sampler, 1 points, 2 packed samples
  int contraction;
  int rd;
  int n_samples;     // points 0: per ray
  int64_t n;         // samples
  float aabb[6];
  float near_p, far_p;
  const float* rays_o;
  const float* rays_d;
  const float* jitter;
  const int* ray_idx;
  const float* t0;
  const float* t1;
  float* per_sample;  // (n, 6): d position, d position * (t0 + t1)/2 + d view dir (points 1: d position, d view)
};

// the sample's position, view direction and (t0 + t1) (0 for points 1), as the forward forms them
__device__ __forceinline__ void rg_point(const RayGradArgs& G, int64_t s, float* pos, float* dir, float* tt) {
#pragma clang fp contract(off)
  if (G.points == 1) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      pos[a] = G.rays_o[s * 3 + a];
      dir[a] = G.rays_d[s * 3 + a];
    }
    *tt = 0.0f;
    return;
  }
  float o[3], t0, t1;
  if (G.points == 2) {
    const int64_t r = G.ray_idx[s];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = G.rays_o[r * 3 + a];
      dir[a] = G.rays_d[r * 3 + a];
    }
    t0 = G.t0[s];
    t1 = G.t1[s];
  } else {
    const int64_t r = s / G.n_samples;
    const int k = (int)(s - r * G.n_samples);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[a] = G.rays_o[r * 3 + a];
      dir[a] = G.rays_d[r * 3 + a];
    }
    const RayGeom g = ray_geom(o, dir, G.aabb, G.near_p, G.far_p);
    sample_interval(g, k, G.jitter[r], G.n_samples, &t0, &t1);
  }
  *tt = t0 + t1;
#pragma unroll
  for (int a = 0; a < 3; ++a) pos[a] = o[a] + __fdiv_rn(dir[a] * *tt, 2.0f);
}

__device__ __forceinline__ void rg_store(const RayGradArgs& G, int64_t s, const float* dpos, const float* ddir,
                                         float tt) {
  float* o = G.per_sample + s * 6;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o[a] = dpos[a];
    o[3 + a] = G.points == 1 ? ddir[a] : fmaf(dpos[a], 0.5f * tt, ddir[a]);
  }
}

// ------------------------------------------------------------------ mlp field
struct RayGradMlp {
  const float* params;  // flat reference-order parameters (den_param_offset)
  const char* dz0;      // workspace tensors of the render (mode layout): dz of L0, L5 (256 wide), Lg (128)
  const char* dz5;
  const char* dzg;
  int64_t bs0, bs5, bsg;  // bytes per wave block of each (den_geom.h SROW_BYTES rows in the BF16 layout)
  float scale;          // the mode's input-column scale (den_geom.h col_scale: 1 in F32, KAPPA in BF16)
};

constexpr int RG_THREADS = 256, RG_OB = 32;

template <int MODE>
__global__ __launch_bounds__(RG_THREADS) void raygrad_mlp_kernel(RayGradArgs G, RayGradMlp M) {
  // weight blocks of RG_OB output rows: W0 (., 63) and the pe columns of W5 (., 256:319), then Wg's
  // view columns (., 256:283); LDS reads are wave-uniform (broadcast)
  __shared__ float w0[RG_OB][PE_PAD], w5[RG_OB][PE_PAD];
  const int64_t s = (int64_t)blockIdx.x * RG_THREADS + threadIdx.x;
  const bool ok = s < G.n;
  const int64_t sc = ok ? s : G.n - 1;
  const int rd = G.rd;
  const float* W0 = M.params + param_offset(rd, 0);
  const float* W5 = M.params + param_offset(rd, 10);
  const float* Wg = M.params + param_offset(rd, 20);
  float gpe[PE_DIM], gve[VE_DIM];
#pragma unroll
  for (int k = 0; k < PE_DIM; ++k) gpe[k] = 0.0f;
#pragma unroll
  for (int k = 0; k < VE_DIM; ++k) gve[k] = 0.0f;
  for (int o0 = 0; o0 < WIDTH; o0 += RG_OB) {
    __syncthreads();
    for (int q = threadIdx.x; q < RG_OB * PE_PAD; q += RG_THREADS) {
      const int oo = q / PE_PAD, k = q % PE_PAD;
      w0[oo][k] = k < PE_DIM ? W0[(o0 + oo) * PE_DIM + k] : 0.0f;
      w5[oo][k] = k < PE_DIM ? W5[(o0 + oo) * (WIDTH + PE_DIM) + WIDTH + k] : 0.0f;
    }
    __syncthreads();
#pragma unroll 1
    for (int oo = 0; oo < RG_OB; oo += 4) {
      float a[4], b[4];
      act_load4<MODE>(M.dz0, M.bs0, sc, o0 + oo, a);
      act_load4<MODE>(M.dz5, M.bs5, sc, o0 + oo, b);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < PE_DIM; ++k) gpe[k] = fmaf(w0[oo + j][k], a[j], fmaf(w5[oo + j][k], b[j], gpe[k]));
    }
  }
  for (int o0 = 0; o0 < WIDTH_COND; o0 += RG_OB) {
    __syncthreads();
    for (int q = threadIdx.x; q < RG_OB * PE_PAD; q += RG_THREADS) {
      const int oo = q / PE_PAD, k = q % PE_PAD;
      w0[oo][k] = k < VE_DIM ? Wg[(o0 + oo) * (WIDTH + VE_DIM) + WIDTH + k] : 0.0f;
    }
    __syncthreads();
#pragma unroll 1
    for (int oo = 0; oo < RG_OB; oo += 4) {
      float a[4];
      act_load4<MODE>(M.dzg, M.bsg, sc, o0 + oo, a);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < VE_DIM; ++k) gve[k] = fmaf(w0[oo + j][k], a[j], gve[k]);
    }
  }
  if (!ok) return;
#pragma unroll
  for (int k = 0; k < PE_DIM; ++k) gpe[k] *= M.scale;
#pragma unroll
  for (int k = 0; k < VE_DIM; ++k) gve[k] *= M.scale;
  float pos[3], dir[3], tt;
  rg_point(G, s, pos, dir, &tt);
  // positional encoding of xc = 2 pi (xhat - 1/2)
  float xc[3], sel;
  contract_point(pos, G.aabb, xc, &sel, G.contraction);
  float dxc[3];
  enc_backward<10>(xc, gpe, dxc);
  float J[3][3];
  contract_unit_jac(pos, G.aabb, G.contraction, J);
  float dpos[3];
#pragma unroll
  for (int b = 0; b < 3; ++b)
    dpos[b] = 6.2831855f * ((dxc[0] * J[0][b] + dxc[1] * J[1][b]) + dxc[2] * J[2][b]);
  // view encoding of pi d
  float dv[3], ddv[3], ddir[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) dv[a] = dir[a] * 3.1415927f;
  enc_backward<4>(dv, gve, ddv);
#pragma unroll
  for (int a = 0; a < 3; ++a) ddir[a] = ddv[a] * 3.1415927f;
  rg_store(G, s, dpos, ddir, tt);
}

// ------------------------------------------------------------------ ngp field
struct RayGradNgp {
  const float* table;
  const float* mlp;
  NgpOff off;
  NgpGrid grid;
  int64_t ld;
  const float* save;  // [NS_ROWS][ld]
  const float* dz;    // [ND_ROWS][ld]
};

// d SH4(v) / dv contracted with g (16): SHEncoder's polynomials (external/sh_encoder.py:55-77)
__device__ __forceinline__ void sh4_backward(const float* v, const float* g, float* dv) {
  const float x = v[0], y = v[1], z = v[2];
  const float x2 = x * x, y2 = y * y, z2 = z * z;
  const float c1 = 0.48860251190291987f, c4 = 1.0925484305920792f, c6 = 0.94617469575755997f,
              c8 = 0.54627421529603959f, c9 = 0.59004358992664352f, c10 = 2.8906114426405538f,
              c11 = 0.45704579946446572f, c12 = 0.3731763325901154f, c14 = 1.4453057213202769f;
  float gx = 0.0f, gy = 0.0f, gz = 0.0f;
  gy += -c1 * g[1];
  gz += c1 * g[2];
  gx += -c1 * g[3];
  gx += c4 * y * g[4];
  gy += c4 * x * g[4];
  gy += -c4 * z * g[5];
  gz += -c4 * y * g[5];
  gz += 2.0f * c6 * z * g[6];
  gx += -c4 * z * g[7];
  gz += -c4 * x * g[7];
  gx += 2.0f * c8 * x * g[8];
  gy += -2.0f * c8 * y * g[8];
  // 9: c9 y (-3 x^2 + y^2)
  gx += c9 * y * (-6.0f * x) * g[9];
  gy += c9 * (-3.0f * x2 + 3.0f * y2) * g[9];
  // 10: c10 x y z
  gx += c10 * y * z * g[10];
  gy += c10 * x * z * g[10];
  gz += c10 * x * y * g[10];
  // 11: c11 y (1 - 5 z^2)
  gy += c11 * (1.0f - 5.0f * z2) * g[11];
  gz += c11 * y * (-10.0f * z) * g[11];
  // 12: c12 z (5 z^2 - 3)
  gz += c12 * (15.0f * z2 - 3.0f) * g[12];
  // 13: c11 x (1 - 5 z^2)
  gx += c11 * (1.0f - 5.0f * z2) * g[13];
  gz += c11 * x * (-10.0f * z) * g[13];
  // 14: c14 z (x^2 - y^2)
  gx += c14 * z * 2.0f * x * g[14];
  gy += c14 * z * (-2.0f * y) * g[14];
  gz += c14 * (x2 - y2) * g[14];
  // 15: c9 x (-x^2 + 3 y^2)
  gx += c9 * (-3.0f * x2 + 3.0f * y2) * g[15];
  gy += c9 * x * 6.0f * y * g[15];
  dv[0] = gx;
  dv[1] = gy;
  dv[2] = gz;
}

__global__ __launch_bounds__(RG_THREADS) void raygrad_ngp_kernel(RayGradArgs G, RayGradNgp Q) {
  const int64_t s = (int64_t)blockIdx.x * RG_THREADS + threadIdx.x;
  if (s >= G.n) return;
  const int64_t ld = Q.ld;
  float xn[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xn[a] = Q.save[(int64_t)(NS_X + a) * ld + s];
  // grid encoding: d features / d xn, level by level
  float dxn[3] = {0.0f, 0.0f, 0.0f};
  for (int l = 0; l < Q.grid.n_levels; ++l) {
    const float g0 = Q.dz[(int64_t)(ND_F + 2 * l) * ld + s];
    const float g1 = Q.dz[(int64_t)(ND_F + 2 * l + 1) * ld + s];
    if (g0 == 0.0f && g1 == 0.0f) continue;
    const NgpLevel V = ngp_level(Q.grid, l);
    float frac[3];
    uint32_t cell[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float p = fmaf(V.scale, xn[d], 0.5f);
      const float fl = floorf(p);
      cell[d] = (uint32_t)(int)fl;
      frac[d] = p - fl;
    }
    float lv[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      uint32_t p[3];
      float wd[3];  // the corner's per-dimension factor
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const bool up = (c >> d) & 1;
        p[d] = cell[d] + (up ? 1 : 0);
        wd[d] = up ? frac[d] : 1.0f - frac[d];
      }
      const uint32_t idx = V.offset + ngp_index(V, Q.grid.hashed, p[0], p[1], p[2]);
      const float2 t = *(const float2*)(Q.table + 2 * (int64_t)idx);
      const float v = g0 * t.x + g1 * t.y;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float sgn = ((c >> d) & 1) ? 1.0f : -1.0f;
        lv[d] += sgn * wd[(d + 1) % 3] * wd[(d + 2) % 3] * v;
      }
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) dxn[d] += V.scale * lv[d];
  }
  // SH input gradient: Wh0[:, 0:16]^T dz_h0
  float gsh[NGP_SH];
#pragma unroll
  for (int k = 0; k < NGP_SH; ++k) gsh[k] = 0.0f;
  const float* W = Q.mlp + Q.off.w[2];
  for (int o = 0; o < NGP_W; ++o) {
    const float dzo = Q.dz[(int64_t)(ND_Z2 + o) * ld + s];
#pragma unroll
    for (int k = 0; k < NGP_SH; ++k) gsh[k] = fmaf(W[o * NGP_HIN + k], dzo, gsh[k]);
  }
  float pos[3], dir[3], tt;
  rg_point(G, s, pos, dir, &tt);
  float J[3][3];
  contract_unit_jac(pos, G.aabb, G.contraction, J);
  float dpos[3], ddir[3];
#pragma unroll
  for (int b = 0; b < 3; ++b) dpos[b] = (dxn[0] * J[0][b] + dxn[1] * J[1][b]) + dxn[2] * J[2][b];
  sh4_backward(dir, gsh, ddir);
  rg_store(G, s, dpos, ddir, tt);
}

// ------------------------------------------------------------------ per-ray reduction
// One wave per ray: its samples are [r S, r S + S) (points 0) or the run of ray r in the sorted
// ray_idx[0 .. n_valid) (points 2; samples past n_valid are padding without gradient).  Overwrites
// d_o / d_d (R, 3).
__global__ void raygrad_reduce_kernel(int n_rays, int points, int n_samples, const int* ray_idx, int64_t n_valid,
                                      const float* per, float* d_o, float* d_d) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= n_rays) return;
  int64_t b, e;
  if (points == 0) {
    b = (int64_t)r * n_samples;
    e = b + n_samples;
  } else {
    // lower bounds of r and r + 1 (every lane runs the same search)
    int64_t lo = 0, hi = n_valid;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ray_idx[mid] < r) lo = mid + 1;
      else hi = mid;
    }
    b = lo;
    hi = n_valid;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ray_idx[mid] <= r) lo = mid + 1;
      else hi = mid;
    }
    e = lo;
  }
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t s = b + lane; s < e; s += 64)
#pragma unroll
    for (int q = 0; q < 6; ++q) acc[q] += per[s * 6 + q];
#pragma unroll
  for (int q = 0; q < 6; ++q) acc[q] = wave_sum(acc[q]);
  if (lane == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      d_o[(int64_t)r * 3 + a] = acc[a];
      d_d[(int64_t)r * 3 + a] = acc[3 + a];
    }
  }
}

// points 1: the per-sample values ARE the gradients of the given points / directions
__global__ void raygrad_split_kernel(int64_t n, const float* per, float* d_x, float* d_dir) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    d_x[s * 3 + a] = per[s * 6 + a];
    d_dir[s * 3 + a] = per[s * 6 + 3 + a];
  }
}

}  // namespace den
