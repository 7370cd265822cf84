// stream_probe.hip -- diagnostic: the hidden backward's memory pattern without its compute.  Per
// 32-sample block a layer launch reads two 16 KiB blocks (dz_l, S'_{l-1}) and writes one (dz_{l-1}, over
// S'_{l-1} in place); here every variant moves exactly those bytes for n_blocks blocks, each workgroup a
// contiguous range, so the byte rate of the pattern can be compared across ways of issuing it:
//   V 0  hidden_bwd_kernel's own: one workgroup of 4 waves per CU, both reads by non-temporal LDS-DMA
//        DEPTH blocks ahead into a ring, counted vmcnt waits + a barrier per block, the written block
//        read back from LDS (ds_read_b128) and stored non-temporally (the in-place output)
//   V 1  the same with the output to a separate buffer
//   V 2  register streaming: W waves per workgroup, global_load_dwordx4 of both reads (non-temporal),
//        UNROLL blocks in flight per wave, the sum of the two stored non-temporally, no LDS
//   V 3  V 2 with plain (cached) stores
// Launch: grid workgroups of 64 * waves threads; the LDS variants 1 per CU (ring size), V 2/3 up to
// occupancy.  No reference counterpart; profiles/stream_probe/stream_probe.py drives it.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 16384;

__device__ __forceinline__ void dma_block(const char* src, char* dst, int waves) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int pc = wave; pc < 16; pc += waves) {
    const int p = __builtin_amdgcn_readfirstlane(pc);
    const char* base = src + p * 1024;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(dst + p * 1024));
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"((uint32_t)lane * 16),
                 "s"(base), "s"(m0) : "memory", "m0");
  }
}

template <bool SEPARATE, int DEPTH>
__global__ __launch_bounds__(256, 1) void lds_stream_kernel(const char* a, char* b, char* c, int64_t n_blocks,
                                                            int64_t per_wg, int64_t stride) {
  constexpr int RING = DEPTH + 1;
  __shared__ __attribute__((aligned(16))) char lds[RING * 2 * BLOCK];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b0 = (int64_t)blockIdx.x * per_wg;
  const int64_t n_it = b0 < n_blocks ? (b0 + per_wg < n_blocks ? per_wg : n_blocks - b0) : 0;
  char* out = SEPARATE ? c : b;
  for (int u = 0; u < DEPTH; ++u)
    if (u < n_it) {
      dma_block(a + (b0 + u) * stride, lds + u * 2 * BLOCK, 4);
      dma_block(b + (b0 + u) * stride, lds + u * 2 * BLOCK + BLOCK, 4);
    }
  __builtin_amdgcn_s_waitcnt(7 << 4);  // vmcnt(0) lgkmcnt(0)
  __syncthreads();
  for (int64_t it = 0; it < n_it; ++it) {
    const int u = (int)(it % RING);
    if (it + DEPTH < n_it) {
      const int v = (u + DEPTH) % RING;
      dma_block(a + (b0 + it + DEPTH) * stride, lds + v * 2 * BLOCK, 4);
      dma_block(b + (b0 + it + DEPTH) * stride, lds + v * 2 * BLOCK + BLOCK, 4);
    }
    // the block's output: wave w writes its 4 KiB quarter (4 x 1 KiB), from both staged reads
    const char* s = lds + u * 2 * BLOCK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int off = (wave * 4 + q) * 1024 + lane * 16;
      const u32x4 x = *(const u32x4*)(s + off), y = *(const u32x4*)(s + BLOCK + off);
      __builtin_nontemporal_store(x ^ y, (u32x4*)(out + (b0 + it) * stride + off));
    }
    // wait for this wave's part of block it + 1: younger than its DMAs (issued DEPTH - 1 iterations
    // ago) are its stores and the DEPTH - 1 later (DMA, stores) pairs: 4 + (DEPTH - 1) * (8 + 4)
    // vector-memory ops (hidden_bwd_kernel's YOUNGER; 28 at DEPTH 3); lgkmcnt(0) for the LDS reads
    constexpr int VM = 4 + (DEPTH - 1) * 12;
    if (it + DEPTH < n_it) __builtin_amdgcn_s_waitcnt((VM & 15) | (7 << 4) | ((VM >> 4) << 14));
    else __builtin_amdgcn_s_waitcnt(7 << 4);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
}

template <int UNROLL, bool NT>
__global__ __launch_bounds__(512) void reg_stream_kernel(const u32x4* a, const u32x4* b, u32x4* c, int64_t n_blocks,
                                                         int64_t per_wg) {
  // the workgroup's waves split each block: 16 KiB = 1024 x 16 B; thread t handles vector t, t + threads, ...
  const int64_t b0 = (int64_t)blockIdx.x * per_wg;
  const int64_t n_it = b0 < n_blocks ? (b0 + per_wg < n_blocks ? per_wg : n_blocks - b0) : 0;
  const int64_t n_vec = n_it * (BLOCK / 16);
  const int64_t base = b0 * (BLOCK / 16);
  const int step = blockDim.x;
  for (int64_t i = threadIdx.x; i < n_vec; i += (int64_t)step * UNROLL) {
    u32x4 x[UNROLL], y[UNROLL];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const int64_t j = i + (int64_t)k * step;
      if (j < n_vec) {
        x[k] = __builtin_nontemporal_load(a + base + j);
        y[k] = __builtin_nontemporal_load(b + base + j);
      }
    }
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
      const int64_t j = i + (int64_t)k * step;
      if (j < n_vec) {
        const u32x4 z = x[k] ^ y[k];
        if (NT) __builtin_nontemporal_store(z, c + base + j);
        else c[base + j] = z;
      }
    }
  }
}

}  // namespace

// stride: bytes from one block of a stream to the next (BLOCK: three separate tensors; larger: the
// streams interleaved in one buffer); variants 4 / 5: the separate-output LDS kernel at DEPTH 2 / 4
extern "C" int stream_probe_launch(int variant, int grid, int waves, const void* a, void* b, void* c,
                                   int64_t n_blocks, int64_t stride, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (grid <= 0 || n_blocks <= 0 || stride < BLOCK) return 1;
  const int64_t per_wg = (n_blocks + grid - 1) / grid;
  switch (variant) {
    case 0:
      hipLaunchKernelGGL((lds_stream_kernel<false, 3>), dim3(grid), dim3(256), 0, s, (const char*)a, (char*)b,
                         (char*)c, n_blocks, per_wg, stride);
      break;
    case 1:
      hipLaunchKernelGGL((lds_stream_kernel<true, 3>), dim3(grid), dim3(256), 0, s, (const char*)a, (char*)b,
                         (char*)c, n_blocks, per_wg, stride);
      break;
    case 4:
      hipLaunchKernelGGL((lds_stream_kernel<true, 2>), dim3(grid), dim3(256), 0, s, (const char*)a, (char*)b,
                         (char*)c, n_blocks, per_wg, stride);
      break;
    case 5:
      hipLaunchKernelGGL((lds_stream_kernel<true, 4>), dim3(grid), dim3(256), 0, s, (const char*)a, (char*)b,
                         (char*)c, n_blocks, per_wg, stride);
      break;
    case 2:
      if (waves < 1 || waves > 8 || stride != BLOCK) return 1;
      hipLaunchKernelGGL((reg_stream_kernel<4, true>), dim3(grid), dim3(64 * waves), 0, s, (const u32x4*)a,
                         (const u32x4*)b, (u32x4*)c, n_blocks, per_wg);
      break;
    case 3:
      if (waves < 1 || waves > 8 || stride != BLOCK) return 1;
      hipLaunchKernelGGL((reg_stream_kernel<4, false>), dim3(grid), dim3(64 * waves), 0, s, (const u32x4*)a,
                         (const u32x4*)b, (u32x4*)c, n_blocks, per_wg);
      break;
    default:
      return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
