// Hand-off transport check for den_hidden.hip hidden_pair_kernel: producer workgroup i writes
// 16 KiB blocks into a ring slot, publishes a counter; consumer workgroup i + 8 (same XCD under
// round-robin placement) waits for the counter and reads the slot.  Variants of the consumer read:
//   0: LDS-DMA sc1, 1: LDS-DMA nt, 2: global_load_dwordx4 sc1 to registers, 3: LDS-DMA after an
//   agent acquire fence.  Producer: sc1 stores, vmcnt(0), barrier, sc1 counter store.
// Every word the consumer sees is compared with the expected pattern; mismatches are counted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 16384, RING = 8, NBLK = 64, THREADS = 256;

__device__ uint32_t pattern(int pair, int blk, int word) { return (uint32_t)(pair * 1000003u + blk * 7919u + word * 31u + 17u); }

__device__ uint32_t g_log[64 * 4];
__device__ void log_bad(uint32_t* bad, int pair, int b, int w, uint32_t got) {
  const uint32_t i = atomicAdd(bad + 2, 1u);
  if (i < 64) { g_log[4 * i] = pair; g_log[4 * i + 1] = b; g_log[4 * i + 2] = w; g_log[4 * i + 3] = got; }
}
template <int V>
__global__ __launch_bounds__(THREADS, 1) void k(char* ring, uint32_t* sync, uint32_t* bad, uint32_t* timeouts) {
  __shared__ __attribute__((aligned(16))) char lds[BLOCK];
  const int g = blockIdx.x / 16, r = blockIdx.x % 16;
  const bool consumer = r >= 8;
  const int pair = g * 8 + (r & 7);
  uint32_t* pub = sync + pair * 64;
  uint32_t* con = pub + 32;
  const int t = threadIdx.x;
  for (int b = 0; b < NBLK; ++b) {
    char* slot = ring + ((int64_t)pair * RING + b % RING) * BLOCK;
    if (!consumer) {
      // wait until the consumer freed the slot
      if (b >= RING) {
        int k = 0;
        while (__hip_atomic_load(con, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)(b - RING + 1) && k < (1 << 22)) { __builtin_amdgcn_s_sleep(2); ++k; }
        if (k == (1 << 22) && t == 0) atomicAdd(timeouts, 1u);
      }
      for (int q = 0; q < BLOCK / 16 / THREADS; ++q) {
        const int w16 = q * THREADS + t;
        i32x4 v = {(int)pattern(pair, b, 4 * w16), (int)pattern(pair, b, 4 * w16 + 1), (int)pattern(pair, b, 4 * w16 + 2), (int)pattern(pair, b, 4 * w16 + 3)};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(slot + w16 * 16), "v"(v) : "memory");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) asm volatile("global_store_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : : "v"(pub), "v"((uint32_t)(b + 1)) : "memory");
    } else {
      int k = 0;
      while (__hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)(b + 1) && k < (1 << 22)) { __builtin_amdgcn_s_sleep(2); ++k; }
      if (k == (1 << 22) && t == 0) atomicAdd(timeouts, 1u);
      if (V == 3) { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
      __syncthreads();
      uint32_t nbad = 0;
      if (V == 2) {
        for (int q = 0; q < BLOCK / 16 / THREADS; ++q) {
          const int w16 = q * THREADS + t;
          i32x4 v;
          asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(slot + w16 * 16) : "memory");
          for (int e = 0; e < 4; ++e)
            if ((uint32_t)v[e] != pattern(pair, b, 4 * w16 + e)) { ++nbad; log_bad(bad, pair, b, 4 * w16 + e, (uint32_t)v[e]); }
        }
      } else {
        const int wave = t >> 6, lane = t & 63;
        for (int q = 0; q < BLOCK / 1024 / 4; ++q) {
          const int pc = __builtin_amdgcn_readfirstlane(q * 4 + wave);
          const char* base = slot + pc * 1024;
          const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(lds + pc * 1024));
          const uint32_t off = lane * 16;
          if (V == 1)
            asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" : : "v"(off), "s"(base), "s"(m0) : "memory", "m0");
          else
            asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 sc1" : : "v"(off), "s"(base), "s"(m0) : "memory", "m0");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int w = t; w < BLOCK / 4; w += THREADS)
          if (((const uint32_t*)lds)[w] != pattern(pair, b, w)) { ++nbad; log_bad(bad, pair, b, w, ((const uint32_t*)lds)[w]); }
      }
      if (nbad) atomicAdd(bad, nbad);
      __syncthreads();
      if (t == 0) asm volatile("global_store_dword %0, %1, off sc1" : : "v"(con), "v"((uint32_t)(b + 1)) : "memory");
    }
  }
}

int main() {
  const int pairs = 128;
  char* ring;
  uint32_t *sync, *cnt;
  (void)hipMalloc(&ring, (size_t)pairs * RING * BLOCK);
  hipMalloc(&sync, pairs * 64 * 4);
  hipMalloc(&cnt, 16);
  // pollute the ring first with other values (stale data a broken hand-off would read)
  hipMemset(ring, 0xAB, (size_t)pairs * RING * BLOCK);
  hipDeviceSynchronize();
  for (int V = 0; V < 4; ++V) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(sync, 0, pairs * 64 * 4);
      hipMemset(cnt, 0, 16);
      if (V == 0) hipLaunchKernelGGL(k<0>, dim3(2 * pairs), dim3(THREADS), 0, 0, ring, sync, cnt, cnt + 1);
      if (V == 1) hipLaunchKernelGGL(k<1>, dim3(2 * pairs), dim3(THREADS), 0, 0, ring, sync, cnt, cnt + 1);
      if (V == 2) hipLaunchKernelGGL(k<2>, dim3(2 * pairs), dim3(THREADS), 0, 0, ring, sync, cnt, cnt + 1);
      if (V == 3) hipLaunchKernelGGL(k<3>, dim3(2 * pairs), dim3(THREADS), 0, 0, ring, sync, cnt, cnt + 1);
      uint32_t h[2];
      hipMemcpy(h, cnt, 8, hipMemcpyDeviceToHost);
      printf("variant %d rep %d: bad words %u / %u, timeouts %u\n", V, rep, h[0], pairs * NBLK * BLOCK / 4, h[1]);
      if (rep == 0) {
        uint32_t lg[64 * 4];
        hipMemcpyFromSymbol(lg, HIP_SYMBOL(g_log), sizeof(lg));
        for (int i = 0; i < 12; ++i) {
          const uint32_t p = lg[4 * i], b = lg[4 * i + 1], w = lg[4 * i + 2];
          const uint32_t exp = p * 1000003u + b * 7919u + w * 31u + 17u;
          long long db = -1;
          for (int bb = 0; bb < NBLK; ++bb) if (p * 1000003u + bb * 7919u + w * 31u + 17u == lg[4 * i + 3]) db = bb;
          printf("   pair %u blk %u word %u got %08x exp %08x (matches block %lld)\n", p, b, w, lg[4 * i + 3], exp, db);
        }
      }
      // re-pollute between reps
      hipMemset(ring, 0xCD + rep, (size_t)pairs * RING * BLOCK);
      hipDeviceSynchronize();
    }
  }
  return 0;
}
