// Store-pattern calibration, round 5 (2): chunks of uneven duration (0..4 extra dependent
// system-scope loads per chunk, as the expansion's rounds and page ends make them), dealt to
// workgroups flat (block order), XCD-static (xcd remap of blockIdx, assumes round-robin placement)
// or XCD-dynamic (each workgroup reads HW_REG_XCC_ID and claims the next chunk group of its XCD's
// eighth from a per-XCD counter, stealing from the other eighths once its own is done).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/store_patterns3 tools/store_patterns3.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef u64 v2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) v2 gv2;

__device__ __forceinline__ void st16(v2* p, v2 v) { __builtin_nontemporal_store(v, (gv2*)p); }
__device__ __forceinline__ u32 sld(const u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

__host__ __device__ __forceinline__ u32 xcd_order(u32 g, u32 n, u32 off) {
  const u32 u = g + off, U = n + off, x = u & 7u, j = u >> 3;
  const u32 q = U >> 3, r = U & 7u;
  const u32 base = x * q + (x < r ? x : r);
  return base + j - (x + 1u < off ? x + 1u : off);
}

// MODE 0 flat, 1 xcd static, 2 xcd dynamic (ctr[8] zeroed before the launch)
template <int MODE, int VAR>
__global__ __launch_bounds__(256) void k_chunks(v2* out, u64 n16, const u32* chain, u32 chain_mask, u32* ctr) {
  extern __shared__ uint8_t lds[];
  __shared__ u32 s_g;
  const u64 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u32 CHT = 16;
  const u64 n_ch = (n16 + 64 * CHT - 1) / (64 * CHT);
  const u32 ng = (u32)((n_ch + 3) / 4);
  u32 g;
  if (MODE == 0) g = blockIdx.x;
  else if (MODE == 1) g = xcd_order(blockIdx.x, gridDim.x, 0);
  else {
    if (threadIdx.x == 0) {
      u32 x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      x &= 7u;
      const u32 q = ng >> 3, r = ng & 7u;
      u32 got = 0xFFFFFFFFu;
      for (u32 k = 0; k < 8 && got == 0xFFFFFFFFu; k++) {
        const u32 y = (x + k) & 7u;
        const u32 cnt = q + (y < r ? 1u : 0u), base = y * q + (y < r ? y : r);
        const u32 t = atomicAdd(ctr + y, 1u);
        if (t < cnt) got = base + t;
      }
      s_g = got;
    }
    __syncthreads();
    g = s_g;
    if (g == 0xFFFFFFFFu) return;
  }
  const u64 c = (u64)g * 4 + wv;
  if (c >= n_ch) return;
  u32 x = (u32)c & chain_mask;
  const int dep = VAR ? (int)((c * 2654435761ull >> 7) % 5) : 4;
  for (int d = 0; d < dep; d++) x = sld(chain + x) & chain_mask;
  if (lane == 0) lds[wv] = (uint8_t)x;
  const u64 b = c * 64 * CHT;
#pragma unroll
  for (u32 t = 0; t < CHT; t++) {
    const u64 i = b + (u64)t * 64 + lane;
    if (i < n16) st16(out + i, v2{i, (u64)x});
  }
}

int main() {
  const u64 bytes = 800000000ull;
  const u64 n16 = bytes / 16;
  v2* out;
  u32 *chain, *ctr;
  const u32 CN = 1u << 20;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&chain, CN * 4) != hipSuccess || hipMalloc(&ctr, 64) != hipSuccess) return 1;
  {
    u32* h = (u32*)malloc(CN * 4);
    u64 s = 88172645463325252ull;
    for (u32 i = 0; i < CN; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (u32)s & (CN - 1); }
    (void)hipMemcpy(chain, h, CN * 4, hipMemcpyHostToDevice);
    free(h);
  }
  const size_t LDS = 26000;
  const u64 n_ch = (n16 + 1023) / 1024, nwg = (n_ch + 3) / 4;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
#define RUN(MODE, VAR)                                                                                     \
  {                                                                                                        \
    float tot = 0;                                                                                         \
    for (int r = -1; r < 20; r++) {                                                                        \
      (void)hipMemsetAsync(ctr, 0, 64);                                                                    \
      (void)hipEventRecord(a);                                                                             \
      hipLaunchKernelGGL((k_chunks<MODE, VAR>), dim3(nwg), dim3(256), LDS, 0, out, n16, chain, CN - 1, ctr); \
      (void)hipEventRecord(b);                                                                             \
      (void)hipEventSynchronize(b);                                                                        \
      float ms;                                                                                            \
      (void)hipEventElapsedTime(&ms, a, b);                                                                \
      if (r >= 0) tot += ms;                                                                               \
    }                                                                                                      \
    const float t = tot / 20;                                                                              \
    printf("mode=%s dep=%s  %.4f ms  %5.0f GB/s\n", MODE == 0 ? "flat   " : MODE == 1 ? "xcd-st " : "xcd-dyn", \
           VAR ? "0..4" : "4   ", t, bytes / t / 1e6);                                                     \
  }
  RUN(0, 0) RUN(1, 0) RUN(2, 0)
  RUN(0, 1) RUN(1, 1) RUN(2, 1)
  RUN(0, 0) RUN(1, 0) RUN(2, 0)
  return 0;
}
