// Store-pattern calibration, round 5: the dictionary expansion's shape (one wave per 16 KiB output
// chunk, 4 waves per workgroup, the fused kernel's ~26.6 KiB of LDS per workgroup) with and without
// a chain of dependent system-scope loads before the first store, and with the chunks dealt to
// workgroups XCD-aware (workgroup b runs on XCD b % 8: each XCD sweeps one contiguous eighth).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/store_patterns2 tools/store_patterns2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef u64 v2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) v2 gv2;

__device__ __forceinline__ void st16(v2* p, v2 v) { __builtin_nontemporal_store(v, (gv2*)p); }
__device__ __forceinline__ u32 sld(const u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// chunk of wave w: XCD=false: w; XCD=true: the workgroup's XCD sweeps its eighth in dispatch order
template <bool XCD>
__device__ __forceinline__ u64 chunk_of(u64 n_ch) {
  const u64 wv = threadIdx.x >> 6;
  if (!XCD) return (u64)blockIdx.x * 4 + wv;
  const u64 nwg = gridDim.x, x = blockIdx.x & 7, j = blockIdx.x >> 3;
  const u64 per_x = (nwg + 7) / 8;  // workgroups per XCD
  return (x * per_x + j) * 4 + wv;
}

// DEP dependent loads (each address from the previous value), then CHT tiles of 1 KiB.
template <bool XCD, int DEP, int CHT>
__global__ __launch_bounds__(256) void k_chunks(v2* out, u64 n16, const u32* chain, u32 chain_mask) {
  extern __shared__ uint8_t lds[];
  const u64 lane = threadIdx.x & 63;
  const u64 n_ch = (n16 + 64 * CHT - 1) / (64 * CHT);
  const u64 c = chunk_of<XCD>(n_ch);
  if (c >= n_ch) return;
  u32 x = (u32)c & chain_mask;
#pragma unroll
  for (int d = 0; d < DEP; d++) x = sld(chain + x) & chain_mask;
  if (lane == 0) lds[threadIdx.x >> 6] = (uint8_t)x;
  const u64 b = c * 64 * CHT;
#pragma unroll
  for (int t = 0; t < CHT; t++) {
    const u64 i = b + (u64)t * 64 + lane;
    if (i < n16) st16(out + i, v2{i, (u64)x});
  }
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < reps; r++) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const u64 bytes = 800000000ull;
  const u64 n16 = bytes / 16;
  v2* out;
  u32* chain;
  const u32 CN = 1u << 20;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&chain, CN * 4) != hipSuccess) return 1;
  {
    u32* h = (u32*)malloc(CN * 4);
    u64 s = 88172645463325252ull;
    for (u32 i = 0; i < CN; i++) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      h[i] = (u32)s & (CN - 1);
    }
    hipMemcpy(chain, h, CN * 4, hipMemcpyHostToDevice);
    free(h);
  }
  const size_t LDS = 26624;
  float t;
  char nm[128];
#define RUN(XCD, DEP, CHT)                                                                                      \
  {                                                                                                             \
    const u64 n_ch = (n16 + 64 * CHT - 1) / (64 * CHT);                                                         \
    const u64 nwg = (n_ch + 3) / 4;                                                                             \
    t = timeit([&] { hipLaunchKernelGGL((k_chunks<XCD, DEP, CHT>), dim3(nwg), dim3(256), LDS, 0, out, n16, chain, \
                                        CN - 1); }, 20);                                                        \
    snprintf(nm, sizeof nm, "chunks %s dep=%d tiles=%d (%llu KiB)", XCD ? "xcd " : "flat", DEP, CHT,          \
             (u64)CHT);                                                                                         \
    printf("%-44s %.4f ms  %5.0f GB/s\n", nm, t, bytes / t / 1e6);                                              \
  }
  RUN(false, 0, 16) RUN(true, 0, 16)
  RUN(false, 2, 16) RUN(true, 2, 16)
  RUN(false, 4, 16) RUN(true, 4, 16)
  RUN(false, 0, 32) RUN(true, 0, 32)
  RUN(false, 4, 32) RUN(true, 4, 32)
  RUN(false, 0, 8) RUN(true, 0, 8)
  RUN(false, 4, 8) RUN(true, 4, 8)
  t = timeit([&] { hipMemsetAsync(out, 0, bytes); }, 20);
  printf("%-44s %.4f ms  %5.0f GB/s\n", "hipMemset", t, bytes / t / 1e6);
  return 0;
}
