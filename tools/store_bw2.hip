// Calibration (diagnostic, not product): write bandwidth of chunked output patterns, 800 MB.
// chunk_fill<NT, CH>: one wave per CH-KiB chunk, 64 lanes x 16 B per store instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
typedef u64 v2 __attribute__((ext_vector_type(2)));

template <int MODE, int CHK>
__global__ __launch_bounds__(256) void chunk_fill(v2* out, u64 n_chunks) {
  const u64 c = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= n_chunks) return;
  const int lane = threadIdx.x & 63;
  __attribute__((address_space(1))) v2* o = (__attribute__((address_space(1))) v2*)(out + c * (CHK * 1024 / 16));
#pragma unroll 4
  for (int t = 0; t < CHK; t++) {
    v2 v = v2{c, (u64)t};
    if (MODE == 0) __builtin_nontemporal_store(v, o + t * 64 + lane);
    else if (MODE == 1) o[t * 64 + lane] = v;
    else __hip_atomic_store((u64*)(o + t * 64 + lane), c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); f();
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
  const u64 bytes = 800ull << 20;
  v2* out;
  hipMalloc(&out, bytes);
  float t;
#define RUN(M, K)                                                                                      \
  {                                                                                                    \
    u64 nc = bytes / (K * 1024);                                                                       \
    t = timeit([&] { hipLaunchKernelGGL((chunk_fill<M, K>), dim3((nc + 3) / 4), dim3(256), 0, 0, out, nc); }, 20); \
    printf("mode %d chunk %3d KiB: %.3f ms  %.0f GB/s\n", M, K, t, bytes / t / 1e6);                  \
  }
  RUN(0, 4) RUN(0, 16) RUN(0, 64) RUN(1, 4) RUN(1, 16) RUN(1, 64)
  t = timeit([&] { hipMemsetAsync(out, 0, bytes, 0); }, 20);
  printf("hipMemset: %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  return 0;
}
