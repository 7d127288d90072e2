// Calibration micro-benchmark (diagnostic, not product): HBM write bandwidth for the
// decode kernel's output pattern: n_pages waves, each writing page_bytes contiguous
// with 16-byte stores (nt or plain), 4 waves per 256-lane workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef unsigned long long u64;
typedef u64 v2 __attribute__((ext_vector_type(2)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void fill(v2* out, int n_pages, u64 elems_per_page) {
  int page = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (page >= n_pages) return;
  int lane = threadIdx.x & 63;
  __attribute__((address_space(1))) v2* o = (__attribute__((address_space(1))) v2*)(out + page * (elems_per_page / 2));
  u64 v = page;
  for (u64 i = lane; i < elems_per_page / 2; i += 64 * U) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      u64 j = i + 64 * u;
      if (j < elems_per_page / 2) {
        if (NT) __builtin_nontemporal_store(v2{v, j}, o + j);
        else o[j] = v2{v, j};
      }
    }
  }
}

// grid-stride over the whole buffer (ideal memset-like pattern)
__global__ __launch_bounds__(256) void fill_flat(v2* out, u64 n) {
  __attribute__((address_space(1))) v2* o = (__attribute__((address_space(1))) v2*)out;
  for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256) __builtin_nontemporal_store(v2{i, i}, o + i);
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
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
  const int n_pages = 5000;
  const u64 epp = 20000;
  const u64 bytes = n_pages * epp * 8;
  v2* out;
  hipMalloc(&out, bytes);
  int grid = (n_pages + 3) / 4;
  float t;
  t = timeit([&] { hipLaunchKernelGGL((fill<true, 1>), dim3(grid), dim3(256), 0, 0, out, n_pages, epp); }, 20);
  printf("per-page waves nt U1: %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL((fill<true, 4>), dim3(grid), dim3(256), 0, 0, out, n_pages, epp); }, 20);
  printf("per-page waves nt U4: %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL((fill<false, 4>), dim3(grid), dim3(256), 0, 0, out, n_pages, epp); }, 20);
  printf("per-page waves plain U4: %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  for (int g : {1024, 2048, 4096, 8192}) {
    t = timeit([&] { hipLaunchKernelGGL(fill_flat, dim3(g), dim3(256), 0, 0, out, bytes / 16); }, 20);
    printf("grid-stride nt grid=%d: %.3f ms  %.0f GB/s\n", g, t, bytes / t / 1e6);
  }
  t = timeit([&] { hipMemsetAsync(out, 0, bytes); }, 20);
  printf("hipMemset: %.3f ms  %.0f GB/s\n", t, bytes / t / 1e6);
  return 0;
}
