// Store-pattern calibration for the dictionary expansion (800 MB of int64 output, the C2
// launch): which assignment of output bytes to waves reaches the highest HBM write rate.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/store_patterns tools/store_patterns.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint64_t u64;
typedef u64 v2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) v2 gv2;

template <bool NT>
__device__ __forceinline__ void st16(v2* p, v2 v) {
  if (NT) __builtin_nontemporal_store(v, (gv2*)p);
  else *(gv2*)p = v;
}

// Each wave writes one contiguous span of `span` bytes (1 KB per store instruction).
template <bool NT>
__global__ __launch_bounds__(256) void k_stream(v2* out, u64 n16, u64 span16) {
  const u64 w = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 lane = threadIdx.x & 63;
  const u64 b = w * span16;
  if (b >= n16) return;
  const u64 e = b + span16 < n16 ? b + span16 : n16;
  for (u64 i = b + lane; i < e; i += 64) st16<NT>(out + i, v2{i, w});
}

// Persistent: workgroup g owns a contiguous region; its 4 waves take chunks of `chunk16`
// round-robin (the k_dict_expand assignment).
template <bool NT>
__global__ __launch_bounds__(256) void k_wg_chunks(v2* out, u64 n16, u64 chunk16, u64 per_wg) {
  const u64 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u64 n_ch = (n16 + chunk16 - 1) / chunk16;
  const u64 c0 = (u64)blockIdx.x * per_wg, c1 = c0 + per_wg < n_ch ? c0 + per_wg : n_ch;
  for (u64 c = c0 + wv; c < c1; c += 4)
    for (u64 i = c * chunk16 + lane; i < (c + 1) * chunk16 && i < n16; i += 64) st16<NT>(out + i, v2{i, c});
}

// Persistent, chunks dealt round-robin over all waves of the grid (grid-stride in chunks).
template <bool NT>
__global__ __launch_bounds__(256) void k_grid_chunks(v2* out, u64 n16, u64 chunk16) {
  const u64 lane = threadIdx.x & 63;
  const u64 w = (u64)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (u64)gridDim.x * 4;
  const u64 n_ch = (n16 + chunk16 - 1) / chunk16;
  for (u64 c = w; c < n_ch; c += nw)
    for (u64 i = c * chunk16 + lane; i < (c + 1) * chunk16 && i < n16; i += 64) st16<NT>(out + i, v2{i, c});
}

// Each lane writes `per_lane` consecutive 16-byte words (lane-contiguous, 64*per_lane*16 B per wave step).
template <bool NT, int PL>
__global__ __launch_bounds__(256) void k_lane_contig(v2* out, u64 n16) {
  const u64 t = (u64)blockIdx.x * 256 + threadIdx.x, nt = (u64)gridDim.x * 256;
  for (u64 base = t * PL; base < n16; base += nt * PL)
#pragma unroll
    for (int u = 0; u < PL; u++)
      if (base + u < n16) st16<NT>(out + base + u, v2{base, (u64)u});
}

// Grid-stride, one 16-byte store per lane per step (the classic fill kernel).
template <bool NT>
__global__ __launch_bounds__(256) void k_gridstride(v2* out, u64 n16) {
  const u64 t = (u64)blockIdx.x * 256 + threadIdx.x, nt = (u64)gridDim.x * 256;
  for (u64 i = t; i < n16; i += nt) st16<NT>(out + i, v2{i, 1});
}

// XCD-aware: workgroup b runs on XCD (b % 8); give each XCD one contiguous eighth of the buffer and
// deal that eighth's chunks to its workgroups in order.
template <bool NT>
__global__ __launch_bounds__(256) void k_xcd_chunks(v2* out, u64 n16, u64 chunk16) {
  const u64 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const u64 xcd = blockIdx.x & 7, j = blockIdx.x >> 3, per_x = (gridDim.x + 7) >> 3;
  const u64 n_ch = (n16 + chunk16 - 1) / chunk16, ch_x = (n_ch + 7) / 8;
  for (u64 c = xcd * ch_x + j * 4 + wv; c < (xcd + 1) * ch_x && c < n_ch; c += per_x * 4)
    for (u64 i = c * chunk16 + lane; i < (c + 1) * chunk16 && i < n16; i += 64) st16<NT>(out + i, v2{i, c});
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
  if (hipMalloc(&out, bytes) != hipSuccess) return 1;
  float t;
#define REPORT(name) printf("%-44s %.3f ms  %5.0f GB/s\n", name, t, bytes / t / 1e6)
  char nm[128];
  for (u64 span : {8192ull, 32768ull, 163840ull, 655360ull}) {
    const u64 s16 = span / 16, waves = (n16 + s16 - 1) / s16;
    t = timeit([&] { hipLaunchKernelGGL(k_stream<true>, dim3((waves + 3) / 4), dim3(256), 0, 0, out, n16, s16); }, 20);
    snprintf(nm, sizeof nm, "stream nt span=%lluKB waves=%llu", span / 1024, waves);
    REPORT(nm);
    t = timeit([&] { hipLaunchKernelGGL(k_stream<false>, dim3((waves + 3) / 4), dim3(256), 0, 0, out, n16, s16); }, 20);
    snprintf(nm, sizeof nm, "stream plain span=%lluKB", span / 1024);
    REPORT(nm);
  }
  for (u64 chunk : {8192ull, 32768ull}) {
    for (u64 wg : {1024ull, 2048ull}) {
      const u64 c16 = chunk / 16, n_ch = (n16 + c16 - 1) / c16, per = (n_ch + wg - 1) / wg;
      t = timeit([&] { hipLaunchKernelGGL(k_wg_chunks<true>, dim3(wg), dim3(256), 0, 0, out, n16, c16, per); }, 20);
      snprintf(nm, sizeof nm, "wg-chunks nt chunk=%lluKB wg=%llu", chunk / 1024, wg);
      REPORT(nm);
      t = timeit([&] { hipLaunchKernelGGL(k_wg_chunks<false>, dim3(wg), dim3(256), 0, 0, out, n16, c16, per); }, 20);
      snprintf(nm, sizeof nm, "wg-chunks plain chunk=%lluKB wg=%llu", chunk / 1024, wg);
      REPORT(nm);
      t = timeit([&] { hipLaunchKernelGGL(k_grid_chunks<true>, dim3(wg), dim3(256), 0, 0, out, n16, c16); }, 20);
      snprintf(nm, sizeof nm, "grid-chunks nt chunk=%lluKB wg=%llu", chunk / 1024, wg);
      REPORT(nm);
    }
  }
  for (u64 g : {1024ull, 2048ull, 8192ull}) {
    t = timeit([&] { hipLaunchKernelGGL((k_lane_contig<true, 4>), dim3(g), dim3(256), 0, 0, out, n16); }, 20);
    snprintf(nm, sizeof nm, "lane-contig x4 nt grid=%llu", g);
    REPORT(nm);
    t = timeit([&] { hipLaunchKernelGGL((k_lane_contig<false, 4>), dim3(g), dim3(256), 0, 0, out, n16); }, 20);
    snprintf(nm, sizeof nm, "lane-contig x4 plain grid=%llu", g);
    REPORT(nm);
  }
  for (u64 g : {1024ull, 2048ull, 4096ull, 16384ull, 65536ull}) {
    t = timeit([&] { hipLaunchKernelGGL(k_gridstride<true>, dim3(g), dim3(256), 0, 0, out, n16); }, 20);
    snprintf(nm, sizeof nm, "gridstride nt grid=%llu", g);
    REPORT(nm);
    t = timeit([&] { hipLaunchKernelGGL(k_gridstride<false>, dim3(g), dim3(256), 0, 0, out, n16); }, 20);
    snprintf(nm, sizeof nm, "gridstride plain grid=%llu", g);
    REPORT(nm);
  }
  for (u64 chunk : {16384ull, 65536ull}) {
    for (u64 g : {2048ull, 8192ull}) {
      t = timeit([&] { hipLaunchKernelGGL(k_xcd_chunks<true>, dim3(g), dim3(256), 0, 0, out, n16, chunk / 16); }, 20);
      snprintf(nm, sizeof nm, "xcd-chunks nt chunk=%lluKB grid=%llu", chunk / 1024, g);
      REPORT(nm);
      t = timeit([&] { hipLaunchKernelGGL(k_xcd_chunks<false>, dim3(g), dim3(256), 0, 0, out, n16, chunk / 16); }, 20);
      snprintf(nm, sizeof nm, "xcd-chunks plain chunk=%lluKB grid=%llu", chunk / 1024, g);
      REPORT(nm);
    }
  }
  t = timeit([&] { hipMemsetAsync(out, 0, bytes); }, 20);
  REPORT("hipMemset");
  t = timeit([&] { hipMemsetD32Async((hipDeviceptr_t)out, 0x12345678, bytes / 4); }, 20);
  REPORT("hipMemsetD32");
  return 0;
}
