// pqgpu_assembly.hip — record assembly of one leaf column on gfx950: repetition / definition
// levels -> the columnar form of the records (offsets of every REPEATED node, validity of every
// OPTIONAL node), the Arrow-style equivalent of the converter events parquet-mr's Dremel
// automaton emits (RecordReaderImplementation.read, parquet-column/.../io/RecordReaderImplementation.java:409-446).
//
// Entries of repetition depth r: the records (r = 0) or the elements of the r-th REPEATED node
// on the path. Slot i begins an entry of depth r when rep[i] <= r and def[i] >= DR[r], DR[r]
// being the definition level of the r-th REPEATED node (DR[0] = 0): that is exactly when the
// automaton opens the node's group (definitionLevelToDepth, :314-324) after closing down to
// nextLevel[rep] (:284-306). Then, per entry of depth r starting at slot i:
//   OPTIONAL node k at depth r:   validity = def[i] >= D(k)
//   REPEATED node at depth r + 1: offsets[entry] = number of depth-(r+1) entries before slot i
// so every output is a function of per-depth exclusive counts: three passes (block counts,
// scan of the block counts, emit) over the levels, HBM-bound on the level bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

constexpr uint32_t ASM_BLOCK = 4096;  // slots per workgroup (256 threads x 16 slots)
constexpr uint32_t ASM_PER_THREAD = 16;

__device__ __forceinline__ uint32_t asm_entries_mask(const AsmParams& P, uint32_t d, uint32_t r) {
  // bit q: slot begins an entry of depth q
  uint32_t m = 0;
#pragma unroll
  for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++)
    if (q <= P.max_rep && r <= q && d >= P.DR[q]) m |= 1u << q;
  return m;
}

__global__ __launch_bounds__(256) void k_asm_count(const uint8_t* __restrict__ def, const uint8_t* __restrict__ rep,
                                                   uint64_t n, AsmParams P, uint64_t* __restrict__ block_counts) {
  __shared__ uint32_t red[4][ASM_MAX_DEPTHS];
  const uint64_t s0 = (uint64_t)blockIdx.x * ASM_BLOCK + (uint64_t)threadIdx.x * ASM_PER_THREAD;
  uint32_t c[ASM_MAX_DEPTHS] = {};
  for (uint32_t j = 0; j < ASM_PER_THREAD; j++) {
    const uint64_t s = s0 + j;
    if (s >= n) break;
    const uint32_t m = asm_entries_mask(P, def ? def[s] : 0u, rep ? rep[s] : 0u);
#pragma unroll
    for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) c[q] += (m >> q) & 1u;
  }
#pragma unroll
  for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) {
    uint32_t v = c[q];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane_id() == 0) red[threadIdx.x >> 6][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < ASM_MAX_DEPTHS) {
    const uint32_t q = threadIdx.x;
    block_counts[(uint64_t)blockIdx.x * ASM_MAX_DEPTHS + q] = (uint64_t)red[0][q] + red[1][q] + red[2][q] + red[3][q];
  }
}

// One workgroup: exclusive scan of every depth's block counts (in place); totals[q] = entries
// of depth q (read by the host, which checks the output capacities before k_asm_emit).
__global__ __launch_bounds__(256) void k_asm_scan(uint64_t* __restrict__ block_counts, uint32_t n_blocks, AsmParams P,
                                                  uint64_t* __restrict__ totals) {
  __shared__ uint64_t wsum[4];
  __shared__ uint64_t carry;
  for (uint32_t q = 0; q <= P.max_rep; q++) {
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < n_blocks; b0 += 256) {
      const uint32_t b = b0 + threadIdx.x;
      const uint64_t v = b < n_blocks ? block_counts[(uint64_t)b * ASM_MAX_DEPTHS + q] : 0;
      uint64_t x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if ((int)lane_id() >= o) x += y;
      }
      if (lane_id() == 63) wsum[threadIdx.x >> 6] = x;
      __syncthreads();
      uint64_t pre = carry;
      for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) pre += wsum[w];
      if (b < n_blocks) block_counts[(uint64_t)b * ASM_MAX_DEPTHS + q] = pre + x - v;
      __syncthreads();
      if (threadIdx.x == 255) carry = pre + x;
      __syncthreads();
    }
    if (threadIdx.x == 0) totals[q] = carry;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_asm_emit(const uint8_t* __restrict__ def, const uint8_t* __restrict__ rep,
                                                  uint64_t n, AsmParams P, const uint64_t* __restrict__ block_counts,
                                                  const uint64_t* __restrict__ totals) {
  __shared__ uint32_t wsum[4][ASM_MAX_DEPTHS];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // closing offsets: offsets[n_entries(r - 1)] = n_entries(r)
    for (uint32_t k = 0; k < P.n_nodes; k++)
      if (P.kind[k] == PQG_REPEATED && P.offsets[k]) gst(P.offsets[k] + totals[P.depth[k] - 1], (int64_t)totals[P.depth[k]]);
  }
  const uint64_t s0 = (uint64_t)blockIdx.x * ASM_BLOCK + (uint64_t)threadIdx.x * ASM_PER_THREAD;
  uint32_t dv[ASM_PER_THREAD], mk[ASM_PER_THREAD];
  uint32_t c[ASM_MAX_DEPTHS] = {};
#pragma unroll
  for (uint32_t j = 0; j < ASM_PER_THREAD; j++) {
    const uint64_t s = s0 + j;
    const bool in = s < n;
    dv[j] = in && def ? def[s] : 0u;
    mk[j] = in ? asm_entries_mask(P, dv[j], rep ? rep[s] : 0u) : 0u;
#pragma unroll
    for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) c[q] += (mk[j] >> q) & 1u;
  }
  // block-exclusive prefix of every depth's count -> the entry index of this thread's first slot
  uint64_t idx[ASM_MAX_DEPTHS];
#pragma unroll
  for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) {
    uint32_t x = c[q];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if ((int)lane_id() >= o) x += y;
    }
    if (lane_id() == 63) wsum[threadIdx.x >> 6][q] = x;
    idx[q] = x - c[q];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) {
    uint64_t pre = block_counts[(uint64_t)blockIdx.x * ASM_MAX_DEPTHS + q];
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) pre += wsum[w][q];
    idx[q] += pre;
  }
  for (uint32_t j = 0; j < ASM_PER_THREAD; j++) {
    const uint32_t m = mk[j];
    if (m) {
      for (uint32_t k = 0; k < P.n_nodes; k++) {
        const uint32_t q = P.depth[k];
        if (P.kind[k] == PQG_OPTIONAL) {
          if (((m >> q) & 1u) && P.validity[k]) gst(P.validity[k] + idx[q], (uint8_t)(dv[j] >= P.D[k] ? 1 : 0));
        } else if (P.kind[k] == PQG_REPEATED) {
          // one list per entry of the enclosing depth: offsets = entries of this depth before the slot
          if (((m >> (q - 1)) & 1u) && P.offsets[k]) gst(P.offsets[k] + idx[q - 1], (int64_t)idx[q]);
        }
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) idx[q] += (m >> q) & 1u;
  }
}

hipError_t launch_assemble(hipStream_t st, const uint8_t* def, const uint8_t* rep, uint64_t n, const AsmParams& P,
                           uint64_t* block_counts, uint32_t n_blocks, uint64_t* totals, int phase) {
  if (phase == 0) {
    if (n_blocks) hipLaunchKernelGGL(k_asm_count, dim3(n_blocks), dim3(256), 0, st, def, rep, n, P, block_counts);
    hipLaunchKernelGGL(k_asm_scan, dim3(1), dim3(256), 0, st, block_counts, n_blocks, P, totals);
  } else if (n_blocks) {
    hipLaunchKernelGGL(k_asm_emit, dim3(n_blocks), dim3(256), 0, st, def, rep, n, P, block_counts, totals);
  }
  return hipGetLastError();
}

}  // namespace pqg
