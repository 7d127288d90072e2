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
// so every output is a function of per-depth exclusive counts: three kernels (block counts, scan
// of the block counts, emit), the level bytes read twice with 16-byte loads, the outputs staged in
// LDS per block and stored as whole dwords / int64 runs; HBM-bound on the level bytes and outputs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

constexpr uint32_t ASM_BLOCK = 4096;  // slots per workgroup (256 threads x 16 slots)
constexpr uint32_t ASM_PER_THREAD = 16;
constexpr uint32_t ASM_SCAN_THREADS = 1024;

__device__ __forceinline__ uint32_t asm_entries_mask(const AsmParams& P, uint32_t d, uint32_t r) {
  // bit q: slot begins an entry of depth q
  uint32_t m = 0;
#pragma unroll
  for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++)
    if (q <= P.max_rep && r <= q && d >= P.DR[q]) m |= 1u << q;
  return m;
}

// The 16 level bytes of thread slot range [s0, s0 + 16): one 16-byte load when the range is whole
// (level arrays from pqg_decode are 256-byte aligned; any other alignment takes bytes), bytes at the tail.
__device__ __forceinline__ void asm_load16(const uint8_t* __restrict__ a, uint64_t s0, uint64_t n, uint32_t (&w)[4]) {
  if (!a) {
    w[0] = w[1] = w[2] = w[3] = 0;
  } else if (s0 + ASM_PER_THREAD <= n && (((uintptr_t)(a + s0)) & 15u) == 0) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)(a + s0));
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  } else {
    w[0] = w[1] = w[2] = w[3] = 0;
    for (uint32_t j = 0; j < ASM_PER_THREAD && s0 + j < n; j++) w[j >> 2] |= (uint32_t)a[s0 + j] << (8 * (j & 3));
  }
}

__device__ __forceinline__ uint32_t bt_at(const uint32_t (&bt)[ASM_MAX_DEPTHS], uint32_t q) {
  uint32_t v = 0;
#pragma unroll
  for (uint32_t d = 0; d < ASM_MAX_DEPTHS; d++) v = d == q ? bt[d] : v;
  return v;
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[4], uint32_t j) { return (w[j >> 2] >> (8 * (j & 3))) & 0xFFu; }

__global__ __launch_bounds__(256) void k_asm_count(const uint8_t* __restrict__ def, const uint8_t* __restrict__ rep,
                                                   uint64_t n, AsmParams P, uint64_t* __restrict__ block_counts) {
  __shared__ uint32_t red[4][ASM_MAX_DEPTHS];
  const uint64_t s0 = (uint64_t)blockIdx.x * ASM_BLOCK + (uint64_t)threadIdx.x * ASM_PER_THREAD;
  uint32_t dw[4], rw[4];
  asm_load16(def, s0, n, dw);
  asm_load16(rep, s0, n, rw);
  uint32_t c[ASM_MAX_DEPTHS] = {};
#pragma unroll
  for (uint32_t j = 0; j < ASM_PER_THREAD; j++) {
    const uint32_t m = s0 + j < n ? asm_entries_mask(P, byte_of(dw, j), byte_of(rw, j)) : 0u;
#pragma unroll
    for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) c[q] += (m >> q) & 1u;
  }
#pragma unroll
  for (uint32_t q = 0; q < ASM_MAX_DEPTHS; q++) {
    uint32_t v = c[q];
    if (q <= P.max_rep) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    }
    if (lane_id() == 0) red[threadIdx.x >> 6][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < ASM_MAX_DEPTHS) {
    const uint32_t q = threadIdx.x;
    block_counts[(uint64_t)blockIdx.x * ASM_MAX_DEPTHS + q] =
        q <= P.max_rep ? (uint64_t)red[0][q] + red[1][q] + red[2][q] + red[3][q] : 0;
  }
}

// One workgroup of 1024 threads: exclusive scan of every depth's block counts (in place); each
// thread sums a contiguous segment of blocks, a workgroup scan of the segment sums gives the
// segment bases, the segment is rewritten. totals[q] = entries of depth q.
__global__ __launch_bounds__(ASM_SCAN_THREADS) void k_asm_scan(uint64_t* __restrict__ block_counts, uint32_t n_blocks,
                                                               AsmParams P, uint64_t* __restrict__ totals) {
  __shared__ uint64_t wsum[ASM_SCAN_THREADS / 64];
  const uint32_t seg = (n_blocks + ASM_SCAN_THREADS - 1) / ASM_SCAN_THREADS;
  const uint32_t b0 = min(n_blocks, threadIdx.x * seg), b1 = min(n_blocks, b0 + seg);
  for (uint32_t q = 0; q <= P.max_rep; q++) {
    uint64_t v = 0;
    for (uint32_t b = b0; b < b1; b++) v += block_counts[(uint64_t)b * ASM_MAX_DEPTHS + q];
    const uint64_t x = wave_incl_scan_u64(v);
    if (lane_id() == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t pre = x - v;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) pre += wsum[w];
    if (threadIdx.x == ASM_SCAN_THREADS - 1) totals[q] = pre + v;
    for (uint32_t b = b0; b < b1; b++) {
      const uint64_t c = block_counts[(uint64_t)b * ASM_MAX_DEPTHS + q];
      block_counts[(uint64_t)b * ASM_MAX_DEPTHS + q] = pre;
      pre += c;
    }
    __syncthreads();
  }
}

// Single pass (outputs): the entry counts before a block come from a decoupled look-back over the
// blocks before it instead of a separate count kernel and scan, so the levels are read once.
// Block order is the order in which workgroups take a ticket (atomicAdd), so every block a
// workgroup waits for is held by a running or finished workgroup: the look-back always ends.
// status[b * ASM_MAX_DEPTHS + q] (zeroed before the launch): ASM_AGG | the block's entry count of
// depth q, then ASM_INC | the inclusive count of blocks 0..b; written and read system-scope (the
// blocks may run on different XCDs, whose L2s are not coherent), the value and its flag in one word.
// Outputs: per node, the block's entries are a contiguous range of the node's output (entries are
// numbered in slot order), so every thread writes its entries' values into an LDS image of the range
// and the workgroup stores the image with wide stores (validity bytes: dwords with byte stores only at
// the ends shared with the neighbouring blocks; offsets: int64 runs).
constexpr uint64_t ASM_AGG = 1ull << 62, ASM_INC = 2ull << 62, ASM_VAL = (1ull << 62) - 1ull;

// MD: repetition depths the kernel tracks (max_rep + 1 <= MD; 2, 4 or 8): per-thread counts, indexes and the
// packed per-slot entry masks sized for it, so a flat LIST column (max_rep 1) runs at 8 workgroups per CU;
// the offsets image holds 32-bit block-relative counts (16 KiB of LDS: the 64-bit image's 32 KiB and 97
// VGPRs allowed 4 workgroups per CU). The look-back reads every depth's status word of a predecessor in one
// round trip (one loop over 64 predecessors for all depths, where each depth had its own loop).
// threads of a one-pass workgroup (8 waves, 8,192 slots): C5 assembly 0.94 ms at 4 waves / 4,096 slots, 0.76 ms
// here, 1.08 ms at 16 waves / 16,384 slots (profiles/r06/asm_blocks)
constexpr uint32_t ASM1_THREADS = 512;
constexpr uint32_t ASM1_BLOCK = ASM1_THREADS * ASM_PER_THREAD;  // slots per one-pass block
constexpr uint32_t ASM1_WAVES = ASM1_THREADS / 64;
template <uint32_t MD>
__global__ __launch_bounds__(ASM1_THREADS) void k_asm_onepass(const uint8_t* __restrict__ def, const uint8_t* __restrict__ rep,
                                                     uint64_t n, AsmParams P, uint64_t* status, uint32_t* ticket,
                                                     uint64_t* __restrict__ totals, uint32_t n_blocks) {
  static_assert(MD == 2 || MD == 4 || MD == 8, "depth classes");
  constexpr uint32_t MB = MD <= 4 ? 4u : 8u;            // mask bits per slot in the packed masks
  constexpr uint32_t NMK = (ASM_PER_THREAD * MB) / 64u;  // 64-bit words of packed masks
  __shared__ uint32_t wsum[ASM1_WAVES][MD];
  __shared__ uint64_t bc[MD];
  __shared__ uint32_t blk_s;
  __shared__ uint32_t img[ASM1_BLOCK];  // 32 KiB: one node's entries of this block (validity bytes / relative offsets)
  if (threadIdx.x == 0) blk_s = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t blk = blk_s;
  const uint32_t max_rep = P.max_rep;
  const uint64_t s0 = (uint64_t)blk * ASM1_BLOCK + (uint64_t)threadIdx.x * ASM_PER_THREAD;
  uint32_t dw[4], rw[4];
  asm_load16(def, s0, n, dw);
  asm_load16(rep, s0, n, rw);
  uint64_t mkp[NMK] = {};
  uint32_t c[MD] = {};
#pragma unroll
  for (uint32_t j = 0; j < ASM_PER_THREAD; j++) {
    const uint32_t m = s0 + j < n ? asm_entries_mask(P, byte_of(dw, j), byte_of(rw, j)) : 0u;
    mkp[(j * MB) / 64u] |= (uint64_t)m << ((j * MB) % 64u);
#pragma unroll
    for (uint32_t q = 0; q < MD; q++) c[q] += (m >> q) & 1u;
  }
  auto mk = [&](uint32_t j) -> uint32_t { return (uint32_t)(mkp[(j * MB) / 64u] >> ((j * MB) % 64u)) & ((1u << MB) - 1u); };
  // block-local exclusive index of this thread's first entry of every depth, block totals
  uint32_t li[MD], bt[MD];
#pragma unroll
  for (uint32_t q = 0; q < MD; q++) {
    uint32_t tot = 0;
    li[q] = q <= max_rep ? wave_excl_scan_u32(c[q], &tot) : 0u;
    if (lane_id() == 0) wsum[threadIdx.x >> 6][q] = tot;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < MD; q++) {
    uint32_t pre = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) pre += wsum[w][q];
    li[q] += pre;
    uint32_t t = 0;
#pragma unroll
    for (uint32_t w = 0; w < ASM1_WAVES; w++) t += wsum[w][q];
    bt[q] = t;
  }
  auto bt_q = [&](uint32_t q) -> uint32_t {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t d = 0; d < MD; d++) v = d == q ? bt[d] : v;
    return v;
  };
  // publish this block's counts, then look back (wave 0): 64 predecessors per step, one lane each, every
  // depth's status word of a predecessor loaded in the same round trip; per depth the nearest predecessor
  // holding an inclusive count ends its look-back, the aggregates of those nearer are added (the decoupled
  // look-back of a single-pass scan)
  if (threadIdx.x <= max_rep)
    sst(status + (uint64_t)blk * ASM_MAX_DEPTHS + threadIdx.x, (blk == 0 ? ASM_INC : ASM_AGG) | (uint64_t)bt_q(threadIdx.x));
  if (threadIdx.x < WAVE) {
    const uint32_t lane = lane_id();
    uint64_t excl[MD] = {};
    uint32_t open = (1u << (max_rep + 1u)) - 1u;  // depths still looking back (uniform)
    int64_t j0 = (int64_t)blk - 1;                 // nearest predecessor of the current step
    const uint64_t t_wait = __builtin_amdgcn_s_memrealtime();
    while (open && j0 >= 0) {
      const int64_t j = j0 - (int64_t)lane;
      uint64_t v[MD];
#pragma unroll
      for (uint32_t q = 0; q < MD; q++)
        v[q] = ((open >> q) & 1u) ? (j >= 0 ? sld(status + (uint64_t)j * ASM_MAX_DEPTHS + q) : ASM_INC) : ASM_INC;
      bool again = false;
      uint32_t first[MD];
#pragma unroll
      for (uint32_t q = 0; q < MD; q++) {
        const uint64_t inc = __ballot((v[q] & ASM_INC) != 0);
        first[q] = inc ? (uint32_t)__builtin_ctzll(inc) : WAVE;  // nearest inclusive (lane)
        const uint64_t upto = first[q] == WAVE ? ~0ull : ((2ull << first[q]) - 1ull);
        if (((open >> q) & 1u) && (__ballot(v[q] == 0) & upto)) again = true;  // not published yet
      }
      if (again) {  // a block up to a depth's nearest inclusive one has not published: read the window again
        __builtin_amdgcn_s_sleep(1);
        // bounded (2 s of s_memrealtime): a block that never publishes leaves a wrong count, not a hang
        if (__builtin_amdgcn_s_memrealtime() - t_wait > 200000000ull) {
          if (lane == 0) totals[ASM_MAX_DEPTHS - 1] = ~0ull;  // flagged to the host as a timeout
          break;
        }
        continue;
      }
#pragma unroll
      for (uint32_t q = 0; q < MD; q++) {
        if (!((open >> q) & 1u)) continue;
        uint64_t x = lane <= first[q] || first[q] == WAVE ? (v[q] & ASM_VAL) : 0ull;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
        excl[q] += x;
        if (first[q] < WAVE) open &= ~(1u << q);
      }
      j0 -= WAVE;
    }
    if (lane == 0) {
#pragma unroll
      for (uint32_t q = 0; q < MD; q++) {
        if (q > max_rep) break;
        const uint32_t agg = bt_q(q);
        if (blk > 0) sst(status + (uint64_t)blk * ASM_MAX_DEPTHS + q, ASM_INC | (excl[q] + agg));
        bc[q] = excl[q];
        if (blk == n_blocks - 1u) totals[q] = excl[q] + agg;
      }
    }
  }
  __syncthreads();
  if (blk == n_blocks - 1u && threadIdx.x == 0) {  // closing offsets: offsets[n_entries(r - 1)] = n_entries(r)
    for (uint32_t k = 0; k < P.n_nodes; k++)
      if (P.kind[k] == PQG_REPEATED && P.offsets[k]) {
        const uint32_t d = P.depth[k];
        gst(P.offsets[k] + bc[d - 1] + bt_q(d - 1), (int64_t)(bc[d] + bt_q(d)));
      }
  }
  uint8_t* img8 = (uint8_t*)img;
  for (uint32_t k = 0; k < P.n_nodes; k++) {
    const uint32_t q = P.depth[k];
    uint32_t li_q = 0, li_p = 0;  // this thread's first entry of depth q (and q - 1)
#pragma unroll
    for (uint32_t d = 0; d < MD; d++) {
      li_q = d == q ? li[d] : li_q;
      li_p = d + 1u == q ? li[d] : li_p;
    }
    if (P.kind[k] == PQG_OPTIONAL && P.validity[k]) {
      const uint32_t Dk = P.D[k];
      uint32_t l = li_q;
#pragma unroll
      for (uint32_t j = 0; j < ASM_PER_THREAD; j++)
        if ((mk(j) >> q) & 1u) img8[l++] = byte_of(dw, j) >= Dk ? 1 : 0;
      __syncthreads();
      // bytes [B, B + cnt) of validity[k]: aligned 16-byte blocks inside (unaligned 32-bit LDS reads of
      // the image), bytes at both ends
      typedef uint32_t __attribute__((aligned(1), may_alias)) u32u;
      uint8_t* g = P.validity[k] + bc[q];
      const uint32_t cnt = bt_q(q);
      const uint32_t mis = (uint32_t)((16u - ((uintptr_t)g & 15u)) & 15u);
      const uint32_t head = mis < cnt ? mis : cnt;
      const uint32_t nd = (cnt - head) >> 4;
      for (uint32_t i = threadIdx.x; i < nd; i += ASM1_THREADS) {
        const uint8_t* s = img8 + head + 16u * i;
        gst((u32x4*)(g + head + 16u * i),
            u32x4{*(const u32u*)s, *(const u32u*)(s + 4), *(const u32u*)(s + 8), *(const u32u*)(s + 12)});
      }
      const uint32_t tail0 = head + 16u * nd;
      if (threadIdx.x < head) gst(g + threadIdx.x, img8[threadIdx.x]);
      if (threadIdx.x >= 64 && threadIdx.x - 64 < cnt - tail0) gst(g + tail0 + (threadIdx.x - 64), img8[tail0 + (threadIdx.x - 64)]);
      __syncthreads();
    } else if (P.kind[k] == PQG_REPEATED && P.offsets[k]) {
      // one list per entry of the enclosing depth q - 1: its offset = entries of depth q before the slot,
      // kept relative to the block's first entry of depth q (bc[q]) in the image
      uint32_t l = li_p;
      uint32_t e = li_q;
#pragma unroll
      for (uint32_t j = 0; j < ASM_PER_THREAD; j++) {
        if ((mk(j) >> (q - 1)) & 1u) img[l++] = e;
        e += (mk(j) >> q) & 1u;
      }
      __syncthreads();
      const uint64_t base = bc[q];
      int64_t* g = P.offsets[k] + bc[q - 1];
      const uint32_t cnt = bt_q(q - 1);
      // pairs as 16-byte stores from the first 16-byte aligned entry on
      const bool al8 = ((uintptr_t)g & 7u) == 0;  // (an int64 array off 8-byte alignment: one entry per store)
      const uint32_t head = (((uintptr_t)g & 15u) != 0 && cnt > 0) ? 1u : 0u;
      const uint32_t np = al8 ? (cnt - head) >> 1 : 0u;
      if (!al8)
        for (uint32_t i = threadIdx.x; i < cnt; i += ASM1_THREADS) gst(g + i, (int64_t)(base + img[i]));
      typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
      for (uint32_t i = threadIdx.x; i < np; i += ASM1_THREADS)
        gst((i64x2*)(g + head + 2u * i),
            i64x2{(int64_t)(base + img[head + 2u * i]), (int64_t)(base + img[head + 2u * i + 1u])});
      if (al8 && threadIdx.x == 0 && head) gst(g, (int64_t)(base + img[0]));
      if (al8 && threadIdx.x == 64 && ((cnt - head) & 1u)) gst(g + cnt - 1u, (int64_t)(base + img[cnt - 1u]));
      __syncthreads();
    }
  }
}

hipError_t launch_assemble(hipStream_t st, const uint8_t* def, const uint8_t* rep, uint64_t n, const AsmParams& P,
                           uint64_t* block_counts, uint32_t n_blocks, uint64_t* totals, uint32_t* ticket, int phase) {
  if (phase == 0) {  // entry counts only
    if (n_blocks) hipLaunchKernelGGL(k_asm_count, dim3(n_blocks), dim3(256), 0, st, def, rep, n, P, block_counts);
    hipLaunchKernelGGL(k_asm_scan, dim3(1), dim3(ASM_SCAN_THREADS), 0, st, block_counts, n_blocks, P, totals);
  } else if (n_blocks) {  // outputs (and totals) in one pass; block_counts = zeroed status words, ticket = 0
    // (blocks of ASM1_BLOCK slots: at most the count pass's n_blocks status words are used)
    const uint32_t n1 = (uint32_t)((n + ASM1_BLOCK - 1) / ASM1_BLOCK);
    if (P.max_rep < 2u)
      hipLaunchKernelGGL(k_asm_onepass<2>, dim3(n1), dim3(ASM1_THREADS), 0, st, def, rep, n, P, block_counts, ticket,
                         totals, n1);
    else if (P.max_rep < 4u)
      hipLaunchKernelGGL(k_asm_onepass<4>, dim3(n1), dim3(ASM1_THREADS), 0, st, def, rep, n, P, block_counts, ticket,
                         totals, n1);
    else
      hipLaunchKernelGGL(k_asm_onepass<8>, dim3(n1), dim3(ASM1_THREADS), 0, st, def, rep, n, P, block_counts, ticket,
                         totals, n1);
  }
  return hipGetLastError();
}

}  // namespace pqg
