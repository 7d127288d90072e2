// pqgpu_device.h — device helpers shared by the CDNA4 (gfx950) kernels of the decoder:
// wave/lane ids, buffer resources with hardware range checks, global/system-scope
// stores and loads, error reporting, the register byte window and the varint readers
// (BytesUtils.readUnsignedVarInt / readUnsignedVarLong / readZigZagVarLong).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_internal.h"

namespace pqg {

constexpr int WAVE = 64;
// Pages per workgroup: one page per wave, 4 waves per 256-lane workgroup. One-wave
// workgroups cap residency by the per-CU workgroup limit (measured: ~2.3k of 5k
// waves resident), so pages are packed 4 to a workgroup.
constexpr int WPB = 4;

__device__ __forceinline__ uint32_t wave_id() {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}
// Page of this wave, or -1 when the grid's last workgroup has fewer pages.
__device__ __forceinline__ int wave_page(const int32_t* list, int n_list) {
  const int i = (int)(blockIdx.x * WPB + wave_id());
  return i < n_list ? list[i] : -1;
}
#ifdef PQG_DIAG
// Diagnostic build only (libpqgpu_diag.so, tools/diag_timeline.py): per-wave
// stamps. Never compiled into the product library.
static __device__ uint64_t* pqg_diag_buf;
static __device__ uint64_t* pqg_diag_wrt;  // per page: s_memrealtime at walk start / publish
static __device__ uint64_t* pqg_diag_xrt;  // per chunk: start, flag seen, end, (page | cu << 32)
static __device__ uint64_t* pqg_diag_wph;  // per page: list-walk cycles (predecode, chain, emit), windows, batches, runs
static __device__ uint64_t* pqg_diag_bp;   // per k_bin_plain tile: start, walked, looked back, end (s_memrealtime), polls, guess ok
#define DIAG_T(v) uint64_t v = __builtin_amdgcn_s_memtime()
#define DIAG_ADD(acc, t0) acc += __builtin_amdgcn_s_memtime() - (t0)
#else
#define DIAG_T(v)
#define DIAG_ADD(acc, t0)
#endif

// Intra-wave ordering of LDS writes before reads by other lanes (no s_barrier:
// the waves of a workgroup work on different pages and do not meet).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint32_t uni(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Exclusive prefix sum over the wave (u32); *total = sum over all lanes.
__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t v, uint32_t* total) {
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((int)(threadIdx.x & 63u) >= o) x += y;
  }
  *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return x - v;
}

// Inclusive prefix sum over the wave (u64, wrapping) with DPP row shifts and row broadcasts
// (no LDS round trips). Call with all 64 lanes active.
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t x) {
#define PQG_DPP_STEP(ctrl, rmask)                                                                        \
  {                                                                                                      \
    const uint32_t lo_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, ctrl, rmask, 0xf, true);         \
    const uint32_t hi_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), ctrl, rmask, 0xf, true); \
    x += ((uint64_t)hi_ << 32) | lo_;                                                                    \
  }
  PQG_DPP_STEP(0x111, 0xf)  // row_shr:1
  PQG_DPP_STEP(0x112, 0xf)  // row_shr:2
  PQG_DPP_STEP(0x114, 0xf)  // row_shr:4
  PQG_DPP_STEP(0x118, 0xf)  // row_shr:8
  PQG_DPP_STEP(0x142, 0xa)  // row_bcast:15 -> rows 1, 3
  PQG_DPP_STEP(0x143, 0xc)  // row_bcast:31 -> rows 2, 3
#undef PQG_DPP_STEP
  return x;
}

// Mask of bytes [jb, je) (clamped) within dword i of a 16-byte block.
__device__ __forceinline__ uint32_t block_byte_mask(int32_t jb, int32_t je, int32_t i) {
  const int32_t lo = jb - 4 * i < 0 ? 0 : (jb - 4 * i > 4 ? 4 : jb - 4 * i);
  const int32_t hi = je - 4 * i < 0 ? 0 : (je - 4 * i > 4 ? 4 : je - 4 * i);
  const uint32_t mh = hi >= 4 ? 0xFFFFFFFFu : (1u << (8 * hi)) - 1u;
  const uint32_t ml = lo >= 4 ? 0xFFFFFFFFu : (1u << (8 * lo)) - 1u;
  return mh & ~ml;
}

// Minimum over the wave (u32), in every lane.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t y = __shfl_xor(v, o);
    v = v < y ? v : y;
  }
  return v;
}

// Maximum over the wave (u32), in every lane.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t y = __shfl_xor(v, o);
    v = v > y ? v : y;
  }
  return v;
}

// Stores through address_space(1) pointers: global_store_* count only in vmcnt.
// (Generic pointers give flat_store_*, which also count in lgkmcnt, so every
// s_waitcnt lgkmcnt(0) for an LDS read would wait for all stores in flight.)
#ifdef PQG_DIAG
static __device__ int pqg_diag_nostore;  // diagnostic ablation: skip output stores (set by pqg_diag_nostore_set)
#define PQG_STORE_GUARD if (!pqg_diag_nostore)
#else
#define PQG_STORE_GUARD
#endif
template <class T>
__device__ __forceinline__ void gst(T* p, T v) {
  PQG_STORE_GUARD *(__attribute__((address_space(1))) T*)p = v;
}
// Streaming output stores (plain stores measured 15 % slower on C2, round 1).
template <class T>
__device__ __forceinline__ void gst_nt(T* p, T v) {
  PQG_STORE_GUARD __builtin_nontemporal_store(v, (__attribute__((address_space(1))) T*)p);
}

// Lane-contiguous runs -> 1 KiB per store instruction. Lane l holds NR consecutive 16-byte rows of a
// wave's contiguous output (rows NR l .. NR l + NR - 1); on return st[i] holds row 64 i + l, so store
// i of the wave writes 1 KiB contiguous. (Each lane writing its own NR rows puts every instruction's 64
// rows NR * 16 bytes apart: 4 rows per lane stored at ~3.6 TB/s against 5.4-6.2 for 1 KiB per
// instruction, profiles/r02/store_patterns.txt 'lane-contig'.) Round a of NR: lane m (r = m % NR)
// fetches for store (a + r) % NR from lane (64 / NR) * ((a + r) % NR) + m / NR, which offers its row
// (c - a) % NR, c = its lane / (64 / NR): every lane is read by exactly one lane per round
// (4 ds_bpermute_b32 per round). All 64 lanes must be active.
template <uint32_t NR>
__device__ __forceinline__ void lane_rows_to_tiles(const u32x4 (&row)[NR], u32x4 (&st)[NR]) {
  static_assert(NR == 2 || NR == 4, "2 or 4 rows per lane");
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t c = lane / (64u / NR), r = lane % NR;
#pragma unroll
  for (uint32_t a = 0; a < NR; a++) {
    const uint32_t sel = (c - a) % NR;
    u32x4 q = row[0];
#pragma unroll
    for (uint32_t j = 1; j < NR; j++) q = sel == j ? row[j] : q;
    const uint32_t ia = (a + r) % NR;
    const int src = (int)((64u / NR) * ia + lane / NR);
    u32x4 got;
    got.x = (uint32_t)__shfl((int)q.x, src);
    got.y = (uint32_t)__shfl((int)q.y, src);
    got.z = (uint32_t)__shfl((int)q.z, src);
    got.w = (uint32_t)__shfl((int)q.w, src);
#pragma unroll
    for (uint32_t i = 0; i < NR; i++) st[i] = ia == i ? got : st[i];
  }
}

// Store the 16-byte output block at `a` (dwords wd) clipped to [o_lo, o_hi): one 16-byte store
// when the block is whole and aligned, dword stores for whole dwords, byte stores at the edges
// (which neighbouring chunks / pages share). have: bit q = dword q whole (0 for an unaligned dst).
__device__ __forceinline__ void store_block16(uint8_t* dst, uint64_t a, uint64_t o_lo, uint64_t o_hi,
                                              const uint32_t (&wd)[4], uint32_t have, bool dst_al16) {
  if (have == 0xFu && dst_al16) {
    gst_nt((u32x4*)(dst + a), u32x4{wd[0], wd[1], wd[2], wd[3]});
    return;
  }
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint64_t d0 = a + 4u * q;
    if ((have >> q) & 1u) {
      gst((uint32_t*)(dst + d0), wd[q]);
    } else {
      for (uint32_t j = 0; j < 4; j++)
        if (d0 + j >= o_lo && d0 + j < o_hi) gst(dst + d0 + j, (uint8_t)(wd[q] >> (8u * j)));
    }
  }
}

// Run records, chunk entries and page status are produced and consumed inside one launch
// by the fused dictionary kernel (different CUs, possibly different XCDs, whose L2s are not
// coherent): they are written and read with system-scope relaxed accesses (sc0 sc1: through
// to memory), ordered by s_waitcnt vmcnt(0) before the page's ready flag is set.
template <class T>
__device__ __forceinline__ void sst(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ T sld(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Buffer resource over [base, base + n) with hardware range checking: loads past
// n return 0 (never fault), so a window may overhang the end of the batch.
__device__ __forceinline__ rsrc_t make_rsrc(const uint8_t* base, uint64_t n) {
  uint64_t b = uni64((uint64_t)(uintptr_t)base);
  uint32_t nr = n > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)n;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)b, (short)0, (int)uni(nr), 0x00020000);
}

__device__ __forceinline__ uint32_t ld32(rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}

// 8 bytes at any byte offset (little endian). Branch-free (v_alignbyte): a load issued on
// only one path leaves the waitcnt pass a "maybe pending" load at every later merge point,
// and it then answers with s_waitcnt vmcnt(0) — draining all stores — in unrelated loops.
__device__ __forceinline__ uint64_t ld8_any(rsrc_t r, uint32_t off) {
  const uint32_t a = off & ~3u, sb = off & 3u;
  const uint32_t w0 = ld32(r, a), w1 = ld32(r, a + 4), w2 = ld32(r, a + 8);
  return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sb) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sb) << 32);
}

__device__ __forceinline__ uint32_t ld4_any(rsrc_t r, uint32_t off) {
  const uint32_t a = off & ~3u, sb = off & 3u;
  return __builtin_amdgcn_alignbyte(ld32(r, a + 4), ld32(r, a), sb);
}

// Record an error: smallest (index << 8 | code) per (page, kind) wins (epoch-tagged, see ErrCount).
__device__ __forceinline__ void report_key(uint64_t* word, ErrCount err_count, uint64_t key) {
  atomicMax((unsigned long long*)word, (unsigned long long)(((uint64_t)err_count.epoch << 48) | (~key & ERR_KEY_MASK)));
  atomicMax(err_count.p, err_count.epoch);
}
__device__ __forceinline__ void report(uint64_t* err, ErrCount err_count, int page, int kind, uint64_t index,
                                       int code) {
  report_key(&err[3 * (uint64_t)page + kind], err_count, (index << 8) | (uint64_t)code);
}

// ---------------------------------------------------------------------------
// Register window over a page: lane l holds bytes [B + 4l, B + 4l + 4) in wa and
// [B + 256 + 4l, ...) in wb. B is wave-uniform; reads are v_readlane.
struct Window {
  rsrc_t rs;
  uint32_t B;
  uint32_t wa, wb;

  __device__ __forceinline__ void seek(uint32_t p) {
    B = p & ~3u;
    wa = ld32(rs, B + 4u * lane_id());
    wb = ld32(rs, B + 256u + 4u * lane_id());
  }
  // Make [p, p + 12) resident. p never moves backwards.
  __device__ __forceinline__ void ensure(uint32_t p) {
    uint32_t k = p - B;
    if (k > 496u) {
      if (k <= 752u) {
        B += 256u;
        wa = wb;
        wb = ld32(rs, B + 256u + 4u * lane_id());
      } else {
        seek(p);
      }
    }
  }
  __device__ __forceinline__ uint32_t dword(uint32_t i) {
    uint32_t a = rdl(wa, i & 63u), b = rdl(wb, i & 63u);
    return i < 64u ? a : b;
  }
  __device__ __forceinline__ uint64_t read8(uint32_t p) {
    ensure(p);
    uint32_t k = p - B, i = k >> 2, sh = (k & 3u) * 8u;
    uint64_t x = (uint64_t)dword(i) | ((uint64_t)dword(i + 1) << 32);
    if (sh) x = (x >> sh) | ((uint64_t)dword(i + 2) << (64u - sh));
    return x;
  }
  __device__ __forceinline__ uint32_t byte(uint32_t p) {
    ensure(p);
    uint32_t k = p - B;
    return (dword(k >> 2) >> ((k & 3u) * 8u)) & 0xFFu;
  }
};

// readUnsignedVarInt (BytesUtils.java:202-211) at p. Sets len; Java int shift masking.
// `lim` = bytes readable before the section end; a varint not terminated within
// them gets len = lim + 1 (the caller's EOF check fails it, as read() would).
__device__ __forceinline__ uint32_t read_uvarint(Window& w, uint32_t p, uint32_t lim, uint32_t& len) {
  uint64_t x = w.read8(p);
  uint32_t b0 = (uint32_t)x & 0xFFu;
  if (!(b0 & 0x80u)) { len = 1; return b0; }
  uint32_t b1 = (uint32_t)(x >> 8) & 0xFFu;
  if (!(b1 & 0x80u)) { len = 2; return (b0 & 0x7Fu) | (b1 << 7); }
  uint32_t value = 0, i = 0, k = 0, b;
  for (;;) {
    b = (k < 8u) ? (uint32_t)(x >> (8u * k)) & 0xFFu : w.byte(p + k);
    if (!(b & 0x80u)) break;
    value |= (b & 0x7Fu) << (i & 31u);
    i += 7;
    k++;
    if (k >= lim) break;
  }
  len = k + 1;
  return value | (b << (i & 31u));
}

// readUnsignedVarLong (BytesUtils.java:260-269), Java long shift masking.
__device__ __forceinline__ uint64_t read_uvarlong(Window& w, uint32_t p, uint32_t lim, uint32_t& len) {
  uint64_t value = 0;
  uint32_t i = 0, k = 0, b;
  uint64_t x = w.read8(p);
  for (;;) {
    b = (k < 8u) ? (uint32_t)(x >> (8u * k)) & 0xFFu : w.byte(p + k);
    if (!(b & 0x80u)) break;
    value |= (uint64_t)(b & 0x7Fu) << (i & 63u);
    i += 7;
    k++;
    if (k >= lim) break;
  }
  len = k + 1;
  return value | ((uint64_t)b << (i & 63u));
}

// readZigZagVarLong (BytesUtils.java:254-258)
__device__ __forceinline__ int64_t zigzag64(uint64_t r) {
  int64_t sign = -(int64_t)(r & 1);
  int64_t temp = ((int64_t)((uint64_t)sign ^ r)) >> 1;
  return (int64_t)((uint64_t)temp ^ (r & 0x8000000000000000ull));
}

}  // namespace pqg
