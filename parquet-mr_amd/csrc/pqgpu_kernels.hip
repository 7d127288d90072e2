// pqgpu_kernels.hip — CDNA4 (gfx950) kernels of the MI355X Parquet page decoder.
//
// Hot path: RLE/bit-packed hybrid decode of dictionary ids and
// levels, dictionary gather, PLAIN copy, DELTA_BINARY_PACKED. All integer /
// byte work: no MFMA. One 64-lane wave decodes one page:
//
//   walk    — the wave reads the page section through a 512-byte register
//             window (one dword per lane, two halves) and follows the run
//             headers with v_readlane on the scalar unit. Each walked run
//             lands in one lane's registers (run r -> lane r % 64), so a batch
//             of 64 runs is a register-resident run table; no LDS.
//   resolve — lanes holding RLE runs fetch their dictionary entry (one gather
//             per run, not per value).
//   expand  — lanes sweep the batch's output range in 16-byte stores; for each
//             chunk a ballot finds the runs overlapping it and a uniform loop
//             over those runs selects each element's run. Bit-packed elements
//             are unpacked from the page bytes (buffer loads hit L1/L2: the
//             walk just touched them) and gathered from the dictionary.
//
// Semantics follow the reference reader value for value:
//   RunLengthBitPackingHybridDecoder.readInt/readNext (rle/…Decoder.java:61-109),
//   DictionaryValuesReader.initFromPage/read* (dictionary/DictionaryValuesReader.java:48-118),
//   PlainValuesReader (plain/PlainValuesReader.java:32-138),
//   DeltaBinaryPackingValuesReader (delta/DeltaBinaryPackingValuesReader.java:59-172),
//   ColumnReaderBase.readPageV1/V2 + levels (impl/ColumnReaderBase.java:650-789).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "pqgpu_device.h"

namespace pqg {

// ---------------------------------------------------------------------------
// RLE / bit-packed hybrid walker (RunLengthBitPackingHybridDecoder.readNext :80-109).
//
// Parallel pre-decode: a 256-byte window [B, B + 256) is held one dword per
// lane (plus the next two dwords), and every lane decodes a run header at each
// of its 4 byte positions as if a run started there (varint, count, RLE value or
// packed data start, next header position). The serial part — following the
// chain of headers from the section start — is then 4 v_readlane per run.

struct PreWin {
  rsrc_t rs;
  // Optional LDS copy of page bytes [seg_lo, seg_lo + SEG_BYTES): windows inside it are read
  // from LDS. (A global load issued after this wave's stores waits for all of them: vmcnt
  // counts stores on CDNA, so the bytes are staged before the first store.)
  uint8_t* seg;
  uint32_t seg_lo;
  uint32_t B;          // uniform: window start (4-aligned, page-relative)
  uint32_t nxt[4];     // per lane, byte b: next header position (0xFFFFFFFF: overflow)
  uint32_t cnt[4];     // run count (values)
  uint32_t val[4];     // RLE: raw value; PACKED: data start
  uint32_t flg;        // byte b: bit0 packed, bit1 slow path, bits 2..4 header length
};

constexpr uint32_t SEG_BYTES = 3072;   // LDS page segment per wave of k_dict_runs (5 workgroups per CU)


// Fill the wave's LDS segment with page bytes [lo, lo + SEG_BYTES) (lo 16-aligned).
__device__ __forceinline__ void seg_fill(PreWin& pw, uint32_t lo) {
  pw.seg_lo = lo;
#pragma unroll
  for (uint32_t i = 0; i < SEG_BYTES; i += 16u * WAVE) {
    const uint32_t o = i + 16u * lane_id();
    if (o < SEG_BYTES) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(pw.rs, (int)(lo + o), 0, 0);
      *(u32x4*)(pw.seg + o) = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// True when bytes [a, a + n) of the page are in the segment.
__device__ __forceinline__ bool seg_has(const PreWin& pw, uint32_t a, uint32_t n) {
  return pw.seg && a >= pw.seg_lo && a + n <= pw.seg_lo + SEG_BYTES;
}

// LDS byte buffers are written as u32x4 and read as u32: may_alias keeps TBAA from
// reordering the two.
typedef uint32_t __attribute__((may_alias)) u32_alias;

__device__ __forceinline__ uint32_t seg32(const PreWin& pw, uint32_t a) {  // a 4-aligned, inside
  return *(const u32_alias*)(pw.seg + (a - pw.seg_lo));
}

// LDS_ONLY: the caller guarantees the whole section is in the segment (no refill,
// no global load: the hot loop then never waits on vmcnt, which would drain stores).
// FAST: headers of at most 4 bytes are parsed branch-free from the position's first dword; a
// 5-byte header (a count / group number of 2^27 or more) is marked slow and left to the scalar
// path, so an RLE value (<= 4 bytes) always lies inside the 8 bytes at the position.
template <bool LDS_ONLY = false, bool FAST = false>
__device__ __forceinline__ void predecode(PreWin& pw, uint32_t B, int w) {
  pw.B = B;
  const uint32_t base = B + 4u * lane_id();
  if (!LDS_ONLY && pw.seg && !seg_has(pw, B, 264u)) seg_fill(pw, B & ~15u);
  uint32_t d0, d1, d2;
  if (LDS_ONLY || pw.seg) {
    d0 = seg32(pw, base);
    d1 = seg32(pw, base + 4);
    d2 = seg32(pw, base + 8);
  } else {
    d0 = ld32(pw.rs, base);
    d1 = ld32(pw.rs, base + 4);
    d2 = ld32(pw.rs, base + 8);
  }
  const uint64_t lo = (uint64_t)d0 | ((uint64_t)d1 << 32);
  const uint32_t nb = ((uint32_t)w + 7u) >> 3;
  uint32_t flg = 0;
#pragma unroll
  for (uint32_t b = 0; b < 4; b++) {
    const uint32_t p = base + b;
    // bytes p .. p+7 in x, byte p+8 .. in hi8
    const uint64_t x = b ? ((lo >> (8 * b)) | ((uint64_t)d2 << (64 - 8 * b))) : lo;
    const uint32_t hi8 = d2 >> (8 * b);
    const uint32_t b0 = (uint32_t)x & 0xFFu, b1 = (uint32_t)(x >> 8) & 0xFFu, b2 = (uint32_t)(x >> 16) & 0xFFu,
                   b3 = (uint32_t)(x >> 24) & 0xFFu, b4 = (uint32_t)(x >> 32) & 0xFFu;
    // readUnsignedVarInt, Java int semantics, up to 5 bytes here (longer: slow path)
    uint32_t v = b0 & 0x7Fu, hl = 1, slow = 0;
    if constexpr (FAST) {
      const uint32_t d = (uint32_t)x, stop = ~d & 0x80808080u;  // stop bit of each of 4 bytes
      slow = stop == 0u;
      hl = stop ? ((uint32_t)__builtin_ctz(stop) >> 3) + 1u : 4u;
      const uint32_t dm = d & (0xFFFFFFFFu >> (32u - 8u * hl));
      v = (dm & 0x7Fu) | ((dm >> 1) & 0x3F80u) | ((dm >> 2) & 0x1FC000u) | ((dm >> 3) & 0xFE00000u);
      (void)b1; (void)b2; (void)b3; (void)b4;
    } else if (b0 & 0x80u) {
      v |= (b1 & 0x7Fu) << 7; hl = 2;
      if (b1 & 0x80u) {
        v |= (b2 & 0x7Fu) << 14; hl = 3;
        if (b2 & 0x80u) {
          v |= (b3 & 0x7Fu) << 21; hl = 4;
          if (b3 & 0x80u) {
            v |= b4 << 28; hl = 5;
            if (b4 & 0x80u) slow = 1;
          }
        }
      }
    }
    uint32_t nx, c, vv, pk;
    if ((v & 1u) == 0) {  // RLE: count, then ceil(w/8) little-endian bytes, not masked
      const uint32_t sh = 8u * hl;
      const uint64_t y = FAST ? x >> sh : (x >> sh) | ((uint64_t)hi8 << (64u - sh));
      vv = nb == 4 ? (uint32_t)y : (uint32_t)y & ((1u << (8u * nb)) - 1u);
      c = v >> 1;
      nx = p + hl + nb;
      pk = 0;
    } else {              // PACKED: (header >>> 1) groups of 8 values, groups * w bytes
      const uint32_t groups = v >> 1;
      if (groups == 0 || groups >= (1u << 28)) slow = 1;
      c = groups * 8u;
      vv = p + hl;
      const uint64_t e = (uint64_t)p + hl + (uint64_t)groups * (uint32_t)w;
      nx = e > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)e;
      pk = 1;
    }
    pw.nxt[b] = nx;
    pw.cnt[b] = c;
    pw.val[b] = vv;
    flg |= (pk | (slow << 1) | (hl << 2)) << (8 * b);
  }
  pw.flg = flg;
}

// Scalar re-decode of one header at `pos` (rare: varints longer than 5 bytes,
// 0 or >= 2^28 groups). Bytes come through uniform buffer loads.
__device__ __forceinline__ uint32_t sbyte(rsrc_t rs, uint32_t p) {
  return uni((ld32(rs, p & ~3u) >> ((p & 3u) * 8u)) & 0xFFu);
}

template <class ByteAt>
__device__ int slow_header_g(ByteAt sbyte_at, uint32_t pos, uint32_t sec_end, int w, uint32_t& hl, uint32_t& m,
                             uint64_t& count, uint32_t& val, uint32_t& next);

__device__ int slow_header(rsrc_t rs, uint32_t pos, uint32_t sec_end, int w, uint32_t& hl, uint32_t& m, uint64_t& count,
                           uint32_t& val, uint32_t& next) {
  return slow_header_g([&](uint32_t p) { return sbyte(rs, p); }, pos, sec_end, w, hl, m, count, val, next);
}

template <class ByteAt>
__device__ int slow_header_g(ByteAt sbyte_at, uint32_t pos, uint32_t sec_end, int w, uint32_t& hl, uint32_t& m,
                             uint64_t& count, uint32_t& val, uint32_t& next) {
  uint32_t value = 0, i = 0, k = 0, bb;
  for (;;) {
    if (pos + k >= sec_end) return PQG_ERR_EOF;
    bb = sbyte_at(pos + k);
    if (!(bb & 0x80u)) break;
    value |= (bb & 0x7Fu) << (i & 31u);
    i += 7;
    k++;
  }
  const uint32_t header = value | (bb << (i & 31u));
  hl = k + 1;
  if ((header & 1u) == 0) {
    const uint32_t nb = ((uint32_t)w + 7u) >> 3;
    if ((uint64_t)pos + hl + nb > sec_end) return PQG_ERR_EOF;
    uint32_t v = 0;
    for (uint32_t j = 0; j < nb; j++) v |= sbyte_at(pos + hl + j) << (8u * j);
    m = 0;
    count = header >> 1;
    val = v;
    next = pos + hl + nb;
    return 0;
  }
  const uint32_t groups = header >> 1;
  if (groups == 0) return PQG_ERR_EMPTY_PACKED_RUN;
  if (groups >= (1u << 28)) return PQG_ERR_CORRUPT;
  m = 1;
  count = (uint64_t)groups * 8u;
  val = pos + hl;
  const uint64_t e = (uint64_t)pos + hl + (uint64_t)groups * (uint32_t)w;
  next = e > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)e;
  return 0;
}

__device__ __forceinline__ uint32_t wbyte(const PreWin& pw, uint32_t p) {
  if (seg_has(pw, p & ~3u, 4)) return uni((seg32(pw, p & ~3u) >> ((p & 3u) * 8u)) & 0xFFu);
  return sbyte(pw.rs, p);
}

__device__ __forceinline__ uint32_t pick4(const uint32_t (&a)[4], uint32_t b, uint32_t l) {
  switch (b) {
    case 0: return rdl(a[0], l);
    case 1: return rdl(a[1], l);
    case 2: return rdl(a[2], l);
    default: return rdl(a[3], l);
  }
}

// Value of element i (page-relative) of a PACKED run [lo, hi) starting at s_r.
__device__ __forceinline__ uint32_t packed_elem(rsrc_t rs, uint32_t lo, uint32_t hi, uint32_t s_r, uint32_t i, int w) {
  if (w == 0) return 0;
  uint64_t bit = (uint64_t)(i - s_r) * (uint32_t)w;
  uint32_t byte = lo + (uint32_t)(bit >> 3);
  uint32_t a = byte & ~3u;
  uint64_t x = (uint64_t)ld32(rs, a) | ((uint64_t)ld32(rs, a + 4) << 32);
  if (a + 8u > hi) {  // truncated final group: bytes past what readFully got are 0 (:96-99)
    int64_t keep = (int64_t)hi - (int64_t)a;
    x = keep <= 0 ? 0 : (x & ((1ull << (8 * keep)) - 1ull));
  }
  x >>= (byte - a) * 8u + (uint32_t)(bit & 7u);
  return w == 32 ? (uint32_t)x : (uint32_t)x & ((1u << w) - 1u);
}

// ---------------------------------------------------------------------------
// Dictionary pages (DictionaryValuesReader): W = 4 or 8 byte values.

template <int W>
struct DictVal;
template <>
struct DictVal<8> {
  typedef uint64_t T;
};
template <>
struct DictVal<4> {
  typedef uint32_t T;
};

template <int W>
__device__ __forceinline__ typename DictVal<W>::T load_dict(rsrc_t d, uint32_t id) {
  if constexpr (W == 8) return ld8_any(d, id * 8u);
  else return ld4_any(d, id * 4u);
}

constexpr uint32_t DICT_LDS_BYTES = 8192;   // dictionary staged in LDS per workgroup when it fits

// Per-wave LDS of k_dict.
struct DictWaveLds {
  uint8_t seg[SEG_BYTES];  // page bytes [seg_lo, seg_lo + SEG_BYTES)
  uint64_t ent[256];       // window position k: next header position | (count | packed << 31) << 32
  uint32_t val[256];       // window position k: RLE raw value, or packed data start
};

// ---------------------------------------------------------------------------
// Dictionary pages in two launches.
//
//   k_dict_runs    one wave per page: follows the run headers of the page's data
//                  section and writes one 8-byte record per run (first value index,
//                  payload: raw RLE id, or 0x80000000 | packed data position), plus,
//                  per output chunk, the record holding the chunk's first value.
//                  No dictionary access, no value stores: latency-bound LDS work.
//   k_dict_expand  one wave per output chunk (CH_TILES x 64 lanes x 16 bytes), a
//                  persistent grid over all chunks of all pages, so the expansion
//                  is balanced regardless of how runs are spread over pages. All
//                  loads of a chunk (records, packed bytes, dictionary) come before
//                  its stores: on CDNA vmcnt counts stores, and a load issued after
//                  stores would wait for all of them.
constexpr uint32_t CH_TILES = DICT_CHUNK_TILES;

__device__ __forceinline__ uint32_t chunk_values(uint32_t E) { return CH_TILES * WAVE * E; }

// Walk -> expansion hand-off inside one launch (walkers and expansion waves on any CU / XCD).
//
// Every datum handed off — run records, chunk -> record entries, page status, page flag — is
// written and read ONLY with system-scope atomics (sst / sld: global_store / global_load with
// sc0 sc1). On gfx950 those bypass the non-coherent per-XCD L2 (stores write through, loads
// miss), so no cache write-back or invalidate is needed for them; what the hand-off needs is
// ORDER:
//   release (walker): the wave's record stores are complete before the status store, and the
//     status before the flag — s_waitcnt vmcnt(0) (stores count in vmcnt; the wait returns once
//     the write-through stores are acknowledged), plus a compiler barrier so no store is moved
//     across it;
//   acquire (expansion): the status / record loads are issued after the flag load returned the
//     epoch — the flag value feeds the loop's scalar branch, so its load has completed (vmcnt)
//     before any later load issues; a compiler barrier keeps those loads below the branch.
// This is the "{sc0 sc1 stores and loads both sides}" hand-off of MI355X_MICROARCH.md
// (inter-workgroup visibility: every handed-off byte stored sc1 and loaded sc1, every storing wave's
// vmcnt(0) before its flag, the polling wave loads only after its poll matched), which needs no
// agent-scope fence. The memory model's fences (buffer_wbl2 sc1 on release, buffer_inv sc1 on
// acquire) write back / invalidate the caches for the expansion's own traffic too; measured on C2
// (tried in round 2: a release store 1.30x the time, an acquire fence 2.45x, both 2.8x;
// profiles/r02/r02_b/ab).
// Variants measured and removed (git history, profiles/r02): an early partial hand-off after the
// walker's first window (C2 181.5 vs 172.6 us per launch, profiles/r02/early_ab: the extra wait on
// the walker's stores costs more than the early chunks gain); the mark-word chain of the window walk
// (the list walk dict_walk_ls replaced it); two chain steps per iteration through a
// successor-of-successor table, a branch-free 4-byte header parse, and the chain on the vector unit
// (ds_bpermute per run): all within +-1 % (profiles/r02/walk_ls/variants, vchain).
__device__ __forceinline__ void handoff_release() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a compiler barrier too (invisible to the waitcnt pass)
}
__device__ __forceinline__ void handoff_acquire() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Saturating inclusive scan over the wave: lane l gets min(v_0 + ... + v_l, cap) (every v <= cap <
// 2^31). DPP row shifts and row broadcasts, no LDS round trip; call with all 64 lanes active.
__device__ __forceinline__ uint32_t wave_incl_scan_sat(uint32_t x, uint32_t cap) {
#define PQG_DPP_SAT(ctrl, rmask)                                                                \
  {                                                                                             \
    const uint32_t y_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rmask, 0xf, true); \
    x = x + y_ < cap ? x + y_ : cap;                                                            \
  }
  PQG_DPP_SAT(0x111, 0xf)  // row_shr:1
  PQG_DPP_SAT(0x112, 0xf)  // row_shr:2
  PQG_DPP_SAT(0x114, 0xf)  // row_shr:4
  PQG_DPP_SAT(0x118, 0xf)  // row_shr:8
  PQG_DPP_SAT(0x142, 0xa)  // row_bcast:15 -> rows 1, 3
  PQG_DPP_SAT(0x143, 0xc)  // row_bcast:31 -> rows 2, 3
#undef PQG_DPP_SAT
  return x;
}

// List walk: the same windows and pre-decode as dict_walk_pj, with the window's chain and its
// records built without per-position masks.
//   chain    the successors of a lane's 4 positions are packed into one dword (byte b: window
//            offset of the successor of position 4 * lane + b, 0 = the chain stops there — a
//            successor is always past its header, so 0 is free); each step is one v_readlane, a
//            byte extract and one lane select that appends the position to a list VGPR (lane t =
//            t-th header of the batch): one loop branch per run, no per-position mark words.
//   records  lane t reads its header's count / payload from an LDS table (one 8-byte entry per
//            window position), a saturating DPP scan gives the first values, and lane t stores
//            record k + t: one store per run instead of a ballot compaction over 256 positions.
// A window with more than 64 headers on its chain is taken in several batches.
// Semantics are those of dict_walk_pj (readNext :80-109, the scalar slow path for long varints,
// 0 / huge group counts and headers crossing the section end).
template <int W, bool SMALL = true>
__device__ __forceinline__ void dict_walk_ls(DictWaveLds& L, PreWin& win, uint32_t N, uint32_t sec_beg,
                                             uint32_t sec_end, int w, uint64_t* rec, uint32_t* chunk_run,
                                             uint32_t CH, uint32_t sh, int page, uint64_t* err, ErrCount err_count,
                                             uint32_t& n_rec, uint32_t& n_ok) {
  typedef uint64_t __attribute__((may_alias)) u64a;
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  typedef u64x2 __attribute__((may_alias)) u64x2a;
  const uint32_t lane = lane_id();
  uint32_t pos = sec_beg + 1;  // RunLengthBitPackingHybridDecoder stream position
  uint32_t produced = 0, k = 0;
  int code = 0;
#ifdef PQG_DIAG
  uint64_t dg_pre = 0, dg_chain = 0, dg_emit = 0, dg_win = 0, dg_bat = 0;
  struct DgOut {
    uint64_t *a, *b, *c, *d, *e;
    uint32_t* k;
    int page;
    __device__ ~DgOut() {
      if (pqg_diag_wph && lane_id() == 0) {
        uint64_t* o = pqg_diag_wph + 8 * (uint64_t)page;
        o[0] = *a; o[1] = *b; o[2] = *c; o[3] = *d; o[4] = *e; o[5] = *k;
      }
    }
  } dg_out{&dg_pre, &dg_chain, &dg_emit, &dg_win, &dg_bat, &k, page};
#endif
  auto put_record = [&](uint32_t start, uint32_t end, uint32_t payload) {
    if (lane == 0) {
      sst(rec + k, (uint64_t)start | ((uint64_t)payload << 32));
      uint32_t j = start == 0 ? 0 : (start + sh + CH - 1) / CH;
      for (; j * CH < end + sh; j++) sst(chunk_run + j, k);
    }
    k++;
  };
  while (true) {
    pos = uni(pos);
    produced = uni(produced);
    k = uni(k);
    if (produced >= N) break;
    if (pos >= sec_end) { code = PQG_ERR_RLE_PAST_END; break; }  // readNext :81
    // A bit-packed run of at least 32 data bytes is taken on the scalar unit, without pre-decoding a
    // 256-byte window that holds at most eight headers (few-entry dictionaries of random ids — C4's
    // flag and mode columns, runs of 504 values at w = 1..3 — have one or two per window). The header
    // test reads one byte; an RLE header (C2's usual one) goes straight to the window.
    {
      if (!SMALL && !seg_has(win, pos & ~3u, 8u)) seg_fill(win, pos & ~15u);
      const uint32_t b0 = uni((seg32(win, pos & ~3u) >> ((pos & 3u) * 8u)) & 0xFFu);
      if (b0 & 1u) {
        uint32_t hl, m, nxs, vv;
        uint64_t cnt64;
        const int c2 = slow_header_g([&](uint32_t p) { return wbyte(win, p); }, pos, sec_end, w, hl, m, cnt64, vv, nxs);
        if (c2 == 0 && m && (cnt64 >> 3) * (uint32_t)w >= 32u) {
          const uint32_t left = N - produced;
          const uint32_t take = cnt64 < left ? (uint32_t)cnt64 : left;
          put_record(produced, produced + take, 0x80000000u | vv);
          produced += take;
          pos = nxs < sec_end ? nxs : sec_end;  // readFully of what is left
          continue;
        }
      }
    }
    const uint32_t B = pos & ~3u;
    DIAG_T(dg_t0);
#ifdef PQG_DIAG
    dg_win++;
#endif
    predecode<SMALL, (bool)0>(win, B, w);
    uint32_t js = 0, nn[4], slowm = 0, inm = 0;
    uint64_t ent[4];
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) {
      const uint32_t p = B + 4u * lane + b;
      const uint32_t f = (win.flg >> (8u * b)) & 0xFFu;
      const uint32_t hl = f >> 2;
      const uint32_t nx = win.nxt[b];
      const bool in = p < sec_end;
      const bool slow = in && ((f & 2u) || p + hl > sec_end || (!(f & 1u) && nx > sec_end));
      nn[b] = (f & 1u) ? (nx < sec_end ? nx : sec_end) : nx;  // packed: readFully of what is left
      const uint32_t j = (!in || slow || nn[b] - B >= 256u) ? 0u : nn[b] - B;
      js |= j << (8u * b);
      slowm |= (slow ? 1u : 0u) << b;
      inm |= (in ? 1u : 0u) << b;
      ent[b] = (uint64_t)win.val[b] | ((uint64_t)(win.cnt[b] | ((f & 1u) << 31)) << 32);
    }
    wave_sync();  // the previous window's table reads are done
    ((u64x2a*)L.ent)[2u * lane] = u64x2{ent[0], ent[1]};
    ((u64x2a*)L.ent)[2u * lane + 1u] = u64x2{ent[2], ent[3]};
    wave_sync();
    DIAG_ADD(dg_pre, dg_t0);
    uint32_t q = pos - B, nq = 0;
    while (true) {  // batches of at most 64 chain positions
      uint32_t t = 0, lst = 0;
      DIAG_T(dg_t1);
#ifdef PQG_DIAG
      dg_bat++;
#endif
      while (true) {
        q = uni(q);
        lst = lane == t ? q : lst;  // v_cmp + v_cndmask
        nq = (rdl(js, q >> 2) >> ((q & 3u) << 3)) & 0xFFu;
        t++;
        if (nq == 0u || t == (uint32_t)WAVE) break;
        q = nq;
      }
      t = uni(t);
      nq = uni(nq);
      DIAG_ADD(dg_chain, dg_t1);
      DIAG_T(dg_t2);
      // the batch's last position q ends the chain here (nq == 0): a run only when it is a
      // fast-path header inside the section (otherwise the scalar path below takes it)
      const uint32_t ql = q >> 2, qb = q & 3u;
      const bool last_run = nq != 0u || (!((rdl(slowm, ql) >> qb) & 1u) && ((rdl(inm, ql) >> qb) & 1u));
      const uint32_t n_v = last_run ? t : t - 1u;
      const uint32_t cap = N - produced;
      uint32_t c = 0, payload = 0;
      if (lane < n_v) {
        const uint64_t e = ((const u64a*)L.ent)[lst];
        const uint32_t cw = (uint32_t)(e >> 32), vv = (uint32_t)e;
        const bool pk = cw >> 31;
        c = cw & 0x7FFFFFFFu;
        if (!pk && c == 0) c = cap;  // Java: currentCount goes negative, the value repeats forever
        c = c < cap ? c : cap;
        payload = pk ? (0x80000000u | vv) : (vv > 0x7FFFFFFFu ? 0x7FFFFFFFu : vv);
      }
      const uint32_t inc = wave_incl_scan_sat(c, cap);
      uint32_t st = __shfl_up(inc, 1);
      if (lane == 0) st = 0;
      const uint32_t total = uni(rdl(inc, WAVE - 1));
      // emitted: the runs that start before the cap (a prefix of the lanes)
      const bool em = c > 0u && st < cap;
      const uint32_t n_em = uni((uint32_t)__builtin_popcountll(__ballot(em)));
      if (em) {
        const uint32_t s_abs = produced + st;
        const uint32_t e_abs = produced + (st + c < cap ? st + c : cap);
        sst(rec + k + lane, (uint64_t)s_abs | ((uint64_t)payload << 32));
        uint32_t j = s_abs == 0 ? 0 : (s_abs + sh + CH - 1) / CH;
        for (; j * CH < e_abs + sh; j++) sst(chunk_run + j, k + lane);
      }
      k = uni(k + n_em);
      produced = uni(produced + total);
      DIAG_ADD(dg_emit, dg_t2);
      if (produced >= N || nq == 0u) break;
      q = nq;  // the chain goes on inside this window: next batch
    }
    if (produced >= N) break;
    // continue after the window's last chain position q
    const uint32_t ql = q >> 2, qb = q & 3u;
    const uint32_t q_slow = (rdl(slowm, ql) >> qb) & 1u;
    const uint32_t q_in = (rdl(inm, ql) >> qb) & 1u;
    if (!q_in) {
      pos = B + q;  // at or past the section end: RLE_PAST_END on the next iteration
    } else if (!q_slow) {
      pos = pick4(nn, qb, ql);  // leaves the window
    } else {
      // scalar re-decode of the header at q (readNext :80-109)
      pos = B + q;
      uint32_t hl, m, nxs, vv;
      uint64_t cnt64;
      code = SMALL ? slow_header_g([&](uint32_t p) { return uni((seg32(win, p & ~3u) >> ((p & 3u) * 8u)) & 0xFFu); },
                                   pos, sec_end, w, hl, m, cnt64, vv, nxs)
                   : slow_header_g([&](uint32_t p) { return wbyte(win, p); }, pos, sec_end, w, hl, m, cnt64, vv, nxs);
      if (code) break;
      if (m == 0 && nxs > sec_end) { code = PQG_ERR_EOF; break; }
      uint64_t cnt = cnt64;
      const uint32_t left = N - produced;
      if (m == 0 && cnt == 0) cnt = left;
      const uint32_t take = cnt < left ? (uint32_t)cnt : left;
      put_record(produced, produced + take, m ? (0x80000000u | vv) : (vv > 0x7FFFFFFFu ? 0x7FFFFFFFu : vv));
      produced += take;
      pos = m ? (nxs < sec_end ? nxs : sec_end) : nxs;
    }
  }
  if (code) {
    if (lane == 0) report(err, err_count, page, 2, produced, code);
    N = produced;
  }
  n_rec = k;
  n_ok = N;
}

// One wave per page (4 per workgroup): the run records of RLE_DICTIONARY / PLAIN_DICTIONARY
// pages (DictionaryValuesReader.initFromPage :48-64 + RunLengthBitPackingHybridDecoder.readNext
// :80-109). The page section is staged in LDS; a 256-byte window is pre-decoded in parallel
// (every lane parses a run header at each of its 4 byte positions) into LDS tables, and the
// serial chain is one ds_read_b64 + ds_read_b32 per run.
// One wave per page (4 per workgroup; `group` is the workgroup's index among the walkers).
template <int W>
__device__ __forceinline__ void dict_runs_body(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                               const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                               const int32_t* __restrict__ list, int n_list, uint64_t* rec,
                                               uint32_t* chunk_run, uint64_t* pstat, uint32_t* flags, uint32_t epoch,
                                               uint64_t* err, ErrCount err_count, uint8_t* lds, uint32_t group) {
  DictWaveLds& L = ((DictWaveLds*)lds)[wave_id()];
  const int i_page = (int)(group * WPB + wave_id());
  if (i_page >= n_list) return;
  const int page = list[i_page];
#ifdef PQG_DIAG
  const uint64_t rt_w0 = __builtin_amdgcn_s_memrealtime();
#endif
  const uint32_t lane = lane_id();
  const PageWork pw = work[page];
  const ColumnDev cd = cols[pw.column];
  uint32_t N = uni(pw.n_values);
  const uint32_t sec_beg = uni(pw.data_begin), sec_end = uni(pw.size);
  constexpr uint32_t E = 16u / W;
  const uint32_t CH = chunk_values(E);
  const uint32_t sh = (uint32_t)(pw.out_offset % (uint64_t)E);
  uint32_t n_rec = 0, n_ok = 0;
  (void)cd;
#ifdef PQG_DIAG
  uint64_t rt_w1 = 0, rt_w2 = 0;
#endif
  if (N > 0) {
    PreWin win;
    win.rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
    win.seg = L.seg;
    if (sec_beg >= sec_end) {
      // empty data section: every read throws "Attempt to read from empty page"
      if (lane == 0) report(err, err_count, page, 2 /*value*/, 0, PQG_ERR_EMPTY_PAGE);
    } else {
      seg_fill(win, sec_beg & ~15u);
      const uint32_t bw = wbyte(win, sec_beg);
#ifdef PQG_DIAG
      rt_w1 = __builtin_amdgcn_s_memrealtime() + (bw > 999u ? 1u : 0u);  // after the staging load
#endif
      if (bw > 32u) {  // RunLengthBitPackingHybridDecoder ctor :55 (thrown at initFromPage)
        if (lane == 0) report(err, err_count, page, 0 /*init*/, 2, PQG_ERR_BIT_WIDTH);
      } else {
        uint64_t* prec = rec + pw.rec_base;
        uint32_t* pcr = chunk_run + pw.chunk_base;
        // SMALL: the whole data section sits in the LDS segment: the walk has no global load
        if (sec_end - win.seg_lo + 264u <= SEG_BYTES)  // every window inside the segment
          dict_walk_ls<W>(L, win, N, sec_beg, sec_end, (int)bw, prec, pcr, CH, sh, page, err, err_count, n_rec, n_ok);
        else
          dict_walk_ls<W, false>(L, win, N, sec_beg, sec_end, (int)bw, prec, pcr, CH, sh, page, err, err_count, n_rec,
                                 n_ok);
      }
    }
  }
  // Publish (see handoff_release): every lane's record / chunk-entry stores, then lane 0's
  // status, then the flag.
#ifdef PQG_DIAG
  rt_w2 = __builtin_amdgcn_s_memrealtime() + (n_rec > 0xFFFFFFF0u ? 1u : 0u);
#endif
  wave_sync();
  handoff_release();
  if (lane == 0) {
    sst(pstat + page, (uint64_t)n_rec | ((uint64_t)n_ok << 32));
    handoff_release();
    sst(flags + page, epoch);
#ifdef PQG_DIAG
    if (pqg_diag_wrt) {
      pqg_diag_wrt[4 * page] = rt_w0;
      pqg_diag_wrt[4 * page + 1] = __builtin_amdgcn_s_memrealtime();
      pqg_diag_wrt[4 * page + 2] = rt_w1;
      pqg_diag_wrt[4 * page + 3] = rt_w2;
    }
#endif
  }
}

template <int W>
__global__ __launch_bounds__(64 * WPB) void k_dict_runs(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                        const PageWork* __restrict__ work,
                                                        const ColumnDev* __restrict__ cols,
                                                        const int32_t* __restrict__ list, int n_list, uint64_t* rec,
                                                        uint32_t* chunk_run, uint64_t* pstat, uint32_t* flags,
                                                        uint32_t epoch, uint64_t* err, ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) DictWaveLds wl_all[WPB];
  dict_runs_body<W>(bytes, n_bytes, work, cols, list, n_list, rec, chunk_run, pstat, flags, epoch, err, err_count,
                    (uint8_t*)wl_all, blockIdx.x);
}

template <int W>
__device__ __forceinline__ typename DictVal<W>::T dict_get_g(bool in_lds, const typename DictVal<W>::T* dict_l,
                                                             rsrc_t drs, uint32_t id) {
  return in_lds ? dict_l[id] : load_dict<W>(drs, id);
}

// One wave per output chunk (CH_TILES tiles of 64 lanes x 16 bytes, i.e. full 1 KB lines).
//
//   load phase  run records of the chunk -> LDS run table {start, payload, value}, RLE
//               values gathered from the dictionary, page bytes of the bit-packed runs ->
//               LDS. Vector loads happen only here, before the wave's first store (on CDNA
//               vmcnt counts stores: a load after stores would wait for all of them).
//   tile sweep  every lane tracks the run holding its element: per tile it advances past
//               the run starts it crossed (usually none), reads the value (RLE) or unpacks
//               the id and gathers (packed), and the wave stores one full 1 KB tile.
constexpr int SPIN_SLEEP = 2;  // s_sleep units (64 cycles) between two polls of a page's ready flag
constexpr uint32_t XT_RUNS = 128;  // run table entries per wave
constexpr uint32_t XT_SEG = 2560;    // LDS bytes for the packed data of one round

constexpr uint32_t XT_LDS_BYTES = DICT_LDS_BYTES + WPB * (XT_RUNS * 16 + XT_SEG);
#ifdef PQG_FAULT_INJECT
// Fault-injection build (tests/build/libpqgpu_faultinject.so, tests/test_gpu_timeout.py only; never
// the product): walker workgroup 0 of every fused launch starts PQG_FAULT_INJECT ticks late, past a
// spin timeout shortened to 0.1 s, so the expansions waiting for its pages time out.
constexpr uint64_t SPIN_TIMEOUT_TICKS = 10000000ull;
#else
constexpr uint64_t SPIN_TIMEOUT_TICKS = 200000000ull;  // 2 s of s_memrealtime (100 MHz)
#endif



// FUSED: launched in the same grid as the walkers (after them in workgroup order, so every
// walker this wave waits for was dispatched first); the page's records are ready once its
// flag holds this launch's epoch.
// IDS: the expansion writes the dictionary ids themselves (u32, into ColumnDev::blen) instead
// of dictionary values: BYTE_ARRAY / FIXED_LEN_BYTE_ARRAY / INT96 dictionaries, whose values
// are materialized by later kernels (k_bin_dict_map + k_bin_copy, k_gather_fixed).
// DD_SUMS (dictionary-direct BYTE_ARRAY columns, ColumnDev::dict_direct; IDS, W = 4): the expansion
// stores the ids compactly (ColumnDev::blen as u8 ids for dict_direct 1, u16 for 2: a quarter / half of
// the u32 id traffic) and the chunk's value bytes, the sum of its ids' entry lengths, to dd[chunk].
// Slots of a page past a walk error (pstat's value count) are left to k_dd_str (empty values).
// DD_IDS (dictionary-direct columns whose dictionary is too large to stage, ColumnDev::dd_global): the
// compact u16 ids only; the chunk sums come from k_dd_gsums, which gathers the entry lengths from HBM.
constexpr int DD_NONE = 0, DD_SUMS = 1, DD_IDS = 2;
constexpr uint32_t DD_ENT_MAX = 2048; // entries of a dictionary page of at most DD_DICT_MAX bytes (4-byte lengths)

// Inclusive prefix sum over the wave (u32) with DPP row shifts / broadcasts; all 64 lanes active.
__device__ __forceinline__ uint32_t wave_incl_scan_u32_dpp(uint32_t x) {
#define PQG_DPP_ADD(ctrl, rmask) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rmask, 0xf, true);
  PQG_DPP_ADD(0x111, 0xf)  // row_shr:1
  PQG_DPP_ADD(0x112, 0xf)  // row_shr:2
  PQG_DPP_ADD(0x114, 0xf)  // row_shr:4
  PQG_DPP_ADD(0x118, 0xf)  // row_shr:8
  PQG_DPP_ADD(0x142, 0xa)  // row_bcast:15 -> rows 1, 3
  PQG_DPP_ADD(0x143, 0xc)  // row_bcast:31 -> rows 2, 3
#undef PQG_DPP_ADD
  return x;
}

template <int W, bool FUSED, bool IDS = false, int DD = DD_NONE>
__device__ __forceinline__ void dict_tiles_body(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                const uint64_t* rec, const uint32_t* chunk_run,
                                                const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                const uint64_t* pstat, const uint32_t* flags, uint32_t epoch,
                                                uint64_t* err, ErrCount err_count, uint8_t* lds, uint32_t group,
                                                uint64_t* dd = nullptr) {
  typedef typename DictVal<W>::T T;
  static_assert(DD == DD_NONE || (IDS && W == 4), "dictionary-direct modes take the ids of a 4-byte expansion");
  constexpr uint32_t E = 16 / W;
  constexpr uint32_t TV = WAVE * E;  // values per tile
  constexpr uint32_t CH = CH_TILES * TV;
  uint8_t* dict_lds = lds;
  u32x4* tab = (u32x4*)(lds + DICT_LDS_BYTES) + wave_id() * XT_RUNS;
  uint8_t* xseg = lds + DICT_LDS_BYTES + WPB * XT_RUNS * 16 + wave_id() * XT_SEG;
  const uint32_t lane = lane_id();
  const uint32_t c = group * WPB + wave_id();
  // (a chunk list entry of page 0xFFFFFFFF is padding: the host aligns each dictionary-direct column's
  // chunks to whole workgroups, so a workgroup's waves share one dictionary)
  const int page = c < n_chunks ? (int)(uint32_t)chunks[c] : -1;
  // the workgroup's dictionary in LDS when its chunks share one that fits
  int* wg_col = (int*)dict_lds;
  if (lane == 0) wg_col[wave_id()] = page >= 0 ? work[page].column : -1;
  __syncthreads();
  int c0 = -1;
  bool same = true;
#pragma unroll
  for (int q = 0; q < WPB; q++) {
    const int cq = wg_col[q];
    if (cq >= 0) {
      if (c0 < 0) c0 = cq;
      else if (cq != c0) same = false;
    }
  }
  __syncthreads();
  bool dict_in_lds = false;
  uint32_t need = 0;
  // the dictionary is loaded into registers first and written to LDS after this wave's hand-off
  // loads, so its latency overlaps the first flag poll instead of preceding it
  u32x4 dreg[DICT_LDS_BYTES / (16u * 64u * WPB)] = {};
  if (!IDS && same && c0 >= 0) {
    const ColumnDev& cd0 = cols[c0];
    need = (uint32_t)((uint64_t)cd0.dict_n * W <= DICT_LDS_BYTES ? (uint64_t)cd0.dict_n * W : DICT_LDS_BYTES + 1u);
    dict_in_lds = need <= DICT_LDS_BYTES && need <= cd0.dict_bytes;
    if (dict_in_lds) {
      rsrc_t d0 = make_rsrc(bytes + cd0.dict_offset, cd0.dict_bytes);
#pragma unroll
      for (uint32_t r = 0; r < DICT_LDS_BYTES / (16u * 64u * WPB); r++) {
        const uint32_t o = 16u * threadIdx.x + r * 16u * 64u * WPB;
        if (o < need)  // any byte alignment; the piece at the buffer's end dword by dword
          dreg[r] = o + 16u <= cd0.dict_bytes
                        ? __builtin_amdgcn_raw_buffer_load_b128(d0, (int)o, 0, 0)
                        : u32x4{ld4_any(d0, o), ld4_any(d0, o + 4), ld4_any(d0, o + 8), ld4_any(d0, o + 12)};
      }
    }
  }
  const T* dict_l = (const T*)dict_lds;
  // ---- this wave's chunk, part 1: page facts and the hand-off (before the workgroup barrier)
  bool go = false;
  int cpage = -1;
  uint32_t j = 0, dict_n = 0, sec_end = 0, db = 0, N = 0, sh = 0, v_lo = 0, v_hi = 0, n_rec = 0, k = 0;
  uint32_t pre_lo = 0xFFFFFFFFu, pre_hi = 0;  // section bytes staged in xseg ahead of the records
  int w = 0;
  uint64_t pf0 = 0, pf1 = 0;  // records [0, 128) of the page (lane l: l and 64 + l)
  PageWork pw{};
  rsrc_t drs = make_rsrc(bytes, 0), prs = drs;
#ifdef PQG_DIAG
  const uint64_t rt_x0 = __builtin_amdgcn_s_memrealtime();
  uint64_t rt_x1 = 0;
  struct XStamp {
    uint64_t t0, *t1;
    uint32_t c;
    bool on;
    __device__ ~XStamp() {
      if (on && pqg_diag_xrt && lane_id() == 0) {
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        pqg_diag_xrt[4 * (uint64_t)c] = t0;
        pqg_diag_xrt[4 * (uint64_t)c + 1] = *t1;
        pqg_diag_xrt[4 * (uint64_t)c + 2] = __builtin_amdgcn_s_memrealtime();
        pqg_diag_xrt[4 * (uint64_t)c + 3] = (uint64_t)hw;
      }
    }
  } xstamp{rt_x0, &rt_x1, c, c < n_chunks};
#endif
  uint32_t NF = 0;  // DD: the page's values (pstat's N stops at a walk error)
  if (page >= 0) {
    cpage = page;
    j = (uint32_t)(chunks[c] >> 32);
    // page / column facts and the page's bit width do not depend on the walk: loaded before the
    // hand-off, so the compiler barrier there does not serialize them behind the flag
    pw = work[cpage];
    const ColumnDev& cd = cols[pw.column];
    dict_n = uni(cd.dict_n);
    drs = make_rsrc(bytes + cd.dict_offset, cd.dict_bytes);
    prs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
    sec_end = uni(pw.size);
    db = uni(pw.data_begin);
    w = (int)uni((ld32(prs, db & ~3u) >> ((db & 3u) * 8u)) & 0xFFu);
    // a data section that fits xseg is staged whole now (input bytes: no hand-off needed), so the
    // packed bytes of its runs need no load after the records
    if (sec_end > db && sec_end + 8u - (db & ~15u) <= XT_SEG) {
      pre_lo = db & ~15u;
      pre_hi = sec_end + 8u;
#pragma unroll
      for (uint32_t i = 0; i < XT_SEG; i += 16u * WAVE) {
        const uint32_t o = i + 16u * lane;
        if (o < pre_hi - pre_lo) *(u32x4*)(xseg + o) = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(pre_lo + o), 0, 0);
      }
      // bytes past the section read as 0 (the truncated final group, :96-99): zeroed once here, so
      // the tile sweep's unpack needs no per-value check
      if (lane < 8u) xseg[sec_end - pre_lo + lane] = 0;
    }
    uint64_t pst = 0;
    bool ok = true;
    if (FUSED) {
      // The flag is polled; once it holds this launch's epoch, handoff_acquire orders the status /
      // record / chunk-entry loads below after it (once per chunk, not per poll).
      uint64_t t_wait = 0;
      while (true) {
        if (uni(sld(flags + cpage)) == epoch) {
          handoff_acquire();
#ifdef PQG_DIAG
          rt_x1 = __builtin_amdgcn_s_memrealtime();
#endif
          break;
        }
        __builtin_amdgcn_s_sleep(SPIN_SLEEP);
        // wall-clock bound (s_memrealtime: constant 100 MHz): a walker that never publishes
        // (descheduled, starved) turns into PQG_ERR_TIMEOUT after SPIN_TIMEOUT_TICKS, not a hang
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t_wait == 0) t_wait = now;
        else if (now - t_wait > SPIN_TIMEOUT_TICKS) {
          if (lane == 0) report(err, err_count, cpage, 2, 0, PQG_ERR_TIMEOUT);
          ok = false;
          break;
        }
      }
    }
    if (ok) {
      // the page status and the chunk's first run in one round trip
      pst = sld(pstat + cpage);
      k = sld(chunk_run + pw.chunk_base + j);
      {  // the page's first 2 x 64 run records in the same round trip
        pf0 = sld(rec + pw.rec_base + lane);
        pf1 = sld(rec + pw.rec_base + WAVE + lane);
      }
      pst = uni64(pst);
      k = uni(k);
      N = (uint32_t)(pst >> 32);  // values covered before a walk error
      NF = DD != DD_NONE ? uni(pw.n_values) : N;
      sh = (uint32_t)(pw.out_offset % (uint64_t)E);
      const uint32_t s_lo = j * CH > sh ? j * CH : sh;
      const uint32_t s_hi = (j + 1) * CH < NF + sh ? (j + 1) * CH : NF + sh;
      go = s_lo < s_hi;
      v_lo = s_lo - sh;
      v_hi = s_hi - sh;
      n_rec = (uint32_t)pst;
    }
  }
  if (dict_in_lds) {
#pragma unroll
    for (uint32_t r = 0; r < DICT_LDS_BYTES / (16u * 64u * WPB); r++) {
      const uint32_t o = 16u * threadIdx.x + r * 16u * 64u * WPB;
      if (o < need) *(u32x4*)(dict_lds + o) = dreg[r];
    }
  }
  // DD_SUMS: the entry lengths
  if constexpr (DD == DD_SUMS) {
    if (same && c0 >= 0) {
      const ColumnDev& cd0 = cols[c0];
      const uint32_t dn = uni(cd0.dict_n);
      dict_in_lds = dn <= DD_ENT_MAX && cd0.dict_bytes <= DD_DICT_MAX;
      if (dict_in_lds) {
        uint32_t* ent = (uint32_t*)dict_lds;
        for (uint32_t i = threadIdx.x; i < dn; i += 64u * WPB) ent[i] = cd0.dict_len[i];
      }
    }
  }
  __syncthreads();
  // ---- part 2: the chunk's run tables and tile sweeps
  auto one_chunk = [&]() {
    const int page = cpage;
    const ColumnDev& cd = cols[pw.column];
    T* const out_base = IDS ? (T*)cd.blen : (T*)cd.values;
    const bool own_dict = dict_in_lds && pw.column == c0;
    const uint64_t* prec = rec + pw.rec_base;
    T* const pag = out_base + (pw.out_offset - sh);  // slot 0 of the page
    const bool out16 = ((uintptr_t)out_base & 15u) == 0;
    const uint32_t wmask = w == 32 ? 0xFFFFFFFFu : (1u << w) - 1u;
    // the walked part of the chunk (DD: slots past a walk error follow as empty values)
    const uint32_t r_hi = DD != DD_NONE ? (v_hi < N ? v_hi : N) : v_hi;
    // DD_SUMS: the lane's byte sum, the column's compact ids (slot 0 of the page), their width
    uint32_t dd_acc = 0;
    const uint32_t* ent_l = (const uint32_t*)dict_lds;
    uint8_t* const idpag = (uint8_t*)cd.blen + (pw.out_offset - sh) * (uint64_t)cd.dict_direct;
    // DD: length of id's entry, 0 past the dictionary. Always from LDS: the plan gives a dictionary-direct
    // column whole workgroups and dictionaries that fit (a global load in the tile loop would make every
    // later wait a vmcnt(0), draining the stores)
    auto dd_entry = [&](uint32_t id) -> uint32_t { return id < dict_n ? ent_l[id] : 0u; };

    uint32_t b_lo = v_lo;
    while (v_lo < r_hi) {
      k = uni(k);
      b_lo = uni(b_lo);
      // ---- load phase: runs k .. k + n_tab - 1 into the table (entry n_tab: end sentinel)
      uint32_t n_tab = 0, b_hi = r_hi, px_lo = 0xFFFFFFFFu, px_hi = 0;
      for (uint32_t t0 = 0; t0 < XT_RUNS; t0 += WAVE) {
        const uint32_t r = k + t0 + lane;
        const bool has = r < n_rec && t0 + lane < XT_RUNS - 1;  // a run of this round
        // records the hand-off prefetched come from the lanes holding them
        const int src = (int)(r & (WAVE - 1u));
        const uint64_t a0 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(pf0 >> 32), src) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)pf0, src);
        const uint64_t a1 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(pf1 >> 32), src) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)pf1, src);
        const uint64_t rr = r >= n_rec ? 0 : (r < WAVE ? a0 : (r < 2u * WAVE ? a1 : sld(prec + r)));
        const uint32_t st = r < n_rec ? (uint32_t)rr : N;        // (past the runs: end sentinel)
        const uint32_t pl = (uint32_t)(rr >> 32);
        const uint32_t q63 = k + t0 + WAVE;
        const uint32_t nx63 = uni(q63 >= n_rec ? N
                                  : (q63 < 2u * WAVE
                                         ? rdl((uint32_t)(q63 < WAVE ? pf0 : pf1), q63 & (WAVE - 1u))
                                         : (uint32_t)sld(prec + q63)));
        const uint32_t en_n = __shfl_down(st, 1);
        const uint32_t en = lane == WAVE - 1 ? nx63 : en_n;  // end of this lane's run
        const bool live = has && st < r_hi;
        uint32_t vlo = 0, vhi = 0;
        if (live && !(pl & 0x80000000u)) {
          if (pl < dict_n) {
            if constexpr (IDS) {
              vlo = pl;
            } else {
              const uint64_t x = (uint64_t)(own_dict ? dict_l[pl] : load_dict<W>(drs, pl));
              vlo = (uint32_t)x;
              vhi = (uint32_t)(x >> 32);
            }
          }
        }
        tab[t0 + lane] = u32x4{st, pl, vlo, vhi};
        // packed bytes needed by this round: [first packed byte, last packed byte + 8)
        if (live && (pl & 0x80000000u)) {
          const uint32_t e_run = en;
          const uint32_t lo = (pl & 0x7FFFFFFFu) + (uint32_t)(((uint64_t)((st > b_lo ? st : b_lo) - st) * (uint32_t)w) >> 3);
          const uint32_t hi_v = (e_run < r_hi ? e_run : r_hi);
          const uint32_t hi = (pl & 0x7FFFFFFFu) + (uint32_t)(((uint64_t)(hi_v > st ? hi_v - st : 0) * (uint32_t)w + 7) >> 3) + 8u;
          px_lo = lo < px_lo ? lo : px_lo;
          px_hi = hi > px_hi ? hi : px_hi;
        }
        const uint64_t inb = __ballot(has && st < r_hi);
        n_tab += (uint32_t)__builtin_popcountll(inb);
        if (!(inb >> 63)) break;  // this batch ends the round
      }
      n_tab = uni(n_tab);
      // wave min / max of the packed byte range
  #pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t a = __shfl_xor(px_lo, o), b = __shfl_xor(px_hi, o);
        px_lo = a < px_lo ? a : px_lo;
        px_hi = b > px_hi ? b : px_hi;
      }
      px_lo = uni(px_lo) & ~15u;
      px_hi = uni(px_hi);
      // round end: the start of the first run not in the table
      if (n_tab >= XT_RUNS - 1) {
        const u32x4 q = tab[XT_RUNS - 1];
        b_hi = uni(q.x) < r_hi ? uni(q.x) : r_hi;
      }
      bool x_lds = true;
      if (px_hi > px_lo && px_lo >= pre_lo && px_hi <= pre_hi) {
        px_lo = pre_lo;  // the section staged before the hand-off covers the round
      } else if (px_hi > px_lo) {
        pre_hi = 0;  // (xseg is overwritten)
        x_lds = px_hi - px_lo <= XT_SEG;
        if (x_lds) {
  #pragma unroll
          for (uint32_t i = 0; i < XT_SEG; i += 16u * WAVE) {
            const uint32_t o = i + 16u * lane;
            if (o < px_hi - px_lo) *(u32x4*)(xseg + o) = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(px_lo + o), 0, 0);
          }
          for (uint32_t o = (sec_end > px_lo ? sec_end - px_lo : 0u) + lane; o < px_hi - px_lo; o += WAVE) xseg[o] = 0;
        }
      }
      // DICT_ID: RLE runs of the round with an id past the dictionary (reported at the first
      // value of the run inside the chunk)
      for (uint32_t t0 = 0; t0 < n_tab; t0 += WAVE) {
        const u32x4 q = tab[t0 + lane];
        const uint32_t en = tab[t0 + lane + 1].x;
        if (t0 + lane < n_tab && !(q.y & 0x80000000u) && q.y >= dict_n && en > b_lo && q.x < b_hi)
          report(err, err_count, page, 2, q.x > b_lo ? q.x : b_lo, PQG_ERR_DICT_ID);
      }
      __builtin_amdgcn_s_waitcnt(0);  // load phase complete (the wave has not stored yet this round)

      // ---- tile sweep
      auto sweep = [&](auto fast_tag) {
        constexpr bool FAST = decltype(fast_tag)::value;
        auto value = [&](uint32_t ci, uint32_t i, const u32x4& q) -> T {
          if (!(q.y & 0x80000000u)) return (T)(((uint64_t)q.w << 32) | q.z);
          uint32_t id;
          if (FAST) {
            // staged bytes (zeroed past the section end), page value counts below 2^27: 32-bit bit
            // positions and one v_alignbit from the dword pair holding the id's first bit
            const uint32_t bit = (i - q.x) * (uint32_t)w;
            const uint32_t byte = (q.y & 0x7FFFFFFFu) + (bit >> 3);
            const uint32_t o = (byte & ~3u) - px_lo;
            id = __builtin_amdgcn_alignbit(*(const u32_alias*)(xseg + o + 4), *(const u32_alias*)(xseg + o),
                                           ((byte & 3u) << 3) + (bit & 7u)) & wmask;
          } else {
            const uint64_t bit = (uint64_t)(i - q.x) * (uint32_t)w;
            const uint32_t byte = (q.y & 0x7FFFFFFFu) + (uint32_t)(bit >> 3);
            const uint32_t a4 = byte & ~3u;
            uint64_t y = (uint64_t)ld32(prs, a4) | ((uint64_t)ld32(prs, a4 + 4) << 32);
            if (a4 + 8u > sec_end) {  // truncated final group: bytes past the section are 0 (:96-99)
              const int64_t keep = (int64_t)sec_end - (int64_t)a4;
              y = keep <= 0 ? 0 : (y & ((1ull << (8 * keep)) - 1ull));
            }
            y >>= (byte - a4) * 8u + (uint32_t)(bit & 7u);
            id = w == 0 ? 0u : (uint32_t)y & wmask;
          }
          if (id >= dict_n) {
            report(err, err_count, page, 2, i, PQG_ERR_DICT_ID);
            return 0;
          }
          if constexpr (IDS) return (T)id;
          else return FAST ? dict_l[id] : dict_get_g<W>(own_dict, dict_l, drs, id);
          (void)ci;
        };
        const uint32_t t_beg = (b_lo + sh) / TV, t_end = (b_hi + sh + TV - 1) / TV;  // page tiles
        // run of the lane's first element: binary search of the table
        uint32_t p0 = t_beg * TV + E * lane - sh;
        uint32_t pe = p0 < b_lo || p0 > 0x7FFFFFFFu ? b_lo : (p0 >= b_hi ? b_hi - 1 : p0);
        uint32_t ci = 0;
  #pragma unroll
        for (uint32_t step = XT_RUNS / 2; step >= 1; step >>= 1)
          if (ci + step < n_tab && tab[ci + step].x <= pe) ci += step;
        u32x4 cq = tab[ci];
        uint32_t ce = tab[ci + 1].x;
        const uint32_t lo_u = b_lo + sh, hi_u = b_hi + sh;  // the round's slot range
        for (uint32_t t = t_beg; t < t_end; t++) {
          t = uni(t);
          const uint32_t ts = t * TV;  // first slot of the tile
          p0 = ts + E * lane - sh;
          pe = p0 < b_lo || p0 > 0x7FFFFFFFu ? b_lo : (p0 >= b_hi ? b_hi - 1 : p0);
          while (pe >= ce) {  // crossed run starts (divergent, usually no lane)
            ci++;
            cq = tab[ci];
            ce = tab[ci + 1].x;
          }
          // elements outside [b_lo, b_hi) are not stored; they are evaluated at a clamped index
          T v[E];
          v[0] = value(ci, pe, cq);
  #pragma unroll
          for (uint32_t e = 1; e < E; e++) {
            const uint32_t x = p0 + e;  // value index of element e (wraps below 0)
            const uint32_t i = x < b_lo || x > 0x7FFFFFFFu ? b_lo : (x >= b_hi ? b_hi - 1 : x);
            if (i < ce) {
              v[e] = value(ci, i, cq);
            } else {  // the element starts a later run
              uint32_t cj = ci + 1;
              while (cj + 1 < n_tab && tab[cj + 1].x <= i) cj++;
              v[e] = value(cj, i, tab[cj]);
            }
          }
          if constexpr (DD != DD_NONE) {
            const bool whole = ts >= lo_u && ts + TV <= hi_u;
            uint8_t* ip = idpag + (uint64_t)(ts + E * lane) * cd.dict_direct;
            if (cd.dict_direct == 1u) {
              if (whole) gst((uint32_t*)ip, (v[0] & 0xFFu) | (v[1] & 0xFFu) << 8 | (v[2] & 0xFFu) << 16 | v[3] << 24);
            } else if (whole) {
              typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
              gst((u32x2*)ip, u32x2{(v[0] & 0xFFFFu) | v[1] << 16, (v[2] & 0xFFFFu) | v[3] << 16});
            }
  #pragma unroll
            for (uint32_t e = 0; e < E; e++) {
              const uint32_t sl = ts + E * lane + e;
              const bool in = sl >= lo_u && sl < hi_u;
              if constexpr (DD == DD_SUMS) dd_acc += in ? dd_entry((uint32_t)v[e]) : 0u;
              if (in && !whole) {
                if (cd.dict_direct == 1u) gst(ip + e, (uint8_t)v[e]);
                else gst((uint16_t*)ip + e, (uint16_t)v[e]);
              }
            }
          } else {
            T* tp = pag + ts + E * lane;
            if (out16 && ts >= lo_u && ts + TV <= hi_u) {
              if constexpr (W == 8) {
                typedef uint64_t v2 __attribute__((ext_vector_type(2)));
                gst_nt((v2*)tp, v2{v[0], v[1]});
              } else {
                gst_nt((u32x4*)tp, u32x4{v[0], v[1], v[2], v[3]});
              }
            } else {
  #pragma unroll
              for (uint32_t e = 0; e < E; e++)
                if (ts + E * lane + e >= lo_u && ts + E * lane + e < hi_u) gst(tp + e, v[e]);
            }
          }
        }
      };
      if ((IDS || own_dict) && x_lds && N < (1u << 27)) sweep(std::true_type{});
      else sweep(std::false_type{});
      if (b_hi >= r_hi) break;
      k += XT_RUNS - 1;
      b_lo = b_hi;
    }
    if constexpr (DD == DD_SUMS) {
      for (int o = 32; o >= 1; o >>= 1) dd_acc += __shfl_xor(dd_acc, o);
      if (lane == 0) gst(dd + c, (uint64_t)dd_acc);
    }
  };
  if (DD == DD_SUMS && go && !(dict_in_lds && pw.column == c0)) {
    // (never with the plan's layout: whole workgroups per column, dictionaries within DD_DICT_MAX / 2,048
    // entries)
    if (lane == 0) report(err, err_count, cpage, 2, v_lo, PQG_ERR_INVALID_ARG);
    go = false;
  }
  if (go) one_chunk();  // one chunk per wave
  else if (DD == DD_SUMS && page >= 0 && lane == 0) gst(dd + c, (uint64_t)0);
}

template <int W, bool IDS = false>
__global__ __launch_bounds__(64 * WPB) void k_dict_tiles(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                         const PageWork* __restrict__ work,
                                                         const ColumnDev* __restrict__ cols, const uint64_t* rec,
                                                         const uint32_t* chunk_run, const uint64_t* __restrict__ chunks,
                                                         uint32_t n_chunks, const uint64_t* pstat, uint64_t* err,
                                                         ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[XT_LDS_BYTES];
  dict_tiles_body<W, false, IDS>(bytes, n_bytes, work, cols, rec, chunk_run, chunks, n_chunks, pstat, nullptr, 0,
                                 err, err_count, lds, blockIdx.x);
}

// Walkers and tiles in one grid: workgroups [0, n_walk) walk pages, the rest expand chunks
// as soon as their page is published, so the expansion overlaps the walk.
template <int W, bool IDS = false>
__global__ __launch_bounds__(64 * WPB) void k_dict_fused(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                         const PageWork* __restrict__ work,
                                                         const ColumnDev* __restrict__ cols,
                                                         const int32_t* __restrict__ list, int n_list,
                                                         uint32_t n_walk, uint64_t* rec, uint32_t* chunk_run,
                                                         const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                         uint64_t* pstat, uint32_t* flags, uint32_t epoch,
                                                         uint64_t* err, ErrCount err_count) {
  constexpr uint32_t LB = sizeof(DictWaveLds) * WPB > XT_LDS_BYTES ? sizeof(DictWaveLds) * WPB : XT_LDS_BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LB];
  // workgroups [0, n_walk) walk (4 pages each), the rest expand (4 chunks each)
  if (blockIdx.x < n_walk) {
#ifdef PQG_FAULT_INJECT
    if (blockIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)PQG_FAULT_INJECT) __builtin_amdgcn_s_sleep(127);
    }
#endif
    dict_runs_body<W>(bytes, n_bytes, work, cols, list, n_list, rec, chunk_run, pstat, flags, epoch, err, err_count,
                      lds, blockIdx.x);
  } else {
    dict_tiles_body<W, true, IDS>(bytes, n_bytes, work, cols, rec, chunk_run, chunks, n_chunks, pstat, flags, epoch,
                                  err, err_count, lds, blockIdx.x - n_walk);
  }
}


// Dictionary-direct BYTE_ARRAY columns (ColumnDev::dict_direct: required, every data page
// dictionary-encoded, the dictionary page at most DD_DICT_MAX bytes): the ids are never stored.
//   k_dict_fused_dd  walkers + DD_SUMS expansion: per output chunk its compact ids and the bytes of its
//                    values (PlainBinaryDictionary entry lengths, PlainValuesDictionary.java:58-134)
//   k_dd_bases       per column: exclusive scan of its chunks' sums (chunks in page order) -> each chunk's
//                    first byte; the total -> bin_total and offsets[n_slots]
//   k_dd_str         per output chunk: the compact ids -> int64 offsets and the value bytes
// (DictionaryValuesReader.readBytes, DictionaryValuesReader.java:75-82, per value: the id's entry)
// DDM = DD_SUMS (dictionary staged in LDS) or DD_IDS (large dictionaries: ids only, k_dd_gsums sums)
template <int DDM>
__global__ __launch_bounds__(64 * WPB) void k_dict_fused_dd(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                            const PageWork* __restrict__ work,
                                                            const ColumnDev* __restrict__ cols,
                                                            const int32_t* __restrict__ list, int n_list,
                                                            uint32_t n_walk, uint64_t* rec, uint32_t* chunk_run,
                                                            const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                            uint64_t* pstat, uint32_t* flags, uint32_t epoch,
                                                            uint64_t* err, ErrCount err_count, uint64_t* sums) {
  constexpr uint32_t LB = sizeof(DictWaveLds) * WPB > XT_LDS_BYTES ? sizeof(DictWaveLds) * WPB : XT_LDS_BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LB];
  if (blockIdx.x < n_walk) {
#ifdef PQG_FAULT_INJECT
    if (blockIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)PQG_FAULT_INJECT) __builtin_amdgcn_s_sleep(127);
    }
#endif
    dict_runs_body<4>(bytes, n_bytes, work, cols, list, n_list, rec, chunk_run, pstat, flags, epoch, err, err_count,
                      lds, blockIdx.x);
  } else {
    dict_tiles_body<4, true, true, DDM>(bytes, n_bytes, work, cols, rec, chunk_run, chunks, n_chunks, pstat, flags,
                                        epoch, err, err_count, lds, blockIdx.x - n_walk, sums);
  }
}

// split mode (pqg_sync's re-run after a fused-kernel timeout): the DD_SUMS / DD_IDS expansion after the walk
template <int DDM>
__global__ __launch_bounds__(64 * WPB) void k_dict_tiles_dd(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                            const PageWork* __restrict__ work,
                                                            const ColumnDev* __restrict__ cols, const uint64_t* rec,
                                                            const uint32_t* chunk_run,
                                                            const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                            const uint64_t* pstat, uint64_t* err, ErrCount err_count,
                                                            uint64_t* sums) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[XT_LDS_BYTES];
  dict_tiles_body<4, false, true, DDM>(bytes, n_bytes, work, cols, rec, chunk_run, chunks, n_chunks, pstat,
                                       nullptr, 0, err, err_count, lds, blockIdx.x, sums);
}

// One workgroup per dictionary-direct column: its chunks are sums[start[2i] .. start[2i + 1]) in page order.
// Exclusive scan in one pass over the column: thread t takes DDB_PER consecutive sums per round (a
// register scan), a workgroup scan of the threads' totals, then each thread writes its bases. (The
// previous 256-sum rounds with two barriers each took 15 us for str_dict's 4,883 chunks.)
constexpr uint32_t DDB_PER = 16;
__global__ __launch_bounds__(256) void k_dd_bases(const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                  const uint64_t* __restrict__ chunks, const int32_t* __restrict__ dd_cols,
                                                  const int32_t* __restrict__ start, uint64_t* sums) {
  __shared__ uint64_t wsum[4];
  const ColumnDev& cd = cols[dd_cols[blockIdx.x]];
  const uint32_t b = (uint32_t)start[2 * blockIdx.x], e = (uint32_t)start[2 * blockIdx.x + 1];
  uint64_t carry = 0;
  for (uint32_t c0 = b; c0 < e; c0 += 256u * DDB_PER) {
    const uint32_t i0 = c0 + threadIdx.x * DDB_PER;
    uint64_t v[DDB_PER], own = 0;
#pragma unroll
    for (uint32_t j = 0; j < DDB_PER; j++) {
      v[j] = i0 + j < e ? sums[i0 + j] : 0;
      own += v[j];
    }
    uint64_t x = own;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o);
      if ((int)lane_id() >= o) x += y;
    }
    if (lane_id() == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t pre = carry + x - own, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
      pre += w < (threadIdx.x >> 6) ? wsum[w] : 0;
      tot += wsum[w];
    }
#pragma unroll
    for (uint32_t j = 0; j < DDB_PER; j++) {
      if (i0 + j < e) sums[i0 + j] = pre;
      pre += v[j];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *cd.bin_total = carry;
    // offsets[n]: n = the column's values = the end of its last page's (the last chunk's page: the host
    // pads before a column's first chunk, never after its last; slots for a required column, the non-null
    // count of a nullable one)
    uint64_t n = cd.n_slots;
    if (e > b) {
      const PageWork& lp = work[(uint32_t)chunks[e - 1]];
      n = lp.out_offset + lp.n_values;
    }
    gst((int64_t*)cd.values + n, (int64_t)carry);
  }
}

// Value bytes of the lane's E values (entry e: ln[e] bytes at LDS dd_lds + sr[e]), bytes [q0, q0 + 4 MD)
// of each: all MD dwords of every value and its tail dword are read first, then the stores (whole
// dwords, then a 2- and a 1-byte store for the last 1-3 bytes inside the range). Reads past an entry
// stay inside the workgroup's LDS or return 0; no store leaves the value's own bytes.
template <uint32_t MD>
__device__ __forceinline__ void dd_put(uint8_t* dst, const uint64_t (&o)[4], const uint32_t (&ln)[4],
                                       const uint32_t (&sr)[4], const uint8_t* dd_lds, uint32_t q0 = 0) {
  typedef uint32_t __attribute__((aligned(1), may_alias)) u32u;
  typedef uint32_t __attribute__((aligned(1), may_alias, address_space(1))) g32u;
  typedef uint16_t __attribute__((aligned(1), may_alias, address_space(1))) g16u;
  uint32_t x[4][MD], tl[4];
#pragma unroll
  for (uint32_t e = 0; e < 4; e++) {
#pragma unroll
    for (uint32_t k = 0; k < MD; k++) x[e][k] = *(const u32u*)(dd_lds + sr[e] + q0 + 4u * k);
    tl[e] = *(const u32u*)(dd_lds + sr[e] + (ln[e] & ~3u));
  }
#pragma unroll
  for (uint32_t e = 0; e < 4; e++) {
    uint8_t* ob = dst + o[e];
#pragma unroll
    for (uint32_t k = 0; k < MD; k++)
      if (q0 + 4u * k + 4u <= ln[e]) *(g32u*)(ob + q0 + 4u * k) = x[e][k];
    const uint32_t q = ln[e] & ~3u, r = ln[e] & 3u;
    if (r && q >= q0 && q < q0 + 4u * MD) {
      if (r & 2u) *(g16u*)(ob + q) = (uint16_t)tl[e];
      if (r & 1u) gst(ob + q + (r & 2u), (uint8_t)(tl[e] >> (8u * (r & 2u))));
    }
  }
}

// Block gather of k_dd_str (entries of 2 .. DDG_MD_MAX bytes): per tile, each wave writes its values'
// tile-relative starts and entries to LDS and, for every 16-byte output block, the value holding the
// block's first byte (each value marks the blocks whose first byte it holds); then every lane composes
// whole blocks from the staged dictionary page (a 16-byte unaligned LDS read per value piece, masked and
// shifted into the block) and stores them as one aligned 16-byte store: 64 KB of value bytes per 4,096
// store instructions, where storing each value's own bytes (dd_put) scattered dword / short / byte stores
// at lane strides (C4: 24.7 M store instructions per launch, the kernel's bound).
constexpr uint32_t DDG_MD_MAX = 32;
constexpr uint32_t DD_SPLIT_MAX_CHUNKS = 16384;  // k_dd_str: a workgroup per chunk up to this many chunks
constexpr uint32_t DDG_FV = (WAVE * 4u * DDG_MD_MAX) / 16u + 2u;
struct DdgLds {
  uint32_t vo[WAVE * 4];  // tile-relative first byte of value v
  uint32_t ve[WAVE * 4];  // entry: source << 16 | length (0: empty / out of range)
  uint16_t fv[DDG_FV];    // block b: the value holding its first byte
};
constexpr uint32_t DDG_WAVE_BYTES = (sizeof(DdgLds) + 15u) & ~15u;

// One wave per output chunk of k_dict_fused_dd (chunks of one column per workgroup: the plan pads the
// chunk list). The chunk's ids are loaded first, all of them (one dword per tile per lane for u8 ids,
// two for u16: no load after the first store, whose wait would drain the stores), then per 256-value
// tile: the entries from the staged table, a wave scan of the lanes' byte counts, the offsets as two
// 16-byte stores per lane, and each value's bytes from the staged dictionary page as unaligned dword
// stores plus a 2- and a 1-byte store for its last 1-3 bytes (no store leaves the value's own bytes).
// Slots of a page past a walk error (pstat) are empty values. dd_region: LDS bytes of the staged page
// (16-byte rounded) + its u32 entry table (source << 16 | length).
template <uint32_t TPW>
__global__ __launch_bounds__(64 * WPB) void k_dd_str(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                     const PageWork* __restrict__ work,
                                                     const ColumnDev* __restrict__ cols,
                                                     const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                     const uint64_t* pstat, const uint64_t* __restrict__ bases,
                                                     uint64_t* err, ErrCount err_count, uint32_t dd_region) {
  typedef uint32_t __attribute__((aligned(1), may_alias, address_space(1))) g32u;
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
  constexpr uint32_t E = 4, TV = WAVE * E, CH = CH_TILES * TV;
  // the staged dictionary page at dd_raw + 16 (16 bytes of slack before it for the block gather's reads)
  extern __shared__ __attribute__((aligned(16))) uint8_t dd_raw[];
  uint8_t* const dd_lds = dd_raw + 16;
  __shared__ int wg_col[WPB];
  // block gather: v_perm selectors taking bytes k .. 15 of a block from the source, the rest from the
  // accumulated block (dd_sel[k], dword d: byte j <- source when 4 d + j >= k)
  __shared__ u32x4 dd_sel[16];
  if (threadIdx.x < 64u) {
    const uint32_t k = threadIdx.x >> 2, d = threadIdx.x & 3u;
    uint32_t sel = 0;
#pragma unroll
    for (uint32_t jb = 0; jb < 4; jb++) sel |= (4u * d + jb >= k ? 4u + jb : jb) << (8u * jb);
    ((uint32_t*)dd_sel)[threadIdx.x] = sel;
  }
  const uint32_t lane = lane_id();
  // TPW = CH_TILES: one chunk per wave. TPW = CH_TILES / WPB: one workgroup per chunk, wave w takes tiles
  // [T0, T1) of it (4x the workgroups: str_dict's 4,883 chunks filled 1.2 rounds of the chip's workgroup
  // slots, the second one a fifth: 0.321 -> 0.274 ms; C4's 122 k chunks keep a chunk per wave, 10.50 vs
  // 10.63 ms; profiles/r05/dd_split)
  static_assert(TPW == CH_TILES || TPW * WPB == CH_TILES, "a chunk per wave or per workgroup");
  constexpr bool SPLIT = TPW < CH_TILES;
  const uint32_t c = SPLIT ? blockIdx.x : blockIdx.x * WPB + wave_id();
  const uint32_t T0 = SPLIT ? wave_id() * TPW : 0u, T1 = T0 + TPW;
  __shared__ uint32_t wsum[WPB];
  const int page = c < n_chunks ? (int)(uint32_t)chunks[c] : -1;
  if (lane == 0) wg_col[wave_id()] = page >= 0 ? work[page].column : -1;
  __syncthreads();
  int c0 = -1;
  bool same = true;
#pragma unroll
  for (int q = 0; q < WPB; q++) {
    const int cq = wg_col[q];
    if (cq >= 0) {
      if (c0 < 0) c0 = cq;
      else if (cq != c0) same = false;
    }
  }
  uint32_t ent_off = 0;
  bool staged = false;
  if (same && c0 >= 0) {  // the dictionary page, then the entry table
    const ColumnDev& cd0 = cols[c0];
    const uint32_t dn = uni(cd0.dict_n);
    ent_off = (uint32_t)((cd0.dict_bytes + 15u) & ~15ull);
    staged = dn <= DD_ENT_MAX && cd0.dict_bytes <= DD_DICT_MAX && ent_off + 4u * dn <= dd_region;
    if (staged) {
      uint32_t* ent = (uint32_t*)(dd_lds + ent_off);
      for (uint32_t i = threadIdx.x; i < dn; i += 64u * WPB) ent[i] = (cd0.dict_src[i] << 16) | cd0.dict_len[i];
      // (a resource over the rest of the batch: a 16-byte load crossing the end of its range would
      // return 0 as a whole; only entry bytes are ever read from the staged page)
      const rsrc_t d0 = make_rsrc(bytes + cd0.dict_offset, n_bytes - cd0.dict_offset);
      for (uint32_t o = 16u * threadIdx.x; o < ent_off; o += 16u * 64u * WPB)
        *(u32x4*)(dd_lds + o) = __builtin_amdgcn_raw_buffer_load_b128(d0, (int)o, 0, 0);
    }
  }
  __syncthreads();
  if (page < 0) return;
  const PageWork pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t j = (uint32_t)(chunks[c] >> 32);
  if (!staged || pw.column != c0) {
    // (never with the plan's layout: whole workgroups per column, dictionaries within DD_DICT_MAX /
    // 2,048 entries and within the launch's dd_region)
    if (lane == 0) report(err, err_count, page, 2, 0, PQG_ERR_INVALID_ARG);
    return;
  }
  const uint32_t dict_n = uni(cd.dict_n), idw = uni(cd.dict_direct);
  // longest entry (its bytes decide the store shapes below) and whether every entry is 1 byte long
  uint32_t md = 0, mn = 0xFFFFu;
  for (uint32_t i = lane; i < dict_n; i += WAVE) {
    const uint32_t l = ((const uint32_t*)(dd_lds + ent_off))[i] & 0xFFFFu;
    md = l > md ? l : md;
    mn = l < mn ? l : mn;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t a = (uint32_t)__shfl_xor((int)md, o), b = (uint32_t)__shfl_xor((int)mn, o);
    md = a > md ? a : md;
    mn = b < mn ? b : mn;
  }
  md = uni(md);
  const bool one = uni(mn) == 1u && md == 1u;
  const uint32_t NF = uni(pw.n_values);
  const uint32_t nok = uni((uint32_t)(sld(pstat + page) >> 32));  // values before a walk error
  const uint32_t sh = (uint32_t)(pw.out_offset % E);
  const uint32_t s_lo = j * CH > sh ? j * CH : sh;
  const uint32_t s_hi = (j + 1) * CH < NF + sh ? (j + 1) * CH : NF + sh;
  if (s_lo >= s_hi) return;
  const uint32_t ok_hi = (nok < NF ? nok : NF) + sh;  // slots [ok_hi, s_hi): empty values
  // the wave's ids: tile T0 + t -> lane's 4 ids (u8: dword t; u16: dwords 2t, 2t + 1)
  const uint8_t* idpag = (const uint8_t*)cd.blen + (pw.out_offset - sh) * (uint64_t)idw;
  uint32_t idr[2 * TPW];
#pragma unroll
  for (uint32_t t = 0; t < TPW; t++) {
    const uint32_t ts = j * CH + (T0 + t) * TV;
    const uint8_t* ip = idpag + (uint64_t)(ts + E * lane) * idw;
    const bool any = ts + E * lane < s_hi;  // (the id array is padded: the ids after a lane's first are readable)
    if (idw == 1u) {
      idr[2 * t] = any ? *(const __attribute__((address_space(1))) uint32_t*)ip : 0u;
      idr[2 * t + 1] = 0u;
    } else {
      const u32x2 x = any ? *(const __attribute__((address_space(1))) u32x2*)ip : u32x2{0u, 0u};
      idr[2 * t] = x.x;
      idr[2 * t + 1] = x.y;
    }
  }
  const uint32_t* ent = (const uint32_t*)(dd_lds + ent_off);
  uint8_t* const dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  int64_t* const opag = (int64_t*)cd.values + (pw.out_offset - sh);  // offsets of the page's slot 0
  const bool o16 = ((uintptr_t)cd.values & 15u) == 0;
  // block gather: entries of 2 .. DDG_MD_MAX bytes into a 16-byte aligned value buffer
  const bool gather = !one && md <= DDG_MD_MAX && ((uintptr_t)dst & 15u) == 0;
  DdgLds& G = *(DdgLds*)(dd_lds + ((dd_region + 15u) & ~15u) + wave_id() * DDG_WAVE_BYTES);
  // a tile's partial last block, finished by the next tile (uniform): bytes [cb_lo, cb_hi) of the block
  // at cb_tal; cx / cxlo: the carrying lane's copy
  bool cb_on = false;
  uint32_t cb_w[4] = {0, 0, 0, 0}, cb_lo = 0, cb_hi = 0, cx[4] = {0, 0, 0, 0}, cxlo = 0;
  uint64_t cb_tal = 0;
  // the wave's first byte: the chunk's plus the bytes of the lower waves' tiles (SPLIT; the waves of a
  // workgroup then share its chunk, so none of them has returned above)
  if constexpr (SPLIT) {
    uint32_t ws = 0;
#pragma unroll
    for (uint32_t t = 0; t < TPW; t++) {
      const uint32_t ts = j * CH + (T0 + t) * TV;
#pragma unroll
      for (uint32_t e = 0; e < E; e++) {
        const uint32_t sl = ts + E * lane + e;
        const uint32_t id = idw == 1u ? (idr[2 * t] >> (8u * e)) & 0xFFu
                                      : (idr[2 * t + (e >> 1)] >> (16u * (e & 1u))) & 0xFFFFu;
        ws += sl >= s_lo && sl < ok_hi && id < dict_n ? ent[id] & 0xFFFFu : 0u;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ws += (uint32_t)__shfl_xor((int)ws, o);
    if (lane == 0) wsum[wave_id()] = ws;
    __syncthreads();
  }
  uint64_t run_base = uni64(bases[c]);
  if constexpr (SPLIT) {
    for (uint32_t w = 0; w < wave_id(); w++) run_base += wsum[w];
    run_base = uni64(run_base);
  }
#pragma unroll 1
  for (uint32_t t = T0; t < T1; t++) {
    const uint32_t ts = uni(j * CH + t * TV);
    if (ts >= s_hi) break;
    uint32_t ln[E], sr[E], ls = 0;
#pragma unroll
    for (uint32_t e = 0; e < E; e++) {
      const uint32_t sl = ts + E * lane + e;
      const uint32_t id = idw == 1u ? (idr[2 * (t - T0)] >> (8u * e)) & 0xFFu
                                    : (idr[2 * (t - T0) + (e >> 1)] >> (16u * (e & 1u))) & 0xFFFFu;
      const uint32_t en = sl >= s_lo && sl < ok_hi && id < dict_n ? ent[id] : 0u;
      ln[e] = en & 0xFFFFu;
      sr[e] = en >> 16;
      ls += ln[e];
    }
    const uint32_t inc = wave_incl_scan_u32_dpp(ls);
    const uint32_t tot = uni(rdl(inc, WAVE - 1));
    uint64_t o[E];
    o[0] = run_base + (inc - ls);
#pragma unroll
    for (uint32_t e = 1; e < E; e++) o[e] = o[e - 1] + ln[e - 1];
    int64_t* op = opag + ts + E * lane;
    if (o16 && ts >= s_lo && ts + TV <= s_hi) {
      gst_nt((i64x2*)op, i64x2{(int64_t)o[0], (int64_t)o[1]});
      gst_nt((i64x2*)(op + 2), i64x2{(int64_t)o[2], (int64_t)o[3]});
    } else {
#pragma unroll
      for (uint32_t e = 0; e < E; e++)
        if (ts + E * lane + e >= s_lo && ts + E * lane + e < s_hi) gst(op + e, (int64_t)o[e]);
    }
    const uint64_t tb = run_base;  // the tile's first byte
    run_base += tot;
    if (run_base <= cap && gather) {
      wave_sync();  // the previous tile's gather reads are done
      // positions relative to the tile's first 16-byte block (32-bit): bytes [rb, re)
      const uint64_t tal = tb & ~15ull;
      const uint32_t rb = (uint32_t)(tb - tal), re = rb + tot;
#pragma unroll
      for (uint32_t e = 0; e < E; e++) {
        G.vo[E * lane + e] = rb + (uint32_t)(o[e] - tb);
        G.ve[E * lane + e] = (sr[e] << 16) | ln[e];
      }
      const uint32_t nblk = (re + 15u) >> 4;
#pragma unroll
      for (uint32_t e = 0; e < E; e++) {
        if (!ln[e]) continue;
        // the blocks whose first byte (16 b, or rb for the tile's first block) this value holds
        const uint32_t g = rb + (uint32_t)(o[e] - tb);
        for (uint32_t b = g == rb ? (g >> 4) : ((g + 15u) >> 4); (b << 4) < g + ln[e]; b++) G.fv[b] = (uint16_t)(E * lane + e);
      }
      wave_sync();
      // the tile's last block, when partial, is finished by the next tile of the chunk (same wave)
      const bool next_tile = t + 1 < T1 && ts + TV < s_hi;
      for (uint32_t b = lane; b < nblk; b += WAVE) {
        const uint32_t gb = b << 4;
        uint32_t bs = gb > rb ? gb : rb;
        const uint32_t be = gb + 16u < re ? gb + 16u : re;
        uint32_t v = G.fv[b];
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        if (b == 0 && cb_on) {  // the previous tile's partial last block (uniform carry)
          a0 = cb_w[0]; a1 = cb_w[1]; a2 = cb_w[2]; a3 = cb_w[3];
          bs = cb_lo;
        }
        uint32_t pos = gb > rb ? gb : rb;
        while (pos < be) {
          const uint32_t g = G.vo[v], ev = G.ve[v];
          const uint32_t ge = g + (ev & 0xFFFFu);
          if (pos < ge) {  // (empty values hold no byte)
            const uint32_t n = (ge < be ? ge : be) - pos;  // bytes of this piece
            const uint32_t k = pos - gb;                    // their place in the block
            // the 16 page bytes that line up with the block: page offset (source of pos) - k, read
            // through the 16 bytes of slack before the staged page
            const uint32_t base = 16u + (ev >> 16) + (pos - g) - k;
            const uint32_t q = base & ~3u, r = base & 3u;
            const uint32_t* w = (const uint32_t*)(dd_raw + q);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
            // block bytes k .. 15 from the source (a later piece overwrites from its own k on; bytes
            // past the block's end are not stored)
            const u32x4 sl = dd_sel[k];
            a0 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w1, w0, r), a0, sl.x);
            a1 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w2, w1, r), a1, sl.y);
            a2 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w3, w2, r), a2, sl.z);
            a3 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w4, w3, r), a3, sl.w);
            pos += n;
          }
          v++;
        }
        const uint32_t wd[4] = {a0, a1, a2, a3};
        if (b == nblk - 1u && be < gb + 16u && next_tile) {  // carried: the lane's values go to the next tile
          cx[0] = a0; cx[1] = a1; cx[2] = a2; cx[3] = a3;
          cxlo = bs - gb;
        } else {
          uint32_t have = 0;
#pragma unroll
          for (uint32_t d = 0; d < 4; d++) have |= (gb + 4u * d >= bs && gb + 4u * d + 4u <= be ? 1u : 0u) << d;
          store_block16(dst, tal + gb, tal + bs, tal + be, wd, have, true);
        }
      }
      // the partial last block of this tile (lane (nblk - 1) % 64) as uniform values for the next tile,
      // whose block 0 is the same 16 bytes (its first byte continues this tile's last)
      const bool carried = nblk && next_tile && (re & 15u) != 0u;
      if (carried) {
        const uint32_t cl = (nblk - 1u) & (WAVE - 1u);
#pragma unroll
        for (uint32_t d = 0; d < 4; d++) cb_w[d] = rdl(cx[d], cl);
        cb_lo = rdl(cxlo, cl);
      } else if (cb_on && nblk == 0) {  // (a tile without bytes: the carried block is stored as is)
        if (lane == 0) {
          uint32_t have = 0;
#pragma unroll
          for (uint32_t d = 0; d < 4; d++) have |= (4u * d >= cb_lo && 4u * d + 4u <= cb_hi ? 1u : 0u) << d;
          store_block16(dst, cb_tal, cb_tal + cb_lo, cb_tal + cb_hi, cb_w, have, true);
        }
      }
      cb_on = carried;
      cb_hi = re & 15u;
      cb_tal = tal + ((uint64_t)(nblk ? nblk - 1u : 0u) << 4);
    } else if (run_base <= cap) {
      if (one && ls == E) {  // 1-byte entries, the lane's 4 values in range: one dword
        uint32_t x = 0;
#pragma unroll
        for (uint32_t e = 0; e < E; e++) x |= (uint32_t)dd_lds[sr[e]] << (8u * e);
        *(g32u*)(dst + o[0]) = x;
      } else if (md <= 4u) {
        dd_put<1>(dst, o, ln, sr, dd_lds);
      } else if (md <= 8u) {
        dd_put<2>(dst, o, ln, sr, dd_lds);
      } else {
        // 16 bytes per value a round: every LDS read of a round before its stores (a read per store
        // waited for the LDS latency once per dword)
        for (uint32_t q0 = 0; q0 < md; q0 += 16u) dd_put<4>(dst, o, ln, sr, dd_lds, q0);
      }
    } else {  // past the capacity (reported at sync with the size needed): the bytes that fit
      if (cb_on) {  // the previous tile's carried partial block: its bytes below the capacity
        if (lane == 0) {
          const uint64_t hi = cb_tal + cb_hi < cap ? cb_tal + cb_hi : cap;
          store_block16(dst, cb_tal, cb_tal + cb_lo, hi, cb_w, 0u, true);
        }
        cb_on = false;
      }
#pragma unroll
      for (uint32_t e = 0; e < E; e++)
        for (uint32_t q = 0; q < ln[e]; q++)
          if (o[e] + q < cap) gst(dst + o[e] + q, dd_lds[sr[e] + q]);
    }
  }
}

// ---------------------------------------------------------------------------
// Dictionary-direct columns whose dictionary page is too large to stage in LDS (ColumnDev::dd_global: over
// DD_DICT_MAX bytes or 2,048 entries, at most 65,536 entries): the walk's expansion stores the u16 ids only
// (DD_IDS); the entries (PlainBinaryDictionary, PlainValuesDictionary.java:58-134: dict_len / dict_src from
// the dictionary walk) and the value bytes are gathered from HBM — a dictionary of a few hundred KB stays
// in L2 — by the two kernels below, with k_dd_bases between them. Ids past the dictionary and slots past a
// walk error are empty values (the walk reports the error), as k_dd_str writes them.

// Byte sum of every chunk: one wave per chunk, all its ids loaded first (two dwords per lane per tile),
// then the walked slots' entry lengths, summed over the wave (no stores but the sum).
__global__ __launch_bounds__(64 * WPB) void k_dd_gsums(const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                     const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                     const uint64_t* pstat, uint64_t* sums) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  constexpr uint32_t E = 4, TV = WAVE * E, CH = CH_TILES * TV;
  const uint32_t lane = lane_id();
  const uint32_t c = blockIdx.x * WPB + wave_id();
  if (c >= n_chunks) return;
  const uint64_t ce = chunks[c];
  if ((uint32_t)ce == 0xFFFFFFFFu) return;  // padding between columns (never summed)
  const int page = (int)(uint32_t)ce;
  const PageWork pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t j = (uint32_t)(ce >> 32);
  const uint32_t dict_n = uni(cd.dict_n), NF = uni(pw.n_values);
  const uint32_t nok = uni((uint32_t)(sld(pstat + page) >> 32));  // values before a walk error
  const uint32_t sh = (uint32_t)(pw.out_offset % E);
  const uint32_t s_lo = j * CH > sh ? j * CH : sh;
  const uint32_t s_hi = (j + 1) * CH < NF + sh ? (j + 1) * CH : NF + sh;
  const uint32_t ok_hi = (nok < NF ? nok : NF) + sh;
  uint64_t acc = 0;
  if (s_lo < s_hi) {
    const uint16_t* idpag = (const uint16_t*)cd.blen + (pw.out_offset - sh);
    u32x2 idr[CH_TILES];
#pragma unroll
    for (uint32_t t = 0; t < CH_TILES; t++) {
      const uint32_t ts = j * CH + t * TV;
      idr[t] = ts + E * lane < s_hi ? *(const __attribute__((address_space(1))) u32x2*)(idpag + ts + E * lane)
                                     : u32x2{0u, 0u};
    }
#pragma unroll
    for (uint32_t t = 0; t < CH_TILES; t++) {
      const uint32_t ts = j * CH + t * TV;
#pragma unroll
      for (uint32_t e = 0; e < E; e++) {
        const uint32_t sl = ts + E * lane + e;
        const uint32_t id = ((e < 2 ? idr[t].x : idr[t].y) >> (16u * (e & 1u))) & 0xFFFFu;
        const bool ok = sl >= s_lo && sl < ok_hi && id < dict_n;
        acc += ok ? cd.dict_len[ok ? id : 0u] : 0u;
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += (uint64_t)__shfl_xor((long long)acc, o);
  if (lane == 0) gst(sums + c, acc);
}

// Offsets and value bytes: one workgroup per 4,096-value chunk, wave w its tiles [4 w, 4 w + 4). The
// wave's ids, then its values' entries (lane: 4 per tile), are loaded before the first store; per tile
// a wave scan of the lengths gives the offsets (two 16-byte stores per lane), and the value bytes of
// entries of at most 32 bytes go through LDS: each value's 32 source bytes (two 16-byte loads from the
// dictionary page, the next tile's requested before this tile's stores) into a staging slot, then every
// lane composes whole 16-byte output blocks from the slots (k_dd_str's block gather) and stores them
// aligned, a tile's edge blocks byte-masked. A tile with a longer entry copies bytes one by one.
constexpr uint32_t DDX_MD = 32;  // longest entry of the block path (= staging bytes per value)
// (16-bit offsets and 8-bit block owners: 39.4 KB per workgroup, 4 workgroups per CU instead of 3)
struct DdxLds {
  uint8_t pre[16];                               // slack before the staging (the gather reads base - k)
  uint32_t stg[WAVE * 4 * DDX_MD / 4 + 8];       // lane l's value e: 32 source bytes at 32 (64 e + l) (+ slack)
  uint16_t vo[WAVE * 4];                         // tile-relative first output byte of value v (< 8,208)
  uint16_t ve[WAVE * 4];                         // staging slot << 6 | length (<= 32)
  uint8_t fv[(WAVE * 4 * DDX_MD) / 16 + 2];      // output block b: the value (< 256) holding its first byte
};
__global__ __launch_bounds__(64 * WPB) void k_dd_gstr(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                    const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                    const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                    const uint64_t* pstat, const uint64_t* __restrict__ bases,
                                                    uint64_t* err, ErrCount err_count) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
  constexpr uint32_t E = 4, TV = WAVE * E, CH = CH_TILES * TV, TPW = CH_TILES / WPB;
  __shared__ __attribute__((aligned(16))) DdxLds lds_all[WPB];
  __shared__ u32x4 dd_sel[16];  // (k_dd_str's selectors: block bytes k .. 15 from the source)
  __shared__ uint32_t wsum[WPB];
  if (threadIdx.x < 64u) {
    const uint32_t k = threadIdx.x >> 2, d = threadIdx.x & 3u;
    uint32_t sel = 0;
#pragma unroll
    for (uint32_t jb = 0; jb < 4; jb++) sel |= (4u * d + jb >= k ? 4u + jb : jb) << (8u * jb);
    ((uint32_t*)dd_sel)[threadIdx.x] = sel;
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  const uint32_t c = blockIdx.x;  // (the workgroup's waves share the chunk: uniform exits below)
  if (c >= n_chunks) return;
  const uint64_t ce = chunks[c];
  if ((uint32_t)ce == 0xFFFFFFFFu) return;
  const int page = (int)(uint32_t)ce;
  const PageWork pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t j = (uint32_t)(ce >> 32);
  const uint32_t dict_n = uni(cd.dict_n), NF = uni(pw.n_values);
  const uint32_t nok = uni((uint32_t)(sld(pstat + page) >> 32));
  const uint32_t sh = (uint32_t)(pw.out_offset % E);
  const uint32_t s_lo = j * CH > sh ? j * CH : sh;
  const uint32_t s_hi = (j + 1) * CH < NF + sh ? (j + 1) * CH : NF + sh;
  if (s_lo >= s_hi) return;
  const uint32_t ok_hi = (nok < NF ? nok : NF) + sh;
  const uint32_t T0 = wave_id() * TPW;
  // ids, then entries (all loads before the first store)
  const uint16_t* idpag = (const uint16_t*)cd.blen + (pw.out_offset - sh);
  u32x2 idr[TPW];
#pragma unroll
  for (uint32_t t = 0; t < TPW; t++) {
    const uint32_t ts = j * CH + (T0 + t) * TV;
    idr[t] = ts + E * lane < s_hi ? *(const __attribute__((address_space(1))) u32x2*)(idpag + ts + E * lane)
                                   : u32x2{0u, 0u};
  }
  uint32_t ln[TPW][E], sr[TPW][E], ws = 0;
#pragma unroll
  for (uint32_t t = 0; t < TPW; t++) {
    const uint32_t ts = j * CH + (T0 + t) * TV;
#pragma unroll
    for (uint32_t e = 0; e < E; e++) {
      const uint32_t sl = ts + E * lane + e;
      const uint32_t id = ((e < 2 ? idr[t].x : idr[t].y) >> (16u * (e & 1u))) & 0xFFFFu;
      const bool ok = sl >= s_lo && sl < ok_hi && id < dict_n;
      const uint64_t en = cd.dict_ent[ok ? id : 0u];  // (branch-free: see ld8_any)
      ln[t][e] = ok ? (uint32_t)en : 0u;
      sr[t][e] = ok ? (uint32_t)(en >> 32) : 0u;
      ws += ln[t][e];
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ws += (uint32_t)__shfl_xor((int)ws, o);
  if (lane == 0) wsum[wave_id()] = ws;
  __syncthreads();
  uint64_t run_base = uni64(bases[c]);
  for (uint32_t w = 0; w < wave_id(); w++) run_base += wsum[w];
  run_base = uni64(run_base);
  uint8_t* const dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  int64_t* const opag = (int64_t*)cd.values + (pw.out_offset - sh);
  const bool o16 = ((uintptr_t)cd.values & 15u) == 0, d16 = ((uintptr_t)dst & 15u) == 0;
  // the dictionary page + the batch's readable slack after it: a load at DDX_OOB is out of range (no access)
  const rsrc_t drs = make_rsrc(bytes + cd.dict_offset, cd.dict_bytes + 64u);
  constexpr uint32_t DDX_OOB = 0x7FFFFFF0u;
  const rsrc_t brs = make_rsrc(bytes + cd.dict_offset, n_bytes - cd.dict_offset);  // (long entries, byte by byte)
  DdxLds& X = lds_all[wave_id()];
  const uint8_t* const xb = (const uint8_t*)&X;  // staged source s is at xb + 16 + s
  // the 32 source bytes of the lane's 4 values of tile t (entries over 32 bytes: the byte path)
  u32x4 pb[E][2];
  auto load_tile = [&](uint32_t t) {
#pragma unroll
    for (uint32_t e = 0; e < E; e++) {  // (out-of-range offsets for empty values / bytes 16.. of short ones)
      pb[e][0] = __builtin_amdgcn_raw_buffer_load_b128(drs, (int)(ln[t][e] ? sr[t][e] : DDX_OOB), 0, 0);
      pb[e][1] = __builtin_amdgcn_raw_buffer_load_b128(drs, (int)(ln[t][e] > 16u ? sr[t][e] + 16u : DDX_OOB), 0, 0);
    }
  };
  load_tile(0);
#pragma unroll
  for (uint32_t t = 0; t < TPW; t++) {
    const uint32_t ts = j * CH + (T0 + t) * TV;
    if (ts >= s_hi) break;  // (uniform)
    uint32_t ls = 0, mx = 0;
#pragma unroll
    for (uint32_t e = 0; e < E; e++) {
      ls += ln[t][e];
      mx = ln[t][e] > mx ? ln[t][e] : mx;
    }
    const uint32_t inc = wave_incl_scan_u32_dpp(ls);
    const uint32_t tot = uni(rdl(inc, WAVE - 1));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t y = (uint32_t)__shfl_xor((int)mx, o);
      mx = y > mx ? y : mx;
    }
    mx = uni(mx);
    uint64_t o[E];
    o[0] = run_base + (inc - ls);
#pragma unroll
    for (uint32_t e = 1; e < E; e++) o[e] = o[e - 1] + ln[t][e - 1];
    const uint64_t tb = run_base;
    run_base += tot;
    const bool gather = mx <= DDX_MD && d16 && run_base <= cap;
    const uint64_t tal = tb & ~15ull;
    const uint32_t rb = (uint32_t)(tb - tal), re = rb + tot;
    if (gather) {
      wave_sync();  // the previous tile's gather reads are done
#pragma unroll
      for (uint32_t e = 0; e < E; e++) {
        // slots 64 e + lane: consecutive lanes 32 bytes apart (slots 4 lane + e, 128 bytes apart, put a
        // 16-byte write of every lane on two bank groups)
        const uint32_t v = E * lane + e, slot = WAVE * e + lane;
        *(u32x4*)&X.stg[8u * slot] = pb[e][0];
        *(u32x4*)&X.stg[8u * slot + 4u] = pb[e][1];
        X.vo[v] = (uint16_t)(rb + (uint32_t)(o[e] - tb));
        X.ve[v] = (uint16_t)((slot << 6) | ln[t][e]);
      }
#pragma unroll
      for (uint32_t e = 0; e < E; e++) {
        if (!ln[t][e]) continue;
        // the blocks whose first byte (16 b, or rb for the tile's first block) this value holds
        const uint32_t g = rb + (uint32_t)(o[e] - tb);
        for (uint32_t b = g == rb ? (g >> 4) : ((g + 15u) >> 4); (b << 4) < g + ln[t][e]; b++)
          X.fv[b] = (uint8_t)(E * lane + e);
      }
    }
    // the next tile's source bytes, requested before this tile's stores
    if (t + 1 < TPW) load_tile(t + 1);
    int64_t* op = opag + ts + E * lane;
    if (o16 && ts >= s_lo && ts + TV <= s_hi) {
      gst_nt((i64x2*)op, i64x2{(int64_t)o[0], (int64_t)o[1]});
      gst_nt((i64x2*)(op + 2), i64x2{(int64_t)o[2], (int64_t)o[3]});
    } else {
#pragma unroll
      for (uint32_t e = 0; e < E; e++)
        if (ts + E * lane + e >= s_lo && ts + E * lane + e < s_hi) gst(op + e, (int64_t)o[e]);
    }
    if (gather) {
      wave_sync();
      const uint32_t nblk = (re + 15u) >> 4;
      for (uint32_t b = lane; b < nblk; b += WAVE) {
        const uint32_t gb = b << 4;
        const uint32_t bs = gb > rb ? gb : rb;
        const uint32_t be = gb + 16u < re ? gb + 16u : re;
        uint32_t v = X.fv[b];
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        uint32_t pos = bs;
        while (pos < be) {
          const uint32_t g = X.vo[v], ev = X.ve[v];
          const uint32_t ge = g + (ev & 63u);
          if (pos < ge) {  // (empty values hold no byte)
            const uint32_t n = (ge < be ? ge : be) - pos;
            const uint32_t k = pos - gb;
            const uint32_t base = 16u + DDX_MD * (ev >> 6) + (pos - g) - k;
            const uint32_t q = base & ~3u, r = base & 3u;
            const uint32_t* w = (const uint32_t*)(xb + q);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
            const u32x4 sl = dd_sel[k];
            a0 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w1, w0, r), a0, sl.x);
            a1 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w2, w1, r), a1, sl.y);
            a2 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w3, w2, r), a2, sl.z);
            a3 = __builtin_amdgcn_perm(__builtin_amdgcn_alignbyte(w4, w3, r), a3, sl.w);
            pos += n;
          }
          v++;
        }
        const uint32_t wd[4] = {a0, a1, a2, a3};
        uint32_t have = 0;
#pragma unroll
        for (uint32_t d = 0; d < 4; d++) have |= (gb + 4u * d >= bs && gb + 4u * d + 4u <= be ? 1u : 0u) << d;
        store_block16(dst, tal + gb, tal + bs, tal + be, wd, have, true);
      }
    } else {  // entries over 32 bytes, an unaligned value buffer, or past the capacity: the bytes that fit
#pragma unroll
      for (uint32_t e = 0; e < E; e++)
        for (uint32_t q = 0; q < ln[t][e]; q++)
          if (o[e] + q < cap) gst(dst + o[e] + q, (uint8_t)(ld32(brs, (sr[t][e] + q) & ~3u) >> (((sr[t][e] + q) & 3u) * 8u)));
    }
  }
  (void)err;
  (void)err_count;
}

// ---------------------------------------------------------------------------
// Levels (def/rep) of nullable columns: ColumnReaderBase.readPageV1/readPageV2,
// RunLengthBitPackingHybridValuesReader.initFromPage (4-byte length prefix),
// newRLEIterator (V2, no prefix). Writes u8 levels, the page's non-null count
// and the data section start; value kernels run afterwards.

// BIT_PACKED (big-endian) level section [beg, end): level i = bits [i*w, (i+1)*w) MSB first
// (Packer.BIG_ENDIAN, ByteBasedBitPackingGenerator getShift msbFirst :153-159); bytes past the
// section read as 0 (ByteBitPackingValuesReader.readMore :49-57). 16 slots per lane, no errors.
__device__ uint32_t decode_levels_be(rsrc_t rs, uint32_t beg, uint32_t end, int w, uint32_t N, uint8_t* out,
                                     uint32_t max_def, bool count_nonnull, uint32_t* nonnull, int* err_code) {
  const uint32_t lane = lane_id();
  uint32_t cnt = 0;
  const uint32_t mask = (1u << w) - 1u;  // w <= 8 (max level <= 254)
  for (uint32_t s0 = 16u * lane; s0 < N; s0 += 16u * WAVE) {
    uint64_t wlo = 0, whi = 0;
    for (uint32_t j = 0; j < 16 && s0 + j < N; j++) {
      const uint64_t bit = (uint64_t)(s0 + j) * (uint32_t)w;
      const uint32_t a = beg + (uint32_t)(bit >> 3);
      uint32_t x = 0;  // bytes a .. a+3, big endian, 0 past the section
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t bq = a + q < end ? (ld32(rs, (a + q) & ~3u) >> (((a + q) & 3u) * 8u)) & 0xFFu : 0u;
        x = (x << 8) | bq;
      }
      const uint32_t v = (x >> (32u - (uint32_t)(bit & 7u) - (uint32_t)w)) & mask;
      if (count_nonnull && v == max_def) cnt++;
      if (j < 8) wlo |= (uint64_t)v << (8 * j);
      else whi |= (uint64_t)v << (8 * (j - 8));
    }
    if (out)
      for (uint32_t j = 0; j < 16 && s0 + j < N; j++)
        gst(out + s0 + j, (uint8_t)((j < 8 ? wlo >> (8 * j) : whi >> (8 * (j - 8))) & 0xFFu));
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (nonnull) *nonnull = cnt;
  *err_code = 0;
  return N;
}

// Per-wave LDS of the level decoder: the page segment, the binary-lifting tables of one 256-byte
// window's header chain, the window's pre-decoded headers, and the window's run table.
// A run of a level section takes at least 2 bytes (w >= 1: header + value byte, or header + >= 1
// group byte), so a window's chain holds at most 128 runs.
constexpr uint32_t LV_RUNS = 128;
struct LevelWaveLds {
  uint8_t seg[SEG_BYTES];     // page bytes [seg_lo, seg_lo + SEG_BYTES)
  uint8_t J[6][256];          // J[r][p]: window offset of the 2^r-th header after p; 0: the chain stops first
  uint32_t ecnt[256];         // position p as a header: run count | packed << 31
  uint16_t eval[256];         // RLE: value (saturated to 255); PACKED: data start - window start
  uint32_t r_start[LV_RUNS];  // first slot of run k of the window
  uint32_t r_pay[LV_RUNS];    // RLE: value (saturated to 255); PACKED: 0x80000000 | data byte position
  uint32_t r_end[LV_RUNS];    // PACKED: end of the bytes read for the run (truncated final group)
  // the partial 16-slot tile a window's expansion ended on (more windows follow): its levels wait
  // here for the next window's part instead of going out as byte stores (expand_level_tiles)
  uint32_t carry[4];
  int32_t carry_s0;       // tile start (slot index relative to the output base)
  uint32_t carry_j;       // valid bytes [carry_j & 255, carry_j >> 8); 0: none
};

// Levels of the runs rs[0 .. n_run) covering slots [s_lo, s_hi) -> out (u8), 16 slots per lane
// with 16-byte stores where the tile is inside [s_lo, s_hi); counts slots == max_def.
// Packed bytes come from the wave's LDS segment of the page when it holds them (a global load
// here would wait for the tile stores before it: vmcnt counts stores).
// Byte mask of bytes [jb, je) (clamped to the tile) in dword i of a 16-byte tile.
__device__ __forceinline__ uint32_t tile_byte_mask(int32_t jb, int32_t je, int32_t i) {
  const int32_t lo = jb - 4 * i < 0 ? 0 : (jb - 4 * i > 4 ? 4 : jb - 4 * i);
  const int32_t hi = je - 4 * i < 0 ? 0 : (je - 4 * i > 4 ? 4 : je - 4 * i);
  const uint32_t mh = hi >= 4 ? 0xFFFFFFFFu : (1u << (8 * hi)) - 1u;
  const uint32_t ml = lo >= 4 ? 0xFFFFFFFFu : (1u << (8 * lo)) - 1u;
  return mh & ~ml;
}

// Run holding slot lo_s: the largest a < n_run (<= 256) with r_start[a] <= lo_s (r_start ascending,
// r_start[0] <= lo_s). Eight fixed steps with unconditional LDS reads instead of this divergent
// bisection loop (whose exec bookkeeping runs on the scalar unit) measured C3 10.01 -> 10.10 ms,
// C5 2.17 -> 2.19 ms (profiles/r02/lv_ab) and were removed.
// Store one tile's levels [j0, j1) (out + s0 is 16-byte aligned): the first tile of a window range merges
// the carried part of the same tile (the previous window ended inside it, so carry_j's end is j0); a tile
// the range ends inside, with more windows to come, becomes the carry; whole tiles go out as one
// 16-byte store, the tiles at the page's edges byte by byte (other pages own the rest).
__device__ __forceinline__ void level_tile_out(LevelWaveLds& L, uint8_t* out, int64_t s0, uint32_t (&acc)[4], int32_t j0,
                                               int32_t j1, uint32_t s_lo, uint32_t s_hi, bool more) {
  if (s0 + j0 == (int64_t)s_lo && j0 > 0) {
    const uint32_t cj = L.carry_j;
    if (cj && L.carry_s0 == (int32_t)s0 && (int32_t)(cj >> 8) == j0) {
#pragma unroll
      for (int32_t c = 0; c < 4; c++) {
        const uint32_t mk = tile_byte_mask(j0, 16, c);
        acc[c] = (acc[c] & mk) | (L.carry[c] & ~mk);
      }
      j0 = (int32_t)(cj & 255u);
      L.carry_j = 0;
    }
  }
  if (more && j1 < 16 && s0 + j1 == (int64_t)s_hi) {
#pragma unroll
    for (int32_t c = 0; c < 4; c++) L.carry[c] = acc[c];
    L.carry_s0 = (int32_t)s0;
    L.carry_j = (uint32_t)j0 | ((uint32_t)j1 << 8);
    return;
  }
  uint8_t* o = out + s0;
  if (j0 == 0 && j1 == 16) {
    gst((u32x4*)o, u32x4{acc[0], acc[1], acc[2], acc[3]});
  } else {
#pragma unroll
    for (int32_t j = 0; j < 16; j++)
      if (j >= j0 && j < j1) gst(o + j, (uint8_t)(acc[j >> 2] >> (8 * (j & 3))));
  }
}

// A carry left when the section's decode stopped early (an error): its levels go out byte by byte.
__device__ __forceinline__ void level_carry_flush(LevelWaveLds& L, uint8_t* out) {
  wave_sync();
  const uint32_t cj = L.carry_j;
  if (cj && out && lane_id() < 16u) {
    const uint32_t j = lane_id();
    if (j >= (cj & 255u) && j < (cj >> 8)) gst(out + L.carry_s0 + (int32_t)j, (uint8_t)(L.carry[j >> 2] >> (8u * (j & 3u))));
  }
  wave_sync();
  if (lane_id() == 0) L.carry_j = 0;
  wave_sync();
}

__device__ __forceinline__ uint32_t level_run_of(const LevelWaveLds& L, uint32_t n_run, uint32_t lo_s) {
  uint32_t a = 0, b = n_run;
  while (b - a > 1) {
    const uint32_t mid = (a + b) >> 1;
    if (L.r_start[mid] <= lo_s) a = mid;
    else b = mid;
  }
  return a;
}

// Bit width WB (1..8) specialisation of expand_level_runs: per tile piece (the part of one run
// inside the lane's 16 slots) the 16 levels are formed without a per-slot loop: an RLE piece is
// its value replicated, a packed piece is 24 bytes at the piece's bit offset, shifted once, then
// 16 bit fields at compile-time positions; a byte mask merges the piece into the tile.
template <int WB>
__device__ __forceinline__ void expand_level_tiles(LevelWaveLds& L, const PreWin& win, uint32_t n_run,
                                                   uint32_t s_lo, uint32_t s_hi, uint8_t* out, uint32_t max_def,
                                                   bool count_nonnull, uint32_t& cnt, bool more) {
  const rsrc_t rs = win.rs;
  const uint32_t lane = lane_id();
  const int64_t mis = out ? (int64_t)((uintptr_t)out & 15u) : 0;
  // width 1 with every RLE value 0 or 1 (the usual flat optional column): the tile's 16 levels
  // are built as a 16-bit mask (3 operations per piece) and spread to bytes once per tile
  bool bits_ok = false;
  if constexpr (WB == 1) {
    bool bad = false;
    for (uint32_t i = lane; i < n_run; i += WAVE) {
      const uint32_t p = L.r_pay[i];
      bad |= !(p & 0x80000000u) && p > 1u;
    }
    bits_ok = !__ballot(bad);
  }
  for (int64_t t = (((int64_t)s_lo + mis) & ~(int64_t)15) - mis; t < (int64_t)s_hi; t += 16 * WAVE) {
    const int64_t s0 = t + 16 * (int64_t)lane;
    if (s0 + 16 <= (int64_t)s_lo || s0 >= (int64_t)s_hi) continue;
    const uint32_t lo_s = (uint32_t)(s0 > (int64_t)s_lo ? s0 : (int64_t)s_lo);
    const uint32_t hi_s = (uint32_t)(s0 + 16 < (int64_t)s_hi ? s0 + 16 : (int64_t)s_hi);
    const uint32_t a = level_run_of(L, n_run, lo_s);
    uint32_t acc[4] = {0u, 0u, 0u, 0u};
    uint32_t cur = lo_s, k = a;
    if (WB == 1 && bits_ok) {
      uint32_t m = 0;  // bit j: level of tile slot j
      while (cur < hi_s) {
        const uint32_t st = L.r_start[k], pay = L.r_pay[k];
        const uint32_t re = k + 1 < n_run ? L.r_start[k + 1] : s_hi;
        const uint32_t stop = hi_s < re ? hi_s : re;
        const uint32_t jb = cur - (uint32_t)s0, je = stop - (uint32_t)s0;
        const uint32_t pm = ((1u << je) - 1u) & ~((1u << jb) - 1u);
        uint32_t bits;
        if (!(pay & 0x80000000u)) {
          bits = pay ? 0xFFFFu : 0u;
        } else {
          // 32 bits of the run's data from slot cur on (bytes at or past the read end are 0)
          const uint32_t rlo = pay & 0x7FFFFFFFu, rhi = L.r_end[k];
          const uint32_t bp = cur - st, byte0 = rlo + (bp >> 3), a4 = byte0 & ~3u;
          uint32_t y0, y1;
          if (seg_has(win, a4, 8u)) {
            y0 = seg32(win, a4);
            y1 = seg32(win, a4 + 4u);
          } else {
            y0 = ld32(rs, a4);
            y1 = ld32(rs, a4 + 4u);
          }
          const int32_t k0 = (int32_t)rhi - (int32_t)a4, k1 = k0 - 4;
          y0 &= k0 >= 4 ? 0xFFFFFFFFu : (k0 <= 0 ? 0u : (1u << (8 * k0)) - 1u);
          y1 &= k1 >= 4 ? 0xFFFFFFFFu : (k1 <= 0 ? 0u : (1u << (8 * k1)) - 1u);
          const uint32_t z = __builtin_amdgcn_alignbyte(y1, y0, byte0 & 3u);
          bits = (z >> (bp & 7u)) << jb;
        }
        m = (m & ~pm) | (bits & pm);
        cur = stop;
        k++;
      }
#pragma unroll
      for (uint32_t c = 0; c < 4; c++) acc[c] = (((m >> (4u * c)) & 0xFu) * 0x204081u) & 0x01010101u;
      const uint32_t j0 = lo_s - (uint32_t)s0, j1 = hi_s - (uint32_t)s0;
      const uint32_t jm = ((1u << j1) - 1u) & ~((1u << j0) - 1u);
      if (count_nonnull) cnt += max_def == 1 ? __builtin_popcount(m & jm) : max_def == 0 ? __builtin_popcount(~m & jm) : 0;
      if (out) level_tile_out(L, out, s0, acc, (int32_t)j0, (int32_t)j1, s_lo, s_hi, more);
      continue;
    }
    while (cur < hi_s) {
      const uint32_t st = L.r_start[k], pay = L.r_pay[k];
      const uint32_t re = k + 1 < n_run ? L.r_start[k + 1] : s_hi;
      const uint32_t stop = hi_s < re ? hi_s : re;
      const int32_t jb = (int32_t)(cur - (uint32_t)s0), je = (int32_t)(stop - (uint32_t)s0);
      uint32_t v[4];
      if (!(pay & 0x80000000u)) {
        const uint32_t rep = pay * 0x01010101u;  // pay <= 255 (saturated)
        v[0] = v[1] = v[2] = v[3] = rep;
      } else {
        // bit offset of tile slot 0 from the run's data start (negative when the run starts
        // inside the tile: those slots are masked off below)
        const uint32_t rlo = pay & 0x7FFFFFFFu, rhi = L.r_end[k];
        const int64_t base = ((int64_t)cur - (int64_t)st - (int64_t)jb) * WB;
        const int64_t byte0 = (int64_t)rlo + (base >> 3);
        const uint32_t bsh = (uint32_t)(base & 7);
        const int64_t a4 = byte0 & ~(int64_t)3;  // may be < 0 near the page start (masked slots only)
        const uint32_t sb = (uint32_t)(byte0 & 3);
        uint32_t y[6];
        if (a4 >= 0 && seg_has(win, (uint32_t)a4, 24u)) {
#pragma unroll
          for (uint32_t c = 0; c < 6; c++) y[c] = seg32(win, (uint32_t)a4 + 4u * c);
        } else {
#pragma unroll
          for (uint32_t c = 0; c < 6; c++) y[c] = a4 + 4 * (int64_t)c >= 0 ? ld32(rs, (uint32_t)(a4 + 4 * (int64_t)c)) : 0u;
        }
        // bytes at or past the run's read end are 0 (readNext :96-99: truncated final group)
#pragma unroll
        for (uint32_t c = 0; c < 6; c++) {
          const int64_t kp = (int64_t)rhi - (a4 + 4 * (int64_t)c);
          y[c] &= kp >= 4 ? 0xFFFFFFFFu : (kp <= 0 ? 0u : (1u << (8 * kp)) - 1u);
        }
        uint32_t z[5], D[5];
#pragma unroll
        for (uint32_t c = 0; c < 5; c++) z[c] = __builtin_amdgcn_alignbyte(y[c + 1], y[c], sb);
#pragma unroll
        for (uint32_t c = 0; c < 4; c++) D[c] = __builtin_amdgcn_alignbit(z[c + 1], z[c], bsh);
        D[4] = z[4] >> bsh;
        v[0] = v[1] = v[2] = v[3] = 0u;
#pragma unroll
        for (uint32_t q = 0; q < 16; q++) {
          constexpr uint32_t M = (1u << WB) - 1u;
          const uint32_t bp = q * WB, wi = bp >> 5, bo = bp & 31u;
          const uint32_t f = (bo + WB <= 32u ? (D[wi] >> bo) : __builtin_amdgcn_alignbit(D[wi + 1], D[wi], bo)) & M;
          v[q >> 2] |= f << (8u * (q & 3u));
        }
      }
#pragma unroll
      for (int32_t c = 0; c < 4; c++) {
        const uint32_t m = tile_byte_mask(jb, je, c);
        acc[c] = (acc[c] & ~m) | (v[c] & m);
      }
      cur = stop;
      k++;
    }
    const int32_t j0 = (int32_t)(lo_s - (uint32_t)s0), j1 = (int32_t)(hi_s - (uint32_t)s0);
    if (count_nonnull) {
      // bytes == max_def inside [j0, j1): zero bytes of acc ^ max_def (per-byte test, no carries)
      const uint32_t rep = max_def * 0x01010101u;
#pragma unroll
      for (int32_t c = 0; c < 4; c++) {
        const uint32_t y = acc[c] ^ rep;
        const uint32_t nz = ((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y;  // bit 7 of a byte: byte != 0
        cnt += (uint32_t)__builtin_popcount(~nz & 0x80808080u & tile_byte_mask(j0, j1, c));
      }
    }
    if (out) level_tile_out(L, out, s0, acc, j0, j1, s_lo, s_hi, more);
  }
}

__device__ __forceinline__ void expand_level_runs_generic(const LevelWaveLds& L, const PreWin& win, uint32_t n_run,
                                                          uint32_t s_lo, uint32_t s_hi, int w, uint8_t* out,
                                                          uint32_t max_def, bool count_nonnull, uint32_t& cnt);

// WB = 1..4: the specialised tile expansion; WB = 0: any width. (A level image in LDS written one run
// per lane, then read 16 slots per lane, measured no faster on C3: 0.990 vs 0.981 ms, profiles/r05/lv_image.)
template <int WB>
__device__ __forceinline__ void expand_level_runs(LevelWaveLds& L, const PreWin& win, uint32_t n_run,
                                                  uint32_t s_lo, uint32_t s_hi, int w, uint8_t* out,
                                                  uint32_t max_def, bool count_nonnull, uint32_t& cnt, bool more) {
  if constexpr (WB > 0) expand_level_tiles<WB>(L, win, n_run, s_lo, s_hi, out, max_def, count_nonnull, cnt, more);
  else expand_level_runs_generic(L, win, n_run, s_lo, s_hi, w, out, max_def, count_nonnull, cnt);
}

__device__ __forceinline__ void expand_level_runs_generic(const LevelWaveLds& L, const PreWin& win, uint32_t n_run,
                                                          uint32_t s_lo, uint32_t s_hi, int w, uint8_t* out,
                                                          uint32_t max_def, bool count_nonnull, uint32_t& cnt) {
  const rsrc_t rs = win.rs;
  const uint32_t lane = lane_id();
  const int64_t mis = out ? (int64_t)((uintptr_t)out & 15u) : 0;
  const uint32_t wmask = w >= 32 ? 0xFFFFFFFFu : (1u << w) - 1u;
  for (int64_t t = (((int64_t)s_lo + mis) & ~(int64_t)15) - mis; t < (int64_t)s_hi; t += 16 * WAVE) {
    const int64_t s0 = t + 16 * (int64_t)lane;
    if (s0 + 16 <= (int64_t)s_lo || s0 >= (int64_t)s_hi) continue;
    const uint32_t lo_s = (uint32_t)(s0 > (int64_t)s_lo ? s0 : (int64_t)s_lo);
    const uint32_t hi_s = (uint32_t)(s0 + 16 < (int64_t)s_hi ? s0 + 16 : (int64_t)s_hi);
    // run holding lo_s: last k with r_start[k] <= lo_s
    const uint32_t a = level_run_of(L, n_run, lo_s);
    uint64_t wlo = 0, whi = 0;
    uint32_t cur = lo_s, k = a;
    while (cur < hi_s) {
      const uint32_t st = L.r_start[k], pay = L.r_pay[k];
      const uint32_t re = k + 1 < n_run ? L.r_start[k + 1] : s_hi;
      const uint32_t stop = hi_s < re ? hi_s : re;
      if (!(pay & 0x80000000u)) {
        for (uint32_t q = cur; q < stop; q++) {
          const uint32_t j = q - (uint32_t)s0;
          if (j < 8) wlo |= (uint64_t)pay << (8 * j);
          else whi |= (uint64_t)pay << (8 * (j - 8));
        }
      } else if (w > 0) {
        const uint32_t rlo = pay & 0x7FFFFFFFu, rhi = L.r_end[k];
        const uint64_t bit0 = (uint64_t)(cur - st) * (uint32_t)w;
        const uint32_t a0 = rlo + (uint32_t)(bit0 >> 3);
        uint64_t x[3];
        const bool in_seg = seg_has(win, a0 & ~3u, 28u);
        uint32_t dw[7];
        if (in_seg) {
#pragma unroll
          for (uint32_t c = 0; c < 7; c++) dw[c] = seg32(win, (a0 & ~3u) + 4u * c);
        }
#pragma unroll
        for (uint32_t c = 0; c < 3; c++) {
          const uint32_t ac = a0 + 8u * c;
          const uint32_t sb = a0 & 3u;
          const uint64_t v = in_seg ? ((uint64_t)__builtin_amdgcn_alignbyte(dw[2 * c + 1], dw[2 * c], sb) |
                                       ((uint64_t)__builtin_amdgcn_alignbyte(dw[2 * c + 2], dw[2 * c + 1], sb) << 32))
                                    : ld8_any(rs, ac);
          const int64_t keep = (int64_t)rhi - (int64_t)ac;  // bytes past the run's read end are 0 (:96-99)
          x[c] = keep >= 8 ? v : (keep <= 0 ? 0 : (v & ((1ull << (8 * keep)) - 1ull)));
        }
        for (uint32_t q = cur; q < stop; q++) {
          const uint32_t sh = (uint32_t)(bit0 & 7u) + (q - cur) * (uint32_t)w;
          const uint32_t c = sh >> 6, o = sh & 63u;
          const uint64_t lo64 = c == 0 ? x[0] : (c == 1 ? x[1] : x[2]);
          const uint64_t hi64 = c == 0 ? x[1] : (c == 1 ? x[2] : 0ull);
          const uint64_t f = o ? ((lo64 >> o) | (hi64 << (64u - o))) : lo64;
          uint32_t v = (uint32_t)f & wmask;
          v = v > 255u ? 255u : v;
          const uint32_t j = q - (uint32_t)s0;
          if (j < 8) wlo |= (uint64_t)v << (8 * j);
          else whi |= (uint64_t)v << (8 * (j - 8));
        }
      }
      cur = stop;
      k++;
    }
    const uint32_t j0 = lo_s - (uint32_t)s0, j1 = hi_s - (uint32_t)s0;
    if (count_nonnull)
      for (uint32_t j = j0; j < j1; j++)
        cnt += (uint32_t)((j < 8 ? wlo >> (8 * j) : whi >> (8 * (j - 8))) & 0xFFu) == max_def ? 1u : 0u;
    if (out) {
      uint8_t* o = out + s0;
      if (j0 == 0 && j1 == 16) {
        typedef uint64_t v2 __attribute__((ext_vector_type(2)));
        gst((v2*)o, v2{wlo, whi});
      } else {
        for (uint32_t j = j0; j < j1; j++) gst(o + j, (uint8_t)((j < 8 ? wlo >> (8 * j) : whi >> (8 * (j - 8))) & 0xFFu));
      }
    }
  }
}

// RLE / bit-packed level section [beg, end) (RunLengthBitPackingHybridDecoder over the section)
// -> out[0 .. N), one 256-byte window at a time:
//   1. pre-decode: every lane parses a run header at each of its 4 byte positions as if one started
//      there (count, value / data start, successor position; branch-free up to 4-byte varints);
//   2. binary lifting: J[0][p] = the successor of p inside the window (0: the chain leaves the window
//      or p is not a fast-path header), J[r+1] = J[r] o J[r] — built only until the chain from the
//      window's entry position ends (J[r][entry] == 0), at most 5 rounds of 4 LDS byte gathers per lane;
//   3. lane t takes the chain's t-th header directly, c_t = J^t(entry), from the bits of t (one LDS
//      gather per bit): no per-position marks, no compaction; a chain of more than 64 headers is taken
//      64 at a time;
//   4. lane t reads its header's pre-decoded count / payload, a saturating DPP scan gives the runs'
//      first slots, lane t writes run t of the window's run table, and the tile expansion writes
//      the slots the window's runs cover.
// Replaced (round 4) the pointer doubling over all 256 positions with a scatter of chain marks per
// round and a ballot compaction of the marked headers (C3: ~15 VALU + 7 SALU per run, 1.05 ms).
// Returns the slots decoded before an error (N when none) and sets *err_code.
template <int WB>
__device__ __forceinline__ uint32_t decode_levels_bl(LevelWaveLds& L, rsrc_t rs, uint32_t beg, uint32_t end, int w,
                                                     uint32_t N, uint8_t* out, uint32_t max_def, bool count_nonnull,
                                                     uint32_t* nonnull, int* err_code, uint64_t* diag = nullptr) {
  const uint32_t lane = lane_id();
  typedef uint32_t __attribute__((may_alias)) u32a;
#ifdef PQG_DIAG
  uint64_t dt[5] = {0, 0, 0, 0, 0}, dm = __builtin_amdgcn_s_memtime();
#define LV_TICK(k) do { if (diag) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); dt[k] += t_ - dm; dm = t_; } } while (0)
#else
#define LV_TICK(k) do { } while (0)
#endif
  PreWin win;
  win.rs = rs;
  win.seg = L.seg;
  win.seg_lo = 0xFFFFF000u;  // nothing staged yet
  uint32_t pos = beg, produced = 0, cnt = 0;
  int code = 0;
  if (lane == 0) L.carry_j = 0;
  wave_sync();
  while (true) {
    pos = uni(pos);
    produced = uni(produced);
    if (produced >= N) break;
    if (pos >= end) { code = PQG_ERR_RLE_PAST_END; break; }  // readNext :81
    const uint32_t B = pos & ~3u;
    predecode<false, true>(win, B, w);  // stages [B, B + 264) in the segment when needed
    uint32_t js = 0, nn[4], slowm = 0, inm = 0, ec[4], ev[4];
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) {
      const uint32_t p = B + 4u * lane + b;
      const uint32_t f = (win.flg >> (8u * b)) & 0xFFu;
      const uint32_t hl = f >> 2;
      const uint32_t nx = win.nxt[b];
      const bool in = p < end;
      const bool slow = in && ((f & 2u) || p + hl > end || (!(f & 1u) && nx > end));
      nn[b] = (f & 1u) ? (nx < end ? nx : end) : nx;  // packed: readFully of what is left
      const uint32_t j = (!in || slow || nn[b] - B >= 256u) ? 0u : nn[b] - B;
      js |= j << (8u * b);
      slowm |= (slow ? 1u : 0u) << b;
      inm |= (in ? 1u : 0u) << b;
      ec[b] = win.cnt[b] | ((f & 1u) << 31);
      ev[b] = (f & 1u) ? ((win.val[b] - B) & 0xFFFFu) : (win.val[b] > 255u ? 255u : win.val[b]);
    }
    wave_sync();  // the previous window's chain / expansion reads are done
    ((u32a*)L.J[0])[lane] = js;
    LV_TICK(0);
    *(u32x4*)(L.ecnt + 4u * lane) = u32x4{ec[0], ec[1], ec[2], ec[3]};
    ((u32a*)L.eval)[2u * lane] = ev[0] | (ev[1] << 16);
    ((u32a*)L.eval)[2u * lane + 1u] = ev[2] | (ev[3] << 16);
    wave_sync();
    // J[r + 1] = J[r] o J[r] until the 2^r-th successor of the entry is missing (chain <= 2^r)
    uint32_t s = pos - B;  // chain entry (window offset)
    uint32_t nt = 1;       // tables built
    {
      uint32_t cur = js;
#pragma unroll 1
      for (uint32_t r = 0; r < 5u; r++) {
        if (uni((uint32_t)L.J[r][s]) == 0u) break;
        uint32_t nx2 = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; b++) {
          const uint32_t j = (cur >> (8u * b)) & 0xFFu;
          const uint32_t jj = L.J[r][j];
          nx2 |= (j ? jj : 0u) << (8u * b);
        }
        ((u32a*)L.J[r + 1])[lane] = nx2;
        cur = nx2;
        nt = r + 2;
        wave_sync();
      }
    }
    nt = uni(nt);
    LV_TICK(1);
    const uint32_t w0 = produced;
    uint32_t n_runs = 0, q = s;
    while (true) {  // batches of at most 64 chain headers
      // lane t: c_t = J^t(s)
      uint32_t c = s;
      bool ok = true;
#pragma unroll 1
      for (uint32_t r = 0; r < nt; r++) {
        const uint32_t x = L.J[r][c];
        const bool take = (lane >> r) & 1u;
        ok = ok && (!take || x != 0u);
        c = take ? x : c;
      }
      ok = ok && lane < (1u << nt);  // nt == 6: every lane
      const uint64_t vm = __ballot(ok);
      const uint32_t n = uni((uint32_t)__builtin_popcountll(vm));  // a prefix of the lanes
      q = uni(rdl(c, n - 1u));
      const uint32_t nq = uni((uint32_t)L.J[0][q]);
      // the batch's last header q: a run unless the chain stops at it (slow / past the section)
      const uint32_t ql = q >> 2, qb = q & 3u;
      const bool last_run = nq != 0u || (!((rdl(slowm, ql) >> qb) & 1u) && ((rdl(inm, ql) >> qb) & 1u));
      const uint32_t n_v = last_run ? n : n - 1u;
      const uint32_t cap = N - produced;
      uint32_t cc = 0, payload = 0, rend = 0;
      if (lane < n_v) {
        const uint32_t e = L.ecnt[c], v = L.eval[c];
        const bool pk = e >> 31;
        const uint32_t raw = e & 0x7FFFFFFFu;
        cc = (!pk && raw == 0u) ? cap : raw;  // Java: currentCount goes negative, the value repeats forever
        cc = cc < cap ? cc : cap;
        if (pk) {
          const uint32_t d = B + v;  // data start
          const uint64_t e2 = (uint64_t)d + (uint64_t)(raw >> 3) * (uint32_t)w;
          rend = e2 < (uint64_t)end ? (uint32_t)e2 : end;
          payload = 0x80000000u | d;
        } else {
          payload = v;
        }
      }
      const uint32_t inc = wave_incl_scan_sat(cc, cap);
      uint32_t st = __shfl_up(inc, 1);
      if (lane == 0) st = 0;
      const uint32_t total = uni(rdl(inc, WAVE - 1));
      const bool em = cc > 0u && st < cap;
      const uint32_t n_em = uni((uint32_t)__builtin_popcountll(__ballot(em)));
      if (em) {
        const uint32_t k = n_runs + lane;
        L.r_start[k] = produced + st;
        L.r_pay[k] = payload;
        L.r_end[k] = rend;
      }
      n_runs = uni(n_runs + n_em);
      produced = uni(produced + total);
      if (produced >= N || nq == 0u) break;
      s = nq;  // the chain goes on inside this window: next batch
    }
    wave_sync();
    LV_TICK(2);
    if (n_runs) expand_level_runs<WB>(L, win, n_runs, w0, produced, w, out, max_def, count_nonnull, cnt, produced < N);
    LV_TICK(3);
#ifdef PQG_DIAG
    dt[4] += 1;
#endif
    if (produced >= N) break;
    // continue after the window's last chain header q
    const uint32_t ql = q >> 2, qb = q & 3u;
    const uint32_t q_slow = (rdl(slowm, ql) >> qb) & 1u;
    const uint32_t q_in = (rdl(inm, ql) >> qb) & 1u;
    if (!q_in) {
      pos = B + q;  // at or past the section end: RLE_PAST_END next
    } else if (!q_slow) {
      pos = pick4(nn, qb, ql);  // leaves the window
    } else {
      // scalar re-decode of the header at q (readNext :80-109)
      pos = B + q;
      uint32_t hl, m, nxs, vv;
      uint64_t cnt64;
      code = slow_header_g([&](uint32_t p) { return wbyte(win, p); }, pos, end, w, hl, m, cnt64, vv, nxs);
      if (code) break;
      if (m == 0 && nxs > end) { code = PQG_ERR_EOF; break; }
      uint64_t c64 = cnt64;
      const uint32_t left = N - produced;
      if (m == 0 && c64 == 0) c64 = left;
      const uint32_t take = c64 < left ? (uint32_t)c64 : left;
      const uint32_t rd_end = m ? (nxs < end ? nxs : end) : nxs;
      wave_sync();
      if (lane == 0) {
        L.r_start[0] = produced;
        L.r_pay[0] = m ? (0x80000000u | vv) : (vv > 255u ? 255u : vv);
        L.r_end[0] = rd_end;
      }
      wave_sync();
      expand_level_runs<WB>(L, win, 1, produced, produced + take, w, out, max_def, count_nonnull, cnt, produced + take < N);
      produced += take;
      pos = rd_end;
    }
  }
  if (WB > 0) level_carry_flush(L, out);
#ifdef PQG_DIAG
  if (diag && lane == 0)
    for (int k = 0; k < 5; k++) diag[k] = dt[k];
#endif
#undef LV_TICK
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (nonnull) *nonnull = cnt;
  *err_code = code;
  return code ? produced : N;
}

// decode_levels_bl with the tile expansion specialised for the section's bit width.
__device__ __forceinline__ uint32_t decode_levels_w(LevelWaveLds& L, rsrc_t rs, uint32_t beg, uint32_t end, int w,
                                                    uint32_t N, uint8_t* out, uint32_t max_def, bool count_nonnull,
                                                    uint32_t* nonnull, int* err_code, uint64_t* diag = nullptr) {
  switch (w) {
    case 1: return decode_levels_bl<1>(L, rs, beg, end, w, N, out, max_def, count_nonnull, nonnull, err_code, diag);
    case 2: return decode_levels_bl<2>(L, rs, beg, end, w, N, out, max_def, count_nonnull, nonnull, err_code, diag);
    case 3: return decode_levels_bl<3>(L, rs, beg, end, w, N, out, max_def, count_nonnull, nonnull, err_code, diag);
    case 4: return decode_levels_bl<4>(L, rs, beg, end, w, N, out, max_def, count_nonnull, nonnull, err_code, diag);
    default: return decode_levels_bl<0>(L, rs, beg, end, w, N, out, max_def, count_nonnull, nonnull, err_code, diag);
  }
}

// 5 waves per SIMD (LDS 6.9 KiB per wave, <= 102 VGPRs): 40,000 C3 pages in 8 rounds instead of 10
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(5))) void k_levels(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                const int32_t* __restrict__ list, int n_list, uint64_t* err,
                                                ErrCount err_count, uint32_t* hint_bad) {
  // hint_bad != nullptr: the plan runs on the V2 header null counts (PQG_PAGE_NULL_COUNT), which the
  // host already put in n_values / data_begin / out_offset and the value kernels are reading beside this
  // kernel; nothing of the page's work entry is written here, the true count is only compared, and a
  // mismatch or any level error raises hint_bad (err_count's epoch): pqg_sync then re-runs level-first
  __shared__ __attribute__((aligned(16))) LevelWaveLds lvl_lds[WPB];
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  LevelWaveLds& LL = lvl_lds[wave_id()];
  PageWork pw = work[page];
  const ColumnDev cd = cols[pw.column];
  const uint32_t lane = lane_id();
  Window win;
  win.rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  const uint32_t size = uni(pw.size);
  const uint32_t nslots = uni(pw.num_slots);
  const int wr = cd.max_rep ? 32 - __builtin_clz((uint32_t)cd.max_rep) : 0;
  const int wd = cd.max_def ? 32 - __builtin_clz((uint32_t)cd.max_def) : 0;
  uint32_t rl_beg = 0, rl_end = 0, dl_beg = 0, dl_end = 0, data_beg = 0;
  bool rl_be = false, dl_be = false;  // V1 BIT_PACKED (big-endian) level sections
  int init_err = 0, init_phase = 0;
  if (pw.version == 2) {
    rl_beg = 0;
    rl_end = pw.rl_len;
    dl_beg = rl_end;
    dl_end = rl_end + pw.dl_len;
    data_beg = dl_end;
    if ((uint64_t)pw.rl_len + pw.dl_len > size) { init_err = PQG_ERR_CORRUPT; init_phase = 0; }
  } else {
    uint32_t p = 0;
    win.seek(0);
    // rl section (RunLengthBitPackingHybridValuesReader.initFromPage :40-46) when max_rep > 0
    for (int which = 0; which < 2 && !init_err; which++) {
      int maxl = which == 0 ? cd.max_rep : cd.max_def;
      int enc = which == 0 ? pw.rl_encoding : pw.dl_encoding;
      uint32_t b = p, e = p;
      if (maxl > 0 && enc == PQG_BIT_PACKED) {
        // deprecated BIT_PACKED levels (ByteBitPackingValuesReader(maxLevel, BIG_ENDIAN).initFromPage
        // :77-88): min(ceil(num_values * w / 8), available) bytes, no length prefix
        const uint32_t wl = 32 - __builtin_clz((uint32_t)maxl);
        const uint64_t want = ((uint64_t)nslots * wl + 7u) / 8u;
        const uint32_t len = (uint32_t)(want < (uint64_t)(size - p) ? want : (uint64_t)(size - p));
        b = p;
        e = p + len;
        p = e;
        if (which == 0) rl_be = true;
        else dl_be = true;
      } else if (maxl > 0) {
        if (enc != PQG_RLE) { init_err = PQG_ERR_UNSUPPORTED; init_phase = which; break; }
        if (p + 4u > size) { init_err = PQG_ERR_EOF; init_phase = which; break; }
        int32_t len = (int32_t)(uint32_t)win.read8(p);
        if (len < 0) { init_err = PQG_ERR_CORRUPT; init_phase = which; break; }
        if ((uint64_t)p + 4u + (uint32_t)len > size) { init_err = PQG_ERR_EOF; init_phase = which; break; }
        b = p + 4u;
        e = b + (uint32_t)len;
        p = e;
      } else if (enc != PQG_RLE && enc != PQG_BIT_PACKED) {
        init_err = PQG_ERR_UNSUPPORTED;
        init_phase = which;
        break;
      }
      if (which == 0) { rl_beg = b; rl_end = e; } else { dl_beg = b; dl_end = e; }
    }
    data_beg = p;
  }
  if (init_err) {
    if (lane == 0) {
      report(err, err_count, page, 0, (uint64_t)init_phase, init_err);
      if (hint_bad) {
        sst(hint_bad, err_count.epoch);
      } else {
        work[page].n_values = 0;
        work[page].data_begin = size;
      }
    }
    return;
  }
  // repetition levels first (ColumnReaderBase.checkRead reads rl then dl per slot)
  uint32_t limit = nslots;
  int code = 0;
  uint8_t* rep_out = cd.rep_levels ? cd.rep_levels + pw.slot_offset : nullptr;
  uint8_t* def_out = cd.def_levels ? cd.def_levels + pw.slot_offset : nullptr;
  uint64_t lvl_err_key = ~0ull;
  if (wr > 0) {
    uint32_t done = rl_be ? decode_levels_be(win.rs, rl_beg, rl_end, wr, nslots, rep_out, 0, false, nullptr, &code)
                          : decode_levels_w(LL, win.rs, rl_beg, rl_end, wr, nslots, rep_out, 0, false, nullptr, &code);
    if (code) {
      limit = done;
      lvl_err_key = ((uint64_t)done << 1) << 8 | (uint64_t)code;
    }
  } else if (rep_out) {
    for (uint32_t i = lane; i < nslots; i += WAVE) gst(rep_out + i, (uint8_t)0);
  }
  uint32_t nonnull = 0;
  if (wd > 0) {
    int code2 = 0;
    uint32_t done = dl_be ? decode_levels_be(win.rs, dl_beg, dl_end, wd, limit, def_out, (uint32_t)cd.max_def, true,
                                             &nonnull, &code2)
                          : decode_levels_w(LL, win.rs, dl_beg, dl_end, wd, limit, def_out, (uint32_t)cd.max_def, true,
                                             &nonnull, &code2,
#ifdef PQG_DIAG
                                            pqg_diag_wph ? pqg_diag_wph + 8 * (uint64_t)page : nullptr
#else
                                            nullptr
#endif
                                             );
    if (code2) {
      uint64_t key = (((uint64_t)done << 1) | 1ull) << 8 | (uint64_t)code2;
      if (key < lvl_err_key) lvl_err_key = key;
    }
  } else {
    nonnull = limit;  // max_def == 0: every slot holds a value
    if (def_out)
      for (uint32_t i = lane; i < limit; i += WAVE) gst(def_out + i, (uint8_t)0);
  }
  if (lane == 0) {
    if (lvl_err_key != ~0ull) {
      // level error key: slot << 1 | (0 = rl, 1 = dl) — host decodes it
      report_key(&err[3 * (uint64_t)page + 1], err_count, lvl_err_key);
    }
    if (hint_bad) {
      if (lvl_err_key != ~0ull || nonnull != pw.n_values || data_beg != pw.data_begin) sst(hint_bad, err_count.epoch);
    } else {
      work[page].n_values = nonnull;
      work[page].data_begin = data_beg;
    }
  }
}

// Exclusive scan of non-null counts per column (one workgroup per column).
__global__ __launch_bounds__(256) void k_scan_offsets(PageWork* __restrict__ work, const int32_t* __restrict__ col_pages,
                                                      const int32_t* __restrict__ col_page_start, int n_cols) {
  // thread t takes SO_PER consecutive pages per round, all loads issued first (two dependent round
  // trips per round instead of per 256 pages), one workgroup scan of the threads' totals
  constexpr int SO_PER = 16;
  const int c = blockIdx.x;
  const int b = col_page_start[c], e = col_page_start[c + 1];
  __shared__ uint64_t warp_sums[4];
  uint64_t carry = 0;
  for (int r0 = b; r0 < e; r0 += 256 * SO_PER) {
    const int i0 = r0 + (int)threadIdx.x * SO_PER;
    int pg[SO_PER];
#pragma unroll
    for (int q = 0; q < SO_PER; q++) pg[q] = i0 + q < e ? col_pages[i0 + q] : -1;
    uint64_t v[SO_PER], own = 0;
#pragma unroll
    for (int q = 0; q < SO_PER; q++) {
      v[q] = pg[q] >= 0 ? work[pg[q]].n_values : 0;
      own += v[q];
    }
    uint64_t x = own;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o);
      if ((int)lane_id() >= o) x += y;
    }
    if (lane_id() == 63) warp_sums[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t pre = carry + x - own, tot = 0;
    for (int wv = 0; wv < 4; wv++) {
      pre += wv < (int)(threadIdx.x >> 6) ? warp_sums[wv] : 0;
      tot += warp_sums[wv];
    }
#pragma unroll
    for (int q = 0; q < SO_PER; q++) {
      if (pg[q] >= 0) gst(&work[pg[q]].out_offset, pre);
      pre += v[q];
    }
    carry += tot;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// PLAIN fixed width (PlainValuesReader / FixedLenByteArrayPlainValuesReader):
// byte copy of n_values * W bytes from the data section, EOF at the first
// value that does not fit.
// A workgroup per page, its WPB waves interleaved over the page's 1 KiB rows (wave w: rows w, w + WPB, ...):
// with one wave per page a page of 160 KB was one wave's serial copy (a load, its wait and a 1 KiB store per
// row), and C5's 14,224 pages took two uneven rounds of the resident waves.
__global__ __launch_bounds__(64 * WPB) void k_plain(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                              const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                              const int32_t* __restrict__ list, int n_list, uint64_t* err,
                                              ErrCount err_count) {
  const int page = (int)blockIdx.x < n_list ? list[blockIdx.x] : -1;
  if (page < 0) return;
  const uint32_t part = wave_id();
  const PageWork pw = work[page];
  const ColumnDev cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint32_t W = uni((uint32_t)cd.elem_width);
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size);
  uint32_t n = uni(pw.n_values);
  const uint32_t avail = end > beg ? end - beg : 0;
  if ((uint64_t)n * W > avail) {
    uint32_t fit = avail / W;
    if (lane == 0 && part == 0) report(err, err_count, page, 2, fit, PQG_ERR_EOF);
    n = fit;
  }
  rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  uint8_t* dst = (uint8_t*)cd.values + pw.out_offset * W;
  const uint64_t nb = (uint64_t)n * W;
  const uint32_t src0 = beg;
  // destination-aligned 16-byte chunks
  const uintptr_t d0 = (uintptr_t)dst, d1 = d0 + nb;
  const uintptr_t a0 = (d0 + 15u) & ~(uintptr_t)15u, a1 = d1 & ~(uintptr_t)15u;
  if (a0 >= a1) {  // tiny: bytewise
    if (part == 0)
      for (uint64_t i = lane; i < nb; i += WAVE) gst(dst + i, (uint8_t)(ld32(rs, (src0 + (uint32_t)i) & ~3u) >> (((src0 + (uint32_t)i) & 3u) * 8u)));
    return;
  }
  const uint32_t head = (uint32_t)(a0 - d0), tail = (uint32_t)(d1 - a1);
  if (part == 0 && lane < head) {
    uint32_t o = src0 + lane;
    gst(dst + lane, (uint8_t)(ld32(rs, o & ~3u) >> ((o & 3u) * 8u)));
  }
  if (part == 0 && lane < tail) {
    uint64_t i = (a1 - d0) + lane;
    uint32_t o = src0 + (uint32_t)i;
    gst(dst + i, (uint8_t)(ld32(rs, o & ~3u) >> ((o & 3u) * 8u)));
  }
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  const uint64_t nchunks = (a1 - a0) >> 4;
  const uint32_t sbase = src0 + head;           // source offset of the first aligned chunk
  const uint32_t mis = sbase & 3u;
  for (uint64_t c = WAVE * part + lane; c < nchunks; c += WAVE * WPB) {
    uint32_t so = sbase + (uint32_t)(c << 4);
    v4 v;
    if (mis == 0) {
      v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)so, 0, 0);
    } else {
      uint32_t a = so & ~3u, sh = mis * 8u;
      uint32_t x0 = ld32(rs, a), x1 = ld32(rs, a + 4), x2 = ld32(rs, a + 8), x3 = ld32(rs, a + 12), x4 = ld32(rs, a + 16);
      v.x = (x0 >> sh) | (x1 << (32u - sh));
      v.y = (x1 >> sh) | (x2 << (32u - sh));
      v.z = (x2 >> sh) | (x3 << (32u - sh));
      v.w = (x3 >> sh) | (x4 << (32u - sh));
    }
    gst_nt((v4*)(a0 + (c << 4)), v);
  }
}

// PLAIN BOOLEAN (BooleanPlainValuesReader -> ByteBitPackingValuesReader(1, LE)):
// bit i of the section (bytes past the section read as 0) -> one byte 0/1.
__global__ __launch_bounds__(64 * WPB) void k_plain_bool(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                   const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                   const int32_t* __restrict__ list, int n_list, uint64_t* err,
                                                   ErrCount err_count) {
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  const PageWork pw = work[page];
  const ColumnDev cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size);
  const uint32_t n = uni(pw.n_values);
  // ByteBitPackingValuesReader.initFromPage :77-88: min(ceil(num_values/8), available) bytes
  uint64_t want = ((uint64_t)pw.num_slots + 7u) / 8u;
  uint32_t avail = end > beg ? end - beg : 0;
  uint32_t lim = beg + (uint32_t)(want < avail ? want : avail);
  rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  uint8_t* dst = (uint8_t*)cd.values + pw.out_offset;
  for (uint32_t i = lane; i < n; i += WAVE) {
    uint32_t o = beg + (i >> 3);
    uint32_t b = o < lim ? (ld32(rs, o & ~3u) >> ((o & 3u) * 8u)) & 0xFFu : 0u;
    gst(dst + i, (uint8_t)((b >> (i & 7u)) & 1u));
  }
}

// BOOLEAN values with encoding RLE (Encoding.RLE.getValuesReader :116-124, getMaxLevel :255-271:
// width 1 for BOOLEAN values; parquet-mr's V2 writer, DefaultV2ValuesWriterFactory
// .getBooleanValuesWriter :77-84): RunLengthBitPackingHybridValuesReader.initFromPage :40-46 reads
// a 4-byte LE length and slices the stream; readBoolean :58-60 = readInteger() != 0. The width-1
// hybrid stream is decoded by the level-section decoder (same decoder class in the reference),
// then an RLE run's unmasked repeated byte is folded to 0 / 1.
__global__ __launch_bounds__(64 * WPB) void k_rle_bool(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                 const PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                 const int32_t* __restrict__ list, int n_list, uint64_t* err,
                                                 ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) LevelWaveLds lvl_lds[WPB];
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  const PageWork pw = work[page];
  const ColumnDev cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint32_t beg = uni(pw.data_begin), size = uni(pw.size), n = uni(pw.n_values);
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  int code = 0;
  uint32_t b = 0, e = 0;
  if ((uint64_t)beg + 4u > size) {
    code = PQG_ERR_EOF;  // readIntLittleEndian
  } else {
    const int32_t len = (int32_t)uni(ld4_any(rs, beg));
    if (len < 0) code = PQG_ERR_CORRUPT;  // sliceStream(negative)
    else if ((uint64_t)beg + 4u + (uint32_t)len > size) code = PQG_ERR_EOF;
    b = beg + 4u;
    e = b + (uint32_t)len;
  }
  if (code) {
    if (lane == 0) report(err, err_count, page, 0, 2, code);
    return;
  }
  uint8_t* out = (uint8_t*)cd.values + pw.out_offset;
  int c2 = 0;
  const uint32_t done = decode_levels_w(lvl_lds[wave_id()], rs, b, e, 1, n, out, 1u, false, nullptr, &c2);
  if (c2 && lane == 0) report(err, err_count, page, 2, done, c2);
  __builtin_amdgcn_s_waitcnt(0);  // this wave's stores are visible to its loads
  for (uint32_t i = lane; i < done; i += WAVE) {
    const uint8_t v = *(const volatile uint8_t*)(out + i);
    if (v > 1u) gst(out + i, (uint8_t)1);
  }
}

// ---------------------------------------------------------------------------
// DELTA_BINARY_PACKED (DeltaBinaryPackingValuesReader.initFromPage :59-77, eager):
// the wave walks block headers (min delta, miniblock widths) into registers
// (block b -> lane b % 64), then per block each lane unpacks its deltas, a
// wave-wide inclusive scan (wrapping int64) turns them into values. INT32 =
// (int) of the long (readInteger :103-107).
//
// LDS segment of the page bytes for the delta decoder: the serial header chain and the
// miniblocks are read from LDS, and the segment is refilled (one coalesced 8 KiB load) only
// every few dozen blocks. Reading the page with global loads between the blocks' stores costs
// a full store drain per block (vmcnt counts stores on CDNA).
constexpr uint32_t DSEG = 8192;
// segment expansion (delta_expand_seg) for miniblocks of a multiple of 16 deltas
// block headers parsed by the vector unit (delta_hdr_v)

struct DSeg {
  rsrc_t rs;
  uint8_t* seg;
  uint32_t lo;  // segment = page bytes [lo, lo + DSEG), lo 16-aligned (uniform)

  __device__ __forceinline__ void fill(uint32_t p) {
    lo = uni(p & ~15u);
#pragma unroll
    for (uint32_t i = 0; i < DSEG; i += 16u * WAVE) {
      const uint32_t o = i + 16u * lane_id();
      *(u32x4*)(seg + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + o), 0, 0);
    }
    wave_sync();
  }
  __device__ __forceinline__ bool has(uint32_t a, uint32_t n) const {
    return a >= lo && (uint64_t)a + n <= (uint64_t)lo + DSEG;
  }
  __device__ __forceinline__ uint32_t w32(uint32_t a4) const { return *(const u32_alias*)(seg + (a4 - lo)); }
  // 8 bytes at uniform p (refills the segment when they are not staged)
  __device__ __forceinline__ uint64_t read8u(uint32_t p) {
    const uint32_t a = p & ~3u, sb = p & 3u;
    if (!has(a, 12)) fill(p);
    const uint32_t x0 = w32(a), x1 = w32(a + 4), x2 = w32(a + 8);
    return (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, sb) |
           ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sb) << 32);
  }
};

// readUnsignedVarInt / readUnsignedVarLong (BytesUtils.java:202-211, 260-269) at uniform p with
// Java shift masking; a varint not terminated within `lim` bytes gets len = lim + 1.
template <bool INT>
__device__ __forceinline__ uint64_t seg_uvar(DSeg& S, uint32_t p, uint32_t lim, uint32_t& len) {
  uint64_t value = 0, x = S.read8u(p);
  uint32_t i = 0, k = 0, b;
  for (;;) {
    b = (k < 8u) ? (uint32_t)(x >> (8u * k)) & 0xFFu : (uint32_t)S.read8u(p + k) & 0xFFu;
    if (!(b & 0x80u)) break;
    value |= (uint64_t)(b & 0x7Fu) << (i & (INT ? 31u : 63u));
    i += 7;
    k++;
    if (k >= lim) break;
  }
  len = k + 1;
  if (INT) return (uint32_t)value | (b << (i & 31u));
  return value | ((uint64_t)b << (i & 63u));
}

// Expansion of nb walked blocks (block b's facts in lane b of b_*): lane l unpacks deltas
// [l*E, l*E + E) of every block, all in one miniblock m (the lane's miniblock index and its
// position in it are the same for every block): unpacked + minDelta (wrapping, as
// loadNewBlockToBuffer :139-142), a DPP scan of the lanes' sums. The value after delta j has
// index blk_first + b*block + j; lane l STORES the E values ending one delta earlier
// (indices blk_first - 1 + b*block + l*E + q, the first taken from lane l - 1 / the carry), so
// that every lane's run is E-aligned and goes out as wide stores. The value after a stream's
// last full block is written by the caller (delta_stream).
template <class T, uint32_t E>
__device__ __forceinline__ void store_run(T* p, const T (&u)[E]) {
  constexpr uint32_t BYTES = E * sizeof(T);
  if constexpr (BYTES >= 16) {
#pragma unroll
    for (uint32_t i = 0; i < BYTES / 16; i++) {
      u32x4 v;
      __builtin_memcpy(&v, (const uint8_t*)u + 16 * i, 16);
      gst((u32x4*)p + i, v);
    }
  } else if constexpr (BYTES == 8) {
    uint64_t v;
    __builtin_memcpy(&v, u, 8);
    gst((uint64_t*)p, v);
  } else {
#pragma unroll
    for (uint32_t q = 0; q < E; q++) gst(p + q, u[q]);
  }
}

template <int W, bool NEG, uint32_t E>
__device__ __forceinline__ void delta_expand(const DSeg& S, uint32_t nb, uint32_t b_data, uint32_t b_wpos,
                                             uint32_t b_lo, uint32_t b_hi, uint32_t b_nmb, uint32_t blk_first,
                                             uint32_t block, uint32_t mbs, uint32_t n_out, uint64_t& carry,
                                             typename DictVal<W>::T* out, int page, uint64_t* err,
                                             ErrCount err_count) {
  typedef typename DictVal<W>::T T;
  const uint32_t lane = lane_id();
  const uint32_t j0 = lane * E;
  const bool lane_in = j0 < block;
  const uint32_t m = lane_in ? j0 / mbs : 0u;
  const uint32_t jm = j0 - m * mbs;
  const uint32_t mb_bytes = mbs / 8u;  // bytes per bit of width
  // wide stores need the run's first value E*W-aligned (runs start at multiples of E from `out`)
  constexpr uint32_t RUN = E * (uint32_t)sizeof(T);
  const bool wide = RUN >= 8 && (((uintptr_t)out + ((uint64_t)(blk_first - 1) * sizeof(T))) % (RUN >= 16 ? 16 : 8)) == 0 &&
                    ((uint64_t)block * sizeof(T)) % (RUN >= 16 ? 16 : 8) == 0;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t data = rdl(b_data, b), wpos = rdl(b_wpos, b), nmb = rdl(b_nmb, b);
    const uint64_t mind = ((uint64_t)rdl(b_hi, b) << 32) | rdl(b_lo, b);
    // the block's miniblock widths (<= 8 bytes at wpos)
    const uint32_t wa = wpos & ~3u, sb = wpos & 3u;
    const uint32_t y0 = S.w32(wa), y1 = S.w32(wa + 4), y2 = S.w32(wa + 8);
    const uint32_t wlo = __builtin_amdgcn_alignbyte(y1, y0, sb), whi = __builtin_amdgcn_alignbyte(y2, y1, sb);
    // width of the lane's miniblock and the byte offset of its data (sum of the widths before it)
    const uint32_t wl = m < nmb ? ((m < 4u ? wlo >> (8u * m) : whi >> (8u * (m - 4u))) & 0xFFu) : 0u;
    const uint32_t blo = m >= 4u ? wlo : (m ? wlo & ((1u << (8u * m)) - 1u) : 0u);
    const uint32_t bhi = m <= 4u ? 0u : whi & ((1u << (8u * (m - 4u))) - 1u);
    const uint32_t off = (__builtin_amdgcn_sad_u8(blo, 0u, 0u) + __builtin_amdgcn_sad_u8(bhi, 0u, 0u)) * mb_bytes;
    const uint64_t mask = wl == 64 ? ~0ull : ((1ull << wl) - 1ull);
    uint64_t loc[E];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < E; q++) {
      uint64_t d = 0;
      if (wl) {
        const uint32_t bit = (jm + q) * wl;
        const uint32_t byte = data + off + (bit >> 3);
        const uint32_t a = byte & ~3u;
        const uint32_t x0 = S.w32(a), x1 = S.w32(a + 4), x2 = S.w32(a + 8);
        const uint32_t sh = (byte - a) * 8u + (bit & 7u);  // < 32
        const uint64_t lo64 = (uint64_t)x0 | ((uint64_t)x1 << 32);
        const uint64_t v = sh == 0 ? lo64 : ((lo64 >> sh) | ((uint64_t)x2 << (64u - sh)));
        d = v & mask;
      }
      sum += lane_in ? d + mind : 0ull;
      loc[q] = sum;
    }
    const uint64_t x = wave_incl_scan_u64(sum);
    const uint64_t base_v = carry + (x - sum);
    // value before this lane's first delta: the previous lane's last value (lane 0: the carry)
    const uint64_t last = base_v + loc[E - 1];
    const uint32_t plo = (uint32_t)__shfl_up((int)(uint32_t)last, 1), phi = (uint32_t)__shfl_up((int)(uint32_t)(last >> 32), 1);
    const uint64_t prev = lane == 0 ? carry : (((uint64_t)phi << 32) | plo);
    const uint64_t k0 = (uint64_t)blk_first - 1u + (uint64_t)b * block + j0;  // index of the run's first value
    T u[E];
#pragma unroll
    for (uint32_t q = 0; q < E; q++) u[q] = (T)(q == 0 ? prev : base_v + loc[q - 1]);
    if (lane_in) {
      if (!NEG && wide && k0 + E <= n_out) {
        store_run<T, E>(out + k0, u);
      } else {
#pragma unroll
        for (uint32_t q = 0; q < E; q++) {
          const uint64_t k = k0 + q;
          if (k < n_out) {
            T v = u[q];
            if (NEG && k > 0 && (int32_t)(uint32_t)v < 0) {
              report(err, err_count, page, 2, k, PQG_ERR_CORRUPT);
              v = 0;
            }
            if (!NEG || k > 0) gst(out + k, v);
          }
        }
      }
    }
    carry += (uint64_t)rdl((uint32_t)x, 63) | ((uint64_t)rdl((uint32_t)(x >> 32), 63) << 32);
  }
}

// Segment expansion of nb walked blocks whose miniblocks hold a multiple of 16 deltas (parquet-mr
// and Arrow write 128 / 4, i.e. 32 per miniblock): lane l of a step takes segment g = 64 * step + l
// of the batch — L = 8 consecutive deltas of one miniblock of block g / (block / L) — unpacks them
// from the LDS segment at its own bit position, keeps their running sums in registers, and one
// 64-bit DPP scan of the 64 segment sums gives every segment its base: 512 deltas per scan and
// per carry step instead of one block (delta_expand: 64 * E). Values, the minDelta addition
// (loadNewBlockToBuffer :139-142, also for the unread miniblocks of a last block, whose values lie
// past the count and are not stored) and the store layout are those of delta_expand: lane l stores
// the L values ending one delta earlier (the first from lane l - 1 / the carry), as wide stores
// when the run is aligned. NEG streams (DELTA_LENGTH lengths) check every value of a step that holds a
// negative one on the per-lane stores.
// In-place inclusive prefix of a lane's deltas in two independent halves joined at the end (half the
// dependent adds of one running sum).
template <class U, uint32_t N>
__device__ __forceinline__ void delta_local_prefix(U (&v)[N]) {
  constexpr uint32_t H = N / 2;
#pragma unroll
  for (uint32_t q = 1; q < H; q++) v[q] += v[q - 1];
#pragma unroll
  for (uint32_t q = H + 1; q < N; q++) v[q] += v[q - 1];
#pragma unroll
  for (uint32_t q = H; q < N; q++) v[q] += v[H - 1];
}

// NEG (DELTA_LENGTH_BYTE_ARRAY lengths): a negative (int) value is reported as CORRUPT at its index and stored
// as 0; a step holding one takes the per-lane stores, which check every value.
template <int W, bool NEG = false>
__device__ __forceinline__ void delta_expand_seg(const DSeg& S, uint32_t nb, uint32_t b_data, uint32_t b_wpos,
                                                 uint32_t b_lo, uint32_t b_hi, uint32_t b_nmb, uint32_t blk_first,
                                                 uint32_t block, uint32_t mbs, uint32_t n_out, uint64_t& carry,
                                                 typename DictVal<W>::T* out, int page = 0, uint64_t* err = nullptr,
                                                 ErrCount err_count = ErrCount{}) {
  typedef typename DictVal<W>::T T;
  // 8 deltas per lane-step (16 measured slower: its 115 VGPRs left 4 waves per SIMD, and 5,000 pages of
  // delta_i64 took 1.2 rounds of them; at 98 VGPRs the LDS segments' 5 waves per SIMD hold every page at
  // once: delta_i64 0.370 -> 0.336 ms, C3 6.68 -> 6.61 ms, C4 10.26 -> 10.12 ms, profiles/r06/delta_l8)
  constexpr uint32_t L = 8;
  const uint32_t lane = lane_id();
  const uint32_t SB = block / L;  // segments per block
  const uint32_t n_seg = nb * SB;
  const uint32_t mb_bytes = mbs / 8u;  // bytes per bit of width
  // Runs are stored shifted by `sft` values so that every lane's L stored values start 16-byte
  // aligned whatever the page's output offset (pages of nullable columns start at any value): lane l
  // stores values [k0 + sft, k0 + sft + L), the last sft of them the first values of lane l + 1's
  // run (its u[1], u[2]: one shuffle each; u[L] is the lane's own last value). The batch's last lane
  // stores only its own values, lane 0 also the sft values before its wide run.
  constexpr uint32_t VPC = 16u / sizeof(T);  // values per 16 bytes
  const uint32_t mis = (uint32_t)((((uintptr_t)out + (uint64_t)(blk_first - 1) * sizeof(T)) % 16u) / sizeof(T));
  const uint32_t sft = mis ? VPC - mis : 0u;
  const bool wide = ((uintptr_t)out % sizeof(T)) == 0 && ((uint64_t)block * sizeof(T)) % 16 == 0;
  for (uint32_t g0 = 0; g0 < n_seg; g0 += WAVE) {
    const uint32_t g = g0 + lane;
    const bool lane_in = g < n_seg;
    const uint32_t bb = lane_in ? g / SB : 0u;
    const uint32_t j0 = (g - bb * SB) * L;  // the segment's first delta in its block
    const uint32_t m = j0 / mbs, jm = j0 - m * mbs;
    const uint32_t data = (uint32_t)__shfl((int)b_data, (int)bb), wpos = (uint32_t)__shfl((int)b_wpos, (int)bb);
    const uint32_t nmb = (uint32_t)__shfl((int)b_nmb, (int)bb);
    const uint64_t mind = ((uint64_t)(uint32_t)__shfl((int)b_hi, (int)bb) << 32) | (uint32_t)__shfl((int)b_lo, (int)bb);
    // the block's miniblock widths (<= 8 bytes at wpos), the lane's width and data offset
    const uint32_t wa = wpos & ~3u, sb = wpos & 3u;
    const uint32_t y0 = S.w32(wa), y1 = S.w32(wa + 4), y2 = S.w32(wa + 8);
    const uint32_t wlo = __builtin_amdgcn_alignbyte(y1, y0, sb), whi = __builtin_amdgcn_alignbyte(y2, y1, sb);
    const uint32_t wl = m < nmb ? ((m < 4u ? wlo >> (8u * m) : whi >> (8u * (m - 4u))) & 0xFFu) : 0u;
    const uint32_t blo = m >= 4u ? wlo : (m ? wlo & ((1u << (8u * m)) - 1u) : 0u);
    const uint32_t bhi = m <= 4u ? 0u : whi & ((1u << (8u * (m - 4u))) - 1u);
    const uint32_t dbase = data + (__builtin_amdgcn_sad_u8(blo, 0u, 0u) + __builtin_amdgcn_sad_u8(bhi, 0u, 0u)) * mb_bytes;
    T u[L + 3];
    uint64_t x;  // the wave scan of the lanes' sums (its last lane: the batch's total)
    if constexpr (W == 4) {
      // 4-byte values: the reader keeps long sums and casts them to int, whose low 32 bits depend on
      // the low 32 bits of every delta and of minDelta only: 32-bit unpack (one v_alignbit from the
      // dword pair holding the delta's first bit), sums and scan
      const uint32_t mask = wl >= 32u ? 0xFFFFFFFFu : (1u << wl) - 1u;
      const uint32_t mind32 = (uint32_t)mind;
      uint32_t loc[L];
      uint32_t sum = 0;
      // bit position relative to the dword holding the miniblock data's first byte (a page-absolute
      // bit position would wrap for data 512 MiB or more into a page)
      const uint32_t abase = dbase & ~3u;
      const uint32_t ab0 = (dbase & 3u) * 8u + jm * wl;
      // every dword pair is read unconditionally (a zero width reads the miniblock's first dword, inside
      // the staged segment, and masks it to 0): a branch per delta put an LDS round trip and its wait
      // between the deltas, 8 serial trips per step instead of one
      uint32_t x0[L], x1[L];
#pragma unroll
      for (uint32_t q = 0; q < L; q++) {
        const uint32_t a = abase + (((ab0 + q * wl) >> 5) << 2);
        x0[q] = S.w32(a);
        x1[q] = S.w32(a + 4);
      }
#pragma unroll
      for (uint32_t q = 0; q < L; q++) {
        const uint32_t d = __builtin_amdgcn_alignbit(x1[q], x0[q], (ab0 + q * wl) & 31u) & mask;
        loc[q] = lane_in ? d + mind32 : 0u;
      }
      delta_local_prefix(loc);
      sum = loc[L - 1];
      const uint32_t x32 = wave_incl_scan_u32_dpp(sum);
      // the value before the lane's first delta: the carry plus every earlier lane's sum (= lane l - 1's last)
      const uint32_t base_v = (uint32_t)carry + (x32 - sum);
#pragma unroll
      for (uint32_t q = 0; q < L + 1; q++) u[q] = (T)(q == 0 ? base_v : base_v + loc[q - 1]);
      x = x32;
    } else {
      const uint64_t mask = wl == 64 ? ~0ull : ((1ull << wl) - 1ull);
      const bool narrow = !__ballot(lane_in && wl > 32u);  // every width <= 32: two dwords per delta
      uint64_t loc[L];
      uint64_t sum = 0;
      // all reads of the step first, no branch per delta (see the 4-byte path): a zero width reads the
      // miniblock's first dwords and masks them to 0
      const uint32_t bit0 = (dbase & 3u) * 8u + jm * wl;  // relative to the dword holding dbase
      const uint32_t abase = dbase & ~3u;
      uint32_t x0[L], x1[L], x2[L];
      auto unpack = [&](auto wide_tag) {
        constexpr bool WIDE = decltype(wide_tag)::value;
#pragma unroll
        for (uint32_t q = 0; q < L; q++) {
          const uint32_t a = abase + (((bit0 + q * wl) >> 5) << 2);
          x0[q] = S.w32(a);
          x1[q] = S.w32(a + 4);
          if (WIDE) x2[q] = S.w32(a + 8);
        }
#pragma unroll
        for (uint32_t q = 0; q < L; q++) {
          const uint32_t sh = (bit0 + q * wl) & 31u;
          const uint64_t lo64 = (uint64_t)x0[q] | ((uint64_t)x1[q] << 32);
          const uint64_t d = (WIDE ? (sh == 0 ? lo64 : ((lo64 >> sh) | ((uint64_t)x2[q] << (64u - sh)))) : (lo64 >> sh)) & mask;
          loc[q] = lane_in ? d + mind : 0ull;
        }
      };
      if (narrow) unpack(std::false_type{});
      else unpack(std::true_type{});
      delta_local_prefix(loc);
      sum = loc[L - 1];
      x = wave_incl_scan_u64(sum);
      // the value before the lane's first delta: the carry plus every earlier lane's sum (= lane l - 1's last)
      const uint64_t base_v = carry + (x - sum);
#pragma unroll
      for (uint32_t q = 0; q < L + 1; q++) u[q] = (T)(q == 0 ? base_v : base_v + loc[q - 1]);
    }
    const uint64_t k0 = (uint64_t)blk_first - 1u + (uint64_t)bb * block + j0;  // index of the run's first value
    // values L + 1, L + 2 of the lane's window: lane l + 1's u[1], u[2] (only for 4-byte values: sft <= 3)
    if constexpr (VPC > 2) {
      u[L + 1] = (T)(uint32_t)__shfl_down((int)(uint32_t)u[1], 1);
      u[L + 2] = (T)(uint32_t)__shfl_down((int)(uint32_t)u[2], 1);
    } else {
      u[L + 1] = u[L + 2] = 0;
    }
    // A full step (64 lanes, its 16-byte rows inside the output): the rows are exchanged between lanes so
    // that every store instruction writes 1 KiB contiguous (lane_rows_to_tiles). Lane-contiguous runs (each
    // lane 64 bytes, four 16-byte stores 64 bytes apart) store at ~3.6 TB/s (profiles/r02/store_patterns.txt
    // 'lane-contig'); the same step with 1 KiB per instruction took delta_i64 0.335 -> 0.245 ms
    // (profiles/r06/delta_tstore). Row r of the step holds values [K + sft + VPC r, + VPC); lane l's run is
    // rows NR l .. NR l + NR - 1; store i of lane m writes row 64 i + m.
    const uint64_t K = (uint64_t)blk_first - 1u + (uint64_t)L * g0;  // value index of lane 0's u[0]
    bool neg_any = false;
    if constexpr (NEG) {
      bool ln = false;
#pragma unroll
      for (uint32_t q = 0; q < L + VPC - 1u; q++) ln |= (int32_t)(uint32_t)u[q] < 0;
      neg_any = __ballot(lane_in && ln) != 0;
    }
    if (wide && (!NEG || !neg_any) && g0 + WAVE <= n_seg && K + sft + (uint64_t)WAVE * L <= n_out) {
      if (lane == 0)  // the sft values before the first row
        for (uint32_t q = 0; q < VPC - 1u; q++)
          if (q < sft) gst(out + K + q, u[q]);
      auto tput = [&](auto s_tag) {
        constexpr uint32_t SF = decltype(s_tag)::value;
        constexpr uint32_t NR = L / VPC;  // rows per lane (4 for 8-byte values, 2 for 4-byte)
        u32x4 row[NR];
#pragma unroll
        for (uint32_t j = 0; j < NR; j++) {
          T v[VPC];
#pragma unroll
          for (uint32_t q = 0; q < VPC; q++) v[q] = u[SF + VPC * j + q];
          __builtin_memcpy(&row[j], v, 16);
        }
        u32x4 st[NR];
        lane_rows_to_tiles<NR>(row, st);
        u32x4* const base = (u32x4*)(out + K + SF);
#pragma unroll
        for (uint32_t i = 0; i < NR; i++) {
          // with 4-byte values and SF >= 2 the step's last row reaches past index K + 64 L (lane 63's last
          // value): only its values up to there go out here, the rest are the next step's head
          if (W == 4 && SF >= 2 && i == NR - 1 && lane == WAVE - 1) {
            const uint32_t* sp = (const uint32_t*)&st[i];
#pragma unroll
            for (uint32_t q = 0; q < 5u - SF; q++) gst((uint32_t*)(base + WAVE * i + lane) + q, sp[q]);
          } else {
            gst(base + WAVE * i + lane, st[i]);
          }
        }
      };
      if (sft == 0) tput(std::integral_constant<uint32_t, 0>{});
      else if (sft == 1) tput(std::integral_constant<uint32_t, 1>{});
      else if constexpr (VPC > 2) {
        if (sft == 2) tput(std::integral_constant<uint32_t, 2>{});
        else tput(std::integral_constant<uint32_t, 3>{});
      }
      if constexpr (W == 4) carry += rdl((uint32_t)x, 63);
      else carry += (uint64_t)rdl((uint32_t)x, 63) | ((uint64_t)rdl((uint32_t)(x >> 32), 63) << 32);
      continue;
    }
    if (lane_in) {
      const bool last_lane = g + 1u >= n_seg || lane == WAVE - 1u;
      // a checked store (NEG: a negative length is CORRUPT at its index and written as 0)
      // (value 0, the stream's first value, was checked and stored by delta_stream: never rewritten here)
      auto put1 = [&](uint64_t k, T v) {
        if constexpr (NEG) {
          if (k == 0) return;
          if ((int32_t)(uint32_t)v < 0) {
            report(err, err_count, page, 2, k, PQG_ERR_CORRUPT);
            v = 0;
          }
        }
        gst(out + k, v);
      };
      if (lane == 0)  // the sft values before lane 0's shifted run
        for (uint32_t q = 0; q < VPC - 1u; q++)
          if (q < sft && k0 + q < n_out) {
            if constexpr (NEG) put1(k0 + q, u[q]);
            else gst(out + k0 + q, u[q]);
          }
      const uint64_t a = k0 + sft;
      if (wide && (!NEG || !neg_any) && !last_lane && a + L <= n_out) {
        // v[q] = u[sft + q]: sft is uniform, so a branch per value of it picks the registers statically
        auto put = [&](auto s_tag) {
          constexpr uint32_t SF = decltype(s_tag)::value;
          T v[L];
#pragma unroll
          for (uint32_t q = 0; q < L; q++) v[q] = u[q + SF];
          store_run<T, L>(out + a, v);
        };
        if (sft == 0) put(std::integral_constant<uint32_t, 0>{});
        else if (sft == 1) put(std::integral_constant<uint32_t, 1>{});
        else if constexpr (VPC > 2) {
          if (sft == 2) put(std::integral_constant<uint32_t, 2>{});
          else put(std::integral_constant<uint32_t, 3>{});
        }
      } else {
        const uint64_t e = last_lane ? k0 + L : a + L;  // the last lane: its own values only
#pragma unroll
        for (uint32_t q = 0; q < L + VPC - 1u; q++) {
          const uint64_t k = k0 + q;
          if (k >= a && k < e && k < n_out) {
            if constexpr (NEG) put1(k, u[q]);
            else gst(out + k, u[q]);
          }
        }
      }
    }
    if constexpr (W == 4) carry += rdl((uint32_t)x, 63);  // (only its low 32 bits are ever stored)
    else carry += (uint64_t)rdl((uint32_t)x, 63) | ((uint64_t)rdl((uint32_t)(x >> 32), 63) << 32);
  }
}

// Any other DeltaBinaryPackingConfig the reference accepts (blocks of more than 512 values or more
// than 8 miniblocks; DuckDB writes 2048 / 8): block by block, miniblock by miniblock, 64 deltas
// per step, page bytes read with buffer loads. Same checks, in the same order, as the batched walk
// below (loadNewBlockToBuffer :118-143): widths of the used miniblocks (> 64: CORRUPT), then
// their bytes (EOF). p = position after the header; the first value is already stored.
// Every byte comes from the wave's LDS segment (refilled when a header or a 64-delta step leaves
// it): a global load between the steps' stores would wait for all of them (vmcnt counts stores),
// one drain per 64 values; with the segment it is one drain per 8 KiB of page bytes.
template <int W, bool NEG>
__device__ int delta_generic(DSeg& S, uint32_t p, uint32_t end, uint32_t block, uint32_t mbn, uint32_t mbs,
                             uint32_t total, uint32_t n_out, uint64_t carry, typename DictVal<W>::T* out, int page,
                             uint64_t* err, ErrCount err_count, uint32_t* p_end, uint32_t buffered0 = 1) {
  typedef typename DictVal<W>::T T;
  const uint32_t lane = lane_id();
  auto byte_at = [&](uint32_t a) -> uint32_t {
    if (!S.has(a & ~3u, 4)) S.fill(a);
    return uni((S.w32(a & ~3u) >> (8u * (a & 3u))) & 0xFFu);
  };
  // (buffered0 > 1: resumed at a block boundary by the batched path, values before it stored)
  uint32_t buffered = buffered0;
  uint64_t k_next = buffered0;  // value index after the next delta
  while (true) {
    p = uni(p);
    buffered = uni(buffered);
    if (buffered >= total) break;
    if (p >= end) return PQG_ERR_EOF;
    // min delta (readZigZagVarLong, Java shift masking)
    uint64_t mraw = 0;
    uint32_t i = 0, k = 0, b;
    for (;;) {
      b = byte_at(p + k);
      if (!(b & 0x80u)) break;
      mraw |= (uint64_t)(b & 0x7Fu) << (i & 63u);
      i += 7;
      k++;
      if (k >= end - p) break;
    }
    mraw |= (uint64_t)b << (i & 63u);
    if ((uint64_t)p + k + 1u > end) return PQG_ERR_EOF;
    const uint64_t mind = (uint64_t)zigzag64(mraw);
    const uint32_t wpos = p + k + 1u;
    if ((uint64_t)wpos + mbn > end) return PQG_ERR_EOF;  // readBitWidthsForMiniBlocks
    uint32_t used = 0, bufd = buffered;
    uint64_t dbytes = 0;
    for (uint32_t m = 0; m < mbn && bufd < total; m++) {
      const uint32_t wm = byte_at(wpos + m);
      if (wm > 64u) return PQG_ERR_CORRUPT;
      dbytes += (uint64_t)wm * (mbs / 8u);
      bufd += mbs;
      used++;
    }
    const uint32_t dpos = wpos + mbn;
    if ((uint64_t)dpos + dbytes > end) return PQG_ERR_EOF;  // in.slice EOF
    uint32_t mo = dpos;  // data of miniblock m
    for (uint32_t m = 0; m < used; m++) {
      const uint32_t w = byte_at(wpos + m);
      const uint64_t mask = w == 64u ? ~0ull : ((1ull << w) - 1ull);
      for (uint32_t c = 0; c < mbs; c += WAVE) {
        const uint32_t q = c + lane;
        const bool in = q < mbs;
        // the step's bytes [mo + c*w/8, mo + (c+64)*w/8 + 12) staged (<= 524 bytes)
        const uint32_t s_lo = (mo + ((c * w) >> 3)) & ~3u, s_hi = mo + (((c + WAVE) * w + 7u) >> 3) + 12u;
        if (w && !S.has(s_lo, s_hi - s_lo)) S.fill(s_lo);
        uint64_t d = 0;
        if (in && w) {
          const uint32_t bit = q * w, byte = mo + (bit >> 3), a = byte & ~3u;
          const uint32_t x0 = S.w32(a), x1 = S.w32(a + 4), x2 = S.w32(a + 8);
          const uint32_t sh = (byte - a) * 8u + (bit & 7u);
          const uint64_t lo64 = (uint64_t)x0 | ((uint64_t)x1 << 32);
          d = (sh == 0 ? lo64 : ((lo64 >> sh) | ((uint64_t)x2 << (64u - sh)))) & mask;
        }
        const uint64_t x = wave_incl_scan_u64(in ? d + mind : 0ull);
        const uint64_t kk = k_next + q;
        if (in && kk < n_out) {
          T v = (T)(carry + x);
          if (NEG && (int32_t)(uint32_t)v < 0) {
            report(err, err_count, page, 2, kk, PQG_ERR_CORRUPT);
            v = 0;
          }
          gst(out + kk, v);
        }
        carry += (uint64_t)rdl((uint32_t)x, 63) | ((uint64_t)rdl((uint32_t)(x >> 32), 63) << 32);
      }
      k_next += mbs;
      mo += w * (mbs / 8u);
    }
    p = dpos + (uint32_t)dbytes;
    buffered = bufd;
  }
  (void)block;
  *p_end = p;
  return 0;
}

// Block header chain step (loadNewBlockToBuffer :118-143: zigzag varlong min delta,
// readBitWidthsForMiniBlocks, the used miniblocks' byte count) on the VECTOR unit at uniform p:
// every lane computes the same values from its LDS copy of 20 bytes (laundered into VGPRs so the
// compiler keeps the arithmetic off the scalar unit, which the CU's four SIMDs share: the scalar
// walk issued ~230 SALU instructions per 128-value block and made k_delta scalar-issue bound).
// Only what the NEXT header's position needs is on this serial path — the varint's length (stop-bit
// mask + ctz), the used widths' byte sum (v_sad_u8) — the min delta's value is decoded afterwards
// by the block's own lane (delta_mind_v), all blocks of a batch at once. Covers the common case —
// a min delta of at most 8 varint bytes, every used width <= 64, header and data inside the
// section — and returns false otherwise, so the scalar walk raises the reference's error.
struct DeltaHdr {
  uint32_t len, wpos, dpos, next, used, dbytes;
};
// (per lane: p need not be uniform; `used` miniblocks are read)
__device__ __forceinline__ bool delta_hdr_parse(const DSeg& S, uint32_t p, uint32_t end, uint32_t mbn, uint32_t mbs,
                                                uint32_t used, DeltaHdr& h) {
  const uint32_t a = p & ~3u, sb = p & 3u;
  if (!S.has(a, 20)) return false;
  uint32_t d[5];
#pragma unroll
  for (int i = 0; i < 5; i++) d[i] = S.w32(a + 4u * i);
  asm volatile("" : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]));
  uint32_t x[4];
#pragma unroll
  for (int i = 0; i < 4; i++) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sb);  // bytes p + 4i ..
  const uint64_t lo = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
  const uint64_t stop = ~lo & 0x8080808080808080ull;  // the varint's last byte has bit 7 clear
  const uint32_t len = stop ? ((uint32_t)__builtin_ctzll(stop) >> 3) + 1u : 9u;
  h.len = len;
  h.wpos = p + len;
  // the <= 8 width bytes: bytes [len, len + 8) of x (len == 8: x[2], x[3])
  const uint32_t q = len >> 2, r = len & 3u;
  const uint32_t xa = q == 0 ? x[0] : (q == 1 ? x[1] : x[2]);
  const uint32_t xb = q == 0 ? x[1] : (q == 1 ? x[2] : x[3]);
  const uint32_t xc = q == 0 ? x[2] : x[3];
  uint32_t wl = __builtin_amdgcn_alignbyte(xb, xa, r), wh = __builtin_amdgcn_alignbyte(xc, xb, r);
  wl &= used >= 4u ? 0xFFFFFFFFu : (1u << (8u * used)) - 1u;
  wh &= used <= 4u ? 0u : (used == 8u ? 0xFFFFFFFFu : (1u << (8u * (used - 4u))) - 1u);
  // a used width > 64 (bit 7 set, or low 7 bits >= 65): the scalar walk reports CORRUPT
  const uint32_t bad = (((wl & 0x7F7F7F7Fu) + 0x3F3F3F3Fu) | wl | ((wh & 0x7F7F7F7Fu) + 0x3F3F3F3Fu) | wh) & 0x80808080u;
  h.used = used;
  h.dbytes = (__builtin_amdgcn_sad_u8(wl, 0u, 0u) + __builtin_amdgcn_sad_u8(wh, 0u, 0u)) * (mbs / 8u);
  h.dpos = h.wpos + mbn;
  h.next = h.dpos + h.dbytes;
  return len <= 8u && !bad && (uint64_t)h.dpos + h.dbytes <= end;  // (implies p + len, wpos + mbn <= end)
}
__device__ __forceinline__ bool delta_hdr_v(const DSeg& S, uint32_t p, uint32_t end, uint32_t mbn, uint32_t mbs,
                                            uint32_t buffered, uint32_t total, DeltaHdr& h) {
  // miniblocks unpacked while buffered < total (:131-135)
  const uint32_t rem = total - buffered;  // > 0
  const uint32_t used = rem >= mbn * mbs ? mbn : (rem + mbs - 1u) / mbs;  // a page's last block only
  const bool ok = delta_hdr_parse(S, p, end, mbn, mbs, used, h);
  return uni(ok ? 1u : 0u) != 0u;
}

// The min delta of a block whose header delta_hdr_v walked: zigzag varlong of `len` (<= 8) bytes at
// hp (readZigZagVarLong), decoded by the block's lane from the LDS segment.
__device__ __forceinline__ uint64_t delta_mind_v(const DSeg& S, uint32_t hp, uint32_t len) {
  const uint32_t a = hp & ~3u, sb = hp & 3u;
  const uint32_t d0 = S.w32(a), d1 = S.w32(a + 4), d2 = S.w32(a + 8);
  const uint64_t lo = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sb) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sb) << 32);
  const uint64_t v = len >= 8u ? lo : lo & ((1ull << (8u * len)) - 1ull);
  const uint64_t raw = (v & 0x7Full) | ((v >> 1) & (0x7Full << 7)) | ((v >> 2) & (0x7Full << 14)) |
                       ((v >> 3) & (0x7Full << 21)) | ((v >> 4) & (0x7Full << 28)) | ((v >> 5) & (0x7Full << 35)) |
                       ((v >> 6) & (0x7Full << 42)) | ((v >> 7) & (0x7Full << 49));
  return (raw >> 1) ^ (0ull - (raw & 1ull));  // zigzag
}

// One stream [p, end) -> out[0 .. min(want, total)). Returns 0 or the init error code (the
// reader decodes eagerly in initFromPage); *p_end = stream position after the used miniblocks,
// *total_out = the header's value count. NEG: a negative (int) value is reported as CORRUPT at
// its index and written as 0 (DELTA_LENGTH_BYTE_ARRAY lengths: in.slice(negative)).
template <int W, bool NEG>
__device__ int delta_stream(DSeg& S, uint32_t p, uint32_t end, uint32_t want, typename DictVal<W>::T* out,
                            int page, uint64_t* err, ErrCount err_count, uint32_t* p_end, uint32_t* total_out) {
  typedef typename DictVal<W>::T T;
  const uint32_t lane = lane_id();
  uint32_t len;
  p = uni(p);
  // header (DeltaBinaryPackingConfig.readConfig :43-45, totalValueCount, first value)
  if (p >= end) return PQG_ERR_EOF;
  const uint32_t block = (uint32_t)seg_uvar<true>(S, p, end - p, len);
  if ((uint64_t)p + len > end) return PQG_ERR_EOF;
  p += len;
  if (p >= end) return PQG_ERR_EOF;
  const uint32_t mbn = (uint32_t)seg_uvar<true>(S, p, end - p, len);
  if ((uint64_t)p + len > end) return PQG_ERR_EOF;
  p += len;
  // DeltaBinaryPackingConfig ctor :34-41 (double division, % 8)
  if (mbn == 0 || (int32_t)mbn < 0 || (int32_t)block < 0) return mbn == 0 ? PQG_ERR_DELTA_CONFIG : PQG_ERR_CORRUPT;
  if ((block % mbn) != 0 || ((block / mbn) % 8u) != 0) return PQG_ERR_DELTA_CONFIG;
  const uint32_t mbs = block / mbn;
  if (mbs == 0) return PQG_ERR_CORRUPT;
  if (p >= end) return PQG_ERR_EOF;
  const uint32_t total = (uint32_t)seg_uvar<true>(S, p, end - p, len);
  if ((uint64_t)p + len > end) return PQG_ERR_EOF;
  p += len;
  if ((int32_t)total < 0) return PQG_ERR_CORRUPT;
  if (p >= end) return PQG_ERR_EOF;
  const uint64_t fraw = seg_uvar<false>(S, p, end - p, len);
  if ((uint64_t)p + len > end) return PQG_ERR_EOF;
  p += len;
  const int64_t first = zigzag64(fraw);
  *total_out = total;
  // values to emit: min(want, total); want > total -> "no more value to read" at index total (caller)
  const uint32_t n_out = want > total ? total : want;
  // Value index k (0-based) of the page: k = 0 is `first`; block b covers
  // k in [1 + b*block, 1 + (b+1)*block).
  uint64_t carry = (uint64_t)first;
  if (lane == 0 && n_out > 0) {
    if (NEG && (int32_t)(uint32_t)carry < 0) {
      report(err, err_count, page, 2, 0, PQG_ERR_CORRUPT);
      gst(out, (T)0);
    } else {
      gst(out, (T)carry);
    }
  }
  // register budget of the batched expansion: block <= 512 values, <= 8 miniblocks (parquet-mr
  // and Arrow write 128 / 4); other configurations take the block-by-block path
  // (blocks of up to 2,048 values in at most 8 miniblocks of a multiple of 16 deltas — DuckDB writes 2048 / 8 —
  // take the batched walk and the segment expansion too, whose per-lane work does not depend on the block)
  const bool seg_big = block <= 2048u && mbn <= 8u && (mbs % 16u) == 0 && ((uint64_t)block * W) % 16u == 0;
  if ((block > 512u || mbn > 8u) && !seg_big)
    return delta_generic<W, NEG>(S, p, end, block, mbn, mbs, total, n_out, carry, out, page, err, err_count, p_end);
  uint32_t buffered = 1;  // Java valuesBuffered (includes the first value)
  uint32_t n_blocks = 0;
  // deltas per lane per block: the power of two >= block / 64 (it divides the block, a multiple
  // of 8, so a lane's deltas never straddle a miniblock)
  const uint32_t E = block <= 64u ? 1u : block <= 128u ? 2u : block <= 256u ? 4u : 8u;
  // bytes a block header may touch: varint (<= 10) + widths (<= 8) + read slack
  constexpr uint32_t HDR_SPAN = 40;
  while (true) {
    buffered = uni(buffered);
    p = uni(p);
    if (buffered >= total) break;
    // a batch starts with its first block fully staged (a block is <= 4126 bytes)
    if (!S.has(p, DSEG / 2 + 64)) S.fill(p);
    // ---- walk up to 64 blocks whose bytes lie in the segment (headers + data offsets)
    uint32_t b_data = 0, b_wpos = 0, b_lo = 0, b_hi = 0, b_nmb = 0, b_mv = 0;
    uint32_t nb = 0;
    const uint32_t blk_first = buffered;
    // Fast chain over the batch's full blocks (every miniblock read): on the serial path only what the
    // next header's position needs — the min delta varint's length (stop-bit mask), the width bytes' sum —
    // while lane b keeps block b's header position; then every check of delta_hdr_v and the staged-data
    // test, one lane per block, all at once. The batch is cut at the first block that fails them (its
    // successor, computed from a bad header, is never used): the loop below takes that block (slow
    // header, error, refill) and the page's last, partial block.
    {
      const uint32_t full = mbn * mbs;                   // values of a full block (<= 512)
      const uint32_t nfull = uni((total - buffered) / full);
      const uint32_t lim = nfull < 64u ? nfull : 64u;
      const uint32_t mb8 = mbs / 8u;
      const uint32_t wml = mbn >= 4u ? 0xFFFFFFFFu : (1u << (8u * mbn)) - 1u;
      const uint32_t wmh = mbn <= 4u ? 0u : (mbn == 8u ? 0xFFFFFFFFu : (1u << (8u * (mbn - 4u))) - 1u);
      uint32_t pc = p, b_p = 0, n_c = 0;
      while (n_c < lim && S.has(pc, HDR_SPAN)) {
        const uint32_t a = pc & ~3u, sb = pc & 3u;
        uint32_t d[5];
#pragma unroll
        for (int i = 0; i < 5; i++) d[i] = S.w32(a + 4u * i);
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; i++) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sb);
        const uint64_t lo = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
        const uint64_t stop = ~lo & 0x8080808080808080ull;
        const uint32_t len = stop ? ((uint32_t)__builtin_ctzll(stop) >> 3) + 1u : 9u;
        const uint32_t q = len >> 2, r = len & 3u;
        const uint32_t xa = q == 0 ? x[0] : (q == 1 ? x[1] : x[2]);
        const uint32_t xb = q == 0 ? x[1] : (q == 1 ? x[2] : x[3]);
        const uint32_t xc = q == 0 ? x[2] : x[3];
        const uint32_t wl = __builtin_amdgcn_alignbyte(xb, xa, r) & wml, wh = __builtin_amdgcn_alignbyte(xc, xb, r) & wmh;
        b_p = lane == n_c ? pc : b_p;
        pc = uni(pc + len + mbn + (__builtin_amdgcn_sad_u8(wl, 0u, 0u) + __builtin_amdgcn_sad_u8(wh, 0u, 0u)) * mb8);
        n_c = uni(n_c + 1u);
      }
      if (n_c) {
        DeltaHdr h{};
        bool ok = false;
        if (lane < n_c)
          ok = delta_hdr_parse(S, b_p, end, mbn, mbs, mbn, h) && S.has(h.dpos, h.dbytes + 12u);
        const uint64_t badm = __ballot(lane < n_c && !ok);
        const uint32_t nk = uni(badm ? (uint32_t)__builtin_ctzll(badm) : n_c);  // blocks kept
        const bool keep = lane < nk;
        b_data = keep ? h.dpos : 0u;
        b_wpos = keep ? h.wpos : 0u;
        b_lo = keep ? b_p : 0u;  // header position and varint length: the min delta follows below
        b_hi = keep ? h.len : 0u;
        b_mv = keep ? 1u : 0u;
        b_nmb = keep ? mbn : 0u;
        if (nk) {
          p = uni(rdl(h.next, nk - 1u));
          buffered = uni(buffered + nk * full);
        }
        nb = nk;
      }
    }
    while (true) {
      nb = uni(nb);
      p = uni(p);
      buffered = uni(buffered);
      if (nb >= 64u || buffered >= total) break;
      if (p >= end) return PQG_ERR_EOF;
      if (!S.has(p, HDR_SPAN)) break;  // nb > 0 here: the batch ends, the next one refills
      {
        DeltaHdr h;
        if (delta_hdr_v(S, p, end, mbn, mbs, buffered, total, h)) {
          // the block's data (+ read slack) must be staged, else the block starts the next batch
          if (!S.has(uni(h.dpos), uni(h.dbytes) + 12u)) break;
          const bool me = lane == nb;
          b_data = me ? h.dpos : b_data;
          b_wpos = me ? h.wpos : b_wpos;
          b_lo = me ? p : b_lo;  // header position and varint length: the min delta follows below
          b_hi = me ? h.len : b_hi;
          b_mv = me ? 1u : b_mv;
          b_nmb = me ? h.used : b_nmb;
          p = uni(h.next);
          buffered = uni(buffered + h.used * mbs);
          nb++;
          continue;
        }
      }
      const uint64_t mraw = seg_uvar<false>(S, p, end - p, len);  // loadNewBlockToBuffer :122-126
      if ((uint64_t)p + len > end) return PQG_ERR_EOF;
      const int64_t mind = zigzag64(mraw);
      const uint32_t wpos = p + len;
      if ((uint64_t)wpos + mbn > end) return PQG_ERR_EOF;  // readBitWidthsForMiniBlocks
      // miniblocks unpacked while buffered < total (:131-135)
      uint32_t used = 0, bufd = buffered;
      uint64_t dbytes = 0;
      const uint64_t wbytes = S.read8u(wpos);  // the <= 8 width bytes
      for (uint32_t m = 0; m < mbn && bufd < total; m++) {
        const uint32_t wm = (uint32_t)(wbytes >> (8u * m)) & 0xFFu;
        if (wm > 64u) return PQG_ERR_CORRUPT;
        dbytes += (uint64_t)wm * (mbs / 8u);
        bufd += mbs;
        used++;
      }
      const uint32_t dpos = wpos + mbn;
      if ((uint64_t)dpos + dbytes > end) return PQG_ERR_EOF;  // in.slice EOF
      // the block's data (+ read slack) must be staged, else the block starts the next batch
      if (!S.has(dpos, (uint32_t)dbytes + 12u)) break;
      const bool me = lane == nb;
      b_data = me ? dpos : b_data;
      b_wpos = me ? wpos : b_wpos;
      b_lo = me ? (uint32_t)(uint64_t)mind : b_lo;
      b_hi = me ? (uint32_t)((uint64_t)mind >> 32) : b_hi;
      b_nmb = me ? used : b_nmb;
      p = dpos + (uint32_t)dbytes;
      buffered = bufd;
      nb++;
    }
    if (nb == 0) {
      // a block whose data does not fit the segment (only blocks over 512 values: > 4 KiB of deltas): the rest of
      // the stream block by block, from this block boundary (the values before it are stored)
      if (block > 512u) {
        if (S.lo != uni(p & ~15u)) {  // a fresh segment from the block on, then the batch again
          S.fill(p);
          continue;
        }
        const uint64_t k = (uint64_t)n_blocks * block;
        if (n_blocks && k < n_out && lane == 0) {  // the value before this block
          T v = (T)carry;
          if (NEG && (int32_t)(uint32_t)v < 0) {
            report(err, err_count, page, 2, k, PQG_ERR_CORRUPT);
            v = 0;
          }
          gst(out + k, v);
        }
        return delta_generic<W, NEG>(S, p, end, block, mbn, mbs, total, n_out, carry, out, page, err, err_count, p_end,
                                     buffered);
      }
      return PQG_ERR_CORRUPT;  // unreachable: a block of at most 512 values always fits
    }
    // min deltas of the blocks delta_hdr_v walked, one lane per block (the segment holds them: it is
    // refilled only at a batch start)
    if (b_mv) {
      const uint64_t md = delta_mind_v(S, b_lo, b_hi);
      b_lo = (uint32_t)md;
      b_hi = (uint32_t)(md >> 32);
    }
    // ---- expand the walked blocks (every read from the LDS segment)
    // (the segment path stores 16-value runs per lane, shifted to 16-byte alignment: pages of
    // nullable columns, which start at any value offset, take it too)
    if ((mbs % 16u) == 0 && ((uint64_t)block * W) % 16u == 0)
      {
        if constexpr (NEG)
          delta_expand_seg<W, NEG>(S, nb, b_data, b_wpos, b_lo, b_hi, b_nmb, blk_first, block, mbs, n_out, carry, out, page,
                                   err, err_count);
        else
          delta_expand_seg<W>(S, nb, b_data, b_wpos, b_lo, b_hi, b_nmb, blk_first, block, mbs, n_out, carry, out);
      }
    else if (E == 1)
      delta_expand<W, NEG, 1>(S, nb, b_data, b_wpos, b_lo, b_hi, b_nmb, blk_first, block, mbs, n_out, carry, out, page, err, err_count);
    else if (E == 2) delta_expand<W, NEG, 2>(S, nb, b_data, b_wpos, b_lo, b_hi, b_nmb, blk_first, block, mbs, n_out, carry, out, page, err, err_count);
    else if (E == 4) delta_expand<W, NEG, 4>(S, nb, b_data, b_wpos, b_lo, b_hi, b_nmb, blk_first, block, mbs, n_out, carry, out, page, err, err_count);
    else delta_expand<W, NEG, 8>(S, nb, b_data, b_wpos, b_lo, b_hi, b_nmb, blk_first, block, mbs, n_out, carry, out, page, err, err_count);
    n_blocks += nb;
  }
  // the value after the last delta of the last block (the expansion stores values up to the one
  // before each block's last delta); only needed when that block was full
  {
    const uint64_t k = (uint64_t)n_blocks * block;
    if (n_blocks && k < n_out && lane == 0) {
      T v = (T)carry;
      if (NEG && (int32_t)(uint32_t)v < 0) {
        report(err, err_count, page, 2, k, PQG_ERR_CORRUPT);
        v = 0;
      }
      gst(out + k, v);
    }
  }
  *p_end = p;
  return 0;
}

// MODE 0: DELTA_BINARY_PACKED values. MODE 1 (DLBA): the lengths of DELTA_LENGTH_BYTE_ARRAY
// pages (DeltaLengthByteArrayValuesReader.initFromPage :44-48 reads them with this reader, then
// takes the remaining stream as the value bytes) -> ColumnDev::blen, value bytes start ->
// PageWork::aux. MODE 2 (DBA): DELTA_BYTE_ARRAY pages (DeltaByteArrayReader.initFromPage :45-48):
// prefix lengths -> bsrc, suffix lengths -> blen, suffix bytes start -> aux; then per value the
// checks of readBytes :57-79 in the reference's order and blen <- prefix + suffix length.
template <int W, int MODE = 0>
__global__ __launch_bounds__(64 * WPB) void k_delta(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                              PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                              const int32_t* __restrict__ list, int n_list, uint64_t* err,
                                              ErrCount err_count, uint32_t* __restrict__ dba_meta = nullptr) {
  typedef typename DictVal<W>::T T;
  __shared__ __attribute__((aligned(16))) uint8_t dseg_all[WPB][DSEG];
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  const PageWork pw = work[page];
  const ColumnDev cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size);
  const uint32_t want = uni(pw.n_values);
  DSeg S;
  S.rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  S.seg = dseg_all[wave_id()];
  S.lo = 0x80000000u;  // nothing staged yet (pages are < 2 GiB)
  uint32_t p_end = beg, total = 0;
  T* out = (MODE == 0 ? (T*)cd.values : MODE == 1 ? (T*)cd.blen : (T*)cd.bsrc) + pw.out_offset;
  int code = delta_stream<W, MODE == 1>(S, beg, end, want, out, page, err, err_count, &p_end, &total);
  if (code) {
    if (lane == 0) report(err, err_count, page, 0, 2, code);
    return;
  }
  uint32_t past_end = want > total ? total : 0xFFFFFFFFu;  // first index with no value
  if constexpr (MODE == 2) {
    uint32_t total2 = 0, p2 = p_end;
    code = delta_stream<4, false>(S, p_end, end, want, cd.blen + pw.out_offset, page, err, err_count, &p2, &total2);
    if (code) {
      if (lane == 0) report(err, err_count, page, 0, 2, code);
      return;
    }
    p_end = p2;
    if (want > total2 && total2 < past_end) past_end = total2;
    // readBytes checks per value i, in order: prefix / suffix length past the streams
    // (DELTA_PAST_END), suffix length < 0 (slice(negative)), suffix bytes past the page (EOF),
    // then for prefix != 0: new byte[prefix + suffix] < 0, arraycopy(previous, 0, out, 0, prefix)
    // with prefix < 0 or > previous.length. blen becomes the value length (0 past an error).
    const uint32_t n_chk = want < past_end ? want : past_end;
    const uint32_t avail = end > p_end ? end - p_end : 0;
    uint32_t* pl = cd.bsrc + pw.out_offset;
    uint32_t* sl = cd.blen + pw.out_offset;
    uint64_t s_carry = 0;
    uint32_t prev_len = 0;  // previous value of the page (empty before the first, :41)
    // PQG_PAGE_DBA_CARRY (PARQUET-246, setPreviousReader :89-95): the first value's previous is the
    // column's value out_offset - 1, known only after the earlier pages: its prefix check is made by
    // k_dba_carry, which copies the page in page order
    const bool carry = (uni(pw.pflags) & PQG_PAGE_DBA_CARRY) != 0;
    // FIXED_LEN_BYTE_ARRAY (Encoding.java :219-222): every value must be type_length bytes to fit the
    // fixed-width output
    const int32_t fixw = cd.physical_type == PQG_FIXED_LEN_BYTE_ARRAY ? cd.type_length : 0;
    uint32_t first_bad = 0xFFFFFFFFu;
    // per BIN_CHUNK-value chunk of the page, for the chunk-parallel value copy (k_dba_tail /
    // k_dba_chain / k_dba_chunks): suffix bytes before the chunk, smallest prefix length in it
    uint32_t* meta = dba_meta + 2u * (uint64_t)pw.chunk_base;
    uint32_t lmax = 0;
    // the lengths were just stored by this wave: wait for them, then read past the L1 (a line
    // shared with a neighbouring page may sit in this CU's L1 from before those stores)
    __builtin_amdgcn_s_waitcnt(0);
    // Rounds of DG chunks (BIN_CHUNK = 256 values: lane l holds values 4 l .. 4 l + 3 of a chunk): every
    // length of a round is loaded before the stores of any of it (a load issued after stores waits for
    // them), and a chunk costs one wave scan, min, max and ballot for 256 values (the lane's 4 values
    // are chained in registers), where one per 64 values left the check at half of the kernel.
    static_assert(BIN_CHUNK == 4 * WAVE, "a chunk is 4 values per lane");
    constexpr uint32_t DG = 4;
    for (uint32_t g0 = 0; g0 < n_chk; g0 += DG * BIN_CHUNK) {
    int32_t pre_g[DG][4], suf_g[DG][4];
#pragma unroll
    for (uint32_t d = 0; d < DG; d++)
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t i = g0 + d * BIN_CHUNK + 4u * lane + q;
        pre_g[d][q] = i < n_chk ? (int32_t)sld(pl + i) : 0;
        suf_g[d][q] = i < n_chk ? (int32_t)sld(sl + i) : 0;
      }
    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
    for (uint32_t d = 0; d < DG; d++) {
      const uint32_t c0 = g0 + d * BIN_CHUNK;  // the chunk's first value
      if (c0 >= n_chk) break;
      const uint32_t ib = c0 + 4u * lane;       // the lane's first value
      uint64_t sv_sum = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) sv_sum += suf_g[d][q] > 0 ? (uint64_t)suf_g[d][q] : 0;
      const uint64_t incl_l = wave_incl_scan_u64(sv_sum);
      uint64_t run = s_carry + incl_l - sv_sum;  // suffix bytes before the lane's first value
      // previous value's length (clamped at 0) for the lane's first value: the last of lane - 1
      const int32_t f3 = (int32_t)((uint32_t)pre_g[d][3] + (uint32_t)suf_g[d][3]);
      const uint32_t up = __shfl_up((uint32_t)(f3 < 0 ? 0 : f3), 1);
      uint32_t prev = lane == 0 ? prev_len : up;
      uint32_t bad_i = 0xFFFFFFFFu;
      int bad_c = 0;
      int32_t full[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t i = ib + q;
        const int32_t pre = pre_g[d][q], suf = suf_g[d][q];
        full[q] = (int32_t)((uint32_t)pre + (uint32_t)suf);
        run += suf > 0 ? (uint64_t)suf : 0;
        int c = 0;
        if (i < n_chk) {
          if (suf < 0) c = PQG_ERR_CORRUPT;
          else if (run > avail) c = PQG_ERR_EOF;
          else if (pre != 0 && (full[q] < 0 || pre < 0 || ((uint32_t)pre > prev && !(carry && i == 0)))) c = PQG_ERR_CORRUPT;
          else if (fixw && full[q] != fixw) c = PQG_ERR_CORRUPT;
        }
        if (c && bad_i == 0xFFFFFFFFu) {
          bad_i = i;
          bad_c = c;
        }
        prev = full[q] < 0 ? 0u : (uint32_t)full[q];
      }
      // the page's first invalid value (the reference throws there): reported once, every value from
      // it on gets length 0
      const uint32_t wb = uni(wave_min_u32(bad_i));
      if (wb != 0xFFFFFFFFu && first_bad == 0xFFFFFFFFu) {
        first_bad = wb;
        if (bad_i == wb) report(err, err_count, page, 2, wb, bad_c);
      }
      const uint32_t fb = uni(first_bad);
      uint32_t pmn = 0xFFFFFFFFu, lmx = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t i = ib + q;
        if (i >= n_chk) break;
        const uint32_t Lf = i >= fb ? 0u : (uint32_t)full[q];
        gst(sl + i, Lf);
        const uint32_t pf = Lf ? (uint32_t)pre_g[d][q] : 0u;  // the copy's prefix: min(prefix, length)
        pmn = pf < pmn ? pf : pmn;
        lmx = Lf > lmx ? Lf : lmx;
      }
      const uint32_t cmin = wave_min_u32(pmn), mx = wave_max_u32(lmx);
      lmax = mx > lmax ? mx : lmax;
      if (lane == 0) {
        gst(meta + 2u * (c0 / BIN_CHUNK), (uint32_t)s_carry);
        gst(meta + 2u * (c0 / BIN_CHUNK) + 1u, cmin);
      }
      prev_len = rdl(prev, WAVE - 1);
      s_carry += rdl((uint32_t)incl_l, WAVE - 1) | ((uint64_t)rdl((uint32_t)(incl_l >> 32), WAVE - 1) << 32);
    }
    }
    // chunks past the checked values hold no bytes
    const uint32_t nch = (uint32_t)(((uint64_t)pw.num_slots + BIN_CHUNK - 1) / BIN_CHUNK);
    for (uint32_t j = (n_chk + BIN_CHUNK - 1) / BIN_CHUNK + lane; j < nch; j += WAVE) {
      gst(meta + 2u * j, (uint32_t)s_carry);
      gst(meta + 2u * j + 1u, 0u);
    }
    // a value longer than the LDS value buffers sends the page to the serial copy
    if (lane == 0) work[page].reserved = carry ? 2u : lmax > DBA_VB ? 1u : 0u;
    // values past an error or past the streams hold length 0 (blen was cleared before the launch)
  }
  if (past_end != 0xFFFFFFFFu && lane == 0) report(err, err_count, page, 2, past_end, PQG_ERR_DELTA_PAST_END);
  if (MODE != 0 && lane == 0) work[page].aux = p_end;
}

// ---------------------------------------------------------------------------
// ParquetReadRouter batch: run r unpacks counts[r] LSB-first values of width w.
__global__ __launch_bounds__(256) void k_unpack_runs(int w, const uint8_t* __restrict__ in, uint64_t in_bytes,
                                                     const uint64_t* __restrict__ in_off, const uint32_t* __restrict__ counts,
                                                     const uint64_t* __restrict__ out_off, int32_t* __restrict__ out,
                                                     int n_runs) {
  const int r = blockIdx.y;
  if (r >= n_runs) return;
  const uint32_t cnt = counts[r];
  rsrc_t rs = make_rsrc(in + in_off[r], in_bytes - in_off[r]);
  int32_t* o = out + out_off[r];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    uint32_t v = 0;
    if (w) {
      uint64_t bit = (uint64_t)i * (uint32_t)w;
      uint32_t byte = (uint32_t)(bit >> 3), a = byte & ~3u;
      uint64_t x = (uint64_t)ld32(rs, a) | ((uint64_t)ld32(rs, a + 4) << 32);
      x >>= (byte - a) * 8u + (uint32_t)(bit & 7u);
      v = w == 32 ? (uint32_t)x : (uint32_t)x & ((1u << w) - 1u);
    }
    gst(o + i, (int32_t)v);
  }
}

#ifdef PQG_DIAG
}  // namespace pqg
extern "C" int pqg_diag_nostore_set(int v) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg::pqg_diag_nostore), &v, sizeof(v)) == hipSuccess ? 0 : 3;
}
extern "C" int pqg_diag_set(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg::pqg_diag_buf), &p, sizeof(p)) == hipSuccess ? 0 : 3;
}
extern "C" int pqg_diag_wph_set(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg::pqg_diag_wph), &p, sizeof(p)) == hipSuccess ? 0 : 3;
}
extern "C" int pqg_diag_rt_set(void* walk, void* chunk) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg::pqg_diag_wrt), &walk, sizeof(walk)) == hipSuccess &&
                 hipMemcpyToSymbol(HIP_SYMBOL(pqg::pqg_diag_xrt), &chunk, sizeof(chunk)) == hipSuccess
             ? 0
             : 3;
}
namespace pqg {
#endif

// ---------------------------------------------------------------------------
// Launchers (host side of this translation unit)

#define PQG_LAUNCH_ARGS bytes, n_bytes, work, cols, list, n, err, err_count

hipError_t launch_dict(int width, hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                       const ColumnDev* cols, const int32_t* list, int n, uint64_t* rec, uint32_t* chunk_run,
                       const uint64_t* chunks, uint32_t n_chunks, uint64_t* pstat, uint32_t* flags, uint32_t epoch,
                       bool fused, uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  const uint32_t n_walk = (uint32_t)(n + WPB - 1) / WPB, n_tile = (n_chunks + WPB - 1) / WPB;
  const dim3 blk(64 * WPB);
  if (fused) {
    if (width == 8)
      hipLaunchKernelGGL(k_dict_fused<8>, dim3(n_walk + n_tile), blk, 0, st, bytes, n_bytes, work, cols, list, n, n_walk,
                         rec, chunk_run, chunks, n_chunks, pstat, flags, epoch, err, err_count);
    else
      hipLaunchKernelGGL(k_dict_fused<4>, dim3(n_walk + n_tile), blk, 0, st, bytes, n_bytes, work, cols, list, n, n_walk,
                         rec, chunk_run, chunks, n_chunks, pstat, flags, epoch, err, err_count);
    return hipGetLastError();
  }
  // split mode (pqg_sync's re-run after a fused-kernel timeout): walk, then expand, two launches
  if (width == 8) {
    hipLaunchKernelGGL(k_dict_runs<8>, dim3(n_walk), blk, 0, st, bytes, n_bytes, work, cols, list, n, rec, chunk_run,
                       pstat, flags, epoch, err, err_count);
    if (n_tile)
      hipLaunchKernelGGL(k_dict_tiles<8>, dim3(n_tile), blk, 0, st, bytes, n_bytes, work, cols, rec, chunk_run, chunks,
                         n_chunks, pstat, err, err_count);
  } else {
    hipLaunchKernelGGL(k_dict_runs<4>, dim3(n_walk), blk, 0, st, bytes, n_bytes, work, cols, list, n, rec, chunk_run,
                       pstat, flags, epoch, err, err_count);
    if (n_tile)
      hipLaunchKernelGGL(k_dict_tiles<4>, dim3(n_tile), blk, 0, st, bytes, n_bytes, work, cols, rec, chunk_run, chunks,
                         n_chunks, pstat, err, err_count);
  }
  return hipGetLastError();
}

hipError_t launch_dict_ids(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const int32_t* list, int n, uint64_t* rec, uint32_t* chunk_run,
                           const uint64_t* chunks, uint32_t n_chunks, uint64_t* pstat, uint32_t* flags,
                           uint32_t epoch, bool fused, uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  const uint32_t n_walk = (uint32_t)(n + WPB - 1) / WPB, n_tile = (n_chunks + WPB - 1) / WPB;
  const dim3 blk(64 * WPB);
  if (fused) {
    hipLaunchKernelGGL((k_dict_fused<4, true>), dim3(n_walk + n_tile), blk, 0, st, bytes, n_bytes, work, cols, list, n,
                       n_walk, rec, chunk_run, chunks, n_chunks, pstat, flags, epoch, err, err_count);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_dict_runs<4>, dim3(n_walk), blk, 0, st, bytes, n_bytes, work, cols, list, n, rec, chunk_run,
                     pstat, flags, epoch, err, err_count);
  if (n_tile)
    hipLaunchKernelGGL((k_dict_tiles<4, true>), dim3(n_tile), blk, 0, st, bytes, n_bytes, work, cols, rec, chunk_run,
                       chunks, n_chunks, pstat, err, err_count);
  return hipGetLastError();
}

hipError_t launch_dict_dd(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                          const ColumnDev* cols, const int32_t* list, int n, uint64_t* rec, uint32_t* chunk_run,
                          const uint64_t* chunks, uint32_t n_chunks, uint64_t* pstat, uint32_t* flags,
                          uint32_t epoch, bool fused, uint64_t* err, ErrCount err_count, uint64_t* sums,
                          const int32_t* dd_cols, const int32_t* dd_start, int n_dd_cols, uint32_t dd_region,
                          bool global, hipEvent_t entries_ready) {
  if (n <= 0) return hipSuccess;
  const uint32_t n_walk = (uint32_t)(n + WPB - 1) / WPB, n_tile = (n_chunks + WPB - 1) / WPB;
  const dim3 blk(64 * WPB);
  if (fused) {
    if (global)
      hipLaunchKernelGGL(k_dict_fused_dd<DD_IDS>, dim3(n_walk + n_tile), blk, 0, st, bytes, n_bytes, work, cols, list, n,
                         n_walk, rec, chunk_run, chunks, n_chunks, pstat, flags, epoch, err, err_count, sums);
    else
      hipLaunchKernelGGL(k_dict_fused_dd<DD_SUMS>, dim3(n_walk + n_tile), blk, 0, st, bytes, n_bytes, work, cols, list, n,
                         n_walk, rec, chunk_run, chunks, n_chunks, pstat, flags, epoch, err, err_count, sums);
  } else {
    hipLaunchKernelGGL(k_dict_runs<4>, dim3(n_walk), blk, 0, st, bytes, n_bytes, work, cols, list, n, rec, chunk_run,
                       pstat, flags, epoch, err, err_count);
    if (n_tile) {
      if (global)
        hipLaunchKernelGGL(k_dict_tiles_dd<DD_IDS>, dim3(n_tile), blk, 0, st, bytes, n_bytes, work, cols, rec, chunk_run,
                           chunks, n_chunks, pstat, err, err_count, sums);
      else
        hipLaunchKernelGGL(k_dict_tiles_dd<DD_SUMS>, dim3(n_tile), blk, 0, st, bytes, n_bytes, work, cols, rec, chunk_run,
                           chunks, n_chunks, pstat, err, err_count, sums);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // (the entries, walked on another queue: the ids above never read them)
  if (entries_ready && hipStreamWaitEvent(st, entries_ready, 0) != hipSuccess) return hipErrorUnknown;
  if (global && n_tile) {  // the chunks' byte sums from the stored ids (entry lengths gathered from HBM)
    hipLaunchKernelGGL(k_dd_gsums, dim3(n_tile), blk, 0, st, work, cols, chunks, n_chunks, pstat, sums);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_dd_bases, dim3(n_dd_cols), dim3(256), 0, st, work, cols, chunks, dd_cols, dd_start, sums);
  e = hipGetLastError();
  if (e != hipSuccess || !n_tile) return e;
  if (global) {  // a workgroup per chunk
    hipLaunchKernelGGL(k_dd_gstr, dim3(n_chunks), blk, 0, st, bytes, n_bytes, work, cols, chunks, n_chunks, pstat, sums,
                       err, err_count);
    return hipGetLastError();
  }
  const uint32_t dd_lds_bytes = 16u + ((dd_region + 15u) & ~15u) + WPB * DDG_WAVE_BYTES;
  if (n_chunks <= DD_SPLIT_MAX_CHUNKS)  // few chunks: a workgroup per chunk
    hipLaunchKernelGGL(k_dd_str<CH_TILES / WPB>, dim3(n_chunks), blk, dd_lds_bytes, st, bytes, n_bytes, work, cols, chunks,
                       n_chunks, pstat, sums, err, err_count, dd_region);
  else
    hipLaunchKernelGGL(k_dd_str<CH_TILES>, dim3(n_tile), blk, dd_lds_bytes, st, bytes, n_bytes, work, cols, chunks, n_chunks,
                       pstat, sums, err, err_count, dd_region);
  return hipGetLastError();
}

hipError_t launch_levels(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work, const ColumnDev* cols,
                         const int32_t* list, int n, uint64_t* err, ErrCount err_count, uint32_t* hint_bad) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_levels, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS, hint_bad);
  return hipGetLastError();
}

hipError_t launch_scan(hipStream_t st, PageWork* work, const int32_t* col_pages, const int32_t* col_page_start,
                       int n_cols) {
  if (n_cols <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan_offsets, dim3(n_cols), dim3(256), 0, st, work, col_pages, col_page_start, n_cols);
  return hipGetLastError();
}

hipError_t launch_plain(int kind, hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                        const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  if (kind == 1) hipLaunchKernelGGL(k_plain_bool, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS);
  else if (kind == 2) hipLaunchKernelGGL(k_rle_bool, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS);
  else hipLaunchKernelGGL(k_plain, dim3(n), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS);  // a workgroup per page
  return hipGetLastError();
}

hipError_t launch_delta(int width, hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                        const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  if (width == 8) hipLaunchKernelGGL(k_delta<8>, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS);
  else hipLaunchKernelGGL(k_delta<4>, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS);
  return hipGetLastError();
}

hipError_t launch_dlba_lengths(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                               const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_delta<4, 1>), dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS);
  return hipGetLastError();
}

hipError_t launch_dba_lengths(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                              const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count,
                              uint32_t* dba_meta) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_delta<4, 2>), dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, PQG_LAUNCH_ARGS, dba_meta);
  return hipGetLastError();
}

hipError_t launch_unpack_runs(hipStream_t st, int w, const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                              const uint32_t* counts, const uint64_t* out_off, int32_t* out, int n_runs,
                              uint32_t max_count) {
  if (n_runs <= 0) return hipSuccess;
  uint32_t gx = (max_count + 255u) / 256u;
  if (gx == 0) gx = 1;
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(k_unpack_runs, dim3(gx, n_runs), dim3(256), 0, st, w, in, in_bytes, in_off, counts, out_off, out,
                     n_runs);
  return hipGetLastError();
}

}  // namespace pqg
