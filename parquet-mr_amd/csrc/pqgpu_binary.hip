// pqgpu_binary.hip — CDNA4 (gfx950) kernels for variable-length and byte-transposed values:
//
//   k_bss            BYTE_STREAM_SPLIT (ByteStreamSplitValuesReader.java:30-114): byte k of value i
//                    sits in stream k; lanes read 4 consecutive values of every stream as dwords
//                    and transpose them in registers.
//   k_bin_walk       PLAIN BYTE_ARRAY (BinaryPlainValuesReader.java:35-61) and the entries of a
//                    BYTE_ARRAY dictionary page (PlainBinaryDictionary, PlainValuesDictionary.java:87-113):
//                    the chain of 4-byte length prefixes, followed in parallel (below).
//   k_bin_dict_map   RLE_DICTIONARY BYTE_ARRAY pages: dictionary id -> (length, source) of the entry.
//   k_gather_fixed   FIXED_LEN_BYTE_ARRAY / INT96 dictionary pages: id -> fixed-width entry bytes.
//   k_bin_scan_*     exclusive scan of value lengths -> int64 offsets of every BYTE_ARRAY column.
//   k_bin_copy       value bytes -> the column's byte buffer, one wave per 256-value chunk,
//                    output-dword parallel (every lane stores whole dwords).
//
// Output of a BYTE_ARRAY column (include/pqgpu.h): offsets[n + 1] (int64) + the concatenated
// bytes — the Binary values the reference's ValuesReader.readBytes returns, in slot order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

// ---------------------------------------------------------------------------
// BYTE_STREAM_SPLIT. initFromPage :67-97: available % W != 0 and "more encoded values than the
// page's value count" fail at init; reading past the encoded values fails at that value
// (nextElementByteOffset :43-50).
__global__ __launch_bounds__(64 * WPB) void k_bss(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                  const PageWork* __restrict__ work,
                                                  const ColumnDev* __restrict__ cols,
                                                  const int32_t* __restrict__ list, int n_list, uint64_t* err,
                                                  ErrCount err_count) {
  // a workgroup per page, its waves interleaved over the page's 256-value steps
  const int page = (int)blockIdx.x < n_list ? list[blockIdx.x] : -1;
  if (page < 0) return;
  const uint32_t part = wave_id();
  const PageWork pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint32_t W = uni((uint32_t)cd.elem_width);
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size);
  const uint32_t avail = end > beg ? end - beg : 0;
  if (W == 0 || avail % W != 0 || pw.num_slots < avail / W) {
    if (lane == 0 && part == 0) report(err, err_count, page, 0, 2, PQG_ERR_CORRUPT);
    return;
  }
  const uint32_t count = avail / W;
  uint32_t n = uni(pw.n_values);
  if (n > count) {
    if (lane == 0 && part == 0) report(err, err_count, page, 2, count, PQG_ERR_EOF);
    n = count;
  }
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  uint8_t* out = (uint8_t*)cd.values + pw.out_offset * W;
  if (W == 4 || W == 8) {
    // lane: values [i0, i0 + 4); stream k -> one dword holding byte k of those 4 values
    for (uint32_t i0 = 4u * (lane + WAVE * part); i0 < n; i0 += 4u * WAVE * WPB) {
      uint32_t d[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) d[k] = k < W ? ld4_any(rs, beg + k * count + i0) : 0u;
      uint32_t lo[4], hi[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        const uint32_t sh = 8u * j;
        lo[j] = ((d[0] >> sh) & 0xFFu) | (((d[1] >> sh) & 0xFFu) << 8) | (((d[2] >> sh) & 0xFFu) << 16) |
                (((d[3] >> sh) & 0xFFu) << 24);
        hi[j] = ((d[4] >> sh) & 0xFFu) | (((d[5] >> sh) & 0xFFu) << 8) | (((d[6] >> sh) & 0xFFu) << 16) |
                (((d[7] >> sh) & 0xFFu) << 24);
      }
      if (W == 4) {
        uint32_t* o = (uint32_t*)out + i0;
        if (i0 + 4 <= n && ((uintptr_t)o & 15u) == 0) {
          gst_nt((u32x4*)o, u32x4{lo[0], lo[1], lo[2], lo[3]});
        } else {
#pragma unroll
          for (uint32_t j = 0; j < 4; j++)
            if (i0 + j < n) gst(o + j, lo[j]);
        }
      } else {
        uint32_t* o = (uint32_t*)out + 2 * i0;
        const uint32_t ib = i0 - 4u * lane;  // the wave's first value this step (uniform)
        if (ib + 4u * WAVE <= n && ((uintptr_t)out & 15u) == 0) {
          // a full step: the lanes' 32-byte runs exchanged so that each store writes 1 KiB contiguous
          const u32x4 row[2] = {u32x4{lo[0], hi[0], lo[1], hi[1]}, u32x4{lo[2], hi[2], lo[3], hi[3]}};
          u32x4 st[2];
          lane_rows_to_tiles<2>(row, st);
          u32x4* const base = (u32x4*)((uint32_t*)out + 2 * ib);
          gst_nt(base + lane, st[0]);
          gst_nt(base + WAVE + lane, st[1]);
        } else if (i0 + 4 <= n && ((uintptr_t)o & 15u) == 0) {
          gst_nt((u32x4*)o, u32x4{lo[0], hi[0], lo[1], hi[1]});
          gst_nt((u32x4*)(o + 4), u32x4{lo[2], hi[2], lo[3], hi[3]});
        } else {
#pragma unroll
          for (uint32_t j = 0; j < 4; j++)
            if (i0 + j < n) {
              gst(o + 2 * j, lo[j]);
              gst(o + 2 * j + 1, hi[j]);
            }
        }
      }
    }
  } else {
    // FIXED_LEN_BYTE_ARRAY of any width: one output byte per lane and step
    const uint64_t nb = (uint64_t)n * W;
    for (uint64_t o = lane + WAVE * part; o < nb; o += WAVE * WPB) {
      const uint32_t i = (uint32_t)(o / W), k = (uint32_t)(o % W);
      const uint32_t a = beg + k * count + i;
      gst(out + o, (uint8_t)(ld32(rs, a & ~3u) >> ((a & 3u) * 8u)));
    }
  }
}

// ---------------------------------------------------------------------------
// Length-prefixed values: [len: 4 bytes LE][len bytes] repeated (BinaryPlainValuesReader.readBytes
// :35-42: readIntLittleEndian, then in.slice(len)).
//
// The chain of positions is serial (each length gives the next position). It is followed a
// 1 KiB window at a time without a serial step per value:
//   1. every lane tests its 16 byte positions p of the window: p is a CANDIDATE when a value
//      could start there (4 length bytes inside the section, 0 <= len, p + 4 + len <= end);
//   2. the candidates are compacted in position order into LDS with their successor p + 4 + len;
//   3. every true value start is a candidate, and the first candidate is the current position.
//      Candidate i is followed by the true chain exactly when succ(i) == pos(i + 1); a batch of
//      64 candidates whose successors all match is accepted in one step. A mismatch (a false
//      candidate inside a value's bytes — rare: a length prefix read from string bytes is
//      almost always larger than the section) is resolved by a search for succ(i) in the list.
// So the per-value work is parallel; the serial steps are one per 64 values plus one per
// false candidate that sits between two true ones.
constexpr uint32_t COPY_BTAB = 320;  // block table entries per wave (chunks of up to 5 KiB)
constexpr uint32_t BW_WIN = 2048;    // window bytes
constexpr uint32_t BW_Q = BW_WIN / 64;     // positions per lane (16 or 32)
constexpr uint32_t BW_CAP = BW_WIN / 4;    // candidates per pass over a tile (more: the tile is taken in parts)
static_assert(BW_Q == 16 || BW_Q == 32, "window of 1 or 2 KiB");

struct BinWalkLds {
  uint2 pn[BW_CAP];       // candidate positions (ascending; bit 31: accepted) and successors (p + 4 + len)
  uint2 mr[WAVE];         // lane l: candidate mask of window offsets [BW_Q l, BW_Q l + BW_Q), index of its first
  uint32_t cut;           // position of candidate BW_CAP (the end of this pass) when there are more
};
static_assert(BW_Q == 32, "window offset -> candidate index through one 32-bit mask per lane");

// Candidate index of window offset so (< BW_WIN), or 0xFFFF when no candidate starts there: the
// owning lane's mask and first index (4.6 KB of LDS per wave instead of a 2,048-entry index table,
// so 6 walking waves fit a SIMD where 4 did).
__device__ __forceinline__ uint32_t bw_index(const BinWalkLds& L, uint32_t so) {
  const uint2 e = L.mr[so >> 5];
  const uint32_t bit = so & 31u;
  return (e.x >> bit) & 1u ? e.y + (uint32_t)__builtin_popcount(e.x & ((1u << bit) - 1u)) : 0xFFFFu;
}

// Window bytes of one lane: [B + BW_Q * lane, + BW_Q + 4) as BW_Q / 4 + 1 dwords.
struct BwBytes {
  u32x4 a, b;  // b unused for 16 positions
  uint32_t x;
};
__device__ __forceinline__ BwBytes bw_load(rsrc_t rs, uint32_t B) {
  const uint32_t o = B + BW_Q * lane_id();
  BwBytes r;
  r.a = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 0);
  if constexpr (BW_Q == 32) r.b = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o + 16u), 0, 0);
  else r.b = u32x4{0, 0, 0, 0};
  r.x = ld32(rs, o + BW_Q);
  return r;
}

// Error of a value whose length prefix starts at p (not a candidate).
__device__ __forceinline__ int bin_value_error(rsrc_t rs, uint32_t p, uint32_t end, bool dict) {
  if ((uint64_t)p + 4u > end) return PQG_ERR_EOF;  // readIntLittleEndian: EOFException
  const int32_t len = (int32_t)ld4_any(rs, p);
  if (len < 0) return PQG_ERR_CORRUPT;             // slice(negative): IllegalArgumentException
  return dict ? PQG_ERR_CORRUPT : PQG_ERR_EOF;     // slice past the end: EOFException (dictionary: CORRUPT)
}

// The window's accepted values are marked in the candidate list (bit 31 of pos) during the walk
// and stored after it, once the next window's bytes have been requested: a load issued after
// stores would wait for them (vmcnt counts stores), so every window costs one memory latency,
// not two.
// Result of a walk: where the chain left it (the next value's position), the values produced, and
// the error that stopped it (0: none).
struct BinWalkEnd {
  uint32_t pos, produced;
  int code;
};

// The walk from `beg` until N values are produced, an error, or (stop, tile-aligned) the chain
// reaches `stop`; values go to out_len / out_src [0, produced).
__device__ __forceinline__ BinWalkEnd bin_walk_core(BinWalkLds& L, rsrc_t rs, uint32_t beg, uint32_t end, uint32_t N,
                                                    uint32_t* out_len, uint32_t* out_src, bool dict,
                                                    uint32_t stop = 0xFFFFFFFFu) {
  const uint32_t lane = lane_id();
  uint32_t pos = uni(beg), produced = 0;
  int code = 0;
  // fixed BW_WIN tiles of the page; the tile after the current one is in flight
  // (a page is one wave's serial chain: with few pages per CU the tile latency is not hidden by
  // other waves, so the wave itself keeps several tiles in flight)
  uint32_t B = pos & ~(BW_WIN - 1u);
  BwBytes cur_b = bw_load(rs, B);
  BwBytes nxt_b = bw_load(rs, B + BW_WIN);
  // Short lengths first (< 256, the usual string): the byte before a length prefix then never reads
  // as a candidate (it is 256 x the true length plus a string byte), so a tile's candidates link one
  // to the next and the binary lifting below is not needed. A value start the short pass does not
  // list (a longer value) sends the tile through the pass with every length.
  bool fast = true;
  while (true) {
    pos = uni(pos);
    produced = uni(produced);
    B = uni(B);
    if (produced >= N || pos >= stop) break;
    if ((uint64_t)pos + 4u > end) { code = PQG_ERR_EOF; break; }
    // ---- candidates of the tile [B, B + BW_WIN) holding pos (its bytes are in cur_b)
    const uint32_t base = B + BW_Q * lane;
    uint32_t d[BW_Q / 4 + 1];
    d[0] = cur_b.a.x; d[1] = cur_b.a.y; d[2] = cur_b.a.z; d[3] = cur_b.a.w;
    if constexpr (BW_Q == 32) {
      d[4] = cur_b.b.x; d[5] = cur_b.b.y; d[6] = cur_b.b.z; d[7] = cur_b.b.w;
    }
    d[BW_Q / 4] = cur_b.x;
    uint32_t m = 0;
    // 32-bit test (pages < 2 GiB): 0 <= len <= end - (p + 4), i.e. rem = end - 4 - p >= 0 and
    // len <= rem as unsigned (a negative len is >= 2^31 > rem)
    const int32_t rem0 = (int32_t)(end - 4u - base);
#pragma unroll
    for (uint32_t q = 0; q < BW_Q; q++) {
      const uint32_t len = __builtin_amdgcn_alignbyte(d[(q >> 2) + 1], d[q >> 2], q & 3u);
      const int32_t rem = rem0 - (int32_t)q;
      const bool c = rem >= 0 && len <= (uint32_t)rem && (!fast || len < 256u);
      m |= (c ? 1u : 0u) << q;
    }
    if (base < pos) m &= pos - base >= BW_Q ? 0u : ~((1u << (pos - base)) - 1u);
    uint32_t total;
    const uint32_t rank = wave_excl_scan_u32((uint32_t)__builtin_popcount(m), &total);
    // one iteration per candidate of this lane (about BW_Q / average value size), not one per
    // position: the per-position form spent most of the walk's scalar and vector instructions
    // on exec-mask branches (profiles/r02/final1/strpmc)
    {
      uint32_t mm = m, r = rank;
      while (mm) {
        const uint32_t q = (uint32_t)__builtin_ctz(mm);
        mm &= mm - 1u;
        if (r < BW_CAP) {
          // d[q / 4] and d[q / 4 + 1] by selects (no dynamic register indexing)
          const uint32_t i = q >> 2;
          uint32_t lo = d[0], hi = d[1];
#pragma unroll
          for (uint32_t t = 1; t < BW_Q / 4; t++) {
            const bool s = i == t;
            lo = s ? d[t] : lo;
            hi = s ? d[t + 1] : hi;
          }
          const uint32_t nx = base + q + 4u + __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
          *(uint64_t*)&L.pn[r] = (uint64_t)(base + q) | ((uint64_t)nx << 32);
        } else if (r == BW_CAP) {
          L.cut = base + q;
        }
        r++;
      }
    }
    L.mr[lane] = uint2{m, rank};
    wave_sync();
    total = uni(total);
    // this pass covers [pos, eff_end): the whole tile, or up to the first candidate past the cap
    const uint32_t eff_end = total > BW_CAP ? uni(L.cut) : B + BW_WIN;
    if (total > BW_CAP) total = BW_CAP;
    if (total == 0 || L.pn[0].x != pos) {  // the current position cannot hold a value
      if (fast) {  // (or a longer one: the tile again with every length)
        fast = false;
        wave_sync();
        continue;
      }
      code = bin_value_error(rs, pos, end, dict);
      break;
    }
    // ---- follow the chain through the candidate list, 64 candidates at a time: every lane
    // looks up the candidate index of its successor (window offset -> index table). Where the
    // candidates link one to the next (the usual case: every candidate is a value start), the
    // batch's chain is the run of consecutive links from lane 0, found by one ballot; otherwise
    // the chain is walked from lane 0 with one v_readlane per value (false candidates — a length
    // read from a shifted prefix, e.g. the byte before a small length — are never reached).
    uint32_t i0 = 0, got = 0;
    bool leave = false;  // next position lies past the window
    bool retry = false;  // the short pass missed a value start: this tile again with every length
    while (true) {
      i0 = uni(i0);
      got = uni(got);
      const uint32_t k = i0 + lane;
      const uint32_t s = k < total ? L.pn[k].y : 0xFFFFFFFFu;
      const uint32_t so = s - B;
      const uint32_t t = so < BW_WIN ? bw_index(L, so) : 0xFFFFu;
      const bool hit = t < total && t > k && t - i0 < WAVE;
      const uint32_t J = hit ? t - i0 : WAVE;
      uint64_t mask = 0;
      uint32_t last = 0;
      // lanes 0 .. run are the chain: lane l < run links to lane l + 1 (lane 63 never "links":
      // its successor is outside the batch); from lane run the chain continues by readlanes only
      // when its successor is a later lane of the batch (a false candidate in between)
      const uint64_t next1 = __ballot(hit && t == k + 1);
      const uint32_t run = ~next1 ? (uint32_t)__builtin_ctzll(~next1) : WAVE - 1u;
      last = run;
      mask = last == WAVE - 1u ? ~0ull : ((1ull << (last + 1u)) - 1ull);
      if (rdl(J, last) < WAVE) {
        // the chain goes on past a false candidate (e.g. the byte before a length prefix, whose
        // shifted "length" fits the page): successors increase, so lane l is on the chain from
        // lane 0 iff binary lifting from lane 0 over the jump tables J^(2^r) stops exactly at l
        uint32_t P[6];
        P[0] = J;
#pragma unroll
        for (int r = 1; r < 6; r++) {
          const uint32_t g = (uint32_t)__shfl((int)P[r - 1], (int)(P[r - 1] & (WAVE - 1u)));
          P[r] = P[r - 1] < WAVE ? g : WAVE;
        }
        uint32_t x = 0;
#pragma unroll
        for (int r = 5; r >= 0; r--) {
          const uint32_t y = (uint32_t)__shfl((int)P[r], (int)x);
          if (y <= lane) x = y;
        }
        mask = __ballot(x == lane);
        last = 63u - (uint32_t)__builtin_clzll(mask);
      }
      const uint32_t n_acc = (uint32_t)__builtin_popcountll(mask);
      const uint32_t room = N - produced - got;
      const uint32_t take = uni(n_acc < room ? n_acc : room);
      const uint32_t rank = (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1ull));
      if (((mask >> lane) & 1ull) && rank < take) L.pn[k].x |= 0x80000000u;  // accepted (k < total)
      got += take;
      if (take == room) break;
      const uint32_t cur = rdl(s, last);  // true successor of the last value of the batch
      pos = cur;
      if (cur >= eff_end) { leave = true; break; }
      const uint32_t a = uni(bw_index(L, cur - B));
      if (a >= total || a <= i0 + last) {  // every position of the window was tested
        if (fast) {  // a longer value: the rest of the tile with every length
          fast = false;
          leave = false;
          retry = true;
          break;
        }
        code = bin_value_error(rs, cur, end, dict);
        break;
      }
      i0 = a;
    }
    // ---- advance to the tile holding the next value (requesting the one after it), then
    // store this tile's values
    // (nB == B: the rest of the same tile after a pass cut at BW_CAP candidates; its bytes are
    // still in cur_b)
    const uint32_t nB = pos & ~(BW_WIN - 1u);
    if (leave && nB != B) {
      if (nB == B + BW_WIN) {
        cur_b = nxt_b;
        nxt_b = bw_load(rs, nB + BW_WIN);
      } else {  // a value longer than a tile: the prefetch missed
        cur_b = bw_load(rs, nB);
        nxt_b = bw_load(rs, nB + BW_WIN);
      }
      B = nB;
    }
    wave_sync();
    got = uni(got);
    for (uint32_t k0 = 0, done = 0; done < got; k0 += WAVE) {
      const uint32_t k = k0 + lane;
      const uint2 e = k < total ? L.pn[k] : uint2{0u, 0u};
      const bool acc = (e.x >> 31) != 0;
      const uint64_t am = __ballot(acc);
      if (acc) {
        const uint32_t o = produced + done + (uint32_t)__builtin_popcountll(am & ((1ull << lane) - 1ull));
        const uint32_t p = e.x & 0x7FFFFFFFu;
        gst(out_len + o, e.y - p - 4u);
        gst(out_src + o, p + 4u);
      }
      done += (uint32_t)__builtin_popcountll(am);
    }
    produced += got;
    if (retry) {  // (pos: the value the short pass could not follow; its tile again, every length)
      wave_sync();
      continue;
    }
    fast = true;
    if (code || !leave) break;
    wave_sync();  // the next window overwrites the list
  }
  return BinWalkEnd{uni(pos), uni(produced), code};
}

__device__ __forceinline__ void bin_walk(BinWalkLds& L, rsrc_t rs, uint32_t beg, uint32_t end, uint32_t N, uint32_t* out_len,
                                         uint32_t* out_src, bool dict, int page, int kind, uint64_t* err, ErrCount err_count) {
  const BinWalkEnd r = bin_walk_core(L, rs, beg, end, N, out_len, out_src, dict);
  if (r.code && lane_id() == 0) report(err, err_count, page, kind, r.produced, r.code);
}

// One wave per page. dict_walk = 0: PLAIN BYTE_ARRAY data pages (values -> blen / bsrc at the
// page's value offset). dict_walk = 1: `list` holds column indices of BYTE_ARRAY dictionaries;
// the dictionary page's entries -> dict_len / dict_src; an error is recorded on the column's
// pseudo page (n_pages + column) as an init error.
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(6))) void k_bin_walk(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                       const PageWork* __restrict__ work,
                                                       const ColumnDev* __restrict__ cols,
                                                       const int32_t* __restrict__ list, int n_list, int dict_walk,
                                                       int n_pages, uint64_t* err, ErrCount err_count) {
  __shared__ BinWalkLds lds_all[WPB];
  const int item = wave_page(list, n_list);
  if (item < 0) return;
  BinWalkLds& L = lds_all[wave_id()];
  if (dict_walk) {
    const ColumnDev& cd = cols[item];
    const rsrc_t rs = make_rsrc(bytes + cd.dict_offset, n_bytes - cd.dict_offset);
    bin_walk(L, rs, 0, (uint32_t)cd.dict_bytes, cd.dict_n, cd.dict_len, cd.dict_src, true, n_pages + item, 0, err,
             err_count);
    return;
  }
  const PageWork& pw = work[item];
  const ColumnDev& cd = cols[pw.column];
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  bin_walk(L, rs, uni(pw.data_begin), uni(pw.size), uni(pw.n_values), cd.blen + pw.out_offset,
           cd.bsrc + pw.out_offset, false, item, 2, err, err_count);
}

// ---- PLAIN BYTE_ARRAY pages walked in segments (plans with few such pages: one wave per page leaves
// most of the chip idle while every page's chain is followed tile after tile).
//
// A page's data section is cut into SEG_B-byte segments (tile-aligned), one wave each, in the order
// the waves take tickets (so a segment's predecessor is always held by a running or finished wave).
// Segment 0 starts at the section start. Segment s > 0 guesses its first value start: the first
// position of its first tile from which SEG_LINKS consecutive length prefixes each land on a
// possible value start (a false start — e.g. the byte before a length prefix, read as a length —
// jumps kilobytes ahead onto string bytes and is rejected within a link or two). Every segment walks
// from its guess to the segment end with the page walk (bin_walk_core), writing its values to its
// own scratch, then waits for its predecessor's publication {where the chain left it, values before
// it}: if that position is not its guess (misspeculation, or no guess), it walks again from there.
// It then publishes its own exit and count and moves its values to their place in the column. Only
// the publication chain is serial (one round trip per segment); errors are reported only when they
// fall inside the page's value count, at the index the one-wave walk would report.
constexpr uint32_t SEG_B = 8 * BW_WIN;       // section bytes per segment
constexpr uint32_t SEG_CAP = SEG_B / 4 + 2;  // values that can start in a segment (each takes >= 4 bytes)
constexpr uint32_t SEG_LINKS = 6;
constexpr uint64_t SG_OK = 1ull << 62, SG_STOP = 2ull << 62;
#ifdef PQG_FAULT_INJECT
// Fault-injection build (tests/build/libpqgpu_faultinject.so, tests/test_gpu_timeout.py only; never the
// product): the wave holding ticket 0 publishes PQG_FAULT_INJECT ticks late, past a wait bound
// shortened to 0.1 s, so the segments after it time out
constexpr uint64_t SEG_TIMEOUT_TICKS = 10000000ull;
#else
constexpr uint64_t SEG_TIMEOUT_TICKS = 200000000ull;  // 2 s of s_memrealtime (100 MHz)
#endif
static_assert(SEG_B == BW_SEG_BYTES && SEG_CAP == BW_SEG_CAP, "host segmentation (pqgpu_internal.h)");
static_assert(BW_WIN == BP_TILE, "host tiling of k_bin_plain (pqgpu_internal.h)");
static_assert(BW_WIN == DENT_TILE && BW_CAP == DENT_CAP, "host tiling of the dictionary entry walk (pqgpu_internal.h)");

// a value could start at p: its 4 length bytes and its bytes inside the section
__device__ __forceinline__ bool seg_candidate(rsrc_t rs, uint32_t p, uint32_t end) {
  if ((uint64_t)p + 4u > end) return false;
  return ld4_any(rs, p) <= end - 4u - p;
}

__device__ uint32_t seg_guess(rsrc_t rs, uint32_t S0, uint32_t end) {
  const uint32_t lim = S0 + BW_WIN < end ? S0 + BW_WIN : end;
  for (uint32_t b = S0; b < lim; b += WAVE) {
    const uint32_t p = b + lane_id();
    bool ok = p < lim && seg_candidate(rs, p, end);
    uint32_t q = p;
    for (uint32_t k = 0; k < SEG_LINKS && ok; k++) {
      q = q + 4u + ld4_any(rs, q);
      if (q >= end) break;  // the chain reaches the section end: nothing contradicts it
      ok = seg_candidate(rs, q, end);
    }
    const uint64_t m = __ballot(ok);
    if (m) return b + (uint32_t)__builtin_ctzll(m);
  }
  return 0xFFFFFFFFu;
}

__global__ __launch_bounds__(64 * WPB) void k_bin_walk_seg(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                           const PageWork* __restrict__ work,
                                                           const ColumnDev* __restrict__ cols,
                                                           const uint64_t* __restrict__ segs, uint32_t n_segs,
                                                           uint64_t* status, uint32_t* ticket, uint32_t* tmp,
                                                           uint64_t* err, ErrCount err_count) {
  __shared__ BinWalkLds lds_all[WPB];
  __shared__ uint32_t tk[WPB];
  const uint32_t lane = lane_id();
  if (lane == 0) tk[wave_id()] = atomicAdd(ticket, 1u);
  wave_sync();
  const uint32_t t = uni(tk[wave_id()]);
  if (t >= n_segs) return;
  BinWalkLds& L = lds_all[wave_id()];
  const uint64_t sg = segs[t];
  const int page = (int)(uint32_t)sg;
  const uint32_t s = (uint32_t)(sg >> 32) & 0x7FFFFFFFu;
  const bool last = (sg >> 63) != 0;
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size), N = uni(pw.n_values);
  const uint32_t A0 = beg & ~(BW_WIN - 1u);
  const uint64_t S0l = s == 0 ? beg : (uint64_t)A0 + (uint64_t)s * SEG_B;
  const uint32_t S0 = S0l < end ? (uint32_t)S0l : end;
  const uint32_t stop = last ? 0xFFFFFFFFu : (uint32_t)((uint64_t)A0 + (uint64_t)(s + 1) * SEG_B < end
                                                             ? (uint64_t)A0 + (uint64_t)(s + 1) * SEG_B : end);
  uint32_t* tl = tmp + (uint64_t)t * 2u * SEG_CAP;
  uint32_t* ts = tl + SEG_CAP;
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  const uint32_t guess = s == 0 ? beg : (S0 < end ? uni(seg_guess(rs, S0, end)) : 0xFFFFFFFFu);
  BinWalkEnd r{guess, 0, 0};
  if (guess != 0xFFFFFFFFu && N > 0) r = bin_walk_core(L, rs, guess, end, SEG_CAP, tl, ts, false, stop);
  // the predecessor's publication: where the chain enters this segment, values before it
  uint32_t entry = beg, before = 0;
  bool stopped = N == 0;
  if (s > 0) {
    uint64_t v = 0;
    const uint64_t t_wait = __builtin_amdgcn_s_memrealtime();
    while (true) {
      v = uni64(sld(status + t - 1));
      if (v) break;
      __builtin_amdgcn_s_sleep(2);
      // bounded (s_memrealtime: 100 MHz): a predecessor that never publishes is PQG_ERR_TIMEOUT, not a hang
      if (__builtin_amdgcn_s_memrealtime() - t_wait > SEG_TIMEOUT_TICKS) {
        if (lane == 0) {
          report(err, err_count, page, 2, 0, PQG_ERR_TIMEOUT);
          sst(status + t, SG_STOP);
        }
        return;
      }
    }
    if (v & SG_STOP) {
      stopped = true;
    } else {
      entry = (uint32_t)(v >> 31) & 0x7FFFFFFFu;
      before = (uint32_t)v & 0x7FFFFFFFu;
    }
  }
  if (stopped || before >= N) {
    if (lane == 0) sst(status + t, SG_STOP);
    return;
  }
  if (s > 0 && guess != entry) {  // misspeculated (or no guess): the walk again from the true entry
    wave_sync();
    r = bin_walk_core(L, rs, entry, end, SEG_CAP, tl, ts, false, stop);
  }
#ifdef PQG_FAULT_INJECT
  if (t == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)PQG_FAULT_INJECT) __builtin_amdgcn_s_sleep(127);
  }
#endif
  const uint32_t room = N - before;
  const uint32_t take = r.produced < room ? r.produced : room;
  bool done = r.produced >= room;
  if (r.code && r.produced < room) {  // an error before the page's values are complete
    if (lane == 0) report(err, err_count, page, 2, before + r.produced, r.code);
    done = true;
  }
  if (lane == 0) sst(status + t, done ? SG_STOP : (SG_OK | ((uint64_t)(r.pos & 0x7FFFFFFFu) << 31) | (uint64_t)(before + r.produced)));
  // this segment's values to their place: read back what this wave stored (completed first)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t* out_len = cd.blen + pw.out_offset + before;
  uint32_t* out_src = cd.bsrc + pw.out_offset + before;
  for (uint32_t i = lane; i < take; i += WAVE) {
    gst(out_len + i, sld(tl + i));
    gst(out_src + i, sld(ts + i));
  }
}

// RLE_DICTIONARY BYTE_ARRAY pages: ids (in blen, written by the dictionary kernel) -> entry
// length and offset in the dictionary page. Invalid ids were reported by the dictionary kernel.
// Workgroup (page, slice): each wave takes 1,024-value chunks of the page (lane l: values
// 64 j + l, j < 16), issues all 16 id loads, then the 32 entry gathers (the tables are small and
// L2-resident), then the 32 stores — one store drain per 1,024 values (a load issued after stores
// waits for them: vmcnt counts stores), where one wave per page looping over 64 values paid one
// per 64 (str_dict: 369 us for 20 M values).
constexpr uint32_t DM_SLICES = 4;  // workgroups per page
constexpr uint32_t DM_J = 16;      // values per lane per chunk
__global__ __launch_bounds__(256) void k_bin_dict_map(const PageWork* __restrict__ work,
                                                      const ColumnDev* __restrict__ cols,
                                                      const int32_t* __restrict__ list, int n_list) {
  if ((int)blockIdx.x >= n_list) return;
  const int page = list[blockIdx.x];
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t n = uni(pw.n_values), dn = uni(cd.dict_n);
  uint32_t* len = cd.blen + pw.out_offset;
  uint32_t* src = cd.bsrc + pw.out_offset;
  const uint32_t lane = lane_id();
  const uint32_t nch = (n + DM_J * WAVE - 1u) / (DM_J * WAVE);
  for (uint32_t c = blockIdx.y * WPB + wave_id(); c < nch; c += DM_SLICES * WPB) {
    const uint32_t b = c * DM_J * WAVE + lane;
    uint32_t id[DM_J], l[DM_J], s[DM_J];
#pragma unroll
    for (uint32_t j = 0; j < DM_J; j++) id[j] = b + WAVE * j < n ? len[b + WAVE * j] : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t j = 0; j < DM_J; j++) {
      const bool ok = id[j] < dn;
      l[j] = ok ? cd.dict_len[id[j]] : 0u;
      s[j] = ok ? cd.dict_src[id[j]] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < DM_J; j++)
      if (b + WAVE * j < n) {
        gst(len + b + WAVE * j, l[j]);
        gst(src + b + WAVE * j, s[j]);
      }
  }
}

// FIXED_LEN_BYTE_ARRAY / INT96 dictionary pages: ids (in blen) -> W-byte entries, one output
// byte per lane and step (the dictionary is small and L2-resident).
__global__ __launch_bounds__(256) void k_gather_fixed(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                      const PageWork* __restrict__ work,
                                                      const ColumnDev* __restrict__ cols,
                                                      const int32_t* __restrict__ list, int n_list) {
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t W = uni((uint32_t)cd.elem_width), dn = uni(cd.dict_n);
  const uint64_t nb = (uint64_t)uni(pw.n_values) * W;
  const uint32_t* ids = cd.blen + pw.out_offset;
  uint8_t* out = (uint8_t*)cd.values + pw.out_offset * W;
  const rsrc_t drs = make_rsrc(bytes + cd.dict_offset, cd.dict_bytes);
  for (uint64_t o = lane_id(); o < nb; o += WAVE) {
    const uint32_t i = (uint32_t)(o / W), k = (uint32_t)(o % W);
    const uint32_t id = ids[i];
    if (id >= dn) continue;
    const uint32_t a = id * W + k;
    gst(out + o, (uint8_t)(ld32(drs, a & ~3u) >> ((a & 3u) * 8u)));
  }
}

// 4 source bytes at staged offset i (any alignment): one unaligned ds_read_b32 (gfx950 runs DS
// accesses in unaligned mode; 32-bit accesses off their alignment take no replay, unlike b64 / b128)
// (the aligned-pair form, two reads and a v_alignbyte, measured the same or slower: profiles/r03/img4)
__device__ __forceinline__ uint32_t img4(const uint32_t* img, uint32_t i) {
  typedef uint32_t __attribute__((aligned(1), may_alias)) u32u;
  return *(const u32u*)((const uint8_t*)img + i);
}

// ---------------------------------------------------------------------------
// Offsets of BYTE_ARRAY columns: exclusive scan of blen over [0, n_slots) (entries past the
// column's decoded values hold 0: blen is cleared before every launch), written as int64
// offsets[0 .. n_slots]. blocks[b] = (column << 32) | block index within the column.

__device__ __forceinline__ uint64_t block_reduce_u64(uint64_t v, uint64_t* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if (lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
  for (uint32_t w = 0; w < blockDim.x / WAVE; w++) t += red[w];
  __syncthreads();
  return t;
}

// A block of SCAN_BLOCK lengths is read as 4 rows of 1,024: in row i thread t holds lengths
// [i * 1024 + 4t, i * 1024 + 4t + 4) (one 16-byte load when the lengths are 16-byte aligned).
static_assert(SCAN_BLOCK == 4096, "scan block layout: 4 rows x 256 threads x 4 lengths");
__device__ __forceinline__ u32x4 scan_row_load(const uint32_t* blen, uint64_t n_slots, uint64_t v) {
  if (v + 4 <= n_slots && ((uintptr_t)(blen + v) & 15u) == 0)
    return *(const __attribute__((address_space(1))) u32x4*)(blen + v);
  u32x4 x;
#pragma unroll
  for (int k = 0; k < 4; k++) x[k] = v + k < n_slots ? blen[v + k] : 0u;
  return x;
}

__global__ __launch_bounds__(256) void k_bin_block_sums(const ColumnDev* __restrict__ cols,
                                                        const uint64_t* __restrict__ blocks) {
  __shared__ uint64_t red[4];
  const uint64_t b = blocks[blockIdx.x];
  const ColumnDev& cd = cols[(uint32_t)(b >> 32)];
  const uint64_t v0 = (uint64_t)(uint32_t)b * SCAN_BLOCK;
  u32x4 x[4];
#pragma unroll
  for (int i = 0; i < 4; i++) x[i] = scan_row_load(cd.blen, cd.n_slots, v0 + 1024u * i + 4u * threadIdx.x);
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) s += (uint64_t)x[i][0] + x[i][1] + (uint64_t)x[i][2] + x[i][3];
  s = block_reduce_u64(s, red);
  if (threadIdx.x == 0) cd.block_sums[(uint32_t)b] = s;
}

// One workgroup per BYTE_ARRAY column: exclusive scan of its block sums (in place) + total.
// Each thread scans 16 consecutive sums serially: one wave scan and one barrier pair per 4,096.
__global__ __launch_bounds__(256) void k_bin_block_bases(const ColumnDev* __restrict__ cols,
                                                         const int32_t* __restrict__ bin_cols) {
  __shared__ uint64_t wsum[4];
  const ColumnDev& cd = cols[bin_cols[blockIdx.x]];
  const uint32_t nb = (uint32_t)((cd.n_slots + SCAN_BLOCK - 1) / SCAN_BLOCK);
  uint64_t* bs = cd.block_sums;
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 16u * 256u) {
    const uint32_t bt = b0 + 16u * threadIdx.x;
    uint64_t v[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      v[k] = bt + k < nb ? bs[bt + k] : 0;
      s += v[k];
    }
    uint64_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o);
      if ((int)lane_id() >= o) x += y;
    }
    if (lane_id() == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t pre = carry, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
      pre += w < (threadIdx.x >> 6) ? wsum[w] : 0;
      tot += wsum[w];
    }
    pre += x - s;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (bt + k < nb) bs[bt + k] = pre;
      pre += v[k];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *cd.bin_total = carry;
}

// Offsets of one scan block: per row, a wave scan of the threads' 4-length sums and the wave
// totals through LDS (4 rows scanned side by side: one barrier per block instead of two per
// 256 lengths); offsets stored as two 16-byte stores per row and thread.
__global__ __launch_bounds__(256) void k_bin_offsets(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                     const ColumnDev* __restrict__ cols,
                                                     const uint64_t* __restrict__ blocks) {
  __shared__ uint64_t wsum[4][4];  // [row][wave]
  const uint64_t b = blocks[blockIdx.x];
  const ColumnDev& cd = cols[(uint32_t)(b >> 32)];
  const uint64_t v0 = (uint64_t)(uint32_t)b * SCAN_BLOCK;
  const uint64_t n_slots = cd.n_slots;
  int64_t* off = (int64_t*)cd.values;
  const uint32_t t = threadIdx.x, wv = t >> 6, lane = lane_id();
  u32x4 x[4];
  uint64_t inc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) x[i] = scan_row_load(cd.blen, n_slots, v0 + 1024u * i + 4u * t);
#pragma unroll
  for (int i = 0; i < 4; i++) inc[i] = (uint64_t)x[i][0] + x[i][1] + (uint64_t)x[i][2] + x[i][3];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint64_t y = __shfl_up(inc[i], o);
      if ((int)lane >= o) inc[i] += y;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int i = 0; i < 4; i++) wsum[i][wv] = inc[i];
  }
  __syncthreads();
  uint64_t base = cd.block_sums[(uint32_t)b];
  const bool vec = ((uintptr_t)off & 15u) == 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t pre = base;
    uint64_t row = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
      pre += w < wv ? wsum[i][w] : 0;
      row += wsum[i][w];
    }
    base += row;
    // exclusive offsets of this thread's 4 lengths
    uint64_t e0 = pre + inc[i] - ((uint64_t)x[i][0] + x[i][1] + (uint64_t)x[i][2] + x[i][3]);
    const uint64_t e1 = e0 + x[i][0], e2 = e1 + x[i][1], e3 = e2 + x[i][2], e4 = e3 + x[i][3];
    const uint64_t v = v0 + 1024u * i + 4u * t;
    if (vec && v + 4 <= n_slots) {
      typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
      gst((i64x2*)(off + v), i64x2{(int64_t)e0, (int64_t)e1});
      gst((i64x2*)(off + v + 2), i64x2{(int64_t)e2, (int64_t)e3});
    } else {
      const uint64_t e[4] = {e0, e1, e2, e3};
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (v + k < n_slots) gst(off + v + k, (int64_t)e[k]);
    }
    // the final offset (the column's byte total) after the last slot
    if (v < n_slots && n_slots <= v + 4) gst(off + n_slots, (int64_t)(n_slots - v == 1 ? e1 : n_slots - v == 2 ? e2
                                                                     : n_slots - v == 3 ? e3 : e4));
  }
}

// ---------------------------------------------------------------------------
// c ? y : x per lane, as v_cndmask the optimizer cannot see through: selects among elements of a
// register array are otherwise turned into an indexed access, which puts the array in scratch (and
// scratch loads wait for every store in flight)
__device__ __forceinline__ uint32_t vsel(uint32_t c, uint32_t x, uint32_t y) {
  uint32_t r;
  asm("v_cmp_ne_u32 vcc, 0, %3\n\tv_cndmask_b32 %0, %1, %2, vcc" : "=v"(r) : "v"(x), "v"(y), "v"(c) : "vcc");
  return r;
}
// a[i], i < 8: a tree of selects on the bits of i
__device__ __forceinline__ uint32_t pick8(const uint32_t (&a)[8], uint32_t i) {
  const uint32_t b0 = i & 1u, b1 = i & 2u, b2 = i & 4u;
  const uint32_t x0 = vsel(b0, a[0], a[1]), x1 = vsel(b0, a[2], a[3]), x2 = vsel(b0, a[4], a[5]), x3 = vsel(b0, a[6], a[7]);
  return vsel(b2, vsel(b1, x0, x1), vsel(b1, x2, x3));
}


// Value bytes of values [i_lo, i_hi) of one page, by one wave (the per-wave path of k_bin_copy,
// for chunks whose source does not fit the workgroup's LDS staging: long values, large
// dictionaries). The offsets and sources are staged in LDS; every lane owns output dwords of the
// range and finds the value of its first byte by binary search (then walks forward). A dword
// inside one value is one unaligned 4-byte source read; a dword that straddles values (or the
// range ends, which other waves share) is assembled and stored byte by byte.
// DELTA_LENGTH_BYTE_ARRAY sources are the page's value bytes (PageWork::aux) + the in-page offset;
// a value running past the page is the reference's "Failed to read N bytes" (EOF) at that value.
constexpr uint32_t CP_VALUES = CP_CHUNK_VALUES;  // values per workgroup chunk of k_bin_copy
constexpr uint32_t CP_WAVE = CP_VALUES / WPB;  // values per wave on the per-wave path
constexpr uint32_t CP_SRC = 48u * CP_VALUES;     // LDS bytes of staged source per workgroup
static_assert(CP_VALUES == CP_CHUNK_VALUES, "host chunking (pqgpu_internal.h)");

struct CopyWaveLds {
  uint64_t off[CP_WAVE + 1];
  uint32_t src[CP_WAVE];
  uint32_t rel[CP_WAVE + 1];
  uint32_t bt[COPY_BTAB];
};

__device__ __forceinline__ void bin_copy_wave(const uint8_t* __restrict__ bytes, uint64_t n_bytes, const PageWork& pw,
                                              const ColumnDev& cd, int page, uint32_t i_lo, uint32_t i_hi,
                                              CopyWaveLds& W, uint64_t* err, ErrCount err_count) {
  uint64_t* off = W.off;
  uint32_t* src = W.src;
  uint32_t* rel = W.rel;
  const uint32_t lane = lane_id();
  if (i_lo >= i_hi) return;
  const uint32_t n = i_hi - i_lo;
  const int64_t* offs = (const int64_t*)cd.values + pw.out_offset;
  const bool dlba = uni(pw.bin_kind) == BIN_DLBA;
  const bool from_dict = uni(pw.bin_kind) == BIN_DICT;
  const uint64_t sbase = from_dict ? cd.dict_offset : pw.base;
  const uint64_t slim = from_dict ? cd.dict_bytes : pw.size;
  const rsrc_t rs = make_rsrc(bytes + sbase, n_bytes - sbase);
  const uint64_t page0 = (uint64_t)offs[0];
  for (uint32_t k = lane; k <= n; k += WAVE) off[k] = (uint64_t)offs[i_lo + k];
  wave_sync();
  // PLAIN / DLBA sources follow from the offsets (see below): only value 0's is needed
  // (PLAIN only: DELTA_LENGTH sources are computed per value below for the EOF check)
  const bool plain_small = !dlba && !from_dict && off[n] - off[0] < 0x7FFF0000ull - 16u;
  const uint32_t n_src = plain_small ? 1u : n;
  for (uint32_t k = lane; k < n_src; k += WAVE) {
    uint32_t s;
    if (dlba) {
      const uint64_t rel = off[k] - page0, len = off[k + 1] - off[k];
      const uint64_t avail = pw.size > pw.aux ? pw.size - pw.aux : 0;
      if (rel + len > avail) report(err, err_count, page, 2, i_lo + k, PQG_ERR_EOF);
      s = (uint32_t)(pw.aux + rel);
    } else {
      s = cd.bsrc[pw.out_offset + i_lo + k];
    }
    src[k] = s;
  }
  wave_sync();
  const uint64_t o_lo = off[0], o_hi0 = off[n];
  const uint64_t o_hi = o_hi0 < cd.binary_capacity ? o_hi0 : cd.binary_capacity;  // overflow: reported at sync
  if (o_lo >= o_hi) return;
  uint8_t* dst = cd.binary_data;
  // every lane fills 16-byte blocks of the output: the value holding the block's first byte by
  // binary search, then per dword the value pieces it contains (one unaligned 4-byte source
  // read per piece, usually one piece per dword)
  const uint64_t a0 = o_lo & ~15ull;
  const bool dst_al16 = ((uintptr_t)dst & 15u) == 0, dst_al4 = ((uintptr_t)dst & 3u) == 0;
  // Blocks are gathered G at a time before any of them is stored: a source load issued
  // after a store waits for that store (vmcnt counts both), so loads and stores are not interleaved.
  constexpr uint32_t G = 4;
  if (o_hi - a0 < 0x7FFF0000ull) {
    // The usual case: the chunk's bytes span < 2 GiB, so offsets are kept chunk-relative in 32
    // bits (relative to the first 16-byte block a0), and PLAIN / DELTA_LENGTH sources follow from
    // them: value k starts at src0 + rel[k] (DLBA) or src0 + rel[k] + 4k (PLAIN: the 4-byte
    // length prefixes); only dictionary entries need the per-value source table.
    for (uint32_t k = lane; k <= n; k += WAVE) rel[k] = (uint32_t)(off[k] - a0);
    wave_sync();
    const uint32_t hole = dlba ? 0u : 4u;
    const uint32_t src0 = src[0];
    const uint32_t r_lo = (uint32_t)(o_lo - a0), r_hi = (uint32_t)(o_hi - a0);
    uint32_t kv = 0;
    // value of every 16-byte block's first byte, when the chunk spans at most COPY_BTAB blocks:
    // bt[j] = the last value starting at or before byte 16j (a value starting inside block j - 1
    // is entered at index ceil(rel / 16), then a running maximum), instead of a binary search
    // per block
    uint32_t* bt = W.bt;
    const uint32_t nblk = (r_hi + 15u) >> 4;
    const bool btab = nblk <= COPY_BTAB;
    if (btab) {
      for (uint32_t i = lane; i < nblk; i += WAVE) bt[i] = 0;
      wave_sync();
      for (uint32_t k = lane; k < n; k += WAVE) {
        const uint32_t blk = (rel[k] + 15u) >> 4;
        if (blk < nblk) atomicMax(&bt[blk], k);
      }
      wave_sync();
      uint32_t carry = 0;
      for (uint32_t i0 = 0; i0 < nblk; i0 += WAVE) {
        uint32_t v = i0 + lane < nblk ? bt[i0 + lane] : 0u;
        v = v > carry ? v : carry;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(v, o);
          if ((int)lane >= o) v = v > y ? v : y;
        }
        if (i0 + lane < nblk) bt[i0 + lane] = v;
        carry = uni(rdl(v, WAVE - 1));
      }
      wave_sync();
    }
    for (uint32_t bg = 16u * lane; bg < r_hi; bg += 16u * WAVE * G) {
      uint32_t wd[G][4];
      uint32_t have[G];
#pragma unroll
      for (uint32_t g = 0; g < G; g++) {
        const uint32_t b = bg + 16u * WAVE * g;  // block start (relative to a0)
        have[g] = 0;
        wd[g][0] = wd[g][1] = wd[g][2] = wd[g][3] = 0;
        if (b >= r_hi) continue;
        const uint32_t b0 = b > r_lo ? b : r_lo;
        if (btab) {
          kv = bt[b >> 4];
        } else
        {
        uint32_t lo = kv, hi = n;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (rel[mid] <= b0) lo = mid;
          else hi = mid;
        }
        kv = lo;
        }
        const uint32_t bend = b + 16u < r_hi ? b + 16u : r_hi;
        // PLAIN / DLBA: the block's source is one stream with a 4-byte hole (PLAIN) at every value
        // start inside the block; with at most 4 such starts the block is composed without loops:
        // 9 aligned source dwords, the 8 dwords a_t at the block's byte alignment, and per output
        // byte i the dword a_{q + cnt_i} (cnt_i = value starts at or before byte i).
        // (not when block byte 0 would lie before the page start: its source offset cannot be
        // expressed, and the block's stored bytes would read as 0)
        const bool compose = !from_dict && !(kv + 5u < n && rel[kv + 5u] < bend) &&
                             !(b < r_lo && src0 + hole * kv < r_lo - b);
        if (compose) {
          uint64_t prof = 0;  // nibble i: value starts at or before byte i of the block (PLAIN)
#pragma unroll
          for (uint32_t j = 1; j <= 4; j++) {
            const uint32_t kk = kv + j;
            const uint32_t pj = kk < n ? rel[kk] : 0xFFFFFFFFu;
            if (pj < bend && hole) prof += 0x1111111111111111ull << (4u * (pj - b));
          }
          const uint32_t S = src0 + (b - r_lo) + hole * kv;  // source of block byte 0 (wraps below: not stored)
          const uint32_t A = S & ~3u, sh = S & 3u;
          const u32x4 w0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)A, 0, 0);
          const u32x4 w1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(A + 16u), 0, 0);
          const uint32_t w8 = ld32(rs, A + 32u);
          const uint32_t wv[9] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w8};
          uint32_t a[8];
#pragma unroll
          for (uint32_t t = 0; t < 8; t++) a[t] = __builtin_amdgcn_alignbyte(wv[t + 1], wv[t], sh);
#pragma unroll
          for (uint32_t q = 0; q < 4; q++) {
            uint32_t word = 0;
            // the dword's bytes come from a[q + c0] and, after at most one value start inside
            // it, a[q + c0 + 1]: one v_perm with the byte selector of the start
            const uint32_t cq = (uint32_t)(prof >> (16u * q)) & 0xFFFFu;  // counts of bytes 4q .. 4q+3
            const uint32_t c0 = cq & 0xFu;
            const uint32_t dn = cq - c0 * 0x1111u;  // nibbles: 0, or 1 from the start on
            if (dn <= 0x1111u && (dn & 0xEEEEu) == 0) {
              const uint32_t A0 = pick8(a, q + c0 < 7u ? q + c0 : 7u), A1 = pick8(a, q + c0 + 1u < 7u ? q + c0 + 1u : 7u);
              const uint32_t hb = (dn & 1u) | ((dn & 0x10u) << 4) | ((dn & 0x100u) << 8) | ((dn & 0x1000u) << 12);
              word = __builtin_amdgcn_perm(A1, A0, 0x03020100u + 4u * hb);
            } else
            {
#pragma unroll
            for (uint32_t e = 0; e < 4; e++) {
              const uint32_t c = (uint32_t)(prof >> (4u * (4u * q + e))) & 0xFu;  // 0..4
              word |= pick8(a, q + c) & (0xFFu << (8u * e));
            }
            }
            const uint32_t d0 = b + 4u * q;
            wd[g][q] = word;
            if (d0 >= r_lo && d0 + 4u <= r_hi) have[g] |= 1u << q;
          }
        } else
        {
        uint32_t k = kv;
        uint32_t k_end = rel[k + 1];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          const uint32_t d0 = b + 4u * q;
          const uint32_t x0 = d0 > r_lo ? d0 : r_lo, x1 = d0 + 4u < r_hi ? d0 + 4u : r_hi;
          uint32_t word = 0;
          for (uint32_t cur = x0; cur < x1;) {
            while (k + 1 < n && cur >= k_end) {
              k++;
              k_end = rel[k + 1];
            }
            const uint32_t seg_end = x1 < k_end ? x1 : k_end;
            const uint32_t sk = from_dict ? src[k] : src0 + (rel[k] - r_lo) + hole * k;
            const uint32_t sp = sk + (cur - rel[k]);
            const uint32_t v = sp < slim ? ld4_any(rs, sp) : 0u;
            const uint32_t nb = seg_end - cur;
            const uint32_t msk = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8u * nb)) - 1u);
            word |= (v & msk) << (8u * (cur - d0));
            cur = seg_end;
          }
          wd[g][q] = word;
          if (x0 == d0 && x1 == d0 + 4u) have[g] |= 1u << q;
        }
        }
        (void)bend;
        if (!dst_al4) have[g] = 0;  // unaligned byte buffer (C ABI caller): byte stores only
      }
#pragma unroll
      for (uint32_t g = 0; g < G; g++) {
        const uint32_t b = bg + 16u * WAVE * g;
        if (b < r_hi) store_block16(dst, a0 + b, o_lo, o_hi, wd[g], have[g], dst_al16);
      }
    }
    return;
  }
  uint32_t kv = 0;  // value of this lane's current byte (monotone across iterations)
  for (uint64_t ag = a0 + 16u * lane; ag < o_hi; ag += 16u * WAVE * G) {
    uint32_t wd[G][4];
    uint32_t have[G];  // bit q: dword q fully inside [o_lo, o_hi)
#pragma unroll
    for (uint32_t g = 0; g < G; g++) {
      const uint64_t a = ag + 16u * WAVE * g;
      have[g] = 0;
      wd[g][0] = wd[g][1] = wd[g][2] = wd[g][3] = 0;
      if (a >= o_hi) continue;
      const uint64_t b0 = a > o_lo ? a : o_lo;
      uint32_t lo = kv, hi = n;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= b0) lo = mid;
        else hi = mid;
      }
      kv = lo;
      uint32_t k = kv;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint64_t d0 = a + 4u * q;
        const uint64_t x0 = d0 > o_lo ? d0 : o_lo, x1 = d0 + 4u < o_hi ? d0 + 4u : o_hi;
        uint32_t word = 0;
        for (uint64_t cur = x0; cur < x1;) {
          while (k + 1 < n && cur >= off[k + 1]) k++;
          const uint64_t vend = off[k + 1];
          const uint64_t seg_end = x1 < vend ? x1 : vend;
          const uint32_t nbytes = (uint32_t)(seg_end - cur);
          const uint64_t sp = (uint64_t)src[k] + (cur - off[k]);
          const uint32_t v = sp < slim ? ld4_any(rs, (uint32_t)sp) : 0u;
          const uint32_t m = nbytes >= 4 ? 0xFFFFFFFFu : ((1u << (8u * nbytes)) - 1u);
          word |= (v & m) << (8u * (uint32_t)(cur - d0));
          cur = seg_end;
        }
        wd[g][q] = word;
        if (x0 == d0 && x1 == d0 + 4u) have[g] |= 1u << q;
      }
      if (!dst_al4) have[g] = 0;  // unaligned byte buffer (C ABI caller): byte stores only
    }
#pragma unroll
    for (uint32_t g = 0; g < G; g++) {
      const uint64_t a = ag + 16u * WAVE * g;
      if (a < o_hi) store_block16(dst, a, o_lo, o_hi, wd[g], have[g], dst_al16);
    }
  }
}

// LDS of one k_bin_copy workgroup: the chunk's value starts (relative to the chunk's first 16-byte
// output block) and dictionary sources, and the staged source bytes; or the per-wave path's tables.
constexpr uint32_t CP_BLOCKS = CP_SRC / 16 + 2;  // 16-byte output blocks of a staged chunk (output <= source)
struct CopyWgLds {
  uint32_t rel[CP_VALUES + 1];
  uint32_t src[CP_VALUES];
  uint16_t bt[CP_BLOCKS];         // output block -> the last value starting at or before its first byte
  uint32_t wmax[WPB];
  uint32_t img[CP_SRC / 4 + 16];  // source bytes [Sa, Sa + CP_SRC) + slack for 9-dword reads
};
union CopyLds {
  CopyWgLds g;
  CopyWaveLds w[WPB];
};


// One 16-byte output block of length-prefixed values composed from staged source bytes: Sv = staged
// offset of the block's byte 0 counting no value start inside the block; prof nibble i = the value
// starts (0..4) at or before byte i, each shifting the source by a 4-byte length prefix. An output
// dword whose bytes shift by at most one start is one v_perm of two byte-aligned source dwords;
// others are taken byte by byte. Reads up to staged byte Sv + 39. (The source dwords are read from
// LDS at the computed offsets: a register array indexed by a start count lands in scratch, whose
// loads wait for every store in flight.)
__device__ __forceinline__ void compose_block(const uint32_t* img, uint32_t Sv, uint64_t prof, uint32_t (&wd)[4]) {
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    uint32_t word = 0;
    const uint32_t cq = (uint32_t)(prof >> (16u * q)) & 0xFFFFu;  // counts of bytes 4q .. 4q+3
    const uint32_t c0 = cq & 0xFu;
    const uint32_t dn = cq - c0 * 0x1111u;  // nibbles: 0, or 1 from a start inside the dword on
    if (dn <= 0x1111u && (dn & 0xEEEEu) == 0) {
      const uint32_t o = Sv + 4u * (q + c0);
      const uint32_t hb = (dn & 1u) | ((dn & 0x10u) << 4) | ((dn & 0x100u) << 8) | ((dn & 0x1000u) << 12);
      word = __builtin_amdgcn_perm(img4(img, o + 4u), img4(img, o), 0x03020100u + 4u * hb);
    } else {
#pragma unroll
      for (uint32_t e = 0; e < 4; e++) {
        const uint32_t c = (uint32_t)(prof >> (4u * (4u * q + e))) & 0xFu;  // 0..4
        word |= img4(img, Sv + 4u * (q + c)) & (0xFFu << (8u * e));
      }
    }
    wd[q] = word;
  }
}

// Value bytes. Workgroups stride over chunks of CP_VALUES values of one page (chunks[c] = page | j << 32).
// The chunk's source is staged in LDS with coalesced 16-byte loads: the page bytes its values come
// from (PLAIN: one stream with a 4-byte length prefix before every value; DELTA_LENGTH: the value
// bytes back to back) or the whole dictionary page (RLE_DICTIONARY: entries in any order). Then
// every thread composes whole 16-byte output blocks from LDS (a block with at most 4 value starts
// from 9 aligned dwords and one v_perm per dword, as the per-wave path does from memory; others
// piece by piece) and stores them: after the staging loads the workgroup issues stores only, so
// no load waits behind a store (vmcnt counts both). Source bytes are read from HBM once, where
// the per-wave path read 36 bytes per 16-byte block. A chunk whose source does not fit CP_SRC
// takes the per-wave path, CP_WAVE values per wave.
__global__ __launch_bounds__(64 * WPB) void k_bin_copy(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                       const PageWork* __restrict__ work,
                                                       const ColumnDev* __restrict__ cols,
                                                       const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                       uint64_t* err, ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) CopyLds S;
  int staged = -1;  // column whose dictionary page is in L.img (kept across this workgroup's chunks)
  for (uint32_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
  __syncthreads();  // the previous chunk's LDS reads are done
  const uint64_t ch = chunks[c];
  const int page = (int)(uint32_t)ch;
  const uint32_t J = (uint32_t)(ch >> 32);
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t nv = uni(pw.n_values);
  const uint32_t i_lo = J * CP_VALUES;
  if (i_lo >= nv) continue;
  const uint32_t i_hi = i_lo + CP_VALUES < nv ? i_lo + CP_VALUES : nv;
  const uint32_t n = i_hi - i_lo;
  const uint32_t t = threadIdx.x;
  const int64_t* offs = (const int64_t*)cd.values + pw.out_offset;
  const uint32_t kind = uni(pw.bin_kind);
  const bool dlba = kind == BIN_DLBA, from_dict = kind == BIN_DICT;
  const uint64_t page0 = (uint64_t)offs[0];
  const uint64_t o_lo = (uint64_t)offs[i_lo], o_hi0 = (uint64_t)offs[i_hi];
  const uint64_t o_hi = o_hi0 < cd.binary_capacity ? o_hi0 : cd.binary_capacity;  // overflow: reported at sync
  const uint64_t a0 = o_lo & ~15ull;
  const uint32_t hole = (dlba || from_dict) ? 0u : 4u;
  // source of the chunk: page-relative (PLAIN, DLBA) or dictionary-relative (DICT) byte range
  const uint64_t slim = from_dict ? cd.dict_bytes : pw.size;
  uint64_t s_lo, s_hi;
  if (from_dict) {
    s_lo = 0;
    s_hi = slim;
  } else {
    s_lo = dlba ? pw.aux + (o_lo - page0) : (uint64_t)cd.bsrc[pw.out_offset + i_lo];
    s_hi = s_lo + (o_hi0 - o_lo) + (uint64_t)hole * (n - 1u);
  }
  const uint64_t Sa = s_lo & ~15ull;
  const bool fit = o_hi0 - a0 < 0x7FFF0000ull && s_hi - Sa <= CP_SRC && s_lo <= slim && o_hi0 - a0 <= 16ull * (CP_BLOCKS - 1);
  if (!fit) {
    // per-wave path: wave w takes values [i_lo + CP_WAVE w, + CP_WAVE)
    const uint32_t w0 = i_lo + CP_WAVE * wave_id();
    bin_copy_wave(bytes, n_bytes, pw, cd, page, w0 < i_hi ? w0 : i_hi, w0 + CP_WAVE < i_hi ? w0 + CP_WAVE : i_hi,
                  S.w[wave_id()], err, err_count);
    staged = -1;
    continue;
  }
  CopyWgLds& L = S.g;
  const uint64_t sbase = from_dict ? cd.dict_offset : pw.base;
  const rsrc_t rs = make_rsrc(bytes + sbase, n_bytes - sbase);
  // ---- staging: source bytes [Sa, s_hi) (bytes at or past slim read as 0), value starts, sources
  const uint32_t n_st = (uint32_t)(s_hi - Sa);
  const bool restage = !(from_dict && staged == pw.column);  // a dictionary page stays staged
  staged = from_dict ? pw.column : -1;
  for (uint32_t o = 16u * t; restage && o < n_st; o += 16u * 64u * WPB) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(Sa + o), 0, 0);
    if (Sa + o + 16u > slim) {
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const int64_t keep = (int64_t)slim - (int64_t)(Sa + o + 4u * q);
        const uint32_t m = keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
        v[q] &= m;
      }
    }
    *(u32x4*)&L.img[o >> 2] = v;
  }
  for (uint32_t k = t; k <= n; k += 64u * WPB) L.rel[k] = (uint32_t)((uint64_t)offs[i_lo + k] - a0);
  if (from_dict)
    for (uint32_t k = t; k < n; k += 64u * WPB) L.src[k] = cd.bsrc[pw.out_offset + i_lo + k];
  if (dlba)  // DeltaLengthByteArrayValuesReader.readBytes: a value past the page is EOF at that value
    for (uint32_t k = t; k < n; k += 64u * WPB) {
      const uint64_t r = (uint64_t)offs[i_lo + k] - page0, len = (uint64_t)offs[i_lo + k + 1] - (uint64_t)offs[i_lo + k];
      const uint64_t avail = pw.size > pw.aux ? pw.size - pw.aux : 0;
      if (r + len > avail) report(err, err_count, page, 2, i_lo + k, PQG_ERR_EOF);
    }
  // Dictionary chunks of short values (C4's flags and modes: 1-17 bytes): every value's bytes are
  // scattered from the staged dictionary into an output image after it in LDS (4 bytes per step), then
  // the image goes out as 16-byte blocks. Composing a 16-byte block that holds many value starts took
  // one LDS round trip per piece (k_bin_copy 7.5 ms of the C4 125M-row shard for 500 M such values).
  const uint32_t ob = (n_st + 15u) & ~15u;  // byte offset of the output image in L.img
  if (from_dict && o_hi0 - a0 <= 16ull * n && ob + (uint32_t)(o_hi0 - a0) + 16u <= CP_SRC) {
    __syncthreads();  // staged dictionary, rel, src
    uint8_t* outb = (uint8_t*)L.img + ob;
    for (uint32_t k = t; k < n; k += 64u * WPB) {
      const uint32_t r = L.rel[k], len = L.rel[k + 1] - r, sp = L.src[k];
      for (uint32_t j = 0; j < len; j += 4u) {
        const uint32_t v = sp + j < n_st ? img4(L.img, sp + j) : 0u;  // (bytes past the value: masked)
#pragma unroll
        for (uint32_t e = 0; e < 4u; e++)
          if (j + e < len) outb[r + j + e] = (uint8_t)(v >> (8u * e));
      }
    }
    __syncthreads();
    if (o_lo >= o_hi) continue;
    uint8_t* dst = cd.binary_data;
    const bool dst_al16 = ((uintptr_t)dst & 15u) == 0, dst_al4 = ((uintptr_t)dst & 3u) == 0;
    const uint32_t r_lo = (uint32_t)(o_lo - a0), r_hi = (uint32_t)(o_hi - a0);
    for (uint32_t b = 16u * t; b < r_hi; b += 16u * 64u * WPB) {
      const u32x4 v4 = *(const u32x4*)(outb + b);
      uint32_t wd[4] = {v4.x, v4.y, v4.z, v4.w};
      uint32_t have = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t d0 = b + 4u * q;
        if (d0 >= r_lo && d0 + 4u <= r_hi) have |= 1u << q;
      }
      if (!dst_al4) have = 0;
      store_block16(dst, a0 + b, o_lo, o_hi, wd, have, dst_al16);
    }
    continue;
  }
  const uint32_t nblk = (uint32_t)((o_hi0 - a0 + 15u) >> 4);
  for (uint32_t i = t; i < nblk; i += 64u * WPB) L.bt[i] = 0;
  __syncthreads();
  // block table: value k enters at block ceil(rel / 16) (the last value entering a block writes it:
  // one writer per block), then a running maximum over the blocks
  for (uint32_t k = t; k < n; k += 64u * WPB) {
    const uint32_t blk = (L.rel[k] + 15u) >> 4;
    if (blk < nblk && (k + 1u == n || ((L.rel[k + 1] + 15u) >> 4) != blk)) L.bt[blk] = (uint16_t)k;
  }
  __syncthreads();
  {
    // running maximum over nblk entries: each thread a run of consecutive blocks, then the runs
    const uint32_t per = (nblk + 64u * WPB - 1u) / (64u * WPB);
    const uint32_t i0 = t * per, i1 = i0 + per < nblk ? i0 + per : nblk;
    uint32_t mx = 0;
    for (uint32_t i = i0; i < i1; i++) mx = L.bt[i] > mx ? L.bt[i] : mx;
    uint32_t inc = mx;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if ((int)lane_id() >= o) inc = y > inc ? y : inc;
    }
    if (lane_id() == 63) L.wmax[wave_id()] = inc;
    __syncthreads();
    uint32_t run = (uint32_t)__shfl_up(inc, 1);
    if (lane_id() == 0) run = 0;
    for (uint32_t w = 0; w < wave_id(); w++) run = L.wmax[w] > run ? L.wmax[w] : run;
    for (uint32_t i = i0; i < i1; i++) {
      run = L.bt[i] > run ? L.bt[i] : run;
      L.bt[i] = (uint16_t)run;
    }
  }
  __syncthreads();
  if (o_lo >= o_hi) continue;
  uint8_t* dst = cd.binary_data;
  const bool dst_al16 = ((uintptr_t)dst & 15u) == 0, dst_al4 = ((uintptr_t)dst & 3u) == 0;
  const uint32_t r_lo = (uint32_t)(o_lo - a0), r_hi = (uint32_t)(o_hi - a0);
  const uint32_t src0 = (uint32_t)(s_lo - Sa);  // staged offset of value 0's first byte (PLAIN, DLBA)
  const uint32_t* img = L.img;
  const uint32_t* rel = L.rel;
  for (uint32_t b = 16u * t; b < r_hi; b += 16u * 64u * WPB) {
    const uint32_t kv = L.bt[b >> 4];  // value of the block's first byte
    const uint32_t bend = b + 16u < r_hi ? b + 16u : r_hi;
    uint32_t wd[4];
    uint32_t have = 0;
    // staged source offset of block byte 0 (PLAIN / DLBA); compose needs it >= 0
    const int64_t Sg = (int64_t)src0 + (int64_t)b - (int64_t)r_lo + (int64_t)hole * kv;
    const bool compose = !from_dict && !(kv + 5u < n && rel[kv + 5u] < bend) && Sg >= 0;
    if (compose) {
      uint64_t prof = 0;  // nibble i: value starts at or before byte i of the block (PLAIN)
#pragma unroll
      for (uint32_t j = 1; j <= 4; j++) {
        const uint32_t kk = kv + j;
        const uint32_t pj = kk < n ? rel[kk] : 0xFFFFFFFFu;
        if (pj < bend && hole) prof += 0x1111111111111111ull << (4u * (pj - b));
      }
      compose_block(img, (uint32_t)Sg, prof, wd);
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t d0 = b + 4u * q;
        if (d0 >= r_lo && d0 + 4u <= r_hi) have |= 1u << q;
      }
    } else {
      uint32_t k = kv;
      uint32_t k_end = rel[k + 1];
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t d0 = b + 4u * q;
        const uint32_t x0 = d0 > r_lo ? d0 : r_lo, x1 = d0 + 4u < r_hi ? d0 + 4u : r_hi;
        uint32_t word = 0;
        for (uint32_t cur = x0; cur < x1;) {
          while (k + 1 < n && cur >= k_end) {
            k++;
            k_end = rel[k + 1];
          }
          const uint32_t seg_end = x1 < k_end ? x1 : k_end;
          const uint32_t sp = from_dict ? L.src[k] + (cur - rel[k]) : src0 + (rel[k] - r_lo) + hole * k + (cur - rel[k]);
          const uint32_t v = sp < n_st ? img4(img, sp) : 0u;  // (DICT: sp is the entry's offset in the page)
          const uint32_t nb = seg_end - cur;
          const uint32_t msk = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8u * nb)) - 1u);
          word |= (v & msk) << (8u * (cur - d0));
          cur = seg_end;
        }
        wd[q] = word;
        if (x0 == d0 && x1 == d0 + 4u) have |= 1u << q;
      }
    }
    if (!dst_al4) have = 0;  // unaligned byte buffer (C ABI caller): byte stores only
    store_block16(dst, a0 + b, o_lo, o_hi, wd, have, dst_al16);
  }
  }
}

// ---------------------------------------------------------------------------
// DELTA_BYTE_ARRAY values (DeltaByteArrayReader.readBytes :57-79): value i = the first prefix_i
// bytes of value i - 1, then suffix i. k_delta MODE 2 left bsrc = prefix length, blen = value
// length (0 from the first invalid value on; the errors are reported there), PageWork::aux = start
// of the suffix bytes and, per chunk of BIN_CHUNK values, {suffix bytes before the chunk, smallest
// prefix length m_c in the chunk} (dba_meta).
//
// The dependency is serial across values, but only through the LAST value of each chunk: value
// i of chunk c needs nothing from before the chunk except the chunk's previous value, i.e. the
// last value T_{c-1} of chunk c - 1, and T_c = the first m_c bytes of T_{c-1}, then bytes that
// come from chunk c's own suffixes. So:
//   k_dba_tail    (one wave per chunk)  writes the own bytes [m_c, |T_c|) of T_c into the output:
//                 value y of the chunk supplies bytes [P_y, min P_{y+1..last}) (suffix minimum);
//   k_dba_chain_par (one wave per chunk) writes the inherited bytes [0, m_c) of every T_c, each
//                 copied from the last earlier T whose own bytes hold it (k_dba_chain: pages of more
//                 than DCP chunks follow T_0, T_1, ... in LDS, one short step per chunk);
//   k_dba_chunks  (one wave per chunk)  with T_{c-1} read back as the previous value, assembles
//                 the chunk's values one after another (LDS, byte-parallel per value).
// A page with a value longer than DBA_VB (PageWork::reserved, set by k_delta) is copied by
// k_dba_copy, the same per-value loop over the whole page with long previous values read back
// from the output.
constexpr uint32_t DBA_SB = 3072;  // LDS suffix staging bytes per batch (a chunk, in k_dba_chunks)
constexpr uint32_t DBA_OB = 4096;  // LDS output bytes of a byte-parallel batch

// LDS of the byte-parallel batch (k_dba_chunks): the batch's values are assembled in obuf, lane
// k writing value k as segments: its suffix [P_k, L_k), then [P_y, P_prev) from the suffix of
// y = the previous value with a strictly smaller prefix length (the bytes every value between
// them inherits unchanged), and so on down to prefix 0 or, past the batch start, the previous
// batch's last value.
struct DbaPar {
  uint8_t obuf_raw[16 + DBA_OB + 32];  // obuf = obuf_raw + 16 (slack for unaligned dword reads)
  uint16_t pmin[6][WAVE];              // pmin[s][x] = min prefix length over values (x - 2^s, x] (<= DBA_VB)
  uint16_t sx[WAVE];                   // suffix offset of value x in the staging buffer (<= DBA_SB)
  uint8_t pse[WAVE];                   // previous value with a smaller prefix length (255: none)
};

// Output byte offset of column value v: BYTE_ARRAY from the offset scan; FIXED_LEN_BYTE_ARRAY
// (every value type_length bytes, checked by k_delta) at v * type_length of `values`.
__device__ __forceinline__ uint64_t dba_off(const ColumnDev& cd, uint64_t v) {
  return cd.physical_type == PQG_FIXED_LEN_BYTE_ARRAY ? v * (uint64_t)(uint32_t)cd.type_length
                                                      : (uint64_t)((const int64_t*)cd.values)[v];
}

// One batch of <= 64 values assembled in LDS and stored (the byte-parallel path): lane k holds value
// k's length L, prefix length P (<= L), suffix offset sx in the staging sb8 and output offset lx in
// the batch (ltot bytes in all, <= DBA_OB; every L <= DBA_VB); prevb is the value before the batch,
// the batch's last value goes to vlast; o_lo: output offset of the batch's first byte.
__device__ __forceinline__ void dba_batch(DbaPar* par, const uint8_t* sb8, const uint8_t* prevb, uint8_t* vlast, bool in,
                                          uint32_t L, uint32_t P, uint32_t sx, uint32_t lx, uint32_t ltot, uint32_t nb,
                                          uint64_t o_lo, uint8_t* dst, uint64_t cap) {
  const uint32_t lane = lane_id();
  uint32_t mv = in ? P : 0xFFFFFFFFu;
#pragma unroll
  for (uint32_t st = 0; st < 6; st++) {
    if (st) {
      const uint32_t y = __shfl_up(mv, 1u << (st - 1));
      if (lane >= (1u << (st - 1))) mv = y < mv ? y : mv;
    }
    par->pmin[st][lane] = (uint16_t)(mv < 0xFFFFu ? mv : 0xFFFFu);
  }
  par->sx[lane] = (uint16_t)sx;
  wave_sync();
  uint32_t ps = 255u;
  if (in && P > 0) {  // max{y < lane : P_y <= P - 1}
    int y = (int)lane - 1;
    const uint32_t th = P - 1u;
#pragma unroll
    for (int st = 5; st >= 0; st--)
      if (y >= (1 << st) - 1 && par->pmin[st][y] > th) y -= 1 << st;
    ps = y < 0 ? 255u : (uint32_t)y;
  }
  par->pse[lane] = (uint8_t)ps;
  wave_sync();
  uint8_t* obuf = par->obuf_raw + 16;
  if (in) {
    uint8_t* ob = obuf + lx;
    uint32_t y = lane, hi = L, lo = P, sxy = sx;
    while (true) {
      for (uint32_t b = lo; b < hi; b++) ob[b] = sb8[sxy + (b - lo)];  // suffix of y
      if (lo == 0) break;
      hi = lo;
      y = par->pse[y];
      if (y == 255u) {  // inherited from before the batch
        for (uint32_t b = 0; b < hi; b++) ob[b] = prevb[b];
        break;
      }
      lo = par->pmin[0][y];
      sxy = par->sx[y];
    }
  }
  wave_sync();
  // the batch's bytes -> output, 16-byte blocks (edges shared with the neighbouring
  // batches / chunks are stored bytewise)
  const uint64_t o_end = o_lo + ltot;
  const uint64_t o_hi = o_end < cap ? o_end : cap;
  const bool dst_al16 = ((uintptr_t)dst & 15u) == 0, dst_al4 = ((uintptr_t)dst & 3u) == 0;
  typedef uint32_t __attribute__((may_alias)) u32a;
  for (uint64_t a = (o_lo & ~15ull) + 16u * lane; a < o_hi; a += 16u * WAVE) {
    const int32_t rel = (int32_t)(int64_t)(a - o_lo);  // >= -15
    const int32_t rb = rel & ~3;
    const uint32_t sb = (uint32_t)rel & 3u;
    uint32_t w[5], wd[4], have = 0;
#pragma unroll
    for (uint32_t c = 0; c < 5; c++) w[c] = *(const u32a*)(obuf + rb + 4 * (int32_t)c);
#pragma unroll
    for (uint32_t c = 0; c < 4; c++) {
      wd[c] = __builtin_amdgcn_alignbyte(w[c + 1], w[c], sb);
      const uint64_t d0 = a + 4u * c;
      if (d0 >= o_lo && d0 + 4u <= o_hi) have |= 1u << c;
    }
    store_block16(dst, a, o_lo, o_hi, wd, dst_al4 ? have : 0u, dst_al16);
  }
  // the batch's last value becomes the previous value
  const uint32_t ll = rdl(L, nb - 1), lxl = rdl(lx, nb - 1);
  for (uint32_t b = lane; b < ll; b += WAVE) vlast[b] = obuf[lxl + b];
}

// Values [i_beg, i_end) of a page, in order. The previous value is in vbuf[cur ^ 1] when
// prev_lds; otherwise at output offset prev_off. sp: page-relative position of value i_beg's suffix.
__device__ __forceinline__ void dba_values(const ColumnDev& cd, uint64_t v0, rsrc_t rs, uint32_t i_beg, uint32_t i_end,
                                           uint32_t sp, uint8_t* vb0, uint8_t* vb1, uint32_t* sbuf, uint32_t cur,
                                           bool prev_lds, uint64_t prev_off, DbaPar* par = nullptr) {
  uint8_t* vbuf[2] = {vb0, vb1};  // value buffers (DBA_VB bytes; one may be par's assembly buffer)
  const uint32_t lane = lane_id();
  uint8_t* dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  const uint8_t* sb8 = (const uint8_t*)sbuf;
  for (uint32_t i0 = i_beg; i0 < i_end; i0 += WAVE) {
    const uint32_t i = i0 + lane;
    const bool in = i < i_end;
    const uint32_t L = in ? cd.blen[v0 + i] : 0u;
    uint32_t P = in ? cd.bsrc[v0 + i] : 0u;
    P = P < L ? P : L;
    const uint32_t S = L - P;
    uint32_t stot;
    const uint32_t sx = wave_excl_scan_u32(S, &stot);
    const uint64_t off = in ? dba_off(cd, v0 + i) : 0;
    const bool staged = stot <= DBA_SB;
    if (staged) {
      for (uint32_t o = 4u * lane; o < stot; o += 4u * WAVE) sbuf[o >> 2] = ld4_any(rs, sp + o);
      wave_sync();
    }
    // the batch's loads are complete before the value loop: otherwise the compiler cannot tell
    // at the loop head whether `off` has arrived and waits with vmcnt(0) — for every store of
    // the previous value — once per value
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t nb = i_end - i0 < WAVE ? i_end - i0 : WAVE;
    if (par && staged && prev_lds) {
      const uint32_t lmax = uni(wave_max_u32(L));
      uint32_t ltot;
      const uint32_t lx = wave_excl_scan_u32(L, &ltot);
      ltot = uni(ltot);
      if (lmax <= DBA_VB && ltot <= DBA_OB) {
        const uint64_t o_lo = ((uint64_t)rdl((uint32_t)(off >> 32), 0) << 32) | rdl((uint32_t)off, 0);
        if (vbuf[cur ^ 1] == par->obuf_raw + 16) {  // the previous value sits in the assembly buffer
          for (uint32_t b = lane; b < DBA_VB; b += WAVE) vbuf[cur][b] = vbuf[cur ^ 1][b];
          wave_sync();
          cur ^= 1;
        }
        // the batch's last value replaces the previous one in the same buffer
        dba_batch(par, sb8, vbuf[cur ^ 1], vbuf[cur ^ 1], in, L, P, sx, lx, ltot, nb, o_lo, dst, cap);
        sp += stot;
        wave_sync();  // the next batch overwrites the staging buffers
        continue;
      }
    }
    for (uint32_t t = 0; t < nb; t++) {
      const uint32_t len = rdl(L, t), pre = rdl(P, t), so = rdl(sx, t);
      const uint64_t o = ((uint64_t)rdl((uint32_t)(off >> 32), t) << 32) | rdl((uint32_t)off, t);
      if (len == 0) {  // empty value (or past an error)
        prev_lds = true;
        cur ^= 1;
        continue;
      }
      const bool fits = len <= DBA_VB;
      if (pre && !prev_lds) __builtin_amdgcn_s_waitcnt(0);  // the previous value's stores, read below
      for (uint32_t j = lane; j < len; j += WAVE) {
        uint32_t b;
        if (j < pre) {
          if (prev_lds) {
            b = vbuf[cur ^ 1][j];
          } else {
            const uint64_t a = prev_off + j;
            b = a < cap ? (sld((const uint32_t*)(dst + (a & ~3ull))) >> ((a & 3u) * 8u)) & 0xFFu : 0u;
          }
        } else {
          const uint32_t q = so + j - pre;
          b = staged ? sb8[q] : (ld32(rs, (sp + q) & ~3u) >> (((sp + q) & 3u) * 8u)) & 0xFFu;
        }
        if (fits) vbuf[cur][j] = (uint8_t)b;
        if (o + j < cap) gst(dst + o + j, (uint8_t)b);
      }
      wave_sync();
      prev_lds = fits;
      prev_off = o;
      cur ^= 1;
    }
    sp += stot;
    wave_sync();  // the next batch overwrites the staging buffer
  }
}

// Serial copy of the pages with a value longer than DBA_VB (PageWork::reserved).
__global__ __launch_bounds__(64 * WPB) void k_dba_copy(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                       const PageWork* __restrict__ work,
                                                       const ColumnDev* __restrict__ cols,
                                                       const int32_t* __restrict__ list, int n_list) {
  __shared__ uint8_t vbuf_all[WPB][2][DBA_VB];
  __shared__ uint32_t sbuf_all[WPB][DBA_SB / 4 + 1];
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  const PageWork& pw = work[page];
  if (uni(pw.reserved) != 1u) return;
  const ColumnDev& cd = cols[pw.column];
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  dba_values(cd, pw.out_offset, rs, 0, uni(pw.n_values), uni(pw.aux), vbuf_all[wave_id()][0], vbuf_all[wave_id()][1],
             sbuf_all[wave_id()], 0,
             true, 0);
}

// Chunk (page, j) of the chunk list -> its value range; false when the chunk holds no value or
// its page takes the serial copy.
__device__ __forceinline__ bool dba_chunk(const PageWork* work, const uint64_t* chunks, uint32_t c, int& page,
                                          uint32_t& j, uint32_t& i_lo, uint32_t& i_hi) {
  const uint64_t ch = chunks[c];
  page = (int)(uint32_t)ch;
  j = (uint32_t)(ch >> 32);
  const PageWork& pw = work[page];
  const uint32_t nv = uni(pw.n_values);
  i_lo = j * BIN_CHUNK;
  if (uni(pw.reserved) || i_lo >= nv) return false;
  i_hi = i_lo + BIN_CHUNK < nv ? i_lo + BIN_CHUNK : nv;
  return true;
}

// Own bytes of the chunk's last value: value y supplies bytes [P_y, R_y), R_y = min(P_{y+1..last})
// (R_last = its length); those intervals tile [m_c, L_last). Byte b's supplier is therefore
// y(b) = max{y : P_y <= b}, found per byte by a descent over a prefix-min table of the chunk's P (the
// batch assembly's previous-smaller search): one lane per byte, every byte's load in flight at once
// (a lane walking its values' byte ranges waited for one load per byte).
__global__ __launch_bounds__(64 * WPB) void k_dba_tail(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                       const PageWork* __restrict__ work,
                                                       const ColumnDev* __restrict__ cols,
                                                       const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                       const uint32_t* __restrict__ meta) {
  static_assert(BIN_CHUNK == 4 * WAVE, "a chunk is 4 values per lane");
  constexpr uint32_t LV = 8;                        // table levels: windows of 1 .. 128 values
  __shared__ uint16_t pm_all[WPB][LV][BIN_CHUNK];   // pm[s][x] = min P over values (x - 2^s, x] (<= DBA_VB)
  __shared__ uint32_t sx_all[WPB][BIN_CHUNK];       // suffix offset of value x in the chunk
  const uint32_t c = blockIdx.x * WPB + wave_id();
  if (c >= n_chunks) return;
  int page;
  uint32_t j, i_lo, i_hi;
  if (!dba_chunk(work, chunks, c, page, j, i_lo, i_hi)) return;
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint64_t v0 = pw.out_offset;
  const uint32_t n = i_hi - i_lo;
  const uint32_t last = n - 1;
  uint16_t(*pm)[BIN_CHUNK] = pm_all[wave_id()];
  uint32_t* sxa = sx_all[wave_id()];
  // lane holds values y = 4 * lane + q of the chunk
  uint32_t Lq[4], Pq[4], s_lane = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint32_t y = 4u * lane + q;
    const bool in = y < n;
    Lq[q] = in ? cd.blen[v0 + i_lo + y] : 0u;
    Pq[q] = in ? cd.bsrc[v0 + i_lo + y] : 0u;
  }
  const uint32_t L_last = uni(cd.blen[v0 + i_lo + last]);
  const uint64_t o_last = dba_off(cd, v0 + i_lo + last);
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  const uint32_t sp = uni(pw.aux) + meta[2u * ((uint64_t)pw.chunk_base + j)];
  if (L_last == 0) return;  // (an error in the chunk leaves its last value empty)
  uint32_t pmin_l = 0xFFFFu;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint32_t y = 4u * lane + q;
    const uint32_t P = y < n ? (Pq[q] < Lq[q] ? Pq[q] : Lq[q]) : 0xFFFFu;
    s_lane += y < n ? Lq[q] - P : 0u;
    pm[0][y] = (uint16_t)P;
  }
  uint32_t stot;
  uint32_t sx = wave_excl_scan_u32(s_lane, &stot);
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint32_t y = 4u * lane + q;
    sxa[y] = sx;
    const uint32_t P = pm[0][y];
    pmin_l = P < pmin_l ? P : pmin_l;
    sx += y < n ? Lq[q] - P : 0u;
  }
  const uint32_t m_c = uni(wave_min_u32(pmin_l));
  wave_sync();
  for (uint32_t sl = 1; sl < LV; sl++) {
    const uint32_t h = 1u << (sl - 1);
    uint32_t v[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint32_t x = 4u * lane + q;
      const uint32_t a = pm[sl - 1][x], b = x >= h ? pm[sl - 1][x - h] : 0xFFFFu;
      v[q] = a < b ? a : b;
    }
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) pm[sl][4u * lane + q] = (uint16_t)v[q];
    wave_sync();
  }
  uint8_t* dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  for (uint32_t b0 = m_c; b0 < L_last; b0 += WAVE) {
    const uint32_t b = b0 + lane;
    if (b < L_last) {
      int y = (int)last;
#pragma unroll
      for (int sl = LV - 1; sl >= 0; sl--)
        if (y >= (1 << sl) - 1 && (uint32_t)pm[sl][y] > b) y -= 1 << sl;
      y = y < 0 ? 0 : y;  // (b >= m_c: found)
      const uint32_t a = sp + sxa[y] + (b - pm[0][y]);
      const uint32_t v = (ld32(rs, a & ~3u) >> ((a & 3u) * 8u)) & 0xFFu;
      if (o_last + b < cap) gst(dst + o_last + b, (uint8_t)v);
    }
  }
}

// Inherited bytes of every chunk's last value, all chunks at once (pages of at most DCP chunks; the
// serial k_dba_chain below takes the others). With k_c = min(m_c, |T_c|) the bytes T_c inherits (k_0 =
// 0: T_0 is all own bytes), T_c[b] = T_{c-1}[b] for b < k_c unrolls to T_c[b] = T_{c*}[b] with
// c* = max{c' < c : k_{c'} <= b}: an own byte of T_{c*}, written by k_dba_tail (an earlier launch). One
// wave per chunk finds c* per byte by a descent over a min table of the page's k (the previous-smaller
// search of the batch assembly, over chunks), then copies the bytes: no per-page serial step.
constexpr uint32_t DCP = 256;     // chunks per page of the parallel chain
constexpr uint32_t DCP_LV = 8;    // table levels: windows of 1 .. 2^(DCP_LV - 1) chunks (descent reach 2^DCP_LV - 1)
__global__ __launch_bounds__(64 * WPB) void k_dba_chain_par(const PageWork* __restrict__ work,
                                                            const ColumnDev* __restrict__ cols,
                                                            const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                            const uint32_t* __restrict__ meta) {
  __shared__ uint16_t mk_all[WPB][DCP_LV][DCP];  // mk[s][x] = min k over chunks (x - 2^s, x]
  const uint32_t cid = blockIdx.x * WPB + wave_id();
  if (cid >= n_chunks) return;
  int page;
  uint32_t j, i_lo, i_hi;
  if (!dba_chunk(work, chunks, cid, page, j, i_lo, i_hi) || j == 0) return;
  const PageWork& pw = work[page];
  const uint32_t nv = uni(pw.n_values);
  const uint32_t nch = (nv + BIN_CHUNK - 1) / BIN_CHUNK;
  if (nch > DCP) return;
  const ColumnDev& cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint64_t v0 = pw.out_offset;
  uint8_t* dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  const uint32_t* m = meta + 2u * (uint64_t)pw.chunk_base;
  uint16_t(*mk)[DCP] = mk_all[wave_id()];
  auto last_of = [&](uint32_t c) __attribute__((always_inline)) {
    return (c + 1) * BIN_CHUNK < nv ? (c + 1) * BIN_CHUNK - 1 : nv - 1;
  };
  // k of chunks 0 .. j (k_j: the bytes this chunk's last value inherits); lengths <= DBA_VB (16 bits)
  uint32_t kq[DCP / WAVE];
#pragma unroll
  for (uint32_t r = 0; r < DCP / WAVE; r++) {
    const uint32_t c = lane + r * WAVE;
    uint32_t k = 0;
    if (c > 0 && c <= j) {
      const uint32_t Ll = cd.blen[v0 + last_of(c)], mc = m[2u * c + 1u];
      k = mc < Ll ? mc : Ll;
    }
    kq[r] = k;
  }
#pragma unroll
  for (uint32_t r = 0; r < DCP / WAVE; r++)
    if (lane + r * WAVE <= j) mk[0][lane + r * WAVE] = (uint16_t)kq[r];
  wave_sync();
  const uint32_t kj = uni((uint32_t)mk[0][j]);
  if (kj == 0) return;
  for (uint32_t s = 1; s < DCP_LV; s++) {
#pragma unroll
    for (uint32_t r = 0; r < DCP / WAVE; r++) {
      const uint32_t x = lane + r * WAVE;
      if (x < j) {
        const uint32_t h = 1u << (s - 1);
        const uint32_t a = mk[s - 1][x], b = x >= h ? mk[s - 1][x - h] : 0xFFFFu;
        mk[s][x] = (uint16_t)(a < b ? a : b);
      }
    }
    wave_sync();
  }
  const uint64_t oj = dba_off(cd, v0 + last_of(j));
  for (uint32_t b0 = 0; b0 < kj; b0 += WAVE) {
    const uint32_t b = b0 + lane;
    if (b >= kj) break;
    // c* = max{c' <= j - 1 : k_{c'} <= b} (k_0 = 0: always found)
    int y = (int)j - 1;
#pragma unroll
    for (int sl = DCP_LV - 1; sl >= 0; sl--)
      if (y >= (1 << sl) - 1 && (uint32_t)mk[sl][y] > b) y -= 1 << sl;
    y = y < 0 ? 0 : y;
    const uint64_t os = dba_off(cd, v0 + last_of((uint32_t)y));
    if (os + b < cap && oj + b < cap) gst(dst + oj + b, dst[os + b]);
  }
}

// Inherited bytes of every chunk's last value, chunk after chunk of one page: T_c[0, m_c) =
// T_{c-1}[0, m_c), with T kept in LDS (the own bytes come from k_dba_tail's output).
__global__ __launch_bounds__(64 * WPB) void k_dba_chain(const PageWork* __restrict__ work,
                                                        const ColumnDev* __restrict__ cols,
                                                        const int32_t* __restrict__ list, int n_list,
                                                        const uint32_t* __restrict__ meta) {
  __shared__ uint8_t tbuf_all[WPB][DBA_VB];
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  const PageWork& pw = work[page];
  if (uni(pw.reserved)) return;
  const ColumnDev& cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint32_t nv = uni(pw.n_values);
  const uint32_t nch = (nv + BIN_CHUNK - 1) / BIN_CHUNK;
  if (nch <= 1 || nch <= DCP) return;  // (pages of <= DCP chunks: k_dba_chain_par)
  const uint64_t v0 = pw.out_offset;
  uint8_t* dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  uint8_t* T = tbuf_all[wave_id()];
  const uint32_t* m = meta + 2u * (uint64_t)pw.chunk_base;
  // T_0 = chunk 0's last value (all own bytes: its first value has prefix 0)
  uint32_t tl = uni(cd.blen[v0 + BIN_CHUNK - 1]);
  {
    const uint64_t o = dba_off(cd, v0 + BIN_CHUNK - 1);
    for (uint32_t b = lane; b < tl; b += WAVE) T[b] = o + b < cap ? dst[o + b] : 0;
  }
  wave_sync();
  for (uint32_t c = 1; c < nch; c++) {
    const uint32_t il = (c + 1) * BIN_CHUNK < nv ? (c + 1) * BIN_CHUNK - 1 : nv - 1;
    const uint32_t Ll = uni(cd.blen[v0 + il]);
    const uint32_t mc = uni(m[2u * c + 1u]);
    const uint64_t o = dba_off(cd, v0 + il);
    const uint32_t k = mc < Ll ? mc : Ll;  // inherited bytes (<= |T_{c-1}| for a valid page)
    // own bytes [k, Ll) were written by k_dba_tail (an earlier launch): load them first
    uint8_t own[DBA_VB / WAVE];
#pragma unroll
    for (uint32_t r = 0; r < DBA_VB / WAVE; r++) {
      const uint32_t b = lane + r * WAVE;
      own[r] = (b >= k && b < Ll && o + b < cap) ? dst[o + b] : 0;
    }
#pragma unroll
    for (uint32_t r = 0; r < DBA_VB / WAVE; r++) {
      const uint32_t b = lane + r * WAVE;
      if (b < k && o + b < cap) gst(dst + o + b, T[b]);
    }
    wave_sync();
#pragma unroll
    for (uint32_t r = 0; r < DBA_VB / WAVE; r++) {
      const uint32_t b = lane + r * WAVE;
      if (b >= k && b < Ll) T[b] = own[r];
    }
    wave_sync();
    tl = Ll;
  }
  (void)tl;
}

// The chunk's values in order, the previous value being T_{c-1} (complete in the output after
// k_dba_tail and k_dba_chain).
__global__ __launch_bounds__(64 * WPB) void k_dba_chunks(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                         const PageWork* __restrict__ work,
                                                         const ColumnDev* __restrict__ cols,
                                                         const uint64_t* __restrict__ chunks, uint32_t n_chunks,
                                                         const uint32_t* __restrict__ meta) {
  __shared__ uint8_t vbuf_all[WPB][DBA_VB];  // the previous value (one buffer: 4 waves per SIMD)
  __shared__ uint32_t sbuf_all[WPB][DBA_SB / 4 + 1];
  __shared__ __attribute__((aligned(16))) DbaPar par_all[WPB];
  const uint32_t c = blockIdx.x * WPB + wave_id();
  if (c >= n_chunks) return;
  int page;
  uint32_t j, i_lo, i_hi;
  if (!dba_chunk(work, chunks, c, page, j, i_lo, i_hi)) return;
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t lane = lane_id();
  const uint64_t v0 = pw.out_offset;
  uint8_t* vb = vbuf_all[wave_id()];
  DbaPar* par = &par_all[wave_id()];
  uint32_t* sbuf = sbuf_all[wave_id()];
  uint8_t* dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  // every load of the chunk at once, so that the chunk costs two memory round trips (these, then its
  // suffix bytes and previous value) instead of two per 64-value batch: lengths and prefix lengths
  // (lane: values 64 q + lane), each batch's output offset, the previous value's length and offset
  static_assert(BIN_CHUNK == 4 * WAVE, "a chunk is 4 batches of 64 values");
  const uint32_t n = i_hi - i_lo;
  uint32_t Lq[4], Pq[4];
  uint64_t oq[4];
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint32_t i = WAVE * q + lane;
    const bool in = i < n;
    Lq[q] = in ? cd.blen[v0 + i_lo + i] : 0u;
    Pq[q] = in ? cd.bsrc[v0 + i_lo + i] : 0u;
    oq[q] = WAVE * q < n ? dba_off(cd, v0 + i_lo + WAVE * q) : 0;
  }
  const uint32_t lp = i_lo ? uni(cd.blen[v0 + i_lo - 1]) : 0u;
  const uint64_t po = i_lo ? dba_off(cd, v0 + i_lo - 1) : 0;
  const uint32_t sp = uni(uni(pw.aux) + meta[2u * ((uint64_t)pw.chunk_base + j)]);
  uint32_t sxq[4], lxq[4], ltq[4], sbase = 0;
  bool fits = true;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    Pq[q] = Pq[q] < Lq[q] ? Pq[q] : Lq[q];
    uint32_t st, lt;
    sxq[q] = sbase + wave_excl_scan_u32(Lq[q] - Pq[q], &st);
    lxq[q] = wave_excl_scan_u32(Lq[q], &lt);
    sbase += uni(st);
    ltq[q] = uni(lt);
    fits = fits && ltq[q] <= DBA_OB;
  }
  fits = fits && sbase <= DBA_SB;
  // the chunk's suffix bytes and the previous value (-> vb)
  if (fits)
    for (uint32_t o = 4u * lane; o < sbase; o += 4u * WAVE) sbuf[o >> 2] = ld4_any(rs, sp + o);
  for (uint32_t b = lane; b < lp; b += WAVE) vb[b] = po + b < cap ? dst[po + b] : 0;
  __builtin_amdgcn_s_waitcnt(0);
  wave_sync();
  if (!fits) {  // batch by batch, with the per-value path for batches past the LDS buffers
    // (the assembly buffer is the per-value path's second value buffer: previous value in vb = vbuf[cur ^ 1])
    dba_values(cd, v0, rs, i_lo, i_hi, sp, par->obuf_raw + 16, vb, sbuf, 0, true, 0, par);
    return;
  }
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    if (WAVE * q >= n) break;
    const uint32_t nb = n - WAVE * q < WAVE ? n - WAVE * q : WAVE;
    // the batch's last value replaces the previous one in vb (read only during the assembly)
    dba_batch(par, (const uint8_t*)sbuf, vb, vb, WAVE * q + lane < n, Lq[q], Pq[q], sxq[q], lxq[q], ltq[q], nb, oq[q],
              dst, cap);
    wave_sync();  // the next batch overwrites the batch tables and reads the value just copied
  }
}

// PQG_PAGE_DBA_CARRY pages (PARQUET-246): one wave per column walks the column's DELTA_BYTE_ARRAY
// pages in page order. A flagged page starts from the column's previous value (value out_offset - 1,
// DeltaByteArrayReader.setPreviousReader :89-95) unless no value was decoded since the last unflagged
// page (the start of a column chunk), whose reader starts empty; its first value's prefix is checked
// against that previous value here (readBytes :72-74: arraycopy past previous.length), then the page
// is copied value after value (dba_values). Unflagged pages were copied by the launches before.
__global__ __launch_bounds__(64) void k_dba_carry(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                  const PageWork* __restrict__ work,
                                                  const ColumnDev* __restrict__ cols,
                                                  const int32_t* __restrict__ list, int n_list,
                                                  const int32_t* __restrict__ carry_cols, uint64_t* err,
                                                  ErrCount err_count) {
  __shared__ uint8_t vbuf[2][DBA_VB];
  __shared__ uint32_t sbuf[DBA_SB / 4 + 1];
  const int col = carry_cols[blockIdx.x];
  const ColumnDev& cd = cols[col];
  const uint32_t lane = lane_id();
  uint8_t* dst = cd.binary_data;
  const uint64_t cap = cd.binary_capacity;
  uint64_t chain_start = 0;  // first value of the current column chunk
  for (int k = 0; k < n_list; k++) {
    const int page = list[k];
    const PageWork& pw = work[page];
    if (uni(pw.column) != col) continue;
    const uint64_t v0 = pw.out_offset;
    if (uni(pw.reserved) != 2u) {
      chain_start = v0;
      continue;
    }
    const uint32_t nv = uni(pw.n_values);
    if (nv == 0) continue;
    bool prev_lds = true;
    uint64_t prev_off = 0;
    const uint32_t lp = v0 > chain_start ? uni(cd.blen[v0 - 1]) : 0u;  // the previous value's length
    {
      const int32_t pre0 = (int32_t)uni(cd.bsrc[v0]);
      const uint32_t L0 = uni(cd.blen[v0]);
      if (L0 != 0 && pre0 > 0 && (uint32_t)pre0 > lp) {
        if (lane == 0) report(err, err_count, page, 2, 0, PQG_ERR_CORRUPT);
        return;  // the reference throws here: nothing after this value is read
      }
    }
    if (lp > 0) {
      const uint64_t o = dba_off(cd, v0 - 1);
      __builtin_amdgcn_s_waitcnt(0);  // this wave's stores of the previous page, read back below
      if (lp <= DBA_VB) {
        for (uint32_t b = lane; b < lp; b += WAVE) {
          const uint64_t a = o + b;
          vbuf[1][b] = a < cap ? (uint8_t)((sld((const uint32_t*)(dst + (a & ~3ull))) >> ((a & 3u) * 8u)) & 0xFFu) : 0;
        }
        wave_sync();
      } else {
        prev_lds = false;
        prev_off = o;
      }
    }
    const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
    dba_values(cd, v0, rs, 0, nv, uni(pw.aux), vbuf[0], vbuf[1], sbuf, 0, prev_lds, prev_off);
  }
}

// ---------------------------------------------------------------------------
// PLAIN BYTE_ARRAY columns in one pass (k_bin_bases + k_bin_plain): the walk, the offsets and the
// value bytes of every 2 KiB tile of a page by one wave, without the per-value length / source
// scratch, the offset scan and the copy kernel of the per-value path.
//
// A PLAIN data section is N values back to back, each a 4-byte length then its bytes
// (BinaryPlainValuesReader.readBytes :35-42), so value i of a page lands at
//   offset_i = base(page) + (P_i - data_begin) - 4 i    (P_i: position of its length prefix)
// in the column's byte buffer, base(page) = the value bytes of the column's earlier pages. A page
// whose N values end exactly at the section end holds (size - data_begin - 4 N) value bytes, so
// base() is a prefix sum known before any walk (k_bin_bases). What a tile still needs is i: the
// number of values that start in the page before it. Each tile walks its own values (the first
// tile of the section from the section start; the others from a guessed first value start, see
// k_bin_walk_seg), publishes that count with the guessed entry and its exit, then looks back over
// up to 64 earlier tiles of the page at once (decoupled look-back): the nearest tile with an
// inclusive count plus the counts of the tiles after it, provided each of those tiles' entry is the
// exit of the tile before it (a misspeculated tile is waited for: it corrects itself). Tiles are
// taken in ticket order, so the tiles looked back on are running or done. The tile then publishes
// its inclusive count, writes its offsets, and composes its value bytes from the staged tile in
// LDS into 16-byte stores.
// A page whose N-th value does not end at the section end (bytes the reader ignores after the
// values) breaks the base() assumption: the tile holding that value raises a flag and pqg_sync
// re-runs the plan on the per-value path (k_bin_walk, offset scan, k_bin_copy), which reads
// exactly N values. Errors are reported at the index the per-value path reports (values past N are
// not read by the reference and raise nothing).
constexpr uint32_t BP_NEXT = 4u * WAVE;         // bytes of the next tile staged too (one dword per lane)
constexpr uint32_t BP_IMG = BW_WIN + BP_NEXT;    // staged bytes per tile (a value reaching past: from memory)
constexpr uint32_t BP_BLK = BW_WIN / 16u + 2u;  // output blocks that can hold a value start
constexpr uint64_t BP_NONE = 0xFFFFFFFFull;     // exit of a tile whose chain stopped (error, section end)

struct BinPlainLds {
  union {
    BinWalkLds w;                   // the tile walk (candidate list)
    uint32_t img[BP_IMG / 4 + 16];  // then: page bytes [B, B + BP_IMG) (+ slack for the compose reads)
  } u;
  union {
    uint32_t pj[BW_CAP];  // the guess's pointer jumping over the candidate list
    struct {
      uint16_t acc[BW_CAP + 2];  // accepted value starts of the tile (offsets from B), ascending
      uint16_t bt[BP_BLK + 2];   // output block -> the last value starting at or before its first byte
    };
  };
};
static_assert(sizeof(BinPlainLds) * WPB <= 160 * 1024 / 6, "6 workgroups of k_bin_plain per CU");

// Candidates of tile [B, B + BW_WIN) from position pos on (see bin_walk_core); returns their number
// (at most BW_CAP: eff_end is then the first candidate not listed).
// fast: only lengths below 256 (a value start of a longer value is then missing from the list, and
// the walk takes the tile again with every length): the byte before a length prefix, read as a
// length, is 256 x the true one plus a string byte, so short-string pages list (almost) only their
// true value starts: half the candidates, and batches whose candidates link one to the next.
__device__ __forceinline__ uint32_t bp_candidates(BinWalkLds& W, const BwBytes& cur, uint32_t B, uint32_t pos,
                                                  uint32_t end, uint32_t& eff_end, bool fast = false) {
  const uint32_t lane = lane_id();
  const uint32_t base = B + BW_Q * lane;
  uint32_t d[BW_Q / 4 + 1];
  d[0] = cur.a.x; d[1] = cur.a.y; d[2] = cur.a.z; d[3] = cur.a.w;
  d[4] = cur.b.x; d[5] = cur.b.y; d[6] = cur.b.z; d[7] = cur.b.w;
  d[8] = cur.x;
  uint32_t m = 0;
  const int32_t rem0 = (int32_t)(end - 4u - base);
  // (a zero-byte SWAR form of the short-length test, 9 dwords per lane, measured slower on C4's comment
  // column: 5.16 vs 5.00 ms, profiles/r05/binplain_swar)
  if (fast) {
#pragma unroll
    for (uint32_t q = 0; q < BW_Q; q++) {
      const uint32_t len = __builtin_amdgcn_alignbyte(d[(q >> 2) + 1], d[q >> 2], q & 3u);
      m |= (len < 256u && (int32_t)(len + q) <= rem0 ? 1u : 0u) << q;
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < BW_Q; q++) {
      const uint32_t len = __builtin_amdgcn_alignbyte(d[(q >> 2) + 1], d[q >> 2], q & 3u);
      const int32_t rem = rem0 - (int32_t)q;
      m |= (rem >= 0 && len <= (uint32_t)rem ? 1u : 0u) << q;
    }
  }
  if (base < pos) m &= pos - base >= BW_Q ? 0u : ~((1u << (pos - base)) - 1u);
  uint32_t total;
  const uint32_t rank = wave_excl_scan_u32((uint32_t)__builtin_popcount(m), &total);
  uint32_t mm = m, r = rank;
  while (mm) {
    const uint32_t q = (uint32_t)__builtin_ctz(mm);
    mm &= mm - 1u;
    if (r < BW_CAP) {
      const uint32_t i = q >> 2;
      uint32_t lo = d[0], hi = d[1];
#pragma unroll
      for (uint32_t t = 1; t < BW_Q / 4; t++) {
        const bool s = i == t;
        lo = s ? d[t] : lo;
        hi = s ? d[t + 1] : hi;
      }
      const uint32_t nx = base + q + 4u + __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
      *(uint64_t*)&W.pn[r] = (uint64_t)(base + q) | ((uint64_t)nx << 32);
    } else if (r == BW_CAP) {
      W.cut = base + q;
    }
    r++;
  }
  W.mr[lane] = uint2{m, rank};
  wave_sync();
  total = uni(total);
  eff_end = total > BW_CAP ? uni(W.cut) : B + BW_WIN;
  return total > BW_CAP ? BW_CAP : total;
}

struct BpWalk {
  uint32_t pos, n;  // where the chain left the tile (or stopped), values accepted
  int code;         // the error that stopped it (PQG_ERR_EOF also at the section end)
};

struct BpGuess {
  uint32_t pos, index, total, eff_end;  // guessed start (0xFFFFFFFF: none), its candidate index, the list
  bool fast;                            // the list holds short lengths only (bp_candidates fast)
};

// The chain from pos through tile [B, B + BW_WIN): accepted value starts to L.acc[0, n). With
// list0 < BW_CAP the candidate list of the whole tile is already in LDS (bp_guess) and pos is its
// candidate list0 (total0 candidates, listed up to eff0).
template <bool FAST, class LdsT>
__device__ BpWalk bp_walk(LdsT& L, const BwBytes& cur, rsrc_t rs, uint32_t B, uint32_t pos, uint32_t end,
                          uint32_t list0 = 0xFFFFFFFFu, uint32_t total0 = 0, uint32_t eff0 = 0, bool list_fast = false) {
  BinWalkLds& W = L.u.w;
  const uint32_t lane = lane_id();
  uint32_t n = 0;
  int code = 0;
  const uint32_t tend = B + BW_WIN;
  bool listed = list0 < BW_CAP;
  bool fast = listed ? list_fast : FAST;  // short lengths first; every length once a value start is missing
  while (true) {
    pos = uni(pos);
    n = uni(n);
    if (pos >= tend) break;
    if ((uint64_t)pos + 4u > end) { code = PQG_ERR_EOF; break; }
    uint32_t eff_end, total, i0 = 0;
    bool fast_pass = false;
    if (listed) {  // the guess's list, from the guessed candidate on
      total = total0;
      eff_end = eff0;
      i0 = list0;
      listed = false;
      fast_pass = fast;
    } else {
      wave_sync();  // the previous pass's list reads are done
      fast_pass = fast;
      total = bp_candidates(W, cur, B, pos, end, eff_end, fast_pass);
    }
    if (total == 0 || W.pn[i0].x != pos) {
      if (fast_pass) {  // pos is a longer value's start: list the tile again with every length
        fast = false;
        continue;
      }
      code = bin_value_error(rs, pos, end, false);
      break;
    }
    bool leave = false;
    while (true) {
      i0 = uni(i0);
      n = uni(n);
      const uint32_t k = i0 + lane;
      const uint32_t s = k < total ? W.pn[k].y : 0xFFFFFFFFu;
      const uint32_t so = s - B;
      const uint32_t t = so < BW_WIN ? bw_index(W, so) : 0xFFFFu;
      const bool hit = t < total && t > k && t - i0 < WAVE;
      const uint32_t J = hit ? t - i0 : WAVE;
      const uint64_t next1 = __ballot(hit && t == k + 1);
      uint32_t last = ~next1 ? (uint32_t)__builtin_ctzll(~next1) : WAVE - 1u;
      uint64_t mask = last == WAVE - 1u ? ~0ull : ((1ull << (last + 1u)) - 1ull);
      if (rdl(J, last) < WAVE) {  // a false candidate inside the batch: binary lifting from lane 0
        uint32_t P[6];
        P[0] = J;
#pragma unroll
        for (int q = 1; q < 6; q++) {
          const uint32_t g = (uint32_t)__shfl((int)P[q - 1], (int)(P[q - 1] & (WAVE - 1u)));
          P[q] = P[q - 1] < WAVE ? g : WAVE;
        }
        uint32_t x = 0;
#pragma unroll
        for (int q = 5; q >= 0; q--) {
          const uint32_t y = (uint32_t)__shfl((int)P[q], (int)x);
          if (y <= lane) x = y;
        }
        mask = __ballot(x == lane);
        last = 63u - (uint32_t)__builtin_clzll(mask);
      }
      const uint32_t rank = (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1ull));
      if ((mask >> lane) & 1ull) L.acc[n + rank] = (uint16_t)(W.pn[k].x - B);
      n += (uint32_t)__builtin_popcountll(mask);
      const uint32_t nxt = rdl(s, last);  // successor of the batch's last value
      pos = nxt;
      if (nxt >= eff_end) { leave = true; break; }
      const uint32_t a = uni(bw_index(W, nxt - B));
      if (a >= total || a <= i0 + last) {
        if (fast_pass) {  // the next value start has a longer length: list the rest again
          fast = false;
          break;
        }
        code = bin_value_error(rs, nxt, end, false);
        break;
      }
      i0 = a;
    }
    if (code) break;
    if (!leave && !(fast_pass && !fast)) break;
  }
  wave_sync();
  return BpWalk{uni(pos), uni(n), code};
}

// Guessed first value start of tile [B, B + BW_WIN) (a tile after the one holding the section
// start). A false candidate (typically the byte before a length prefix, which reads as a length of
// 256 x the true one) jumps far and lands, by chance, on the true chain about once in 20 tiles: a
// "first candidate whose links hold" rule picks it then. So every candidate's chain is followed to
// where it leaves the tile (pointer jumping over the candidate list: 9 rounds for 512 candidates)
// and the guess is the candidate with the most values on its chain among the first 64 whose chains
// stay on candidates (the true start's chain holds every true value start of the tile; a false chain
// that merges into it skips the values it jumps over), ties to the earliest; a chain that leaves the
// tile within SEG_LINKS links is checked on in memory. 0xFFFFFFFF when no candidate qualifies.
__device__ BpGuess bp_guess(BinPlainLds& L, const BwBytes& cur, rsrc_t rs, uint32_t B, uint32_t end) {
  BinWalkLds& W = L.u.w;
  uint32_t eff_end;
  const uint32_t lane = lane_id();
  {  // short-length candidates that link one to the next from the first to one leaving the tile: the
     // first is the guess (no pointer jumping; short-string pages, where false candidates are rare)
    const uint32_t tf = bp_candidates(W, cur, B, B, end, eff_end, true);
    bool ok = tf > 0;
    for (uint32_t k0 = 0; k0 < tf && ok; k0 += WAVE) {
      const uint32_t k = k0 + lane;
      bool good = true;
      if (k < tf) {
        const uint32_t sc = W.pn[k].y, so = sc - B;
        good = k + 1u < tf ? (so < BW_WIN && bw_index(W, so) == k + 1u) : sc >= eff_end;
      }
      ok = __ballot(!good) == 0ull;
    }
    if (ok) {
      const uint32_t g = uni(W.pn[0].x);
      wave_sync();
      return BpGuess{g, 0, tf, eff_end, true};
    }
    wave_sync();  // the exact list replaces it
  }
  const uint32_t total = bp_candidates(W, cur, B, B, end, eff_end);
  // node i: J = successor index, or (last index | 0x8000) once the chain leaves the list, 0xFFFF when
  // it breaks; D = values on the chain so far (L.pj: J | D << 16). 6 rounds: a chain of more than 64
  // values is not followed to its end but ranked by where its 64th value lies (the true start's chain
  // holds every value, so it gets there soonest)
  constexpr uint32_t NP = BW_CAP / WAVE;  // nodes per lane
  constexpr uint32_t XF = 0x8000u, BAD = 0xFFFFu;
  uint32_t v[NP];
#pragma unroll
  for (uint32_t j = 0; j < NP; j++) {
    const uint32_t i = lane + WAVE * j;
    uint32_t e = BAD | (1u << 16);
    if (i < total) {
      const uint32_t q = W.pn[i].y;
      const uint32_t t = q < eff_end ? bw_index(W, q - B) : 0xFFFFu;
      e = (q >= eff_end || q == end ? (i | XF) : (t < total ? t : BAD)) | (1u << 16);  // (end: the last value)
    }
    v[j] = e;
    L.pj[i] = e;
  }
  wave_sync();
  for (uint32_t r = 0; r < 6; r++) {
#pragma unroll
    for (uint32_t j = 0; j < NP; j++) {
      const uint32_t e = v[j];
      const uint32_t J = e & 0xFFFFu;
      if (J < XF) {  // not terminal: jump
        const uint32_t f = L.pj[J];
        v[j] = (f & 0xFFFFu) == BAD ? (BAD | (e & 0xFFFF0000u)) : ((f & 0xFFFFu) | ((e >> 16) + (f >> 16)) << 16);
      }
    }
    wave_sync();
#pragma unroll
    for (uint32_t j = 0; j < NP; j++) L.pj[lane + WAVE * j] = v[j];
    wave_sync();
  }
  const uint32_t e = lane < total ? v[0] : BAD;  // candidate `lane` (one of the first 64)
  const uint32_t J = e & 0xFFFFu;
  const uint32_t d = e >> 16;
  const bool term = J != BAD && (J & XF) != 0, lng = J < XF;
  bool ok = lane < total && (term || lng);
  uint32_t dmax = ok ? (lng ? 0xFFFFu : d) : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)dmax, o);
    dmax = y > dmax ? y : dmax;
  }
  // a chain of SEG_LINKS values inside the tile needs no further check; otherwise (long values) the
  // chains that leave the tile early are checked on in memory
  if (uni(dmax) < SEG_LINKS && ok) {
    uint32_t q = W.pn[J & 0x1FFu].y;
    for (uint32_t i = d; i < SEG_LINKS && ok; i++) {
      if (q >= end) break;  // the chain reaches the section end: nothing contradicts it
      ok = seg_candidate(rs, q, end);
      q = q + 4u + ld4_any(rs, q);
    }
  }
  // rank: long chains by where their 64th value lies (sooner first), then chains that leave the tile
  // by their values; ties to the earliest candidate
  const uint32_t score = lng ? 0x10000u + (0xFFFFu - (W.pn[J].x - B)) : d;
  uint32_t key = ok ? (score << 8) | (255u - lane) : 0u;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)key, o);
    key = y > key ? y : key;
  }
  key = uni(key);
  const uint32_t gi = 255u - (key & 0xFFu);
  const uint32_t g = key ? uni(W.pn[gi].x) : 0xFFFFFFFFu;
  wave_sync();
  return BpGuess{g, gi, total, eff_end, false};
}

// bp_emit for tiles whose values are all at least 4 bytes long, whose output fits 2 KiB and whose
// sources lie in img (C3's 4-32 byte strings, C4's comments): no block table. Output byte x (relative
// to the 16-byte aligned a0) of value k comes from img[x + C + 4 k], C = P_0 + 4 - B - r_lo, and k is
// the number of value starts 1..m-1 at or before x: the starts go into a 2,048-bit LDS bitmap (one
// dword per lane: lane l owns output bytes [32 l, 32 l + 32)), a wave scan of their popcounts gives
// each lane its first k, and each of its 8 output dwords is one unaligned LDS read (a start inside the
// dword: two, and a v_perm). Returns false (nothing written) when the tile does not qualify.
__device__ __forceinline__ bool bp_emit_fast(uint32_t* bm, const uint32_t* img, uint32_t img_len, const uint16_t* acc,
                                             uint32_t B, uint32_t beg, uint32_t rn, uint32_t rpos, uint32_t before,
                                             uint32_t m, const PageWork& pw, const ColumnDev& cd) {
  uint32_t lane = lane_id();
  asm volatile("" : "+v"(lane));  // (see bp_emit)
  auto pos_k = [&](uint32_t k) -> uint32_t { return k < rn ? B + acc[k] : rpos; };
  const uint64_t bb = pw.bin_base;
  const uint32_t P0 = uni(pos_k(0)), Pm = uni(pos_k(m));
  const uint64_t o_lo = bb + (uint64_t)(P0 - beg) - 4ull * before;
  const uint64_t o_hi0 = bb + (uint64_t)(Pm - beg) - 4ull * (uint64_t)(before + m);
  const uint64_t o_hi = o_hi0 < cd.binary_capacity ? o_hi0 : cd.binary_capacity;
  const uint64_t a0 = o_lo & ~15ull;
  if (o_lo >= o_hi || o_hi - a0 > 2048u || Pm - B + 8u > img_len) return false;
  bool short_v = false;
  for (uint32_t k = lane; k < m; k += WAVE) short_v |= pos_k(k + 1u) - pos_k(k) < 8u;  // value bytes < 4
  if (__ballot(short_v)) return false;
  const uint32_t r_lo = (uint32_t)(o_lo - a0), r_hi = (uint32_t)(o_hi - a0);
  // offsets of values before .. before + m (the last one: the end of value m - 1)
  int64_t* offs = (int64_t*)cd.values + pw.out_offset + before;
  for (uint32_t k = lane; k <= m; k += WAVE)
    gst(offs + k, (int64_t)(bb + (uint64_t)(pos_k(k) - beg) - 4ull * (uint64_t)(before + k)));
  // starts of values 1 .. m - 1 (output positions relative to a0; distinct: every value >= 4 bytes)
  bm[lane] = 0u;
  wave_sync();
  for (uint32_t k = lane + 1u; k < m; k += WAVE) {
    const uint32_t x = (pos_k(k) - P0) - 4u * k + r_lo;
    if (x < 2048u) __hip_atomic_fetch_or(&bm[x >> 5], 1u << (x & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  wave_sync();
  // starts before each 32-byte word of the output (lane w: word w), then lane l composes output blocks
  // l and 64 + l (bytes [16 l, + 16) and [1024 + 16 l, + 16)): each store instruction covers 1 KiB
  // of consecutive output (two blocks per lane side by side left every instruction's lines half
  // written: C4's comment column wrote 7.3 GB for 4.4 GB of output, profiles/r05/c4)
  uint32_t tot;
  const uint32_t kw = wave_excl_scan_u32((uint32_t)__builtin_popcount(bm[lane]), &tot);
  const uint32_t C = P0 + 4u - B - r_lo;
  uint8_t* dst = cd.binary_data;
  const bool dst_al16 = ((uintptr_t)dst & 15u) == 0, dst_al4 = ((uintptr_t)dst & 3u) == 0;
#pragma unroll
  for (uint32_t g = 0; g < 2; g++) {
    const uint32_t blk = 64u * g + lane, w = blk >> 1, half = 16u * (blk & 1u);
    const uint32_t bits = bm[w];
    const uint32_t k0 = (uint32_t)__shfl((int)kw, (int)w);  // starts before word w
    const uint32_t b = 16u * blk;
    uint32_t wd[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint32_t bo = half + 4u * q, x0 = b + 4u * q;
      const uint32_t k = k0 + (uint32_t)__builtin_popcount(bits & (0xFFFFFFFFu >> (31u - bo)));  // starts <= x0
      const uint32_t inner = (bits >> (bo + 1u)) & 7u;  // a start at x0 + 1 .. x0 + 3 (at most one)
      const int32_t s0 = (int32_t)(x0 + C + 4u * k);
      const uint32_t lo = img4(img, s0 > 0 ? (uint32_t)s0 : 0u);
      const uint32_t hi = img4(img, (uint32_t)(s0 + 4 > 0 ? s0 + 4 : 0));
      const uint32_t j = inner ? (uint32_t)__builtin_ctz(inner) + 1u : 4u;  // first byte of the next value
      const uint32_t sel = 0x03020100u + (0x04040404u & ~(j >= 4u ? 0xFFFFFFFFu : (1u << (8u * j)) - 1u));
      wd[q] = __builtin_amdgcn_perm(hi, lo, sel);
    }
    if (b >= r_hi) continue;
    uint32_t have = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint32_t d0 = b + 4u * q;
      if (d0 >= r_lo && d0 + 4u <= r_hi) have |= 1u << q;
    }
    if (!dst_al4) have = 0;
    store_block16(dst, a0 + b, o_lo, o_hi, wd, have, dst_al16);
  }
  return true;
}

// Offsets and value bytes of values [before, before + m) of a page, m <= rn: the rn values the walk
// accepted in tile [B, B + BW_WIN) start at B + acc[k], the chain left the tile at rpos; img holds the
// staged page bytes [B, B + img_len) (a value reaching further: the rest from memory). The offsets
// (offset_k = base(page) + (P_k - data_begin) - 4 k, the last one the end of value m - 1) go to the
// column's offsets, the value bytes are composed from img into 16-byte output blocks.
__device__ __forceinline__ void bp_emit(const uint32_t* img, uint32_t img_len, const uint16_t* acc, uint16_t* bt,
                                        rsrc_t rs, uint32_t B, uint32_t beg, uint32_t rn, uint32_t rpos,
                                        uint32_t before, uint32_t m, const PageWork& pw, const ColumnDev& cd) {
  // the lane index laundered through an empty volatile asm: lane-derived constants are recomputed per
  // call instead of being hoisted out of the caller's tile loop, where they were spilled to scratch
  // (a scratch reload waits for every store in flight)
  uint32_t lane = lane_id();
  asm volatile("" : "+v"(lane));
  // ---- offsets of values before .. before + m (the last one: the end of value m - 1)
  auto pos_k = [&](uint32_t k) -> uint32_t { return k < rn ? B + acc[k] : rpos; };
  int64_t* offs = (int64_t*)cd.values + pw.out_offset + before;
  const uint64_t bb = pw.bin_base;
  for (uint32_t k = lane; k <= m; k += WAVE)
    gst(offs + k, (int64_t)(bb + (uint64_t)(pos_k(k) - beg) - 4ull * (uint64_t)(before + k)));
  const uint64_t o_lo = bb + (uint64_t)(pos_k(0) - beg) - 4ull * before;
  const uint64_t o_hi0 = bb + (uint64_t)(pos_k(m) - beg) - 4ull * (uint64_t)(before + m);
  const uint64_t o_hi = o_hi0 < cd.binary_capacity ? o_hi0 : cd.binary_capacity;  // overflow: reported at sync
  if (o_lo >= o_hi) return;
  // ---- value bytes: 16-byte output blocks composed from the staged bytes
  const uint64_t a0 = o_lo & ~15ull;
  const uint32_t r_lo = (uint32_t)(o_lo - a0), r_hi = (uint32_t)(o_hi - a0);
  const uint32_t P0 = pos_k(0);
  auto rel = [&](uint32_t k) -> uint32_t { return (pos_k(k) - P0) - 4u * k + r_lo; };  // k <= m
  for (uint32_t i = lane; i < BP_BLK; i += WAVE) bt[i] = 0;
  wave_sync();
  for (uint32_t k = lane; k < m; k += WAVE) {
    const uint32_t blk = (rel(k) + 15u) >> 4;
    if (blk < BP_BLK && (k + 1u == m || ((rel(k + 1u) + 15u) >> 4) != blk)) bt[blk] = (uint16_t)k;
  }
  wave_sync();
  {  // running maximum over the blocks: 3 consecutive entries per lane, then across lanes
    constexpr uint32_t PER = (BP_BLK + WAVE - 1u) / WAVE;
    uint32_t v[PER], mx = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t i = PER * lane + j;
      v[j] = i < BP_BLK ? bt[i] : 0u;
      mx = v[j] > mx ? v[j] : mx;
    }
    uint32_t inc = mx;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
      if ((int)lane >= o) inc = y > inc ? y : inc;
    }
    uint32_t run = (uint32_t)__shfl_up((int)inc, 1);
    if (lane == 0) run = 0;
    wave_sync();
#pragma unroll
    for (uint32_t j = 0; j < PER; j++) {
      const uint32_t i = PER * lane + j;
      run = v[j] > run ? v[j] : run;
      if (i < BP_BLK) bt[i] = (uint16_t)run;
    }
  }
  wave_sync();
  uint8_t* dst = cd.binary_data;
  const bool dst_al16 = ((uintptr_t)dst & 15u) == 0, dst_al4 = ((uintptr_t)dst & 3u) == 0;
  for (uint32_t b = 16u * lane; b < r_hi; b += 16u * WAVE) {
    const uint32_t kv = (b >> 4) < BP_BLK ? bt[b >> 4] : m - 1u;  // value of the block's first byte
    const uint32_t bend = b + 16u < r_hi ? b + 16u : r_hi;
    const uint32_t rkv = rel(kv);
    const int64_t Sg = (int64_t)(pos_k(kv) + 4u - B) + (int64_t)b - (int64_t)rkv;  // staged offset of block byte 0
    uint32_t wd[4];
    uint32_t have = 0;
    const bool compose = !(kv + 5u < m && rel(kv + 5u) < bend) && Sg >= 0 && Sg + 36 <= (int64_t)img_len;
    if (compose) {
      uint64_t prof = 0;  // nibble i: value starts at or before byte i of the block
#pragma unroll
      for (uint32_t j = 1; j <= 4; j++) {
        const uint32_t kk = kv + j;
        const uint32_t pj = kk < m ? rel(kk) : 0xFFFFFFFFu;
        if (pj < bend) prof += 0x1111111111111111ull << (4u * (pj - b));
      }
      compose_block(img, (uint32_t)Sg, prof, wd);
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t d0 = b + 4u * q;
        if (d0 >= r_lo && d0 + 4u <= r_hi) have |= 1u << q;
      }
    } else {
      uint32_t k = kv;
      uint32_t k_end = rel(k + 1u);
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint32_t d0 = b + 4u * q;
        const uint32_t x0 = d0 > r_lo ? d0 : r_lo, x1 = d0 + 4u < r_hi ? d0 + 4u : r_hi;
        uint32_t word = 0;
        for (uint32_t c = x0; c < x1;) {
          while (k + 1u < m && c >= k_end) {
            k++;
            k_end = rel(k + 1u);
          }
          const uint32_t seg_end = x1 < k_end ? x1 : k_end;
          const uint32_t sp = pos_k(k) + 4u - B + (c - rel(k));  // page-relative: B + sp
          const uint32_t v = sp + 4u <= img_len ? img4(img, sp) : ld4_any(rs, B + sp);
          const uint32_t nb = seg_end - c;
          const uint32_t msk = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8u * nb)) - 1u);
          word |= (v & msk) << (8u * (c - d0));
          c = seg_end;
        }
        wd[q] = word;
        if (x0 == d0 && x1 == d0 + 4u) have |= 1u << q;
      }
    }
    if (!dst_al4) have = 0;  // unaligned byte buffer (C ABI caller): byte stores only
    store_block16(dst, a0 + b, o_lo, o_hi, wd, have, dst_al16);
  }
}


__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(6))) void k_bin_plain(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                        const PageWork* __restrict__ work,
                                                        const ColumnDev* __restrict__ cols,
                                                        const uint64_t* __restrict__ segs, uint32_t n_segs,
                                                        uint64_t* aggw, uint64_t* incw, uint32_t* ticket,
                                                        uint32_t epoch, uint32_t* inexact, uint32_t flag_epoch,
                                                        uint64_t* err, ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) BinPlainLds lds_all[WPB];
  const uint32_t lane = lane_id();
  // Tile t = workgroup order: workgroups are dispatched in index order, so the tiles a tile waits for
  // hold a slot (one atomic ticket per 2 KiB tile serialized on one address and dominated the kernel).
  // That order is not promised by the programming model: a wait that times out hands the plan to the
  // per-value path (the inexact flag) instead of failing the decode.
  const uint32_t t = blockIdx.x * WPB + wave_id();
  (void)ticket;
  if (t >= n_segs) return;
#ifdef PQG_DIAG
  const uint64_t dg0 = __builtin_amdgcn_s_memrealtime();
  uint64_t dg1 = 0, dg2 = 0, dg_polls = 0, dg_guess = 0;
#endif
  BinPlainLds& L = lds_all[wave_id()];
  const uint64_t sg = segs[t];
  const int page = (int)(uint32_t)sg;
  const uint32_t s = (uint32_t)(sg >> 32);  // tile of the page: bytes [s BW_WIN, (s + 1) BW_WIN)
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size), N = uni(pw.n_values);
  const uint32_t B = s * BW_WIN;
  const uint64_t E = (uint64_t)epoch << 56;
  const uint32_t s0 = beg / BW_WIN;  // the tile holding the section start
  if (s < s0 || N == 0 || beg >= end || B >= end) {  // no value starts here
    if (lane == 0) {
      sst(incw + t, E | BP_NONE);
      if (s == 0 && N > 0 && beg >= end) report(err, err_count, page, 2, 0, PQG_ERR_EOF);  // no section: value 0
      if (s == 0 && N == 0 && beg < end) sst(inexact, flag_epoch);  // bytes but no values: base() assumes none
    }
    return;
  }
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  const BwBytes cur = bw_load(rs, B);
  const uint32_t nxt = ld32(rs, B + BW_WIN + 4u * lane);  // the next tile's first BP_NEXT bytes
  const bool first = s == s0;
  const BpGuess gs = first ? BpGuess{beg, 0xFFFFFFFFu, 0, 0, false} : bp_guess(L, cur, rs, B, end);
  uint32_t entry = gs.pos;
#ifdef PQG_DIAG
  dg_polls = __builtin_amdgcn_s_memrealtime() + (entry == 7u ? 1u : 0u);  // (after the guess; polls below)
#endif
  BpWalk r{entry, 0, 0};
  if (entry != 0xFFFFFFFFu) {
    r = first ? bp_walk<true>(L, cur, rs, B, entry, end)
              : bp_walk<true>(L, cur, rs, B, entry, end, gs.index, gs.total, gs.eff_end, gs.fast);
    if (!first && lane == 0)  // speculative: count, guessed entry, exit, stop
      sst(aggw + t, E | ((uint64_t)r.n << 46) | ((uint64_t)(entry - B) << 35) | ((uint64_t)(r.code ? 1u : 0u) << 34) |
                        (uint64_t)r.pos);
  }
  uint32_t before = 0;
  bool stopped = false;
#ifdef PQG_DIAG
  dg1 = __builtin_amdgcn_s_memrealtime() + (r.n > 0xFFFFFFF0u ? 1u : 0u);
#endif
  if (!first) {
    const uint64_t t_wait = __builtin_amdgcn_s_memrealtime();
    while (true) {
      // lane l: the tile l + 1 before this one (down to the first tile of the section)
      const bool valid = s >= s0 + 1u + lane;
      const uint32_t u = t - 1u - lane;
      const uint64_t iw = valid ? sld(incw + u) : 0ull;
      const bool inc = valid && (uint32_t)(iw >> 56) == epoch;
      const uint64_t aw = valid && !inc ? sld(aggw + u) : 0ull;
      const bool agg = valid && !inc && (uint32_t)(aw >> 56) == epoch;
      const uint64_t bi = __ballot(inc);
      const uint32_t F = bi ? (uint32_t)__builtin_ctzll(bi) : WAVE;  // the nearest inclusive count
      const uint64_t below = F >= WAVE ? ~0ull : ((1ull << F) - 1ull);
      if (F < WAVE && (__ballot(agg) & below) == below) {
        const uint32_t ex = inc ? (uint32_t)iw : (uint32_t)aw;
        const bool stp = inc ? ex == 0xFFFFFFFFu : ((aw >> 34) & 1ull) != 0;
        const uint32_t cnt = inc ? (uint32_t)(iw >> 32) & 0xFFFFFFu : (uint32_t)(aw >> 46) & 0x3FFu;
        const uint32_t ent = (s - 1u - lane) * BW_WIN + ((uint32_t)(aw >> 35) & 0x7FFu);
        // the earliest stopped tile from F on (highest lane): the tiles after it hold no values
        const uint64_t bs = __ballot(stp && lane <= F);
        const uint32_t S = bs ? 63u - (uint32_t)__builtin_clzll(bs) : WAVE;
        const uint32_t lo = S < WAVE ? S : 0u;
        const uint32_t nex = (uint32_t)__shfl_down((int)ex, 1);  // exit of the tile before this lane's
        const bool link = lane < lo || lane >= F || ent == nex;
        if (__ballot(!link) == 0ull) {
          const uint32_t c = lane >= lo && lane <= F ? cnt : 0u;
          uint32_t sum = c;
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o);
          before = uni(sum);
          if (S < WAVE) {
            stopped = true;
          } else {
            const uint32_t ex0 = uni(rdl(ex, 0));  // where the chain enters this tile
#ifdef PQG_DIAG
            dg_guess = ex0 == entry ? 1u : 0u;
#endif
            if (ex0 != entry) {                    // misspeculated (or no guess): walk from there
              entry = ex0;
              r = ex0 >= B + BW_WIN ? BpWalk{ex0, 0, 0} : bp_walk<true>(L, cur, rs, B, ex0, end);
            }
          }
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
      // bounded (s_memrealtime: 100 MHz): a tile that never publishes sends the plan to the per-value
      // path (pqg_sync re-runs it), not a hang
      if (__builtin_amdgcn_s_memrealtime() - t_wait > 200000000ull) {
        if (lane == 0) {
          sst(inexact, flag_epoch);
          sst(incw + t, E | BP_NONE);
        }
        return;
      }
    }
  }
  const uint32_t n = stopped ? 0u : r.n;
  const uint32_t incl = before + n < 0xFFFFFFu ? before + n : 0xFFFFFFu;
#ifdef PQG_DIAG
  dg2 = __builtin_amdgcn_s_memrealtime() + (n > 0xFFFFFFF0u ? 1u : 0u);
  struct DgBp {
    uint64_t a, *b, *c, *d, *e;
    uint32_t t;
    __device__ ~DgBp() {
      if (pqg_diag_bp && lane_id() == 0) {
        uint64_t* o = pqg_diag_bp + 8 * (uint64_t)t;
        o[0] = a; o[1] = *b; o[2] = *c; o[3] = __builtin_amdgcn_s_memrealtime(); o[4] = *d; o[5] = *e;
      }
    }
  } dg_out{dg0, &dg1, &dg2, &dg_polls, &dg_guess, t};
#endif
  if (lane == 0) sst(incw + t, E | ((uint64_t)incl << 32) | (stopped || r.code ? BP_NONE : (uint64_t)r.pos));
  if (stopped || before >= N) return;
  if (r.code && before + r.n < N && lane == 0) report(err, err_count, page, 2, before + r.n, r.code);
  if (before + r.n >= N) {  // the page's last value is here: it must end at the section end
    const uint32_t q = N - 1u - before;
    const uint32_t e_last = q + 1u < r.n ? B + L.acc[q + 1u] : r.pos;
    if ((q + 1u < r.n || e_last != end) && lane == 0) sst(inexact, flag_epoch);
  }
  const uint32_t m = r.n < N - before ? r.n : N - before;
  if (m == 0) return;
  wave_sync();  // the walk's candidate list is dead: stage the tile and the start of the next one
  {
    uint32_t* img = L.u.img;
    *(u32x4*)&img[8u * lane] = cur.a;
    *(u32x4*)&img[8u * lane + 4u] = cur.b;
    img[BW_WIN / 4u + lane] = nxt;
  }
  wave_sync();
  if (!bp_emit_fast((uint32_t*)L.bt, L.u.img, BP_IMG, L.acc, B, beg, r.n, r.pos, before, m, pw, cd))
    bp_emit(L.u.img, BP_IMG, L.acc, L.bt, rs, B, beg, r.n, r.pos, before, m, pw, cd);
}

// One-pass PLAIN BYTE_ARRAY for plans with many PLAIN pages (k_bin_plain_pg): one wave per page
// follows its chain tile after tile from the section start (bp_walk from a known position: no guess,
// no look-back, the values before a tile are the wave's running count) and emits every tile's offsets
// and value bytes from the tile and the next one staged in LDS (bp_emit). The next tile's bytes are
// in registers before the current tile's stores, the one after it is requested before them. With
// thousands of pages one wave per page fills the chip; the tile kernel (k_bin_plain) spreads few pages
// over many waves. Same semantics as k_bin_plain: errors at the per-value path's index, a page whose
// values do not end at its section end raises the inexact flag (pqg_sync re-runs the plan per value).
struct BinPageLds {
  union {
    BinWalkLds w;                         // the tile walk (candidate list)
    uint32_t img[2u * BW_WIN / 4u + 16];  // then: page bytes [B, B + 2 BW_WIN) (+ slack for the compose reads)
  } u;
  uint16_t acc[BW_CAP + 2];  // accepted value starts of the tile (offsets from B), ascending
  uint16_t bt[BP_BLK + 2];   // output block -> the last value starting at or before its first byte
};
static_assert(sizeof(BinPageLds) * WPB <= 160 * 1024 / 6, "6 workgroups of k_bin_plain_pg per CU");

// 5 waves per SIMD: 94 VGPRs hold the tile being walked and the next one without spills (at 6, the
// next tile's registers went to scratch, whose store waited for the prefetch on every tile)
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(5))) void k_bin_plain_pg(
    const uint8_t* __restrict__ bytes, uint64_t n_bytes, const PageWork* __restrict__ work,
    const ColumnDev* __restrict__ cols, const int32_t* __restrict__ list, int n_list, uint32_t* inexact,
    uint32_t flag_epoch, uint64_t* err, ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) BinPageLds lds_all[WPB];
  const int page = wave_page(list, n_list);
  if (page < 0) return;
  BinPageLds& L = lds_all[wave_id()];
  const uint32_t lane = lane_id();
  const PageWork& pw = work[page];
  const ColumnDev& cd = cols[pw.column];
  const uint32_t beg = uni(pw.data_begin), end = uni(pw.size), N = uni(pw.n_values);
  if (N == 0 || beg >= end) {
    if (lane == 0) {
      if (N > 0) report(err, err_count, page, 2, 0, PQG_ERR_EOF);  // no section: value 0
      else if (beg < end) sst(inexact, flag_epoch);                // bytes but no values: base() assumes none
    }
    return;
  }
  const rsrc_t rs = make_rsrc(bytes + pw.base, n_bytes - pw.base);
  uint32_t pos = beg, before = 0;
  uint32_t B = beg & ~(BW_WIN - 1u);
  // Two tile buffers in ping-pong (the loop body is written for (cur, nxt) = (X, Y), then (Y, X)): a
  // "cur = nxt" copy made the compiler wait for the freshly issued load of the next tile at once
  // (its registers were moved into place), a full memory latency per tile.
  BwBytes X = bw_load(rs, B), Y = bw_load(rs, B + BW_WIN);
  // one tile; returns true when the page is done
  auto tile = [&](BwBytes& cur, BwBytes& nxt) __attribute__((always_inline)) -> bool {
    pos = uni(pos);
    before = uni(before);
    B = uni(B);
    const BpWalk r = bp_walk<true>(L, cur, rs, B, pos, end);
    if (r.code && before + r.n < N && lane == 0) report(err, err_count, page, 2, before + r.n, r.code);
    bool last = r.code != 0;
    if (before + r.n >= N) {  // the page's last value is here: it must end at the section end
      const uint32_t q = N - 1u - before;
      const uint32_t e_last = q + 1u < r.n ? B + L.acc[q + 1u] : r.pos;
      if ((q + 1u < r.n || e_last != end) && lane == 0) sst(inexact, flag_epoch);
      last = true;
    }
    const uint32_t m = r.n < N - before ? r.n : N - before;
    wave_sync();  // the walk's candidate list is dead: stage this tile and the next one
    *(u32x4*)&L.u.img[8u * lane] = cur.a;
    *(u32x4*)&L.u.img[8u * lane + 4u] = cur.b;
    *(u32x4*)&L.u.img[BW_WIN / 4u + 8u * lane] = nxt.a;
    *(u32x4*)&L.u.img[BW_WIN / 4u + 8u * lane + 4u] = nxt.b;
    // the tile holding the next value (r.pos >= B + BW_WIN: the walk left this tile) and the one after
    // it, requested before this tile's stores
    const uint32_t nB = r.pos & ~(BW_WIN - 1u);
    if (!last) {
      if (nB == B + BW_WIN) {  // the next call walks nxt; this buffer takes the tile after it
        cur = bw_load(rs, nB + BW_WIN);
      } else {  // a value longer than a tile: both again (next call: nxt = tile nB, cur = the one after)
        nxt = bw_load(rs, nB);
        cur = bw_load(rs, nB + BW_WIN);
      }
    }
    wave_sync();
    if (m)
      if (!bp_emit_fast((uint32_t*)L.bt, L.u.img, 2u * BW_WIN, L.acc, B, beg, r.n, r.pos, before, m, pw, cd))
        bp_emit(L.u.img, 2u * BW_WIN, L.acc, L.bt, rs, B, beg, r.n, r.pos, before, m, pw, cd);
    if (last) return true;
    before += r.n;
    pos = r.pos;
    B = nB;
    wave_sync();  // the emit's LDS reads are done before the next walk's list
    return false;
  };
  while (!tile(X, Y) && !tile(Y, X)) {
  }
}

// base(page) of every page of the PLAIN-only BYTE_ARRAY columns (one workgroup per column, pages in
// column order): the value bytes of the column's earlier pages, each page taken as filling its data
// section (size - data_begin - 4 n_values; k_bin_plain checks it); the column total -> bin_total
// (compared with binary_capacity at sync).
__global__ __launch_bounds__(256) void k_bin_bases(PageWork* __restrict__ work, const ColumnDev* __restrict__ cols,
                                                   const int32_t* __restrict__ col_pages,
                                                   const int32_t* __restrict__ col_start) {
  // thread t takes BB_PER consecutive pages per round: all their loads issued before any use (two
  // dependent round trips per round: the page list, then the pages' facts), a register scan, one
  // workgroup scan of the threads' totals. (The previous 256-page rounds paid both round trips and
  // three barriers per 256 pages: C3's two columns of 5,000 pages took 290-640 us on the strings'
  // queue, ahead of k_bin_plain_pg.)
  constexpr int BB_PER = 16;
  const int b = col_start[blockIdx.x], e = col_start[blockIdx.x + 1];
  __shared__ uint64_t wsum[4];
  uint64_t carry = 0;
  for (int r0 = b; r0 < e; r0 += 256 * BB_PER) {
    const int i0 = r0 + (int)threadIdx.x * BB_PER;
    int pg[BB_PER];
#pragma unroll
    for (int q = 0; q < BB_PER; q++) pg[q] = i0 + q < e ? col_pages[i0 + q] : -1;
    uint64_t v[BB_PER], own = 0;
#pragma unroll
    for (int q = 0; q < BB_PER; q++) {
      v[q] = 0;
      if (pg[q] >= 0) {
        const PageWork& w = work[pg[q]];
        const uint64_t need = (uint64_t)w.data_begin + 4ull * w.n_values;
        v[q] = w.size > need ? w.size - need : 0;
      }
      own += v[q];
    }
    uint64_t x = own;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o);
      if ((int)lane_id() >= o) x += y;
    }
    if (lane_id() == 63) wsum[threadIdx.x >> 6] = x;
    __syncthreads();
    uint64_t pre = carry + x - own, tot = 0;
    for (int w = 0; w < 4; w++) {
      pre += w < (int)(threadIdx.x >> 6) ? wsum[w] : 0;
      tot += wsum[w];
    }
#pragma unroll
    for (int q = 0; q < BB_PER; q++) {
      if (pg[q] >= 0) gst(&work[pg[q]].bin_base, pre);
      pre += v[q];
    }
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && e > b) {
    const ColumnDev& cd = cols[work[col_pages[b]].column];
    gst(cd.bin_total, carry);
    gst((int64_t*)cd.values, (int64_t)0);  // offsets[0] (also when the column has no values)
  }
}

// ---------------------------------------------------------------------------
// Launchers

#define PQG_BIN_ARGS bytes, n_bytes, work, cols, list, n, err, err_count

hipError_t launch_bss(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work, const ColumnDev* cols,
                      const int32_t* list, int n, uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bss, dim3(n), dim3(64 * WPB), 0, st, PQG_BIN_ARGS);  // a workgroup per page
  return hipGetLastError();
}

// ---- BYTE_ARRAY dictionary pages of DENT_MIN bytes or more (PlainBinaryDictionary ctor,
// PlainValuesDictionary.java:58-134: dict_n entries of [u32 length][bytes] read one after the other),
// walked in parallel. The one-wave walk (k_bin_walk, dict_walk = 1) follows a 360 KB page of 16,384
// entries tile after tile in ~550 us (profiles/r06); here every 2 KiB tile is walked at once from a
// guessed first entry, as the one-pass PLAIN tiles do, but without inter-workgroup waits:
//   k_dent_walk     one wave per tile: bp_guess (tile 0: the page start), the tile's chain (bp_walk), its
//                   accepted starts (u16 tile offsets) to the tile's scratch, the record {guess, exit, count,
//                   code}
//   k_dent_resolve  one wave per dictionary: the true entry of tile t is the exit of tile t - 1; a tile
//                   whose guess is not that entry (rare) is walked again from it by this wave (64 tiles at a
//                   time by a count scan while every guess holds: 44 -> 6 us for 16,384 entries); tile t's first
//                   entry index = the counts before it (capped at dict_n); the chain's first error before
//                   dict_n entries is the dictionary's error (bin_value_error's dictionary codes, as the
//                   one-wave walk reports them)
//   k_dent_scatter  one wave per tile: its entries' lengths and sources to dict_len / dict_src
__global__ __launch_bounds__(64 * WPB) void k_dent_walk(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                       const ColumnDev* __restrict__ cols, const uint64_t* __restrict__ tiles,
                                                       uint32_t n_tiles, uint64_t* rec, uint16_t* scr) {
  __shared__ __attribute__((aligned(16))) BinPlainLds lds_all[WPB];
  const uint32_t t = blockIdx.x * WPB + wave_id();
  if (t >= n_tiles) return;
  const uint32_t lane = lane_id();
  BinPlainLds& L = lds_all[wave_id()];
  const uint64_t tv = tiles[t];
  const ColumnDev& cd = cols[(uint32_t)tv];
  const uint32_t s = (uint32_t)(tv >> 32), B = s * BW_WIN, end = uni((uint32_t)cd.dict_bytes);
  const rsrc_t rs = make_rsrc(bytes + cd.dict_offset, n_bytes - cd.dict_offset);
  const BwBytes cur = bw_load(rs, B);
  const BpGuess gs = s == 0 ? BpGuess{0u, 0xFFFFFFFFu, 0, 0, false} : bp_guess(L, cur, rs, B, end);
  BpWalk r{gs.pos, 0, 0};
  if (gs.pos != 0xFFFFFFFFu)
    r = s == 0 ? bp_walk<true>(L, cur, rs, B, 0u, end)
               : bp_walk<true>(L, cur, rs, B, gs.pos, end, gs.index, gs.total, gs.eff_end, gs.fast);
  for (uint32_t k = lane; k < r.n; k += WAVE) gst(scr + (uint64_t)t * BW_CAP + k, L.acc[k]);
  if (lane == 0) {
    gst(rec + 2u * t, (uint64_t)gs.pos | ((uint64_t)r.pos << 32));
    gst(rec + 2u * t + 1u, (uint64_t)r.n | ((uint64_t)(uint32_t)r.code << 32));
  }
}

__global__ __launch_bounds__(64) void k_dent_resolve(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                    const ColumnDev* __restrict__ cols, const int32_t* __restrict__ dcols,
                                                    const int32_t* __restrict__ dstart, const uint64_t* rec, uint16_t* scr,
                                                    uint64_t* tb, int n_pages, uint64_t* err, ErrCount err_count) {
  __shared__ __attribute__((aligned(16))) BinPlainLds L;
  const uint32_t lane = lane_id();
  const int col = dcols[blockIdx.x];
  const ColumnDev& cd = cols[col];
  const uint32_t t0 = (uint32_t)dstart[blockIdx.x], t1 = (uint32_t)dstart[blockIdx.x + 1];
  const uint32_t N = uni(cd.dict_n), end = uni((uint32_t)cd.dict_bytes);
  const rsrc_t rs = make_rsrc(bytes + cd.dict_offset, n_bytes - cd.dict_offset);
  uint32_t entry = 0, before = 0, t = t0;
  int code = 0;
  bool done = N == 0;
  uint64_t r0 = 0, r1 = 0;  // lane l: the records of tile (t - t0) rounded down to 64, + l
  for (; t < t1 && !done; t++) {
    const uint32_t s = t - t0, j = s & (WAVE - 1u);
    if (j == 0) {  // the next 64 records, one per lane
      const bool in = t + lane < t1;
      r0 = in ? sld(rec + 2u * (t + lane)) : 0ull;
      r1 = in ? sld(rec + 2u * (t + lane) + 1u) : 0ull;
      // the whole batch at once when every tile still needed was walked from its true entry (its guess is
      // the previous tile's exit) and ends without an error: first entries by a scan of the counts
      const uint32_t n_in = t1 - t < WAVE ? t1 - t : WAVE;
      const uint32_t g = (uint32_t)r0, x = (uint32_t)(r0 >> 32), c = in ? (uint32_t)r1 : 0u;
      const uint32_t cc = (uint32_t)(r1 >> 32);
      uint32_t px = __shfl_up(x, 1);
      if (lane == 0) px = entry;
      uint32_t inc = c;
      for (int o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if ((int)lane >= o) inc += y;
      }
      const uint32_t bef = before + (inc - c);  // (counts <= BW_CAP per tile: no overflow)
      const bool live = in && bef < N;
      const bool ok = !live || ((t + lane == t0 || g == px) && (cc == 0u || bef + c >= N));
      if (__ballot(!ok) == 0ull) {
        if (in) {
          const uint32_t b2 = bef < N ? bef : N, take = live ? (c < N - bef ? c : N - bef) : 0u;
          gst(tb + t + lane, (uint64_t)b2 | ((uint64_t)take << 32));
        }
        const uint32_t after = uni(before + rdl(inc, n_in - 1u));
        before = after < N ? after : N;
        entry = uni(rdl(x, n_in - 1u));
        done = before >= N;
        t += n_in - 1u;
        continue;
      }
    }
    const uint32_t B = s * BW_WIN;
    if (entry >= B + BW_WIN) {  // a value spans the whole tile: no entry starts in it
      if (lane == 0) gst(tb + t, (uint64_t)before);
      continue;
    }
    const uint32_t guess = uni(rdl((uint32_t)r0, j));
    uint32_t ex = uni(rdl((uint32_t)(r0 >> 32), j)), cnt = uni(rdl((uint32_t)r1, j));
    uint32_t cd_code = uni(rdl((uint32_t)(r1 >> 32), j));
    if (s != 0 && guess != entry) {  // misspeculated (or no guess): this wave walks the tile from its true entry
      const BwBytes cur = bw_load(rs, B);
      const BpWalk rr = bp_walk<true>(L, cur, rs, B, entry, end);
      for (uint32_t k = lane; k < rr.n; k += WAVE) gst(scr + (uint64_t)t * BW_CAP + k, L.acc[k]);
      ex = rr.pos;
      cnt = rr.n;
      cd_code = (uint32_t)rr.code;
      wave_sync();
    }
    const uint32_t take = cnt < N - before ? cnt : N - before;
    if (lane == 0) gst(tb + t, (uint64_t)before | ((uint64_t)take << 32));
    before += take;
    if (before >= N) {
      done = true;
    } else if (cd_code) {  // the chain stopped (an error, or the section end) before dict_n entries
      code = bin_value_error(rs, ex, end, true);
      done = true;
    } else {
      entry = ex;
    }
  }
  if (!done) code = bin_value_error(rs, entry, end, true);  // past the last tile before dict_n entries
  for (uint32_t u = t + lane; u < t1; u += WAVE) gst(tb + u, (uint64_t)before);  // tiles past the end: none
  if (code && lane == 0) report(err, err_count, n_pages + col, 0, before, code);
}

__global__ __launch_bounds__(64 * WPB) void k_dent_scatter(const uint8_t* __restrict__ bytes, uint64_t n_bytes,
                                                          const ColumnDev* __restrict__ cols,
                                                          const uint64_t* __restrict__ tiles, uint32_t n_tiles,
                                                          const uint16_t* __restrict__ scr, const uint64_t* __restrict__ tb) {
  const uint32_t t = blockIdx.x * WPB + wave_id();
  if (t >= n_tiles) return;
  const uint64_t tv = tiles[t];
  const ColumnDev& cd = cols[(uint32_t)tv];
  const uint32_t B = (uint32_t)(tv >> 32) * BW_WIN;
  const uint64_t v = tb[t];
  const uint32_t base = (uint32_t)v, cnt = (uint32_t)(v >> 32);
  const rsrc_t rs = make_rsrc(bytes + cd.dict_offset, n_bytes - cd.dict_offset);
  for (uint32_t k = lane_id(); k < cnt; k += WAVE) {
    const uint32_t p = B + scr[(uint64_t)t * BW_CAP + k];
    const uint32_t len = ld4_any(rs, p);
    gst(cd.dict_len + base + k, len);
    gst(cd.dict_src + base + k, p + 4u);
    if (cd.dict_ent) gst(cd.dict_ent + base + k, ((uint64_t)(p + 4u) << 32) | len);
  }
}

hipError_t launch_dict_entries(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, const ColumnDev* cols,
                               const uint64_t* tiles, uint32_t n_tiles, const int32_t* dcols, const int32_t* dstart,
                               int n_dcols, uint64_t* rec, uint16_t* scr, uint64_t* tb, int n_pages, uint64_t* err,
                               ErrCount err_count) {
  if (!n_tiles || n_dcols <= 0) return hipSuccess;
  const dim3 grid((n_tiles + WPB - 1) / WPB), blk(64 * WPB);
  hipLaunchKernelGGL(k_dent_walk, grid, blk, 0, st, bytes, n_bytes, cols, tiles, n_tiles, rec, scr);
  hipLaunchKernelGGL(k_dent_resolve, dim3(n_dcols), dim3(64), 0, st, bytes, n_bytes, cols, dcols, dstart, rec, scr, tb,
                     n_pages, err, err_count);
  hipLaunchKernelGGL(k_dent_scatter, grid, blk, 0, st, bytes, n_bytes, cols, tiles, n_tiles, scr, tb);
  return hipGetLastError();
}

hipError_t launch_bin_walk(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const int32_t* list, int n, int dict_walk, int n_pages,
                           uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bin_walk, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols, list, n,
                     dict_walk, n_pages, err, err_count);
  return hipGetLastError();
}

hipError_t launch_bin_walk_seg(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                               const ColumnDev* cols, const uint64_t* segs, uint32_t n_segs, uint64_t* status,
                               uint32_t* ticket, uint32_t* tmp, uint64_t* err, ErrCount err_count) {
  if (n_segs == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bin_walk_seg, dim3((n_segs + WPB - 1) / WPB), dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols,
                     segs, n_segs, status, ticket, tmp, err, err_count);
  return hipGetLastError();
}

hipError_t launch_bin_plain(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work, const ColumnDev* cols,
                            const int32_t* col_pages, const int32_t* col_start, int n_cols, const uint64_t* segs,
                            uint32_t n_segs, uint64_t* aggw, uint64_t* incw, uint32_t* ticket, uint32_t epoch,
                            uint32_t* inexact, uint32_t flag_epoch, uint64_t* err, ErrCount err_count,
                            bool per_page, int n_pages_total) {
  if (n_cols <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bin_bases, dim3(n_cols), dim3(256), 0, st, work, cols, col_pages, col_start);
  if (per_page) {  // one wave per page of col_pages
    const int n = n_pages_total;
    if (n > 0)
      hipLaunchKernelGGL(k_bin_plain_pg, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols,
                         col_pages, n, inexact, flag_epoch, err, err_count);
  } else if (n_segs) {
    hipLaunchKernelGGL(k_bin_plain, dim3((n_segs + WPB - 1) / WPB), dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols,
                       segs, n_segs, aggw, incw, ticket, epoch, inexact, flag_epoch, err, err_count);
  }
  return hipGetLastError();
}

hipError_t launch_bin_dict_map(hipStream_t st, PageWork* work, const ColumnDev* cols, const int32_t* list, int n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bin_dict_map, dim3(n, DM_SLICES), dim3(64 * WPB), 0, st, work, cols, list, n);
  return hipGetLastError();
}

hipError_t launch_gather_fixed(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                               const ColumnDev* cols, const int32_t* list, int n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_fixed, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols,
                     list, n);
  return hipGetLastError();
}

hipError_t launch_bin_scan(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, const ColumnDev* cols,
                           const int32_t* bin_cols, int n_bin_cols, const uint64_t* blocks, uint32_t n_blocks) {
  if (n_bin_cols <= 0 || n_blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bin_block_sums, dim3(n_blocks), dim3(256), 0, st, cols, blocks);
  hipLaunchKernelGGL(k_bin_block_bases, dim3(n_bin_cols), dim3(256), 0, st, cols, bin_cols);
  hipLaunchKernelGGL(k_bin_offsets, dim3(n_blocks), dim3(256), 0, st, bytes, n_bytes, cols, blocks);
  return hipGetLastError();
}

hipError_t launch_dba_copy(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const int32_t* list, int n, const uint64_t* chunks,
                           uint32_t n_chunks, const uint32_t* dba_meta, const int32_t* carry_cols, int n_carry_cols,
                           uint64_t* err, ErrCount err_count) {
  if (n <= 0) return hipSuccess;
  if (n_chunks) {
    const dim3 gc((n_chunks + WPB - 1) / WPB);
    hipLaunchKernelGGL(k_dba_tail, gc, dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols, chunks, n_chunks, dba_meta);
    hipLaunchKernelGGL(k_dba_chain_par, gc, dim3(64 * WPB), 0, st, work, cols, chunks, n_chunks, dba_meta);
    hipLaunchKernelGGL(k_dba_chain, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, work, cols, list, n, dba_meta);
    hipLaunchKernelGGL(k_dba_chunks, gc, dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols, chunks, n_chunks, dba_meta);
  }
  hipLaunchKernelGGL(k_dba_copy, dim3((n + WPB - 1) / WPB), dim3(64 * WPB), 0, st, bytes, n_bytes, work, cols, list, n);
  if (n_carry_cols > 0)
    hipLaunchKernelGGL(k_dba_carry, dim3(n_carry_cols), dim3(64), 0, st, bytes, n_bytes, work, cols, list, n, carry_cols,
                       err, err_count);
  return hipGetLastError();
}

hipError_t launch_bin_copy(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const uint64_t* chunks, uint32_t n_chunks, uint64_t* err,
                           ErrCount err_count) {
  if (n_chunks == 0) return hipSuccess;
  // one resident round of workgroups (by LDS: 5 per CU at ~31 KiB each; by VGPRs at most 7) striding
  // over the chunks: a dictionary page stays staged across a workgroup's chunks of the same column
  constexpr uint32_t CP_VGPR_WG = 5u;  // 95 VGPRs: 5 waves per SIMD
  constexpr uint32_t CP_PER_CU = (160u * 1024u) / (uint32_t)sizeof(CopyLds) < CP_VGPR_WG ? (160u * 1024u) / (uint32_t)sizeof(CopyLds) : CP_VGPR_WG;
  constexpr uint32_t CP_GRID = 256u * CP_PER_CU;
  hipLaunchKernelGGL(k_bin_copy, dim3(n_chunks < CP_GRID ? n_chunks : CP_GRID), dim3(64 * WPB), 0, st, bytes, n_bytes,
                     work, cols, chunks, n_chunks, err, err_count);
  return hipGetLastError();
}

}  // namespace pqg

#ifdef PQG_DIAG
// Diagnostic build only (tools/diag_binplain.py): per k_bin_plain tile, 8 u64 (see pqg_diag_bp).
extern "C" int pqg_diag_bp_set(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg::pqg_diag_bp), &p, sizeof(p)) == hipSuccess ? 0 : 3;
}
#endif
