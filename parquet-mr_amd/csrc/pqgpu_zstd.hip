// pqgpu_zstd.hip — ZSTD page decompression on gfx950 (pqg_zstd_decompress).
//
// parquet-mr decompresses a ZSTD page through zstd-jni's streaming decoder (ZstandardCodec ->
// ZstdDecompressorStream, parquet-hadoop/src/main/java/org/apache/parquet/hadoop/codec/
// ZstdDecompressorStream.java:31-46; libzstd underneath) and keeps exactly the header's
// uncompressed size (ColumnChunkPageReadStore.java:144-172). The format is RFC 8878; the CPU
// restatement every test checks against is oracle/zstd_ref.c.
//
// One 64-lane wave per job (page). Decoding a ZSTD block has two serial parts and one parallel:
//   * literals: Huffman streams decoded by lanes 0..3 (one stream each, 4-stream blocks) or lane 0,
//     with the decoding table in LDS, into a per-job literal buffer in global scratch;
//   * sequences: the three FSE state machines and the backward bitstream, wave-uniform code (the
//     scalar unit does the bookkeeping), the bitstream read through a 1 KiB LDS window;
//   * execution: each sequence's literal copy and match copy by all 64 lanes, the last 4 KiB of
//     output mirrored in an LDS ring so that overlapping / near matches read LDS; older bytes
//     are read back from the output with system-scope (L1-bypassing) loads after a store drain
//     every 2 KiB of output.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

constexpr uint32_t ZS_RING = 4096;  // LDS mirror of the most recent output
constexpr uint32_t ZS_WIN = 1024;     // LDS window of the sequence bitstream
constexpr uint32_t ZS_HWIN = 256;     // LDS window per Huffman stream
constexpr uint32_t ZS_LIT_MAX = 131072;
constexpr uint32_t ZS_SB = 64;        // sequences per execution batch (lane k: sequence k)
constexpr uint32_t ZS_CAP = 512;      // output bytes per execution batch
constexpr uint32_t ZS_LIT = 0x80000000u;  // byte source tag: a literal of the batch (| its index)
constexpr uint32_t ZS_FLUSH = 1024;   // ring bytes written to HBM once this many are pending

// Sequence-section decoder state of the current block, kept in LDS between batches: the decode loop
// (zseq_decode) is a function of its own, so its state lives in SGPRs without the register pressure
// of the whole job's code around it (inlined, the loop's state was spilled to VGPR lanes and every
// uniform test went through the vector unit: ~2,200 cycles per sequence).
struct ZSeq {
  uint64_t src, src_len;          // the job's input (the function builds its own buffer resource)
  uint64_t c;                     // bit container (BackBits)
  int32_t bits, cbit;
  uint32_t wlo, base, n;
  uint32_t sl, so, sm;            // FSE states
  uint32_t rep0, rep1, rep2;      // repeat offsets
  uint32_t i, nseq;               // sequences decoded / in the block
  uint32_t outp, lits, regen, frame0;  // output position and literals after the decoded sequences
  uint32_t m, T, blit, pend;      // result of a call: batch size, bytes, literals; 1: a sequence is
                                  // carried to the next batch, 2: it is longer than a batch
};

// The literal / table-description phase of a block and its sequence execution never overlap, so
// their scratch shares LDS (18.2 KiB per wave instead of 20.8: 8 waves per CU instead of 7).
struct ZLitLds {
  uint32_t hw[64];                     // FSE table of compressed Huffman weights (accuracy <= 6)
  uint8_t hwin[4][ZS_HWIN + 16];
  int16_t norm[256];
  uint8_t wts[256];
  uint16_t nxt[256];
};
struct ZExecLds {
  uint32_t src[ZS_CAP];                // batch output byte -> literal index (| ZS_LIT) or output position
  uint8_t lseg[ZS_CAP + 16];           // the batch's literal bytes
};
struct ZWaveLds {
  uint32_t ll[512], ml[512], of[256];  // FSE decoding entries: sym | nb << 8 | base << 16
  uint16_t huf[2048];                  // Huffman decoding entries: sym | nb << 8 (kept for treeless blocks)
  uint8_t ring[ZS_RING];
  uint8_t win[ZS_WIN + 16];
  union {
    ZLitLds t;
    ZExecLds x;
  } ph;
  uint32_t flag;
  uint32_t sq_ll[ZS_SB + 1], sq_ml[ZS_SB + 1], sq_of[ZS_SB + 1];  // decoded sequences of one batch (+ the carried one)
  uint32_t llcode[36], mlcode[53];     // literal / match length codes: baseline | extra bits << 24
  ZSeq ss;
#ifdef PQG_DIAG
  uint64_t diag[12];                  // diagnostic build: cycles per phase of the current job
#endif
};

#ifdef PQG_DIAG
// Diagnostic build only (tools/diag_zstd.py): per job 8 u64 = cycles in literals (Huffman), sequence
// tables, sequence decode, batch execution, long sequences, whole job; sequences; literal bytes.
static __device__ uint64_t* pqg_zdiag;
extern "C" int pqg_diag_zstd_set(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg_zdiag), &p, sizeof(p)) == hipSuccess ? 0 : 3;
}
#define ZD_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ZD_ADD(L, i, t0) ((L).diag[i] += __builtin_amdgcn_s_memtime() - (t0))
#define ZD_CNT(L, i, n) ((L).diag[i] += (n))
#define ZQ(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define ZQ_ADD(acc, a, b) (acc) += (b) - (a)
#else
#define ZQ(v)
#define ZQ_ADD(acc, a, b)
#define ZD_T(v)
#define ZD_ADD(L, i, t0)
#define ZD_CNT(L, i, n)
#endif

__constant__ int16_t ZLL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t ZML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t ZOF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t ZLL_BASE[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32, 40,
                                      48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t ZLL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t ZML_BASE[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29,
                                      30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099,
                                      8195, 16387, 32771, 65539};
__constant__ uint8_t ZML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                     0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

__device__ __forceinline__ int zhigh(uint32_t v) { return v ? 31 - __builtin_clz(v) : -1; }

// Reads of bytes this wave stored earlier (literal buffer, output), after the s_waitcnt that
// completed the stores: system-scope loads (L1 and L2 bypassed). A workgroup-scope load
// measured the same (71.7 ms on 100 M int64 PLAIN pages, profiles/r02/zstd_ab):
// the kernel is not bound by these round trips.
__device__ __forceinline__ uint32_t zld(const uint32_t* p) {
  return sld(p);
}

// one input byte at `o` of the job's input (uniform reads: every lane loads the same dword)
__device__ __forceinline__ uint32_t zbyte(rsrc_t rs, uint32_t o) { return (ld32(rs, o & ~3u) >> ((o & 3u) * 8u)) & 0xFFu; }

// Forward little-endian bit reader over the input (FSE table descriptions), uniform.
struct FwdBits {
  rsrc_t rs;
  uint32_t lim;     // input bytes readable (the description's end)
  uint64_t bitpos;  // absolute bit position
  bool bad;
  __device__ uint32_t get(int k) {
    uint32_t v = 0;
    const uint64_t b0 = bitpos;
    if (((b0 + (uint64_t)k + 7) >> 3) > lim) { bad = true; bitpos += (uint64_t)k; return 0; }
    const uint32_t byte = (uint32_t)(b0 >> 3);
    const uint64_t w = ld8_any(rs, byte);
    v = (uint32_t)((w >> (b0 & 7)) & ((1ull << k) - 1ull));
    bitpos += (uint64_t)k;
    return v;
  }
};

// Backward bitstream (RFC 8878 §4.1) whose bytes [0, n) start at input offset `base` (wave-uniform).
// Reads come from a 64-bit register container holding stream bits [cbit, cbit + 64), refilled with 8
// bytes from an LDS window of the stream (the whole wave refills the window): most reads are a
// shift and a mask, where reading every field from LDS put an LDS round trip on the sequence
// decoder's serial chain per field (6 per sequence).
struct BackBits {
  rsrc_t rs;
  uint32_t base, n;
  int32_t bits;      // unread bits
  uint32_t wlo;      // window covers stream bytes [wlo, wlo + ZS_WIN)
  uint8_t* win;
  uint64_t c;        // container: stream bits [cbit, cbit + 64)
  int32_t cbit;
  __device__ bool init(rsrc_t r, uint32_t b, uint32_t len, uint8_t* w) {
    rs = r; base = b; n = len; win = w; wlo = 0xFFFFFFFFu;
    cbit = INT32_MAX;
    c = 0;
    if (len == 0) return false;
    const uint32_t last = zbyte(rs, base + len - 1);
    if (!last) return false;
    bits = (int32_t)(len - 1) * 8 + zhigh(last);
    return true;
  }
  __device__ void refill(uint32_t need_end) {  // window ending at stream byte need_end
    const uint32_t lo = need_end > ZS_WIN ? need_end - ZS_WIN : 0;
    wlo = lo;
    const uint32_t o = 16u * lane_id();
    *(u32x4*)(win + o) = u32x4{ld4_any(rs, base + lo + o), ld4_any(rs, base + lo + o + 4),
                               ld4_any(rs, base + lo + o + 8), ld4_any(rs, base + lo + o + 12)};
    wave_sync();
  }
  // container for reads ending at bit `end` (exclusive): bits [ceil8(end) - 64, ceil8(end)), from 0
  __device__ void fill(int32_t end) {
    const int32_t e8 = (end + 7) & ~7;
    cbit = e8 > 64 ? e8 - 64 : 0;
    const uint32_t b0 = (uint32_t)cbit >> 3, b1 = b0 + 8u < n ? b0 + 8u : n;  // bytes [b0, b1)
    if (wlo == 0xFFFFFFFFu || b0 < wlo || b1 > wlo + ZS_WIN) refill(b1 + 8u < n ? b1 + 8u : n);
    typedef uint32_t __attribute__((may_alias)) u32a;
    const uint32_t rel = b0 - wlo, r4 = rel & ~3u, sft = rel & 3u;
    const uint32_t d0 = *(const u32a*)(win + r4), d1 = *(const u32a*)(win + r4 + 4), d2 = *(const u32a*)(win + r4 + 8);
    uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sft) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sft) << 32);
    const uint32_t nb = b1 - b0;  // bytes past the stream's end read as 0
    if (nb < 8u) v &= (1ull << (8u * nb)) - 1ull;
    c = uni64(v);
  }
  // k <= 32 bits; bits below the stream start read as 0 (overflow: bits < 0 afterwards)
  __device__ uint32_t read(int k) {
    if (k == 0) return 0;
    bits -= k;
    int32_t a = bits;
    int sh = 0;
    if (a < 0) { sh = -a; a = 0; }
    const int kk = k - sh;
    if (kk <= 0) return 0;
    if (a < cbit || a + kk > cbit + 64) fill(a + kk);
    const uint32_t v = (uint32_t)((c >> (uint32_t)(a - cbit)) & ((1ull << kk) - 1ull));
    return v << sh;
  }
  // Sequence decoding (one container check per group of fields instead of one per field):
  // need(n) makes n <= 57 unread bits available in the container (all that is left near the
  // stream start); get(n), n <= 31, then reads them. Reading past the start gives garbage and
  // leaves bits < 0, which the caller reports as corrupt before the values are used.
  __device__ __forceinline__ void need(int32_t k) {
    if (bits - cbit < k && cbit > 0) fill(bits);
  }
  __device__ __forceinline__ uint32_t get(int32_t k) {
    bits -= k;
    return (uint32_t)(c >> ((uint32_t)(bits - cbit) & 63u)) & ((1u << k) - 1u);
  }
};

// Per-lane backward bitstream for one Huffman stream: its own LDS window (lane-private use) and a
// 64-bit register container of stream bits [cbit, cbit + 64), so a symbol costs one LDS access (its
// decoding entry) instead of two dependent ones.
struct LaneBits {
  uint32_t base, n, wlo;
  int64_t bits;
  uint8_t* win;
  uint64_t c;
  int64_t cbit;
  __device__ void refill(rsrc_t rs, uint32_t need_end) {
    const uint32_t lo = need_end > ZS_HWIN ? need_end - ZS_HWIN : 0;
    wlo = lo;
    for (uint32_t o = 0; o < ZS_HWIN; o += 16)
      *(u32x4*)(win + o) = u32x4{ld4_any(rs, base + lo + o), ld4_any(rs, base + lo + o + 4),
                                 ld4_any(rs, base + lo + o + 8), ld4_any(rs, base + lo + o + 12)};
  }
  __device__ void fill(rsrc_t rs, int64_t end) {
    const int64_t e8 = (end + 7) & ~7ll;
    cbit = e8 > 64 ? e8 - 64 : 0;
    const uint32_t b0 = (uint32_t)(cbit >> 3), b1 = b0 + 8u < n ? b0 + 8u : n;
    if (wlo == 0xFFFFFFFFu || b0 < wlo || b1 > wlo + ZS_HWIN) refill(rs, b1 + 8u < n ? b1 + 8u : n);
    typedef uint32_t __attribute__((may_alias)) u32a;
    const uint32_t rel = b0 - wlo, r4 = rel & ~3u, sft = rel & 3u;
    const uint32_t d0 = *(const u32a*)(win + r4), d1 = *(const u32a*)(win + r4 + 4), d2 = *(const u32a*)(win + r4 + 8);
    uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sft) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sft) << 32);
    const uint32_t nb = b1 - b0;
    if (nb < 8u) v &= (1ull << (8u * nb)) - 1ull;
    c = v;
  }
  __device__ uint32_t peek(rsrc_t rs, int k) {  // the next k bits without consuming (zeros past the start)
    int64_t a = bits - k;
    int sh = 0;
    if (a < 0) { sh = (int)-a; a = 0; }
    const int kk = k - sh;
    if (kk <= 0) return 0;
    if (a < cbit || a + kk > cbit + 64) fill(rs, a + kk);
    return (uint32_t)((c >> (uint32_t)(a - cbit)) & ((1ull << kk) - 1ull)) << sh;
  }
};

// FSE decoding table from normalized counts (RFC 8878 §4.1.1), wave-uniform; entries in `tab`.
__device__ bool zfse_build(ZWaveLds& L, uint32_t* tab, int nsym, int log) {
  int16_t* norm = L.ph.t.norm;
  uint16_t* nxt = L.ph.t.nxt;
  const int size = 1 << log;
  int high = size - 1;
  const uint32_t lane = lane_id();
  if (lane == 0) {
    for (int s = 0; s < nsym; s++) {
      if (norm[s] == -1) { tab[high--] = (uint32_t)s; nxt[s] = 1; }
      else nxt[s] = (uint16_t)norm[s];
    }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int pos = 0;
    for (int s = 0; s < nsym; s++)
      for (int i = 0; i < norm[s]; i++) {
        tab[pos] = (uint32_t)s;
        do { pos = (pos + step) & mask; } while (pos > high);
      }
    L.flag = pos != 0;  // the spread must end where it started
    if (pos == 0)
      for (int u = 0; u < size; u++) {
        const uint32_t s = tab[u] & 0xFFu;
        const uint32_t ns = nxt[s]++;
        const int nb = log - zhigh(ns);
        tab[u] = s | ((uint32_t)nb << 8) | (((ns << nb) - (uint32_t)size) << 16);
      }
  }
  wave_sync();
  return uni(L.flag) == 0;
}

// Normalized counts (FSE table description) at input offset `o`; returns bytes or -1.
__device__ int64_t zread_ncount(rsrc_t rs, uint32_t o, uint32_t lim, int max_log, int max_sym, int16_t* norm, int* nsym,
                                int* log) {
  FwdBits f{rs, lim, (uint64_t)o * 8u, false};
  const int accuracy = 5 + (int)f.get(4);
  if (accuracy > max_log) return -1;
  *log = accuracy;
  int remaining = (1 << accuracy) + 1, sym = 0;
  while (remaining > 1 && sym <= max_sym && !f.bad) {
    const int nbits = zhigh((uint32_t)remaining) + 1;
    const uint32_t maxv = (1u << nbits) - 1u - (uint32_t)remaining;
    uint32_t v = f.get(nbits - 1);
    if (v >= maxv) {
      v |= f.get(1) << (nbits - 1);
      if (v >= (1u << (nbits - 1))) v -= maxv;
    }
    const int prob = (int)v - 1;
    if (lane_id() == 0) norm[sym] = (int16_t)prob;
    sym++;
    remaining -= prob < 0 ? -prob : prob;
    if (prob == 0 && sym <= max_sym) {
      uint32_t rep;
      do {
        rep = f.get(2);
        for (uint32_t r = 0; r < rep && sym <= max_sym; r++) {
          if (lane_id() == 0) norm[sym] = 0;
          sym++;
        }
      } while (rep == 3 && !f.bad);
    }
  }
  wave_sync();
  if (f.bad || remaining != 1 || sym > max_sym + 1) return -1;
  *nsym = sym;
  return (int64_t)((f.bitpos + 7) >> 3) - o;
}

// Sequence table for one mode (RFC 8878 §3.1.1.3.2.1): predefined / RLE / FSE-compressed / repeat.
__device__ bool zseq_table(ZWaveLds& L, uint32_t* tab, int* tlog, bool& have, int mode, rsrc_t rs, uint32_t& q,
                           uint32_t lim, const int16_t* def, int def_n, int def_log, int max_log, int max_sym) {
  if (mode == 0) {
    if (lane_id() < (uint32_t)def_n) L.ph.t.norm[lane_id()] = def[lane_id()];
    wave_sync();
    *tlog = def_log;
    have = zfse_build(L, tab, def_n, def_log);
    return have;
  }
  if (mode == 1) {
    if (q >= lim) return false;
    const uint32_t s = zbyte(rs, q);
    q++;
    if ((int)s > max_sym) return false;
    if (lane_id() == 0) tab[0] = s;
    wave_sync();
    *tlog = 0;
    have = true;
    return true;
  }
  if (mode == 2) {
    int ns, lg;
    const int64_t u = zread_ncount(rs, q, lim, max_log, max_sym, L.ph.t.norm, &ns, &lg);
    if (u < 0) return false;
    q += (uint32_t)u;
    *tlog = lg;
    have = zfse_build(L, tab, ns, lg);
    return have;
  }
  return have;  // repeat
}

// Huffman decoding table from weights L.ph.t.wts[0, nsym) (+ the implied last weight), RFC 8878 §4.2.1.
__device__ int zhuf_build(ZWaveLds& L, int nsym) {
  uint32_t total = 0;
  for (int s = 0; s < nsym; s++) {
    const uint32_t w = L.ph.t.wts[s];
    if (w > 11) return -1;
    if (w) total += 1u << (w - 1);
  }
  if (!total) return -1;
  const int max_bits = zhigh(total) + 1;
  const uint32_t left = (1u << max_bits) - total;
  if (max_bits > 11 || (left & (left - 1u))) return -1;
  if (lane_id() == 0) L.ph.t.wts[nsym] = (uint8_t)(zhigh(left) + 1);
  wave_sync();
  nsym++;
  uint32_t next = 0;
  for (int wt = 1; wt <= max_bits; wt++) {
    const uint32_t nb = (uint32_t)(max_bits + 1 - wt), len = 1u << (wt - 1);
    for (int s = 0; s < nsym; s++) {
      if (L.ph.t.wts[s] != wt) continue;
      for (uint32_t e = lane_id(); e < len; e += WAVE) L.huf[next + e] = (uint16_t)(s | (nb << 8));
      next += len;
    }
  }
  wave_sync();
  return next == (1u << max_bits) ? max_bits : -1;
}

// Huffman tree description at q; returns max_bits (> 0) and advances q, or -1.
__device__ int zhuf_tree(ZWaveLds& L, rsrc_t rs, uint32_t& q, uint32_t lim) {
  if (q >= lim) return -1;
  const uint32_t hdr = zbyte(rs, q);
  int nsym = 0;
  if (hdr >= 128) {
    nsym = (int)hdr - 127;
    const uint32_t nb = (uint32_t)(nsym + 1) / 2;
    if (q + 1 + nb > lim) return -1;
    for (int s = (int)lane_id(); s < nsym; s += WAVE) {
      const uint32_t b = zbyte(rs, q + 1 + (uint32_t)s / 2);
      L.ph.t.wts[s] = (uint8_t)((s & 1) ? (b & 15u) : (b >> 4));
    }
    wave_sync();
    q += 1 + nb;
  } else {
    const uint32_t cs = hdr;
    if (q + 1 + cs > lim) return -1;
    int ns, lg;
    const int64_t hb = zread_ncount(rs, q + 1, q + 1 + cs, 6, 255, L.ph.t.norm, &ns, &lg);
    if (hb < 0) return -1;
    // its own table: a later block may repeat the sequence tables (LL / OF / ML mode 3)
    if (!zfse_build(L, L.ph.t.hw, ns, lg)) return -1;
    BackBits b;
    if (!b.init(rs, q + 1 + (uint32_t)hb, cs - (uint32_t)hb, L.win)) return -1;
    uint32_t s1 = b.read(lg), s2 = b.read(lg);
    // at most 255 decoded weights (libzstd HUF_readStats: FSE output capacity hwSize - 1)
    for (;;) {
      if (nsym >= 255) return -1;
      uint32_t e = L.ph.t.hw[s1];
      if (lane_id() == 0) L.ph.t.wts[nsym] = (uint8_t)(e & 0xFFu);
      nsym++;
      s1 = (e >> 16) + b.read((int)((e >> 8) & 0xFFu));
      if (b.bits < 0) {
        if (nsym >= 255) return -1;
        if (lane_id() == 0) L.ph.t.wts[nsym] = (uint8_t)(L.ph.t.hw[s2] & 0xFFu);
        nsym++;
        break;
      }
      if (nsym >= 255) return -1;
      e = L.ph.t.hw[s2];
      if (lane_id() == 0) L.ph.t.wts[nsym] = (uint8_t)(e & 0xFFu);
      nsym++;
      s2 = (e >> 16) + b.read((int)((e >> 8) & 0xFFu));
      if (b.bits < 0) {
        if (nsym >= 255) return -1;
        if (lane_id() == 0) L.ph.t.wts[nsym] = (uint8_t)(L.ph.t.hw[s1] & 0xFFu);
        nsym++;
        break;
      }
    }
    wave_sync();
    q += 1 + cs;
  }
  return zhuf_build(L, nsym);
}

// ---- output: global bytes + the LDS ring of the last ZS_RING bytes
struct ZOut {
  uint8_t* dst;
  uint32_t cap;        // job's output size: bytes past it are dropped (the page reader stops there)
  uint32_t pos;        // bytes produced (the newest ZS_RING of them are in the LDS ring)
  uint32_t frame0;     // output position of the current frame's start
  uint32_t drained;    // every store below this position has completed
  uint32_t flushed;    // output below this position has been stored from the ring to HBM
};

// Output bytes are produced into the LDS ring and stored to HBM from there ZS_FLUSH bytes at a time,
// as dwords aligned to the destination (byte stores only at the ends): one store instruction moves
// 256 bytes, where a byte store per output byte moved at most 64 (and usually 8: one match).
__device__ __forceinline__ void zput(ZOut& O, ZWaveLds& L, uint32_t p, uint32_t v) {
  (void)O;
  L.ring[p & (ZS_RING - 1u)] = (uint8_t)v;
}

__device__ __forceinline__ void zflush(ZOut& O, ZWaveLds& L) {
  const uint32_t a = O.flushed, e = O.pos < O.cap ? O.pos : O.cap;
  O.flushed = O.pos;
  if (a >= e) return;
  typedef uint32_t __attribute__((may_alias)) u32a;
  const u32a* ring32 = (const u32a*)L.ring;
  const uint32_t oal = (uint32_t)(uintptr_t)O.dst & 3u;
  const uint32_t base = ((a + oal) & ~3u) - oal;  // dst + base is dword aligned (base <= a, may wrap)
  const uint32_t skip = a - base, span = e - base;
  for (uint32_t d0 = 0; d0 < span; d0 += 4u * WAVE) {
    const uint32_t d = d0 + 4u * lane_id();
    if (d < span) {
      const uint32_t t = base + d, r = t & (ZS_RING - 1u) & ~3u;
      const uint32_t v = __builtin_amdgcn_alignbyte(ring32[((r + 4u) & (ZS_RING - 1u)) >> 2], ring32[r >> 2], t & 3u);
      if (d >= skip && d + 4u <= span) {
        gst((uint32_t*)(O.dst + t), v);
      } else {
#pragma unroll
        for (uint32_t j = 0; j < 4u; j++)
          if (d + j >= skip && d + j < span) gst(O.dst + (t + j), (uint8_t)(v >> (8u * j)));
      }
    }
  }
}

__device__ __forceinline__ void zmaybe_flush(ZOut& O, ZWaveLds& L) {
  wave_sync();
  if (O.pos - O.flushed >= ZS_FLUSH) zflush(O, L);
}

// output byte q (< pos): from the ring when recent, else from memory (system-scope load after a
// drain; the line may sit in this CU's L1 from before it was written)
__device__ __forceinline__ uint32_t zget(const ZOut& O, const ZWaveLds& L, uint32_t q, uint32_t pos) {
  if (pos - q <= ZS_RING - WAVE) return L.ring[q & (ZS_RING - 1u)];
  if (q >= O.cap) return 0;
  const uint32_t w = zld((const uint32_t*)(O.dst + (q & ~3u)));
  return (w >> ((q & 3u) * 8u)) & 0xFFu;
}

// every output byte produced so far stored and complete in HBM
__device__ __forceinline__ void zdrain(ZOut& O, ZWaveLds& L) {
  zflush(O, L);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  O.drained = O.pos;
}

// literal byte k of the block's literals: from the input at src + k (raw), the single byte `src`
// (RLE) or the literal buffer at src + k (Huffman-decoded)
__device__ __forceinline__ uint32_t zlit(int kind, rsrc_t rs, uint32_t src, const uint8_t* litbuf, uint32_t k) {
  if (kind == 0) return zbyte(rs, src + k);
  if (kind == 1) return src;
  const uint32_t a = src + k;
  return (zld((const uint32_t*)(litbuf + (a & ~3u))) >> ((a & 3u) * 8u)) & 0xFFu;
}

// copy n literal bytes (see zlit) to the output, 64 per round through the ring
__device__ __forceinline__ void zcopy_lits(ZOut& O, ZWaveLds& L, int kind, rsrc_t rs, uint32_t src, const uint8_t* litbuf,
                           uint32_t n) {
  const uint32_t p0 = O.pos;
  for (uint32_t k0 = 0; k0 < n; k0 += WAVE) {
    const uint32_t k = k0 + lane_id();
    if (k < n) zput(O, L, p0 + k, zlit(kind, rs, src, litbuf, k));
    wave_sync();
    const uint32_t done = p0 + (k0 + WAVE < n ? k0 + WAVE : n);
    if (done - O.flushed >= ZS_FLUSH) {  // keep the unflushed part well inside the ring
      O.pos = done;
      zflush(O, L);
    }
  }
  O.pos = p0 + n;
  zmaybe_flush(O, L);
}

// match: n bytes from `off` back; in rounds of min(off, 64) so a round only reads finished bytes
__device__ __forceinline__ void zcopy_match(ZOut& O, ZWaveLds& L, uint32_t off, uint32_t n) {
  const uint32_t step = off < WAVE ? off : WAVE;
  const uint32_t p0 = O.pos;
  for (uint32_t k0 = 0; k0 < n; k0 += step) {
    const uint32_t cur = p0 + k0;
    // a far match reads memory: every byte this round reads must have been stored
    if (off > ZS_RING - WAVE && cur + step - off > O.drained) {
      O.pos = cur;
      zdrain(O, L);
    }
    const uint32_t k = k0 + lane_id();
    if (lane_id() < step && k < n) zput(O, L, p0 + k, zget(O, L, p0 + k - off, cur));
    wave_sync();
    if (cur + step - O.flushed >= ZS_FLUSH) {  // keep the unflushed part well inside the ring
      O.pos = k0 + step < n ? cur + step : p0 + n;
      zflush(O, L);
    }
  }
  O.pos = p0 + n;
  zmaybe_flush(O, L);
}

// One batch of m decoded sequences (L.sq_*, lane k: sequence k) producing T <= ZS_CAP bytes: every
// output byte gets its source (a literal of the batch, or the output position it copies), pointer
// jumping follows in-batch copies of copies until every source is a literal or lies before the
// batch, then the bytes are gathered from the literal segment / the ring / HBM (older than the
// ring) at once. Sequences are dependent chains (a match of 8 bytes at offset 8 after 2 literals,
// again and again, in int64 data): they resolve in log2(depth) rounds instead of one at a time.
__device__ __forceinline__ void zexec_batch(ZOut& O, ZWaveLds& L, uint32_t m, int lit_kind, rsrc_t rs, uint32_t lit_src,
                            const uint8_t* litbuf, uint32_t lit_pos, int32_t lw_rel = -1) {
  const uint32_t lane = lane_id();
  const uint32_t ll = lane < m ? L.sq_ll[lane] : 0u, ml = lane < m ? L.sq_ml[lane] : 0u, of = lane < m ? L.sq_of[lane] : 0u;
  uint32_t T, LT;
  const uint32_t ob = wave_excl_scan_u32(ll + ml, &T);
  const uint32_t lb = wave_excl_scan_u32(ll, &LT);
  T = uni(T);
  LT = uni(LT);
  // the batch's literals [lit_pos, lit_pos + LT)
  for (uint32_t i = lane; i < LT; i += WAVE)
    L.ph.x.lseg[i] = lw_rel >= 0 ? L.win[(uint32_t)lw_rel + i]  // staged (replay): see zblock
                                 : (uint8_t)zlit(lit_kind, rs, lit_src, litbuf, lit_pos + i);
  const uint32_t op = O.pos;
  for (uint32_t i = 0; i < ll; i++) L.ph.x.src[ob + i] = ZS_LIT | (lb + i);
  for (uint32_t i = 0; i < ml; i++) L.ph.x.src[ob + ll + i] = op + ob + ll + i - of;
  wave_sync();
  constexpr uint32_t NB = ZS_CAP / WAVE;
  uint32_t sv[NB];
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint32_t b = lane + WAVE * j;
    sv[j] = b < T ? L.ph.x.src[b] : ZS_LIT;
  }
#pragma unroll 1
  for (uint32_t r = 0; r < 12u; r++) {  // branch-free rounds (the index is clamped to the table)
    bool more = false, hop = false;
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const bool inb = !(sv[j] & ZS_LIT) && sv[j] >= op;
      const uint32_t nv = L.ph.x.src[(sv[j] - op) & (ZS_CAP - 1u)];
      sv[j] = inb ? nv : sv[j];
      hop |= inb;
      more |= inb && !(nv & ZS_LIT) && nv >= op;
    }
    if (!__ballot(hop)) break;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) L.ph.x.src[lane + WAVE * j] = sv[j];  // entries >= T hold ZS_LIT
    wave_sync();
    if (!__ballot(more)) break;
  }
  // bytes: literals from the segment, earlier output from the ring or, older, from HBM
  uint32_t bv[NB];
  bool far = false;
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint32_t v = sv[j];
    bv[j] = (v & ZS_LIT) ? L.ph.x.lseg[v & (ZS_CAP - 1u)] : L.ring[v & (ZS_RING - 1u)];
    far |= lane + WAVE * j < T && !(v & ZS_LIT) && v + ZS_RING < op + WAVE;
  }
  if (__ballot(far)) {
    zdrain(O, L);
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const uint32_t v = sv[j];
      if (lane + WAVE * j < T && !(v & ZS_LIT) && v + ZS_RING < op + WAVE) bv[j] = zget(O, L, v, 0xFFFFFFFFu);
    }
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint32_t b = lane + WAVE * j;
    if (b < T) L.ring[(op + b) & (ZS_RING - 1u)] = (uint8_t)bv[j];
  }
  O.pos = op + T;
  zmaybe_flush(O, L);
}

// Decodes the block's next sequences into L.sq_* (RFC 8878 §3.1.1.3.2.1, §3.1.1.5): up to ZS_SB of
// them and ZS_CAP output bytes, stopping before one that does not fit (carried: pend 1) or after one
// longer than ZS_CAP (pend 2, in slot ZS_SB); a carried sequence opens the next batch. Returns 0 or
// PQG_ERR_CORRUPT.
__device__ __attribute__((noinline)) int zseq_decode(ZWaveLds& L) {
  ZSeq& S = L.ss;
  BackBits b;
  b.rs = make_rsrc((const uint8_t*)uni64(S.src), uni64(S.src_len));  // scalar (an argument would be VGPRs)
  b.win = L.win;
  b.base = uni(S.base);
  b.n = uni(S.n);
  b.wlo = uni(S.wlo);
  b.c = uni64(S.c);
  b.bits = (int32_t)uni((uint32_t)S.bits);
  b.cbit = (int32_t)uni((uint32_t)S.cbit);
  uint32_t sl = uni(S.sl), so = uni(S.so), sm = uni(S.sm);
  uint32_t r0 = uni(S.rep0), r1 = uni(S.rep1), r2 = uni(S.rep2);
  uint32_t i = uni(S.i);
  const uint32_t nseq = uni(S.nseq), regen = uni(S.regen), frame0 = uni(S.frame0);
  uint32_t outp = uni(S.outp), lits = uni(S.lits);
  const bool lane0 = lane_id() == 0;
  uint32_t m = 0, T = 0, blit = 0, pend = 0;
  int code = 0;
  if (uni(S.pend) == 1u) {  // the sequence carried from the last batch opens this one
    const uint32_t ll = uni(L.sq_ll[ZS_SB]), ml = uni(L.sq_ml[ZS_SB]);
    if (lane0) {
      L.sq_ll[0] = ll;
      L.sq_ml[0] = ml;
      L.sq_of[0] = L.sq_of[ZS_SB];
    }
    m = 1;
    T = ll + ml;
    blit = ll;
  }
  while (i < nseq) {
    const uint32_t el = uni(L.ll[sl]), eo = uni(L.of[so]), em = uni(L.ml[sm]);
    const uint32_t llc = el & 0xFFu, ofc = eo & 0xFFu, mlc = em & 0xFFu;
    if (llc > 35 || mlc > 52 || ofc > 31) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t mle = uni(L.mlcode[mlc]), lle = uni(L.llcode[llc]);
    const int32_t mlb = (int32_t)(mle >> 24), llb = (int32_t)(lle >> 24);
    b.need((int32_t)ofc);  // offset, match length, literal length extra bits
    const uint32_t ofv = (1u << ofc) + b.get((int32_t)ofc);
    b.need(mlb + llb);
    const uint32_t ml = (mle & 0xFFFFFFu) + b.get(mlb);
    const uint32_t ll = (lle & 0xFFFFFFu) + b.get(llb);
    uint32_t off;
    if (ofv > 3) {
      off = ofv - 3u;
      r2 = r1; r1 = r0; r0 = off;
    } else {
      uint32_t idx = ofv - 1u;
      if (ll == 0) idx++;
      if (idx == 0) {
        off = r0;
      } else if (idx == 3) {
        off = r0 - 1u;
        if (off == 0) { code = PQG_ERR_CORRUPT; break; }
        r2 = r1; r1 = r0; r0 = off;
      } else {
        off = idx == 1 ? r1 : r2;
        if (idx == 2) r2 = r1;
        r1 = r0;
        r0 = off;
      }
    }
    i++;
    if (i < nseq) {  // state updates: literal length, match length, offset
      const int32_t nl = (int32_t)((el >> 8) & 0xFFu), nm = (int32_t)((em >> 8) & 0xFFu), no = (int32_t)((eo >> 8) & 0xFFu);
      b.need(nl + nm + no);  // <= 26 bits
      sl = (el >> 16) + b.get(nl);
      sm = (em >> 16) + b.get(nm);
      so = (eo >> 16) + b.get(no);
    }
    if (b.bits < 0 || lits + ll > regen) { code = PQG_ERR_CORRUPT; break; }
    if (off == 0 || off > outp + ll - frame0) { code = PQG_ERR_CORRUPT; break; }
    lits += ll;
    outp += ll + ml;
    const bool big = (uint64_t)ll + ml > ZS_CAP;
    if (big || T + ll + ml > ZS_CAP || m == ZS_SB) {
      if (lane0) {
        L.sq_ll[ZS_SB] = ll;
        L.sq_ml[ZS_SB] = ml;
        L.sq_of[ZS_SB] = off;
      }
      pend = big ? 2u : 1u;
      break;
    }
    if (lane0) {
      L.sq_ll[m] = ll;
      L.sq_ml[m] = ml;
      L.sq_of[m] = off;
    }
    m++;
    T += ll + ml;
    blit += ll;
  }
  if (lane0) {
    S.c = b.c; S.bits = b.bits; S.cbit = b.cbit; S.wlo = b.wlo;
    S.sl = sl; S.so = so; S.sm = sm;
    S.rep0 = r0; S.rep1 = r1; S.rep2 = r2;
    S.i = i; S.outp = outp; S.lits = lits;
    S.m = m; S.T = T; S.blit = blit; S.pend = pend;
  }
  wave_sync();
  return code;
}

// One compressed block [q, q + bs) of the job's input. Returns 0 or an error code.
__device__ __forceinline__ int zblock(ZWaveLds& L, ZOut& O, rsrc_t rs, uint32_t q, uint32_t bs, uint8_t* litbuf, bool& have_huf,
                      int& huf_bits, bool* have_tab, int* tlog, uint32_t* rep, const uint64_t* rec, uint32_t& rc) {
  const uint32_t lim = q + bs;
  if (bs < 1) return PQG_ERR_CORRUPT;
  const uint32_t b0 = zbyte(rs, q);
  const int lt = (int)(b0 & 3u), sf = (int)((b0 >> 2) & 3u);
  uint32_t regen = 0, comp = 0, hl = 0;
  if (lt <= 1) {
    if (sf == 0 || sf == 2) { regen = b0 >> 3; hl = 1; }
    else if (sf == 1) { regen = (b0 >> 4) + (zbyte(rs, q + 1) << 4); hl = 2; }
    else { regen = (b0 >> 4) + (zbyte(rs, q + 1) << 4) + (zbyte(rs, q + 2) << 12); hl = 3; }
  } else {
    const uint64_t v = ld8_any(rs, q);
    if (sf <= 1) { regen = (uint32_t)(v >> 4) & 0x3FFu; comp = (uint32_t)(v >> 14) & 0x3FFu; hl = 3; }
    else if (sf == 2) { regen = (uint32_t)(v >> 4) & 0x3FFFu; comp = (uint32_t)(v >> 18) & 0x3FFFu; hl = 4; }
    else { regen = (uint32_t)(v >> 4) & 0x3FFFFu; comp = (uint32_t)(v >> 22) & 0x3FFFFu; hl = 5; }
  }
  if (q + hl > lim || regen > ZS_LIT_MAX) return PQG_ERR_CORRUPT;
  uint32_t p = q + hl;
  ZD_T(t_lit);
  int lit_kind;          // 0 raw (input at lit_src), 1 RLE (byte lit_src), 2 decoded into litbuf
  uint32_t lit_src = 0;
  if (lt == 0) {
    if (p + regen > lim) return PQG_ERR_CORRUPT;
    lit_kind = 0; lit_src = p; p += regen;
  } else if (lt == 1) {
    if (p + 1 > lim) return PQG_ERR_CORRUPT;
    lit_kind = 1; lit_src = zbyte(rs, p); p += 1;
  } else {
    if (p + comp > lim) return PQG_ERR_CORRUPT;
    uint32_t c = p;
    const uint32_t cend = p + comp;
    if (lt == 2) {
      huf_bits = zhuf_tree(L, rs, c, cend);
      if (huf_bits < 0) return PQG_ERR_CORRUPT;
      have_huf = true;
    } else if (!have_huf) {
      return PQG_ERR_CORRUPT;
    }
    // streams: 1 (lane 0) or 4 (lanes 0..3), each decoded into its part of litbuf
    uint32_t sb[4] = {c, 0, 0, 0}, sn[4] = {cend - c, 0, 0, 0}, cnt[4] = {regen, 0, 0, 0}, dst0[4] = {0, 0, 0, 0};
    int ns = 1;
    if (sf != 0) {
      if (cend - c < 6) return PQG_ERR_CORRUPT;
      const uint32_t s1 = zbyte(rs, c) | (zbyte(rs, c + 1) << 8), s2 = zbyte(rs, c + 2) | (zbyte(rs, c + 3) << 8),
                     s3 = zbyte(rs, c + 4) | (zbyte(rs, c + 5) << 8);
      const uint32_t tot = cend - c - 6;
      if ((uint64_t)s1 + s2 + s3 > tot) return PQG_ERR_CORRUPT;
      const uint32_t seg = (regen + 3) / 4;
      if (3 * seg > regen) return PQG_ERR_CORRUPT;
      sb[0] = c + 6; sn[0] = s1;
      sb[1] = sb[0] + s1; sn[1] = s2;
      sb[2] = sb[1] + s2; sn[2] = s3;
      sb[3] = sb[2] + s3; sn[3] = tot - s1 - s2 - s3;
      cnt[0] = cnt[1] = cnt[2] = seg; cnt[3] = regen - 3 * seg;
      dst0[1] = seg; dst0[2] = 2 * seg; dst0[3] = 3 * seg;
      ns = 4;
    }
    const uint32_t lane = lane_id();
    int bad = 0;
    if ((int)lane < ns) {
      uint32_t mb = 0, mn = 0, mc = 0, md = 0;
#pragma unroll
      for (int i = 0; i < 4; i++)
        if ((int)lane == i) { mb = sb[i]; mn = sn[i]; mc = cnt[i]; md = dst0[i]; }
      LaneBits lb{mb, mn, 0xFFFFFFFFu, 0, L.ph.t.hwin[lane], 0, INT64_MAX};
      const uint32_t last = mn ? zbyte(rs, mb + mn - 1) : 0u;
      if (!last) {
        bad = 1;
      } else {
        lb.bits = (int64_t)(mn - 1) * 8 + zhigh(last);
        uint32_t acc = 0;
        for (uint32_t i = 0; i < mc; i++) {
          const uint32_t e = L.huf[lb.peek(rs, huf_bits)];
          lb.bits -= (int64_t)(e >> 8);
          if (lb.bits < 0) { bad = 1; break; }
          const uint32_t o = md + i;
          acc |= (e & 0xFFu) << ((o & 3u) * 8u);
          if ((o & 3u) == 3u || i + 1 == mc) {  // flush a (partial) dword: byte stores keep neighbours
            if ((o & 3u) == 3u && (o & ~3u) >= md) {
              gst((uint32_t*)(litbuf + (o & ~3u)), acc);  // a whole dword of this stream
            } else {
              for (uint32_t j = (o & ~3u) > md ? (o & ~3u) : md; j <= o; j++) gst(litbuf + j, (uint8_t)(acc >> ((j & 3u) * 8u)));
            }
            acc = 0;
          }
        }
        if (!bad && lb.bits != 0) bad = 1;
      }
    }
    if (__ballot(bad)) return PQG_ERR_CORRUPT;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // literals in memory before they are read back
    lit_kind = 2;
    p += comp;
  }
  ZD_ADD(L, 0, t_lit);
  ZD_CNT(L, 7, regen);
  // ---- sequences
  if (p >= lim) return PQG_ERR_CORRUPT;
  uint32_t nseq = zbyte(rs, p);
  if (nseq == 0) {
    p += 1;
    zcopy_lits(O, L, lit_kind, rs, lit_src, litbuf, regen);
    return p == lim ? 0 : PQG_ERR_CORRUPT;
  }
  if (nseq < 128) { p += 1; }
  else if (nseq < 255) { nseq = ((nseq - 128) << 8) + zbyte(rs, p + 1); p += 2; }
  else { nseq = zbyte(rs, p + 1) + (zbyte(rs, p + 2) << 8) + 0x7F00u; p += 3; }
  if (p >= lim) return PQG_ERR_CORRUPT;
  if (rec) {  // replay: k_zstd_seq decoded (and checked) this block's sequences
    ZD_T(t_rep);
    const uint32_t lane = lane_id();
    uint32_t i = 0, lit_pos = 0;
    // record queue: records [qb, qe) of the block, lane l of q_j holding record qb + 64 j + l (one
    // load round per 256 records instead of one per batch)
    uint64_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    uint32_t qb = 0, qe = 0;
    // raw / Huffman-decoded literals staged ZS_WIN bytes at a time in L.win (free in replay: no
    // bitstream): one load round per ~1 KiB of literals instead of one per batch. Source address of
    // literal k: lit_src + k in the input (raw), k in litbuf (decoded); window [lw, lw + ZS_WIN).
    uint32_t lw = 0xFFFFFFFFu;
    const uint32_t sa0 = lit_kind == 0 ? lit_src : 0u;
    auto stage = [&](uint32_t k) {
      lw = (sa0 + k) & ~3u;
      for (uint32_t j = lane; j < ZS_WIN / 4u; j += WAVE) {
        const uint32_t a = lw + 4u * j;
        const uint32_t v = lit_kind == 0 ? ld32(rs, a) : zld((const uint32_t*)(litbuf + a));
        *(uint32_t*)(L.win + 4u * j) = v;
      }
      wave_sync();
    };
    auto shfl64 = [](uint64_t v, uint32_t l) -> uint64_t {
      return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, (int)l) | ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)l) << 32);
    };
    while (i < nseq) {
      if (i + WAVE > qe && qe < nseq) {
        qb = i;
        qe = i + 4u * WAVE < nseq ? i + 4u * WAVE : nseq;
        const uint32_t b = i + lane;
        q0 = b < nseq ? rec[rc + b] : 0ull;
        q1 = b + WAVE < nseq ? rec[rc + b + WAVE] : 0ull;
        q2 = b + 2u * WAVE < nseq ? rec[rc + b + 2u * WAVE] : 0ull;
        q3 = b + 3u * WAVE < nseq ? rec[rc + b + 3u * WAVE] : 0ull;
      }
      const uint32_t k = i + lane;
      const uint32_t d = uni(i - qb), s0 = d >> 6, l = (d + lane) & (WAVE - 1u);
      const bool upper = (d & (WAVE - 1u)) + lane >= WAVE;  // the lane's record sits in slot s0 + 1
      const uint64_t A = s0 == 0 ? q0 : s0 == 1 ? q1 : s0 == 2 ? q2 : q3;
      const uint64_t Bq = s0 == 0 ? q1 : s0 == 1 ? q2 : s0 == 2 ? q3 : 0ull;
      const uint64_t ra = shfl64(A, l), rb = shfl64(Bq, l);
      const uint64_t r = k < nseq ? (upper ? rb : ra) : 0ull;
      const uint32_t ll = (uint32_t)r & 0x3FFFFu, ml = (uint32_t)(r >> 18) & 0x3FFFFu, off = (uint32_t)(r >> 36);
      const uint32_t tot = ll + ml;
      const bool big = tot > ZS_CAP;
      const uint32_t cum = (uint32_t)wave_incl_scan_u64(big ? (uint64_t)ZS_CAP + 1u : tot);
      const uint64_t stop = __ballot(k >= nseq || big || cum > ZS_CAP);
      const uint32_t m = stop ? (uint32_t)__builtin_ctzll(stop) : WAVE;
      if (lane < m) {
        L.sq_ll[lane] = ll;
        L.sq_ml[lane] = ml;
        L.sq_of[lane] = off;
      }
      uint32_t blit;
      (void)wave_excl_scan_u32(lane < m ? ll : 0u, &blit);
      blit = uni(blit);
      wave_sync();
      if (m) {
        int32_t rel = -1;
        if (lit_kind != 1 && blit) {
          if (lw == 0xFFFFFFFFu || sa0 + lit_pos < lw || sa0 + lit_pos + blit > lw + ZS_WIN) stage(lit_pos);
          rel = (int32_t)(sa0 + lit_pos - lw);
        }
        zexec_batch(O, L, m, lit_kind, rs, lit_src, litbuf, lit_pos, rel);
        lit_pos += blit;
      }
      i += m;
      if (m < WAVE && i < nseq && uni(rdl(big ? 1u : 0u, m))) {  // a sequence longer than a batch: through the ring
        const uint32_t bll = uni(rdl(ll, m)), bml = uni(rdl(ml, m)), bof = uni(rdl(off, m));
        if (bll) zcopy_lits(O, L, lit_kind, rs, lit_kind == 1 ? lit_src : lit_src + lit_pos, litbuf, bll);
        lit_pos += bll;
        zcopy_match(O, L, bof, bml);
        i++;
      }
    }
    rc += nseq;
    ZD_ADD(L, 2, t_rep);
    if (regen > lit_pos) zcopy_lits(O, L, lit_kind, rs, lit_kind == 1 ? lit_src : lit_src + lit_pos, litbuf, regen - lit_pos);
    return 0;
  }
  ZD_T(t_tab);
  const uint32_t modes = zbyte(rs, p++);
  if (modes & 3u) return PQG_ERR_CORRUPT;
  if (!zseq_table(L, L.ll, &tlog[0], have_tab[0], (int)(modes >> 6), rs, p, lim, ZLL_DEF, 36, 6, 9, 35)) return PQG_ERR_CORRUPT;
  if (!zseq_table(L, L.of, &tlog[1], have_tab[1], (int)((modes >> 4) & 3u), rs, p, lim, ZOF_DEF, 29, 5, 8, 31)) return PQG_ERR_CORRUPT;
  if (!zseq_table(L, L.ml, &tlog[2], have_tab[2], (int)((modes >> 2) & 3u), rs, p, lim, ZML_DEF, 53, 6, 9, 52)) return PQG_ERR_CORRUPT;
  BackBits b;
  if (!b.init(rs, p, lim - p, L.win)) return PQG_ERR_CORRUPT;
  b.need(tlog[0] + tlog[1] + tlog[2]);  // <= 27 bits
  const uint32_t sl0 = b.get(tlog[0]);
  const uint32_t so0 = b.get(tlog[1]);
  const uint32_t sm0 = b.get(tlog[2]);
  ZD_ADD(L, 1, t_tab);
  ZD_CNT(L, 6, nseq);
  ZD_T(t_seq);
  // Sequences are decoded one after another (the three FSE states and the backward bitstream are
  // serial) by zseq_decode, a batch at a time (up to ZS_SB sequences, ZS_CAP output bytes, in LDS),
  // and each batch is executed at once (zexec_batch); a sequence longer than ZS_CAP runs on its own
  // through the ring.
  if (lane_id() == 0) {
    ZSeq& S = L.ss;
    S.c = b.c; S.bits = b.bits; S.cbit = b.cbit; S.wlo = b.wlo; S.base = b.base; S.n = b.n;
    S.sl = sl0; S.so = so0; S.sm = sm0;
    S.rep0 = rep[0]; S.rep1 = rep[1]; S.rep2 = rep[2];
    S.i = 0; S.nseq = nseq; S.outp = O.pos; S.lits = 0; S.regen = regen; S.frame0 = O.frame0;
    S.pend = 0;
  }
  wave_sync();
  uint32_t lit_pos = 0;  // literals consumed by executed sequences
  while (true) {
    if (zseq_decode(L)) return PQG_ERR_CORRUPT;
    const uint32_t m = uni(L.ss.m), blit = uni(L.ss.blit), pend = uni(L.ss.pend);
    if (m) {
      ZD_T(t_ex);
      zexec_batch(O, L, m, lit_kind, rs, lit_src, litbuf, lit_pos);
      ZD_ADD(L, 3, t_ex);
      lit_pos += blit;
    }
    if (pend == 2u) {  // a long sequence: through the ring
      ZD_T(t_long);
      const uint32_t ll = uni(L.sq_ll[ZS_SB]), ml = uni(L.sq_ml[ZS_SB]), off = uni(L.sq_of[ZS_SB]);
      if (ll) zcopy_lits(O, L, lit_kind, rs, lit_kind == 1 ? lit_src : lit_src + lit_pos, litbuf, ll);
      lit_pos += ll;
      zcopy_match(O, L, off, ml);
      if (lane_id() == 0) L.ss.pend = 0;
      wave_sync();
      ZD_ADD(L, 4, t_long);
    }
    if (pend == 0u && uni(L.ss.i) == nseq) break;
  }
  rep[0] = uni(L.ss.rep0);
  rep[1] = uni(L.ss.rep1);
  rep[2] = uni(L.ss.rep2);
  ZD_ADD(L, 2, t_seq);
  if ((int32_t)uni((uint32_t)L.ss.bits) != 0) return PQG_ERR_CORRUPT;
  if (regen > lit_pos) zcopy_lits(O, L, lit_kind, rs, lit_kind == 1 ? lit_src : lit_src + lit_pos, litbuf, regen - lit_pos);
  return 0;
}

// XXH64 of the frame's output [a, e) (content checksum), lane 0 alone: the output is re-read from
// memory after a drain. Only for frames that carry a checksum.
__device__ uint64_t zxxh64(const uint8_t* p, uint32_t n) {
  constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                     P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  const uint32_t mis = (uint32_t)(uintptr_t)p & 3u;
  const uint32_t* base = (const uint32_t*)(p - mis);
  const uint32_t last_w = n ? (n - 1u + mis) >> 2 : 0u;  // the output's last dword: nothing past it is read
  auto rd = [&](uint32_t o, int bytes) {  // little-endian bytes [o, o + bytes) of the output, bytes <= 8
    const uint32_t a = o + mis, w = a >> 2, s = a & 3u;
    const uint32_t d0 = zld(base + w), d1 = w + 1u <= last_w ? zld(base + w + 1) : 0u,
                   d2 = s && w + 2u <= last_w ? zld(base + w + 2) : 0u;
    uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
    return bytes == 8 ? v : v & ((1ull << (8 * bytes)) - 1ull);
  };
  auto round = [&](uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl(acc, 31); return acc * P1; };
  uint32_t o = 0;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; o + 32 <= n; o += 32) {
      v1 = round(v1, rd(o, 8)); v2 = round(v2, rd(o + 8, 8)); v3 = round(v3, rd(o + 16, 8)); v4 = round(v4, rd(o + 24, 8));
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) { h ^= round(0, v); h = h * P1 + P4; }
  } else {
    h = P5;
  }
  h += n;
  for (; o + 8 <= n; o += 8) { h ^= round(0, rd(o, 8)); h = rotl(h, 27) * P1 + P4; }
  if (o + 4 <= n) { h ^= rd(o, 4) * P1; h = rotl(h, 23) * P2 + P3; o += 4; }
  for (; o < n; o++) { h ^= rd(o, 1) * P5; h = rotl(h, 11) * P1; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

// ---- Sequence pre-pass (k_zstd_seq): one LANE per job ------------------------------------------------
// The sequence section is a serial chain per block (three FSE states and one backward bitstream), and
// decoded by a wave's scalar unit it costs ~150 scalar instructions per sequence, which the CU's one
// scalar unit issues for all of its waves: 100 M int64 PLAIN pages took 44 ms, scalar-issue bound.
// Here every lane decodes the sequences of its own job (page) with vector instructions — one
// instruction advances 16 pages — and writes them as 8-byte records {ll:18, ml:18, offset:28} in
// stream order to `seqs` (job j's records at dst_offset / 5, capacity (dst_offset + dst_size) / 5 -
// dst_offset / 5: disjoint because the jobs' outputs are). k_zstd then replays them (literals, match
// execution, checksums) instead of decoding. The pre-pass checks everything the inline decoder
// checks in the sequence section; anything it does not take (a malformed or unusual stream, a page
// of >= 2^28 bytes, more sequences than its capacity) marks the job for the inline path, which then
// reports exactly what it always did. Per lane: its FSE tables (one u32 per state: next-state base,
// state bits, the symbol's extra bits and baseline: 5 KiB for LL 512 + ML 512 + OF 256 states; 12
// lanes per workgroup, 2 workgroups per CU) and a 512-byte LDS window of
// its bitstream. Window refills are collective: when any lane of the sequence loop could read below
// its window in the next sequence, every lane in the loop re-centres its window at its position, so
// the wave waits for one round of loads per ~150 sequences instead of once per lane's refill
// (measured: per-lane refills at uncorrelated times stalled the wave every few sequences).
constexpr uint32_t ZQ_JOBS = 12;  // lanes (jobs) per workgroup
#ifdef PQG_DIAG
// Diagnostic build only (tools/diag_zstd.py): per job 6 u64 = pre-pass cycles (whole job, tables,
// sequence loops), sequences, window re-centrings, compressed blocks.
static __device__ uint64_t* pqg_zqdiag;
extern "C" int pqg_diag_zq_set(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pqg_zqdiag), &p, sizeof(p)) == hipSuccess ? 0 : 3;
}
struct ZqDiag {
  uint64_t tab, loop, seqs, rec, blocks;
};
#define ZQD_ARG , ZqDiag& zd
#define ZQD_PASS , zd
#else
#define ZQD_ARG
#define ZQD_PASS
#endif
constexpr uint32_t ZQ_WIN = 512;
constexpr uint32_t ZQ_LL = 0, ZQ_ML = 512, ZQ_OF = 1024;  // table regions (entries)
constexpr int32_t ZQ_REPLAY = 0, ZQ_INLINE = 1;

struct ZqLane {
  uint8_t win[ZQ_WIN + 16];  // bitstream bytes [wlo, wlo + ZQ_WIN) of the job's input (absolute offsets)
  uint32_t e[1280];          // FSE entries (zq_entry): next-state base, state bits, the symbol's extra bits and baseline
  int16_t norm[56];
  uint16_t nxt[56];
};
struct ZqLds {
  ZqLane l[ZQ_JOBS];
  uint32_t llcode[36], mlcode[53];
  int16_t def_ll[36], def_ml[53], def_of[29];
};

// A decoding entry carries what the sequence step needs from its symbol, so a state costs one LDS
// read: next-state base (bits 0-8) | state bits << 9 | the symbol's extra bits << 13 | its baseline
// << 18 (0x3FFF: a baseline of >= 16,383, which for every such code is (1 << extra bits) + ZQ_ADD:
// LL codes 33-35, ML codes 50-52 (+3), offset codes >= 14).
constexpr uint32_t ZQ_BIG = 0x3FFFu;
__device__ __forceinline__ uint32_t zq_sym_entry(const ZqLds& L, int kind, uint32_t sy) {
  uint32_t xb, bl;
  if (kind == 0) { xb = L.llcode[sy] >> 24; bl = L.llcode[sy] & 0xFFFFFFu; }
  else if (kind == 1) { xb = L.mlcode[sy] >> 24; bl = L.mlcode[sy] & 0xFFFFFFu; }
  else { xb = sy; bl = 1u << sy; }
  return (xb << 13) | ((bl >= ZQ_BIG ? ZQ_BIG : bl) << 18);
}
__device__ __forceinline__ uint32_t zq_baseline(uint32_t e, uint32_t add) {
  const uint32_t bl = e >> 18;
  return bl != ZQ_BIG ? bl : (1u << ((e >> 13) & 31u)) + add;
}

// FSE decoding table of `nsym` normalized counts (T.norm) with accuracy `log` into region `r`
// (kind 0 LL, 1 ML, 2 OF: which code table the symbols index).
__device__ bool zq_build(const ZqLds& L, ZqLane& T, uint32_t r, int nsym, int log, int kind) {
  const int size = 1 << log, mask = size - 1;
  int high = size - 1;
  for (int s = 0; s < nsym; s++) {
    if (T.norm[s] == -1) {
      T.e[r + high--] = (uint32_t)s;
      T.nxt[s] = 1;
    } else {
      T.nxt[s] = (uint16_t)T.norm[s];
    }
  }
  const int step = (size >> 1) + (size >> 3) + 3;
  int pos = 0;
  for (int s = 0; s < nsym; s++)
    for (int i = 0; i < T.norm[s]; i++) {
      T.e[r + pos] = (uint32_t)s;
      do { pos = (pos + step) & mask; } while (pos > high);
    }
  if (pos != 0) return false;
  for (int u = 0; u < size; u++) {
    const uint32_t sy = T.e[r + u];
    const uint32_t ns = T.nxt[sy]++;
    const int nb = log - zhigh(ns);
    T.e[r + u] = ((ns << nb) - (uint32_t)size) | ((uint32_t)nb << 9) | zq_sym_entry(L, kind, sy);
  }
  return true;
}

// Normalized counts at input offset o (absolute) into T.norm; returns bytes read or -1.
__device__ int64_t zq_ncount(ZqLane& T, rsrc_t rs, uint32_t o, uint32_t lim, int max_log, int max_sym, int* nsym, int* log) {
  FwdBits f{rs, lim, (uint64_t)o * 8u, false};
  const int accuracy = 5 + (int)f.get(4);
  if (accuracy > max_log) return -1;
  *log = accuracy;
  int remaining = (1 << accuracy) + 1, sym = 0;
  while (remaining > 1 && sym <= max_sym && !f.bad) {
    const int nbits = zhigh((uint32_t)remaining) + 1;
    const uint32_t maxv = (1u << nbits) - 1u - (uint32_t)remaining;
    uint32_t v = f.get(nbits - 1);
    if (v >= maxv) {
      v |= f.get(1) << (nbits - 1);
      if (v >= (1u << (nbits - 1))) v -= maxv;
    }
    const int prob = (int)v - 1;
    T.norm[sym] = (int16_t)prob;
    sym++;
    remaining -= prob < 0 ? -prob : prob;
    if (prob == 0 && sym <= max_sym) {
      uint32_t rep;
      do {
        rep = f.get(2);
        for (uint32_t r = 0; r < rep && sym <= max_sym; r++) T.norm[sym++] = 0;
      } while (rep == 3 && !f.bad);
    }
  }
  if (f.bad || remaining != 1 || sym > max_sym + 1) return -1;
  *nsym = sym;
  return (int64_t)((f.bitpos + 7) >> 3) - o;
}

// One sequence table (mode: predefined / RLE / FSE-compressed / repeat), as zseq_table.
__device__ bool zq_table(const ZqLds& L, int kind, ZqLane& T, uint32_t r, int* tlog, bool& have, int mode, rsrc_t rs,
                         uint32_t& q, uint32_t lim,
                         const int16_t* def, int def_n, int def_log, int max_log, int max_sym) {
  if (mode == 0) {
    for (int i = 0; i < def_n; i++) T.norm[i] = def[i];
    *tlog = def_log;
    have = zq_build(L, T, r, def_n, def_log, kind);
    return have;
  }
  if (mode == 1) {
    if (q >= lim) return false;
    const uint32_t sy = zbyte(rs, q);
    q++;
    if ((int)sy > max_sym) return false;
    T.e[r] = zq_sym_entry(L, kind, sy);
    *tlog = 0;
    have = true;
    return true;
  }
  if (mode == 2) {
    int ns, lg;
    const int64_t u = zq_ncount(T, rs, q, lim, max_log, max_sym, &ns, &lg);
    if (u < 0) return false;
    q += (uint32_t)u;
    *tlog = lg;
    have = zq_build(L, T, r, ns, lg, kind);
    return have;
  }
  return have;
}

// The sequences of one compressed block's sequence section [q, lim) (absolute input offsets). Returns
// false for anything the inline path must handle.
__device__ bool zq_block_seqs(ZqLds& L, ZqLane& T, rsrc_t rs, uint32_t q, uint32_t lim, uint32_t regen, uint32_t& outp,
                              uint32_t frame0, uint32_t* rep, bool* have_tab, int* tlog, uint64_t* rec, uint32_t& cnt,
                              uint32_t cap ZQD_ARG) {
  if (q >= lim) return false;
  uint32_t nseq = zbyte(rs, q);
  if (nseq == 0) {
    outp += regen;
    return q + 1u == lim;
  }
  if (nseq < 128) { q += 1; }
  else if (nseq < 255) { nseq = ((nseq - 128) << 8) + zbyte(rs, q + 1); q += 2; }
  else { nseq = zbyte(rs, q + 1) + (zbyte(rs, q + 2) << 8) + 0x7F00u; q += 3; }
  if (q >= lim) return false;
  const uint32_t modes = zbyte(rs, q++);
  if (modes & 3u) return false;
#ifdef PQG_DIAG
  const uint64_t zt0 = __builtin_amdgcn_s_memtime();
  zd.blocks++;
#endif
  if (!zq_table(L, 0, T, ZQ_LL, &tlog[0], have_tab[0], (int)(modes >> 6), rs, q, lim, L.def_ll, 36, 6, 9, 35)) return false;
  if (!zq_table(L, 2, T, ZQ_OF, &tlog[1], have_tab[1], (int)((modes >> 4) & 3u), rs, q, lim, L.def_of, 29, 5, 8, 31))
    return false;
  if (!zq_table(L, 1, T, ZQ_ML, &tlog[2], have_tab[2], (int)((modes >> 2) & 3u), rs, q, lim, L.def_ml, 53, 6, 9, 52))
    return false;
  // backward bitstream [q, lim): container c = stream bits [cbit, cbit + 64), from the LDS window
  const uint32_t sb = q, sn = lim - q;
  if (sn == 0) return false;
  const uint32_t lastb = zbyte(rs, sb + sn - 1u);
  if (!lastb) return false;
  int32_t bits = (int32_t)(sn - 1u) * 8 + zhigh(lastb), cbit = 0;
  uint32_t wlo = 0xFFFFFFFFu;
  uint64_t c = 0;
  typedef uint32_t __attribute__((may_alias)) u32a;
  auto recenter = [&](uint32_t b0) {  // window [wlo, wlo + ZQ_WIN) with b0 16-32 bytes below its top
    const uint32_t top = (b0 + 16u) & ~15u;
    wlo = top >= ZQ_WIN - 16u ? top - (ZQ_WIN - 16u) : 0u;
#pragma unroll
    for (uint32_t o = 0; o < ZQ_WIN; o += 16)
      *(u32x4*)(T.win + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(wlo + o), 0, 0);
  };
  auto fill = [&](int32_t end) {
    const int32_t e8 = (end + 7) & ~7;
    cbit = e8 > 64 ? e8 - 64 : 0;
    const uint32_t b0 = sb + ((uint32_t)cbit >> 3);  // absolute
    const uint32_t b1 = b0 + 8u < sb + sn ? b0 + 8u : sb + sn;
    if (wlo == 0xFFFFFFFFu || b0 < wlo || b0 + 12u > wlo + ZQ_WIN) recenter(b0);
    const uint32_t rel = b0 - wlo, r4 = rel & ~3u, sft = rel & 3u;
    const uint32_t d0 = *(const u32a*)(T.win + r4), d1 = *(const u32a*)(T.win + r4 + 4), d2 = *(const u32a*)(T.win + r4 + 8);
    uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sft) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sft) << 32);
    const uint32_t nb = b1 - b0;
    if (nb < 8u) v &= (1ull << (8u * nb)) - 1ull;
    c = v;
  };
  auto need = [&](int32_t k) {
    if (bits - cbit < k && cbit > 0) fill(bits);
  };
  auto get = [&](int32_t k) -> uint32_t {
    bits -= k;
    return (uint32_t)(c >> ((uint32_t)(bits - cbit) & 63u)) & ((1u << k) - 1u);
  };
  fill(bits);
#ifdef PQG_DIAG
  const uint64_t zt1 = __builtin_amdgcn_s_memtime();
  zd.tab += zt1 - zt0;
#endif
  need(tlog[0] + tlog[1] + tlog[2]);
  uint32_t sl = get(tlog[0]), so = get(tlog[1]), sm = get(tlog[2]);
  uint32_t r0 = rep[0], r1 = rep[1], r2 = rep[2], lits = 0;
  // record room for the block's sequences, checked once. The record fields need no check per sequence:
  // literal and match lengths stay below 2^17 (LL code 35: 65536 + 16 extra bits; ML code 52: 65539 +
  // 16 bits; the tables hold valid codes only), and an offset that passes the window check is at most
  // the output so far (< 2^27 + 2^18: jobs of < 2^27 bytes)
  if (cnt + nseq > cap) return false;
  // One sequence = one pass with no data-dependent branch on the common path: the table entries and
  // 20 window bytes at the read position are loaded together; the sequence's bits (offset, match and
  // literal length extras, then the LL / ML / OF state bits: T <= 64 of them, else the inline path
  // takes the job) come out of one 64-bit funnel shift; repeat offsets are selects.
  // re-centring threshold: the window holds stream bits [bits - 160, bits) while bits >= rthr
  // (sb + max(bits - 160, 0) / 8 >= wlo), recomputed when the window moves
  int32_t rthr = wlo > sb ? (int32_t)(wlo - sb) * 8 + 160 : INT32_MIN;
  for (uint32_t i = 0; i < nseq; i++) {
    {  // a sequence reads at most 64 bits below `bits`: re-centre every window of the loop together
      const bool want = bits < rthr;
      if (__ballot(want)) {
        recenter(sb + ((uint32_t)(bits > 0 ? bits : 0) >> 3));
        rthr = wlo > sb ? (int32_t)(wlo - sb) * 8 + 160 : INT32_MIN;
#ifdef PQG_DIAG
        zd.rec++;
#endif
      }
    }
    // every load of the step first (table entries, window bytes), one exit test at the end: an early
    // return per check sinks the loads below it and costs an exec-mask region each
    const uint32_t el = T.e[ZQ_LL + sl], eo = T.e[ZQ_OF + so], em = T.e[ZQ_ML + sm];
    // stream bits [cb, cb + 160) from the window: cb <= bits - 64 < cb + 32
    const int32_t lowbit = bits - 64 > 0 ? bits - 64 : 0;
    const uint32_t a = (sb + ((uint32_t)lowbit >> 3)) & ~3u;
    const int32_t cb = ((int32_t)a - (int32_t)sb) * 8;
    const uint32_t rel = a - wlo;
    const uint32_t d0 = *(const u32a*)(T.win + rel), d1 = *(const u32a*)(T.win + rel + 4),
                   d2 = *(const u32a*)(T.win + rel + 8), d3 = *(const u32a*)(T.win + rel + 12),
                   d4 = *(const u32a*)(T.win + rel + 16);
    bool bad = false;  // (the tables hold valid symbols only: zq_ncount / zq_table check them)
    const uint32_t ofc = (eo >> 13) & 31u, mlb = (em >> 13) & 31u, llb = (el >> 13) & 31u;
    const bool more = i + 1u < nseq;
    const uint32_t nl = more ? (el >> 9) & 15u : 0u, nm = more ? (em >> 9) & 15u : 0u, no = more ? (eo >> 9) & 15u : 0u;
    uint32_t tt = ofc + mlb + llb + nl + nm + no;
    bad |= tt > 64u;
    tt = tt > 64u ? 64u : tt;
    bits -= (int32_t)tt;
    const int32_t off = bits - cb;  // in [0, 96) unless the stream is overrun (bits < 0: failed below)
    const uint32_t ix = (uint32_t)off >> 5, sh = (uint32_t)off & 31u;
    const uint32_t x0 = ix == 0 ? d0 : ix == 1 ? d1 : d2;
    const uint32_t x1 = ix == 0 ? d1 : ix == 1 ? d2 : d3;
    const uint32_t x2 = ix == 0 ? d2 : ix == 1 ? d3 : d4;
    const uint64_t Y = (uint64_t)__builtin_amdgcn_alignbit(x1, x0, sh) |
                       ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32);  // stream bits [bits, bits + 64)
    uint32_t t = tt;
    auto fld = [&](uint32_t k) -> uint32_t {  // the next k <= 31 bits, from the top of Y down
      t -= k;
      return (uint32_t)(Y >> t) & ((1u << k) - 1u);
    };
    const uint32_t ofv = zq_baseline(eo, 0u) + fld(ofc);
    const uint32_t ml = zq_baseline(em, 3u) + fld(mlb);
    const uint32_t ll = zq_baseline(el, 0u) + fld(llb);
    const uint32_t nsl = (el & 0x1FFu) + fld(nl);
    const uint32_t nsm = (em & 0x1FFu) + fld(nm);
    const uint32_t nso = (eo & 0x1FFu) + fld(no);
    // repeat offsets (RFC 8878 3.1.1.5)
    const bool big = ofv > 3u;
    const uint32_t ri = ofv - 1u + (ll == 0u ? 1u : 0u);
    uint32_t roff = r0;  // a chain of selects (nested conditionals compile to exec-mask branches)
    roff = ri == 1u ? r1 : roff;
    roff = ri == 2u ? r2 : roff;
    roff = ri == 3u ? r0 - 1u : roff;
    roff = big ? ofv - 3u : roff;
    const uint32_t n2 = (big || ri >= 2u) ? r1 : r2, n1 = (big || ri >= 1u) ? r0 : r1;
    r2 = n2;
    r1 = n1;
    r0 = roff;
    if (more) {
      sl = nsl;
      sm = nsm;
      so = nso;
    }
    bad |= bits < 0 || lits + ll > regen || roff == 0 || roff > outp + ll - frame0;
    if (bad) return false;
    gst(rec + cnt, (uint64_t)ll | ((uint64_t)ml << 18) | ((uint64_t)roff << 36));
    cnt++;
    lits += ll;
    outp += ll + ml;
  }
#ifdef PQG_DIAG
  zd.loop += __builtin_amdgcn_s_memtime() - zt1;
  zd.seqs += nseq;
#endif
  if (bits != 0) return false;
  rep[0] = r0;
  rep[1] = r1;
  rep[2] = r2;
  outp += regen - lits;
  return true;
}

// The sequence pre-pass of one job (lane): frames and blocks as zstd_job walks them, stopping where
// it stops (the block that reaches the page's size is still decoded whole). Returns ZQ_REPLAY or
// ZQ_INLINE.
__device__ int32_t zq_job(ZqLds& L, ZqLane& T, rsrc_t rs, const pqg_snappy_job& jb, uint64_t* seqs ZQD_ARG) {
  const uint64_t so64 = jb.src_offset, n = jb.src_size;
  if (so64 + n >= 0xFFFFFF00ull || jb.dst_size >= (1u << 27)) return ZQ_INLINE;
  const uint32_t so = (uint32_t)so64, cap = jb.dst_size;
  const uint64_t base = jb.dst_offset / 5u;
  const uint32_t rcap = (uint32_t)((jb.dst_offset + jb.dst_size) / 5u - base);
  uint64_t* rec = seqs + base;
  uint32_t cnt = 0, outp = 0, p = so;
  const uint32_t end = so + (uint32_t)n;
  while (p < end && outp < cap) {
    if (end - p < 4) return ZQ_INLINE;
    const uint32_t magic = ld4_any(rs, p);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      if (end - p < 8) return ZQ_INLINE;
      const uint32_t sz = ld4_any(rs, p + 4);
      if (sz > end - p - 8) return ZQ_INLINE;
      p += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) return ZQ_INLINE;
    p += 4;
    if (p >= end) return ZQ_INLINE;
    const uint32_t fhd = zbyte(rs, p++);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, checksum = (fhd >> 2) & 1u, did_flag = fhd & 3u;
    if (fhd & 8u) return ZQ_INLINE;
    if (!single) p++;
    const uint32_t did_sz = did_flag == 3 ? 4u : did_flag;
    uint32_t did = 0;
    for (uint32_t i = 0; i < did_sz; i++) did |= zbyte(rs, p + i) << (8 * i);
    p += did_sz;
    if (did) return ZQ_INLINE;
    const uint32_t fcs_sz = fcs_flag == 0 ? single : (fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u);
    if (p + fcs_sz > end) return ZQ_INLINE;
    uint64_t fcs = 0;
    for (uint32_t i = 0; i < fcs_sz; i++) fcs |= (uint64_t)zbyte(rs, p + i) << (8 * i);
    if (fcs_sz == 2) fcs += 256;
    p += fcs_sz;
    const uint32_t frame0 = outp;
    uint32_t rep[3] = {1, 4, 8};
    bool have_tab[3] = {false, false, false};
    int tlog[3] = {0, 0, 0};
    bool cut = false;
    while (true) {
      if (outp >= cap) { cut = true; break; }
      if (p + 3 > end) return ZQ_INLINE;
      const uint32_t bh = zbyte(rs, p) | (zbyte(rs, p + 1) << 8) | (zbyte(rs, p + 2) << 16);
      p += 3;
      const uint32_t last = bh & 1u, type = (bh >> 1) & 3u, bs = bh >> 3;
      if (type == 3) return ZQ_INLINE;
      if (type == 1) {
        if (p + 1 > end) return ZQ_INLINE;
        outp += bs;
        p += 1;
      } else if (type == 0) {
        if (p + bs > end) return ZQ_INLINE;
        outp += bs;
        p += bs;
      } else {
        if (p + bs > end || bs < 1) return ZQ_INLINE;
        const uint32_t lim = p + bs, before = outp;
        // literals section header (the literals themselves are k_zstd's)
        const uint32_t b0 = zbyte(rs, p);
        const int lt = (int)(b0 & 3u), sf = (int)((b0 >> 2) & 3u);
        uint32_t regen = 0, comp = 0, hl = 0;
        if (lt <= 1) {
          if (sf == 0 || sf == 2) { regen = b0 >> 3; hl = 1; }
          else if (sf == 1) { regen = (b0 >> 4) + (zbyte(rs, p + 1) << 4); hl = 2; }
          else { regen = (b0 >> 4) + (zbyte(rs, p + 1) << 4) + (zbyte(rs, p + 2) << 12); hl = 3; }
        } else {
          const uint64_t v = ld8_any(rs, p);
          if (sf <= 1) { regen = (uint32_t)(v >> 4) & 0x3FFu; comp = (uint32_t)(v >> 14) & 0x3FFu; hl = 3; }
          else if (sf == 2) { regen = (uint32_t)(v >> 4) & 0x3FFFu; comp = (uint32_t)(v >> 18) & 0x3FFFu; hl = 4; }
          else { regen = (uint32_t)(v >> 4) & 0x3FFFFu; comp = (uint32_t)(v >> 22) & 0x3FFFFu; hl = 5; }
        }
        if (p + hl > lim || regen > ZS_LIT_MAX) return ZQ_INLINE;
        uint32_t q = p + hl;
        const uint32_t lsz = lt == 0 ? regen : lt == 1 ? 1u : comp;
        if (q + lsz > lim) return ZQ_INLINE;
        q += lsz;
        if (!zq_block_seqs(L, T, rs, q, lim, regen, outp, frame0, rep, have_tab, tlog, rec, cnt, rcap ZQD_PASS))
          return ZQ_INLINE;
        if (outp - before > ZS_LIT_MAX) return ZQ_INLINE;
        p += bs;
      }
      if (last) break;
    }
    if (cut) break;
    if ((fcs_flag || single) && (uint64_t)(outp - frame0) != fcs) return ZQ_INLINE;
    if (checksum) {
      if (p + 4 > end) return ZQ_INLINE;
      p += 4;
    }
  }
  return ZQ_REPLAY;
}

__global__ __launch_bounds__(64) void k_zstd_seq(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                                 const pqg_snappy_job* __restrict__ jobs, int n_jobs,
                                                 uint64_t* __restrict__ seqs, int32_t* __restrict__ mode) {
  __shared__ __attribute__((aligned(16))) ZqLds L;
  const uint32_t lane = lane_id();
  for (uint32_t i = lane; i < 53u; i += WAVE) {
    if (i < 36u) {
      L.llcode[i] = ZLL_BASE[i] | (uint32_t)ZLL_BITS[i] << 24;
      L.def_ll[i] = ZLL_DEF[i];
    }
    if (i < 29u) L.def_of[i] = ZOF_DEF[i];
    L.mlcode[i] = ZML_BASE[i] | (uint32_t)ZML_BITS[i] << 24;
    L.def_ml[i] = ZML_DEF[i];
  }
  wave_sync();
  const int j = (int)(blockIdx.x * ZQ_JOBS + lane);
  if (lane >= ZQ_JOBS || j >= n_jobs) return;  // (no cross-lane operation follows)
  const rsrc_t rs = make_rsrc(src, src_bytes);
  const pqg_snappy_job jb = jobs[j];
#ifdef PQG_DIAG
  ZqDiag zd{0, 0, 0, 0, 0};
  const uint64_t zj0 = __builtin_amdgcn_s_memtime();
  mode[j] = zq_job(L, L.l[lane], rs, jb, seqs, zd);
  if (pqg_zqdiag) {
    uint64_t* o = pqg_zqdiag + 6 * (uint64_t)j;
    o[0] = __builtin_amdgcn_s_memtime() - zj0;
    o[1] = zd.tab;
    o[2] = zd.loop;
    o[3] = zd.seqs;
    o[4] = zd.rec;
    o[5] = zd.blocks;
  }
#else
  mode[j] = zq_job(L, L.l[lane], rs, jb, seqs);
#endif
}

// One wave per job: the frames of src[job] -> dst[job] (exactly dst_size bytes kept). The grid is at
// most ZS_GRID waves; wave w takes jobs w, w + grid, ... and owns literal scratch slot w, so the
// scratch is bounded whatever the number of pages.
__device__ __forceinline__ void zstd_job(ZWaveLds& L, const uint8_t* __restrict__ src, uint64_t src_bytes, uint8_t* dst,
                         uint64_t dst_bytes, const pqg_snappy_job& jb, int j, int32_t* status, uint8_t* litbuf,
                         const uint64_t* rec);

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_zstd(const uint8_t* __restrict__ src, uint64_t src_bytes, uint8_t* dst,
                                             uint64_t dst_bytes, const pqg_snappy_job* __restrict__ jobs, int n_jobs,
                                             int32_t* status, uint8_t* scratch, uint64_t lit_stride,
                                             const uint64_t* __restrict__ seqs, const int32_t* __restrict__ mode) {
  __shared__ __attribute__((aligned(16))) ZWaveLds L;
  uint8_t* litbuf = scratch + (uint64_t)blockIdx.x * lit_stride;
  for (uint32_t i = lane_id(); i < 53u; i += WAVE) {
    if (i < 36u) L.llcode[i] = ZLL_BASE[i] | (uint32_t)ZLL_BITS[i] << 24;
    L.mlcode[i] = ZML_BASE[i] | (uint32_t)ZML_BITS[i] << 24;
  }
  wave_sync();
  for (int j = (int)blockIdx.x; j < n_jobs; j += (int)gridDim.x) {
    const pqg_snappy_job jb = jobs[j];
    const bool replay = seqs && (int32_t)uni((uint32_t)mode[j]) == ZQ_REPLAY;
    zstd_job(L, src, src_bytes, dst, dst_bytes, jb, j, status, litbuf, replay ? seqs + jb.dst_offset / 5u : nullptr);
    wave_sync();
  }
}

__device__ __forceinline__ void zstd_job(ZWaveLds& L, const uint8_t* __restrict__ src, uint64_t src_bytes, uint8_t* dst,
                         uint64_t dst_bytes, const pqg_snappy_job& jb, int j, int32_t* status, uint8_t* litbuf,
                         const uint64_t* rec) {
  const rsrc_t rs = make_rsrc(src + jb.src_offset, src_bytes - jb.src_offset);
  if (lane_id() == 0) {
    L.ss.src = (uint64_t)(uintptr_t)(src + jb.src_offset);
    L.ss.src_len = src_bytes - jb.src_offset;
  }
  const uint32_t n = uni(jb.src_size);
#ifdef PQG_DIAG
  for (int i = 0; i < 12; i++) L.diag[i] = 0;
  ZD_T(t_job);
#endif
  ZOut O{dst + jb.dst_offset, uni(jb.dst_size), 0, 0, 0, 0};
  int code = 0;
  uint32_t p = 0, rc = 0;  // rc: replayed sequences so far
  if (jb.dst_offset + jb.dst_size > dst_bytes || jb.src_offset + jb.src_size > src_bytes) code = PQG_ERR_INVALID_ARG;
  while (!code && p < n && O.pos < O.cap) {
    p = uni(p);
    if (n - p < 4) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t magic = ld4_any(rs, p);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (n - p < 8) { code = PQG_ERR_CORRUPT; break; }
      const uint32_t sz = ld4_any(rs, p + 4);
      if (sz > n - p - 8) { code = PQG_ERR_CORRUPT; break; }
      p += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) { code = PQG_ERR_CORRUPT; break; }
    p += 4;
    if (p >= n) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t fhd = zbyte(rs, p++);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, checksum = (fhd >> 2) & 1u, did_flag = fhd & 3u;
    if (fhd & 8u) { code = PQG_ERR_CORRUPT; break; }
    if (!single) p++;  // Window_Descriptor: the whole frame is decoded in place
    const uint32_t did_sz = did_flag == 3 ? 4u : did_flag;
    uint32_t did = 0;
    for (uint32_t i = 0; i < did_sz; i++) did |= zbyte(rs, p + i) << (8 * i);
    p += did_sz;
    if (did) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t fcs_sz = fcs_flag == 0 ? single : (fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u);
    if (p + fcs_sz > n) { code = PQG_ERR_CORRUPT; break; }
    uint64_t fcs = 0;
    for (uint32_t i = 0; i < fcs_sz; i++) fcs |= (uint64_t)zbyte(rs, p + i) << (8 * i);
    if (fcs_sz == 2) fcs += 256;
    p += fcs_sz;
    O.frame0 = O.pos;
    uint32_t rep[3] = {1, 4, 8};
    bool have_huf = false, have_tab[3] = {false, false, false};
    int huf_bits = 0, tlog[3] = {0, 0, 0};
    bool cut = false;
    while (!code) {
      if (O.pos >= O.cap) { cut = true; break; }  // the page reader stops at its size
      if (p + 3 > n) { code = PQG_ERR_CORRUPT; break; }
      const uint32_t bh = zbyte(rs, p) | (zbyte(rs, p + 1) << 8) | (zbyte(rs, p + 2) << 16);
      p += 3;
      const uint32_t last = bh & 1u, type = (bh >> 1) & 3u, bs = bh >> 3;
      if (type == 3) { code = PQG_ERR_CORRUPT; break; }
      if (type == 1) {
        if (p + 1 > n) { code = PQG_ERR_CORRUPT; break; }
        zcopy_lits(O, L, 1, rs, zbyte(rs, p), litbuf, bs);
        p += 1;
      } else if (type == 0) {
        if (p + bs > n) { code = PQG_ERR_CORRUPT; break; }
        zcopy_lits(O, L, 0, rs, p, litbuf, bs);
        p += bs;
      } else {
        if (p + bs > n) { code = PQG_ERR_CORRUPT; break; }
        const uint32_t before = O.pos;
        code = zblock(L, O, rs, p, bs, litbuf, have_huf, huf_bits, have_tab, tlog, rep, rec, rc);
        if (!code && O.pos - before > ZS_LIT_MAX) code = PQG_ERR_CORRUPT;
        p += bs;
      }
      if (last) break;
    }
    if (code || cut) break;
    if ((fcs_flag || single) && (uint64_t)(O.pos - O.frame0) != fcs) { code = PQG_ERR_CORRUPT; break; }
    if (checksum) {
      if (p + 4 > n) { code = PQG_ERR_CORRUPT; break; }
      const uint32_t want = ld4_any(rs, p);
      p += 4;
      if (O.pos <= O.cap) {
        zdrain(O, L);
        const uint32_t got = (uint32_t)zxxh64(O.dst + O.frame0, O.pos - O.frame0);
        if (uni(got) != want) { code = PQG_ERR_CORRUPT; break; }
      }
    }
  }
  zflush(O, L);
#ifdef PQG_DIAG
  L.diag[5] = __builtin_amdgcn_s_memtime() - t_job;
  if (pqg_zdiag && lane_id() < 12) pqg_zdiag[12 * (uint64_t)j + lane_id()] = L.diag[lane_id()];
#endif
  if (!code && O.pos < O.cap) code = PQG_ERR_EOF;  // the frames end before the page's size
  if (lane_id() == 0 && status) status[j] = code;
}

hipError_t launch_zstd(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                       const pqg_snappy_job* jobs, int n_jobs, int32_t* status, uint8_t* scratch, uint64_t* seqs,
                       int32_t* mode) {
  if (n_jobs <= 0) return hipSuccess;
  if (seqs && mode) {
    hipLaunchKernelGGL(k_zstd_seq, dim3((n_jobs + (int)ZQ_JOBS - 1) / (int)ZQ_JOBS), dim3(64), 0, st, src, src_bytes,
                       jobs, n_jobs, seqs, mode);
  } else {
    seqs = nullptr;
    mode = nullptr;
  }
  hipLaunchKernelGGL(k_zstd, dim3(n_jobs < (int)ZSTD_GRID ? n_jobs : (int)ZSTD_GRID), dim3(64), 0, st, src, src_bytes,
                     dst, dst_bytes, jobs, n_jobs, status, scratch, (uint64_t)ZS_LIT_MAX, seqs, mode);
  return hipGetLastError();
}

}  // namespace pqg
