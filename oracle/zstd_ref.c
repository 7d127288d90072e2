/*
 * zstd_ref.c — ORACLE TEST INFRASTRUCTURE: a plain C restatement of Zstandard decompression, the
 * checker for the GPU codec kernel (parquet-mr_amd/csrc/pqgpu_zstd.hip). Never linked into the
 * product.
 *
 * parquet-mr decompresses a ZSTD page with zstd-jni 1.5.6-2 (third-party, absent here):
 * ZstandardCodec -> ZstdDecompressorStream (parquet-hadoop/src/main/java/org/apache/parquet/hadoop/
 * codec/ZstdDecompressorStream.java:31-46) -> com.github.luben.zstd.ZstdInputStream, i.e. libzstd's
 * streaming decoder, and the page reader takes exactly the header's uncompressed size from it
 * (BytesInput.from(stream, uncompressedSize), ColumnChunkPageReadStore.java:144-172). What is
 * restated is the published format, RFC 8878 (Zstandard Compression and the application/zstd
 * Media Type): frames (and skippable frames) one after another, Raw / RLE / Compressed blocks,
 * literals (raw, RLE, Huffman with 1 or 4 streams, treeless), sequences (predefined / RLE / FSE /
 * repeat tables), repeat offsets, the optional XXH64 content checksum. Parity is pinned on frames
 * produced by libzstd itself (pyarrow's codec, tests/golden/zstd/) and ZSTD parquet files.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pqref.h"

enum { ZR_OK = 0, ZR_CORRUPT = 18, ZR_EOF = 10 };

/* ---- XXH64 (content checksum: low 32 bits of XXH64(content, seed 0)) ---- */
static const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                      P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t xround(uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl64(acc, 31); return acc * P1; }
static uint64_t xmerge(uint64_t acc, uint64_t v) { v = xround(0, v); acc ^= v; return acc * P1 + P4; }

uint64_t pqr_xxh64(const uint8_t* p, uint64_t n, uint64_t seed) {
  const uint8_t* end = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8)); v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + P5;
  }
  h += n;
  while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rotl64(h, 27) * P1 + P4; p += 8; }
  if (p + 4 <= end) { h ^= (uint64_t)rd32(p) * P1; h = rotl64(h, 23) * P2 + P3; p += 4; }
  while (p < end) { h ^= (*p) * P5; h = rotl64(h, 11) * P1; p++; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

/* ---- backward bit stream (RFC 8878 §4.1: read from the end, the last byte's highest set bit is
 * the start marker) ---- */
typedef struct { const uint8_t* p; int64_t n; int64_t bits; } BitB;  /* bits = unread bits left */
static int bitb_init(BitB* b, const uint8_t* p, int64_t n) {
  if (n <= 0 || p[n - 1] == 0) return -1;
  int hb = 7;
  while (!((p[n - 1] >> hb) & 1)) hb--;
  b->p = p; b->n = n; b->bits = (n - 1) * 8 + hb;
  return 0;
}
/* read k bits (k <= 32); past the start they read as 0 (the caller checks overflow) */
static uint32_t bitb_read(BitB* b, int k) {
  uint32_t v = 0;
  for (int i = 0; i < k; i++) {
    b->bits--;
    uint32_t bit = 0;
    if (b->bits >= 0) bit = (b->p[b->bits >> 3] >> (b->bits & 7)) & 1;
    v = (v << 1) | bit;
  }
  return v;
}

/* ---- FSE (RFC 8878 §4.1.1) ---- */
typedef struct { uint8_t sym, nb; uint16_t base; } FseEnt;
typedef struct { int log; FseEnt t[512]; } FseTab;

static int highbit(uint32_t v) { int r = -1; while (v) { v >>= 1; r++; } return r; }

static int fse_build(FseTab* T, const int16_t* norm, int nsym, int log) {
  const int size = 1 << log;
  int high = size - 1;
  uint16_t next[256];
  T->log = log;
  for (int s = 0; s < nsym; s++) {
    if (norm[s] == -1) { T->t[high--].sym = (uint8_t)s; next[s] = 1; }
    else next[s] = (uint16_t)norm[s];
  }
  const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  int pos = 0;
  for (int s = 0; s < nsym; s++)
    for (int i = 0; i < norm[s]; i++) {
      T->t[pos].sym = (uint8_t)s;
      do { pos = (pos + step) & mask; } while (pos > high);
    }
  if (pos != 0) return -1;
  for (int u = 0; u < size; u++) {
    const int s = T->t[u].sym;
    const uint32_t ns = next[s]++;
    const int nb = log - highbit(ns);
    T->t[u].nb = (uint8_t)nb;
    T->t[u].base = (uint16_t)((ns << nb) - size);
  }
  return 0;
}

/* FSE table description (normalized counts) at p (forward little-endian bit reading);
 * returns bytes consumed or -1. */
static int64_t fse_read_ncount(const uint8_t* p, int64_t n, int max_log, int max_sym, int16_t* norm, int* nsym, int* log) {
  int64_t bitpos = 0;
  /* forward little-endian bit reader */
  #define GETB(k, out) do { uint32_t v_ = 0; for (int i_ = 0; i_ < (k); i_++) { int64_t q_ = bitpos + i_; \
      if ((q_ >> 3) >= n) { return -1; } \
      v_ |= (uint32_t)((p[q_ >> 3] >> (q_ & 7)) & 1) << i_; } bitpos += (k); (out) = v_; } while (0)
  uint32_t a;
  GETB(4, a);
  const int accuracy = 5 + (int)a;
  if (accuracy > max_log) return -1;
  *log = accuracy;
  int remaining = (1 << accuracy) + 1, sym = 0;
  while (remaining > 1 && sym <= max_sym) {
    const int nbits = highbit((uint32_t)remaining) + 1;
    const uint32_t maxv = (1u << nbits) - 1 - (uint32_t)remaining;  /* values below: nbits - 1 bits */
    uint32_t v;
    GETB(nbits - 1, v);
    if (v >= maxv) {
      uint32_t hi;
      GETB(1, hi);
      v |= hi << (nbits - 1);
      if (v >= (1u << (nbits - 1))) v -= maxv;
    }
    const int prob = (int)v - 1;
    norm[sym++] = (int16_t)prob;
    remaining -= prob < 0 ? -prob : prob;
    if (prob == 0 && sym <= max_sym) {  /* FSE_readNCount reads repeat flags only while symbols remain */
      uint32_t rep;
      do {
        GETB(2, rep);
        for (uint32_t r = 0; r < rep && sym <= max_sym; r++) norm[sym++] = 0;
      } while (rep == 3);
    }
  }
  #undef GETB
  if (remaining != 1 || sym > max_sym + 1) return -1;
  *nsym = sym;
  return (bitpos + 7) >> 3;
}

static const int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t LL_BASE[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32, 40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t ML_BASE[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29,
                                     30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099,
                                     8195, 16387, 32771, 65539};
static const uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

/* ---- Huffman literals (RFC 8878 §4.2) ---- */
typedef struct { int max_bits; uint8_t sym[2048]; uint8_t nb[2048]; } HufTab;  /* max_bits <= 11 */

static int huf_build(HufTab* H, const uint8_t* w, int nsym) {
  uint32_t total = 0;
  for (int s = 0; s < nsym; s++)
    if (w[s]) total += 1u << (w[s] - 1);
  if (!total) return -1;
  const int max_bits = highbit(total) + 1;
  const uint32_t left = (1u << max_bits) - total;  /* the implied last weight */
  if (left & (left - 1)) return -1;
  uint8_t W[256];
  memcpy(W, w, (size_t)nsym);
  W[nsym] = (uint8_t)(highbit(left) + 1);
  nsym++;
  if (max_bits > 11) return -1;
  H->max_bits = max_bits;
  /* canonical prefix codes: ranks by weight, weight 1 (longest codes) first */
  uint32_t next = 0;
  for (int wt = 1; wt <= max_bits; wt++) {
    const int nb = max_bits + 1 - wt;
    for (int s = 0; s < nsym; s++) {
      if (W[s] != wt) continue;
      const uint32_t len = 1u << (wt - 1);  /* table entries of this code */
      for (uint32_t e = 0; e < len; e++) { H->sym[next + e] = (uint8_t)s; H->nb[next + e] = (uint8_t)nb; }
      next += len;
    }
  }
  return next == (1u << max_bits) ? 0 : -1;
}

/* Huffman tree description at p; returns bytes consumed or -1 */
static int64_t huf_read_tree(HufTab* H, const uint8_t* p, int64_t n) {
  if (n < 1) return -1;
  uint8_t w[256];
  int nsym = 0;
  const uint32_t hdr = p[0];
  int64_t used;
  if (hdr >= 128) {  /* direct: 4-bit weights */
    nsym = (int)hdr - 127;
    const int64_t nb = (nsym + 1) / 2;
    if (1 + nb > n) return -1;
    for (int s = 0; s < nsym; s++) w[s] = (s & 1) ? (p[1 + s / 2] & 15) : (p[1 + s / 2] >> 4);
    used = 1 + nb;
  } else {  /* FSE-compressed weights, two interleaved states */
    const int64_t cs = hdr;
    if (1 + cs > n) return -1;
    int16_t norm[256];
    int ns, log;
    const int64_t hb = fse_read_ncount(p + 1, cs, 6, 255, norm, &ns, &log);
    if (hb < 0) return -1;
    FseTab T;
    if (fse_build(&T, norm, ns, log)) return -1;
    BitB b;
    if (bitb_init(&b, p + 1 + hb, cs - hb)) return -1;
    uint32_t s1 = bitb_read(&b, log), s2 = bitb_read(&b, log);
    for (;;) {
      if (nsym >= 255) return -1;
      w[nsym++] = T.t[s1].sym;
      s1 = T.t[s1].base + bitb_read(&b, T.t[s1].nb);
      if (b.bits < 0) { if (nsym >= 255) return -1; w[nsym++] = T.t[s2].sym; break; }
      if (nsym >= 255) return -1;
      w[nsym++] = T.t[s2].sym;
      s2 = T.t[s2].base + bitb_read(&b, T.t[s2].nb);
      if (b.bits < 0) { if (nsym >= 255) return -1; w[nsym++] = T.t[s1].sym; break; }
    }
    used = 1 + cs;
  }
  for (int s = 0; s < nsym; s++) if (w[s] > 11) return -1;
  return huf_build(H, w, nsym) ? -1 : used;
}

static int huf_stream(const HufTab* H, const uint8_t* p, int64_t n, uint8_t* out, int64_t cnt) {
  BitB b;
  if (bitb_init(&b, p, n)) return -1;
  for (int64_t i = 0; i < cnt; i++) {
    /* peek max_bits (bits past the start read as 0) */
    BitB t = b;
    const uint32_t v = bitb_read(&t, H->max_bits);
    out[i] = H->sym[v];
    b.bits -= H->nb[v];
    if (b.bits < 0) return -1;
  }
  return b.bits == 0 ? 0 : -1;  /* the stream is consumed exactly */
}

/* ---- frame decoding ---- */
typedef struct {
  uint8_t* dst;
  int64_t cap, pos;        /* output written so far (bytes past cap are dropped, not an error) */
  int64_t frame_start;     /* output position where the current frame began */
  HufTab huf;
  int have_huf;
  FseTab ll, of, ml;
  int have_ll, have_of, have_ml;
  uint32_t rep[3];
  uint8_t lit[131072];
} ZState;

static void out_byte(ZState* Z, uint8_t v) {
  if (Z->pos < Z->cap) Z->dst[Z->pos] = v;
  Z->pos++;
}

static int seq_table(FseTab* T, int* have, int mode, const uint8_t* p, int64_t n, int64_t* used, const int16_t* def,
                     int def_n, int def_log, int max_log, int max_sym) {
  *used = 0;
  switch (mode) {
    case 0: fse_build(T, def, def_n, def_log); *have = 1; return 0;
    case 1:
      if (n < 1 || p[0] > max_sym) return -1;
      T->log = 0; T->t[0].sym = p[0]; T->t[0].nb = 0; T->t[0].base = 0;
      *used = 1; *have = 1; return 0;
    case 2: {
      int16_t norm[64];
      int ns, log;
      const int64_t u = fse_read_ncount(p, n, max_log, max_sym, norm, &ns, &log);
      if (u < 0 || fse_build(T, norm, ns, log)) return -1;
      *used = u; *have = 1; return 0;
    }
    default: return *have ? 0 : -1;
  }
}

static int block_compressed(ZState* Z, const uint8_t* p, int64_t n, int64_t window_bytes) {
  (void)window_bytes;
  if (n < 1) return -1;
  /* literals section */
  const int lt = p[0] & 3, sf = (p[0] >> 2) & 3;
  int64_t regen, comp = 0, hl;
  if (lt <= 1) {
    if (sf == 0 || sf == 2) { regen = p[0] >> 3; hl = 1; }
    else if (sf == 1) { if (n < 2) return -1; regen = (p[0] >> 4) + ((int64_t)p[1] << 4); hl = 2; }
    else { if (n < 3) return -1; regen = (p[0] >> 4) + ((int64_t)p[1] << 4) + ((int64_t)p[2] << 12); hl = 3; }
  } else {
    if (sf <= 1) { if (n < 3) return -1; uint32_t v = p[0] | (p[1] << 8) | ((uint32_t)p[2] << 16); regen = (v >> 4) & 0x3FF; comp = (v >> 14) & 0x3FF; hl = 3; }
    else if (sf == 2) { if (n < 4) return -1; uint32_t v = rd32(p); regen = (v >> 4) & 0x3FFF; comp = (v >> 18) & 0x3FFF; hl = 4; }
    else { if (n < 5) return -1; uint64_t v = rd32(p) | ((uint64_t)p[4] << 32); regen = (v >> 4) & 0x3FFFF; comp = (v >> 22) & 0x3FFFF; hl = 5; }
  }
  if (regen > 131072) return -1;
  int64_t q = hl;
  if (lt == 0) {
    if (q + regen > n) return -1;
    memcpy(Z->lit, p + q, (size_t)regen);
    q += regen;
  } else if (lt == 1) {
    if (q + 1 > n) return -1;
    memset(Z->lit, p[q], (size_t)regen);
    q += 1;
  } else {
    if (q + comp > n) return -1;
    const uint8_t* c = p + q;
    int64_t cn = comp;
    if (lt == 2) {
      const int64_t u = huf_read_tree(&Z->huf, c, cn);
      if (u < 0) return -1;
      Z->have_huf = 1;
      c += u; cn -= u;
    } else if (!Z->have_huf) {
      return -1;
    }
    if (sf == 0) {
      if (huf_stream(&Z->huf, c, cn, Z->lit, regen)) return -1;
    } else {
      if (cn < 6) return -1;
      const int64_t s1 = c[0] | (c[1] << 8), s2 = c[2] | (c[3] << 8), s3 = c[4] | (c[5] << 8);
      const int64_t s4 = cn - 6 - s1 - s2 - s3;
      if (s4 < 0) return -1;
      const int64_t seg = (regen + 3) / 4, last = regen - 3 * seg;
      if (last < 0) return -1;
      const uint8_t* d = c + 6;
      if (huf_stream(&Z->huf, d, s1, Z->lit, seg) || huf_stream(&Z->huf, d + s1, s2, Z->lit + seg, seg) ||
          huf_stream(&Z->huf, d + s1 + s2, s3, Z->lit + 2 * seg, seg) ||
          huf_stream(&Z->huf, d + s1 + s2 + s3, s4, Z->lit + 3 * seg, last))
        return -1;
    }
    q += comp;
  }
  /* sequences section */
  if (q >= n) return -1;
  int64_t nseq = p[q];
  if (nseq == 0) {
    q += 1;
    for (int64_t i = 0; i < regen; i++) out_byte(Z, Z->lit[i]);
    return q == n ? 0 : -1;
  }
  if (nseq < 128) { q += 1; }
  else if (nseq < 255) { if (q + 2 > n) return -1; nseq = ((nseq - 128) << 8) + p[q + 1]; q += 2; }
  else { if (q + 3 > n) return -1; nseq = p[q + 1] + ((int64_t)p[q + 2] << 8) + 0x7F00; q += 3; }
  if (q >= n) return -1;
  const uint8_t modes = p[q++];
  if (modes & 3) return -1;
  int64_t u;
  if (seq_table(&Z->ll, &Z->have_ll, modes >> 6, p + q, n - q, &u, LL_DEF, 36, 6, 9, 35)) return -1;
  q += u;
  if (seq_table(&Z->of, &Z->have_of, (modes >> 4) & 3, p + q, n - q, &u, OF_DEF, 29, 5, 8, 31)) return -1;
  q += u;
  if (seq_table(&Z->ml, &Z->have_ml, (modes >> 2) & 3, p + q, n - q, &u, ML_DEF, 53, 6, 9, 52)) return -1;
  q += u;
  BitB b;
  if (bitb_init(&b, p + q, n - q)) return -1;
  uint32_t sl = bitb_read(&b, Z->ll.log), so = bitb_read(&b, Z->of.log), sm = bitb_read(&b, Z->ml.log);
  int64_t lit_pos = 0;
  for (int64_t i = 0; i < nseq; i++) {
    const int llc = Z->ll.t[sl].sym, ofc = Z->of.t[so].sym, mlc = Z->ml.t[sm].sym;
    if (llc > 35 || mlc > 52 || ofc > 31) return -1;
    uint64_t ofv = ((uint64_t)1 << ofc) + (ofc ? bitb_read(&b, ofc > 32 ? 32 : ofc) : 0);
    const uint32_t ml = ML_BASE[mlc] + (ML_BITS[mlc] ? bitb_read(&b, ML_BITS[mlc]) : 0);
    const uint32_t ll = LL_BASE[llc] + (LL_BITS[llc] ? bitb_read(&b, LL_BITS[llc]) : 0);
    /* repeat offsets (RFC 8878 §3.1.1.5) */
    uint32_t off;
    if (ofv > 3) {
      off = (uint32_t)(ofv - 3);
      Z->rep[2] = Z->rep[1]; Z->rep[1] = Z->rep[0]; Z->rep[0] = off;
    } else {
      uint32_t idx = (uint32_t)ofv - 1;  /* 0..2 */
      if (ll == 0) idx++;                /* shifted by one when the literal length is 0 */
      if (idx == 0) {
        off = Z->rep[0];
      } else if (idx == 3) {
        off = Z->rep[0] - 1;
        if (off == 0) return -1;
        Z->rep[2] = Z->rep[1]; Z->rep[1] = Z->rep[0]; Z->rep[0] = off;
      } else {
        off = Z->rep[idx];
        if (idx == 2) Z->rep[2] = Z->rep[1];
        Z->rep[1] = Z->rep[0];
        Z->rep[0] = off;
      }
    }
    if (i + 1 < nseq) {
      sl = Z->ll.t[sl].base + bitb_read(&b, Z->ll.t[sl].nb);
      sm = Z->ml.t[sm].base + bitb_read(&b, Z->ml.t[sm].nb);
      so = Z->of.t[so].base + bitb_read(&b, Z->of.t[so].nb);
    }
    if (b.bits < 0) return -1;
    if (lit_pos + ll > regen) return -1;
    for (uint32_t k = 0; k < ll; k++) out_byte(Z, Z->lit[lit_pos + k]);
    lit_pos += ll;
    if (off == 0 || (int64_t)off > Z->pos - Z->frame_start) return -1;  /* before the frame's start (no dictionary) */
    for (uint32_t k = 0; k < ml; k++) {
      const int64_t s = Z->pos - off;
      out_byte(Z, s < Z->cap ? Z->dst[s] : 0);
    }
  }
  if (b.bits != 0) return -1;
  for (int64_t k = lit_pos; k < regen; k++) out_byte(Z, Z->lit[k]);
  return 0;
}

/* Decompress the concatenated frames in src[0, n) into dst[0, expect): ZR_OK when at least
 * `expect` bytes were produced (the page reader takes exactly that many), *out_len = bytes
 * produced. Errors: ZR_CORRUPT (malformed / checksum), ZR_EOF (frames end before `expect`). */
static int zstd_frames(ZState* Z, const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len);

int pqr_zstd_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len) {
  ZState* Z = (ZState*)malloc(sizeof(ZState));
  if (!Z) return ZR_CORRUPT;
  const int rc = zstd_frames(Z, src, n, dst, expect, out_len);
  free(Z);
  return rc;
}

static int zstd_frames(ZState* Z, const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len) {
  Z->dst = dst; Z->cap = expect; Z->pos = 0;
  int64_t p = 0;
  *out_len = 0;
  while (p < n && Z->pos < expect) {
    if (n - p < 4) return ZR_CORRUPT;
    const uint32_t magic = rd32(src + p);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  /* skippable frame */
      if (n - p < 8) return ZR_CORRUPT;
      const uint32_t sz = rd32(src + p + 4);
      if ((uint64_t)sz > (uint64_t)(n - p - 8)) return ZR_CORRUPT;
      p += 8 + (int64_t)sz;
      continue;
    }
    if (magic != 0xFD2FB528u) return ZR_CORRUPT;
    p += 4;
    if (p >= n) return ZR_CORRUPT;
    const uint8_t fhd = src[p++];
    const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (fhd & 8) return ZR_CORRUPT;  /* reserved bit */
    int64_t window = 0;  /* Window_Size (not needed to decode a whole frame in memory) */
    if (!single) {
      if (p >= n) return ZR_CORRUPT;
      const uint8_t wd = src[p++];
      const int exp = wd >> 3, mant = wd & 7;
      const uint64_t base = 1ull << (10 + exp);
      window = (int64_t)(base + (base / 8) * (uint64_t)mant);
    }
    const int did_sz[4] = {0, 1, 2, 4};
    if (p + did_sz[did_flag] > n) return ZR_CORRUPT;
    uint32_t did = 0;
    for (int i = 0; i < did_sz[did_flag]; i++) did |= (uint32_t)src[p + i] << (8 * i);
    p += did_sz[did_flag];
    if (did) return ZR_CORRUPT;  /* a dictionary: parquet pages never use one, none is available */
    const int fcs_sz = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
    if (p + fcs_sz > n) return ZR_CORRUPT;
    uint64_t fcs = 0;
    for (int i = 0; i < fcs_sz; i++) fcs |= (uint64_t)src[p + i] << (8 * i);
    if (fcs_sz == 2) fcs += 256;
    p += fcs_sz;
    if (single) window = (int64_t)fcs;
    const int64_t frame_start = Z->pos;
    Z->frame_start = frame_start;
    Z->rep[0] = 1; Z->rep[1] = 4; Z->rep[2] = 8;
    Z->have_huf = Z->have_ll = Z->have_of = Z->have_ml = 0;
    for (;;) {
      /* the page reader stops after `expect` bytes: later blocks are never decoded */
      if (Z->pos >= Z->cap) { *out_len = Z->pos; return ZR_OK; }
      if (p + 3 > n) return ZR_CORRUPT;
      const uint32_t bh = src[p] | (src[p + 1] << 8) | ((uint32_t)src[p + 2] << 16);
      p += 3;
      const int last = bh & 1, type = (bh >> 1) & 3;
      const int64_t bs = bh >> 3;
      if (type == 3) return ZR_CORRUPT;
      if (type == 1) {
        if (p + 1 > n) return ZR_CORRUPT;
        for (int64_t k = 0; k < bs; k++) out_byte(Z, src[p]);
        p += 1;
      } else {
        if (p + bs > n) return ZR_CORRUPT;
        if (type == 0) {
          for (int64_t k = 0; k < bs; k++) out_byte(Z, src[p + k]);
        } else {
          const int64_t before = Z->pos;
          if (block_compressed(Z, src + p, bs, window)) return ZR_CORRUPT;
          if (Z->pos - before > 131072) return ZR_CORRUPT;
        }
        p += bs;
      }
      if (last) break;
    }
    if (fcs_flag || single) {
      if ((uint64_t)(Z->pos - frame_start) != fcs) return ZR_CORRUPT;
    }
    if (checksum) {
      if (p + 4 > n) return ZR_CORRUPT;
      const uint32_t want = rd32(src + p);
      p += 4;
      if (Z->pos <= Z->cap) {  /* a frame cut by the page size is not checked (deviation) */
        const uint32_t got = (uint32_t)pqr_xxh64(dst + frame_start, (uint64_t)(Z->pos - frame_start), 0);
        if (got != want) return ZR_CORRUPT;
      }
    }
  }
  *out_len = Z->pos;
  return Z->pos >= expect ? ZR_OK : ZR_EOF;
}
