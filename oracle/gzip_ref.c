/* gzip_ref.c — ORACLE (test infrastructure only): GZIP page decompression restated from RFC 1952
 * (gzip member: header, DEFLATE data, CRC-32, ISIZE) and RFC 1951 (DEFLATE: stored, fixed-Huffman and
 * dynamic-Huffman blocks, LZ77 back-references up to 32 KiB).
 *
 * parquet-mr decompresses a GZIP page through Hadoop's GzipCodec (CompressionCodecName.GZIP,
 * parquet-common/.../hadoop/metadata/CompressionCodecName.java:28; CodecFactory.HeapBytesDecompressor,
 * parquet-hadoop/.../hadoop/CodecFactory.java:155-182: codec.createInputStream, then
 * BytesInput.from(is, decompressedSize) reads exactly the header's uncompressed size). Hadoop's
 * GzipCodec / zlib are third-party code absent here; this restatement is pinned to Python's zlib /
 * gzip round trips and to pyarrow-written GZIP parquet files (tests/test_gpu_gzip.py).
 *
 * Semantics kept: concatenated members are read one after the other; reading stops once `expect`
 * bytes are produced (readFully of the page size: neither output beyond it nor the trailer of the
 * member that completes the page is read); a member that ends before the page is complete has its
 * CRC-32 and ISIZE checked before the next member's header; fewer than `expect` bytes -> PQG_ERR_EOF
 * (EOFException); malformed data -> PQG_ERR_CORRUPT (ZipException / IOException).
 *
 * Credit: the inflate part (gz_build's canonical-code construction with its over-subscription /
 * incomplete-code checks, gz_decode's bit-at-a-time canonical decode, the length / distance base and
 * extra-bit tables, the code-length-code order and the dynamic-block header checks) follows the
 * structure of puff.c, Mark Adler's reference inflate in zlib's contrib/puff (Copyright (C) 2002-2013
 * Mark Adler, zlib license). This file is an altered version of that code: restated in this
 * repository's style, with gzip member framing, page-size truncation and this oracle's error codes
 * added. It is the test checker only; nothing in the product uses it. */
#include <stdint.h>
#include <string.h>

#include "pqref.h"

typedef struct {
  const uint8_t* s;
  int64_t n, p;   /* input, size, next byte */
  uint32_t bitbuf;
  int bitcnt;
  int err;
} gz_in;

static uint32_t gz_bits(gz_in* in, int need) {
  uint32_t v = in->bitbuf;
  while (in->bitcnt < need) {
    if (in->p >= in->n) { in->err = PQG_ERR_CORRUPT; return 0; }
    v |= (uint32_t)in->s[in->p++] << in->bitcnt;
    in->bitcnt += 8;
  }
  in->bitbuf = v >> need;
  in->bitcnt -= need;
  return v & ((1u << need) - 1u);
}

typedef struct {
  int16_t count[16];   /* codes per length */
  int16_t symbol[320]; /* symbols in canonical order */
} gz_huff;

/* canonical code from lengths (RFC 1951 3.2.2); 0 ok (incomplete codes allowed only for a single
 * distance code, as zlib accepts), -1 over-subscribed */
static int gz_build(gz_huff* h, const uint8_t* len, int n) {
  int16_t offs[16];
  memset(h->count, 0, sizeof(h->count));
  for (int s = 0; s < n; s++) h->count[len[s]]++;
  if (h->count[0] == n) return 0;
  int left = 1;
  for (int l = 1; l < 16; l++) {
    left <<= 1;
    left -= h->count[l];
    if (left < 0) return -1;
  }
  offs[1] = 0;
  for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + h->count[l];
  for (int s = 0; s < n; s++)
    if (len[s]) h->symbol[offs[len[s]]++] = (int16_t)s;
  return left;
}

static int gz_decode(gz_in* in, const gz_huff* h) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    code |= (int)gz_bits(in, 1);
    if (in->err) return -1;
    const int count = h->count[l];
    if (code - count < first) return h->symbol[index + (code - first)];
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  in->err = PQG_ERR_CORRUPT;
  return -1;
}

static const uint16_t LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                   35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                   1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static uint32_t gz_crc_table[256];
static void gz_crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    gz_crc_table[i] = c;
  }
}

/* one member's DEFLATE stream into dst[op..]; output past `expect` is not kept and stops the decode
 * (*full = 1). Returns 0 or an error; *op advanced. */
static int gz_inflate(gz_in* in, uint8_t* dst, int64_t* opp, int64_t expect, int* full, int64_t member_start) {
  int64_t op = *opp;
  int last;
  do {
    last = (int)gz_bits(in, 1);
    const int type = (int)gz_bits(in, 2);
    if (in->err) return in->err;
    if (type == 0) {  /* stored */
      in->bitbuf = 0;
      in->bitcnt = 0;
      if (in->p + 4 > in->n) return PQG_ERR_CORRUPT;
      const uint32_t len = in->s[in->p] | (in->s[in->p + 1] << 8);
      const uint32_t nlen = in->s[in->p + 2] | (in->s[in->p + 3] << 8);
      in->p += 4;
      if (len != (~nlen & 0xFFFFu)) return PQG_ERR_CORRUPT;
      if (in->p + len > in->n) return PQG_ERR_CORRUPT;
      for (uint32_t i = 0; i < len; i++) {
        if (op >= expect) { *full = 1; *opp = op; return 0; }
        dst[op++] = in->s[in->p + i];
      }
      in->p += len;
      continue;
    }
    gz_huff lit, dist;
    uint8_t lens[320];
    if (type == 1) {
      for (int s = 0; s < 144; s++) lens[s] = 8;
      for (int s = 144; s < 256; s++) lens[s] = 9;
      for (int s = 256; s < 280; s++) lens[s] = 7;
      for (int s = 280; s < 288; s++) lens[s] = 8;
      gz_build(&lit, lens, 288);
      for (int s = 0; s < 30; s++) lens[s] = 5;
      gz_build(&dist, lens, 30);
    } else if (type == 2) {
      static const uint8_t ORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      const int nlen = (int)gz_bits(in, 5) + 257, ndist = (int)gz_bits(in, 5) + 1, ncode = (int)gz_bits(in, 4) + 4;
      if (in->err) return in->err;
      if (nlen > 286 || ndist > 30) return PQG_ERR_CORRUPT;
      uint8_t cl[19] = {0};
      for (int i = 0; i < ncode; i++) cl[ORD[i]] = (uint8_t)gz_bits(in, 3);
      if (in->err) return in->err;
      gz_huff clh;
      if (gz_build(&clh, cl, 19) != 0) return PQG_ERR_CORRUPT;  /* must be complete */
      int idx = 0;
      while (idx < nlen + ndist) {
        int sym = gz_decode(in, &clh);
        if (sym < 0) return PQG_ERR_CORRUPT;
        if (sym < 16) {
          lens[idx++] = (uint8_t)sym;
        } else {
          int rep, val = 0;
          if (sym == 16) {
            if (idx == 0) return PQG_ERR_CORRUPT;
            val = lens[idx - 1];
            rep = 3 + (int)gz_bits(in, 2);
          } else if (sym == 17) {
            rep = 3 + (int)gz_bits(in, 3);
          } else {
            rep = 11 + (int)gz_bits(in, 7);
          }
          if (in->err) return in->err;
          if (idx + rep > nlen + ndist) return PQG_ERR_CORRUPT;
          while (rep--) lens[idx++] = (uint8_t)val;
        }
      }
      if (lens[256] == 0) return PQG_ERR_CORRUPT;  /* no end-of-block code */
      const int e1 = gz_build(&lit, lens, nlen);
      if (e1 < 0 || (e1 > 0 && nlen - lit.count[0] != 1)) return PQG_ERR_CORRUPT;
      const int e2 = gz_build(&dist, lens + nlen, ndist);
      if (e2 < 0 || (e2 > 0 && ndist - dist.count[0] != 1)) return PQG_ERR_CORRUPT;
    } else {
      return PQG_ERR_CORRUPT;
    }
    for (;;) {
      const int sym = gz_decode(in, &lit);
      if (sym < 0) return PQG_ERR_CORRUPT;
      if (sym < 256) {
        if (op >= expect) { *full = 1; *opp = op; return 0; }
        dst[op++] = (uint8_t)sym;
      } else if (sym == 256) {
        break;
      } else {
        const int li = sym - 257;
        if (li >= 29) return PQG_ERR_CORRUPT;
        const int len = LBASE[li] + (int)gz_bits(in, LEXT[li]);
        const int ds = gz_decode(in, &dist);
        if (ds < 0 || ds >= 30) return PQG_ERR_CORRUPT;
        const int64_t d = DBASE[ds] + (int64_t)gz_bits(in, DEXT[ds]);
        if (in->err) return in->err;
        if (d > op - member_start) return PQG_ERR_CORRUPT;  /* before the member's first byte */
        for (int i = 0; i < len; i++) {
          if (op >= expect) { *full = 1; *opp = op; return 0; }
          dst[op] = dst[op - d];
          op++;
        }
      }
    }
  } while (!last);
  *opp = op;
  return 0;
}

int pqr_gzip_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len) {
  if (!gz_crc_table[1]) gz_crc_init();
  gz_in in = {src, n, 0, 0, 0, 0};
  int64_t op = 0;
  while (op < expect) {
    if (in.p >= n) return PQG_ERR_EOF;  /* the stream ends before the page's size */
    /* member header (RFC 1952 2.3) */
    if (in.p + 10 > n) return PQG_ERR_CORRUPT;
    const uint8_t* h = src + in.p;
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || (h[3] & 0xE0)) return PQG_ERR_CORRUPT;
    const uint8_t flg = h[3];
    in.p += 10;
    if (flg & 4) {
      if (in.p + 2 > n) return PQG_ERR_CORRUPT;
      const int64_t xlen = src[in.p] | (src[in.p + 1] << 8);
      in.p += 2 + xlen;
    }
    if (flg & 8) { while (in.p < n && src[in.p]) in.p++; in.p++; }
    if (flg & 16) { while (in.p < n && src[in.p]) in.p++; in.p++; }
    if (flg & 2) in.p += 2;
    if (in.p > n) return PQG_ERR_CORRUPT;
    in.bitbuf = 0;
    in.bitcnt = 0;
    const int64_t start = op;
    int full = 0;
    const int rc = gz_inflate(&in, dst, &op, expect, &full, start);
    if (rc) return rc;
    if (full || op >= expect) break;  /* the page is complete: its reader stops before the trailer */
    /* trailer: CRC-32 and ISIZE of the member */
    if (in.p + 8 > n) return PQG_ERR_CORRUPT;
    uint32_t crc = 0xFFFFFFFFu;
    for (int64_t i = start; i < op; i++) crc = gz_crc_table[(crc ^ dst[i]) & 0xFF] ^ (crc >> 8);
    crc ^= 0xFFFFFFFFu;
    const uint32_t want = src[in.p] | (src[in.p + 1] << 8) | (src[in.p + 2] << 16) | ((uint32_t)src[in.p + 3] << 24);
    const uint32_t isz = src[in.p + 4] | (src[in.p + 5] << 8) | (src[in.p + 6] << 16) | ((uint32_t)src[in.p + 7] << 24);
    if (crc != want || isz != (uint32_t)(op - start)) return PQG_ERR_CORRUPT;
    in.p += 8;
  }
  *out_len = op;
  return 0;
}
