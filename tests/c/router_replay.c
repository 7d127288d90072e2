/*
 * router_replay.c — a Spark-style caller loop over ParquetReadRouter, driven through the C ABI.
 *
 * Spark's VectorizedRleValuesReader.readNextGroup reads a run header, and for a bit-packed run calls
 * ParquetReadRouter.read(bitWidth, in, currentCount, currentBuffer) and consumes currentBuffer right
 * after the call returns (ParquetReadRouter.java:57-66: the values are there on return). This driver
 * does the same with pqg_router_read_page, one reused buffer per stream, and records every packed
 * read's values the moment the call returns, before the next call may overwrite the buffer.
 *
 * usage: router_replay <case file> <out file> [tail]
 *   case file: "PQGS" | i32 n_streams | per stream: i32 bit_width | i64 n_values | u64 section_len |
 *              u64 stream_len | stream bytes [stream_len]
 *              (the hybrid section is the first section_len bytes; the caller's stream may run past it:
 *              stream_left is measured to stream_len, as a reader whose stream is the rest of the page)
 *   out file:  per packed read, the values of that read (int32), back to back; per stream, the
 *              decoded values (int32) after the packed reads of all streams
 * prints: CALL <stream> <position> <count> per packed read, then STREAM <i> <code> <n decoded>,
 *         then STATS <hits> <misses>
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pqgpu.h"
#include "pqgpu_reader.h"

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  char magic[4];
  int32_t n_streams;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "PQGS", 4) || fread(&n_streams, 4, 1, f) != 1 || n_streams < 0)
    return 2;
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;
  pqg_ctx* ctx = NULL;
  int rc = pqg_ctx_create(0, NULL, &ctx);
  if (rc) {
    printf("CTX_ERROR %d\n", rc);
    return 0;
  }
  int32_t** decoded = calloc((size_t)n_streams + 1, sizeof(int32_t*));
  int64_t* n_dec = calloc((size_t)n_streams + 1, sizeof(int64_t));
  int* codes = calloc((size_t)n_streams + 1, sizeof(int));
  for (int s = 0; s < n_streams; s++) {
    int32_t w;
    int64_t n;
    uint64_t sec_len, len;
    if (fread(&w, 4, 1, f) != 1 || fread(&n, 8, 1, f) != 1 || fread(&sec_len, 8, 1, f) != 1 ||
        fread(&len, 8, 1, f) != 1 || n < 0 || sec_len > len)
      return 2;
    uint8_t* in = malloc(len + 1);
    if (!in || fread(in, 1, len, f) != len) return 2;
    int32_t* vals = calloc((size_t)n + 1, 4);
    int32_t* buf = NULL; /* currentBuffer, grown as Spark grows it */
    int64_t cap = 0, got = 0;
    uint64_t pos = 0;
    int code = 0;
    while (got < n) {
      /* readNextGroup: BytesUtils.readUnsignedVarInt */
      uint32_t hdr = 0, sh = 0, b;
      for (;;) {
        if (pos >= sec_len) { code = PQG_ERR_EOF; break; }
        b = in[pos++];
        if (!(b & 0x80u)) break;
        hdr |= (b & 0x7Fu) << (sh & 31u);
        sh += 7;
      }
      if (code) break;
      hdr |= b << (sh & 31u);
      if (!(hdr & 1u)) { /* RLE: count, readIntLittleEndianPaddedOnBitWidth */
        const uint32_t nb = ((uint32_t)w + 7u) / 8u;
        uint32_t v = 0;
        for (uint32_t j = 0; j < nb; j++) v |= (pos + j < sec_len ? (uint32_t)in[pos + j] : 0u) << (8u * j);
        pos += nb;
        int64_t c = (int64_t)(hdr >> 1);
        if (c > n - got) c = n - got;
        for (int64_t j = 0; j < c; j++) vals[got + j] = (int32_t)v;
        got += c;
        continue;
      }
      const int32_t count = (int32_t)((hdr >> 1) * 8u);
      if (count > cap) {
        free(buf);
        cap = count;
        buf = malloc((size_t)cap * 4 + 4);
      }
      /* ParquetReadRouter.read(bitWidth, in, currentCount, currentBuffer): stream at pos, len - pos left */
      rc = pqg_router_read_page(ctx, w, in + pos, (size_t)(len - pos), count, buf);
      if (rc) { code = rc; break; }
      /* consume currentBuffer now: record it and take the values the page still needs */
      printf("CALL %d %" PRIu64 " %d\n", s, pos, count);
      if (count && fwrite(buf, 4, (size_t)count, o) != (size_t)count) return 2;
      int64_t c = count < n - got ? count : n - got;
      memcpy(vals + got, buf, (size_t)c * 4);
      got += c;
      pos += (uint64_t)count * (uint64_t)w / 8u;
      /* the buffer is the caller's: scribble over it, as the next group's decode would */
      memset(buf, 0xA5, (size_t)count * 4);
    }
    decoded[s] = vals;
    n_dec[s] = got;
    codes[s] = code;
    free(buf);
    free(in);
  }
  fclose(f);
  for (int s = 0; s < n_streams; s++) {
    printf("STREAM %d %d %" PRId64 "\n", s, codes[s], n_dec[s]);
    if (n_dec[s] && fwrite(decoded[s], 4, (size_t)n_dec[s], o) != (size_t)n_dec[s]) return 2;
    free(decoded[s]);
  }
  fclose(o);
  uint64_t hits = 0, misses = 0;
  pqg_router_cache_stats(ctx, &hits, &misses);
  printf("STATS %" PRIu64 " %" PRIu64 "\n", hits, misses);
  pqg_ctx_destroy(ctx);
  free(decoded);
  free(n_dec);
  free(codes);
  return 0;
}
