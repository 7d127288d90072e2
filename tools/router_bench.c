/*
 * router_bench.c — the ParquetReadRouter caller loop (Spark's readNextGroup: header, then
 * ParquetReadRouter.read for a bit-packed run, values consumed from currentBuffer at once) timed over
 * a set of hybrid streams, with the router call served three ways:
 *   page     pqg_router_read_page   (GPU: one device round trip per page, later runs from the cache)
 *   run      pqg_router_read        (GPU: one device round trip per run)
 *   cpu      pqr_router_read_batch  (the oracle's restatement of ParquetReadRouter.readBatch, one core;
 *                                    the CPU baseline, not the product)
 * Each mode's decoded values are checked against the cpu mode's before timing.
 *
 * usage: router_bench <case file (tests/c/router_replay.c format)> <reps>
 * prints one JSON line per mode.
 */
#define _POSIX_C_SOURCE 199309L
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pqgpu.h"
#include "../oracle/pqref.h"

typedef struct {
  int32_t w;
  int64_t n;
  uint64_t sec_len, len;
  uint8_t* in;
} stream_t;

enum { M_PAGE = 0, M_RUN = 1, M_CPU = 2 };

static pqg_ctx* g_ctx;
static int32_t* g_buf;

/* one pass of the caller loop over every stream; returns the number of packed reads, -1 on error */
static int64_t replay(const stream_t* ss, int n_streams, int mode, int32_t* vals_out) {
  int64_t calls = 0, at = 0;
  for (int s = 0; s < n_streams; s++) {
    const stream_t* st = &ss[s];
    const uint8_t* in = st->in;
    int64_t got = 0;
    uint64_t pos = 0;
    while (got < st->n) {
      uint32_t hdr = 0, sh = 0, b;
      for (;;) {
        if (pos >= st->sec_len) return -1;
        b = in[pos++];
        if (!(b & 0x80u)) break;
        hdr |= (b & 0x7Fu) << (sh & 31u);
        sh += 7;
      }
      hdr |= b << (sh & 31u);
      if (!(hdr & 1u)) {
        const uint32_t nb = ((uint32_t)st->w + 7u) / 8u;
        uint32_t v = 0;
        for (uint32_t j = 0; j < nb; j++) v |= (uint32_t)in[pos + j] << (8u * j);
        pos += nb;
        int64_t c = (int64_t)(hdr >> 1);
        if (c > st->n - got) c = st->n - got;
        for (int64_t j = 0; j < c; j++) vals_out[at + got + j] = (int32_t)v;
        got += c;
        continue;
      }
      const int32_t count = (int32_t)((hdr >> 1) * 8u);
      int rc = 0;
      if (mode == M_PAGE) rc = pqg_router_read_page(g_ctx, st->w, in + pos, (size_t)(st->len - pos), count, g_buf);
      else if (mode == M_RUN) rc = pqg_router_read(g_ctx, st->w, in + pos, (size_t)(st->len - pos), count, g_buf);
      else rc = pqr_router_read_batch(st->w, in + pos, (int64_t)(st->len - pos), count, g_buf) < 0;
      if (rc) return -1;
      calls++;
      const int64_t c = count < st->n - got ? count : st->n - got;
      memcpy(vals_out + at + got, g_buf, (size_t)c * 4);
      got += c;
      pos += (uint64_t)count * (uint64_t)st->w / 8u;
    }
    at += st->n;
  }
  return calls;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int reps = atoi(argv[2]);
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  char magic[4];
  int32_t n_streams;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "PQGS", 4) || fread(&n_streams, 4, 1, f) != 1 || n_streams <= 0)
    return 2;
  stream_t* ss = calloc((size_t)n_streams, sizeof(stream_t));
  int64_t total = 0, total_bytes = 0;
  for (int s = 0; s < n_streams; s++) {
    stream_t* st = &ss[s];
    if (fread(&st->w, 4, 1, f) != 1 || fread(&st->n, 8, 1, f) != 1 || fread(&st->sec_len, 8, 1, f) != 1 ||
        fread(&st->len, 8, 1, f) != 1)
      return 2;
    st->in = malloc(st->len + 1);
    if (fread(st->in, 1, st->len, f) != st->len) return 2;
    total += st->n;
    total_bytes += (int64_t)st->sec_len;
  }
  fclose(f);
  if (pqg_ctx_create(0, NULL, &g_ctx)) return 3;
  g_buf = malloc(4u << 20);
  int32_t* ref = malloc((size_t)total * 4 + 4);
  int32_t* got = malloc((size_t)total * 4 + 4);
  if (replay(ss, n_streams, M_CPU, ref) < 0) return 4;
  const char* names[3] = {"pqg_router_read_page (GPU, one round trip per page)",
                          "pqg_router_read (GPU, one round trip per run)",
                          "pqr_router_read_batch (oracle readBatch restated, 1 CPU core)"};
  for (int mode = 0; mode < 3; mode++) {
    memset(got, 0, (size_t)total * 4);
    const int64_t calls = replay(ss, n_streams, mode, got);
    if (calls < 0 || memcmp(got, ref, (size_t)total * 4)) {
      printf("{\"mode\": \"%s\", \"error\": \"mismatch\"}\n", names[mode]);
      return 5;
    }
    const int r = mode == M_RUN ? (reps + 9) / 10 : reps;
    uint64_t h0 = 0, m0 = 0, h1 = 0, m1 = 0;
    pqg_router_cache_stats(g_ctx, &h0, &m0);
    const double t0 = now_s();
    for (int k = 0; k < r; k++) replay(ss, n_streams, mode, got);
    const double dt = (now_s() - t0) / r;
    pqg_router_cache_stats(g_ctx, &h1, &m1);
    printf("{\"mode\": \"%s\", \"streams\": %d, \"values\": %" PRId64 ", \"section_bytes\": %" PRId64
           ", \"packed_reads\": %" PRId64 ", \"reps\": %d, \"ms_per_pass\": %.4f, \"values_per_s\": %.4g, "
           "\"us_per_stream\": %.3f, \"device_round_trips_per_pass\": %.1f}\n",
           names[mode], n_streams, total, total_bytes, calls, r, dt * 1e3, (double)total / dt, dt * 1e6 / n_streams,
           mode == M_PAGE ? (double)(m1 - m0) / r : mode == M_RUN ? (double)calls : 0.0);
    fflush(stdout);
  }
  pqg_ctx_destroy(g_ctx);
  return 0;
}
