/*
 * router.c — C driver of the batched ParquetReadRouter entry (pqg_router_read_runs), the call the
 * JNI shim's PqGpu.routerReadBatch makes for a page's bit-packed runs.
 *
 * usage: router <case file> <out file>
 *   case file: "PQGR" | i32 bit_width | i32 n_runs | u64 in_len | u64 in_offsets[n_runs] |
 *              u32 counts[n_runs] | in bytes            (written by tests/test_c_harness.py)
 *   out file:  the int32 values of all runs back to back
 * prints: ROUTER <code> <exception|-> <n values>
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
  int32_t bw, n;
  uint64_t in_len;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "PQGR", 4) || fread(&bw, 4, 1, f) != 1 || fread(&n, 4, 1, f) != 1 ||
      fread(&in_len, 8, 1, f) != 1 || n < 0)
    return 2;
  uint64_t* offs = calloc((size_t)n + 1, 8);
  uint32_t* counts = calloc((size_t)n + 1, 4);
  uint8_t* in = malloc(in_len + 1);
  if ((n && (fread(offs, 8, (size_t)n, f) != (size_t)n || fread(counts, 4, (size_t)n, f) != (size_t)n)) ||
      fread(in, 1, in_len, f) != in_len)
    return 2;
  fclose(f);
  uint64_t total = 0;
  for (int r = 0; r < n; r++) total += counts[r];
  int32_t* out = calloc((size_t)total + 1, 4);
  pqg_ctx* ctx = NULL;
  int rc = pqg_ctx_create(0, NULL, &ctx);
  if (!rc) rc = pqg_router_read_runs(ctx, bw, in, (size_t)in_len, offs, counts, n, out);
  const char* e = pqg_java_exception(rc);
  printf("ROUTER %d %s %" PRIu64 "\n", rc, e ? e : "-", total);
  FILE* o = fopen(argv[2], "wb");
  if (!o || fwrite(out, 4, (size_t)total, o) != (size_t)total) return 2;
  fclose(o);
  if (ctx) pqg_ctx_destroy(ctx);
  return 0;
}
