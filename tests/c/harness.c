/*
 * harness.c — C driver of the drop-in boundary, the way the JNI shim drives it (no ctypes):
 * raw column-chunk bytes -> pqg_frame_chunk (CRC verified) -> pqg_pages_from_headers ->
 * pqg_decode_host -> one pqg_values_reader per page (initFromPage, readX / skip(n)), with every
 * failure mapped to the Java exception class the shim throws (pqg_java_exception).
 *
 * usage: harness <case file> <mode>
 *   case file: "PQGC" | i32 physical_type, type_length, max_def, max_rep, flags, codec | i64 num_values |
 *              u64 chunk_len | chunk bytes            (written by tests/test_c_harness.py)
 *   mode:      all   read every value of every page with the column type's read call
 *              skip  per page: skip(3), read 2, repeated (ValuesReader.skip(int n))
 * output, one line each:
 *   FRAME <n headers> | FRAME_ERROR <code> <exception> <page>
 *   CTX_ERROR <code> <exception>
 *   DECODE <code> <exception|-> <page> <value_index>
 *   PAGE <p> <n values> | PAGE <p> INIT_ERROR <code> <exception>
 *   V <page> <index in page> <value>        (ints decimal, float / double bit patterns hex, bytes hex)
 *   END <page> <code> <exception>            (the read that ended the page: EOF past the last value)
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pqgpu.h"
#include "pqgpu_reader.h"

static const char* exc(int code) {
  const char* e = pqg_java_exception(code);
  return e ? e : "-";
}

static void print_bytes(const uint8_t* d, uint32_t n) {
  if (n == 0) printf("-");
  for (uint32_t i = 0; i < n; i++) printf("%02x", d[i]);
}

/* one read of the column's type; 0 and a printed value, or the error code */
static int read_one(pqg_values_reader* r, int page, uint64_t k) {
  int rc;
  if (r->ids) {
    int32_t v;
    if ((rc = pqg_vr_read_dictionary_id(r, &v))) return rc;
    printf("V %d %" PRIu64 " %d\n", page, k, v);
    return 0;
  }
  switch (r->physical_type) {
    case PQG_BOOLEAN: {
      int32_t v;
      if ((rc = pqg_vr_read_boolean(r, &v))) return rc;
      printf("V %d %" PRIu64 " %d\n", page, k, v);
      return 0;
    }
    case PQG_INT32: {
      int32_t v;
      if ((rc = pqg_vr_read_integer(r, &v))) return rc;
      printf("V %d %" PRIu64 " %d\n", page, k, v);
      return 0;
    }
    case PQG_INT64: {
      int64_t v;
      if ((rc = pqg_vr_read_long(r, &v))) return rc;
      printf("V %d %" PRIu64 " %" PRId64 "\n", page, k, v);
      return 0;
    }
    case PQG_FLOAT: {
      float v;
      uint32_t b;
      if ((rc = pqg_vr_read_float(r, &v))) return rc;
      memcpy(&b, &v, 4);
      printf("V %d %" PRIu64 " %08x\n", page, k, b);
      return 0;
    }
    case PQG_DOUBLE: {
      double v;
      uint64_t b;
      if ((rc = pqg_vr_read_double(r, &v))) return rc;
      memcpy(&b, &v, 8);
      printf("V %d %" PRIu64 " %016" PRIx64 "\n", page, k, b);
      return 0;
    }
    default: {
      const uint8_t* d;
      uint32_t n;
      if ((rc = pqg_vr_read_bytes(r, &d, &n))) return rc;
      printf("V %d %" PRIu64 " ", page, k);
      print_bytes(d, n);
      printf("\n");
      return 0;
    }
  }
}

/* a read call of another type must be refused (UnsupportedOperationException) */
static int wrong_type_refused(pqg_values_reader* r) {
  int32_t i32;
  int64_t i64;
  if (r->ids) return pqg_vr_read_long(r, &i64) == PQG_ERR_UNSUPPORTED;
  if (r->physical_type == PQG_INT32) return pqg_vr_read_long(r, &i64) == PQG_ERR_UNSUPPORTED;
  return pqg_vr_read_integer(r, &i32) == PQG_ERR_UNSUPPORTED && pqg_vr_read_dictionary_id(r, &i32) == PQG_ERR_UNSUPPORTED;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <case file> all|skip\n", argv[0]);
    return 2;
  }
  const int skip_mode = strcmp(argv[2], "skip") == 0;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  char magic[4];
  int32_t hdr[6];
  int64_t num_values;
  uint64_t chunk_len;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "PQGC", 4) || fread(hdr, 4, 6, f) != 6 ||
      fread(&num_values, 8, 1, f) != 1 || fread(&chunk_len, 8, 1, f) != 1)
    return 2;
  const uint64_t pad = 1024;
  uint8_t* chunk = calloc(chunk_len + pad, 1);
  if (!chunk || fread(chunk, 1, chunk_len, f) != chunk_len) return 2;
  fclose(f);

  /* ParquetFileReader.Chunk.readAllPages: headers, CRC */
  pqg_status st;
  int n_hdr = 0;
  pqg_page_header* hdrs = calloc(4096, sizeof(pqg_page_header));
  int rc = pqg_frame_chunk(chunk, chunk_len, num_values, 1, hdrs, 4096, &n_hdr, &st);
  if (rc) {
    printf("FRAME_ERROR %d %s %d\n", rc, exc(rc), st.page);
    return 0;
  }
  printf("FRAME %d\n", n_hdr);
  pqg_column_desc col;
  memset(&col, 0, sizeof(col));
  col.physical_type = hdr[0];
  col.type_length = hdr[1];
  col.max_def = hdr[2];
  col.max_rep = hdr[3];
  col.flags = hdr[4];
  col.dict_offset = -1;
  pqg_page_desc* pages = calloc((size_t)n_hdr + 1, sizeof(pqg_page_desc));
  int n_pages = 0;
  /* the chunk's ColumnMetaData.codec decides which pages are compressed (ColumnChunkPageReadStore) */
  rc = pqg_pages_from_headers(hdrs, n_hdr, hdr[5], 0, 0, &col, pages, n_hdr + 1, &n_pages, &st);
  if (rc) {
    printf("FRAME_ERROR %d %s %d\n", rc, exc(rc), st.page);
    return 0;
  }

  pqg_ctx* ctx = NULL;
  rc = pqg_ctx_create(0, NULL, &ctx);
  if (rc) {
    printf("CTX_ERROR %d %s\n", rc, exc(rc));
    return 0;
  }
  uint64_t slots = 0;
  for (int p = 0; p < n_pages; p++) slots += pages[p].num_values;
  const int bin = col.physical_type == PQG_BYTE_ARRAY && !(col.flags & PQG_COLUMN_DICTIONARY_IDS);
  int w = 16;  /* >= every element width (INT96 12; FLBA up to type_length) */
  if (col.physical_type == PQG_FIXED_LEN_BYTE_ARRAY && col.type_length > w) w = col.type_length;
  col.values = calloc(slots + 1, (size_t)w);
  col.values_capacity = slots + (bin ? 1 : 0);
  uint8_t* dl = calloc(slots + 1, 1);
  uint8_t* rl = calloc(slots + 1, 1);
  col.def_levels = col.max_def > 0 ? dl : NULL;
  col.rep_levels = col.max_rep > 0 ? rl : NULL;
  col.levels_capacity = slots;
  uint64_t bcap = bin ? chunk_len + 64 : 0;
  col.binary_data = bin ? malloc(bcap) : NULL;
  col.binary_capacity = bcap;
  uint32_t* counts = calloc((size_t)n_pages + 1, sizeof(uint32_t));
  rc = pqg_decode_host(ctx, chunk, chunk_len, &col, 1, pages, n_pages, counts, &st);
  if (rc == PQG_ERR_INVALID_ARG && st.page == -1 && strncmp(st.message, "binary capacity", 15) == 0) {
    /* the dictionary values expand past the first estimate: allocate what the library reports */
    bcap = (uint64_t)st.value_index + 64;
    free(col.binary_data);
    col.binary_data = malloc(bcap);
    col.binary_capacity = bcap;
    rc = pqg_decode_host(ctx, chunk, chunk_len, &col, 1, pages, n_pages, counts, &st);
  }
  printf("DECODE %d %s %d %" PRId64 "\n", rc, exc(rc), rc ? st.page : -1, rc ? st.value_index : (int64_t)-1);

  int refused_ok = 1;
  for (int p = 0; p < n_pages; p++) {
    pqg_values_reader r;
    const int irc = pqg_vr_init_from_page(&r, &col, pages, counts, n_pages, p, rc, &st);
    if (irc) {
      printf("PAGE %d INIT_ERROR %d %s\n", p, irc, exc(irc));
      continue;
    }
    printf("PAGE %d %" PRIu64 "\n", p, pqg_vr_remaining(&r));
    if (pqg_vr_remaining(&r) && !wrong_type_refused(&r)) refused_ok = 0;
    uint64_t k = 0;
    int e = 0;
    while (!e) {
      if (skip_mode) {
        e = pqg_vr_skip_n(&r, 3);
        if (e) break;
        k += 3;
        for (int j = 0; j < 2 && !e; j++) e = read_one(&r, p, k++);
      } else {
        e = read_one(&r, p, k++);
      }
    }
    printf("END %d %d %s\n", p, e, exc(e));
  }
  printf("REFUSED_WRONG_TYPE %d\n", refused_ok);
  pqg_ctx_destroy(ctx);
  return 0;
}
