/*
 * harness.c — C driver of the drop-in boundary, the way the JNI shim drives it (no ctypes):
 * raw column-chunk bytes -> pqg_frame_chunk (CRC verified) -> pqg_pages_from_headers ->
 * pqg_decode_host or the staged path (pqg_host_input / pqg_decode_staged / pqg_staged_column,
 * what shim/jni/pqgpu_jni.c calls) -> per page the level readers (pqg_lr_*) and the values reader
 * (pqg_vr_*), every failure mapped to the Java exception class the shim throws
 * (pqg_java_exception).
 *
 * usage: harness <case file> <mode> [<case file> ...]
 *   case file: "PQGC" | i32 physical_type, type_length, max_def, max_rep, flags, codec | i64 num_values |
 *              u64 chunk_len | chunk bytes            (written by tests/test_c_harness.py)
 *              Several case files are several columns of one batch (chunks laid out back to back,
 *              16-byte aligned, decoded in one call).
 *   mode:      all     read every value of every page with the column type's read call (pqg_decode_host)
 *              skip    per page: skip(3), read 2, repeated (ValuesReader.skip(int n)) (pqg_decode_host)
 *              staged  as `all`, through the staged path
 *              levels  ColumnReaderBase.checkRead per slot through the staged path: rl, dl, and the value
 *                      when dl == max_def (ColumnReaderBase.java:650-676)
 * output, one line each:
 *   FRAME <n headers> | FRAME_ERROR <code> <exception> <page>
 *   CTX_ERROR <code> <exception>
 *   DECODE <code> <exception|-> <page> <value_index>
 *   PERR <page> <code> <phase> <index>       (pqg_page_errors, pages with an error only)
 *   PAGECOL <page> <column>
 *   PAGE <p> <n values> | PAGE <p> INIT_ERROR <code> <exception>
 *   V <page> <index in page> <value>        (ints decimal, float / double bit patterns hex, bytes hex)
 *   L <page> <slot> <r> <d>                 (levels mode)
 *   END <page> <code> <exception>            (the read that ended the page: EOF past the last value;
 *                                            levels mode: the failing read, or 0 after the last slot)
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

typedef struct {
  int32_t hdr[6]; /* physical_type, type_length, max_def, max_rep, flags, codec */
  int64_t num_values;
  uint64_t len;
  uint8_t* bytes;
} case_t;

static int load_case(const char* path, case_t* c) {
  FILE* f = fopen(path, "rb");
  if (!f) return 0;
  char magic[4];
  int ok = fread(magic, 1, 4, f) == 4 && memcmp(magic, "PQGC", 4) == 0 && fread(c->hdr, 4, 6, f) == 6 &&
           fread(&c->num_values, 8, 1, f) == 1 && fread(&c->len, 8, 1, f) == 1;
  if (ok) {
    c->bytes = malloc(c->len + 1);
    ok = c->bytes && fread(c->bytes, 1, c->len, f) == c->len;
  }
  fclose(f);
  return ok;
}

/* the element width of a column's values in a host array */
static int host_width(const pqg_column_desc* col) {
  if (col->flags & PQG_COLUMN_DICTIONARY_IDS) return 4;
  switch (col->physical_type) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return col->type_length;
    default: return 8; /* INT64, DOUBLE, BYTE_ARRAY offsets */
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <case file> all|skip|staged|levels [<case file> ...]\n", argv[0]);
    return 2;
  }
  const char* mode = argv[2];
  const int skip_mode = strcmp(mode, "skip") == 0;
  const int levels_mode = strcmp(mode, "levels") == 0;
  const int staged = levels_mode || strcmp(mode, "staged") == 0;
  const int n_cols = argc - 2;
  case_t* cs = calloc((size_t)n_cols, sizeof(case_t));
  const char** paths = calloc((size_t)n_cols, sizeof(char*));
  paths[0] = argv[1];
  for (int i = 1; i < n_cols; i++) paths[i] = argv[2 + i];
  uint64_t total = 0;
  for (int i = 0; i < n_cols; i++) {
    if (!load_case(paths[i], &cs[i])) return 2;
    total = ((total + 15) & ~(uint64_t)15) + cs[i].len;
  }
  const uint64_t pad = 1024;
  uint8_t* batch = calloc(total + pad, 1);
  pqg_column_desc* cols = calloc((size_t)n_cols, sizeof(pqg_column_desc));
  pqg_page_desc* pages = calloc(8192, sizeof(pqg_page_desc));
  int n_pages = 0;
  uint64_t at = 0;
  pqg_status st;
  for (int i = 0; i < n_cols; i++) {
    case_t* c = &cs[i];
    at = (at + 15) & ~(uint64_t)15;
    memcpy(batch + at, c->bytes, c->len);
    /* ParquetFileReader.Chunk.readAllPages: headers, CRC */
    int n_hdr = 0;
    pqg_page_header* hdrs = calloc(4096, sizeof(pqg_page_header));
    int rc = pqg_frame_chunk(c->bytes, c->len, c->num_values, 1, hdrs, 4096, &n_hdr, &st);
    if (rc) {
      printf("FRAME_ERROR %d %s %d\n", rc, exc(rc), st.page);
      return 0;
    }
    printf("FRAME %d\n", n_hdr);
    pqg_column_desc* col = &cols[i];
    col->physical_type = c->hdr[0];
    col->type_length = c->hdr[1];
    col->max_def = c->hdr[2];
    col->max_rep = c->hdr[3];
    col->flags = c->hdr[4];
    col->dict_offset = -1;
    int np = 0;
    /* the chunk's ColumnMetaData.codec decides which pages are compressed (ColumnChunkPageReadStore) */
    rc = pqg_pages_from_headers(hdrs, n_hdr, c->hdr[5], at, i, col, pages + n_pages, 8192 - n_pages, &np, &st);
    free(hdrs);
    if (rc) {
      printf("FRAME_ERROR %d %s %d\n", rc, exc(rc), st.page);
      return 0;
    }
    for (int p = n_pages; p < n_pages + np; p++) printf("PAGECOL %d %d\n", p, i);
    n_pages += np;
    at += c->len;
  }

  pqg_ctx* ctx = NULL;
  int rc = pqg_ctx_create(0, NULL, &ctx);
  if (rc) {
    printf("CTX_ERROR %d %s\n", rc, exc(rc));
    return 0;
  }
  uint64_t* slots = calloc((size_t)n_cols, sizeof(uint64_t));
  for (int p = 0; p < n_pages; p++) slots[pages[p].column] += pages[p].num_values;
  uint32_t* counts = calloc((size_t)n_pages + 1, sizeof(uint32_t));
  if (staged) {
    /* the JNI shim's sequence: bytes into the library's pinned input, decode, copy the outputs out
     * into arrays of its own (Set<Type>ArrayRegion) */
    uint8_t* in = NULL;
    rc = pqg_host_input(ctx, total, &in);
    if (!rc) {
      memcpy(in, batch, total);
      rc = pqg_decode_staged(ctx, total, cols, n_cols, pages, n_pages, counts, &st);
    }
    for (int i = 0; i < n_cols && rc != PQG_ERR_HIP; i++) {
      pqg_staged_output o;
      if (pqg_staged_column(ctx, i, &o)) break;
      const int w = host_width(&cols[i]);
      const int bin = cols[i].physical_type == PQG_BYTE_ARRAY && !(cols[i].flags & PQG_COLUMN_DICTIONARY_IDS);
      cols[i].values = calloc(o.n_values + 2, (size_t)w);
      memcpy(cols[i].values, o.values, (o.n_values + (bin ? 1 : 0)) * (size_t)w);
      cols[i].def_levels = o.def_levels ? malloc(o.n_slots + 1) : NULL;
      cols[i].rep_levels = o.rep_levels ? malloc(o.n_slots + 1) : NULL;
      if (o.def_levels) memcpy(cols[i].def_levels, o.def_levels, o.n_slots);
      if (o.rep_levels) memcpy(cols[i].rep_levels, o.rep_levels, o.n_slots);
      cols[i].binary_data = bin ? malloc(o.n_binary + 1) : NULL;
      if (bin && o.binary) pqg_copy_out(cols[i].binary_data, o.binary, o.n_binary);
    }
  } else {
    for (int i = 0; i < n_cols; i++) {
      pqg_column_desc* col = &cols[i];
      const int bin = col->physical_type == PQG_BYTE_ARRAY && !(col->flags & PQG_COLUMN_DICTIONARY_IDS);
      int w = 16; /* >= every element width (INT96 12; FLBA up to type_length) */
      if (col->physical_type == PQG_FIXED_LEN_BYTE_ARRAY && col->type_length > w) w = col->type_length;
      col->values = calloc(slots[i] + 1, (size_t)w);
      col->values_capacity = slots[i] + (bin ? 1 : 0);
      col->def_levels = col->max_def > 0 ? calloc(slots[i] + 1, 1) : NULL;
      col->rep_levels = col->max_rep > 0 ? calloc(slots[i] + 1, 1) : NULL;
      col->levels_capacity = slots[i];
      col->binary_capacity = bin ? cs[i].len + 64 : 0;
      col->binary_data = bin ? malloc(col->binary_capacity) : NULL;
    }
    rc = pqg_decode_host(ctx, batch, total, cols, n_cols, pages, n_pages, counts, &st);
    if (rc == PQG_ERR_INVALID_ARG && st.page == -1 && strncmp(st.message, "binary capacity", 15) == 0) {
      /* the dictionary values expand past the first estimate: allocate what the library reports */
      int c = 0;
      sscanf(st.message, "binary capacity: column %d", &c);
      cols[c].binary_capacity = (uint64_t)st.value_index + 64;
      free(cols[c].binary_data);
      cols[c].binary_data = malloc(cols[c].binary_capacity);
      rc = pqg_decode_host(ctx, batch, total, cols, n_cols, pages, n_pages, counts, &st);
    }
  }
  printf("DECODE %d %s %d %" PRId64 "\n", rc, exc(rc), rc ? st.page : -1, rc ? st.value_index : (int64_t)-1);
  pqg_page_error* perr = calloc((size_t)n_pages + 1, sizeof(pqg_page_error));
  const pqg_page_error* pe = NULL;
  if (rc && pqg_page_errors(ctx, perr, n_pages) == PQG_OK) pe = perr;
  for (int p = 0; pe && p < n_pages; p++)
    if (pe[p].code) printf("PERR %d %d %d %" PRId64 "\n", p, pe[p].code, pe[p].phase, pe[p].index);

  int refused_ok = 1;
  for (int p = 0; p < n_pages; p++) {
    const pqg_column_desc* col = &cols[pages[p].column];
    pqg_values_reader r;
    if (levels_mode) {
      /* readPageV1 / V2: rl reader, dl reader, then the data reader (initDataReader) */
      pqg_levels_reader rl, dl;
      int irc = pqg_lr_init_from_page(&rl, col, PQG_LEVELS_REP, pages, n_pages, p, pe);
      if (!irc) irc = pqg_lr_init_from_page(&dl, col, PQG_LEVELS_DEF, pages, n_pages, p, pe);
      if (!irc) irc = pqg_vr_init_from_page(&r, col, pages, counts, n_pages, p, pe);
      if (irc) {
        printf("PAGE %d INIT_ERROR %d %s\n", p, irc, exc(irc));
        continue;
      }
      printf("PAGE %d %" PRIu64 "\n", p, pqg_vr_remaining(&r));
      uint64_t k = 0;
      int e = 0;
      for (uint32_t s = 0; s < pages[p].num_values && !e; s++) {
        int32_t rv = 0, dv = 0;
        if ((e = pqg_lr_read_integer(&rl, &rv)) || (e = pqg_lr_read_integer(&dl, &dv))) break;
        printf("L %d %u %d %d\n", p, s, rv, dv);
        if (dv == col->max_def) e = read_one(&r, p, k++);
      }
      printf("END %d %d %s\n", p, e, exc(e));
      continue;
    }
    const int irc = pqg_vr_init_from_page(&r, col, pages, counts, n_pages, p, pe);
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
