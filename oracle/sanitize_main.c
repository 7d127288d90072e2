/*
 * sanitize_main.c — ORACLE TEST INFRASTRUCTURE: runs oracle/pqref.c under AddressSanitizer +
 * UndefinedBehaviorSanitizer (host code only; built by tests/test_oracle_sanitize.py with
 * -fsanitize=address,undefined -fno-sanitize-recover=all, so any finding aborts).
 *
 * usage: sanitize_main <case file>...
 *   case file: "PQGB" | u32 n_cols | u32 n_pages | u64 n_bytes | pqg_column_desc[n_cols] (pointers 0)
 *              | pqg_page_desc[n_pages] | bytes[n_bytes]
 * Every case is decoded by pqr_decode into exactly-sized heap outputs (values, levels, BYTE_ARRAY
 * bytes of the capacity the case asks for), so an out-of-bounds read of the page bytes or write past
 * an output is caught. Prints "<file> rc=<code>" per case.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pqref.h"

static int elem_width(int t, int tl) {
  switch (t) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return tl > 0 ? tl : 1;
    default: return 8;  /* BYTE_ARRAY offsets */
  }
}

int main(int argc, char** argv) {
  for (int a = 1; a < argc; a++) {
    FILE* f = fopen(argv[a], "rb");
    if (!f) return 2;
    char magic[4];
    uint32_t n_cols, n_pages;
    uint64_t n_bytes;
    if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "PQGB", 4) || fread(&n_cols, 4, 1, f) != 1 ||
        fread(&n_pages, 4, 1, f) != 1 || fread(&n_bytes, 8, 1, f) != 1)
      return 2;
    pqg_column_desc* cols = calloc(n_cols + 1, sizeof(*cols));
    pqg_page_desc* pages = calloc(n_pages + 1, sizeof(*pages));
    /* exactly n_bytes: the oracle must not read past the batch */
    uint8_t* bytes = malloc(n_bytes ? n_bytes : 1);
    if (fread(cols, sizeof(*cols), n_cols, f) != n_cols || fread(pages, sizeof(*pages), n_pages, f) != n_pages ||
        fread(bytes, 1, n_bytes, f) != n_bytes)
      return 2;
    fclose(f);
    void** bufs = calloc(4 * (size_t)n_cols + 1, sizeof(void*));
    for (uint32_t i = 0; i < n_cols; i++) {
      uint64_t slots = 0;
      for (uint32_t p = 0; p < n_pages; p++)
        if (pages[p].column == (int32_t)i) slots += pages[p].num_values;
      const int bin = cols[i].physical_type == PQG_BYTE_ARRAY;
      const uint64_t cap = slots + (bin ? 1 : 0);
      bufs[4 * i] = malloc(cap * (uint64_t)elem_width(cols[i].physical_type, cols[i].type_length) + 1);
      cols[i].values = bufs[4 * i];
      cols[i].values_capacity = cap;
      if (cols[i].max_def > 0) cols[i].def_levels = bufs[4 * i + 1] = malloc(slots + 1);
      if (cols[i].max_rep > 0) cols[i].rep_levels = bufs[4 * i + 2] = malloc(slots + 1);
      cols[i].levels_capacity = slots;
      if (bin) {
        /* the case's binary_capacity field holds the capacity to test with */
        cols[i].binary_data = bufs[4 * i + 3] = malloc(cols[i].binary_capacity + 1);
      }
    }
    uint32_t* counts = calloc(n_pages + 1, sizeof(uint32_t));
    pqg_status st;
    const int rc = pqr_decode(bytes, n_bytes, cols, (int)n_cols, pages, (int)n_pages, counts, &st);
    printf("%s rc=%d\n", argv[a], rc);
    for (uint32_t j = 0; j < 4 * n_cols; j++) free(bufs[j]);
    free(bufs);
    free(counts);
    free(bytes);
    free(pages);
    free(cols);
  }
  return 0;
}
