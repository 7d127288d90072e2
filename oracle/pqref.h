/* pqref.h — ORACLE (test infrastructure only): CPU restatement of parquet-mr's
 * page readers. See pqref.c for the reference citations. Not part of the product. */
#ifndef PQREF_H
#define PQREF_H
#include <stdint.h>
#include "../include/pqgpu.h"
#ifdef __cplusplus
extern "C" {
#endif
int pqr_width_from_max_int(int32_t bound);
void pqr_unpack8_int(int w, const uint8_t* in, int32_t* out);
void pqr_unpack8_long(int w, const uint8_t* in, int64_t* out);
void pqr_unpack8_int_be(int w, const uint8_t* in, int32_t* out);
int pqr_rle_decode(int bit_width, const uint8_t* buf, int64_t len, int64_t n, int32_t* out,
                   int64_t* err_index, int64_t* consumed);
int64_t pqr_router_read_batch(int bit_width, const uint8_t* in, int64_t in_len, int count, int32_t* out);
int64_t pqr_delta_decode(const uint8_t* buf, int64_t len, int64_t* out, int64_t cap, int64_t* consumed);
/* Snappy raw block (page codec SNAPPY): 0 or PQG_ERR_CORRUPT; the length must equal `expect`. */
int pqr_snappy_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len);
/* Zstandard (RFC 8878) frames -> dst (zstd_ref.c); XXH64 of the content checksum */
int pqr_zstd_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len);
/* LZ4 raw block (Lz4RawDecompressor; LZ4 block format restated): 0, or PQG_ERR_CORRUPT. */
int pqr_lz4_raw_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len);
/* GZIP members (RFC 1952 / 1951 restated, gzip_ref.c): 0, PQG_ERR_EOF (short) or PQG_ERR_CORRUPT. */
int pqr_gzip_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len);
uint64_t pqr_xxh64(const uint8_t* p, uint64_t n, uint64_t seed);
int pqr_decode(const uint8_t* bytes, uint64_t n_bytes, pqg_column_desc* cols, int n_cols,
               const pqg_page_desc* pages, int n_pages, uint32_t* page_value_counts, pqg_status* st);
const char* pqg_error_name_ref(int code);
#ifdef __cplusplus
}
#endif
#endif
