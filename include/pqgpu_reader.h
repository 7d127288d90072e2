/*
 * pqgpu_reader.h — parquet-mr's ValuesReader contract over a decoded page batch (host, C).
 *
 * The JNI shim's GpuValuesReader (shim/java/) keeps no decode logic of its own:
 * a batch of pages is decoded in one pqg_decode_host call, and each page's ValuesReader then
 * serves that page's slice of the dense column. This header is that per-page reader in C, so the
 * JNI glue (shim/jni/pqgpu_jni.c) is a thin translation and the contract is testable without a
 * JVM (tests/c/harness.c):
 *
 *   ValuesReader (parquet-column/src/main/java/org/apache/parquet/column/values/ValuesReader.java)
 *     initFromPage(valueCount, in)   :107-114 -> pqg_vr_init_from_page (the page's section is the
 *                                               page's whole data section; nothing is left to consume)
 *     readValueDictionaryId()        :142-144 -> pqg_vr_read_dictionary_id (columns decoded with
 *                                               PQG_COLUMN_DICTIONARY_IDS; DictionaryValuesReader.java:67-73)
 *     readBoolean/readBytes/readFloat/readDouble/readInteger/readLong :149-189 -> pqg_vr_read_*
 *     skip() / skip(n)               :191-203 -> pqg_vr_skip / pqg_vr_skip_n
 *   An operation the page's reader does not support returns PQG_ERR_UNSUPPORTED
 *   (UnsupportedOperationException: e.g. readInteger on an INT64 page, readValueDictionaryId on a
 *   column not decoded to ids). A decode error of the batch surfaces exactly where the reference's
 *   lazy reader would throw it: init / level errors at pqg_vr_init_from_page of that page, a value
 *   error at the read of that value (the reads before it succeed).
 *   pqg_java_exception(code) names the Java exception class the shim throws for a code.
 */
#ifndef PQGPU_READER_H
#define PQGPU_READER_H

#include "pqgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pqg_values_reader {
  int32_t physical_type;
  int32_t type_length;
  int32_t ids;               /* the column holds dictionary ids (PQG_COLUMN_DICTIONARY_IDS) */
  int32_t error_code;        /* decode error that surfaces in this page at value `error_at` (0: none) */
  const uint8_t* values;     /* dense values of the column (host), or int64 offsets for BYTE_ARRAY */
  const uint8_t* binary;     /* BYTE_ARRAY value bytes */
  uint64_t pos;              /* next value (index into the column) */
  uint64_t end;              /* one past the page's last value */
  uint64_t error_at;         /* column value index at which error_code is raised */
} pqg_values_reader;

/* Position `r` on page `page` of a batch decoded by pqg_decode_host: `col` is the page's column
 * descriptor after the call (values / binary_data / values_written), `page_value_counts` the
 * per-page counts it wrote, `decode_rc` / `decode_status` its result. Returns the page's init /
 * level error (the reference's initFromPage / level reader throws), else PQG_OK. */
int pqg_vr_init_from_page(pqg_values_reader* r, const pqg_column_desc* col, const pqg_page_desc* pages,
                          const uint32_t* page_value_counts, int n_pages, int page, int decode_rc,
                          const pqg_status* decode_status);

/* Values left in the page. */
uint64_t pqg_vr_remaining(const pqg_values_reader* r);

int pqg_vr_read_dictionary_id(pqg_values_reader* r, int32_t* out);
int pqg_vr_read_boolean(pqg_values_reader* r, int32_t* out);
int pqg_vr_read_integer(pqg_values_reader* r, int32_t* out);
int pqg_vr_read_long(pqg_values_reader* r, int64_t* out);
int pqg_vr_read_float(pqg_values_reader* r, float* out);
int pqg_vr_read_double(pqg_values_reader* r, double* out);
/* BYTE_ARRAY: pointer into the decoded bytes + length; FIXED_LEN_BYTE_ARRAY / INT96: the fixed-width
 * value. Zero-copy (Binary.fromConstantByteBuffer on the Java side). */
int pqg_vr_read_bytes(pqg_values_reader* r, const uint8_t** data, uint32_t* len);
int pqg_vr_skip(pqg_values_reader* r);
int pqg_vr_skip_n(pqg_values_reader* r, uint64_t n);

/* JNI class name of the exception the reference raises for `code` (e.g.
 * "org/apache/parquet/io/ParquetDecodingException", "java/lang/UnsupportedOperationException"). */
const char* pqg_java_exception(int code);

#ifdef __cplusplus
}
#endif

#endif /* PQGPU_READER_H */
