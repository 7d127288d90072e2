/*
 * pqgpu_reader.h — parquet-mr's ValuesReader contract over a decoded page batch (host, C).
 *
 * The JNI shim's readers (shim/java/) keep no decode logic of their own: a batch
 * of pages is decoded in one host call (pqg_decode_host / pqg_decode_staged), and each page's
 * readers then serve that page's slice of the dense column and of its level arrays. This header
 * is those per-page readers in C, so the JNI glue is a thin translation and the contract is
 * testable without a JVM (tests/c/harness.c):
 *
 *   ValuesReader (parquet-column/src/main/java/org/apache/parquet/column/values/ValuesReader.java)
 *     initFromPage(valueCount, in)   :107-114 -> pqg_vr_init_from_page (the page's section is the
 *                                               page's whole data section; nothing is left to consume)
 *     readValueDictionaryId()        :142-144 -> pqg_vr_read_dictionary_id (columns decoded with
 *                                               PQG_COLUMN_DICTIONARY_IDS; DictionaryValuesReader.java:67-73)
 *     readBoolean/readBytes/readFloat/readDouble/readInteger/readLong :149-189 -> pqg_vr_read_*
 *     skip() / skip(n)               :191-203 -> pqg_vr_skip / pqg_vr_skip_n
 *   Level readers (ColumnReaderBase.readPageV1 :738-758 builds rl / dl ValuesReaders from
 *   page.getRlEncoding() / getDlEncoding() — RunLengthBitPackingHybridValuesReader.java:40-65,
 *   ByteBitPackingValuesReader for BIT_PACKED, ZeroIntegerValuesReader when the max level is 0 —
 *   and readPageV2 :760-771 an RLEIntIterator over RunLengthBitPackingHybridDecoder
 *   (newRLEIterator :779-789) or a NullIntIterator when the max level is 0):
 *     initFromPage / RLEIntIterator ctor          -> pqg_lr_init_from_page (PQG_LEVELS_REP / _DEF)
 *     readInteger() / nextInt()                   -> pqg_lr_read_integer
 *     skip()                                      -> pqg_lr_skip
 *   An operation the page's reader does not support returns PQG_ERR_UNSUPPORTED
 *   (UnsupportedOperationException: e.g. readInteger on an INT64 page, readValueDictionaryId on a
 *   column not decoded to ids).
 *
 * Errors (pqg_page_errors of the decode call, include/pqgpu.h) surface exactly where the
 * reference's lazy readers would throw them, per column (a failing column does not affect the
 * others, as a ColumnReader fails on its own):
 *   - the column's dictionary page: every reader of the column's pages fails at init;
 *   - RL_INIT / DL_INIT / DATA_INIT: that reader's init fails (and the readers readPageV1 creates
 *     after it: rl, then dl, then data);
 *   - RL_READ / DL_READ at slot s: the reads of that level array before s succeed, its read of slot
 *     s fails; the other level array is served up to where checkRead would read it (dl up to s-1
 *     after an rl error, rl up to s after a dl error) and fails there with the same error;
 *   - VALUE at value v: the reads before v succeed, the read of v fails;
 *   - a page after its column's first failing page: init fails with that page's error (the
 *     reference's column reader threw there and never reads further).
 * pqg_java_exception(code) names the Java exception class the shim throws for a code.
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

/* Position `r` on page `page` of a decoded batch: `col` is the page's column descriptor with the
 * host outputs (values / binary_data; pqg_decode_host fills them, a staged caller points them at
 * its copies), `page_value_counts` the per-page counts the call wrote, `page_errors` the call's
 * pqg_page_errors (NULL: the call succeeded). Returns the error the reference's initFromPage (or an
 * earlier read of this column) throws, else PQG_OK. */
int pqg_vr_init_from_page(pqg_values_reader* r, const pqg_column_desc* col, const pqg_page_desc* pages,
                          const uint32_t* page_value_counts, int n_pages, int page,
                          const pqg_page_error* page_errors);

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

/* Level reader of one page: the repetition or definition levels of its slots. */
enum pqg_levels_kind { PQG_LEVELS_REP = 0, PQG_LEVELS_DEF = 1 };

typedef struct pqg_levels_reader {
  int32_t max_level;         /* 0: ZeroIntegerValuesReader / NullIntIterator (every read is 0) */
  int32_t error_code;        /* error raised at slot `error_at` (0: none) */
  const uint8_t* levels;     /* the column's u8 level array (host), NULL when max_level == 0 */
  uint64_t pos;              /* next slot (index into the column's level array) */
  uint64_t end;              /* one past the page's last slot */
  uint64_t error_at;
} pqg_levels_reader;

/* Position `r` on the `kind` levels of page `page`: slots of the column's pages before it are
 * skipped (num_values each, the header's slot count); `col->rep_levels` / `def_levels` hold the
 * decoded levels (host). Returns the page's init error for this reader, else PQG_OK. */
int pqg_lr_init_from_page(pqg_levels_reader* r, const pqg_column_desc* col, int kind, const pqg_page_desc* pages,
                          int n_pages, int page, const pqg_page_error* page_errors);
/* Slots left in the page. */
uint64_t pqg_lr_remaining(const pqg_levels_reader* r);
/* The next slot's level. Past the page's slots: PQG_ERR_EOF (the RLE stream is exhausted: the
 * reference fails with a wrapped EOF / past-the-stream error there); a zero reader never ends. */
int pqg_lr_read_integer(pqg_levels_reader* r, int32_t* out);
int pqg_lr_skip(pqg_levels_reader* r);

/* JNI class name of the exception the reference raises for `code` (e.g.
 * "org/apache/parquet/io/ParquetDecodingException", "java/lang/UnsupportedOperationException"). */
const char* pqg_java_exception(int code);

#ifdef __cplusplus
}
#endif

#endif /* PQGPU_READER_H */
