/*
 * pqgpu.h — C ABI of the MI355X-native Parquet column-page decoder.
 *
 * This is the drop-in boundary for parquet-mr's page-decode hot path
 * (SURVEY.md §8b). Every entry point uses plain C types: pointers and sizes,
 * no C++ or torch types. A JNI shim binds it the way
 * parquet-mr would bind a native ValuesReader / ParquetReadRouter backend.
 *
 * Reference interfaces replaced (apache/parquet-mr 1.15.0-SNAPSHOT):
 *   - ValuesReader.initFromPage / readX
 *     parquet-column/src/main/java/org/apache/parquet/column/values/ValuesReader.java:36-203
 *     -> pqg_decode (many pages per call; dense values + levels per column)
 *   - ColumnReaderBase.readPageV1 / readPageV2 / newRLEIterator (page split, levels)
 *     parquet-column/src/main/java/org/apache/parquet/column/impl/ColumnReaderBase.java:738-789
 *     -> pqg_decode (levels decoded on device, data section located on device)
 *   - Encoding.getValuesReader / getDictionaryBasedValuesReader / initDictionary
 *     parquet-column/src/main/java/org/apache/parquet/column/Encoding.java:61-320
 *     -> the (physical_type, encoding) dispatch inside pqg_decode
 *   - ParquetReadRouter.read(bitWidth, in, currentCount, int[] out)
 *     parquet-plugins/parquet-encoding-vector/src/main/java/org/apache/parquet/column/values/bitpacking/ParquetReadRouter.java:57-66
 *     -> pqg_unpack_runs (device batch) / pqg_router_read (host buffers)
 *
 * Threading: a pqg_ctx owns one HIP stream and its device scratch; it is not
 * shared between threads (one ctx per thread per GPU), like a ValuesReader.
 * All pqg_decode / pqg_plan_launch work is asynchronous on the ctx stream
 * until pqg_sync (a launch may fan out to three internal queues of the ctx
 * and joins them back into the ctx stream before it returns). Outputs are
 * valid only after pqg_sync returns: two rare cases are repaired by pqg_sync
 * itself with a host-driven re-launch (a PLAIN BYTE_ARRAY page with bytes
 * after its values, pqg_plan_plain_fallbacks; a fused-kernel timeout,
 * pqg_plan_timeout_fallbacks; a wrong V2 header null count,
 * pqg_plan_null_hint_fallbacks), so work ordered after a launch on the ctx
 * stream by events alone may see outputs that pqg_sync later rewrites.
 * No exception crosses this ABI: every function returns a pqg_error code and
 * fills an optional pqg_status.
 *
 * ABI 4 (this version): pqg_page_desc carries the V2 header's num_nulls
 * (PQG_PAGE_NULL_COUNT, 56-byte descriptor), pqg_plan_null_hint_fallbacks.
 * ABI 3: per-page errors (pqg_page_errors) so that a failure
 * surfaces in its own column only; the staged host path (pqg_host_input /
 * pqg_decode_staged / pqg_staged_column) for callers that must not hold host
 * arrays across device work (JNI critical regions); the host batch of router
 * runs (pqg_router_read_runs); levels readers (pqgpu_reader.h).
 */
#ifndef PQGPU_H
#define PQGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQG_ABI_VERSION 4

/* parquet-format `Type` values (parquet.thrift). */
enum pqg_physical_type {
  PQG_BOOLEAN = 0,
  PQG_INT32 = 1,
  PQG_INT64 = 2,
  PQG_INT96 = 3,
  PQG_FLOAT = 4,
  PQG_DOUBLE = 5,
  PQG_BYTE_ARRAY = 6,
  PQG_FIXED_LEN_BYTE_ARRAY = 7
};

/* parquet-format `Encoding` values (parquet.thrift); see Encoding.java:61-253. */
enum pqg_encoding {
  PQG_PLAIN = 0,
  PQG_PLAIN_DICTIONARY = 2,
  PQG_RLE = 3,
  PQG_BIT_PACKED = 4,
  PQG_DELTA_BINARY_PACKED = 5,
  PQG_DELTA_LENGTH_BYTE_ARRAY = 6,
  PQG_DELTA_BYTE_ARRAY = 7,
  PQG_RLE_DICTIONARY = 8,
  PQG_BYTE_STREAM_SPLIT = 9
};

/*
 * Error codes. Each decode error names the Java exception the reference
 * reader raises for the same bytes, so the JNI shim can rethrow it as
 * ParquetDecodingException (io/ParquetDecodingException.java) with the same
 * meaning. The first failing (page, value index) in page order is reported,
 * which is the value at which the reference's lazy reader would throw.
 */
enum pqg_error {
  PQG_OK = 0,
  PQG_ERR_INVALID_ARG = 1,      /* API misuse (null pointer, bad count, capacity too small) */
  PQG_ERR_UNSUPPORTED = 2,      /* (type, encoding) has no reader: Encoding.java:84,193; UnsupportedOperationException */
  PQG_ERR_HIP = 3,              /* HIP runtime failure */
  PQG_ERR_NO_DEVICE = 4,        /* no HIP device / extension unusable */
  PQG_ERR_TIMEOUT = 5,          /* a fused-kernel wave waited > 2 s of wall time for its page's walk (the
                                   walker was descheduled or starved); not a decode error: the chunk's
                                   output is incomplete, relaunch the plan */
  PQG_ERR_EOF = 10,             /* java.io.EOFException: read past the end of a page section
                                   (SingleBufferInputStream.read :50-55, LittleEndianDataInputStream.readInt/readLong) */
  PQG_ERR_RLE_PAST_END = 11,    /* IllegalArgumentException "Reading past RLE/BitPacking stream."
                                   (RunLengthBitPackingHybridDecoder.java:81) */
  PQG_ERR_BIT_WIDTH = 12,       /* IllegalArgumentException "bitWidth must be >= 0 and <= 32"
                                   (RunLengthBitPackingHybridDecoder.java:55) */
  PQG_ERR_DICT_ID = 13,         /* ArrayIndexOutOfBoundsException in Dictionary.decodeToX
                                   (PlainValuesDictionary.java:159-161 etc.) */
  PQG_ERR_EMPTY_PAGE = 14,      /* IOException "Attempt to read from empty page" (DictionaryValuesReader.java:57-62) */
  PQG_ERR_EMPTY_PACKED_RUN = 15,/* bit-packed run header with 0 groups: AIOOBE on currentBuffer[] (:71) */
  PQG_ERR_DELTA_CONFIG = 16,    /* IllegalArgumentException "miniBlockSize must be multiple of 8"
                                   (DeltaBinaryPackingConfig.java:39) */
  PQG_ERR_DELTA_PAST_END = 17,  /* ParquetDecodingException "no more value to read, total value count is N"
                                   (DeltaBinaryPackingValuesReader.java:115-119) */
  PQG_ERR_CORRUPT = 18,         /* section lengths inconsistent with the page (negative/oversized length prefix) */
  PQG_ERR_NO_DICTIONARY = 19,   /* "could not read page ... as the dictionary was missing" (ColumnReaderBase.java:709-712) */
  PQG_ERR_DICT_ENCODING = 20,   /* "Dictionary data encoding type not supported" (PlainValuesDictionary.java:49-52) */
  PQG_ERR_CRC = 21              /* ParquetDecodingException "could not verify page integrity, CRC checksum
                                   verification failed" (ParquetFileReader.java:1805-1813) */
};

/*
 * One data page, already decompressed, located inside the batch byte buffer.
 * Mirrors DataPageV1 (DataPageV1.java:26-141) and DataPageV2 (DataPageV2.java:26-247).
 */
typedef struct pqg_page_desc {
  uint64_t offset;         /* byte offset of the page body in the batch buffer (16-B aligned is fastest) */
  uint32_t size;           /* page body length in bytes (V1: rl + dl + data sections; V2: rl + dl + data) */
  uint32_t num_values;     /* header num_values: level slots including nulls */
  int32_t column;          /* index into the pqg_column_desc table */
  int32_t version;         /* 1 = DataPageV1, 2 = DataPageV2 */
  int32_t encoding;        /* value encoding (pqg_encoding) */
  int32_t rl_encoding;     /* V1 only: RLE or BIT_PACKED (ignored when max_rep == 0) */
  int32_t dl_encoding;     /* V1 only: RLE or BIT_PACKED (ignored when max_def == 0) */
  uint32_t rl_byte_length; /* V2 only: repetition_levels_byte_length */
  uint32_t dl_byte_length; /* V2 only: definition_levels_byte_length */
  uint32_t flags;          /* PQG_PAGE_* (0 for a page written by a current writer) */
  uint32_t num_nulls;      /* V2 only, read when flags has PQG_PAGE_NULL_COUNT: DataPageHeaderV2.num_nulls (ABI 4) */
  uint32_t reserved;       /* 0 (sizeof(pqg_page_desc) = 56) */
} pqg_page_desc;

/* pqg_page_desc.flags: PQG_PAGE_DBA_CARRY — a DELTA_BYTE_ARRAY page whose reader takes the previous
 * page's last value as its starting `previous` (PARQUET-246: DeltaByteArrayWriter before parquet-mr
 * 1.8.0 did not reset `previous` between pages, so the first value of every page after the first may
 * carry a prefix of the previous page's last value). The reader side is
 * ColumnReaderBase.initDataReader (parquet-column/.../column/impl/ColumnReaderBase.java:730-735) ->
 * DeltaByteArrayReader.setPreviousReader (.../values/deltastrings/DeltaByteArrayReader.java:89-95),
 * applied when CorruptDeltaByteArrays.requiresSequentialReads(created_by, DELTA_BYTE_ARRAY)
 * (parquet-column/src/main/java/org/apache/parquet/CorruptDeltaByteArrays.java:31-84) holds: the caller
 * sets the flag on every DELTA_BYTE_ARRAY page of such a column chunk except its first page. The
 * previous page of the column in the batch must be a DELTA_BYTE_ARRAY page (the reference casts its
 * reader to DeltaByteArrayReader), otherwise PQG_ERR_UNSUPPORTED. Flagged pages are decoded in page
 * order, one column at a time. */
#define PQG_PAGE_DBA_CARRY 1

/* pqg_page_desc.flags: PQG_PAGE_NULL_COUNT — `num_nulls` holds the DataPageV2 header's null count
 * (DataPageV2.getNullCount, parquet-column/src/main/java/org/apache/parquet/column/page/DataPageV2.java:197-199;
 * pqg_pages_from_headers sets it for every V2 page). The reference never trusts that count: it decodes
 * the definition levels and reads a value for every slot with dl == max_def (ColumnReaderBase.java:650-676,
 * readPageV2 :760-771). The decoder uses it as a verified hint: when every page of every nullable column
 * of a plan is a V2 page carrying it, each page's value count (num_values - num_nulls) and output offset
 * are known on the host, so the value kernels start at the launch's start beside the level kernel instead
 * of after it. The level kernel still decodes every level section and compares each page's true count;
 * a mismatch (or any level / level-init error on such a page) makes pqg_sync re-run the plan with the
 * counts taken from the levels, as without the hint (pqg_plan_null_hint_fallbacks counts these re-runs),
 * so results and errors are those of the reference whatever the header says. */
#define PQG_PAGE_NULL_COUNT 2

/*
 * One column chunk: the ColumnDescriptor facts the decoder needs (physical
 * type, type length, max rep/def level), its dictionary page (optional) and
 * where its decoded output goes.
 *
 * Output layout (Java-equivalent "dense" form): `values` receives only the
 * non-null values, in slot order, exactly the sequence the reference's
 * ValuesReader returns for slots with dl == max_def (ColumnReaderBase.java:650-676).
 * `def_levels` / `rep_levels` receive one byte per slot (the Java int level;
 * level values above 255 are stored saturated to 255 and therefore never
 * equal max_def, which is limited to <= 254). Element widths: INT32/FLOAT 4,
 * INT64/DOUBLE 8, INT96 12, FIXED_LEN_BYTE_ARRAY type_length, BOOLEAN 1.
 * For pqg_decode these are device pointers; the per-page value counts are
 * written to `page_value_counts` (device, one uint32 per page of the batch, optional).
 */
/* pqg_column_desc.flags: PQG_COLUMN_DICTIONARY_IDS — `values` receives the uint32 dictionary id of
 * every non-null value instead of the value (DictionaryValuesReader.readValueDictionaryId,
 * parquet-column/src/main/java/org/apache/parquet/column/values/dictionary/DictionaryValuesReader.java:67-73),
 * any physical type; a page of the column that is not dictionary-encoded fails with
 * PQG_ERR_UNSUPPORTED (ValuesReader.readValueDictionaryId throws UnsupportedOperationException,
 * ValuesReader.java:142-144). */
#define PQG_COLUMN_DICTIONARY_IDS 1

typedef struct pqg_column_desc {
  int32_t physical_type;     /* pqg_physical_type */
  int32_t type_length;       /* FIXED_LEN_BYTE_ARRAY length */
  int32_t max_rep;           /* ColumnDescriptor.getMaxRepetitionLevel() */
  int32_t max_def;           /* ColumnDescriptor.getMaxDefinitionLevel() */
  int64_t dict_offset;       /* byte offset of the dictionary page body in the batch buffer, -1 if none */
  uint32_t dict_size;        /* dictionary page body bytes */
  uint32_t dict_num_values;  /* DictionaryPageHeader.num_values */
  int32_t dict_encoding;     /* PLAIN or PLAIN_DICTIONARY */
  int32_t flags;             /* PQG_COLUMN_* (0: decode values) */
  void* values;              /* dense output values */
  uint64_t values_capacity;  /* capacity in elements */
  uint8_t* def_levels;       /* per-slot definition levels (may be NULL) */
  uint8_t* rep_levels;       /* per-slot repetition levels (may be NULL) */
  uint64_t levels_capacity;  /* capacity in slots */
  uint8_t* binary_data;      /* BYTE_ARRAY only: value bytes; `values` then holds int64 offsets[n+1] */
  uint64_t binary_capacity;  /* BYTE_ARRAY only: capacity of binary_data in bytes */
  uint64_t values_written;   /* OUT (after pqg_sync / host calls): non-null values decoded */
} pqg_column_desc;

/* First decode error of a call, in (page, value) order. */
typedef struct pqg_status {
  int32_t code;              /* pqg_error */
  int32_t page;              /* index into the page table, -1 if not page-specific */
  int64_t value_index;       /* value index inside the page (data values for value errors, slots for level errors) */
  char message[240];
} pqg_status;

typedef struct pqg_ctx pqg_ctx;
typedef struct pqg_plan pqg_plan;

/* ---- context ------------------------------------------------------------ */

/* Library / ABI version (PQG_ABI_VERSION). */
int pqg_abi_version(void);

/* Number of visible HIP devices (0 when none). */
int pqg_device_count(void);

/* Create a context on `device`. `hip_stream` may be NULL (the ctx creates its
 * own non-blocking stream) or an existing hipStream_t to run on. */
int pqg_ctx_create(int device, void* hip_stream, pqg_ctx** out);
int pqg_ctx_destroy(pqg_ctx* ctx);
/* The hipStream_t the ctx launches on. */
void* pqg_ctx_stream(pqg_ctx* ctx);

/* Kernel-choice overrides for plans created on the ctx afterwards (tests and A/B measurements;
 * the defaults are the measured choices). Decoded results are the same under every setting.
 *   PQG_DISPATCH_PLAIN_ONE_PASS  PLAIN-only BYTE_ARRAY columns: 0 = per-value path (walk, offset
 *                                scan, copy), 1 = one pass, tiles, 2 = one pass, tiles below 4,096
 *                                PLAIN pages and one wave per page from there (default), 3 = one
 *                                pass, one wave per page
 *   PQG_DISPATCH_DICT_DIRECT     dictionary BYTE_ARRAY columns with small dictionaries: 1 = ids
 *                                mapped straight to lengths and bytes (default), 0 = ids, then map
 *   PQG_DISPATCH_DICT_FUSED      dictionary pages: 1 = walk and expansion in one launch (default),
 *                                0 = two launches (the mode a fused launch that timed out re-runs in)
 *   PQG_DISPATCH_NULL_HINTS      nullable columns of V2 pages: 1 = value kernels start from the header
 *                                null counts beside the level decode, which verifies them (default;
 *                                PQG_PAGE_NULL_COUNT), 0 = levels first
 *   PQG_DISPATCH_GZIP_PREPASS_MIN pqg_gzip_decompress: pages of at least `value` output bytes take the
 *                                token pre-pass + replay, smaller ones the one-wave decoder (default
 *                                16384; 0 = every page); applies to later pqg_gzip_decompress calls
 * Returns PQG_ERR_INVALID_ARG for an unknown key or value. Not thread-safe (like the ctx). */
enum pqg_dispatch {
  PQG_DISPATCH_PLAIN_ONE_PASS = 1,
  PQG_DISPATCH_DICT_DIRECT = 2,
  PQG_DISPATCH_GZIP_PREPASS_MIN = 3,
  PQG_DISPATCH_DICT_FUSED = 4,
  PQG_DISPATCH_NULL_HINTS = 5
};
int pqg_ctx_set_dispatch(pqg_ctx* ctx, int key, int value);

/* ---- device-resident batch decode ----------------------------------------
 * `d_bytes` is a 4-byte aligned DEVICE buffer holding every page body (and
 * dictionary page) the descriptors refer to, padded by at least 64 readable
 * bytes after the last page; `n_bytes` is its readable size INCLUDING that
 * padding (device loads are range-checked per dword against it, so a page that
 * ends at an unaligned offset needs the padding inside n_bytes). Page offsets may
 * have any alignment (raw file bytes); 16-B aligned is fastest. Column output
 * pointers are DEVICE pointers. Pages of one column
 * must appear in page order; pages of several columns may be interleaved.
 * Asynchronous: errors are reported by pqg_sync. */
int pqg_decode(pqg_ctx* ctx, const uint8_t* d_bytes, uint64_t n_bytes,
               pqg_column_desc* cols, int n_cols,
               const pqg_page_desc* pages, int n_pages,
               uint32_t* d_page_value_counts, pqg_status* st);

/* Wait for all work on the ctx stream; returns the first decode error of the
 * calls since the previous pqg_sync (every plan launched since then, in launch
 * order, is checked and repaired as described above) and fills
 * cols[i].values_written for the most recent pqg_decode. */
int pqg_sync(pqg_ctx* ctx, pqg_status* st);

/* ---- per-page errors ---------------------------------------------------------
 * pqg_status names the batch's first failing page. A column reader in the
 * reference fails on its own (ColumnReaderBase.readPage / checkRead /
 * readValue, ColumnReaderBase.java:590-676, 738-771): the other columns of the
 * row group stay readable. pqg_page_errors gives every page's own first error
 * in the reference's read order of that page:
 *   DICTIONARY  the column's dictionary page (ColumnReaderBase ctor :448-472; set on the column's
 *               first page of the batch)
 *   RL_INIT / DL_INIT / DATA_INIT   rlReader / dlReader / data reader initFromPage (readPageV1
 *               :738-758; a V2 page's level lengths past the page: RL_INIT)
 *   RL_READ / DL_READ   repetitionLevelColumn / definitionLevelColumn .nextInt() of slot `index`
 *               (checkRead :650-676 reads rl then dl per slot)
 *   VALUE       the read of value `index` of the page (readValue :584-626)
 * Values are decoded only for slots before a level error, and a page's value count
 * (page_value_counts) stops there. A caller serving the pages of one column in
 * order stops at that column's first failing page (pqgpu_reader.h does). */
enum pqg_phase {
  PQG_PHASE_NONE = 0,
  PQG_PHASE_DICTIONARY = 1,
  PQG_PHASE_RL_INIT = 2,
  PQG_PHASE_DL_INIT = 3,
  PQG_PHASE_DATA_INIT = 4,
  PQG_PHASE_RL_READ = 5,
  PQG_PHASE_DL_READ = 6,
  PQG_PHASE_VALUE = 7
};

typedef struct pqg_page_error {
  int32_t code;     /* pqg_error; PQG_OK when the page decoded cleanly */
  int32_t phase;    /* pqg_phase */
  int64_t index;    /* RL_READ / DL_READ: slot in the page; VALUE: value in the page; else -1 */
} pqg_page_error;

/* Every page's error of the most recent pqg_decode / pqg_decode_host / pqg_decode_staged on the
 * ctx, after its pqg_sync (the host calls sync themselves). `n_pages` must equal that call's page
 * count. API / device failures (no page) are not listed: they are the call's return code. */
int pqg_page_errors(pqg_ctx* ctx, pqg_page_error* out, int n_pages);
/* The same for a plan's most recent launch, after pqg_sync. */
int pqg_plan_page_errors(pqg_plan* plan, pqg_page_error* out, int n_pages);

/* ---- prepared plans (bench / steady-state) --------------------------------
 * A plan uploads descriptors once; pqg_plan_launch re-runs the decode of the
 * same page batch with no host work beyond the kernel launches. */
int pqg_plan_create(pqg_ctx* ctx, const uint8_t* d_bytes, uint64_t n_bytes,
                    const pqg_column_desc* cols, int n_cols,
                    const pqg_page_desc* pages, int n_pages, pqg_plan** out, pqg_status* st);
int pqg_plan_launch(pqg_plan* plan);
/* Number of kernel launches one pqg_plan_launch issues. */
int pqg_plan_kernel_count(pqg_plan* plan);
/* Dictionary pages decode in one fused launch (walk + expansion, the expansion waiting for its
 * page's walk). Should an expansion wait longer than 2 s (the GPU did not dispatch the walker it
 * waits for), that launch reports PQG_ERR_TIMEOUT internally and pqg_sync re-runs the plan with the
 * walk and the expansion as two launches; the plan keeps that mode and the caller sees the normal
 * result. The same holds for a segment of a segmented PLAIN BYTE_ARRAY page walk (per-value path,
 * few large pages) whose predecessor segment did not publish within 2 s: the plan re-runs with those
 * pages walked one wave each, and keeps that mode. Returns how many launches of the plan were re-run
 * either way. */
int pqg_plan_timeout_fallbacks(pqg_plan* plan);
/* BYTE_ARRAY columns whose pages are all PLAIN decode in one pass per 2 KiB tile of the pages (walk,
 * offsets and value bytes together), which takes each page's values to fill its data section, as
 * every writer lays them out. A page with bytes after its num_values values (which the reader
 * ignores) is detected on the device, and pqg_sync re-runs the plan on the per-value path (value
 * walk, offset scan, byte copy), which reads exactly num_values values; the plan keeps that path.
 * Returns how many launches of the plan were re-run that way. */
int pqg_plan_plain_fallbacks(pqg_plan* plan);
/* Plans whose nullable columns are all V2 pages with PQG_PAGE_NULL_COUNT start their value kernels
 * from the header null counts (see PQG_PAGE_NULL_COUNT). Returns how many launches of the plan pqg_sync
 * re-ran with the counts taken from the levels because a header count was wrong (the plan then keeps
 * the level-first order). */
int pqg_plan_null_hint_fallbacks(pqg_plan* plan);
int pqg_plan_destroy(pqg_plan* plan);

/* ---- host-buffer decode (the JNI shim's entry: file bytes in, arrays out) --
 * Copies `h_bytes` to the device through pinned staging (hipMemcpyAsync),
 * decodes, and copies values / levels back into the HOST pointers of `cols`.
 * Synchronous. */
int pqg_decode_host(pqg_ctx* ctx, const uint8_t* h_bytes, uint64_t n_bytes,
                    pqg_column_desc* cols, int n_cols,
                    const pqg_page_desc* pages, int n_pages,
                    uint32_t* h_page_value_counts, pqg_status* st);

/* ---- staged host path -------------------------------------------------------
 * pqg_decode_host reads and writes the caller's host arrays while the device works, which a JNI
 * caller may not allow (a Get*ArrayCritical region must not span blocking calls). The staged path
 * keeps the caller's arrays out of device work: the library owns the pinned input and output
 * buffers, and the caller copies in before and out after.
 *   1. pqg_host_input(ctx, n_bytes, &p): pinned buffer of at least n_bytes (+ padding, zeroed by the
 *      decode); the caller writes the page bytes to p[0 .. n_bytes) (JNI: GetByteArrayRegion, or a
 *      memcpy from a direct buffer). Valid until the next pqg_host_input / host call on ctx.
 *   2. pqg_decode_staged(ctx, n_bytes, cols, ...): as pqg_decode_host over those bytes. The output
 *      fields of `cols` (pointers and capacities) are ignored: the values of every column and the
 *      levels of every column with max_def / max_rep > 0 are produced into library memory, sized by
 *      the library. Returns after the outputs are in pinned host memory.
 *   3. pqg_staged_column(ctx, col, &out): where column `col`'s outputs are in that memory; valid
 *      until the next host call on ctx. Copy them out with any memcpy (JNI: Set<Type>ArrayRegion,
 *      or pqg_copy_out inside a short critical region: a plain multi-threaded memcpy, no device call).
 * Codes, statuses and per-page errors as pqg_decode_host. */
typedef struct pqg_staged_output {
  const void* values;        /* n_values elements (BYTE_ARRAY: int64 offsets[n_values + 1]) */
  const uint8_t* def_levels; /* n_slots bytes, NULL if not wanted / max_def == 0 */
  const uint8_t* rep_levels; /* n_slots bytes, NULL if not wanted / max_rep == 0 */
  const uint8_t* binary;     /* BYTE_ARRAY: n_binary value bytes */
  uint64_t n_values;
  uint64_t n_slots;
  uint64_t n_binary;
} pqg_staged_output;

int pqg_host_input(pqg_ctx* ctx, uint64_t n_bytes, uint8_t** buf);
int pqg_decode_staged(pqg_ctx* ctx, uint64_t n_bytes, pqg_column_desc* cols, int n_cols,
                      const pqg_page_desc* pages, int n_pages, uint32_t* h_page_value_counts, pqg_status* st);
int pqg_staged_column(pqg_ctx* ctx, int col, pqg_staged_output* out);
/* memcpy of n bytes spread over up to 8 host threads (large copies out of pinned memory). */
void pqg_copy_out(void* dst, const void* src, uint64_t n);

/* ---- ParquetReadRouter boundary --------------------------------------------
 * Batch of bit-packed runs on the device: run r unpacks counts[r] (multiple of 8)
 * LSB-first values of `bit_width` bits from d_in + in_offsets[r] into
 * d_out + out_offsets[r] (int32). Bit-exact with Packer.LITTLE_ENDIAN
 * BytePacker.unpack8Values (ByteBasedBitPackingGenerator.java:258-308). */
int pqg_unpack_runs(pqg_ctx* ctx, int bit_width, const uint8_t* d_in,
                    const uint64_t* d_in_offsets, const uint32_t* d_counts,
                    const uint64_t* d_out_offsets, int32_t* d_out, int n_runs);

/* ParquetReadRouter.read equivalent on host buffers: consumes
 * count*bit_width/8 bytes of `in` (in_len must cover them, else PQG_ERR_EOF as
 * SingleBufferInputStream.slice throws EOFException) and writes `count` ints.
 * The unpack runs on the GPU (H2D, kernel, D2H); synchronous. A parity entry for the router's
 * call shape: one call per run pays a PCIe round trip, so batch runs through pqg_unpack_runs
 * (device buffers) or decode whole pages with pqg_decode. */
int pqg_router_read(pqg_ctx* ctx, int bit_width, const uint8_t* in, size_t in_len,
                    int count, int32_t* out);

/* Many router reads in one round trip (host buffers): run r is ParquetReadRouter.read(bit_width,
 * in positioned at in_offsets[r], counts[r], ...) and its counts[r] ints go to out + (sum of the
 * earlier counts). One H2D of the bytes the runs cover, one kernel, one D2H, one synchronisation
 * for the whole batch (a page's bit-packed runs, say). counts[r] must be a multiple of 8 (a
 * bit-packed run's currentCount); a run whose counts[r] * bit_width / 8 bytes pass in_len ->
 * PQG_ERR_EOF with nothing written (SingleBufferInputStream.slice throws EOFException before the
 * unpack). Synchronous. */
int pqg_router_read_runs(pqg_ctx* ctx, int bit_width, const uint8_t* in, size_t in_len,
                         const uint64_t* in_offsets, const uint32_t* counts, int n_runs, int32_t* out);

/* ParquetReadRouter.read (parquet-plugins/parquet-encoding-vector/.../ParquetReadRouter.java:57-66)
 * with its contract kept — out[0 .. count) holds the run's values when the call returns — at one
 * device round trip per page instead of per run. `in` is the caller's stream at the run's data start
 * and `stream_left` the bytes left in that stream (ByteBufferInputStream.available(): the run's bytes
 * and everything after them). On a miss the hybrid stream after the run is walked on the host
 * (RunLengthBitPackingHybridDecoder.readNext header forms), this run and every later bit-packed run
 * found are unpacked in one pqg_router_read_runs call, and the results are kept in the context; a
 * later call for a walked run (same width, count, position from the end, and bytes) is served from
 * host memory with no device work. The caller advances its stream by count*bit_width/8 bytes, as
 * after readBatch. Errors as pqg_router_read: count not a multiple of 8 -> INVALID_ARG; the run's
 * bytes past stream_left -> PQG_ERR_EOF (SingleBufferInputStream.slice) with nothing written. */
int pqg_router_read_page(pqg_ctx* ctx, int bit_width, const uint8_t* in, size_t stream_left, int count,
                         int32_t* out);

/* The cache probe of pqg_router_read_page alone (host only, never a device call): needs only the
 * run's count*bit_width/8 bytes at `run`. *hit = 1 with out filled, or 0 with nothing written (then
 * call pqg_router_read_page with the whole stream tail). For callers whose stream tail costs a copy
 * (the JNI shim's heap arrays). */
int pqg_router_cache_lookup(pqg_ctx* ctx, int bit_width, const uint8_t* run, size_t stream_left, int count,
                            int32_t* out, int* hit);

/* Reads served from the page cache (hits) and device round trips (misses) since the context was
 * created. */
int pqg_router_cache_stats(pqg_ctx* ctx, uint64_t* hits, uint64_t* misses);

/* ---- record assembly ---------------------------------------------------------
 * Dremel assembly of ONE leaf column into the columnar form of its records: the
 * Arrow-style equivalent of the converter events parquet-mr's automaton emits
 * (RecordReaderImplementation.read, parquet-column/src/main/java/org/apache/parquet/io/RecordReaderImplementation.java:409-446,
 * built by MessageColumnIO.getRecordReader, io/MessageColumnIO.java:77-130).
 *
 * `path` lists the schema nodes from the root's child down to the leaf. Entries of
 * repetition depth r are the records (r = 0) or the elements of the r-th REPEATED node.
 * A non-REPEATED node has one entry per entry of its depth (the number of REPEATED nodes
 * at or above it); a REPEATED node's entries are its elements. Outputs (device pointers):
 *   OPTIONAL node: validity[entry] = 1 when the node is present (a group the automaton opens,
 *                  or a non-null leaf value);
 *   REPEATED node: offsets[e] for every entry e of the enclosing depth, plus offsets[n] =
 *                  this node's entry count (a list's elements are offsets[e] .. offsets[e+1]).
 * The leaf's non-null values are the dense values pqg_decode wrote for the column.
 * d_def_levels / d_rep_levels: the u8 levels pqg_decode wrote (NULL when the max level is 0).
 * Synchronous. When an output is too small, returns PQG_ERR_INVALID_ARG with every
 * n_entries filled in (nothing written). Outputs sized for the bound (validity: n_slots
 * entries, offsets: n_slots + 1) are written in one pass with a single synchronisation;
 * smaller ones are checked against the counted entries first (one extra round trip). */
enum pqg_repetition { PQG_REQUIRED = 0, PQG_OPTIONAL = 1, PQG_REPEATED = 2 };

typedef struct pqg_assembly_node {
  int32_t repetition;      /* pqg_repetition (parquet-format FieldRepetitionType) */
  int32_t reserved;
  uint8_t* validity;       /* OPTIONAL: 1 byte per entry; may be NULL */
  int64_t* offsets;        /* REPEATED: offsets[n_enclosing_entries + 1]; may be NULL */
  uint64_t capacity;       /* elements the validity / offsets array holds */
  uint64_t n_entries;      /* OUT: entries of this node */
} pqg_assembly_node;

int pqg_assemble(pqg_ctx* ctx, const uint8_t* d_def_levels, const uint8_t* d_rep_levels, uint64_t n_slots,
                 pqg_assembly_node* path, int depth, uint64_t* n_records, pqg_status* st);

/* Record assembly of every leaf of a schema: the columnar form of what the automaton emits when it
 * interleaves all leaves of each record (RecordReaderImplementation ctor :253-330 builds the
 * transitions between leaves — nextColumnIdxForRepLevel, levelToClose — and read() :409-446 walks
 * them). `nodes` is the schema below the message root in depth-first order, each naming its parent
 * (-1: a child of the root); `leaves` gives the levels pqg_decode wrote for each leaf node. Every
 * node's outputs (validity / offsets, as in pqg_assembly_node) come from the first leaf under it in
 * schema order; the other leaves under a node must agree on its entry count, and all leaves on the
 * record count, or the call fails with PQG_ERR_CORRUPT (st->page = the leaf, st->value_index = the
 * node). Synchronous. */
typedef struct pqg_schema_node {
  int32_t parent;          /* index of the parent node (< this index), -1 for a child of the root */
  int32_t repetition;      /* pqg_repetition */
  uint8_t* validity;       /* OPTIONAL: 1 byte per entry; may be NULL */
  int64_t* offsets;        /* REPEATED: offsets[n_enclosing_entries + 1]; may be NULL */
  uint64_t capacity;       /* elements the validity / offsets array holds */
  uint64_t n_entries;      /* OUT: entries of this node */
} pqg_schema_node;

typedef struct pqg_schema_leaf {
  int32_t node;            /* index of the leaf in `nodes` */
  int32_t reserved;
  const uint8_t* d_def_levels;  /* device, NULL when the leaf's max definition level is 0 */
  const uint8_t* d_rep_levels;  /* device, NULL when the leaf's max repetition level is 0 */
  uint64_t n_slots;
} pqg_schema_leaf;

int pqg_assemble_schema(pqg_ctx* ctx, pqg_schema_node* nodes, int n_nodes, const pqg_schema_leaf* leaves, int n_leaves,
                        uint64_t* n_records, pqg_status* st);

/* ---- page decompression (codec SNAPPY) --------------------------------------
 * Replaces the decompression step between the page reader and the value readers:
 * ColumnChunkPageReadStore.readPage (parquet-hadoop/src/main/java/org/apache/parquet/hadoop/ColumnChunkPageReadStore.java:144-172
 * for V1 pages, :218-247 for the data section of compressed V2 pages) calling
 * BytesInputDecompressor.decompress -> SnappyDecompressor (parquet-hadoop/.../hadoop/codec/SnappyDecompressor.java),
 * i.e. xerial Snappy.uncompress of one raw Snappy block into a buffer of the header's
 * uncompressed size. Job j decompresses d_src[src_offset, src_offset + src_size) into
 * d_dst[dst_offset, dst_offset + dst_size); a block whose length varint differs from dst_size
 * or that is malformed fails with PQG_ERR_CORRUPT. d_jobs is a DEVICE array; d_status (device,
 * n_jobs int32, may be NULL) receives each job's code. Asynchronous on the context's stream;
 * pqg_snappy_sync reports the first failing job (st->page = job index). */
typedef struct pqg_snappy_job {
  uint64_t src_offset;
  uint64_t dst_offset;
  uint32_t src_size;
  uint32_t dst_size;
} pqg_snappy_job;

int pqg_snappy_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                          const pqg_snappy_job* d_jobs, int n_jobs, int32_t* d_status);
int pqg_snappy_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st);

/* ---- page decompression (codec ZSTD) ------------------------------------------
 * The same step for ZSTD pages: ZstandardCodec -> ZstdDecompressorStream
 * (parquet-hadoop/src/main/java/org/apache/parquet/hadoop/codec/ZstdDecompressorStream.java:31-46,
 * zstd-jni's ZstdInputStream over libzstd) read for exactly the header's uncompressed size
 * (ColumnChunkPageReadStore.java:144-172). Job j decodes the Zstandard frames (RFC 8878; skippable
 * frames skipped, concatenated frames in order) in d_src[src_offset, + src_size) and keeps the first
 * dst_size bytes at d_dst + dst_offset. Frames that end before dst_size -> PQG_ERR_EOF; a malformed
 * frame, a frame content size or content checksum (XXH64) that does not match -> PQG_ERR_CORRUPT;
 * dictionaries are not supported (a frame naming one -> CORRUPT). Asynchronous on the context's
 * stream; the context keeps 128 KiB of device scratch per decoding wave (at most 4,096 waves, each
 * looping over the jobs: 512 MiB at most, whatever the number of pages); the output is read back
 * only inside each job's [dst_offset, dst_offset + dst_size) (no padding needed). pqg_zstd_sync reports the first
 * failing job (st->page = job index). */
typedef pqg_snappy_job pqg_zstd_job;

int pqg_zstd_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                        const pqg_zstd_job* d_jobs, int n_jobs, int32_t* d_status);
int pqg_zstd_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st);

/* LZ4_RAW pages (ColumnChunkPageReadStore.readPage -> Lz4RawDecompressor, parquet-hadoop/.../hadoop/
 * codec/Lz4RawDecompressor.java:26-50, aircompressor's Lz4Decompressor underneath): every job is one
 * raw LZ4 block (lz4 block format) decompressed into exactly dst_size bytes (the header's
 * uncompressed size; another length, or a malformed block -> PQG_ERR_CORRUPT in the job's status).
 * Same job table and calling sequence as pqg_snappy_decompress; pqg_lz4_raw_sync reports the first
 * failing job (st->page = job index). */
typedef pqg_snappy_job pqg_lz4_job;

int pqg_lz4_raw_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                           const pqg_lz4_job* d_jobs, int n_jobs, int32_t* d_status);
int pqg_lz4_raw_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st);

/* GZIP pages (ColumnChunkPageReadStore.readPage -> CodecFactory.HeapBytesDecompressor.decompress,
 * parquet-hadoop/.../hadoop/CodecFactory.java:155-182, Hadoop's GzipCodec stream read for exactly the
 * page's size): every job is gzip members (RFC 1952) of DEFLATE data (RFC 1951) read until dst_size
 * bytes are produced. The member completing the page has its trailer unread; an earlier member's ISIZE
 * is checked (its CRC-32 is not recomputed on the device). Fewer bytes than dst_size -> PQG_ERR_EOF,
 * malformed data -> PQG_ERR_CORRUPT in the job's status. Same job table and calling sequence as
 * pqg_snappy_decompress; pqg_gzip_sync reports the first failing job (st->page = job index). */
typedef pqg_snappy_job pqg_gzip_job;

int pqg_gzip_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                        const pqg_gzip_job* d_jobs, int n_jobs, int32_t* d_status);
int pqg_gzip_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st);

/* ---- page framing (host) ----------------------------------------------------
 * File bytes in: the page headers of one raw column chunk, as
 * ParquetFileReader.Chunk.readAllPages reads them
 * (parquet-hadoop/src/main/java/org/apache/parquet/hadoop/ParquetFileReader.java:1824-1979;
 * header = Thrift compact PageHeader, Util.readPageHeader,
 * parquet-format-structures/src/main/java/org/apache/parquet/format/Util.java:127-131).
 * Host code: no device needed. */
enum pqg_page_type { PQG_DATA_PAGE = 0, PQG_INDEX_PAGE = 1, PQG_DICTIONARY_PAGE = 2, PQG_DATA_PAGE_V2 = 3 };

typedef struct pqg_page_header {
  int32_t type;                          /* pqg_page_type */
  int32_t uncompressed_page_size;
  int32_t compressed_page_size;
  int32_t has_crc;
  uint32_t crc;
  int32_t num_values;                    /* data pages: slots; dictionary page: entries */
  int32_t encoding;                      /* values encoding / dictionary page encoding */
  int32_t definition_level_encoding;     /* DataPageHeader (V1) */
  int32_t repetition_level_encoding;     /* DataPageHeader (V1) */
  int32_t num_nulls;                     /* DataPageHeaderV2 */
  int32_t num_rows;                      /* DataPageHeaderV2 */
  int32_t definition_levels_byte_length; /* DataPageHeaderV2 */
  int32_t repetition_levels_byte_length; /* DataPageHeaderV2 */
  int32_t is_compressed;                 /* DataPageHeaderV2 (default 1) */
  int32_t is_sorted;                     /* DictionaryPageHeader */
  int32_t reserved;
  uint64_t header_offset;                /* offset of the header in the chunk buffer */
  uint64_t body_offset;                  /* offset of the page body (compressed_page_size bytes) */
} pqg_page_header;

/* CRC-32 (java.util.zip.CRC32) of n bytes, continuing from `crc` (0 to start). */
uint32_t pqg_crc32(uint32_t crc, const uint8_t* data, uint64_t n);

/* Walk the page headers of the chunk bytes [chunk, chunk + chunk_len) until `value_count` data
 * values have been read (ColumnMetaData.num_values; < 0: every header up to the end).
 * DICTIONARY_PAGE, DATA_PAGE and DATA_PAGE_V2 headers go to `headers` in order; other page types
 * are skipped (as readAllPages does). verify_crc != 0: pages whose header has a crc are checked
 * (CRC-32 of the page's compressed bytes) -> PQG_ERR_CRC with st->page = the page.
 * Errors: a second dictionary page, unreadable header, V2 level lengths past the page -> CORRUPT;
 * a body past the chunk -> EOF; value count mismatch at the end -> CORRUPT ("Expected N values in
 * column chunk ..."). *n_headers = headers found; capacity too small -> INVALID_ARG with
 * st->value_index = the count needed. */
int pqg_frame_chunk(const uint8_t* chunk, uint64_t chunk_len, int64_t value_count, int verify_crc,
                    pqg_page_header* headers, int capacity, int* n_headers, pqg_status* st);

/* ColumnMetaData.codec (parquet.thrift CompressionCodec; CompressionCodecName in parquet-mr). */
enum pqg_codec {
  PQG_CODEC_UNCOMPRESSED = 0, PQG_CODEC_SNAPPY = 1, PQG_CODEC_GZIP = 2, PQG_CODEC_LZO = 3,
  PQG_CODEC_BROTLI = 4, PQG_CODEC_LZ4 = 5, PQG_CODEC_ZSTD = 6, PQG_CODEC_LZ4_RAW = 7
};

/* Headers of a chunk placed at byte `chunk_offset` of a batch buffer -> the pqg_page_desc entries
 * of its data pages (column index `column`) and the dictionary fields of `col` (may be NULL).
 * `codec` is the chunk's ColumnMetaData.codec; it alone decides which pages are compressed, as
 * ColumnChunkPageReadStore.readPage does (ColumnChunkPageReadStore.java:147-181, :218-257,
 * readDictionaryPage :313-316): with a codec other than UNCOMPRESSED every V1 data page and the
 * dictionary page are compressed whatever their sizes, a V2 page when its is_compressed flag is set.
 * A compressed page -> PQG_ERR_UNSUPPORTED with st->page = its header index (decompress first:
 * pqg_snappy_decompress / pqg_zstd_decompress, then describe the decompressed layout). An
 * UNCOMPRESSED chunk's pages are taken as they are (CodecFactory.NO_OP_DECOMPRESSOR). A codec
 * outside pqg_codec -> PQG_ERR_INVALID_ARG. Replaces the page loop of
 * ParquetFileReader.Chunk.readAllPages (ParquetFileReader.java:1824-1979) + the decompressor choice. */
int pqg_pages_from_headers(const pqg_page_header* headers, int n_headers, int codec, uint64_t chunk_offset,
                           int column, pqg_column_desc* col, pqg_page_desc* pages, int capacity, int* n_pages,
                           pqg_status* st);

/* Human-readable name of an error code. */
const char* pqg_error_name(int code);

#ifdef __cplusplus
}
#endif

#endif /* PQGPU_H */
