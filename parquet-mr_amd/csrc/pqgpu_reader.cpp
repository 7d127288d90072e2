// pqgpu_reader.cpp — the ValuesReader contract over a decoded page batch (include/pqgpu_reader.h).
//
// Host code of libpqgpu.so; what the JNI shim's GpuValuesReader / GpuLevelsReader do per call. Reference:
// ValuesReader (parquet-column/src/main/java/org/apache/parquet/column/values/ValuesReader.java:36-203)
// and the readers it dispatches to (PlainValuesReader, BooleanPlainValuesReader,
// BinaryPlainValuesReader, FixedLenByteArrayPlainValuesReader, DictionaryValuesReader,
// DeltaBinaryPackingValuesReader, ...): each supports only the read of its type and throws
// UnsupportedOperationException for the others. Level readers: ColumnReaderBase.readPageV1 / readPageV2 /
// newRLEIterator (parquet-column/src/main/java/org/apache/parquet/column/impl/ColumnReaderBase.java:738-789),
// RunLengthBitPackingHybridValuesReader (.../values/rle/RunLengthBitPackingHybridValuesReader.java:40-65),
// ZeroIntegerValuesReader.
#include <cstdint>
#include <cstring>

#include "../../include/pqgpu_reader.h"

namespace {

int elem_width(int t, int tl) {
  switch (t) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return tl;
    default: return 0;
  }
}

// the next value's index, or the error raised at it
int take(pqg_values_reader* r, uint64_t* i) {
  if (r->error_code && r->pos >= r->error_at) return r->error_code;
  // past the page's values: the reference readers fail with an EOF / "past the stream" error that
  // their read methods wrap in ParquetDecodingException
  if (r->pos >= r->end) return PQG_ERR_EOF;
  *i = r->pos++;
  return PQG_OK;
}

}  // namespace

extern "C" {

int pqg_vr_init_from_page(pqg_values_reader* r, const pqg_column_desc* col, const pqg_page_desc* pages,
                          const uint32_t* page_value_counts, int n_pages, int page,
                          const pqg_page_error* page_errors) {
  if (!r || !col || !pages || !page_value_counts || page < 0 || page >= n_pages) return PQG_ERR_INVALID_ARG;
  std::memset(r, 0, sizeof(*r));
  r->physical_type = col->physical_type;
  r->type_length = col->type_length;
  r->ids = (col->flags & PQG_COLUMN_DICTIONARY_IDS) != 0;
  r->values = (const uint8_t*)col->values;
  r->binary = col->binary_data;
  const int column = pages[page].column;
  uint64_t first = 0;
  for (int p = 0; p < page; p++)
    if (pages[p].column == column) {
      // the column reader threw on an earlier page and reads no further
      if (page_errors && page_errors[p].code) return page_errors[p].code;
      first += page_value_counts[p];
    }
  r->pos = first;
  r->end = first + page_value_counts[page];
  if (page_errors && page_errors[page].code) {
    const pqg_page_error& e = page_errors[page];
    switch (e.phase) {
      case PQG_PHASE_VALUE:
        // DictionaryValuesReader / DeltaBinaryPackingValuesReader / ...: the reads before the
        // failing value succeed, the failing read throws
        r->error_code = e.code;
        r->error_at = first + (uint64_t)e.index;
        break;
      case PQG_PHASE_RL_READ:
      case PQG_PHASE_DL_READ:
        // the page's values stop at the slots before the level error (page_value_counts)
        break;
      default:  // the dictionary (ColumnReaderBase ctor) or an initFromPage threw
        return e.code;
    }
  }
  return PQG_OK;
}

int pqg_lr_init_from_page(pqg_levels_reader* r, const pqg_column_desc* col, int kind, const pqg_page_desc* pages,
                          int n_pages, int page, const pqg_page_error* page_errors) {
  if (!r || !col || !pages || page < 0 || page >= n_pages || (kind != PQG_LEVELS_REP && kind != PQG_LEVELS_DEF))
    return PQG_ERR_INVALID_ARG;
  std::memset(r, 0, sizeof(*r));
  const bool rep = kind == PQG_LEVELS_REP;
  r->max_level = rep ? col->max_rep : col->max_def;
  r->levels = r->max_level > 0 ? (rep ? col->rep_levels : col->def_levels) : nullptr;
  if (r->max_level > 0 && !r->levels) return PQG_ERR_INVALID_ARG;
  const int column = pages[page].column;
  uint64_t first = 0;
  for (int p = 0; p < page; p++)
    if (pages[p].column == column) {
      if (page_errors && page_errors[p].code) return page_errors[p].code;
      first += pages[p].num_values;
    }
  r->pos = first;
  r->end = first + pages[page].num_values;
  if (page_errors && page_errors[page].code) {
    const pqg_page_error& e = page_errors[page];
    switch (e.phase) {
      case PQG_PHASE_DICTIONARY:
      case PQG_PHASE_RL_INIT:  // readPageV1: rl init throws before the dl reader exists
        return e.code;
      case PQG_PHASE_DL_INIT:  // rl initialised, dl init throws
        if (!rep) return e.code;
        break;
      case PQG_PHASE_RL_READ:  // rl(s) throws; checkRead never reads dl(s)
        r->error_code = e.code;
        r->error_at = first + (uint64_t)e.index;
        break;
      case PQG_PHASE_DL_READ:  // rl(s) was read, dl(s) throws
        r->error_code = e.code;
        r->error_at = first + (uint64_t)e.index + (rep ? 1u : 0u);
        break;
      default:  // DATA_INIT (after both level readers) / VALUE: the levels are served
        break;
    }
  }
  return PQG_OK;
}

uint64_t pqg_lr_remaining(const pqg_levels_reader* r) { return r && r->end > r->pos ? r->end - r->pos : 0; }

int pqg_lr_read_integer(pqg_levels_reader* r, int32_t* out) {
  if (!r || !out) return PQG_ERR_INVALID_ARG;
  if (r->error_code && r->pos >= r->error_at) return r->error_code;
  if (r->max_level == 0) {  // ZeroIntegerValuesReader.readInteger / NullIntIterator.nextInt: 0, forever
    *out = 0;
    r->pos++;
    return PQG_OK;
  }
  if (r->pos >= r->end) return PQG_ERR_EOF;
  *out = r->levels[r->pos++];
  return PQG_OK;
}

int pqg_lr_skip(pqg_levels_reader* r) {
  int32_t v;
  return pqg_lr_read_integer(r, &v);
}

uint64_t pqg_vr_remaining(const pqg_values_reader* r) { return r && r->end > r->pos ? r->end - r->pos : 0; }

int pqg_vr_read_dictionary_id(pqg_values_reader* r, int32_t* out) {
  if (!r || !out) return PQG_ERR_INVALID_ARG;
  if (!r->ids) return PQG_ERR_UNSUPPORTED;
  uint64_t i;
  const int rc = take(r, &i);
  if (rc) return rc;
  std::memcpy(out, r->values + 4 * i, 4);
  return PQG_OK;
}

#define PQG_VR_FIXED(NAME, TYPE, PHYS)                                  \
  int NAME(pqg_values_reader* r, TYPE* out) {                           \
    if (!r || !out) return PQG_ERR_INVALID_ARG;                         \
    if (r->ids || r->physical_type != (PHYS)) return PQG_ERR_UNSUPPORTED; \
    uint64_t i;                                                         \
    const int rc = take(r, &i);                                         \
    if (rc) return rc;                                                  \
    std::memcpy(out, r->values + sizeof(TYPE) * i, sizeof(TYPE));       \
    return PQG_OK;                                                      \
  }

PQG_VR_FIXED(pqg_vr_read_integer, int32_t, PQG_INT32)
PQG_VR_FIXED(pqg_vr_read_long, int64_t, PQG_INT64)
PQG_VR_FIXED(pqg_vr_read_float, float, PQG_FLOAT)
PQG_VR_FIXED(pqg_vr_read_double, double, PQG_DOUBLE)
#undef PQG_VR_FIXED

int pqg_vr_read_boolean(pqg_values_reader* r, int32_t* out) {
  if (!r || !out) return PQG_ERR_INVALID_ARG;
  if (r->ids || r->physical_type != PQG_BOOLEAN) return PQG_ERR_UNSUPPORTED;
  uint64_t i;
  const int rc = take(r, &i);
  if (rc) return rc;
  *out = r->values[i] != 0;
  return PQG_OK;
}

int pqg_vr_read_bytes(pqg_values_reader* r, const uint8_t** data, uint32_t* len) {
  if (!r || !data || !len) return PQG_ERR_INVALID_ARG;
  const int t = r->physical_type;
  if (r->ids || (t != PQG_BYTE_ARRAY && t != PQG_FIXED_LEN_BYTE_ARRAY && t != PQG_INT96)) return PQG_ERR_UNSUPPORTED;
  uint64_t i;
  const int rc = take(r, &i);
  if (rc) return rc;
  if (t == PQG_BYTE_ARRAY) {
    int64_t a, b;
    std::memcpy(&a, r->values + 8 * i, 8);
    std::memcpy(&b, r->values + 8 * (i + 1), 8);
    *data = r->binary + a;
    *len = (uint32_t)(b - a);
  } else {
    const int w = elem_width(t, r->type_length);
    *data = r->values + (uint64_t)w * i;
    *len = (uint32_t)w;
  }
  return PQG_OK;
}

int pqg_vr_skip(pqg_values_reader* r) {
  if (!r) return PQG_ERR_INVALID_ARG;
  uint64_t i;
  return take(r, &i);
}

int pqg_vr_skip_n(pqg_values_reader* r, uint64_t n) {
  // ValuesReader.skip(int n): skip() n times (:198-203) — stops at the first failing skip
  if (!r) return PQG_ERR_INVALID_ARG;
  uint64_t lim = r->end > r->pos ? r->end - r->pos : 0;  // skips that succeed
  if (r->error_code && r->error_at >= r->pos && r->error_at - r->pos < lim) lim = r->error_at - r->pos;
  if (n <= lim) {
    r->pos += n;
    return PQG_OK;
  }
  r->pos += lim;
  uint64_t i;
  return take(r, &i);  // the failing skip
}

const char* pqg_java_exception(int code) {
  switch (code) {
    case PQG_OK: return nullptr;
    case PQG_ERR_UNSUPPORTED: return "java/lang/UnsupportedOperationException";
    case PQG_ERR_RLE_PAST_END:  // RunLengthBitPackingHybridDecoder.readNext :81 checkArgument
    case PQG_ERR_BIT_WIDTH:     // RunLengthBitPackingHybridDecoder ctor :55
    case PQG_ERR_DELTA_CONFIG:  // DeltaBinaryPackingConfig :39
      return "java/lang/IllegalArgumentException";
    case PQG_ERR_DICT_ID:          // Dictionary.decodeToX array access
    case PQG_ERR_EMPTY_PACKED_RUN: // currentBuffer[] of length 0
      return "java/lang/ArrayIndexOutOfBoundsException";
    case PQG_ERR_EOF:            // EOFException, wrapped by the readers' read methods
    case PQG_ERR_EMPTY_PAGE:     // IOException "Attempt to read from empty page", wrapped
    case PQG_ERR_DELTA_PAST_END:
    case PQG_ERR_CORRUPT:
    case PQG_ERR_NO_DICTIONARY:
    case PQG_ERR_DICT_ENCODING:
    case PQG_ERR_CRC:
      return "org/apache/parquet/io/ParquetDecodingException";
    case PQG_ERR_INVALID_ARG: return "java/lang/IllegalArgumentException";
    default:  // PQG_ERR_HIP, PQG_ERR_NO_DEVICE, PQG_ERR_TIMEOUT: the native backend failed, not the data
      return "java/lang/IllegalStateException";
  }
}

}  // extern "C"
