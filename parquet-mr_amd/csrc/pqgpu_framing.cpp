// pqgpu_framing.cpp — page framing of a raw column chunk (host code of libpqgpu.so).
//
// Restates ParquetFileReader.Chunk.readAllPages
// (parquet-hadoop/src/main/java/org/apache/parquet/hadoop/ParquetFileReader.java:1824-1979):
// page headers are read one after another (Util.readPageHeader,
// parquet-format-structures/src/main/java/org/apache/parquet/format/Util.java:127-131, Thrift
// TCompactProtocol over the parquet.thrift PageHeader) until the chunk's value count is reached;
// DICTIONARY_PAGE / DATA_PAGE / DATA_PAGE_V2 are kept, other page types skipped; with checksum
// verification on, each page's stored CRC32 is compared with the CRC32 of its (compressed) bytes
// (verifyCrc :1805-1813; V2: the level sections and the values together :1925-1931).
//
// The Thrift walk is a plain recursive-descent reader of the compact protocol: only PageHeader's
// fields are interpreted, everything else (statistics, unknown fields) is skipped by type.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/pqgpu.h"

namespace {

void pqg_set_status(pqg_status* st, int code, int page, int64_t idx, const char* what) {
  if (!st) return;
  st->code = code;
  st->page = page;
  st->value_index = idx;
  std::snprintf(st->message, sizeof(st->message), "%s", what);
}

enum : int { T_STOP = 0, T_TRUE = 1, T_FALSE = 2, T_BYTE = 3, T_I16 = 4, T_I32 = 5, T_I64 = 6, T_DOUBLE = 7,
             T_BINARY = 8, T_LIST = 9, T_SET = 10, T_MAP = 11, T_STRUCT = 12 };

struct ThriftReader {
  const uint8_t* p;
  uint64_t pos, end;
  bool bad = false;
  int depth = 0;

  uint32_t byte() {
    if (pos >= end) { bad = true; return 0; }
    return p[pos++];
  }
  uint64_t varint() {
    uint64_t r = 0;
    for (int shift = 0; shift < 70; shift += 7) {
      const uint32_t b = byte();
      if (bad) return 0;
      r |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return r;
    }
    bad = true;
    return 0;
  }
  int64_t zigzag() {
    const uint64_t n = varint();
    return (int64_t)(n >> 1) ^ -(int64_t)(n & 1);
  }
  void skip(int t) {
    if (++depth > 64) { bad = true; return; }
    switch (t) {
      case T_TRUE: case T_FALSE: break;
      case T_BYTE: byte(); break;
      case T_I16: case T_I32: case T_I64: varint(); break;
      case T_DOUBLE: if (end - pos < 8) bad = true; else pos += 8; break;
      case T_BINARY: {
        const uint64_t n = varint();
        if (n > end - pos) bad = true; else pos += n;
        break;
      }
      case T_LIST: case T_SET: {
        const uint32_t h = byte();
        uint64_t n = h >> 4;
        if (n == 15) n = varint();
        for (uint64_t i = 0; i < n && !bad; i++) skip((int)(h & 15));
        break;
      }
      case T_MAP: {
        const uint64_t n = varint();
        if (n) {
          const uint32_t kv = byte();
          for (uint64_t i = 0; i < n && !bad; i++) { skip((int)(kv >> 4)); skip((int)(kv & 15)); }
        }
        break;
      }
      case T_STRUCT: struct_fields([](int, int, ThriftReader&) { return false; }); break;
      default: bad = true;
    }
    depth--;
  }
  // on(fid, type, reader) -> true when it consumed the value
  template <class F>
  void struct_fields(F&& on) {
    int16_t last = 0;
    while (!bad) {
      const uint32_t h = byte();
      if (bad) return;
      const int t = (int)(h & 15);
      if (t == T_STOP) return;
      const int delta = (int)(h >> 4);
      const int16_t fid = delta ? (int16_t)(last + delta) : (int16_t)zigzag();
      last = fid;
      if (!on(fid, t, *this)) skip(t);
    }
  }
};

// i32 field value (compact protocol: zigzag varint); false for another type
bool i32_field(int t, ThriftReader& r, int32_t& out) {
  if (t != T_I32 && t != T_I16 && t != T_I64) return false;
  out = (int32_t)r.zigzag();
  return true;
}

// Util.readPageHeader: one PageHeader at r.pos.
bool read_page_header(ThriftReader& r, pqg_page_header& h, bool& has_type, bool& has_csize) {
  std::memset(&h, 0, sizeof(h));
  h.is_compressed = 1;  // DataPageHeaderV2.is_compressed defaults to true (parquet.thrift)
  has_type = has_csize = false;
  r.struct_fields([&](int fid, int t, ThriftReader& rr) {
    switch (fid) {
      case 1: has_type = i32_field(t, rr, h.type); return has_type;
      case 2: return i32_field(t, rr, h.uncompressed_page_size);
      case 3: has_csize = i32_field(t, rr, h.compressed_page_size); return has_csize;
      case 4: {
        int32_t c;
        if (!i32_field(t, rr, c)) return false;
        h.has_crc = 1;
        h.crc = (uint32_t)c;
        return true;
      }
      case 5:  // DataPageHeader
        if (t != T_STRUCT) return false;
        rr.struct_fields([&](int f, int tt, ThriftReader& q) {
          switch (f) {
            case 1: return i32_field(tt, q, h.num_values);
            case 2: return i32_field(tt, q, h.encoding);
            case 3: return i32_field(tt, q, h.definition_level_encoding);
            case 4: return i32_field(tt, q, h.repetition_level_encoding);
            default: return false;
          }
        });
        return true;
      case 7:  // DictionaryPageHeader
        if (t != T_STRUCT) return false;
        rr.struct_fields([&](int f, int tt, ThriftReader& q) {
          switch (f) {
            case 1: return i32_field(tt, q, h.num_values);
            case 2: return i32_field(tt, q, h.encoding);
            case 3: if (tt == T_TRUE || tt == T_FALSE) { h.is_sorted = tt == T_TRUE; return true; } return false;
            default: return false;
          }
        });
        return true;
      case 8:  // DataPageHeaderV2
        if (t != T_STRUCT) return false;
        rr.struct_fields([&](int f, int tt, ThriftReader& q) {
          switch (f) {
            case 1: return i32_field(tt, q, h.num_values);
            case 2: return i32_field(tt, q, h.num_nulls);
            case 3: return i32_field(tt, q, h.num_rows);
            case 4: return i32_field(tt, q, h.encoding);
            case 5: return i32_field(tt, q, h.definition_levels_byte_length);
            case 6: return i32_field(tt, q, h.repetition_levels_byte_length);
            case 7: if (tt == T_TRUE || tt == T_FALSE) { h.is_compressed = tt == T_TRUE; return true; } return false;
            default: return false;
          }
        });
        return true;
      default: return false;
    }
  });
  return !r.bad && has_type && has_csize;
}

// CRC-32 (IEEE 802.3, reflected 0xEDB88320) — java.util.zip.CRC32, which verifyCrc uses.
// Slicing by 8: eight 256-entry tables, 8 bytes per step.
struct Crc32Tables {
  uint32_t t[8][256];
  Crc32Tables() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
      for (int s = 1; s < 8; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Crc32Tables& crc_tables() {
  static const Crc32Tables tabs;
  return tabs;
}

}  // namespace

extern "C" {

uint32_t pqg_crc32(uint32_t crc, const uint8_t* data, uint64_t n) {
  const Crc32Tables& T = crc_tables();
  uint32_t c = ~crc;
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, data + i, 4);
    std::memcpy(&hi, data + i + 4, 4);
    lo ^= c;
    c = T.t[7][lo & 0xFF] ^ T.t[6][(lo >> 8) & 0xFF] ^ T.t[5][(lo >> 16) & 0xFF] ^ T.t[4][lo >> 24] ^
        T.t[3][hi & 0xFF] ^ T.t[2][(hi >> 8) & 0xFF] ^ T.t[1][(hi >> 16) & 0xFF] ^ T.t[0][hi >> 24];
  }
  for (; i < n; i++) c = T.t[0][(c ^ data[i]) & 0xFF] ^ (c >> 8);
  return ~c;
}

int pqg_frame_chunk(const uint8_t* chunk, uint64_t chunk_len, int64_t value_count, int verify_crc,
                    pqg_page_header* headers, int capacity, int* n_headers, pqg_status* st) {
  if (st) std::memset(st, 0, sizeof(*st));
  if ((!chunk && chunk_len) || !n_headers || capacity < 0 || (capacity > 0 && !headers)) {
    pqg_set_status(st, PQG_ERR_INVALID_ARG, -1, -1, "pqg_frame_chunk: bad arguments");
    return PQG_ERR_INVALID_ARG;
  }
  *n_headers = 0;
  uint64_t pos = 0;
  int64_t seen = 0;
  int n = 0, n_pages_read = 0;
  bool have_dict = false;
  // hasMorePages (:1981-1985) without an offset index: until the chunk's value count is read;
  // value_count < 0: every page header up to the end of the buffer
  while (value_count >= 0 ? seen < value_count : pos < chunk_len) {
    ThriftReader r{chunk, pos, chunk_len};
    pqg_page_header h;
    bool has_type, has_csize;
    if (!read_page_header(r, h, has_type, has_csize)) {
      char msg[160];
      std::snprintf(msg, sizeof(msg), "could not read page header at chunk offset %llu (%s)",
                    (unsigned long long)pos, pos >= chunk_len ? "end of chunk" :
                    (!r.bad && (!has_type || !has_csize)) ? "required field missing" : "truncated / invalid thrift");
      pqg_set_status(st, pos >= chunk_len ? PQG_ERR_EOF : PQG_ERR_CORRUPT, n_pages_read, (int64_t)pos, msg);
      *n_headers = n;
      return st ? st->code : PQG_ERR_CORRUPT;
    }
    h.header_offset = pos;
    h.body_offset = r.pos;
    if (h.compressed_page_size < 0 || (uint64_t)h.compressed_page_size > chunk_len - r.pos) {
      // readAsBytesInput of more bytes than the chunk holds: EOFException
      pqg_set_status(st, PQG_ERR_EOF, n_pages_read, (int64_t)pos, "page body runs past the end of the column chunk");
      *n_headers = n;
      return PQG_ERR_EOF;
    }
    const uint8_t* body = chunk + r.pos;
    pos = r.pos + (uint64_t)h.compressed_page_size;
    const bool keep = h.type == PQG_DICTIONARY_PAGE || h.type == PQG_DATA_PAGE || h.type == PQG_DATA_PAGE_V2;
    if (!keep) continue;  // "skipping page of type ..." (:1952-1955)
    if (h.type == PQG_DICTIONARY_PAGE) {
      if (have_dict) {
        pqg_set_status(st, PQG_ERR_CORRUPT, n_pages_read, (int64_t)h.header_offset,
                       "more than one dictionary page in column");
        *n_headers = n;
        return PQG_ERR_CORRUPT;
      }
      have_dict = true;
    } else {
      if (h.type == PQG_DATA_PAGE_V2 &&
          (h.repetition_levels_byte_length < 0 || h.definition_levels_byte_length < 0 ||
           (int64_t)h.repetition_levels_byte_length + h.definition_levels_byte_length > h.compressed_page_size)) {
        pqg_set_status(st, PQG_ERR_CORRUPT, n_pages_read, (int64_t)h.header_offset,
                       "DataPageV2 level byte lengths exceed the page");
        *n_headers = n;
        return PQG_ERR_CORRUPT;
      }
      seen += h.num_values;
    }
    if (verify_crc && h.has_crc && pqg_crc32(0, body, (uint64_t)h.compressed_page_size) != h.crc) {
      pqg_set_status(st, PQG_ERR_CRC, n_pages_read, (int64_t)h.header_offset,
                     h.type == PQG_DICTIONARY_PAGE
                         ? "could not verify dictionary page integrity, CRC checksum verification failed"
                         : "could not verify page integrity, CRC checksum verification failed");
      *n_headers = n;
      return PQG_ERR_CRC;
    }
    if (n < capacity) headers[n] = h;
    n++;
    n_pages_read++;
  }
  *n_headers = n;
  if (value_count >= 0 && seen != value_count) {
    char msg[160];
    std::snprintf(msg, sizeof(msg), "Expected %lld values in column chunk but got %lld values instead over %d pages",
                  (long long)value_count, (long long)seen, n);
    pqg_set_status(st, PQG_ERR_CORRUPT, -1, -1, msg);
    return PQG_ERR_CORRUPT;
  }
  if (n > capacity) {
    pqg_set_status(st, PQG_ERR_INVALID_ARG, -1, n, "pqg_frame_chunk: header capacity too small (value_index = needed)");
    return PQG_ERR_INVALID_ARG;
  }
  return PQG_OK;
}

int pqg_pages_from_headers(const pqg_page_header* headers, int n_headers, int codec, uint64_t chunk_offset,
                           int column, pqg_column_desc* col, pqg_page_desc* pages, int capacity, int* n_pages,
                           pqg_status* st) {
  if (st) std::memset(st, 0, sizeof(*st));
  if ((n_headers > 0 && !headers) || !n_pages || capacity < 0 || (capacity > 0 && !pages) || codec < PQG_CODEC_UNCOMPRESSED ||
      codec > PQG_CODEC_LZ4_RAW) {
    pqg_set_status(st, PQG_ERR_INVALID_ARG, -1, -1, "pqg_pages_from_headers: bad arguments");
    return PQG_ERR_INVALID_ARG;
  }
  int n = 0;
  for (int i = 0; i < n_headers; i++) {
    const pqg_page_header& h = headers[i];
    // Whether the page body goes through the chunk's decompressor is decided by the codec, never by
    // the sizes (ColumnChunkPageReadStore.readPage): a V1 data page (:147-181) and the dictionary
    // page (readDictionaryPage :313-316) always do; a V2 page only when is_compressed (:218, :232,
    // :253). UNCOMPRESSED is CodecFactory.NO_OP_DECOMPRESSOR (CodecFactory.java:60-83), whose
    // BytesInput form returns the bytes as they are. A compressed page must be decompressed first
    // (pqg_snappy / zstd / lz4_raw / gzip_decompress) into a layout of its own.
    const bool compressed = codec != PQG_CODEC_UNCOMPRESSED && (h.type != PQG_DATA_PAGE_V2 || h.is_compressed);
    if (compressed && (h.type == PQG_DICTIONARY_PAGE || h.type == PQG_DATA_PAGE || h.type == PQG_DATA_PAGE_V2)) {
      pqg_set_status(st, PQG_ERR_UNSUPPORTED, i, -1,
                     "compressed page: decompress the chunk (pqg_snappy / zstd / lz4_raw / gzip_decompress) and "
                     "describe the decompressed pages");
      return PQG_ERR_UNSUPPORTED;
    }
    if (h.type == PQG_DICTIONARY_PAGE) {
      if (col) {
        col->dict_offset = (int64_t)(chunk_offset + h.body_offset);
        col->dict_size = (uint32_t)h.compressed_page_size;
        col->dict_num_values = (uint32_t)h.num_values;
        col->dict_encoding = h.encoding;
      }
      continue;
    }
    if (h.type != PQG_DATA_PAGE && h.type != PQG_DATA_PAGE_V2) continue;
    if (n < capacity) {
      pqg_page_desc& p = pages[n];
      std::memset(&p, 0, sizeof(p));
      p.offset = chunk_offset + h.body_offset;
      p.size = (uint32_t)h.compressed_page_size;
      p.num_values = (uint32_t)h.num_values;
      p.column = column;
      p.version = h.type == PQG_DATA_PAGE_V2 ? 2 : 1;
      p.encoding = h.encoding;
      p.rl_encoding = h.repetition_level_encoding;
      p.dl_encoding = h.definition_level_encoding;
      p.rl_byte_length = (uint32_t)h.repetition_levels_byte_length;
      p.dl_byte_length = (uint32_t)h.definition_levels_byte_length;
      if (p.version == 2 && h.num_nulls >= 0) {  // DataPageV2.getNullCount: a hint the decoder verifies
        p.flags |= PQG_PAGE_NULL_COUNT;
        p.num_nulls = (uint32_t)h.num_nulls;
      }
    }
    n++;
  }
  *n_pages = n;
  if (n > capacity) {
    pqg_set_status(st, PQG_ERR_INVALID_ARG, -1, n, "pqg_pages_from_headers: page capacity too small (value_index = needed)");
    return PQG_ERR_INVALID_ARG;
  }
  return PQG_OK;
}

}  // extern "C"
