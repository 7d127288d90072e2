/*
 * pqref.c — ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, value-at-a-time restatement of apache/parquet-mr's page readers
 * (1.15.0-SNAPSHOT, /root/reference). It is the checker for the MI355X decoder
 * and the CPU baseline that bench.py times beside it; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product path (libpqgpu.so) never links or calls anything in this directory.
 *
 * Pinning: the reference is Java and cannot be built or run here (no JDK, no
 * Maven). This restatement is pinned by the reference's own
 * known-answer tests and round trips (tests/test_oracle_*.py), by the
 * parquet-mr-written fixture files under parquet-hadoop/src/test/resources
 * (copied to tests/golden/, decoded here and compared with the values pyarrow
 * reads from the same files), and by pyarrow-written pages as an independent
 * writer. See DESIGN.md "Oracle".
 *
 * Every function names the Java method (file:line) it follows. Java integer
 * semantics are kept where they change results: `<<` masks its shift count,
 * int arithmetic wraps, RLE values are not masked to the bit width, a
 * truncated final bit-packed group is zero-filled, and DELTA sums wrap mod 2^64.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#include "../include/pqgpu.h"
#include "pqref.h"

/* ------------------------------------------------------------------------ */
/* L0 byte stream: SingleBufferInputStream (parquet-common/.../bytes/SingleBufferInputStream.java) */

typedef struct {
  const uint8_t* buf;
  int64_t pos;
  int64_t end;
} jstream;

static inline int64_t js_available(const jstream* s) { return s->end - s->pos; }

/* SingleBufferInputStream.read :50-55 — EOFException at end. */
static inline int js_read(jstream* s, int* b) {
  if (s->pos >= s->end) return PQG_ERR_EOF;
  *b = s->buf[s->pos++];
  return PQG_OK;
}

/* SingleBufferInputStream.slice :114-125 — EOFException when fewer than
 * `length` bytes remain; a negative length makes ByteBuffer.limit throw
 * IllegalArgumentException (reported as PQG_ERR_CORRUPT). */
static int js_slice(jstream* s, int64_t length, jstream* out) {
  if (length < 0) return PQG_ERR_CORRUPT;
  if (js_available(s) < length) return PQG_ERR_EOF;
  out->buf = s->buf;
  out->pos = s->pos;
  out->end = s->pos + length;
  s->pos += length;
  return PQG_OK;
}

/* ------------------------------------------------------------------------ */
/* BytesUtils (parquet-common/.../bytes/BytesUtils.java) */

/* getWidthFromMaxInt :49-51 */
int pqr_width_from_max_int(int32_t bound) {
  uint32_t b = (uint32_t)bound;
  int w = 0;
  while (b) { w++; b >>= 1; }
  return w;
}

/* readIntLittleEndian(InputStream) :86-95 */
static int read_int_le(jstream* s, int32_t* out) {
  if (js_available(s) < 4) { s->pos = s->end; return PQG_ERR_EOF; }
  const uint8_t* p = s->buf + s->pos;
  *out = (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
  s->pos += 4;
  return PQG_OK;
}

/* readIntLittleEndianPaddedOnBitWidth :124-142 — ceil(w/8) bytes, NOT masked to w. */
static int read_int_le_padded(jstream* s, int bit_width, int32_t* out) {
  int bytes = (bit_width + 7) / 8;
  uint32_t v = 0;
  for (int i = 0; i < bytes; i++) {
    int b;
    int e = js_read(s, &b);
    if (e) return e;
    v |= (uint32_t)b << (8 * i);
  }
  *out = (int32_t)v;
  return PQG_OK;
}

/* readUnsignedVarInt :202-211 — Java int `<<` masks the shift count to 5 bits. */
static int read_uvarint(jstream* s, int32_t* out) {
  uint32_t value = 0;
  int i = 0, b, e;
  for (;;) {
    if ((e = js_read(s, &b))) return e;
    if ((b & 0x80) == 0) break;
    value |= (uint32_t)(b & 0x7F) << (i & 31);
    i += 7;
  }
  *out = (int32_t)(value | ((uint32_t)b << (i & 31)));
  return PQG_OK;
}

/* readUnsignedVarLong :260-269 — Java long `<<` masks the shift count to 6 bits. */
static int read_uvarlong(jstream* s, int64_t* out) {
  uint64_t value = 0;
  int i = 0, b, e;
  for (;;) {
    if ((e = js_read(s, &b))) return e;
    if ((b & 0x80) == 0) break;
    value |= (uint64_t)(b & 0x7F) << (i & 63);
    i += 7;
  }
  *out = (int64_t)(value | ((uint64_t)b << (i & 63)));
  return PQG_OK;
}

/* readZigZagVarLong :254-258 */
static int read_zigzag_varlong(jstream* s, int64_t* out) {
  int64_t raw;
  int e = read_uvarlong(s, &raw);
  if (e) return e;
  uint64_t r = (uint64_t)raw;
  int64_t sign = -(int64_t)(r & 1);                        /* (raw << 63) >> 63 */
  int64_t temp = ((int64_t)((uint64_t)sign ^ r)) >> 1;     /* arithmetic >> of a Java long */
  *out = (int64_t)((uint64_t)temp ^ (r & 0x8000000000000000ULL));
  return PQG_OK;
}

/* ------------------------------------------------------------------------ */
/* L1 bit unpackers: Packer.LITTLE_ENDIAN (parquet-encoding/.../Packer.java:56-86),
 * generated code per ByteBasedBitPackingGenerator.generateUnpack :258-308 with
 * getShift's LSB-first branch :160-167: value i occupies bits [i*w, (i+1)*w) of
 * the input, byte 0 bit 0 first. Width 0 writes nothing (:264). */

void pqr_unpack8_int(int w, const uint8_t* in, int32_t* out) {
  if (w == 0) return;
  for (int i = 0; i < 8; i++) {
    int bit = i * w;
    uint64_t acc = 0;
    int first = bit >> 3, last = (bit + w - 1) >> 3;
    for (int b = first; b <= last; b++) acc |= (uint64_t)in[b] << (8 * (b - first));
    acc >>= (bit & 7);
    out[i] = (int32_t)(uint32_t)(w == 32 ? acc : (acc & ((1ULL << w) - 1)));
  }
}

void pqr_unpack8_long(int w, const uint8_t* in, int64_t* out) {
  if (w == 0) return;
  for (int i = 0; i < 8; i++) {
    int bit = i * w;
    uint64_t v = 0;
    for (int k = 0; k < w; k++) {
      int pb = bit + k;
      v |= (uint64_t)((in[pb >> 3] >> (pb & 7)) & 1) << k;
    }
    out[i] = (int64_t)v;
  }
}

/* ------------------------------------------------------------------------ */
/* RunLengthBitPackingHybridDecoder (parquet-column/.../rle/RunLengthBitPackingHybridDecoder.java) */

enum { MODE_NONE = 0, MODE_RLE = 1, MODE_PACKED = 2 };

typedef struct {
  int bit_width;
  jstream in;
  int mode;
  int32_t current_count;   /* Java int semantics, may go negative (zero-count RLE run) */
  int32_t current_value;
  /* PACKED: the run's bytes are unpacked lazily (same values as unpack8Values
   * over the zero-padded byte[] of :95-103) */
  int64_t packed_pos;      /* stream offset of the run's first data byte */
  int64_t packed_avail;    /* bytes actually present (readFully of min(needed, available)) */
  int32_t packed_len;      /* currentBuffer.length = numGroups*8 */
  int empty_page;          /* DictionaryValuesReader :57-62 stand-in decoder */
} rle_dec;

/* ctor :52-59 */
static int rle_init(rle_dec* d, int bit_width, jstream in) {
  memset(d, 0, sizeof(*d));
  if (bit_width < 0 || bit_width > 32) return PQG_ERR_BIT_WIDTH;
  d->bit_width = bit_width;
  d->in = in;
  return PQG_OK;
}

static inline uint32_t packed_value(const rle_dec* d, int32_t idx) {
  int w = d->bit_width;
  if (w == 0) return 0;
  int64_t bit = (int64_t)idx * w;
  uint64_t acc = 0;
  int64_t first = bit >> 3, last = (bit + w - 1) >> 3;
  for (int64_t b = first; b <= last; b++) {
    uint64_t byte = (b < d->packed_avail) ? d->in.buf[d->packed_pos + b] : 0; /* zero fill :96-99 */
    acc |= byte << (8 * (b - first));
  }
  acc >>= (bit & 7);
  return (uint32_t)(w == 32 ? acc : (acc & ((1ULL << w) - 1)));
}

/* readNext :80-109 */
static int rle_read_next(rle_dec* d) {
  if (js_available(&d->in) <= 0) return PQG_ERR_RLE_PAST_END;    /* :81 */
  int32_t header;
  int e = read_uvarint(&d->in, &header);
  if (e) return e;
  if ((header & 1) == 0) {
    d->mode = MODE_RLE;
    d->current_count = (int32_t)((uint32_t)header >> 1);          /* :86 */
    e = read_int_le_padded(&d->in, d->bit_width, &d->current_value); /* :88 */
    if (e) return e;
  } else {
    d->mode = MODE_PACKED;
    uint32_t num_groups = (uint32_t)header >> 1;
    if (num_groups >= (1u << 28)) return PQG_ERR_CORRUPT;        /* Java: int overflow / NegativeArraySize */
    d->current_count = (int32_t)(num_groups * 8);                 /* :92 */
    d->packed_len = d->current_count;
    int64_t bytes_to_read = ((int64_t)d->current_count * d->bit_width + 7) / 8; /* :97 */
    int64_t avail = js_available(&d->in);
    if (bytes_to_read > avail) bytes_to_read = avail;              /* :98 */
    d->packed_pos = d->in.pos;
    d->packed_avail = bytes_to_read;
    d->in.pos += bytes_to_read;                                    /* readFully :99 */
  }
  return PQG_OK;
}

/* readInt :61-78 */
static int rle_read_int(rle_dec* d, int32_t* out) {
  if (d->empty_page) return PQG_ERR_EMPTY_PAGE;
  if (d->current_count == 0) {
    int e = rle_read_next(d);
    if (e) return e;
  }
  --d->current_count;
  if (d->mode == MODE_RLE) {
    *out = d->current_value;
  } else {
    int64_t idx = (int64_t)d->packed_len - 1 - d->current_count;  /* :71 */
    if (idx < 0 || idx >= d->packed_len) return PQG_ERR_EMPTY_PACKED_RUN;
    *out = (int32_t)packed_value(d, (int32_t)idx);
  }
  return PQG_OK;
}

/* Public single-stream decode used by the known-answer tests:
 * decodes n ints like n calls of readInt(); returns the first error and the
 * index of the value that raised it. */
int pqr_rle_decode(int bit_width, const uint8_t* buf, int64_t len, int64_t n, int32_t* out,
                   int64_t* err_index, int64_t* consumed) {
  rle_dec d;
  jstream s = {buf, 0, len};
  int e = rle_init(&d, bit_width, s);
  if (e) { if (err_index) *err_index = 0; return e; }
  for (int64_t i = 0; i < n; i++) {
    e = rle_read_int(&d, &out[i]);
    if (e) { if (err_index) *err_index = i; if (consumed) *consumed = d.in.pos; return e; }
  }
  if (consumed) *consumed = d.in.pos;
  return PQG_OK;
}

/* ParquetReadRouter.readBatch (parquet-plugins/.../ParquetReadRouter.java:107-116):
 * per 8 values in.slice(bitWidth) then unpack8Values. Returns bytes consumed or <0. */
int64_t pqr_router_read_batch(int bit_width, const uint8_t* in, int64_t in_len, int count, int32_t* out) {
  int64_t pos = 0;
  for (int v = 0; v < count; v += 8) {
    if (in_len - pos < bit_width) return -PQG_ERR_EOF;
    pqr_unpack8_int(bit_width, in + pos, out + v);
    pos += bit_width;
  }
  return pos;
}

/* ------------------------------------------------------------------------ */
/* Dictionaries: PlainValuesDictionary (parquet-column/.../dictionary/PlainValuesDictionary.java) */

typedef struct {
  int present;
  int physical_type;
  int elem_width;           /* fixed-width types */
  uint32_t n;
  const uint8_t* fixed;     /* n * elem_width bytes (LE, in the page) */
  const uint8_t** bin_ptr;  /* BYTE_ARRAY entries */
  int32_t* bin_len;
} jdict;

static int elem_width_of(int physical_type, int type_length) {
  switch (physical_type) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return type_length;
    default: return 0;
  }
}

/* PlainValuesDictionary ctor :47-53, Plain{Long,Integer,Double,Float}Dictionary
 * :147-156/:231-240/:189-198/:273-282 (LittleEndianDataInputStream reads; EOF when
 * short), PlainBinaryDictionary :87-113 (length-prefixed or fixed length). */
static int dict_init(jdict* D, const pqg_column_desc* c, const uint8_t* bytes) {
  memset(D, 0, sizeof(*D));
  if (c->dict_offset < 0) return PQG_OK;
  D->present = 1;
  if (c->dict_encoding != PQG_PLAIN && c->dict_encoding != PQG_PLAIN_DICTIONARY) return PQG_ERR_DICT_ENCODING;
  D->physical_type = c->physical_type;
  D->n = c->dict_num_values;
  const uint8_t* p = bytes + c->dict_offset;
  int64_t size = c->dict_size;
  switch (c->physical_type) {
    case PQG_INT32: case PQG_INT64: case PQG_FLOAT: case PQG_DOUBLE:
    case PQG_INT96: case PQG_FIXED_LEN_BYTE_ARRAY: {
      int w = elem_width_of(c->physical_type, c->type_length);
      if (c->physical_type == PQG_FIXED_LEN_BYTE_ARRAY && w <= 0) return PQG_ERR_CORRUPT; /* :107 */
      D->elem_width = w;
      if ((int64_t)D->n * w > size) {
        /* INT32/INT64/FLOAT/DOUBLE: readInt/readLong EOF. FLBA/INT96: Binary.fromConstantByteBuffer
         * over the buffer past its limit -> IndexOutOfBounds; both are a short page. */
        return PQG_ERR_EOF;
      }
      D->fixed = p;
      return PQG_OK;
    }
    case PQG_BYTE_ARRAY: {
      D->bin_ptr = (const uint8_t**)malloc(sizeof(uint8_t*) * (D->n ? D->n : 1));
      D->bin_len = (int32_t*)malloc(sizeof(int32_t) * (D->n ? D->n : 1));
      int64_t off = 0;
      for (uint32_t i = 0; i < D->n; i++) {
        if (off + 4 > size) return PQG_ERR_EOF;
        int32_t len = (int32_t)((uint32_t)p[off] | ((uint32_t)p[off + 1] << 8) |
                                ((uint32_t)p[off + 2] << 16) | ((uint32_t)p[off + 3] << 24));
        off += 4;
        if (len < 0 || off + len > size) return PQG_ERR_CORRUPT;
        D->bin_ptr[i] = p + off;
        D->bin_len[i] = len;
        off += len;
      }
      return PQG_OK;
    }
    default:
      return PQG_ERR_UNSUPPORTED; /* Encoding.PLAIN.initDictionary :106-108 (BOOLEAN) */
  }
}

static void dict_free(jdict* D) {
  free(D->bin_ptr);
  free(D->bin_len);
  D->bin_ptr = NULL;
  D->bin_len = NULL;
}

/* ------------------------------------------------------------------------ */
/* Output sink: dense values, Java-equivalent order. */

typedef struct {
  pqg_column_desc* c;
  int elem_width;
  uint64_t n_values;        /* values written so far (column) */
  uint64_t n_slots;         /* level slots written so far (column) */
  uint64_t bin_bytes;       /* BYTE_ARRAY bytes written */
  jdict dict;
  int dict_err;
  int dict_checked;
  /* the previous page's data reader (ColumnReaderBase.initDataReader :702, previousReader): its kind and,
   * for DELTA_BYTE_ARRAY, its `previous` value (PARQUET-246 carry-over, PQG_PAGE_DBA_CARRY) */
  int last_kind;            /* 0: no page yet */
  uint8_t* dba_prev;
  int64_t dba_prev_len;
} colstate;

static int emit_fixed(colstate* cs, const uint8_t* src) {
  if (cs->n_values >= cs->c->values_capacity) return PQG_ERR_INVALID_ARG;
  memcpy((uint8_t*)cs->c->values + cs->n_values * cs->elem_width, src, cs->elem_width);
  cs->n_values++;
  return PQG_OK;
}

/* BYTE_ARRAY output: values = int64 offsets[n+1] into binary_data. */
static int emit_binary(colstate* cs, const uint8_t* src, int32_t len) {
  pqg_column_desc* c = cs->c;
  if (cs->n_values + 1 >= c->values_capacity) return PQG_ERR_INVALID_ARG;
  if (cs->bin_bytes + (uint64_t)len > c->binary_capacity) return PQG_ERR_INVALID_ARG;
  int64_t* offs = (int64_t*)c->values;
  memcpy(c->binary_data + cs->bin_bytes, src, (size_t)len);
  cs->bin_bytes += (uint64_t)len;
  offs[cs->n_values] = (int64_t)(cs->bin_bytes - (uint64_t)len);
  offs[cs->n_values + 1] = (int64_t)cs->bin_bytes;
  cs->n_values++;
  return PQG_OK;
}

/* ------------------------------------------------------------------------ */
/* Value readers: one struct with a tagged union of the reference's readers. */

enum { VR_DICT = 1, VR_PLAIN_FIXED, VR_PLAIN_BOOL, VR_PLAIN_BINARY, VR_DELTA, VR_DLBA, VR_DBA, VR_BSS, VR_RLE_BOOL };

/* DeltaBinaryPackingValuesReader state: the eagerly decoded page (valuesBuffer). */
typedef struct {
  int64_t* buf;
  int32_t total;
  int32_t read;
} jdelta;

typedef struct {
  int kind;
  jstream in;
  int width;
  /* dictionary */
  rle_dec rle;
  const jdict* dict;
  /* boolean (ByteBitPackingValuesReader(1, LITTLE_ENDIAN), ByteBitPackingValuesReader.java:41-89) */
  int64_t bool_read;
  /* DELTA_BINARY_PACKED values; DELTA_LENGTH_BYTE_ARRAY lengths; DELTA_BYTE_ARRAY suffix lengths */
  jdelta delta;
  /* DELTA_BYTE_ARRAY prefix lengths and the previous value (DeltaByteArrayReader.previous) */
  jdelta prefix;
  uint8_t* prev;
  int64_t prev_len;
  /* BYTE_STREAM_SPLIT: encoded stream count and index (ByteStreamSplitValuesReader :32-50) */
  int64_t bss_count;
  int64_t bss_index;
} vreader;

/* DeltaBinaryPackingValuesReader.initFromPage :59-77 (eager), allocateValuesBuffer :83-87,
 * loadNewBlockToBuffer :121-143, unpack8Values :156-162, readBitWidthsForMiniBlocks :164-172,
 * DeltaBinaryPackingConfig :30-51. */
static int delta_init(jdelta* r, jstream* s) {
  int32_t block_size, mb_num, total;
  int e;
  if ((e = read_uvarint(s, &block_size))) return e;
  if ((e = read_uvarint(s, &mb_num))) return e;
  /* DeltaBinaryPackingConfig ctor :34-41: miniSize = (double)block/mbNum must be a multiple of 8 */
  if (mb_num == 0) return PQG_ERR_DELTA_CONFIG;   /* block/0 = Inf or NaN: Inf % 8 is NaN != 0 */
  double mini = (double)block_size / (double)mb_num;
  if (mini != mini || mini - 8.0 * (double)(int64_t)(mini / 8.0) != 0.0) return PQG_ERR_DELTA_CONFIG;
  int32_t mb_size = (int32_t)mini;
  if (mb_num < 0 || mb_size <= 0) return PQG_ERR_CORRUPT;
  if ((e = read_uvarint(s, &total))) return e;
  if (total < 0) return PQG_ERR_CORRUPT;
  int64_t mb_count = ((int64_t)total + mb_size - 1) / mb_size;   /* Math.ceil :84 */
  int64_t cap = mb_count * mb_size + 1;
  r->buf = (int64_t*)calloc((size_t)cap, sizeof(int64_t));
  r->total = total;
  r->read = 0;
  int32_t* widths = (int32_t*)calloc((size_t)mb_num, sizeof(int32_t));
  int64_t buffered = 0;
  if ((e = read_zigzag_varlong(s, &r->buf[buffered]))) { free(widths); return e; }
  buffered++;
  while (buffered < total) {
    int64_t min_delta;
    if ((e = read_zigzag_varlong(s, &min_delta))) { free(widths); return e; }
    for (int32_t i = 0; i < mb_num; i++) {
      int b;
      if ((e = js_read(s, &b))) { free(widths); return e; }
      widths[i] = b;
    }
    int32_t i;
    for (i = 0; i < mb_num && buffered < total; i++) {
      int w = widths[i];
      if (w > 64) { free(widths); return PQG_ERR_CORRUPT; } /* Packer has no packer for w > 64 */
      for (int32_t j = 0; j < mb_size; j += 8) {
        jstream sl;
        if ((e = js_slice(s, w, &sl))) { free(widths); return e; }
        pqr_unpack8_long(w, sl.buf + sl.pos, &r->buf[buffered]);
        buffered += 8;
      }
    }
    int64_t unpacked = (int64_t)i * mb_size;
    for (int64_t j = buffered - unpacked; j < buffered; j++)
      r->buf[j] = (int64_t)((uint64_t)r->buf[j] + (uint64_t)min_delta + (uint64_t)r->buf[j - 1]);
  }
  free(widths);
  return PQG_OK;
}

/* readLong :109-113 with checkRead :115-119 ("no more value to read"). */
static int delta_next(jdelta* r, int64_t* v) {
  if (r->read >= r->total) return PQG_ERR_DELTA_PAST_END;
  *v = r->buf[r->read++];
  return PQG_OK;
}

/* DeltaLengthByteArrayValuesReader.readBytes :51-58: length = lengthReader.readInteger()
 * ((int) of the long), then in.slice(length): negative -> IllegalArgumentException from
 * ByteBuffer.limit (CORRUPT), short -> EOFException ("Failed to read N bytes"). */
static int dlba_next(vreader* r, const uint8_t** p, int32_t* len) {
  int64_t l64;
  int e = delta_next(&r->delta, &l64);
  if (e) return e;
  int32_t l = (int32_t)(uint32_t)(uint64_t)l64;
  jstream sl;
  if ((e = js_slice(&r->in, l, &sl))) return e;
  *p = sl.buf + sl.pos;
  *len = l;
  return PQG_OK;
}

/* Encoding dispatch: Encoding.java getValuesReader / getDictionaryBasedValuesReader :61-253,
 * ColumnReaderBase.initDataReader :701-736 (then dataColumn.initFromPage). */
static int vreader_init(vreader* r, const pqg_page_desc* pg, colstate* cs, jstream* s, int32_t value_count) {
  memset(r, 0, sizeof(*r));
  const pqg_column_desc* c = cs->c;
  int enc = pg->encoding;
  int t = c->physical_type;
  if (enc == PQG_PLAIN_DICTIONARY || enc == PQG_RLE_DICTIONARY) {
    if (!cs->dict.present) return PQG_ERR_NO_DICTIONARY;                 /* :709-712 */
    if (cs->dict_err) return cs->dict_err;
    if (t == PQG_BOOLEAN) return PQG_ERR_UNSUPPORTED;                     /* Encoding.java :246-248 */
    r->kind = VR_DICT;
    r->dict = &cs->dict;
    /* DictionaryValuesReader.initFromPage :48-64: remainingStream(); 1-byte bit width */
    jstream in = *s;
    s->pos = s->end;
    if (js_available(&in) > 0) {
      int bw = 0;
      js_read(&in, &bw);   /* readIntLittleEndianOnOneByte */
      return rle_init(&r->rle, bw, in);
    }
    rle_init(&r->rle, 1, in);
    r->rle.empty_page = 1;
    return PQG_OK;
  }
  if (enc == PQG_PLAIN) {
    /* PlainValuesReader.initFromPage :38-41 etc.: remainingStream() */
    if (t == PQG_BOOLEAN) {
      /* ByteBitPackingValuesReader.initFromPage :77-88 with valueCount = page value count */
      int64_t length = ((int64_t)value_count * 1 + 7) / 8;
      if (length > js_available(s)) length = js_available(s);
      jstream sl;
      js_slice(s, length, &sl);
      r->kind = VR_PLAIN_BOOL;
      r->in = sl;
      return PQG_OK;
    }
    r->in = *s;
    s->pos = s->end;
    if (t == PQG_BYTE_ARRAY) { r->kind = VR_PLAIN_BINARY; return PQG_OK; }
    r->kind = VR_PLAIN_FIXED;
    r->width = elem_width_of(t, c->type_length);
    if (r->width <= 0) return PQG_ERR_UNSUPPORTED;
    return PQG_OK;
  }
  if (enc == PQG_DELTA_BINARY_PACKED) {
    if (t != PQG_INT32 && t != PQG_INT64) return PQG_ERR_UNSUPPORTED;   /* Encoding.java :190-193 */
    r->kind = VR_DELTA;
    return delta_init(&r->delta, s);
  }
  if (enc == PQG_DELTA_LENGTH_BYTE_ARRAY) {
    if (t != PQG_BYTE_ARRAY) return PQG_ERR_UNSUPPORTED;                /* Encoding.java :204-207 */
    /* DeltaLengthByteArrayValuesReader.initFromPage :44-48: lengths (eager), then remainingStream() */
    r->kind = VR_DLBA;
    int e = delta_init(&r->delta, s);
    if (e) return e;
    r->in = *s;
    s->pos = s->end;
    return PQG_OK;
  }
  if (enc == PQG_DELTA_BYTE_ARRAY) {
    /* Encoding.java :219-222: BYTE_ARRAY and FIXED_LEN_BYTE_ARRAY; the FLBA output here is fixed
     * width, so a decoded value of another length is reported as PQG_ERR_CORRUPT (vreader_read) */
    if (t != PQG_BYTE_ARRAY && !(t == PQG_FIXED_LEN_BYTE_ARRAY && c->type_length > 0)) return PQG_ERR_UNSUPPORTED;
    /* DeltaByteArrayReader.initFromPage :45-48: prefix lengths, then the suffixes' DLBA reader */
    r->kind = VR_DBA;
    int e = delta_init(&r->prefix, s);
    if (e) return e;
    if ((e = delta_init(&r->delta, s))) return e;
    r->in = *s;
    s->pos = s->end;
    r->prev = NULL;     /* previous = empty (:41) */
    r->prev_len = 0;
    if (pg->flags & PQG_PAGE_DBA_CARRY) {
      /* ColumnReaderBase.initDataReader :730-735 -> setPreviousReader :89-95 (PARQUET-246): previous =
       * the previous page reader's previous; that reader must be a DeltaByteArrayReader (cast) */
      if (cs->last_kind && cs->last_kind != VR_DBA) return PQG_ERR_UNSUPPORTED;
      if (cs->last_kind && cs->dba_prev_len > 0) {
        r->prev = (uint8_t*)malloc((size_t)cs->dba_prev_len);
        memcpy(r->prev, cs->dba_prev, (size_t)cs->dba_prev_len);
        r->prev_len = cs->dba_prev_len;
      }
    }
    return PQG_OK;
  }
  if (enc == PQG_BYTE_STREAM_SPLIT) {
    /* Encoding.java :127-145; ByteStreamSplitValuesReader.initFromPage :67-97 */
    if (t != PQG_FLOAT && t != PQG_DOUBLE && t != PQG_INT32 && t != PQG_INT64 && t != PQG_FIXED_LEN_BYTE_ARRAY)
      return PQG_ERR_UNSUPPORTED;
    int w = elem_width_of(t, c->type_length);
    if (w <= 0) return PQG_ERR_UNSUPPORTED;
    int64_t avail = js_available(s);
    if (avail % w != 0) return PQG_ERR_CORRUPT;               /* "Invalid ByteStreamSplit stream" :74-79 */
    if ((int64_t)value_count < avail / w) return PQG_ERR_CORRUPT;  /* upper bound check :83-88 */
    r->kind = VR_BSS;
    r->width = w;
    r->in = *s;
    s->pos = s->end;
    r->bss_count = avail / w;
    r->bss_index = 0;
    return PQG_OK;
  }
  if (enc == PQG_RLE) {
    /* Encoding.RLE.getValuesReader :116-124: VALUES only for BOOLEAN (getMaxLevel :255-271, width 1;
     * parquet-mr's V2 writer, DefaultV2ValuesWriterFactory.getBooleanValuesWriter :77-84).
     * RunLengthBitPackingHybridValuesReader.initFromPage :40-46: 4-byte LE length, sliceStream */
    if (t != PQG_BOOLEAN) return PQG_ERR_UNSUPPORTED;
    int32_t length;
    int e = read_int_le(s, &length);
    if (e) return e;
    jstream sl;
    if ((e = js_slice(s, length, &sl))) return e;
    r->kind = VR_RLE_BOOL;
    return rle_init(&r->rle, 1, sl);
  }
  return PQG_ERR_UNSUPPORTED;
}

static void vreader_free(vreader* r) {
  free(r->delta.buf);
  free(r->prefix.buf);
  free(r->prev);
  r->delta.buf = NULL;
  r->prefix.buf = NULL;
  r->prev = NULL;
}

/* Reads one value through the reader and emits it (readLong/readInteger/...). */
static int vreader_read(vreader* r, colstate* cs) {
  const pqg_column_desc* c = cs->c;
  int e;
  switch (r->kind) {
    case VR_DICT: {
      int32_t id;
      if ((e = rle_read_int(&r->rle, &id))) return e;
      const jdict* D = r->dict;
      /* Dictionary.decodeToX(id): array index, AIOOBE outside [0, n) */
      if (id < 0 || (uint32_t)id >= D->n) return PQG_ERR_DICT_ID;
      if (c->physical_type == PQG_BYTE_ARRAY) return emit_binary(cs, D->bin_ptr[id], D->bin_len[id]);
      return emit_fixed(cs, D->fixed + (int64_t)id * D->elem_width);
    }
    case VR_PLAIN_FIXED: {
      /* LittleEndianDataInputStream.readInt/readLong :334-377 (EOF), FixedLenByteArray slice (EOF) */
      if (js_available(&r->in) < r->width) return PQG_ERR_EOF;
      e = emit_fixed(cs, r->in.buf + r->in.pos);
      r->in.pos += r->width;
      return e;
    }
    case VR_PLAIN_BOOL: {
      /* ByteBitPackingValuesReader.readInteger/readMore :48-75: groups of 8 bits, zero fill */
      int64_t bit = r->bool_read++;
      int64_t byte = bit >> 3;
      uint8_t v = 0;
      if (byte < js_available(&r->in)) v = (r->in.buf[r->in.pos + byte] >> (bit & 7)) & 1;
      return emit_fixed(cs, &v);
    }
    case VR_RLE_BOOL: {
      /* RunLengthBitPackingHybridValuesReader.readBoolean :58-60: readInteger() != 0 */
      int32_t x;
      if ((e = rle_read_int(&r->rle, &x))) return e;
      uint8_t v = x != 0;
      return emit_fixed(cs, &v);
    }
    case VR_PLAIN_BINARY: {
      /* BinaryPlainValuesReader.readBytes :35-42 */
      int32_t len;
      if ((e = read_int_le(&r->in, &len))) return e;
      jstream sl;
      if ((e = js_slice(&r->in, len, &sl))) return e;
      return emit_binary(cs, sl.buf + sl.pos, len);
    }
    case VR_DELTA: {
      /* readLong :109-113, checkRead :115-119; readInteger :103-107 = (int) readLong() */
      int64_t v;
      if ((e = delta_next(&r->delta, &v))) return e;
      if (c->physical_type == PQG_INT32) {
        int32_t i32 = (int32_t)(uint32_t)(uint64_t)v;
        return emit_fixed(cs, (const uint8_t*)&i32);
      }
      return emit_fixed(cs, (const uint8_t*)&v);
    }
    case VR_DLBA: {
      const uint8_t* p;
      int32_t len;
      if ((e = dlba_next(r, &p, &len))) return e;
      return emit_binary(cs, p, len);
    }
    case VR_DBA: {
      /* DeltaByteArrayReader.readBytes :57-79 */
      int64_t pl64;
      if ((e = delta_next(&r->prefix, &pl64))) return e;
      int32_t prefix = (int32_t)(uint32_t)(uint64_t)pl64;
      const uint8_t* sp;
      int32_t slen;
      if ((e = dlba_next(r, &sp, &slen))) return e;
      int64_t length = (int64_t)(int32_t)((uint32_t)prefix + (uint32_t)slen);  /* int addition */
      if (prefix != 0) {
        /* new byte[length] (NegativeArraySizeException), arraycopy(previous, 0, out, 0, prefix)
         * (IndexOutOfBounds when prefix < 0 or prefix > previous.length) */
        if (length < 0 || prefix < 0 || prefix > r->prev_len) return PQG_ERR_CORRUPT;
        uint8_t* out = (uint8_t*)malloc((size_t)(length ? length : 1));
        memcpy(out, r->prev, (size_t)prefix);
        memcpy(out + prefix, sp, (size_t)slen);
        free(r->prev);
        r->prev = out;
        r->prev_len = length;
      } else {
        uint8_t* out = (uint8_t*)malloc((size_t)(slen ? slen : 1));
        memcpy(out, sp, (size_t)slen);
        free(r->prev);
        r->prev = out;
        r->prev_len = slen;
      }
      if (c->physical_type == PQG_FIXED_LEN_BYTE_ARRAY) {
        if (r->prev_len != c->type_length) return PQG_ERR_CORRUPT;  /* no room in the fixed-width output */
        return emit_fixed(cs, r->prev);
      }
      return emit_binary(cs, r->prev, (int32_t)r->prev_len);
    }
    case VR_BSS: {
      /* nextElementByteOffset :43-50; value bytes k = stream k at index i (decodeData :53-64) */
      if (r->bss_index >= r->bss_count) return PQG_ERR_EOF;   /* "Byte-stream data was already exhausted." */
      uint8_t tmp[64];
      uint8_t* buf = r->width <= 64 ? tmp : (uint8_t*)malloc((size_t)r->width);
      for (int k = 0; k < r->width; k++) buf[k] = r->in.buf[r->in.pos + r->bss_index + (int64_t)k * r->bss_count];
      r->bss_index++;
      e = emit_fixed(cs, buf);
      if (buf != tmp) free(buf);
      return e;
    }
  }
  return PQG_ERR_UNSUPPORTED;
}

/* ------------------------------------------------------------------------ */
/* Level readers: V1 via Encoding.getValuesReader(.., REPETITION/DEFINITION_LEVEL)
 * (Encoding.java :116-125 RLE, :152-157 BIT_PACKED; maxLevel 0 -> ZeroIntegerValuesReader
 * or BIT_PACKED width 0 = no bytes); RunLengthBitPackingHybridValuesReader.initFromPage
 * :40-46 (4-byte LE length then sliceStream). V2 via ColumnReaderBase.newRLEIterator :779-789
 * (no length prefix; maxLevel 0 -> NullIntIterator). */

typedef struct {
  int zero;
  rle_dec rle;
  /* BIT_PACKED (BIG_ENDIAN) levels: ByteBitPackingValuesReader(maxLevel, BIG_ENDIAN) */
  int be;
  int be_width;
  jstream be_in;
  int64_t be_read;
} lreader;

/* BE (MSB-first) unpack: Packer.BIG_ENDIAN, ByteBasedBitPackingGenerator getShift msbFirst branch
 * (:153-159): value i = bits [i*w, (i+1)*w) of the stream, bit 0 = MSB of byte 0. */
static uint32_t be_value(const uint8_t* buf, int64_t avail, int64_t idx, int w) {
  uint32_t v = 0;
  for (int k = 0; k < w; k++) {
    int64_t bit = idx * w + k;
    int64_t byte = bit >> 3;
    uint32_t b = byte < avail ? buf[byte] : 0;   /* readMore :49-57: zero fill past the section */
    v = (v << 1) | ((b >> (7 - (bit & 7))) & 1u);
  }
  return v;
}

void pqr_unpack8_int_be(int w, const uint8_t* in, int32_t* out) {
  for (int i = 0; i < 8; i++) out[i] = (int32_t)be_value(in, w, i, w);
}

static int lreader_init_v1(lreader* L, int enc, int max_level, jstream* s, int32_t value_count) {
  memset(L, 0, sizeof(*L));
  int w = pqr_width_from_max_int(max_level);
  if (w == 0) {
    if (enc == PQG_RLE || enc == PQG_BIT_PACKED) { L->zero = 1; return PQG_OK; }
    return PQG_ERR_UNSUPPORTED;
  }
  if (enc == PQG_BIT_PACKED) {
    /* ByteBitPackingValuesReader.initFromPage :77-88: min(ceil(valueCount * w / 8), available)
     * bytes, valueCount = the page's num_values */
    int64_t length = ((int64_t)value_count * w + 7) / 8;
    if (length > js_available(s)) length = js_available(s);
    jstream sl;
    js_slice(s, length, &sl);
    L->be = 1;
    L->be_width = w;
    L->be_in = sl;
    return PQG_OK;
  }
  if (enc != PQG_RLE) return PQG_ERR_UNSUPPORTED;
  int32_t length;
  int e = read_int_le(s, &length);
  if (e) return e;
  jstream sl;
  if ((e = js_slice(s, length, &sl))) return e;
  return rle_init(&L->rle, w, sl);
}

static int lreader_init_v2(lreader* L, int max_level, jstream sec) {
  memset(L, 0, sizeof(*L));
  int w = pqr_width_from_max_int(max_level);
  if (max_level == 0) { L->zero = 1; return PQG_OK; }
  return rle_init(&L->rle, w, sec);
}

static inline int lreader_next(lreader* L, int32_t* v) {
  if (L->zero) { *v = 0; return PQG_OK; }
  if (L->be) {
    *v = (int32_t)be_value(L->be_in.buf + L->be_in.pos, js_available(&L->be_in), L->be_read++, L->be_width);
    return PQG_OK;
  }
  return rle_read_int(&L->rle, v);
}

/* ------------------------------------------------------------------------ */
/* Column decode: ColumnReaderBase ctor (dictionary) :448-472, readPageV1 :738-758,
 * readPageV2 :760-771, checkRead :650-676 (rl, dl per slot; value when dl == maxDl). */

static void set_status(pqg_status* st, int code, int page, int64_t idx, const char* what) {
  if (!st) return;
  st->code = code;
  st->page = page;
  st->value_index = idx;
  snprintf(st->message, sizeof(st->message), "%s: %s (page %d, index %lld)", what, pqg_error_name_ref(code),
           page, (long long)idx);
}

int pqr_decode(const uint8_t* bytes, uint64_t n_bytes, pqg_column_desc* cols, int n_cols,
               const pqg_page_desc* pages, int n_pages, uint32_t* page_value_counts, pqg_status* st) {
  if (st) { memset(st, 0, sizeof(*st)); st->page = -1; }
  if (!bytes && n_bytes) return PQG_ERR_INVALID_ARG;
  colstate* cs = (colstate*)calloc((size_t)(n_cols > 0 ? n_cols : 1), sizeof(colstate));
  for (int i = 0; i < n_cols; i++) {
    cs[i].c = &cols[i];
    cs[i].elem_width = elem_width_of(cols[i].physical_type, cols[i].type_length);
    cols[i].values_written = 0;
  }
  int rc = PQG_OK;
  for (int p = 0; p < n_pages && rc == PQG_OK; p++) {
    const pqg_page_desc* pg = &pages[p];
    if (pg->column < 0 || pg->column >= n_cols || pg->offset + pg->size > n_bytes) {
      rc = PQG_ERR_INVALID_ARG;
      set_status(st, rc, p, -1, "bad page descriptor");
      break;
    }
    colstate* C = &cs[pg->column];
    pqg_column_desc* c = C->c;
    if (!C->dict_checked) {   /* ColumnReaderBase ctor :455-466 reads the dictionary page once */
      C->dict_checked = 1;
      C->dict_err = dict_init(&C->dict, c, bytes);
      if (C->dict_err) { rc = C->dict_err; set_status(st, rc, p, -1, "dictionary page"); break; }
    }
    jstream page = {bytes + pg->offset, 0, pg->size};
    lreader rl, dl;
    vreader vr;
    memset(&vr, 0, sizeof(vr));
    int e;
    int32_t nv = (int32_t)pg->num_values;
    if (pg->version == 2) {
      /* DataPageV2: rl bytes, dl bytes, data (DataPageV2.java:201-213) */
      if ((uint64_t)pg->rl_byte_length + pg->dl_byte_length > pg->size) {
        rc = PQG_ERR_CORRUPT; set_status(st, rc, p, 0, "V2 level lengths"); break;
      }
      jstream rls = {page.buf, 0, pg->rl_byte_length};
      jstream dls = {page.buf, pg->rl_byte_length, (int64_t)pg->rl_byte_length + pg->dl_byte_length};
      jstream data = {page.buf, (int64_t)pg->rl_byte_length + pg->dl_byte_length, pg->size};
      if ((e = lreader_init_v2(&rl, c->max_rep, rls))) { rc = e; set_status(st, rc, p, 0, "rl init"); break; }
      if ((e = lreader_init_v2(&dl, c->max_def, dls))) { rc = e; set_status(st, rc, p, 0, "dl init"); break; }
      if ((e = vreader_init(&vr, pg, C, &data, nv))) {
        rc = e; set_status(st, rc, p, 0, "data init"); vreader_free(&vr); break;
      }
    } else {
      if ((e = lreader_init_v1(&rl, pg->rl_encoding, c->max_rep, &page, nv))) {
        rc = e; set_status(st, rc, p, 0, "rl init"); break;
      }
      if ((e = lreader_init_v1(&dl, pg->dl_encoding, c->max_def, &page, nv))) {
        rc = e; set_status(st, rc, p, 0, "dl init"); break;
      }
      if ((e = vreader_init(&vr, pg, C, &page, nv))) {
        rc = e; set_status(st, rc, p, 0, "data init"); vreader_free(&vr); break;
      }
    }
    uint64_t before = C->n_values;
    for (int32_t slot = 0; slot < nv; slot++) {
      int32_t r, d;
      if ((e = lreader_next(&rl, &r))) { rc = e; set_status(st, rc, p, slot, "rl decode"); break; }
      if ((e = lreader_next(&dl, &d))) { rc = e; set_status(st, rc, p, slot, "dl decode"); break; }
      if (C->n_slots >= c->levels_capacity && (c->def_levels || c->rep_levels)) {
        rc = PQG_ERR_INVALID_ARG; set_status(st, rc, p, slot, "levels capacity"); break;
      }
      if (c->def_levels) c->def_levels[C->n_slots] = (uint8_t)((uint32_t)d > 255u ? 255u : (uint32_t)d);
      if (c->rep_levels) c->rep_levels[C->n_slots] = (uint8_t)((uint32_t)r > 255u ? 255u : (uint32_t)r);
      C->n_slots++;
      if (d == c->max_def) {
        if ((e = vreader_read(&vr, C))) {
          rc = e; set_status(st, rc, p, (int64_t)(C->n_values - before), "value decode"); break;
        }
      }
    }
    if (page_value_counts) page_value_counts[p] = (uint32_t)(C->n_values - before);
    C->last_kind = vr.kind;
    if (vr.kind == VR_DBA) {  /* keep `previous` for the next page's setPreviousReader */
      free(C->dba_prev);
      C->dba_prev = vr.prev;
      C->dba_prev_len = vr.prev_len;
      vr.prev = NULL;
    }
    vreader_free(&vr);
  }
  for (int i = 0; i < n_cols; i++) {
    cols[i].values_written = cs[i].n_values;
    dict_free(&cs[i].dict);
    free(cs[i].dba_prev);
  }
  free(cs);
  return rc;
}

/* DeltaBinaryPackingValuesReader over one section (known-answer tests): returns
 * number of values (header total) or <0; consumed bytes via *consumed. */
int64_t pqr_delta_decode(const uint8_t* buf, int64_t len, int64_t* out, int64_t cap, int64_t* consumed) {
  jstream s = {buf, 0, len};
  vreader r;
  memset(&r, 0, sizeof(r));
  int e = delta_init(&r.delta, &s);
  if (e) { vreader_free(&r); return -e; }
  int64_t n = r.delta.total;
  if (n > cap) { vreader_free(&r); return -PQG_ERR_INVALID_ARG; }
  memcpy(out, r.delta.buf, (size_t)n * sizeof(int64_t));
  if (consumed) *consumed = s.pos;
  vreader_free(&r);
  return n;
}

const char* pqg_error_name_ref(int code) {
  switch (code) {
    case PQG_OK: return "OK";
    case PQG_ERR_INVALID_ARG: return "INVALID_ARG";
    case PQG_ERR_UNSUPPORTED: return "UNSUPPORTED";
    case PQG_ERR_HIP: return "HIP";
    case PQG_ERR_NO_DEVICE: return "NO_DEVICE";
    case PQG_ERR_EOF: return "EOF";
    case PQG_ERR_RLE_PAST_END: return "RLE_PAST_END";
    case PQG_ERR_BIT_WIDTH: return "BIT_WIDTH";
    case PQG_ERR_DICT_ID: return "DICT_ID";
    case PQG_ERR_EMPTY_PAGE: return "EMPTY_PAGE";
    case PQG_ERR_EMPTY_PACKED_RUN: return "EMPTY_PACKED_RUN";
    case PQG_ERR_DELTA_CONFIG: return "DELTA_CONFIG";
    case PQG_ERR_DELTA_PAST_END: return "DELTA_PAST_END";
    case PQG_ERR_CORRUPT: return "CORRUPT";
    case PQG_ERR_NO_DICTIONARY: return "NO_DICTIONARY";
    case PQG_ERR_DICT_ENCODING: return "DICT_ENCODING";
    default: return "UNKNOWN";
  }
}

/* ------------------------------------------------------------------------------------------
 * Snappy raw block decompression (ORACLE). parquet-mr decompresses a SNAPPY page with
 * SnappyDecompressor.decompress (parquet-hadoop/.../hadoop/codec/SnappyDecompressor.java), which
 * calls Snappy.uncompress of xerial snappy-java (a third-party library absent here, pinned in
 * parquet-mr's pom as org.xerial.snappy:snappy-java); the page is decompressed into a buffer of
 * the header's uncompressed size (ColumnChunkPageReadStore.java:150-172 V1, :223-247 V2 data
 * section). This restates the published Snappy block format (google/snappy
 * format_description.txt): varint uncompressed length, then elements — literal (tag & 3 == 0,
 * length - 1 in the tag or 1..4 following bytes), copy with 1-, 2- or 4-byte offset — where a
 * copy may overlap its own output (byte-at-a-time semantics). Returns 0 and *out_len, or
 * PQG_ERR_CORRUPT for malformed input or a length different from `expect`.
 * ------------------------------------------------------------------------------------------ */
int pqr_snappy_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len) {
  int64_t p = 0;
  uint64_t ulen = 0;
  int shift = 0;
  for (;;) {
    if (p >= n || shift > 28) return PQG_ERR_CORRUPT;
    uint8_t b = src[p++];
    ulen |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) break;
    shift += 7;
  }
  if (ulen > 0xFFFFFFFFull || (int64_t)ulen != expect) return PQG_ERR_CORRUPT;
  int64_t op = 0;
  while (op < (int64_t)ulen) {
    if (p >= n) return PQG_ERR_CORRUPT;
    const uint8_t tag = src[p++];
    if ((tag & 3) == 0) {
      int64_t len = tag >> 2;
      if (len >= 60) {
        const int nb = (int)len - 59;
        if (p + nb > n) return PQG_ERR_CORRUPT;
        len = 0;
        for (int i = 0; i < nb; i++) len |= (int64_t)src[p + i] << (8 * i);
        p += nb;
      }
      len += 1;
      if (p + len > n || op + len > (int64_t)ulen) return PQG_ERR_CORRUPT;
      memcpy(dst + op, src + p, (size_t)len);
      p += len;
      op += len;
    } else {
      int64_t len, off;
      if ((tag & 3) == 1) {
        if (p + 1 > n) return PQG_ERR_CORRUPT;
        len = 4 + ((tag >> 2) & 7);
        off = ((int64_t)(tag >> 5) << 8) | src[p];
        p += 1;
      } else if ((tag & 3) == 2) {
        if (p + 2 > n) return PQG_ERR_CORRUPT;
        len = 1 + (tag >> 2);
        off = (int64_t)src[p] | ((int64_t)src[p + 1] << 8);
        p += 2;
      } else {
        if (p + 4 > n) return PQG_ERR_CORRUPT;
        len = 1 + (tag >> 2);
        off = (int64_t)src[p] | ((int64_t)src[p + 1] << 8) | ((int64_t)src[p + 2] << 16) | ((int64_t)src[p + 3] << 24);
        p += 4;
      }
      if (off == 0 || off > op || op + len > (int64_t)ulen) return PQG_ERR_CORRUPT;
      for (int64_t i = 0; i < len; i++) dst[op + i] = dst[op - off + i];
      op += len;
    }
  }
  *out_len = op;
  return 0;
}

/* ------------------------------------------------------------------------------------------
 * LZ4 raw block decompression (ORACLE). parquet-mr decompresses an LZ4_RAW page with
 * Lz4RawDecompressor (parquet-hadoop/.../hadoop/codec/Lz4RawDecompressor.java:26-50, a
 * NonBlockedDecompressor over a buffer of the header's uncompressed size), which calls
 * io.airlift.compress.lz4.Lz4Decompressor (aircompressor, a third-party library absent here, pinned
 * in parquet-mr's pom as io.airlift:aircompressor). This restates the published LZ4 block format
 * (lz4/lz4 doc/lz4_Block_format.md): a sequence is a token (literal length in the high nibble,
 * match length - 4 in the low nibble; 15 continues with bytes added while they are 255), the
 * literals, a 2-byte little-endian offset (0 is invalid) and the match, which may overlap its own
 * output; the block ends with a sequence of literals only, at the end of the input. An empty
 * output is the single byte 0. Returns 0 and *out_len, or PQG_ERR_CORRUPT for malformed input or an
 * output length different from `expect`. Parity unpinned for blocks that break the format's
 * end-of-block rules (last 5 bytes literals, last match >= 12 bytes before the end): they are not
 * checked here (nor by k_lz4raw), while aircompressor may reject them.
 * ------------------------------------------------------------------------------------------ */
int pqr_lz4_raw_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expect, int64_t* out_len) {
  if (n <= 0) return PQG_ERR_CORRUPT;
  int64_t p = 0, op = 0;
  for (;;) {
    if (p >= n) return PQG_ERR_CORRUPT;
    const uint32_t token = src[p++];
    int64_t ll = token >> 4;
    if (ll == 15) {
      uint32_t b;
      do {
        if (p >= n) return PQG_ERR_CORRUPT;
        b = src[p++];
        ll += b;
      } while (b == 255);
    }
    if (p + ll > n || op + ll > expect) return PQG_ERR_CORRUPT;
    memcpy(dst + op, src + p, (size_t)ll);
    p += ll;
    op += ll;
    if (p == n) break;  /* the last sequence: literals only */
    if (p + 2 > n) return PQG_ERR_CORRUPT;
    const int64_t off = (int64_t)src[p] | ((int64_t)src[p + 1] << 8);
    p += 2;
    if (off == 0 || off > op) return PQG_ERR_CORRUPT;
    int64_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (p >= n) return PQG_ERR_CORRUPT;
        b = src[p++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (op + ml > expect) return PQG_ERR_CORRUPT;
    for (int64_t i = 0; i < ml; i++) dst[op + i] = dst[op - off + i];
    op += ml;
  }
  if (op != expect) return PQG_ERR_CORRUPT;
  *out_len = op;
  return 0;
}
