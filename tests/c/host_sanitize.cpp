/*
 * host_sanitize.cpp — the product's host code (csrc/pqgpu_framing.cpp: Thrift compact page headers,
 * CRC, page descriptors; csrc/pqgpu_reader.cpp: the ValuesReader contract over decoded arrays) under
 * AddressSanitizer + UndefinedBehaviorSanitizer, without HIP. Built by tests/test_host_sanitize.py
 * with -fsanitize=address,undefined -fno-sanitize-recover=all, so any finding aborts the run.
 *
 * The reference walks the same untrusted bytes in ParquetFileReader.Chunk.readAllPages
 * (parquet-hadoop/.../ParquetFileReader.java:1824-1979) and Util.readPageHeader (Thrift).
 *
 * usage: host_sanitize <case file>...
 *   case file: "PQGF" | i32 codec | i32 physical_type | i32 type_length | i32 flags | i64 value_count
 *              | u64 chunk_len | chunk bytes
 * Every buffer the library reads or writes is an exactly-sized heap allocation (the chunk bytes,
 * the header / page descriptor arrays, the decoded arrays the readers serve), so a read or write
 * one byte past any of them is caught. Prints one line per case:
 *   <file> frame=<rc> pages=<rc> n=<pages> reads=<values read> errs=<reader errors>
 */
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pqgpu.h"
#include "pqgpu_reader.h"

static int width_of(int t, int tl) {
  switch (t) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return tl > 0 ? tl : 1;
    default: return 8;  // BYTE_ARRAY: int64 offsets
  }
}

// one read of the reader's type; 0 or the error code
static int read_one(pqg_values_reader* r) {
  int32_t i32;
  int64_t i64;
  float f;
  double d;
  const uint8_t* p;
  uint32_t n;
  if (r->ids) return pqg_vr_read_dictionary_id(r, &i32);
  switch (r->physical_type) {
    case PQG_BOOLEAN: return pqg_vr_read_boolean(r, &i32);
    case PQG_INT32: return pqg_vr_read_integer(r, &i32);
    case PQG_INT64: return pqg_vr_read_long(r, &i64);
    case PQG_FLOAT: return pqg_vr_read_float(r, &f);
    case PQG_DOUBLE: return pqg_vr_read_double(r, &d);
    default: {
      const int rc = pqg_vr_read_bytes(r, &p, &n);
      if (rc == 0 && n) {
        volatile uint8_t s = p[0] ^ p[n - 1];  // touch the first and last byte of the value
        (void)s;
      }
      return rc;
    }
  }
}

// Serve every page of the framed chunk from exactly-sized "decoded" arrays; with a simulated decode
// error (value error in page err_page at err_index, or an init error) for the error paths.
static void read_pages(const pqg_column_desc& col0, const pqg_page_desc* pages, int np, int mode, uint64_t* reads,
                       uint64_t* errs) {
  uint64_t total = 0;
  for (int p = 0; p < np; p++) total += pages[p].num_values;
  if (total > (1u << 24)) return;  // lying headers: do not allocate gigabytes
  std::vector<uint32_t> counts((size_t)np + 1, 0);
  for (int p = 0; p < np; p++) counts[(size_t)p] = pages[p].num_values;
  const int w = (col0.flags & PQG_COLUMN_DICTIONARY_IDS) ? 4 : width_of(col0.physical_type, col0.type_length);
  const bool bin = col0.physical_type == PQG_BYTE_ARRAY && !(col0.flags & PQG_COLUMN_DICTIONARY_IDS);
  const size_t vbytes = (size_t)(bin ? total + 1 : total) * (size_t)w;
  uint8_t* values = (uint8_t*)std::malloc(vbytes ? vbytes : 1);
  uint8_t* binary = nullptr;
  uint64_t nbin = 0;
  if (bin) {
    int64_t* offs = (int64_t*)values;
    for (uint64_t i = 0; i <= total; i++) offs[i] = (int64_t)(3 * i);  // value i = 3 bytes
    nbin = 3 * total;
    binary = (uint8_t*)std::malloc(nbin ? nbin : 1);
    for (uint64_t i = 0; i < nbin; i++) binary[i] = (uint8_t)i;
  } else {
    for (size_t i = 0; i < vbytes; i++) values[i] = (uint8_t)(i * 7);
  }
  pqg_column_desc col = col0;
  col.values = values;
  col.values_capacity = bin ? total + 1 : total;
  col.binary_data = binary;
  col.binary_capacity = nbin;
  col.values_written = total;
  // exactly-sized level arrays (one byte per slot) for the level readers
  uint8_t* dl = (uint8_t*)std::malloc(total ? total : 1);
  uint8_t* rl = (uint8_t*)std::malloc(total ? total : 1);
  for (uint64_t i = 0; i < total; i++) dl[i] = rl[i] = (uint8_t)(i % 3);
  col.max_def = col.max_def > 0 ? col.max_def : 2;
  col.max_rep = col.max_rep > 0 ? col.max_rep : 1;
  col.def_levels = dl;
  col.rep_levels = rl;
  std::vector<pqg_page_error> pe((size_t)np + 1, pqg_page_error{PQG_OK, PQG_PHASE_NONE, -1});
  if (mode == 1 && np > 0) {  // a value error in the middle page
    pe[(size_t)np / 2] = {PQG_ERR_DICT_ID, PQG_PHASE_VALUE, (int64_t)pages[np / 2].num_values / 2};
  } else if (mode == 2 && np > 0) {  // an init error in the last page
    pe[(size_t)np - 1] = {PQG_ERR_CORRUPT, PQG_PHASE_DATA_INIT, -1};
  } else if (mode == 3 && np > 0) {  // a level error in the first page
    pe[0] = {PQG_ERR_RLE_PAST_END, PQG_PHASE_DL_READ, (int64_t)pages[0].num_values / 3};
  }
  const pqg_page_error* perr = mode ? pe.data() : nullptr;
  for (int p = 0; p < np; p++) {
    pqg_levels_reader lr[2];
    for (int kind = 0; kind < 2; kind++) {
      if (pqg_lr_init_from_page(&lr[kind], &col, kind, pages, np, p, perr)) {
        (*errs)++;
        continue;
      }
      for (;;) {  // reads past the page's slots end in EOF
        int32_t v;
        if (pqg_lr_read_integer(&lr[kind], &v)) {
          (*errs)++;
          break;
        }
        (*reads)++;
      }
      (void)pqg_lr_remaining(&lr[kind]);
    }
    pqg_values_reader r;
    const int irc = pqg_vr_init_from_page(&r, &col, pages, counts.data(), np, p, perr);
    if (irc) {
      (*errs)++;
      continue;
    }
    // skip(3), read 2, ..., then reads past the end
    for (int k = 0;; k++) {
      const int e = (k % 5 < 3) ? pqg_vr_skip(&r) : read_one(&r);
      if (e) {
        (*errs)++;
        break;
      }
      (*reads)++;
    }
    (void)pqg_vr_skip_n(&r, 1u << 20);
    (void)pqg_vr_remaining(&r);
    (void)pqg_java_exception(read_one(&r));
  }
  std::free(dl);
  std::free(rl);
  std::free(values);
  std::free(binary);
}

int main(int argc, char** argv) {
  for (int a = 1; a < argc; a++) {
    FILE* f = std::fopen(argv[a], "rb");
    if (!f) return 2;
    char magic[4];
    int32_t hdr[4];
    int64_t value_count;
    uint64_t len;
    if (std::fread(magic, 1, 4, f) != 4 || std::memcmp(magic, "PQGF", 4) || std::fread(hdr, 4, 4, f) != 4 ||
        std::fread(&value_count, 8, 1, f) != 1 || std::fread(&len, 8, 1, f) != 1)
      return 2;
    uint8_t* chunk = (uint8_t*)std::malloc(len ? len : 1);  // exactly the chunk: no padding to hide overreads
    if (std::fread(chunk, 1, len, f) != len) return 2;
    std::fclose(f);
    (void)pqg_crc32(0, chunk, len);
    // headers: start from a one-entry array, then exactly the count the library asks for
    int cap = 1, n = 0;
    pqg_status st;
    pqg_page_header* h = (pqg_page_header*)std::malloc(sizeof(pqg_page_header) * (size_t)cap);
    int frc = pqg_frame_chunk(len ? chunk : nullptr, len, value_count, 1, h, cap, &n, &st);
    if (frc == PQG_ERR_INVALID_ARG && n > cap) {
      cap = n;
      h = (pqg_page_header*)std::realloc(h, sizeof(pqg_page_header) * (size_t)cap);
      frc = pqg_frame_chunk(len ? chunk : nullptr, len, value_count, 1, h, cap, &n, &st);
    }
    int prc = -1, np = 0;
    uint64_t reads = 0, errs = 0;
    if (frc == PQG_OK) {
      pqg_column_desc col;
      std::memset(&col, 0, sizeof(col));
      col.physical_type = hdr[1];
      col.type_length = hdr[2];
      col.flags = hdr[3];
      col.dict_offset = -1;
      int pcap = 1;
      pqg_page_desc* pages = (pqg_page_desc*)std::malloc(sizeof(pqg_page_desc) * (size_t)pcap);
      prc = pqg_pages_from_headers(h, n, hdr[0], 0, 0, &col, pages, pcap, &np, &st);
      if (prc == PQG_ERR_INVALID_ARG && np > pcap) {
        pcap = np;
        pages = (pqg_page_desc*)std::realloc(pages, sizeof(pqg_page_desc) * (size_t)pcap);
        prc = pqg_pages_from_headers(h, n, hdr[0], 0, 0, &col, pages, pcap, &np, &st);
      }
      if (prc == PQG_OK)
        for (int mode = 0; mode < 4; mode++) read_pages(col, pages, np, mode, &reads, &errs);
      std::free(pages);
    }
    std::printf("%s frame=%d pages=%d n=%d reads=%" PRIu64 " errs=%" PRIu64 "\n", argv[a], frc, prc, np, reads, errs);
    std::free(h);
    std::free(chunk);
  }
  return 0;
}
