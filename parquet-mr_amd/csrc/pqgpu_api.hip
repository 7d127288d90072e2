// pqgpu_api.hip — the C ABI of include/pqgpu.h.
//
// Host work here is descriptor bookkeeping only (page tables, class lists,
// prefix sums of header value counts, error resolution); every byte of page
// data is decoded by the kernels in pqgpu_kernels.hip. There is no CPU decode
// fallback: without a usable HIP device every entry point returns
// PQG_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <new>
#include <atomic>
#include <thread>
#include <vector>

#include "pqgpu_internal.h"

using pqg::ColumnDev;
using pqg::PageWork;

namespace {

const char* kNames[] = {"OK", "INVALID_ARG", "UNSUPPORTED", "HIP", "NO_DEVICE"};

void set_status(pqg_status* st, int code, int page, int64_t idx, const char* what) {
  if (!st) return;
  st->code = code;
  st->page = page;
  st->value_index = idx;
  std::snprintf(st->message, sizeof(st->message), "%s: %s (page %d, index %lld)", what, pqg_error_name(code), page,
                (long long)idx);
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, n ? n : 16);
    if (e == hipSuccess) cap = n ? n : 16;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, n ? n : 16, hipHostMallocDefault);
    if (e == hipSuccess) cap = n ? n : 16;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

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

// PQG_COLUMN_DICTIONARY_IDS columns write uint32 ids; BYTE_ARRAY columns otherwise write offsets + bytes
bool ids_mode(const pqg_column_desc& c) { return (c.flags & PQG_COLUMN_DICTIONARY_IDS) != 0; }
bool bin_out(const pqg_column_desc& c) { return c.physical_type == PQG_BYTE_ARRAY && !ids_mode(c); }
int out_width(const pqg_column_desc& c) { return ids_mode(c) ? 4 : elem_width(c.physical_type, c.type_length); }

// Error words: 3 per page + 3 per column (dictionary pages), padded to 16 bytes; the error
// counter follows them in the same allocation.
size_t err_region_bytes(int n_pages, int n_cols) {
  return (sizeof(uint64_t) * 3 * (size_t)(n_pages + std::max(n_cols, 1)) + 15) & ~(size_t)15;
}

// Kernel classes, in launch order after the level pass.
//   C_IDS   dictionary pages whose values are not 4 / 8 bytes (BYTE_ARRAY, FLBA, INT96): ids first
//   C_BINP  PLAIN BYTE_ARRAY          C_DLBA  DELTA_LENGTH_BYTE_ARRAY      C_BSS  BYTE_STREAM_SPLIT
//   C_DBA   DELTA_BYTE_ARRAY (lengths here; values by k_dba_copy after the offset scan)
//   C_DD    dictionary pages of dictionary-direct BYTE_ARRAY columns (ColumnDev::dict_direct): walk + chunk
//           byte sums, per-column scan, offsets + value bytes (launch_dict_dd), no ids stored
//   C_DDG   the same for dictionary-direct columns whose dictionary is gathered from HBM (ColumnDev::dd_global)
enum Cls { C_DICT4 = 0, C_DICT8, C_IDS, C_PLAIN, C_BOOL, C_DELTA4, C_DELTA8, C_BSS, C_BINP, C_DLBA, C_DBA, C_RLEBOOL, C_DD,
           C_DDG, C_NCLS };
constexpr int N_DICT_CLS = 3;  // C_DICT4, C_DICT8, C_IDS: run-record walk + chunk expansion

struct HostErr {
  int page;
  int kind;  // 0 init, 2 value
  int64_t index;
  int code;
};

}  // namespace

struct pqg_plan {
  pqg_ctx* ctx = nullptr;
  const uint8_t* d_bytes = nullptr;
  uint64_t n_bytes = 0;
  int n_pages = 0;
  int n_cols = 0;
  DevBuf work, cols, lists, col_pages, col_page_start, err;
  DevBuf rec, chunk_run, chunks;      // dictionary pages: run records, chunk -> record, chunk work list
  DevBuf pstat, flags;                // per page: {records, values} and ready epoch (fused dictionary kernel)
  uint32_t epoch = 0;
  uint32_t err_epoch = pqg::ERR_EPOCH_MAX;  // error-word epoch of the last launch (first launch wraps: zeroes the region)
  bool dict_fused = true;
  uint32_t chunk_off[N_DICT_CLS] = {0, 0, 0}, chunk_n[N_DICT_CLS] = {0, 0, 0};  // ranges in `chunks`
  // C_DD: its chunks in `chunks` (per column in page order, each column's first at a multiple of 4:
  // padding entries of page 0xFFFFFFFF between columns), the per-chunk byte sums / first bytes in
  // bscratch, the columns and their chunk ranges in bin_lists, the LDS of the staged dictionaries
  // ([0]: C_DD, dictionaries staged in LDS; [1]: C_DDG, dictionaries gathered from HBM)
  uint32_t dd_chunk_off[2] = {0, 0}, dd_chunk_n[2] = {0, 0}, dd_region = 16;
  uint64_t dd_sums_off[2] = {~0ull, ~0ull};
  int n_dd_cols[2] = {0, 0}, off_dd_cols[2] = {0, 0}, off_dd_start[2] = {0, 0};
  // fused dictionary kernel: persistent walker / tile workgroup counts (0: one page / 4 chunks per WG)
  // BYTE_ARRAY / fixed-width-dictionary scratch (ColumnDev::blen, bsrc, dict_len, dict_src, block_sums,
  // bin_total), dictionary walks, post-passes, offset-scan blocks, copy chunks
  DevBuf bscratch, bin_lists, bin_blocks, bin_chunks, dba_chunks;
  uint64_t blen_bytes = 0;            // leading part of bscratch cleared before every launch
  int n_dict_walk = 0, n_bind = 0, n_fixd = 0, n_bin_cols = 0, n_carry = 0;
  // BYTE_ARRAY dictionary pages of at least DENT_MIN bytes: walked per tile (launch_dict_entries)
  DevBuf dent_tiles;
  uint32_t n_dent_tiles = 0;
  int n_dent_cols = 0, off_dent_cols = 0, off_dent_start = 0;
  uint64_t dent_rec_off = 0, dent_scr_off = 0, dent_tb_off = 0;
  int off_dict_walk = 0, off_bind = 0, off_fixd = 0, off_bin_cols = 0, off_carry = 0;  // into bin_lists
  uint32_t n_bin_blocks = 0, n_bin_chunks = 0, n_dba_chunks = 0;
  uint64_t dba_meta_off = ~0ull;  // DELTA_BYTE_ARRAY per-chunk {suffix base, smallest prefix} in bscratch
  uint32_t* dba_meta() const {
    return dba_meta_off == ~0ull ? nullptr : (uint32_t*)((uint8_t*)bscratch.p + dba_meta_off);
  }
  std::vector<uint64_t> bin_total_off;  // per column: byte offset of its bin_total in bscratch (or ~0)
  std::vector<uint64_t> bin_capacity;
  std::vector<int> col_first_page;
  std::vector<void*> empty_bin_values; // BYTE_ARRAY columns without slots: offsets[0] = 0
  std::vector<PageWork> h_work;
  std::vector<int> cls_off, cls_n;  // into lists
  int levels_off = 0, levels_n = 0;
  int n_scan_cols = 0;
  std::vector<int> page_cls;        // -1 if not launched
  std::vector<uint8_t> col_nullable;
  std::vector<uint64_t> col_required_values;
  std::vector<HostErr> host_errs;
  std::vector<pqg_page_error> page_errs;  // per page, resolved by pqg_sync (pqg_page_errors)
  int kernels = 0;
  DevBuf segs;                        // PLAIN BYTE_ARRAY segments (k_bin_walk_seg): page | s << 32 | last << 63
  uint32_t n_segs = 0;
  uint64_t seg_status_off = 0, seg_tmp_off = 0;  // in bscratch: status words + ticket (cleared per launch), scratch
  int timeout_fallbacks = 0;           // launches re-run in split mode after PQG_ERR_TIMEOUT (pqg_sync)
  // PLAIN-only BYTE_ARRAY columns in one pass (k_bin_bases + k_bin_plain); the per-value path's lists
  // hold those columns' entries last, so plain_fused launches skip them (pqg_sync turns plain_fused
  // off when a page's values do not fill its data section)
  bool plain_fused = false;
  bool plain_pg = false;  // ... through k_bin_plain_pg (one wave per page) instead of the tiles
  int n_pcp = 0;          // pages of those columns (pcol_pages)
  int plain_fallbacks = 0;
  DevBuf psegs, pstatus, pcol_pages, pcol_start;  // tiles (page | tile << 32); aggw + incw per tile; column page lists
  uint32_t n_psegs = 0, pseg_epoch = 0;
  int n_pcols = 0;
  uint64_t pticket_off = 0, pflag_off = 0;  // in bscratch: ticket (cleared per launch), inexact flag (epoch-tagged)
  uint64_t blen_bytes_nf = 0;               // cleared part of bscratch when plain_fused
  int n_binp_fused = 0, n_bin_cols_nf = 0;  // tails of cls_lists[C_BINP] / bin_cols that belong to those columns
  // pages k_bin_walk_seg walks (the last n_binp_seg of cls_lists[C_BINP], after the one-pass columns'
  // pages); seg_walk false: one wave per page instead (pqg_sync's re-run after a segment wait timed out)
  int n_binp_seg = 0;
  bool seg_walk = true;
  uint32_t n_bin_blocks_nf = 0, n_bin_chunks_nf = 0;
  // V2 header null counts (PQG_PAGE_NULL_COUNT): every nullable page of the plan carries one, so the
  // host filled those pages' n_values / data_begin / out_offset and the value kernels start beside
  // k_levels, which verifies the counts into the epoch-tagged word at hint_off (bscratch); a mismatch
  // makes pqg_sync re-run level-first, and the plan keeps that order (null_hints false)
  bool null_hints = false;
  uint64_t hint_off = 0;
  int hint_fallbacks = 0;
  uint32_t* d_counts = nullptr;  // pqg_decode's d_page_value_counts (refreshed after a re-run)
};

// pqg_router_read_page: the bit-packed runs of a hybrid stream's tail, walked on the host at the first
// read of a page, unpacked on the device in one round trip and served from host memory by the later
// reads (ParquetReadRouter.read: the values are in the caller's buffer when the call returns).
struct RouterCache {
  int w = -1;
  uint64_t tail_len = 0;        // bytes from the walked tail's start to the stream's end
  std::vector<uint8_t> bytes;   // the tail (a cached run is served only when its bytes equal the request's)
  std::vector<uint64_t> off;    // run data start, relative to the tail start (ascending)
  std::vector<uint32_t> cnt;    // values of the run
  std::vector<uint64_t> vo;     // first value of the run in vals
  std::vector<int32_t> vals;
  uint64_t hits = 0, misses = 0;
};

struct pqg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  pqg_plan* last = nullptr;          // plan of the most recent pqg_decode (owned)
  pqg_plan* last_launched = nullptr; // plan of the most recent launch (decode or plan_launch)
  std::vector<pqg_plan*> unsynced;   // plans launched since the last pqg_sync, in launch order
  std::vector<pqg_staged_output> staged;  // pqg_decode_staged: where each column's outputs are in pin_out
  pqg_column_desc* last_cols = nullptr;
  PinnedBuf pin_in, pin_out, pin_err;
  DevBuf host_bytes, host_out, host_counts, host_runs;
  DevBuf asm_scratch;                // pqg_assemble: block counts + totals
  hipStream_t copy_stream = nullptr; // pqg_decode_host: second D2H queue (odd output chunks)
  DevBuf zstd_scratch;               // pqg_zstd_decompress: literal buffers, ZSTD_LIT_SCRATCH per grid wave
  DevBuf zstd_seqs, zstd_mode;       // pqg_zstd_decompress: sequence records of the lane-per-page pre-pass, per-job mode
  DevBuf gzip_recs, gzip_mode;       // pqg_gzip_decompress: back-reference records of the token pre-pass, per-job count
  // pqg_plan_launch: the one-pass PLAIN BYTE_ARRAY kernel runs on a second queue beside the other
  // columns' kernels (forked after the levels, joined before the launch ends)
  hipStream_t side_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // ... and the BYTE_ARRAY kernels of the other columns (dictionary walk / ids / map, per-value walks,
  // offset scan, copies) on a third, beside the fixed-width columns' kernels
  hipStream_t bin_stream = nullptr;
  hipEvent_t ev_join_bin = nullptr;
  // ... and the fixed-width columns' kernels on a fourth. The three are created one after the other
  // with the context, so that HIP's round-robin puts them on different hardware queues; the caller's
  // stream only waits while they run (a queue shared with it costs nothing then).
  hipStream_t fix_stream = nullptr;
  hipEvent_t ev_join_fix = nullptr;
  // ... and the tile walk of large dictionaries beside the id walk of their dictionary-direct pages, whose
  // ids need no entries (C_DDG: the entries are first read by k_dd_gsums, which waits for ev_dent)
  hipStream_t dent_stream = nullptr;
  hipEvent_t ev_dent_fork = nullptr, ev_dent = nullptr;
  // pqg_ctx_set_dispatch: kernel-choice overrides for the plans created on this ctx
  int plain_mode = 2;       // PQG_DISPATCH_PLAIN_ONE_PASS
  bool dict_direct = true;  // PQG_DISPATCH_DICT_DIRECT
  bool dict_fused = true;   // PQG_DISPATCH_DICT_FUSED
  bool null_hints = true;   // PQG_DISPATCH_NULL_HINTS
  uint32_t gz_prepass_min = pqg::GZ_PREPASS_MIN;  // PQG_DISPATCH_GZIP_PREPASS_MIN
  RouterCache router;  // pqg_router_read_page
};

extern "C" {

int pqg_abi_version(void) { return PQG_ABI_VERSION; }

const char* pqg_error_name(int code) {
  switch (code) {
    case PQG_OK: case PQG_ERR_INVALID_ARG: case PQG_ERR_UNSUPPORTED: case PQG_ERR_HIP: case PQG_ERR_NO_DEVICE:
      return kNames[code];
    case PQG_ERR_TIMEOUT: return "TIMEOUT";
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
    case PQG_ERR_CRC: return "CRC";
    default: return "UNKNOWN";
  }
}

int pqg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pqg_ctx_create(int device, void* hip_stream, pqg_ctx** out) {
  if (!out) return PQG_ERR_INVALID_ARG;
  *out = nullptr;
  int n = pqg_device_count();
  if (n <= 0) return PQG_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(device) != hipSuccess) return PQG_ERR_HIP;
  pqg_ctx* c = new (std::nothrow) pqg_ctx();
  if (!c) return PQG_ERR_INVALID_ARG;
  c->device = device;
  if (hip_stream) {
    c->stream = (hipStream_t)hip_stream;
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      return PQG_ERR_HIP;
    }
    c->own_stream = true;
  }
  if (hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking) != hipSuccess) c->side_stream = nullptr;
  if (hipStreamCreateWithFlags(&c->bin_stream, hipStreamNonBlocking) != hipSuccess) c->bin_stream = nullptr;
  if (hipStreamCreateWithFlags(&c->fix_stream, hipStreamNonBlocking) != hipSuccess) c->fix_stream = nullptr;
  *out = c;
  return PQG_OK;
}

void* pqg_ctx_stream(pqg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int pqg_ctx_set_dispatch(pqg_ctx* ctx, int key, int value) {
  if (!ctx) return PQG_ERR_INVALID_ARG;
  switch (key) {
    case PQG_DISPATCH_PLAIN_ONE_PASS:
      if (value < 0 || value > 3) return PQG_ERR_INVALID_ARG;
      ctx->plain_mode = value;
      return PQG_OK;
    case PQG_DISPATCH_DICT_DIRECT:
      if (value != 0 && value != 1) return PQG_ERR_INVALID_ARG;
      ctx->dict_direct = value != 0;
      return PQG_OK;
    case PQG_DISPATCH_GZIP_PREPASS_MIN:
      if (value < 0) return PQG_ERR_INVALID_ARG;
      ctx->gz_prepass_min = (uint32_t)value;
      return PQG_OK;
    case PQG_DISPATCH_DICT_FUSED:
      if (value != 0 && value != 1) return PQG_ERR_INVALID_ARG;
      ctx->dict_fused = value != 0;
      return PQG_OK;
    case PQG_DISPATCH_NULL_HINTS:
      if (value != 0 && value != 1) return PQG_ERR_INVALID_ARG;
      ctx->null_hints = value != 0;
      return PQG_OK;
    default: return PQG_ERR_INVALID_ARG;
  }
}

int pqg_plan_destroy(pqg_plan* p);

int pqg_ctx_destroy(pqg_ctx* c) {
  if (!c) return PQG_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->last) pqg_plan_destroy(c->last);
  c->pin_in.release();
  c->pin_out.release();
  c->pin_err.release();
  c->host_bytes.release();
  c->host_out.release();
  c->host_counts.release();
  c->host_runs.release();
  c->asm_scratch.release();
  c->zstd_scratch.release();
  c->zstd_seqs.release();
  c->zstd_mode.release();
  c->gzip_recs.release();
  c->gzip_mode.release();
  if (c->copy_stream) {
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamDestroy(c->copy_stream);
  }
  if (c->side_stream) {
    (void)hipStreamSynchronize(c->side_stream);
    (void)hipStreamDestroy(c->side_stream);
  }
  if (c->bin_stream) {
    (void)hipStreamSynchronize(c->bin_stream);
    (void)hipStreamDestroy(c->bin_stream);
  }
  if (c->ev_join_bin) (void)hipEventDestroy(c->ev_join_bin);
  if (c->fix_stream) {
    (void)hipStreamSynchronize(c->fix_stream);
    (void)hipStreamDestroy(c->fix_stream);
  }
  if (c->ev_join_fix) (void)hipEventDestroy(c->ev_join_fix);
  if (c->dent_stream) {
    (void)hipStreamSynchronize(c->dent_stream);
    (void)hipStreamDestroy(c->dent_stream);
  }
  if (c->ev_dent_fork) (void)hipEventDestroy(c->ev_dent_fork);
  if (c->ev_dent) (void)hipEventDestroy(c->ev_dent);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return PQG_OK;
}

// valid_bytes: the caller's data ends there (page and dictionary extents are checked against it); the
// kernels may read up to n_bytes (pqg_decode_host's zero padding past the caller's bytes)
// Kernels one launch of the plan runs (in its current modes).
static int count_kernels(const pqg_plan* P) {
  const bool pf = P->plain_fused;
  int k = (P->levels_n ? 1 : 0) + (P->n_scan_cols && !P->null_hints ? 1 : 0);
  for (int c = 0; c < C_NCLS; c++) {
    const int n = P->cls_n[(size_t)c] - (c == C_BINP ? P->n_binp_seg + (pf ? P->n_binp_fused : 0) : 0);
    if (n && c == C_DD) k += P->dict_fused ? 3 : 4;
    else if (n && c == C_DDG) k += P->dict_fused ? 4 : 5;
    else if (n) k += (c == C_DICT4 || c == C_DICT8 || c == C_IDS) && !P->dict_fused ? 2 : 1;
  }
  k += (P->n_dict_walk ? 1 : 0) + (P->n_dent_tiles ? 3 : 0) + (P->n_bind ? 1 : 0) + (P->n_fixd ? 1 : 0) +
       ((pf ? P->n_bin_blocks_nf : P->n_bin_blocks) ? 3 : 0) + ((pf ? P->n_bin_chunks_nf : P->n_bin_chunks) ? 1 : 0) +
       (P->cls_n[C_DBA] ? (P->n_dba_chunks ? 4 : 1) : 0) + (P->n_carry ? 1 : 0) + (P->n_segs ? 1 : 0) +
       (pf ? 2 : 0);
  return k;
}

static int plan_create_impl(pqg_ctx* ctx, const uint8_t* d_bytes, uint64_t n_bytes, uint64_t valid_bytes,
                            const pqg_column_desc* cols, int n_cols, const pqg_page_desc* pages, int n_pages,
                            pqg_plan** out, pqg_status* st) {
  if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
  if (!ctx || !out || n_cols < 0 || n_pages < 0 || (n_cols && !cols) || (n_pages && !pages) || (n_bytes && !d_bytes) ||
      ((uintptr_t)d_bytes & 3u)) {  // the batch buffer is read as dwords (scalar loads): 4-byte aligned
    set_status(st, PQG_ERR_INVALID_ARG, -1, -1, "plan arguments");
    return PQG_ERR_INVALID_ARG;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  pqg_plan* P = new (std::nothrow) pqg_plan();
  if (!P) return PQG_ERR_INVALID_ARG;
  P->ctx = ctx;
  P->dict_fused = ctx->dict_fused;
  P->d_bytes = d_bytes;
  P->n_bytes = n_bytes;
  P->n_pages = n_pages;
  P->n_cols = n_cols;
  // ---- columns
  std::vector<ColumnDev> hc((size_t)std::max(n_cols, 1));
  std::vector<int> col_err((size_t)std::max(n_cols, 1), 0);
  std::vector<int> col_first_page((size_t)std::max(n_cols, 1), -1);
  P->col_nullable.assign((size_t)std::max(n_cols, 1), 0);
  P->col_required_values.assign((size_t)std::max(n_cols, 1), 0);
  for (int i = 0; i < n_cols; i++) {
    const pqg_column_desc& c = cols[i];
    ColumnDev& d = hc[(size_t)i];
    std::memset(&d, 0, sizeof(d));
    d.physical_type = c.physical_type;
    d.type_length = c.type_length;
    d.max_rep = c.max_rep;
    d.max_def = c.max_def;
    d.elem_width = elem_width(c.physical_type, c.type_length);
    d.values = c.values;
    d.binary_data = c.binary_data;
    d.binary_capacity = bin_out(c) ? c.binary_capacity : 0;
    d.def_levels = c.max_def > 0 ? c.def_levels : nullptr;
    d.rep_levels = c.max_rep > 0 ? c.rep_levels : nullptr;
    P->col_nullable[(size_t)i] = (c.max_def > 0 || c.max_rep > 0) ? 1 : 0;
    if (c.max_def > 254 || c.max_rep > 254 || c.max_def < 0 || c.max_rep < 0) col_err[(size_t)i] = PQG_ERR_UNSUPPORTED;
    if (c.dict_offset >= 0) {
      // PlainValuesDictionary ctor :47-53 and the typed readers: validated from the descriptor
      if (c.dict_encoding != PQG_PLAIN && c.dict_encoding != PQG_PLAIN_DICTIONARY) {
        col_err[(size_t)i] = PQG_ERR_DICT_ENCODING;
      } else if (c.physical_type == PQG_BOOLEAN) {
        col_err[(size_t)i] = PQG_ERR_UNSUPPORTED;
      } else if (c.physical_type == PQG_FIXED_LEN_BYTE_ARRAY && c.type_length <= 0) {
        col_err[(size_t)i] = PQG_ERR_CORRUPT;  // PlainBinaryDictionary :106 checkArgument(length > 0)
      } else if ((uint64_t)c.dict_offset + c.dict_size > valid_bytes) {
        col_err[(size_t)i] = PQG_ERR_INVALID_ARG;
      } else if (d.elem_width > 0 && (uint64_t)c.dict_num_values * (uint64_t)d.elem_width > c.dict_size) {
        col_err[(size_t)i] = PQG_ERR_EOF;
      }
      d.dict_n = c.dict_num_values;
      d.dict_offset = (uint64_t)c.dict_offset;
      d.dict_bytes = c.dict_size;
    }
  }
  // ---- pages
  P->h_work.resize((size_t)std::max(n_pages, 1));
  P->page_cls.assign((size_t)std::max(n_pages, 1), -1);
  std::vector<std::vector<int>> cls_lists(C_NCLS);
  std::vector<int> lvl_list;
  std::vector<std::vector<int>> col_pages((size_t)std::max(n_cols, 1));
  std::vector<uint64_t> slot_acc((size_t)std::max(n_cols, 1), 0), val_acc((size_t)std::max(n_cols, 1), 0);
  // per column: class of its previous page (-2: none yet; PQG_PAGE_DBA_CARRY needs a DELTA_BYTE_ARRAY
  // one), FIXED_LEN_BYTE_ARRAY with DELTA_BYTE_ARRAY pages, any carry page
  std::vector<int> col_last_cls((size_t)std::max(n_cols, 1), -2);
  std::vector<uint8_t> dba_fixed((size_t)std::max(n_cols, 1), 0), dba_carry((size_t)std::max(n_cols, 1), 0);
  for (int p = 0; p < n_pages; p++) {
    const pqg_page_desc& g = pages[p];
    PageWork& w = P->h_work[(size_t)p];
    std::memset(&w, 0, sizeof(w));
    if (g.column < 0 || g.column >= n_cols || g.offset + g.size > valid_bytes || g.offset + g.size < g.offset || (g.version != 1 && g.version != 2)) {
      set_status(st, PQG_ERR_INVALID_ARG, p, -1, "page descriptor");
      delete P;
      return PQG_ERR_INVALID_ARG;
    }
    const int ci = g.column;
    const pqg_column_desc& c = cols[ci];
    if (col_first_page[(size_t)ci] < 0) {
      col_first_page[(size_t)ci] = p;
      if (col_err[(size_t)ci]) P->host_errs.push_back(HostErr{p, 0, -1, col_err[(size_t)ci]});
    }
    w.base = g.offset;
    w.size = g.size;
    w.num_slots = g.num_values;
    w.column = ci;
    w.version = g.version;
    w.rl_encoding = g.rl_encoding;
    w.dl_encoding = g.dl_encoding;
    w.rl_len = g.rl_byte_length;
    w.dl_len = g.dl_byte_length;
    w.pflags = g.flags;
    w.slot_offset = slot_acc[(size_t)ci];
    slot_acc[(size_t)ci] += g.num_values;
    const bool nullable = P->col_nullable[(size_t)ci] != 0;
    if (!nullable) {
      // required column: no level sections are consumed (ZeroIntegerValuesReader / BIT_PACKED
      // width 0 / NullIntIterator), values = header num_values
      if (g.version == 1 && ((g.rl_encoding != PQG_RLE && g.rl_encoding != PQG_BIT_PACKED) ||
                             (g.dl_encoding != PQG_RLE && g.dl_encoding != PQG_BIT_PACKED))) {
        P->host_errs.push_back(HostErr{p, 0, 0, PQG_ERR_UNSUPPORTED});
        continue;
      }
      uint64_t lv = g.version == 2 ? (uint64_t)g.rl_byte_length + g.dl_byte_length : 0;
      if (lv > g.size) {
        P->host_errs.push_back(HostErr{p, 0, 0, PQG_ERR_CORRUPT});
        continue;
      }
      w.data_begin = (uint32_t)lv;
      w.n_values = g.num_values;
      w.out_offset = val_acc[(size_t)ci];
      val_acc[(size_t)ci] += g.num_values;
    } else {
      lvl_list.push_back(p);
      col_pages[(size_t)ci].push_back(p);
    }
    const int last_cls = col_last_cls[(size_t)ci];
    col_last_cls[(size_t)ci] = -1;
    if (col_err[(size_t)ci]) continue;  // dictionary page unusable: ColumnReaderBase ctor threw
    // value class (Encoding.getValuesReader / getDictionaryBasedValuesReader dispatch)
    const int t = c.physical_type;
    const int ew = elem_width(t, c.type_length);
    int cls = -1, herr = 0;
    if (ids_mode(c)) {
      // readValueDictionaryId: dictionary pages give their ids (any physical type, k_dict_fused<4, IDS>
      // writing straight into the column's uint32 values); other readers throw (ValuesReader.java:123-125)
      if (g.encoding != PQG_PLAIN_DICTIONARY && g.encoding != PQG_RLE_DICTIONARY) herr = PQG_ERR_UNSUPPORTED;
      else if (c.dict_offset < 0) herr = PQG_ERR_NO_DICTIONARY;
      else if (t == PQG_BOOLEAN) herr = PQG_ERR_UNSUPPORTED;
      else cls = C_IDS;
    } else
    switch (g.encoding) {
      case PQG_PLAIN_DICTIONARY:
      case PQG_RLE_DICTIONARY:
        if (c.dict_offset < 0) herr = PQG_ERR_NO_DICTIONARY;
        else if (t == PQG_BOOLEAN) herr = PQG_ERR_UNSUPPORTED;
        else if (t == PQG_BYTE_ARRAY) { cls = C_IDS; w.bin_kind = pqg::BIN_DICT; }
        else if (ew == 8) cls = C_DICT8;
        else if (ew == 4) cls = C_DICT4;
        else if (ew > 0) cls = C_IDS;      // FLBA / INT96: ids, then k_gather_fixed
        else herr = PQG_ERR_UNSUPPORTED;
        break;
      case PQG_PLAIN:
        if (t == PQG_BOOLEAN) cls = C_BOOL;
        else if (t == PQG_BYTE_ARRAY) { cls = C_BINP; w.bin_kind = pqg::BIN_PLAIN; }
        else if (ew > 0) cls = C_PLAIN;
        else herr = PQG_ERR_UNSUPPORTED;
        break;
      case PQG_RLE:  // Encoding.RLE values: BOOLEAN only (getMaxLevel :255-271)
        if (t == PQG_BOOLEAN) cls = C_RLEBOOL;
        else herr = PQG_ERR_UNSUPPORTED;
        break;
      case PQG_DELTA_BINARY_PACKED:
        if (t == PQG_INT64) cls = C_DELTA8;
        else if (t == PQG_INT32) cls = C_DELTA4;
        else herr = PQG_ERR_UNSUPPORTED;
        break;
      case PQG_DELTA_LENGTH_BYTE_ARRAY:
        if (t == PQG_BYTE_ARRAY) { cls = C_DLBA; w.bin_kind = pqg::BIN_DLBA; }
        else herr = PQG_ERR_UNSUPPORTED;   // Encoding.java :204-207
        break;
      case PQG_BYTE_STREAM_SPLIT:
        if (t == PQG_FLOAT || t == PQG_DOUBLE || t == PQG_INT32 || t == PQG_INT64 ||
            (t == PQG_FIXED_LEN_BYTE_ARRAY && ew > 0))
          cls = C_BSS;
        else
          herr = PQG_ERR_UNSUPPORTED;      // Encoding.java :130-143
        break;
      case PQG_DELTA_BYTE_ARRAY:
        // Encoding.java :219-222: BYTE_ARRAY and FIXED_LEN_BYTE_ARRAY (whose values must then be
        // type_length bytes each: k_delta reports any other length as PQG_ERR_CORRUPT)
        if (t == PQG_BYTE_ARRAY || (t == PQG_FIXED_LEN_BYTE_ARRAY && ew > 0)) {
          cls = C_DBA;
          w.bin_kind = pqg::BIN_DBA;
          if (t == PQG_FIXED_LEN_BYTE_ARRAY) dba_fixed[(size_t)ci] = 1;
          if (g.flags & PQG_PAGE_DBA_CARRY) {
            // setPreviousReader casts the previous page's reader to DeltaByteArrayReader
            if (last_cls != -2 && last_cls != C_DBA) { cls = -1; herr = PQG_ERR_UNSUPPORTED; }
            else dba_carry[(size_t)ci] = 1;
          }
        } else {
          herr = PQG_ERR_UNSUPPORTED;
        }
        break;
      default:
        herr = PQG_ERR_UNSUPPORTED;
    }
    if (herr) {
      P->host_errs.push_back(HostErr{p, 0, 2, herr});
      continue;
    }
    P->page_cls[(size_t)p] = cls;
    col_last_cls[(size_t)ci] = cls;
    cls_lists[(size_t)cls].push_back(p);
  }
  for (int i = 0; i < n_cols; i++) P->col_required_values[(size_t)i] = val_acc[(size_t)i];
  P->col_first_page = col_first_page;
  // V2 header null counts as a verified hint (PQG_PAGE_NULL_COUNT): only when every nullable page of the
  // plan carries a usable one, so that no value kernel has to wait for k_levels
  if (ctx->null_hints && !lvl_list.empty()) {
    bool all = true;
    for (int p : lvl_list) {
      const pqg_page_desc& g = pages[p];
      all = all && g.version == 2 && (g.flags & PQG_PAGE_NULL_COUNT) && g.num_nulls <= g.num_values &&
            (uint64_t)g.rl_byte_length + g.dl_byte_length <= g.size;
    }
    if (all) {
      std::vector<uint64_t> acc((size_t)std::max(n_cols, 1), 0);
      for (int p : lvl_list) {  // (page order within each column)
        const pqg_page_desc& g = pages[p];
        PageWork& w = P->h_work[(size_t)p];
        w.n_values = g.num_values - g.num_nulls;
        w.data_begin = g.rl_byte_length + g.dl_byte_length;
        w.out_offset = acc[(size_t)g.column];
        acc[(size_t)g.column] += w.n_values;
      }
      P->null_hints = true;
    }
  }
  // ---- BYTE_ARRAY and fixed-width dictionary columns: scratch layout, dictionary walks,
  // post-passes, offset-scan blocks and copy chunks
  std::vector<int32_t> dict_walk, bind, fixd, bin_cols, carry_cols, dent_cols;
  std::vector<uint64_t> bin_blocks, bin_chunks;
  std::vector<uint64_t> blen_off((size_t)std::max(n_cols, 1), ~0ull), bsrc_off = blen_off, dlen_off = blen_off,
      dsrc_off = blen_off, bsum_off = blen_off, dent_off = blen_off;
  P->bin_total_off.assign((size_t)std::max(n_cols, 1), ~0ull);
  P->bin_capacity.assign((size_t)std::max(n_cols, 1), 0);
  uint64_t sc = 0;
  auto take = [&](uint64_t bytes) { uint64_t o = sc; sc = (sc + bytes + 255) & ~uint64_t(255); return o; };
  std::vector<uint8_t> needs_ids((size_t)std::max(n_cols, 1), 0);
  for (int p : cls_lists[C_IDS]) needs_ids[(size_t)P->h_work[(size_t)p].column] = 1;
  // PLAIN-only BYTE_ARRAY columns (every page PLAIN, no descriptor error, < 2^24 - 1 slots per page):
  // one pass: k_bin_bases + k_bin_plain over 2 KiB tiles of their pages when the plan has fewer than
  // BW_SEG_MAX_PAGES PLAIN pages, k_bin_plain_pg (one wave per page, which fills the chip) with more
  // (there the tiles measured slower than the per-value walk + copy: C3 10.4 vs 6.4 ms, profiles/r03/plain_ab)
  // pqg_ctx_set_dispatch(PQG_DISPATCH_PLAIN_ONE_PASS) overrides the choice (tests and A/B): 0 = no
  // one-pass path (every plan per value), 3 = every plan one wave per page
  const int plain_mode = ctx->plain_mode;
  const bool many_plain = (cls_lists[C_BINP].size() >= pqg::BW_SEG_MAX_PAGES && plain_mode != 1) || plain_mode == 3;
  P->plain_pg = many_plain;
  std::vector<uint8_t> plain_col((size_t)std::max(n_cols, 1), 0);
  std::vector<uint64_t> psegs;
  std::vector<int32_t> pcp, pcs(1, 0);
  {
    std::vector<int> npg((size_t)std::max(n_cols, 1), 0), nplain((size_t)std::max(n_cols, 1), 0);
    std::vector<std::vector<int>> cpg((size_t)std::max(n_cols, 1));
    for (int p = 0; p < n_pages; p++) {
      const int c = P->h_work[(size_t)p].column;
      npg[(size_t)c]++;
      cpg[(size_t)c].push_back(p);
      if (P->page_cls[(size_t)p] == C_BINP && P->h_work[(size_t)p].num_slots < (1u << 24) - 1u) nplain[(size_t)c]++;
    }
    for (int i = 0; i < n_cols; i++) {
      plain_col[(size_t)i] = bin_out(cols[i]) && !ids_mode(cols[i]) && !col_err[(size_t)i] && !dba_fixed[(size_t)i] &&
                             npg[(size_t)i] > 0 && nplain[(size_t)i] == npg[(size_t)i] && plain_mode != 0;
      if (!plain_col[(size_t)i]) continue;
      for (int p : cpg[(size_t)i]) {
        pcp.push_back(p);
        if (many_plain) continue;
        const uint32_t ntile = std::max<uint32_t>((P->h_work[(size_t)p].size + pqg::BP_TILE - 1) / pqg::BP_TILE, 1u);
        for (uint32_t k = 0; k < ntile; k++) psegs.push_back((uint64_t)(uint32_t)p | ((uint64_t)k << 32));
      }
      pcs.push_back((int32_t)pcp.size());
    }
  }
  // dictionary-direct BYTE_ARRAY columns (ColumnDev::dict_direct): every data page dictionary-encoded,
  // the dictionary page small enough to stage (DD_DICT_MAX bytes, at most 2,048 entries): their pages
  // leave C_IDS for C_DD (no ids stored, no offset scan or copy of their own). Nullable and nested
  // columns too (round 6): the walk decodes a page's n_values ids from its data section, which k_levels
  // (or the V2 header counts) give, and values are indexed by out_offset like every other class.
  // Larger dictionaries (at most 65,536 entries: u16 ids) take C_DDG: their entries and value bytes are
  // gathered from HBM instead of LDS (k_dd_gsums / k_dd_gstr; round 6)
  std::vector<uint8_t> dict_direct((size_t)std::max(n_cols, 1), 0), dd_glob((size_t)std::max(n_cols, 1), 0);
  {
    std::vector<int> npg((size_t)std::max(n_cols, 1), 0), nids((size_t)std::max(n_cols, 1), 0);
    for (int p = 0; p < n_pages; p++) {
      const int c = P->h_work[(size_t)p].column;
      npg[(size_t)c]++;
      if (P->page_cls[(size_t)p] == C_IDS) nids[(size_t)c]++;
    }
    for (int i = 0; i < n_cols; i++)
      dict_direct[(size_t)i] = cols[i].physical_type == PQG_BYTE_ARRAY && bin_out(cols[i]) && !ids_mode(cols[i]) &&
                               !col_err[(size_t)i] && !dba_fixed[(size_t)i] && !plain_col[(size_t)i] &&
                               cols[i].dict_offset >= 0 && cols[i].dict_num_values <= 65536 &&
                               npg[(size_t)i] > 0 && nids[(size_t)i] == npg[(size_t)i] && ctx->dict_direct;
    for (int i = 0; i < n_cols; i++)
      dd_glob[(size_t)i] = dict_direct[(size_t)i] &&
                           (cols[i].dict_size > pqg::DD_DICT_MAX || cols[i].dict_num_values > 2048);
    std::vector<int> keep, dd, ddg;
    for (int p : cls_lists[C_IDS]) {
      const int c = P->h_work[(size_t)p].column;
      (!dict_direct[(size_t)c] ? keep : dd_glob[(size_t)c] ? ddg : dd).push_back(p);
    }
    auto by_col = [&](int a, int b) { return P->h_work[(size_t)a].column < P->h_work[(size_t)b].column; };
    std::stable_sort(dd.begin(), dd.end(), by_col);
    std::stable_sort(ddg.begin(), ddg.end(), by_col);
    for (int p : dd) P->page_cls[(size_t)p] = C_DD;
    for (int p : ddg) P->page_cls[(size_t)p] = C_DDG;
    cls_lists[C_IDS].swap(keep);
    cls_lists[C_DD].swap(dd);
    cls_lists[C_DDG].swap(ddg);
  }
  // PLAIN BYTE_ARRAY pages walked in segments when there are few of them (k_bin_walk_seg)
  std::vector<uint64_t> segs;
  std::vector<uint8_t> seg_page((size_t)std::max(n_pages, 1), 0);
  if (!cls_lists[C_BINP].empty() && cls_lists[C_BINP].size() < pqg::BW_SEG_MAX_PAGES) {
    for (int p : cls_lists[C_BINP]) {
      const PageWork& w = P->h_work[(size_t)p];
      if (plain_col[(size_t)w.column]) continue;  // one pass (k_bin_plain); the per-value fallback walks per page
      const uint32_t nseg = (w.size + pqg::BW_SEG_BYTES - 1) / pqg::BW_SEG_BYTES + 1;  // + 1: tile alignment of the start
      if (nseg < 3) continue;
      seg_page[(size_t)p] = 1;
      for (uint32_t k = 0; k < nseg; k++)
        segs.push_back((uint64_t)(uint32_t)p | ((uint64_t)k << 32) | (k + 1 == nseg ? (1ull << 63) : 0ull));
    }
  }
  // blen first: the part cleared before every launch (with the one-pass columns' last: not cleared
  // while they take the one-pass path)
  for (int pass = 0; pass < 2; pass++) {
    for (int i = 0; i < n_cols; i++) {
      if (ids_mode(cols[i]) || dict_direct[(size_t)i] || (plain_col[(size_t)i] != 0) != (pass == 1))
        continue;  // ids go straight to the values; dictionary-direct columns store none
      if (bin_out(cols[i]) || needs_ids[(size_t)i] || dba_fixed[(size_t)i])
        blen_off[(size_t)i] = take(4 * (slot_acc[(size_t)i] + 1));
    }
    if (pass == 0) {
      if (!segs.empty()) P->seg_status_off = take(8 * (segs.size() + 1));  // + the ticket counter
      if (!pcp.empty()) P->pticket_off = take(8);
      P->blen_bytes_nf = sc;
    }
  }
  P->blen_bytes = sc;
  // dictionary-direct columns: compact ids (u8 for dictionaries of at most 256 entries, else u16), written
  // by k_dict_fused_dd for every slot k_dd_str reads (not cleared; padded: k_dd_str reads whole dwords)
  for (int i = 0; i < n_cols; i++)
    if (dict_direct[(size_t)i])
      blen_off[(size_t)i] = take((cols[i].dict_num_values <= 256 && !dd_glob[(size_t)i] ? 1u : 2u) * (slot_acc[(size_t)i] + 16));
  if (!pcp.empty()) P->pflag_off = take(8);
  if (P->null_hints) P->hint_off = take(8);
  if (!segs.empty()) P->seg_tmp_off = take(4 * 2 * (uint64_t)pqg::BW_SEG_CAP * segs.size());
  P->n_segs = (uint32_t)segs.size();
  for (int i = 0; i < n_cols; i++) {
    if (dba_fixed[(size_t)i]) bsrc_off[(size_t)i] = take(4 * (slot_acc[(size_t)i] + 1));  // prefix lengths
    if (dba_carry[(size_t)i]) carry_cols.push_back(i);
  }
  for (int i0 = 0; i0 < 2 * n_cols; i0++) {  // the one-pass columns last
    const int i = i0 % n_cols;
    if (!bin_out(cols[i]) || (plain_col[(size_t)i] != 0) != (i0 >= n_cols)) continue;
    P->bin_capacity[(size_t)i] = cols[i].binary_capacity;
    if (dict_direct[(size_t)i]) {  // the byte total (k_dd_bases) and the dictionary's entries only
      P->bin_total_off[(size_t)i] = take(8);
      // (dictionaries gathered from HBM: always the tile walk, whose scatter also packs their entries)
      ((cols[i].dict_size >= pqg::DENT_MIN || dd_glob[(size_t)i]) && cols[i].dict_num_values ? dent_cols : dict_walk)
          .push_back(i);
      if (dd_glob[(size_t)i]) dent_off[(size_t)i] = take(8 * ((uint64_t)cols[i].dict_num_values + 1));
      dlen_off[(size_t)i] = take(4 * ((uint64_t)cols[i].dict_num_values + 1));
      dsrc_off[(size_t)i] = take(4 * ((uint64_t)cols[i].dict_num_values + 1));
      continue;
    }
    bin_cols.push_back(i);
    bsrc_off[(size_t)i] = take(4 * (slot_acc[(size_t)i] + 1));
    const uint64_t nb = (slot_acc[(size_t)i] + pqg::SCAN_BLOCK - 1) / pqg::SCAN_BLOCK;
    bsum_off[(size_t)i] = take(8 * (nb + 1));
    P->bin_total_off[(size_t)i] = take(8);
    for (uint64_t b = 0; b < nb; b++) bin_blocks.push_back(((uint64_t)(uint32_t)i << 32) | b);
    if (nb == 0 && cols[i].values) P->empty_bin_values.push_back(cols[i].values);
    if (cols[i].dict_offset >= 0 && !col_err[(size_t)i]) {
      (cols[i].dict_size >= pqg::DENT_MIN && cols[i].dict_num_values ? dent_cols : dict_walk).push_back(i);
      dlen_off[(size_t)i] = take(4 * ((uint64_t)cols[i].dict_num_values + 1));
      dsrc_off[(size_t)i] = take(4 * ((uint64_t)cols[i].dict_num_values + 1));
    }
  }
  {  // bin_cols / bin_blocks of the one-pass columns form the tails
    int nf = 0;
    for (int c : bin_cols) nf += plain_col[(size_t)c] ? 0 : 1;
    P->n_bin_cols_nf = nf;
    uint32_t nb = 0;
    for (uint64_t b : bin_blocks) nb += plain_col[(size_t)(b >> 32)] ? 0 : 1;
    P->n_bin_blocks_nf = nb;
  }
  std::vector<uint64_t> plain_chunks;  // copy chunks of the one-pass columns (per-value fallback only)
  for (int k : {C_IDS, C_BINP, C_DLBA})
    for (int p : cls_lists[(size_t)k]) {
      const PageWork& w = P->h_work[(size_t)p];
      if (k == C_BINP && plain_col[(size_t)w.column]) {
        const uint32_t nch = (w.num_slots + pqg::CP_CHUNK_VALUES - 1) / pqg::CP_CHUNK_VALUES;
        for (uint32_t j = 0; j < nch; j++) plain_chunks.push_back((uint64_t)(uint32_t)p | ((uint64_t)j << 32));
        continue;
      }
      if (k == C_IDS && ids_mode(cols[w.column])) continue;  // the ids are the output
      if (k == C_IDS && dict_direct[(size_t)w.column]) continue;  // the offset scan writes the bytes
      if (k == C_IDS && cols[w.column].physical_type != PQG_BYTE_ARRAY) {
        fixd.push_back(p);
        continue;
      }
      if (k == C_IDS) bind.push_back(p);
      const uint32_t nch = (w.num_slots + pqg::CP_CHUNK_VALUES - 1) / pqg::CP_CHUNK_VALUES;
      for (uint32_t j = 0; j < nch; j++) bin_chunks.push_back((uint64_t)(uint32_t)p | ((uint64_t)j << 32));
    }
  P->n_bin_chunks_nf = (uint32_t)bin_chunks.size();
  bin_chunks.insert(bin_chunks.end(), plain_chunks.begin(), plain_chunks.end());
  {  // PLAIN pages: walked by k_bin_walk_seg (not listed), one wave per page, the one-pass columns last
    std::vector<int> keep, tail, seg;
    for (int p : cls_lists[C_BINP]) {
      if (plain_col[(size_t)P->h_work[(size_t)p].column]) tail.push_back(p);
      else if (!seg_page[(size_t)p]) keep.push_back(p);
      else seg.push_back(p);
    }
    P->n_binp_fused = (int)tail.size();
    P->n_binp_seg = (int)seg.size();
    keep.insert(keep.end(), tail.begin(), tail.end());
    keep.insert(keep.end(), seg.begin(), seg.end());
    cls_lists[C_BINP].swap(keep);
  }
  // ---- DELTA_BYTE_ARRAY pages: BIN_CHUNK-value chunks (upper bound from the slot count)
  std::vector<uint64_t> dba_chunks;
  for (int p : cls_lists[C_DBA]) {
    PageWork& w = P->h_work[(size_t)p];
    w.chunk_base = (uint32_t)dba_chunks.size();
    w.reserved = 0;
    const uint32_t nch = (w.num_slots + pqg::BIN_CHUNK - 1) / pqg::BIN_CHUNK;
    for (uint32_t j = 0; j < nch; j++) dba_chunks.push_back((uint64_t)(uint32_t)p | ((uint64_t)j << 32));
  }
  if (!dba_chunks.empty()) P->dba_meta_off = take(8 * dba_chunks.size());
  P->n_dba_chunks = (uint32_t)dba_chunks.size();
  // ---- dictionary pages: run-record capacity (a run covers >= 1 value and its header takes
  // >= 1 byte) and output chunks (slots [j*CH, (j+1)*CH) of the page, upper bound from the slot count)
  std::vector<uint64_t> chunk_list;
  uint64_t rec_total = 0;
  uint32_t chunk_total = 0;
  for (int k = C_DICT4; k < C_DICT4 + N_DICT_CLS; k++) {
    P->chunk_off[k - C_DICT4] = (uint32_t)chunk_list.size();
    for (int p : cls_lists[(size_t)k]) {
      PageWork& w = P->h_work[(size_t)p];
      const int ew = k == C_DICT8 ? 8 : 4;
      const uint32_t ch = pqg::dict_chunk_values(ew);
      w.rec_base = rec_total;
      rec_total += (uint64_t)std::min<uint32_t>(w.num_slots, w.size) + 1;
      w.chunk_base = chunk_total;
      const uint32_t nch = (uint32_t)(((uint64_t)w.num_slots + (uint32_t)(16 / ew) - 1 + ch - 1) / ch);
      for (uint32_t j = 0; j < nch; j++) chunk_list.push_back((uint64_t)(uint32_t)p | ((uint64_t)j << 32));
      chunk_total += nch;
    }
    P->chunk_n[k - C_DICT4] = (uint32_t)chunk_list.size() - P->chunk_off[k - C_DICT4];
  }
  std::vector<int32_t> dd_cols[2], dd_start[2];
  for (int g = 0; g < 2; g++) {  // C_DD, then C_DDG
    P->dd_chunk_off[g] = (uint32_t)chunk_list.size();
    for (int p : cls_lists[g ? C_DDG : C_DD]) {  // (sorted by column)
      PageWork& w = P->h_work[(size_t)p];
      if (dd_cols[g].empty() || dd_cols[g].back() != w.column) {  // dd_start: [begin, end) of each column's chunks
        if (!dd_cols[g].empty()) dd_start[g].push_back((int32_t)(chunk_list.size() - P->dd_chunk_off[g]));
        while ((chunk_list.size() - P->dd_chunk_off[g]) % (uint32_t)pqg::DICT_WPB) {  // whole workgroups per column
          chunk_list.push_back(0xFFFFFFFFull);
          chunk_total++;
        }
        dd_cols[g].push_back(w.column);
        dd_start[g].push_back((int32_t)(chunk_list.size() - P->dd_chunk_off[g]));
        const pqg_column_desc& cc = cols[w.column];
        if (!g)
          P->dd_region = std::max<uint32_t>(P->dd_region, (uint32_t)(((uint64_t)cc.dict_size + 15u) & ~15ull) +
                                                              4u * (uint32_t)cc.dict_num_values);
      }
      const uint32_t ch = pqg::dict_chunk_values(4);
      w.rec_base = rec_total;
      rec_total += (uint64_t)std::min<uint32_t>(w.num_slots, w.size) + 1;
      w.chunk_base = chunk_total;
      const uint32_t nch = (uint32_t)(((uint64_t)w.num_slots + 3u + ch - 1) / ch);
      for (uint32_t j = 0; j < nch; j++) chunk_list.push_back((uint64_t)(uint32_t)p | ((uint64_t)j << 32));
      chunk_total += nch;
    }
    if (!dd_cols[g].empty()) dd_start[g].push_back((int32_t)(chunk_list.size() - P->dd_chunk_off[g]));
    P->dd_chunk_n[g] = (uint32_t)chunk_list.size() - P->dd_chunk_off[g];
    P->n_dd_cols[g] = (int)dd_cols[g].size();
    if (P->dd_chunk_n[g]) P->dd_sums_off[g] = take(8 * (uint64_t)P->dd_chunk_n[g]);
  }
  // ---- flatten lists: [levels][class 0]...[class n]
  std::vector<int32_t> flat(lvl_list.begin(), lvl_list.end());
  P->levels_off = 0;
  P->levels_n = (int)lvl_list.size();
  P->cls_off.assign(C_NCLS, 0);
  P->cls_n.assign(C_NCLS, 0);
  for (int k = 0; k < C_NCLS; k++) {
    P->cls_off[(size_t)k] = (int)flat.size();
    P->cls_n[(size_t)k] = (int)cls_lists[(size_t)k].size();
    flat.insert(flat.end(), cls_lists[(size_t)k].begin(), cls_lists[(size_t)k].end());
  }
  std::vector<int32_t> cp, cps;
  cps.push_back(0);
  for (int i = 0; i < n_cols; i++) {
    if (col_pages[(size_t)i].empty()) continue;
    cp.insert(cp.end(), col_pages[(size_t)i].begin(), col_pages[(size_t)i].end());
    cps.push_back((int32_t)cp.size());
  }
  P->n_scan_cols = (int)cps.size() - 1;
  // bin_lists: [dictionary walks (columns)][BYTE_ARRAY dictionary pages][FLBA/INT96 dictionary pages][BYTE_ARRAY columns]
  std::vector<int32_t> bl;
  P->off_dict_walk = (int)bl.size(); P->n_dict_walk = (int)dict_walk.size(); bl.insert(bl.end(), dict_walk.begin(), dict_walk.end());
  P->off_bind = (int)bl.size(); P->n_bind = (int)bind.size(); bl.insert(bl.end(), bind.begin(), bind.end());
  P->off_fixd = (int)bl.size(); P->n_fixd = (int)fixd.size(); bl.insert(bl.end(), fixd.begin(), fixd.end());
  P->off_bin_cols = (int)bl.size(); P->n_bin_cols = (int)bin_cols.size(); bl.insert(bl.end(), bin_cols.begin(), bin_cols.end());
  P->off_carry = (int)bl.size(); P->n_carry = (int)carry_cols.size(); bl.insert(bl.end(), carry_cols.begin(), carry_cols.end());
  std::vector<uint64_t> dent_tiles;
  {  // large BYTE_ARRAY dictionaries: 2 KiB tiles of their pages, per column in dent_cols order
    std::vector<int32_t> dstart(1, 0);
    for (int i : dent_cols) {
      const uint32_t nt = (cols[i].dict_size + pqg::DENT_TILE - 1) / pqg::DENT_TILE;
      for (uint32_t t = 0; t < nt; t++) dent_tiles.push_back((uint64_t)(uint32_t)i | ((uint64_t)t << 32));
      dstart.push_back((int32_t)dent_tiles.size());
    }
    P->off_dent_cols = (int)bl.size(); P->n_dent_cols = (int)dent_cols.size(); bl.insert(bl.end(), dent_cols.begin(), dent_cols.end());
    P->off_dent_start = (int)bl.size(); bl.insert(bl.end(), dstart.begin(), dstart.end());
    P->n_dent_tiles = (uint32_t)dent_tiles.size();
    if (P->n_dent_tiles) {
      P->dent_rec_off = take(16ull * P->n_dent_tiles);
      P->dent_scr_off = take(2ull * pqg::DENT_CAP * P->n_dent_tiles);
      P->dent_tb_off = take(8ull * P->n_dent_tiles);
    }
  }
  for (int g = 0; g < 2; g++) {
    P->off_dd_cols[g] = (int)bl.size(); bl.insert(bl.end(), dd_cols[g].begin(), dd_cols[g].end());
    P->off_dd_start[g] = (int)bl.size(); bl.insert(bl.end(), dd_start[g].begin(), dd_start[g].end());
  }
  P->n_bin_blocks = (uint32_t)bin_blocks.size();
  P->n_bin_chunks = (uint32_t)bin_chunks.size();
  // ---- upload
  hipStream_t s = ctx->stream;
  bool ok = P->work.ensure(sizeof(PageWork) * P->h_work.size()) == hipSuccess &&
            P->cols.ensure(sizeof(ColumnDev) * hc.size()) == hipSuccess &&
            P->lists.ensure(sizeof(int32_t) * std::max<size_t>(flat.size(), 1)) == hipSuccess &&
            P->col_pages.ensure(sizeof(int32_t) * std::max<size_t>(cp.size(), 1)) == hipSuccess &&
            P->col_page_start.ensure(sizeof(int32_t) * cps.size()) == hipSuccess &&
            P->err.ensure(err_region_bytes(n_pages, n_cols) + 16) == hipSuccess &&
            P->bscratch.ensure(std::max<uint64_t>(sc, 256)) == hipSuccess &&
            P->bin_lists.ensure(sizeof(int32_t) * std::max<size_t>(bl.size(), 1)) == hipSuccess &&
            P->bin_blocks.ensure(sizeof(uint64_t) * std::max<size_t>(bin_blocks.size(), 1)) == hipSuccess &&
            P->bin_chunks.ensure(sizeof(uint64_t) * std::max<size_t>(bin_chunks.size(), 1)) == hipSuccess &&
            P->dba_chunks.ensure(sizeof(uint64_t) * std::max<size_t>(dba_chunks.size(), 1)) == hipSuccess &&
            P->segs.ensure(sizeof(uint64_t) * std::max<size_t>(segs.size(), 1)) == hipSuccess &&
            P->dent_tiles.ensure(sizeof(uint64_t) * std::max<size_t>(dent_tiles.size(), 1)) == hipSuccess &&
            P->psegs.ensure(sizeof(uint64_t) * std::max<size_t>(psegs.size(), 1)) == hipSuccess &&
            P->pstatus.ensure(2 * sizeof(uint64_t) * std::max<size_t>(psegs.size(), 1)) == hipSuccess &&
            P->pcol_pages.ensure(sizeof(int32_t) * std::max<size_t>(pcp.size(), 1)) == hipSuccess &&
            P->pcol_start.ensure(sizeof(int32_t) * pcs.size()) == hipSuccess &&

            P->rec.ensure(sizeof(uint64_t) * (rec_total + 2 * 64 + 16)) == hipSuccess &&  // the expansion prefetches a page's first 128
            P->chunk_run.ensure(sizeof(uint32_t) * std::max<uint32_t>(chunk_total, 1)) == hipSuccess &&
            P->chunks.ensure(sizeof(uint64_t) * std::max<size_t>(chunk_list.size(), 1)) == hipSuccess &&
            P->pstat.ensure(sizeof(uint64_t) * (size_t)std::max(n_pages, 1)) == hipSuccess &&
            P->flags.ensure(sizeof(uint32_t) * (size_t)std::max(n_pages, 1)) == hipSuccess;
  ok = ok && hipMemsetAsync(P->flags.p, 0, sizeof(uint32_t) * (size_t)std::max(n_pages, 1), s) == hipSuccess;
  {
    uint8_t* scb = (uint8_t*)P->bscratch.p;
    auto at = [&](uint64_t o) -> void* { return o == ~0ull ? nullptr : (void*)(scb + o); };
    for (int i = 0; i < n_cols; i++) {
      ColumnDev& d = hc[(size_t)i];
      d.blen = ids_mode(cols[i]) ? (uint32_t*)cols[i].values : (uint32_t*)at(blen_off[(size_t)i]);
      d.bsrc = (uint32_t*)at(bsrc_off[(size_t)i]);
      d.dict_len = (uint32_t*)at(dlen_off[(size_t)i]);
      d.dict_src = (uint32_t*)at(dsrc_off[(size_t)i]);
      d.dict_ent = (uint64_t*)at(dent_off[(size_t)i]);
      d.block_sums = (uint64_t*)at(bsum_off[(size_t)i]);
      d.bin_total = (uint64_t*)at(P->bin_total_off[(size_t)i]);
      d.n_slots = slot_acc[(size_t)i];
      d.dict_direct = dict_direct[(size_t)i] ? (cols[i].dict_num_values <= 256 && !dd_glob[(size_t)i] ? 1u : 2u) : 0u;  // id bytes
      d.dd_global = dd_glob[(size_t)i];
      if (dba_fixed[(size_t)i]) {  // DELTA_BYTE_ARRAY values go straight to the fixed-width output
        d.binary_data = (uint8_t*)cols[i].values;
        d.binary_capacity = slot_acc[(size_t)i] * (uint64_t)d.elem_width;
      }
    }
  }
  if (!bl.empty())
    ok = ok && hipMemcpyAsync(P->bin_lists.p, bl.data(), sizeof(int32_t) * bl.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!bin_blocks.empty())
    ok = ok && hipMemcpyAsync(P->bin_blocks.p, bin_blocks.data(), sizeof(uint64_t) * bin_blocks.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!bin_chunks.empty())
    ok = ok && hipMemcpyAsync(P->bin_chunks.p, bin_chunks.data(), sizeof(uint64_t) * bin_chunks.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!segs.empty())
    ok = ok && hipMemcpyAsync(P->segs.p, segs.data(), sizeof(uint64_t) * segs.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!dent_tiles.empty())
    ok = ok && hipMemcpyAsync(P->dent_tiles.p, dent_tiles.data(), sizeof(uint64_t) * dent_tiles.size(), hipMemcpyHostToDevice,
                              s) == hipSuccess;
  if (!psegs.empty()) {
    ok = ok && hipMemcpyAsync(P->psegs.p, psegs.data(), sizeof(uint64_t) * psegs.size(), hipMemcpyHostToDevice, s) == hipSuccess;
    ok = ok && hipMemsetAsync(P->pstatus.p, 0, 2 * sizeof(uint64_t) * psegs.size(), s) == hipSuccess;
  }
  if (!pcp.empty()) {
    ok = ok && hipMemcpyAsync(P->pcol_pages.p, pcp.data(), sizeof(int32_t) * pcp.size(), hipMemcpyHostToDevice, s) == hipSuccess;
    ok = ok && hipMemcpyAsync(P->pcol_start.p, pcs.data(), sizeof(int32_t) * pcs.size(), hipMemcpyHostToDevice, s) == hipSuccess;
    ok = ok && hipMemsetAsync((uint8_t*)P->bscratch.p + P->pflag_off, 0, 8, s) == hipSuccess;
  }
  if (P->null_hints) ok = ok && hipMemsetAsync((uint8_t*)P->bscratch.p + P->hint_off, 0, 8, s) == hipSuccess;
  P->n_psegs = (uint32_t)psegs.size();
  P->n_pcols = (int)pcs.size() - 1;
  P->plain_fused = !pcp.empty();
  P->n_pcp = (int)pcp.size();
  if (!dba_chunks.empty())
    ok = ok && hipMemcpyAsync(P->dba_chunks.p, dba_chunks.data(), sizeof(uint64_t) * dba_chunks.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!chunk_list.empty())
    ok = ok && hipMemcpyAsync(P->chunks.p, chunk_list.data(), sizeof(uint64_t) * chunk_list.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  ok = ok && hipMemcpyAsync(P->work.p, P->h_work.data(), sizeof(PageWork) * P->h_work.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  ok = ok && hipMemcpyAsync(P->cols.p, hc.data(), sizeof(ColumnDev) * hc.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!flat.empty()) ok = ok && hipMemcpyAsync(P->lists.p, flat.data(), sizeof(int32_t) * flat.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  if (!cp.empty()) ok = ok && hipMemcpyAsync(P->col_pages.p, cp.data(), sizeof(int32_t) * cp.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  ok = ok && hipMemcpyAsync(P->col_page_start.p, cps.data(), sizeof(int32_t) * cps.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  // the host vectors above die at return: wait for the copies
  ok = ok && hipStreamSynchronize(s) == hipSuccess;
  if (!ok) {
    set_status(st, PQG_ERR_HIP, -1, -1, "plan upload");
    pqg_plan_destroy(P);
    return PQG_ERR_HIP;
  }
  P->kernels = count_kernels(P);
  *out = P;
  return PQG_OK;
}

int pqg_plan_kernel_count(pqg_plan* P) { return P ? P->kernels : 0; }

int pqg_plan_timeout_fallbacks(pqg_plan* P) { return P ? P->timeout_fallbacks : 0; }

int pqg_plan_plain_fallbacks(pqg_plan* P) { return P ? P->plain_fallbacks : 0; }

int pqg_plan_null_hint_fallbacks(pqg_plan* P) { return P ? P->hint_fallbacks : 0; }

int pqg_plan_launch(pqg_plan* P) {
  if (!P) return PQG_ERR_INVALID_ARG;
  pqg_ctx* ctx = P->ctx;
  hipStream_t s = ctx->stream;
  uint64_t* err = (uint64_t*)P->err.p;
  // error words and the error counter share one allocation; both are tagged with the launch's
  // error epoch (pqg::ErrCount), so the region is zeroed only when the epoch wraps
  const size_t err_bytes = err_region_bytes(P->n_pages, P->n_cols);
  if (++P->err_epoch > pqg::ERR_EPOCH_MAX) {
    P->err_epoch = 1;
    if (hipMemsetAsync(P->err.p, 0, err_bytes + 16, s) != hipSuccess) return PQG_ERR_HIP;
    if (P->n_pcp && hipMemsetAsync((uint8_t*)P->bscratch.p + P->pflag_off, 0, 8, s) != hipSuccess) return PQG_ERR_HIP;
    if (P->null_hints && hipMemsetAsync((uint8_t*)P->bscratch.p + P->hint_off, 0, 8, s) != hipSuccess) return PQG_ERR_HIP;
  }
  const pqg::ErrCount ecount{(uint32_t*)((uint8_t*)P->err.p + err_bytes), P->err_epoch};
  PageWork* work = (PageWork*)P->work.p;
  const ColumnDev* cols = (const ColumnDev*)P->cols.p;
  const int32_t* lists = (const int32_t*)P->lists.p;
  const bool pf = P->plain_fused;
  const uint64_t clear = pf ? P->blen_bytes_nf : P->blen_bytes;
  if (clear && hipMemsetAsync(P->bscratch.p, 0, clear, s) != hipSuccess) return PQG_ERR_HIP;
  if (pf && ++P->pseg_epoch > 255u) {  // k_bin_plain tile words are tagged with 1..255
    P->pseg_epoch = 1;
    if (hipMemsetAsync(P->pstatus.p, 0, 2 * sizeof(uint64_t) * P->n_psegs, s) != hipSuccess) return PQG_ERR_HIP;
  }
  for (void* v : P->empty_bin_values)
    if (hipMemsetAsync(v, 0, sizeof(int64_t), s) != hipSuccess) return PQG_ERR_HIP;
  // page ready flags compare against the launch epoch (even); a walker's early partial status is
  // flagged epoch - 1. Reset on wrap.
  P->epoch += 2;
  if (P->epoch == 0) {
    P->epoch = 2;
    if (hipMemsetAsync(P->flags.p, 0, sizeof(uint32_t) * (size_t)std::max(P->n_pages, 1), s) != hipSuccess)
      return PQG_ERR_HIP;
  }
  hipError_t e = hipSuccess;
  // level-first order: k_levels + k_scan_offsets give the nullable pages' counts and offsets before any
  // value kernel; with V2 header null counts (null_hints) the host has them and k_levels only verifies
  // them, on the caller's stream beside the forked value kernels (launched after the fork below)
  const bool hints = P->null_hints && P->levels_n;
  const int32_t* bl = (const int32_t*)P->bin_lists.p;
  auto launch_dent = [&](hipStream_t st) -> hipError_t {  // large dictionaries' entries, per 2 KiB tile
    uint8_t* scb = (uint8_t*)P->bscratch.p;
    return pqg::launch_dict_entries(st, P->d_bytes, P->n_bytes, cols, (const uint64_t*)P->dent_tiles.p, P->n_dent_tiles,
                                    bl + P->off_dent_cols, bl + P->off_dent_start, P->n_dent_cols,
                                    (uint64_t*)(scb + P->dent_rec_off), (uint16_t*)(scb + P->dent_scr_off),
                                    (uint64_t*)(scb + P->dent_tb_off), P->n_pages, err, ecount);
  };
  // every large dictionary's column dictionary-direct with HBM entries (C_DDG only): its tile walk runs
  // on a queue of its own from the start, beside the levels and the id walk (k_dict_fused_dd<DD_IDS>)
  bool dent_fork = false;
  if (e == hipSuccess && P->n_dent_tiles && P->cls_n[C_DDG] && !P->cls_n[C_DD] && !P->cls_n[C_IDS] && !P->n_bind) {
    dent_fork = (ctx->dent_stream || hipStreamCreateWithFlags(&ctx->dent_stream, hipStreamNonBlocking) == hipSuccess) &&
                (ctx->ev_dent_fork || hipEventCreateWithFlags(&ctx->ev_dent_fork, hipEventDisableTiming) == hipSuccess) &&
                (ctx->ev_dent || hipEventCreateWithFlags(&ctx->ev_dent, hipEventDisableTiming) == hipSuccess) &&
                hipEventRecord(ctx->ev_dent_fork, s) == hipSuccess &&
                hipStreamWaitEvent(ctx->dent_stream, ctx->ev_dent_fork, 0) == hipSuccess;
    if (dent_fork) {
      e = launch_dent(ctx->dent_stream);
      if (e == hipSuccess && hipEventRecord(ctx->ev_dent, ctx->dent_stream) != hipSuccess) e = hipErrorUnknown;
    }
  }
  auto launch_dict_walks = [&](hipStream_t st) -> hipError_t {
    hipError_t r = hipSuccess;
    if (P->n_dict_walk)  // BYTE_ARRAY dictionary entries (PlainBinaryDictionary ctor)
      r = pqg::launch_bin_walk(st, P->d_bytes, P->n_bytes, work, cols, bl + P->off_dict_walk, P->n_dict_walk, 1,
                               P->n_pages, err, ecount);
    if (r == hipSuccess && P->n_dent_tiles && !dent_fork) r = launch_dent(st);
    return r;
  };
  if (e == hipSuccess && P->levels_n && !hints) {
    e = pqg::launch_levels(s, P->d_bytes, P->n_bytes, work, cols, lists + P->levels_off, P->levels_n, err, ecount, nullptr);
    if (e == hipSuccess)
      e = pqg::launch_scan(s, work, (const int32_t*)P->col_pages.p, (const int32_t*)P->col_page_start.p, P->n_scan_cols);
  }
  // The one-pass PLAIN BYTE_ARRAY kernel is latency / issue bound (~1 TB/s) and independent of the other
  // columns' kernels (most of them HBM bound): with other pages in the plan it runs on a second queue,
  // forked after the levels and joined at the end, so the two kinds share the chip.
  // The BYTE_ARRAY kernels of the other columns likewise go to a third queue when fixed-width columns'
  // kernels (HBM bound) are in the plan to share the chip with.
  bool fork = false, fork_bin = false, fork_fix = false;
  const bool has_fixed = P->cls_n[C_DICT4] || P->cls_n[C_DICT8] || P->cls_n[C_PLAIN] || P->cls_n[C_BOOL] ||
                         P->cls_n[C_RLEBOOL] || P->cls_n[C_DELTA4] || P->cls_n[C_DELTA8] || P->cls_n[C_BSS];
  const bool has_bin = P->n_dict_walk || P->n_dent_tiles || P->cls_n[C_IDS] || P->cls_n[C_DD] || P->cls_n[C_DDG] || P->cls_n[C_BINP] - P->n_binp_seg - (pf ? P->n_binp_fused : 0) > 0 ||
                       P->cls_n[C_DLBA] || P->cls_n[C_DBA] || P->n_segs;
  const bool want = e == hipSuccess && ((pf && (has_fixed || has_bin)) || (has_bin && has_fixed) ||
                                        (hints && (pf || has_bin || has_fixed)));
  const bool ev_ok = want && (ctx->ev_fork || hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) == hipSuccess) &&
                     hipEventRecord(ctx->ev_fork, s) == hipSuccess;
  if (ev_ok && pf) {
    fork = (ctx->side_stream || hipStreamCreateWithFlags(&ctx->side_stream, hipStreamNonBlocking) == hipSuccess) &&
           (ctx->ev_join || hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming) == hipSuccess) &&
           hipStreamWaitEvent(ctx->side_stream, ctx->ev_fork, 0) == hipSuccess;
  }
  if (ev_ok && has_bin && (has_fixed || hints)) {
    fork_bin = (ctx->bin_stream || hipStreamCreateWithFlags(&ctx->bin_stream, hipStreamNonBlocking) == hipSuccess) &&
               (ctx->ev_join_bin || hipEventCreateWithFlags(&ctx->ev_join_bin, hipEventDisableTiming) == hipSuccess) &&
               hipStreamWaitEvent(ctx->bin_stream, ctx->ev_fork, 0) == hipSuccess;
  }
  if (ev_ok && (fork || fork_bin || hints) && has_fixed)
    fork_fix = (ctx->fix_stream || hipStreamCreateWithFlags(&ctx->fix_stream, hipStreamNonBlocking) == hipSuccess) &&
               (ctx->ev_join_fix || hipEventCreateWithFlags(&ctx->ev_join_fix, hipEventDisableTiming) == hipSuccess) &&
               hipStreamWaitEvent(ctx->fix_stream, ctx->ev_fork, 0) == hipSuccess;
  if (e == hipSuccess && hints)  // the level sections, verified against the header counts, beside the value kernels
    e = pqg::launch_levels(s, P->d_bytes, P->n_bytes, work, cols, lists + P->levels_off, P->levels_n, err, ecount,
                           (uint32_t*)((uint8_t*)P->bscratch.p + P->hint_off));
  if (e == hipSuccess && pf) {  // PLAIN-only BYTE_ARRAY columns: one pass (after the levels: n_values, out_offset)
    uint8_t* scb = (uint8_t*)P->bscratch.p;
    uint64_t* ps = (uint64_t*)P->pstatus.p;
    e = pqg::launch_bin_plain(fork ? ctx->side_stream : s, P->d_bytes, P->n_bytes, work, cols, (const int32_t*)P->pcol_pages.p,
                              (const int32_t*)P->pcol_start.p, P->n_pcols, (const uint64_t*)P->psegs.p, P->n_psegs, ps,
                              ps + P->n_psegs, (uint32_t*)(scb + P->pticket_off), P->pseg_epoch,
                              (uint32_t*)(scb + P->pflag_off), P->err_epoch, err, ecount, P->plain_pg, P->n_pcp);
    if (fork && hipEventRecord(ctx->ev_join, ctx->side_stream) != hipSuccess) e = hipErrorUnknown;
  }
  const hipStream_t sb = fork_bin ? ctx->bin_stream : s;  // BYTE_ARRAY kernels of the other columns
  const hipStream_t sf = fork_fix ? ctx->fix_stream : s;  // fixed-width columns
  if (e == hipSuccess) e = launch_dict_walks(sb);
  for (int k = 0; k < C_NCLS && e == hipSuccess; k++) {
    int n = P->cls_n[(size_t)k] - (k == C_BINP ? P->n_binp_seg + (pf ? P->n_binp_fused : 0) : 0);
    if (!n) continue;
    const int32_t* l = lists + P->cls_off[(size_t)k];
    switch (k) {
      case C_DICT4:
      case C_DICT8: {
        const int i = k - C_DICT4;
        e = pqg::launch_dict(k == C_DICT8 ? 8 : 4, sf, P->d_bytes, P->n_bytes, work, cols, l, n, (uint64_t*)P->rec.p,
                             (uint32_t*)P->chunk_run.p, (const uint64_t*)P->chunks.p + P->chunk_off[i], P->chunk_n[i],
                             (uint64_t*)P->pstat.p, (uint32_t*)P->flags.p, P->epoch, P->dict_fused, err, ecount);
        break;
      }
      case C_IDS: {
        const int i = k - C_DICT4;
        e = pqg::launch_dict_ids(sb, P->d_bytes, P->n_bytes, work, cols, l, n, (uint64_t*)P->rec.p,
                                 (uint32_t*)P->chunk_run.p, (const uint64_t*)P->chunks.p + P->chunk_off[i],
                                 P->chunk_n[i], (uint64_t*)P->pstat.p, (uint32_t*)P->flags.p, P->epoch, P->dict_fused, err, ecount);
        break;
      }
      case C_DD:
      case C_DDG: {
        const int g = k == C_DDG ? 1 : 0;
        e = pqg::launch_dict_dd(sb, P->d_bytes, P->n_bytes, work, cols, l, n, (uint64_t*)P->rec.p,
                                (uint32_t*)P->chunk_run.p, (const uint64_t*)P->chunks.p + P->dd_chunk_off[g],
                                P->dd_chunk_n[g], (uint64_t*)P->pstat.p, (uint32_t*)P->flags.p, P->epoch, P->dict_fused,
                                err, ecount, (uint64_t*)((uint8_t*)P->bscratch.p + P->dd_sums_off[g]),
                                bl + P->off_dd_cols[g], bl + P->off_dd_start[g], P->n_dd_cols[g], P->dd_region, g == 1,
                                g == 1 && dent_fork ? ctx->ev_dent : nullptr);
        break;
      }
      case C_BSS: e = pqg::launch_bss(sf, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
      case C_BINP:
        e = pqg::launch_bin_walk(sb, P->d_bytes, P->n_bytes, work, cols, l, n, 0, P->n_pages, err, ecount);
        break;
      case C_DLBA: e = pqg::launch_dlba_lengths(sb, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
      case C_DBA:
        e = pqg::launch_dba_lengths(sb, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount, P->dba_meta());
        break;
      case C_PLAIN: e = pqg::launch_plain(0, sf, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
      case C_BOOL: e = pqg::launch_plain(1, sf, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
      case C_RLEBOOL: e = pqg::launch_plain(2, sf, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
      case C_DELTA4: e = pqg::launch_delta(4, sf, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
      case C_DELTA8: e = pqg::launch_delta(8, sf, P->d_bytes, P->n_bytes, work, cols, l, n, err, ecount); break;
    }
  }
  if (e == hipSuccess && P->n_segs && !P->seg_walk)  // the segmented pages one wave each (after a timeout)
    e = pqg::launch_bin_walk(sb, P->d_bytes, P->n_bytes, work, cols,
                             lists + P->cls_off[C_BINP] + (P->cls_n[C_BINP] - P->n_binp_seg), P->n_binp_seg, 0,
                             P->n_pages, err, ecount);
  if (e == hipSuccess && P->n_segs && P->seg_walk) {  // PLAIN BYTE_ARRAY pages in segments (status + ticket cleared above)
    uint8_t* scb = (uint8_t*)P->bscratch.p;
    e = pqg::launch_bin_walk_seg(sb, P->d_bytes, P->n_bytes, work, cols, (const uint64_t*)P->segs.p, P->n_segs,
                                 (uint64_t*)(scb + P->seg_status_off), (uint32_t*)(scb + P->seg_status_off) + 2u * P->n_segs,
                                 (uint32_t*)(scb + P->seg_tmp_off), err, ecount);
  }
  // post-passes: dictionary ids -> BYTE_ARRAY entries / fixed-width entries; offsets; value bytes
  if (e == hipSuccess && P->n_bind) e = pqg::launch_bin_dict_map(sb, work, cols, bl + P->off_bind, P->n_bind);
  if (e == hipSuccess && P->n_fixd)
    e = pqg::launch_gather_fixed(sb, P->d_bytes, P->n_bytes, work, cols, bl + P->off_fixd, P->n_fixd);
  const uint32_t n_blocks = pf ? P->n_bin_blocks_nf : P->n_bin_blocks;
  if (e == hipSuccess && n_blocks)
    e = pqg::launch_bin_scan(sb, P->d_bytes, P->n_bytes, cols, bl + P->off_bin_cols, pf ? P->n_bin_cols_nf : P->n_bin_cols,
                             (const uint64_t*)P->bin_blocks.p, n_blocks);
  const uint32_t n_chunks = pf ? P->n_bin_chunks_nf : P->n_bin_chunks;
  if (e == hipSuccess && n_chunks)
    e = pqg::launch_bin_copy(sb, P->d_bytes, P->n_bytes, work, cols, (const uint64_t*)P->bin_chunks.p, n_chunks, err,
                             ecount);
  if (e == hipSuccess && P->cls_n[C_DBA])
    e = pqg::launch_dba_copy(sb, P->d_bytes, P->n_bytes, work, cols, lists + P->cls_off[C_DBA], P->cls_n[C_DBA],
                             (const uint64_t*)P->dba_chunks.p, P->n_dba_chunks, P->dba_meta(), bl + P->off_carry,
                             P->n_carry, err, ecount);
  if (fork && hipStreamWaitEvent(s, ctx->ev_join, 0) != hipSuccess) e = hipErrorUnknown;
  if (fork_bin && (hipEventRecord(ctx->ev_join_bin, ctx->bin_stream) != hipSuccess ||
                   hipStreamWaitEvent(s, ctx->ev_join_bin, 0) != hipSuccess))
    e = hipErrorUnknown;
  if (fork_fix && (hipEventRecord(ctx->ev_join_fix, ctx->fix_stream) != hipSuccess ||
                   hipStreamWaitEvent(s, ctx->ev_join_fix, 0) != hipSuccess))
    e = hipErrorUnknown;
  ctx->last_launched = P;
  if (std::find(ctx->unsynced.begin(), ctx->unsynced.end(), P) == ctx->unsynced.end()) ctx->unsynced.push_back(P);
  return e == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

int pqg_plan_destroy(pqg_plan* P) {
  if (!P) return PQG_OK;
  if (P->ctx) {
    (void)hipStreamSynchronize(P->ctx->stream);
    if (P->ctx->last_launched == P) P->ctx->last_launched = nullptr;
    if (P->ctx->last == P) P->ctx->last = nullptr;
    auto& u = P->ctx->unsynced;
    u.erase(std::remove(u.begin(), u.end(), P), u.end());
  }
  P->work.release();
  P->cols.release();
  P->lists.release();
  P->col_pages.release();
  P->col_page_start.release();
  P->err.release();
  P->rec.release();
  P->chunk_run.release();
  P->psegs.release();
  P->pstatus.release();
  P->pcol_pages.release();
  P->pcol_start.release();
  P->chunks.release();
  P->pstat.release();
  P->flags.release();
  P->bscratch.release();
  P->bin_lists.release();
  P->bin_blocks.release();
  P->bin_chunks.release();
  P->dba_chunks.release();
  P->segs.release();
  P->dent_tiles.release();
  delete P;
  return PQG_OK;
}

}  // extern "C"

namespace {

int resolve_page_errors(pqg_plan* P, pqg_status* st, const std::vector<uint64_t>& errs);

// Resolve the first error of a launched plan in (page, value) order.
// Per page: init errors (rl init < dl init < data init) first; then value errors
// (values are decoded only for slots before a level error, so a value error is
// always earlier in the reference's read order); then level errors.
int resolve_errors(pqg_plan* P, pqg_status* st, std::vector<PageWork>* work_out) {
  pqg_ctx* ctx = P->ctx;
  hipStream_t s = ctx->stream;
  if (ctx->pin_err.ensure(16) != hipSuccess) return PQG_ERR_HIP;
  uint32_t* cnt = (uint32_t*)ctx->pin_err.p;
  if (hipMemcpyAsync(cnt, (uint8_t*)P->err.p + err_region_bytes(P->n_pages, P->n_cols), sizeof(uint32_t),
                     hipMemcpyDeviceToHost, s) != hipSuccess)
    return PQG_ERR_HIP;
  bool need_work = false;
  for (auto v : P->col_nullable) need_work = need_work || v;
  if (need_work && work_out) {
    work_out->resize(P->h_work.size());
    if (hipMemcpyAsync(work_out->data(), P->work.p, sizeof(PageWork) * P->h_work.size(), hipMemcpyDeviceToHost, s) != hipSuccess)
      return PQG_ERR_HIP;
  }
  if (hipStreamSynchronize(s) != hipSuccess) return PQG_ERR_HIP;
  std::vector<uint64_t> errs;
  if (*cnt == P->err_epoch) {  // a kernel of the last launch reported (see pqg::ErrCount)
    errs.resize(3 * (size_t)(P->n_pages + std::max(P->n_cols, 1)));
    if (hipMemcpy(errs.data(), P->err.p, sizeof(uint64_t) * errs.size(), hipMemcpyDeviceToHost) != hipSuccess) return PQG_ERR_HIP;
    for (uint64_t& w : errs)  // words of earlier launches are stale: no error in this one
      w = (w >> 48) == P->err_epoch ? (~w & pqg::ERR_KEY_MASK) : ~0ull;
  }
  int rc = resolve_page_errors(P, st, errs);
  if (rc) return rc;
  // BYTE_ARRAY output capacity (API misuse, after the decode errors: values past a decode error
  // are not meaningful and may inflate the byte count)
  for (int i = 0; i < P->n_cols; i++) {
    if (P->bin_total_off[(size_t)i] == ~0ull) continue;
    uint64_t total = 0;
    if (hipMemcpy(&total, (uint8_t*)P->bscratch.p + P->bin_total_off[(size_t)i], sizeof(total), hipMemcpyDeviceToHost) !=
        hipSuccess)
      return PQG_ERR_HIP;
    if (total > P->bin_capacity[(size_t)i]) {
      if (st) {
        st->code = PQG_ERR_INVALID_ARG;
        st->page = -1;
        st->value_index = (int64_t)total;
        std::snprintf(st->message, sizeof(st->message),
                      "binary capacity: column %d needs %llu bytes of binary_data (capacity %llu)", i,
                      (unsigned long long)total, (unsigned long long)P->bin_capacity[(size_t)i]);
      }
      return PQG_ERR_INVALID_ARG;
    }
  }
  return PQG_OK;
}

int resolve_page_errors(pqg_plan* P, pqg_status* st, const std::vector<uint64_t>& errs) {
  // every page's own first error (pqg_page_errors), then the batch's first in page order (st)
  P->page_errs.assign((size_t)P->n_pages, pqg_page_error{PQG_OK, PQG_PHASE_NONE, -1});
  if (P->host_errs.empty() && errs.empty()) return PQG_OK;
  std::vector<const HostErr*> herr((size_t)std::max(P->n_pages, 1), nullptr);
  for (const HostErr& h : P->host_errs)
    if (!herr[(size_t)h.page]) herr[(size_t)h.page] = &h;
  int first = -1;
  for (int p = 0; p < P->n_pages; p++) {
    pqg_page_error& pe = P->page_errs[(size_t)p];
    const HostErr* h = herr[(size_t)p];
    // device-detected dictionary page errors (BYTE_ARRAY dictionary walk, pseudo page n_pages + column):
    // the ColumnReaderBase ctor reads the dictionary before the column's first page
    const int col = P->h_work[(size_t)p].column;
    const uint64_t d = (!errs.empty() && col >= 0 && col < P->n_cols && P->col_first_page[(size_t)col] == p)
                           ? errs[3 * (size_t)(P->n_pages + col)] : ~0ull;
    uint64_t init = errs.empty() ? ~0ull : errs[3 * (size_t)p];
    uint64_t lvl = errs.empty() ? ~0ull : errs[3 * (size_t)p + 1];
    uint64_t val = errs.empty() ? ~0ull : errs[3 * (size_t)p + 2];
    if (d != ~0ull) {
      pe = {(int32_t)(d & 0xFF), PQG_PHASE_DICTIONARY, -1};
    } else if (h && h->index == -1) {  // host-detected dictionary page error: before any page is read
      pe = {h->code, PQG_PHASE_DICTIONARY, -1};
    } else if (h || init != ~0ull) {   // init-phase errors: key = phase (0 rl, 1 dl, 2 data) << 8 | code
      const uint64_t hkey = h ? (((uint64_t)h->index << 8) | (uint64_t)h->code) : ~0ull;
      const uint64_t k = std::min(hkey, init);
      const int ph = (int)(k >> 8);
      pe = {(int32_t)(k & 0xFF), ph == 0 ? PQG_PHASE_RL_INIT : ph == 1 ? PQG_PHASE_DL_INIT : PQG_PHASE_DATA_INIT, -1};
    } else if (val != ~0ull) {
      // values are decoded only for slots before a level error: a value error comes first
      pe = {(int32_t)(val & 0xFF), PQG_PHASE_VALUE, (int64_t)(val >> 8)};
    } else if (lvl != ~0ull) {         // key = (slot << 1 | 0 rl / 1 dl) << 8 | code
      pe = {(int32_t)(lvl & 0xFF), ((lvl >> 8) & 1) ? PQG_PHASE_DL_READ : PQG_PHASE_RL_READ, (int64_t)(lvl >> 9)};
    }
    if (pe.code != PQG_OK && first < 0) first = p;
  }
  if (first < 0) return PQG_OK;
  const pqg_page_error& pe = P->page_errs[(size_t)first];
  switch (pe.phase) {
    case PQG_PHASE_DICTIONARY: set_status(st, pe.code, first, -1, "dictionary page"); break;
    case PQG_PHASE_DATA_INIT: set_status(st, pe.code, first, 0, "data init"); break;
    case PQG_PHASE_RL_INIT: case PQG_PHASE_DL_INIT: set_status(st, pe.code, first, 0, "level init"); break;
    case PQG_PHASE_VALUE: set_status(st, pe.code, first, pe.index, "value decode"); break;
    default: set_status(st, pe.code, first, pe.index, "level decode"); break;
  }
  return pe.code;
}

}  // namespace

namespace {

// pqg_sync for one launched plan: the PLAIN one-pass re-run, error resolution, the fused-kernel
// timeout re-run. `work` receives the plan's PageWork (nullable columns' value counts).
int sync_plan(pqg_plan* P, pqg_status* st, std::vector<PageWork>* work) {
  pqg_ctx* ctx = P->ctx;
  if (P->null_hints && P->levels_n) {
    // A V2 header null count that disagrees with the page's definition levels (or a level error on such
    // a page): the value kernels ran on wrong counts / offsets. The reference decodes by the levels
    // (ColumnReaderBase.java:650-676, 760-771), so the launch is re-run level-first, which rewrites every
    // output; the plan keeps that order.
    uint32_t flag = 0;
    if (hipMemcpy(&flag, (uint8_t*)P->bscratch.p + P->hint_off, sizeof(flag), hipMemcpyDeviceToHost) != hipSuccess)
      return PQG_ERR_HIP;
    if (flag == P->err_epoch) {
      P->null_hints = false;
      P->kernels = count_kernels(P);
      P->hint_fallbacks++;
      const int lrc = pqg_plan_launch(P);
      if (lrc != PQG_OK) return lrc;
      if (P->d_counts &&  // pqg_decode's per-page counts, copied after the first launch
          hipMemcpy2DAsync(P->d_counts, sizeof(uint32_t), (const uint8_t*)P->work.p + offsetof(PageWork, n_values),
                           sizeof(PageWork), sizeof(uint32_t), (size_t)P->n_pages, hipMemcpyDeviceToDevice,
                           ctx->stream) != hipSuccess)
        return PQG_ERR_HIP;
      if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
    }
  }
  if (P->plain_fused) {
    // A PLAIN page whose values do not end at its section end (bytes the reader ignores after them)
    // breaks the one-pass path's byte bases: the launch is re-run on the per-value path (k_bin_walk,
    // offset scan, k_bin_copy), which reads exactly n_values values per page; the plan keeps that path.
    uint32_t flag = 0;
    if (hipMemcpy(&flag, (uint8_t*)P->bscratch.p + P->pflag_off, sizeof(flag), hipMemcpyDeviceToHost) != hipSuccess)
      return PQG_ERR_HIP;
    if (flag == P->err_epoch) {
      P->plain_fused = false;
      P->kernels = count_kernels(P);
      P->plain_fallbacks++;
      const int lrc = pqg_plan_launch(P);
      if (lrc != PQG_OK) return lrc;
      if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
    }
  }
  int rc = resolve_errors(P, st, work);
  // only a timeout of the fused dictionary kernel's hand-off is re-run in split mode (a PLAIN
  // BYTE_ARRAY segment walk that timed out waiting for its predecessor reaches the caller)
  const int tpage = st ? (int)st->page : -1;
  const int tcls = tpage >= 0 && tpage < P->n_pages ? P->page_cls[(size_t)tpage] : -1;
  if (rc == PQG_ERR_TIMEOUT && P->dict_fused && (tcls == C_DICT4 || tcls == C_DICT8 || tcls == C_IDS || tcls == C_DD || tcls == C_DDG)) {
    // The fused dictionary kernel's hand-off relies on the walker workgroups being dispatched before
    // the expansion workgroups that wait for them, which HIP does not promise. A launch in which an
    // expansion waited past SPIN_TIMEOUT_TICKS (it then stops and reports PQG_ERR_TIMEOUT; the walkers
    // still finish, so the grid drains) is re-run with the walk and the expansion as two launches,
    // which have no inter-workgroup waits; the plan keeps that mode. Every output of the re-run is
    // written again, so the result is the same bit for bit.
    P->dict_fused = false;
    P->kernels = count_kernels(P);
    P->timeout_fallbacks++;
    rc = pqg_plan_launch(P);
    if (rc == PQG_OK) {
      if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
      work->clear();
      rc = resolve_errors(P, st, work);
    }
  }
  // likewise a segment of a segmented PLAIN BYTE_ARRAY page that waited past its bound for its
  // predecessor's publication (k_bin_walk_seg; the predecessor always holds an earlier ticket, so this
  // needs a starved wave): the plan re-runs with those pages one wave each and keeps that mode
  const int tpage2 = st ? (int)st->page : -1;
  const int tcls2 = tpage2 >= 0 && tpage2 < P->n_pages ? P->page_cls[(size_t)tpage2] : -1;
  if (rc == PQG_ERR_TIMEOUT && P->n_segs && P->seg_walk && tcls2 == C_BINP) {
    P->seg_walk = false;
    P->kernels = count_kernels(P);
    P->timeout_fallbacks++;
    rc = pqg_plan_launch(P);
    if (rc == PQG_OK) {
      if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
      work->clear();
      rc = resolve_errors(P, st, work);
    }
  }
  return rc;
}

}  // namespace

extern "C" {

int pqg_sync(pqg_ctx* ctx, pqg_status* st) {
  if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
  if (!ctx) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
    set_status(st, PQG_ERR_HIP, -1, -1, hipGetErrorString(hipGetLastError()));
    return PQG_ERR_HIP;
  }
  // every plan launched since the last sync, in launch order (re-runs inside sync_plan append the
  // plan again; the list is taken first and cleared at the end)
  std::vector<pqg_plan*> plans;
  plans.swap(ctx->unsynced);
  int rc = PQG_OK;
  for (pqg_plan* P : plans) {
    // sync_plan can return PQG_ERR_HIP before anything sets the status: start from "no error"
    pqg_status pst;
    std::memset(&pst, 0, sizeof(pst));
    pst.page = -1;
    std::vector<PageWork> work;
    const int prc = sync_plan(P, &pst, &work);
    if (prc != PQG_OK && pst.code == 0 && pst.message[0] == '\0')
      set_status(&pst, prc, -1, -1, prc == PQG_ERR_HIP ? hipGetErrorString(hipGetLastError()) : "plan sync failed");
    if (prc != PQG_OK && rc == PQG_OK) {
      rc = prc;
      if (st) *st = pst;
    }
    if (prc == PQG_ERR_HIP) break;
    if (ctx->last_cols && P == ctx->last) {
      for (int i = 0; i < P->n_cols; i++) {
        uint64_t n = P->col_required_values[(size_t)i];
        if (P->col_nullable[(size_t)i] && !work.empty()) {
          n = 0;
          for (int p = 0; p < P->n_pages; p++)
            if (work[(size_t)p].column == i) n += work[(size_t)p].n_values;
        }
        ctx->last_cols[i].values_written = n;
      }
    }
  }
  ctx->unsynced.clear();
  return rc;
}

int pqg_plan_page_errors(pqg_plan* P, pqg_page_error* out, int n_pages) {
  if (!P || n_pages != P->n_pages || (n_pages && !out)) return PQG_ERR_INVALID_ARG;
  for (int p = 0; p < n_pages; p++)
    out[p] = (size_t)p < P->page_errs.size() ? P->page_errs[(size_t)p] : pqg_page_error{PQG_OK, PQG_PHASE_NONE, -1};
  return PQG_OK;
}

int pqg_page_errors(pqg_ctx* ctx, pqg_page_error* out, int n_pages) {
  if (!ctx || !ctx->last) return PQG_ERR_INVALID_ARG;
  return pqg_plan_page_errors(ctx->last, out, n_pages);
}

int pqg_plan_create(pqg_ctx* ctx, const uint8_t* d_bytes, uint64_t n_bytes, const pqg_column_desc* cols, int n_cols,
                    const pqg_page_desc* pages, int n_pages, pqg_plan** out, pqg_status* st) {
  return plan_create_impl(ctx, d_bytes, n_bytes, n_bytes, cols, n_cols, pages, n_pages, out, st);
}

static int decode_impl(pqg_ctx* ctx, const uint8_t* d_bytes, uint64_t n_bytes, uint64_t valid_bytes,
                       pqg_column_desc* cols, int n_cols, const pqg_page_desc* pages, int n_pages,
                       uint32_t* d_page_value_counts, pqg_status* st) {
  if (!ctx || n_cols < 0 || n_pages < 0 || (n_cols && !cols) || (n_pages && !pages)) return PQG_ERR_INVALID_ARG;
  // capacity checks (descriptor arithmetic)
  {
    std::vector<uint64_t> slots((size_t)std::max(n_cols, 1), 0);
    for (int p = 0; p < n_pages; p++)
      if (pages[p].column >= 0 && pages[p].column < n_cols) slots[(size_t)pages[p].column] += pages[p].num_values;
    for (int i = 0; i < n_cols; i++) {
      bool lv = cols[i].max_def > 0 || cols[i].max_rep > 0;
      const uint64_t need = slots[(size_t)i] + (bin_out(cols[i]) ? 1 : 0);  // offsets[n + 1]
      if (need > cols[i].values_capacity || (need && !cols[i].values) ||
          (lv && ((cols[i].max_def > 0 && cols[i].def_levels) || (cols[i].max_rep > 0 && cols[i].rep_levels)) &&
           slots[(size_t)i] > cols[i].levels_capacity)) {
        set_status(st, PQG_ERR_INVALID_ARG, -1, i, "output capacity");
        return PQG_ERR_INVALID_ARG;
      }
    }
  }
  if (ctx->last) {
    pqg_plan_destroy(ctx->last);
    ctx->last = nullptr;
  }
  pqg_plan* P = nullptr;
  int rc = plan_create_impl(ctx, d_bytes, n_bytes, valid_bytes, cols, n_cols, pages, n_pages, &P, st);
  if (rc) return rc;
  ctx->last = P;
  ctx->last_cols = cols;
  rc = pqg_plan_launch(P);
  P->d_counts = n_pages > 0 ? d_page_value_counts : nullptr;
  if (rc == PQG_OK && d_page_value_counts && n_pages > 0) {
    // n_values of every page (strided in PageWork) -> dense uint32 array
    rc = hipMemcpy2DAsync(d_page_value_counts, sizeof(uint32_t), (const uint8_t*)P->work.p + offsetof(PageWork, n_values),
                          sizeof(PageWork), sizeof(uint32_t), (size_t)n_pages, hipMemcpyDeviceToDevice,
                          ctx->stream) == hipSuccess
             ? PQG_OK
             : PQG_ERR_HIP;
  }
  return rc;
}

int pqg_decode(pqg_ctx* ctx, const uint8_t* d_bytes, uint64_t n_bytes, pqg_column_desc* cols, int n_cols,
               const pqg_page_desc* pages, int n_pages, uint32_t* d_page_value_counts, pqg_status* st) {
  return decode_impl(ctx, d_bytes, n_bytes, n_bytes, cols, n_cols, pages, n_pages, d_page_value_counts, st);
}

// ---- host copies of the host path (pinned staging <-> caller arrays): one thread moves ~10 GB/s,
// so large copies are spread over up to 8 threads, and the D2H of the outputs is issued in chunks
// whose copies out of pinned memory start as each chunk lands.
namespace {
struct HostCopy {
  uint8_t* dst;
  uint64_t src;  // offset in the pinned buffer
  uint64_t len;
};
// D2H piece: each is copied out by one thread as soon as it lands, so the copy of the last piece is the
// tail after the link (32 MiB pieces: d2h+copy 21-24 ms for 800 MB against 14 ms of link, r05u)
constexpr uint64_t HOST_CHUNK = 8ull << 20;
inline int host_threads(uint64_t bytes) {
  const unsigned hw = std::thread::hardware_concurrency();
  const uint64_t want = bytes / (8ull << 20) + 1;
  // (16 threads measured 38.4 vs 36.9 GB/s for 8 on an 800 MB output: host memory bound, profiles/r05/e2e)
  return (int)std::min<uint64_t>({want, 8ull, hw ? (uint64_t)hw : 1ull});
}
// the parts of `jobs` inside [lo, hi) of the pinned buffer `base`
void copy_range(const std::vector<HostCopy>& jobs, const uint8_t* base, uint64_t lo, uint64_t hi) {
  for (const HostCopy& j : jobs) {
    const uint64_t a = std::max(lo, j.src), b = std::min(hi, j.src + j.len);
    if (a < b) std::memcpy(j.dst + (a - j.src), base + a, b - a);
  }
}
void par_memcpy(void* dst, const void* src, uint64_t n) {
  const int t = host_threads(n);
  if (t <= 1) { std::memcpy(dst, src, n); return; }
  std::vector<std::thread> th;
  const uint64_t per = (n / (uint64_t)t + 4095) & ~4095ull;
  for (int k = 0; k < t; k++) {
    const uint64_t a = std::min(n, per * (uint64_t)k), b = std::min(n, a + per);
    if (a < b) th.emplace_back([=] { std::memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, b - a); });
  }
  for (auto& x : th) x.join();
}
}  // namespace

// The host path. h_bytes == nullptr: staged (pqg_decode_staged) — the bytes are already in ctx->pin_in,
// the outputs stay in ctx->pin_out and ctx->staged describes them; otherwise the caller's arrays.
static int host_path(pqg_ctx* ctx, const uint8_t* h_bytes, uint64_t n_bytes, pqg_column_desc* cols, int n_cols,
                     const pqg_page_desc* pages, int n_pages, uint32_t* h_page_value_counts, pqg_status* st) {
  if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
  const bool staged = h_bytes == nullptr;
  if (!ctx || n_cols < 0 || n_pages < 0 || (n_cols && !cols) || (n_pages && !pages)) return PQG_ERR_INVALID_ARG;
  if (staged && ctx->pin_in.cap < n_bytes + 1024) return PQG_ERR_INVALID_ARG;  // pqg_host_input first
  ctx->staged.clear();
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  hipStream_t s = ctx->stream;
  // PQG_HOST_TIMING=1: phase times of this call on stderr (diagnostics)
  static const bool timing = std::getenv("PQG_HOST_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    if (!timing) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "pqg_decode_host %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t_last).count());
    t_last = now;
  };
  const uint64_t pad = 1024;
  const size_t nc = (size_t)std::max(n_cols, 1);
  std::vector<uint64_t> slots(nc, 0), page_bytes(nc, 0);
  for (int p = 0; p < n_pages; p++)
    if (pages[p].column >= 0 && pages[p].column < n_cols) {
      slots[(size_t)pages[p].column] += pages[p].num_values;
      page_bytes[(size_t)pages[p].column] += pages[p].size;
    }
  // BYTE_ARRAY bytes on the device: PLAIN / DELTA_LENGTH values fit in their pages; dictionary
  // columns may expand, so the first attempt may come back short and is then re-run once at the
  // exact size the device counted
  std::vector<uint64_t> bin_cap(nc, 0);
  for (int i = 0; i < n_cols; i++)
    if (bin_out(cols[i]))
      bin_cap[(size_t)i] = page_bytes[(size_t)i] + (cols[i].dict_offset >= 0 ? 2 * (uint64_t)cols[i].dict_size : 0) + 64;
  if (ctx->host_bytes.ensure(n_bytes + pad) != hipSuccess || ctx->pin_in.ensure(n_bytes + pad) != hipSuccess ||
      ctx->host_counts.ensure(sizeof(uint32_t) * (size_t)std::max(n_pages, 1)) != hipSuccess) {
    set_status(st, PQG_ERR_HIP, -1, -1, "device buffers");
    return PQG_ERR_HIP;
  }
  // host -> pinned -> device (staged: the caller wrote the bytes into pin_in)
  if (!staged) par_memcpy(ctx->pin_in.p, h_bytes, n_bytes);
  std::memset((uint8_t*)ctx->pin_in.p + n_bytes, 0, pad);
  phase("stage-in");
  if (hipMemcpyAsync(ctx->host_bytes.p, ctx->pin_in.p, n_bytes + pad, hipMemcpyHostToDevice, s) != hipSuccess) return PQG_ERR_HIP;
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  std::vector<uint64_t> off_v(nc), off_d(nc), off_r(nc), off_b(nc);
  std::vector<pqg_column_desc> dcols(cols, cols + n_cols);
  // levels wanted: staged -> every column with a max level > 0; else where the caller gave an array
  std::vector<uint8_t> want_d(nc, 0), want_r(nc, 0);
  for (int i = 0; i < n_cols; i++) {
    want_d[(size_t)i] = cols[i].max_def > 0 && (staged || cols[i].def_levels);
    want_r[(size_t)i] = cols[i].max_rep > 0 && (staged || cols[i].rep_levels);
  }
  uint64_t total = 0;
  int rc = PQG_OK;
  pqg_status st2;
  for (int attempt = 0; attempt < 2; attempt++) {
    // device layout of outputs: per column values | def | rep | binary bytes, 256-B aligned
    total = 0;
    for (int i = 0; i < n_cols; i++) {
      const bool bin = bin_out(cols[i]);
      int w = out_width(cols[i]);
      if (w <= 0) w = 8;
      off_v[(size_t)i] = total;
      total = al(total + (slots[(size_t)i] + (bin ? 1 : 0)) * (uint64_t)w);
      off_d[(size_t)i] = total;
      if (want_d[(size_t)i]) total = al(total + slots[(size_t)i]);
      off_r[(size_t)i] = total;
      if (want_r[(size_t)i]) total = al(total + slots[(size_t)i]);
      off_b[(size_t)i] = total;
      if (bin) total = al(total + bin_cap[(size_t)i]);
    }
    if (ctx->host_out.ensure(total + 256) != hipSuccess || ctx->pin_out.ensure(total + 256) != hipSuccess) {
      set_status(st, PQG_ERR_HIP, -1, -1, "device buffers");
      return PQG_ERR_HIP;
    }
    uint8_t* dout = (uint8_t*)ctx->host_out.p;
    for (int i = 0; i < n_cols; i++) {
      const bool bin = bin_out(cols[i]);
      dcols[(size_t)i].values = dout + off_v[(size_t)i];
      dcols[(size_t)i].values_capacity = slots[(size_t)i] + (bin ? 1 : 0);
      dcols[(size_t)i].def_levels = want_d[(size_t)i] ? dout + off_d[(size_t)i] : nullptr;
      dcols[(size_t)i].rep_levels = want_r[(size_t)i] ? dout + off_r[(size_t)i] : nullptr;
      dcols[(size_t)i].levels_capacity = slots[(size_t)i];
      dcols[(size_t)i].binary_data = bin ? dout + off_b[(size_t)i] : nullptr;
      dcols[(size_t)i].binary_capacity = bin_cap[(size_t)i];
    }
    // the zero padding is part of the readable range: loads are range-checked per dword against it, and
    // a page ending at an unaligned offset close to n_bytes (raw file bytes) needs its last dword whole
    rc = decode_impl(ctx, (const uint8_t*)ctx->host_bytes.p, n_bytes + pad, n_bytes, dcols.data(), n_cols, pages,
                     n_pages, (uint32_t*)ctx->host_counts.p, st);
    if (rc) return rc;
    rc = pqg_sync(ctx, &st2);
    if (rc != PQG_ERR_INVALID_ARG || st2.page != -1 || !ctx->last || attempt == 1) break;
    // binary capacity: size every BYTE_ARRAY column to the byte count the device produced
    bool grew = false;
    for (int i = 0; i < n_cols; i++) {
      const uint64_t o = ctx->last->bin_total_off[(size_t)i];
      if (o == ~0ull) continue;
      uint64_t t = 0;
      if (hipMemcpy(&t, (uint8_t*)ctx->last->bscratch.p + o, sizeof(t), hipMemcpyDeviceToHost) != hipSuccess) return PQG_ERR_HIP;
      if (t > bin_cap[(size_t)i]) { bin_cap[(size_t)i] = t; grew = true; }
    }
    if (!grew) break;
  }
  for (int i = 0; i < n_cols; i++) cols[i].values_written = dcols[(size_t)i].values_written;
  if (rc && st) *st = st2;
  phase("h2d+decode");
  // device -> pinned -> host arrays (decoded values are valid up to the first error): the D2H goes
  // in HOST_CHUNK pieces, each followed by an event; worker threads copy the fixed-width values
  // and levels out of each piece as it lands
  uint8_t* dout = (uint8_t*)ctx->host_out.p;
  const uint8_t* po = (const uint8_t*)ctx->pin_out.p;
  std::vector<HostCopy> jobs;
  for (int i = 0; i < n_cols && !staged; i++) {
    const int w = out_width(cols[i]);
    const uint64_t n = std::min<uint64_t>(cols[i].values_written, cols[i].values_capacity);
    if (!bin_out(cols[i]) && cols[i].values && n)
      jobs.push_back({(uint8_t*)cols[i].values, off_v[(size_t)i], n * (uint64_t)w});
    if (cols[i].max_def > 0 && cols[i].def_levels)
      jobs.push_back({cols[i].def_levels, off_d[(size_t)i], std::min(slots[(size_t)i], cols[i].levels_capacity)});
    if (cols[i].max_rep > 0 && cols[i].rep_levels)
      jobs.push_back({cols[i].rep_levels, off_r[(size_t)i], std::min(slots[(size_t)i], cols[i].levels_capacity)});
  }
  const uint64_t n_chunks = (total + HOST_CHUNK - 1) / HOST_CHUNK;
  std::vector<hipEvent_t> ev((size_t)n_chunks, nullptr);
  bool ok = true;
  // odd chunks on a second stream (a second DMA queue), after the decode
  hipStream_t s2 = s;
  hipEvent_t dec_done = nullptr;
  if (n_chunks > 1) {
    if (!ctx->copy_stream && hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess)
      ctx->copy_stream = nullptr;
    if (ctx->copy_stream && hipEventCreateWithFlags(&dec_done, hipEventDisableTiming) == hipSuccess &&
        hipEventRecord(dec_done, s) == hipSuccess && hipStreamWaitEvent(ctx->copy_stream, dec_done, 0) == hipSuccess)
      s2 = ctx->copy_stream;
  }
  // The copy threads start first and take each piece once it is queued and its event has completed:
  // hipMemcpyAsync into pinned memory measured blocking here (its events had all completed when the
  // threads started, r05w), so a queue-then-copy order ran the host copies after the whole D2H.
  std::vector<std::atomic<int>> queued((size_t)n_chunks);
  for (auto& q : queued) q.store(0, std::memory_order_relaxed);
  const int T = std::max(1, std::min<int>(host_threads(total), (int)n_chunks));
  std::vector<int> wok((size_t)T, 1);
  std::vector<std::thread> th;
  std::vector<double> t_dma((size_t)n_chunks, 0.0);  // (PQG_HOST_TIMING: when each piece was seen landed)
  const auto t_d0 = std::chrono::steady_clock::now();
  for (int t = 0; t < T && !staged; t++)
    th.emplace_back([&, t] {
      if (hipSetDevice(ctx->device) != hipSuccess) { wok[(size_t)t] = 0; return; }
      for (uint64_t k = (uint64_t)t; k < n_chunks; k += (uint64_t)T) {
        int q;
        while ((q = queued[(size_t)k].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        if (q < 0 || hipEventSynchronize(ev[(size_t)k]) != hipSuccess) { wok[(size_t)t] = 0; return; }
        if (timing) t_dma[(size_t)k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_d0).count();
        copy_range(jobs, po, k * HOST_CHUNK, std::min(total, (k + 1) * HOST_CHUNK));
      }
    });
  for (uint64_t k = 0; k < n_chunks; k++) {
    const uint64_t a = k * HOST_CHUNK, len = std::min(HOST_CHUNK, total - a);
    hipStream_t sk = (k & 1) ? s2 : s;
    ok = ok && hipMemcpyAsync((uint8_t*)ctx->pin_out.p + a, dout + a, len, hipMemcpyDeviceToHost, sk) == hipSuccess &&
         hipEventCreateWithFlags(&ev[(size_t)k], hipEventDisableTiming) == hipSuccess &&
         hipEventRecord(ev[(size_t)k], sk) == hipSuccess;
    queued[(size_t)k].store(ok ? 1 : -1, std::memory_order_release);  // (-1: the threads stop)
  }
  std::vector<uint32_t> counts((size_t)std::max(n_pages, 1));
  if (ok && n_pages)
    ok = hipMemcpyAsync(counts.data(), ctx->host_counts.p, sizeof(uint32_t) * (size_t)n_pages, hipMemcpyDeviceToHost, s) == hipSuccess;
  for (auto& x : th) x.join();
  for (int v : wok) ok = ok && v;
  if (timing && n_chunks && !staged)
    std::fprintf(stderr, "pqg_decode_host   last D2H piece seen landed %.3f ms after the copy threads started (%d threads)\n",
                 *std::max_element(t_dma.begin(), t_dma.end()), T);
  if (s2 != s && hipStreamSynchronize(s2) != hipSuccess) ok = false;
  for (hipEvent_t e : ev)
    if (e) (void)hipEventDestroy(e);
  if (dec_done) (void)hipEventDestroy(dec_done);
  if (!ok || hipStreamSynchronize(s) != hipSuccess) return PQG_ERR_HIP;
  phase("d2h+copy");
  if (staged) {
    // outputs stay in pin_out: describe them (pqg_staged_column)
    ctx->staged.resize(nc);
    for (int i = 0; i < n_cols; i++) {
      pqg_staged_output& o = ctx->staged[(size_t)i];
      o.values = po + off_v[(size_t)i];
      o.def_levels = want_d[(size_t)i] ? po + off_d[(size_t)i] : nullptr;
      o.rep_levels = want_r[(size_t)i] ? po + off_r[(size_t)i] : nullptr;
      o.n_values = std::min<uint64_t>(cols[i].values_written, slots[(size_t)i]);
      o.n_slots = slots[(size_t)i];
      o.binary = nullptr;
      o.n_binary = 0;
      if (bin_out(cols[i])) {
        const uint64_t nb = (uint64_t)((const int64_t*)o.values)[o.n_values];
        if (nb > bin_cap[(size_t)i]) {  // the device's count did not fit even after the resize
          if (rc == PQG_OK) {
            rc = PQG_ERR_INVALID_ARG;
            set_status(st, rc, -1, (int64_t)nb, "binary capacity");
          }
        } else {
          o.binary = po + off_b[(size_t)i];
          o.n_binary = nb;
        }
      }
    }
    if (h_page_value_counts && n_pages) std::memcpy(h_page_value_counts, counts.data(), sizeof(uint32_t) * (size_t)n_pages);
    return rc;
  }
  for (int i = 0; i < n_cols; i++) {
    if (!bin_out(cols[i])) continue;
    // offsets[n + 1] and the bytes they span
    const uint64_t n = std::min<uint64_t>(cols[i].values_written, cols[i].values_capacity ? cols[i].values_capacity - 1 : 0);
    const int64_t* offs = (const int64_t*)(po + off_v[(size_t)i]);
    if (cols[i].values && cols[i].values_capacity) par_memcpy(cols[i].values, offs, (n + 1) * sizeof(int64_t));
    const uint64_t nb = (uint64_t)offs[n];
    if (nb > cols[i].binary_capacity) {
      if (rc == PQG_OK) {
        rc = PQG_ERR_INVALID_ARG;
        if (st) {
          st->code = rc;
          st->page = -1;
          st->value_index = (int64_t)nb;
          std::snprintf(st->message, sizeof(st->message), "binary capacity: column %d needs %llu bytes", i,
                        (unsigned long long)nb);
        }
      }
    } else if (cols[i].binary_data && nb) {
      par_memcpy(cols[i].binary_data, po + off_b[(size_t)i], nb);
    }
  }
  if (h_page_value_counts && n_pages) std::memcpy(h_page_value_counts, counts.data(), sizeof(uint32_t) * (size_t)n_pages);
  phase("binary");
  return rc;
}

int pqg_decode_host(pqg_ctx* ctx, const uint8_t* h_bytes, uint64_t n_bytes, pqg_column_desc* cols, int n_cols,
                    const pqg_page_desc* pages, int n_pages, uint32_t* h_page_value_counts, pqg_status* st) {
  static const uint8_t empty = 0;
  if (n_bytes && !h_bytes) {
    if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
    return PQG_ERR_INVALID_ARG;
  }
  return host_path(ctx, h_bytes ? h_bytes : &empty, n_bytes, cols, n_cols, pages, n_pages, h_page_value_counts, st);
}

int pqg_host_input(pqg_ctx* ctx, uint64_t n_bytes, uint8_t** buf) {
  if (!ctx || !buf) return PQG_ERR_INVALID_ARG;
  *buf = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  // the decode pads with 1,024 zero bytes after n_bytes (host_path's `pad`)
  if (ctx->pin_in.ensure(n_bytes + 1024) != hipSuccess) return PQG_ERR_HIP;
  ctx->staged.clear();
  *buf = (uint8_t*)ctx->pin_in.p;
  return PQG_OK;
}

int pqg_decode_staged(pqg_ctx* ctx, uint64_t n_bytes, pqg_column_desc* cols, int n_cols, const pqg_page_desc* pages,
                      int n_pages, uint32_t* h_page_value_counts, pqg_status* st) {
  return host_path(ctx, nullptr, n_bytes, cols, n_cols, pages, n_pages, h_page_value_counts, st);
}

int pqg_staged_column(pqg_ctx* ctx, int col, pqg_staged_output* out) {
  if (!ctx || !out || col < 0 || (size_t)col >= ctx->staged.size()) return PQG_ERR_INVALID_ARG;
  *out = ctx->staged[(size_t)col];
  return PQG_OK;
}

void pqg_copy_out(void* dst, const void* src, uint64_t n) {
  if (n && dst && src) par_memcpy(dst, src, n);
}

int pqg_assemble(pqg_ctx* ctx, const uint8_t* d_def_levels, const uint8_t* d_rep_levels, uint64_t n_slots,
                 pqg_assembly_node* path, int depth, uint64_t* n_records, pqg_status* st) {
  if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
  if (!ctx || !path || depth <= 0 || depth > (int)pqg::ASM_MAX_NODES) {
    set_status(st, PQG_ERR_INVALID_ARG, -1, -1, "assembly arguments");
    return PQG_ERR_INVALID_ARG;
  }
  // levels of every node (ColumnIO repetition / definition level)
  pqg::AsmParams P;
  std::memset(&P, 0, sizeof(P));
  P.n_nodes = (uint32_t)depth;
  uint32_t r = 0, d = 0;
  for (int k = 0; k < depth; k++) {
    const int rp = path[k].repetition;
    if (rp != PQG_REQUIRED && rp != PQG_OPTIONAL && rp != PQG_REPEATED) {
      set_status(st, PQG_ERR_INVALID_ARG, -1, k, "assembly node repetition");
      return PQG_ERR_INVALID_ARG;
    }
    if (rp == PQG_REPEATED) {
      r++;
      d++;
      if (r >= pqg::ASM_MAX_DEPTHS) {
        set_status(st, PQG_ERR_UNSUPPORTED, -1, k, "assembly: more than 7 repetition levels");
        return PQG_ERR_UNSUPPORTED;
      }
      P.DR[r] = d;
    } else if (rp == PQG_OPTIONAL) {
      d++;
    }
    P.kind[k] = rp;
    P.depth[k] = r;
    P.D[k] = d;
    P.validity[k] = rp == PQG_OPTIONAL ? path[k].validity : nullptr;
    P.offsets[k] = rp == PQG_REPEATED ? path[k].offsets : nullptr;
  }
  P.max_rep = r;
  if (d > 254) {
    set_status(st, PQG_ERR_UNSUPPORTED, -1, -1, "assembly: definition level above 254");
    return PQG_ERR_UNSUPPORTED;
  }
  if (n_slots && ((d > 0 && !d_def_levels) || (r > 0 && !d_rep_levels))) {
    set_status(st, PQG_ERR_INVALID_ARG, -1, -1, "assembly levels");
    return PQG_ERR_INVALID_ARG;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  hipStream_t s = ctx->stream;
  const uint32_t n_blocks = (uint32_t)((n_slots + 4095) / 4096);
  const size_t cnt_bytes = sizeof(uint64_t) * pqg::ASM_MAX_DEPTHS * (size_t)std::max<uint32_t>(n_blocks, 1);
  if (ctx->asm_scratch.ensure(cnt_bytes + 256) != hipSuccess || ctx->pin_err.ensure(256) != hipSuccess) return PQG_ERR_HIP;
  uint64_t* counts = (uint64_t*)ctx->asm_scratch.p;  // block counts (count pass) / look-back status words
  uint64_t* totals = (uint64_t*)((uint8_t*)ctx->asm_scratch.p + cnt_bytes);
  uint32_t* ticket = (uint32_t*)(totals + pqg::ASM_MAX_DEPTHS);
  bool any_out = false, bounded = true;
  for (int k = 0; k < depth; k++) {
    any_out = any_out || P.validity[k] || P.offsets[k];
    // entries of any depth <= n_slots: outputs sized for that bound need no count round trip
    if ((P.validity[k] && path[k].capacity < n_slots) || (P.offsets[k] && path[k].capacity < n_slots + 1)) bounded = false;
  }
  const uint8_t* dl = d > 0 ? d_def_levels : nullptr;
  const uint8_t* rl = r > 0 ? d_rep_levels : nullptr;
  // the single pass: status words, totals and the ticket zeroed, then one kernel (outputs + totals)
  auto emit = [&]() -> hipError_t {
    hipError_t e2 = hipMemsetAsync(ctx->asm_scratch.p, 0, cnt_bytes + sizeof(uint64_t) * pqg::ASM_MAX_DEPTHS + 16, s);
    if (e2 == hipSuccess) e2 = pqg::launch_assemble(s, dl, rl, n_slots, P, counts, n_blocks, totals, ticket, 1);
    if (e2 == hipSuccess && n_blocks == 0)  // no slots: closing offsets only (offsets[0] = 0)
      for (int k = 0; k < depth && e2 == hipSuccess; k++)
        if (P.kind[k] == PQG_REPEATED && P.offsets[k]) e2 = hipMemsetAsync(P.offsets[k], 0, sizeof(int64_t), s);
    return e2;
  };
  const bool one_pass = any_out && bounded;
  hipError_t e = one_pass ? emit() : pqg::launch_assemble(s, dl, rl, n_slots, P, counts, n_blocks, totals, ticket, 0);
  uint64_t* h_tot = (uint64_t*)ctx->pin_err.p;
  if (e == hipSuccess) e = hipMemcpyAsync(h_tot, totals, sizeof(uint64_t) * pqg::ASM_MAX_DEPTHS, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    set_status(st, PQG_ERR_HIP, -1, -1, hipGetErrorString(e));
    return PQG_ERR_HIP;
  }
  if (h_tot[pqg::ASM_MAX_DEPTHS - 1] == ~0ull) {  // a look-back wait timed out (k_asm_onepass)
    set_status(st, PQG_ERR_TIMEOUT, -1, -1, "assembly look-back");
    return PQG_ERR_TIMEOUT;
  }
  if (n_records) *n_records = h_tot[0];
  int bad = -1;
  for (int k = 0; k < depth; k++) {
    path[k].n_entries = h_tot[P.depth[k]];
    uint64_t need = 0;
    if (P.kind[k] == PQG_OPTIONAL && P.validity[k]) need = h_tot[P.depth[k]];
    if (P.kind[k] == PQG_REPEATED && P.offsets[k]) need = h_tot[P.depth[k] - 1] + 1;
    if (need > path[k].capacity && bad < 0) bad = k;
  }
  if (bad >= 0) {
    set_status(st, PQG_ERR_INVALID_ARG, -1, bad, "assembly output capacity");
    return PQG_ERR_INVALID_ARG;
  }
  if (!any_out || one_pass) return PQG_OK;  // counts only, or already emitted
  e = emit();
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    set_status(st, PQG_ERR_HIP, -1, -1, hipGetErrorString(e));
    return PQG_ERR_HIP;
  }
  return PQG_OK;
}

int pqg_assemble_schema(pqg_ctx* ctx, pqg_schema_node* nodes, int n_nodes, const pqg_schema_leaf* leaves, int n_leaves,
                        uint64_t* n_records, pqg_status* st) {
  if (st) { std::memset(st, 0, sizeof(*st)); st->page = -1; }
  if (!ctx || !nodes || n_nodes <= 0 || (n_leaves > 0 && !leaves) || n_leaves < 0) {
    set_status(st, PQG_ERR_INVALID_ARG, -1, -1, "schema assembly arguments");
    return PQG_ERR_INVALID_ARG;
  }
  for (int k = 0; k < n_nodes; k++)
    if (nodes[k].parent >= k || nodes[k].parent < -1) {
      set_status(st, PQG_ERR_INVALID_ARG, -1, k, "schema node parent");
      return PQG_ERR_INVALID_ARG;
    }
  std::vector<int> owner((size_t)n_nodes, -1);  // leaf whose pass wrote the node's outputs
  uint64_t records = 0;
  for (int li = 0; li < n_leaves; li++) {
    const pqg_schema_leaf& lf = leaves[li];
    if (lf.node < 0 || lf.node >= n_nodes) {
      set_status(st, PQG_ERR_INVALID_ARG, li, -1, "schema leaf node");
      return PQG_ERR_INVALID_ARG;
    }
    for (int k = 0; k < n_nodes; k++)
      if (nodes[k].parent == lf.node) {
        set_status(st, PQG_ERR_INVALID_ARG, li, k, "schema leaf has children");
        return PQG_ERR_INVALID_ARG;
      }
    // the leaf's path: root's child .. leaf
    std::vector<int> chain;
    for (int k = lf.node; k >= 0; k = nodes[k].parent) chain.push_back(k);
    std::reverse(chain.begin(), chain.end());
    if (chain.size() > pqg::ASM_MAX_NODES) {
      set_status(st, PQG_ERR_UNSUPPORTED, li, -1, "schema assembly: path too deep");
      return PQG_ERR_UNSUPPORTED;
    }
    std::vector<pqg_assembly_node> path(chain.size());
    for (size_t q = 0; q < chain.size(); q++) {
      const pqg_schema_node& n = nodes[chain[q]];
      pqg_assembly_node& a = path[q];
      std::memset(&a, 0, sizeof(a));
      a.repetition = n.repetition;
      if (owner[(size_t)chain[q]] < 0) {  // first leaf under this node: it writes the outputs
        a.validity = n.validity;
        a.offsets = n.offsets;
        a.capacity = n.capacity;
      }
    }
    uint64_t nrec = 0;
    const int rc = pqg_assemble(ctx, lf.d_def_levels, lf.d_rep_levels, lf.n_slots, path.data(), (int)path.size(), &nrec, st);
    if (rc) {
      if (st) st->page = li;
      if (st && rc == PQG_ERR_INVALID_ARG && st->value_index >= 0 && st->value_index < (int64_t)chain.size())
        st->value_index = chain[(size_t)st->value_index];  // path position -> node index
      return rc;
    }
    if (li > 0 && nrec != records) {
      set_status(st, PQG_ERR_CORRUPT, li, -1, "schema assembly: leaves disagree on the record count");
      return PQG_ERR_CORRUPT;
    }
    records = nrec;
    for (size_t q = 0; q < chain.size(); q++) {
      const int k = chain[q];
      if (owner[(size_t)k] < 0) {
        owner[(size_t)k] = li;
        nodes[k].n_entries = path[q].n_entries;
      } else if (nodes[k].n_entries != path[q].n_entries) {
        set_status(st, PQG_ERR_CORRUPT, li, k, "schema assembly: leaves disagree on a node's entries");
        return PQG_ERR_CORRUPT;
      }
    }
  }
  if (n_records) *n_records = records;
  return PQG_OK;
}

int pqg_unpack_runs(pqg_ctx* ctx, int bit_width, const uint8_t* d_in, const uint64_t* d_in_offsets,
                    const uint32_t* d_counts, const uint64_t* d_out_offsets, int32_t* d_out, int n_runs) {
  if (!ctx || bit_width < 0 || bit_width > 32 || n_runs < 0) return PQG_ERR_INVALID_ARG;
  if (n_runs == 0) return PQG_OK;
  if (!d_in || !d_in_offsets || !d_counts || !d_out_offsets || !d_out) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  // the kernel grid-strides inside each run; 64 blocks x 256 lanes per run
  hipError_t e = pqg::launch_unpack_runs(ctx->stream, bit_width, d_in, ~0ull >> 1, d_in_offsets, d_counts, d_out_offsets,
                                         d_out, n_runs, 1u << 14);
  return e == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

static_assert(sizeof(pqg_snappy_job) == 24, "pqg_snappy_job layout");

int pqg_snappy_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                          const pqg_snappy_job* d_jobs, int n_jobs, int32_t* d_status) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (n_jobs == 0) return PQG_OK;
  if (!d_src || !d_dst || !d_jobs) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  const hipError_t e = pqg::launch_snappy(ctx->stream, d_src, src_bytes, d_dst, dst_bytes, d_jobs, n_jobs, d_status);
  return e == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

int pqg_snappy_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
  if (st) set_status(st, PQG_OK, -1, -1, "snappy");
  if (!d_status || n_jobs == 0) return PQG_OK;
  std::vector<int32_t> h((size_t)n_jobs);
  if (hipMemcpy(h.data(), d_status, sizeof(int32_t) * (size_t)n_jobs, hipMemcpyDeviceToHost) != hipSuccess)
    return PQG_ERR_HIP;
  for (int j = 0; j < n_jobs; j++)
    if (h[(size_t)j]) {
      set_status(st, h[(size_t)j], j, -1, "snappy block");
      return h[(size_t)j];
    }
  return PQG_OK;
}

int pqg_lz4_raw_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                           const pqg_lz4_job* d_jobs, int n_jobs, int32_t* d_status) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (n_jobs == 0) return PQG_OK;
  if (!d_src || !d_dst || !d_jobs) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  const hipError_t e = pqg::launch_lz4raw(ctx->stream, d_src, src_bytes, d_dst, dst_bytes, d_jobs, n_jobs, d_status);
  return e == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

int pqg_lz4_raw_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
  if (st) set_status(st, PQG_OK, -1, -1, "lz4_raw");
  if (!d_status || n_jobs == 0) return PQG_OK;
  std::vector<int32_t> h((size_t)n_jobs);
  if (hipMemcpy(h.data(), d_status, sizeof(int32_t) * (size_t)n_jobs, hipMemcpyDeviceToHost) != hipSuccess)
    return PQG_ERR_HIP;
  for (int j = 0; j < n_jobs; j++)
    if (h[(size_t)j]) {
      set_status(st, h[(size_t)j], j, -1, "lz4_raw block");
      return h[(size_t)j];
    }
  return PQG_OK;
}

int pqg_gzip_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                        const pqg_gzip_job* d_jobs, int n_jobs, int32_t* d_status) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (n_jobs == 0) return PQG_OK;
  if (!d_src || !d_dst || !d_jobs) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  // token pre-pass scratch: dst_bytes / 3 + 2 eight-byte records and one word per job; without it
  // every job takes the scalar decoder
  uint64_t* recs = nullptr;
  int32_t* mode = nullptr;
  {
    const size_t need_r = 8u * (size_t)(dst_bytes / 3u + 2u), need_m = 4u * (size_t)n_jobs;
    if (ctx->gzip_recs.cap < need_r || ctx->gzip_mode.cap < need_m) {
      if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
      if (ctx->gzip_recs.ensure(need_r) != hipSuccess || ctx->gzip_mode.ensure(need_m) != hipSuccess) {
        (void)hipGetLastError();
        ctx->gzip_recs.release();
        ctx->gzip_mode.release();
      }
    }
    if (ctx->gzip_recs.cap >= need_r && ctx->gzip_mode.cap >= need_m) {
      recs = (uint64_t*)ctx->gzip_recs.p;
      mode = (int32_t*)ctx->gzip_mode.p;
    }
  }
  const hipError_t e = pqg::launch_gzip(ctx->stream, d_src, src_bytes, d_dst, dst_bytes, d_jobs, n_jobs, d_status,
                                        recs, mode, ctx->gz_prepass_min);
  return e == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

int pqg_gzip_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
  if (st) set_status(st, PQG_OK, -1, -1, "gzip");
  if (!d_status || n_jobs == 0) return PQG_OK;
  std::vector<int32_t> h((size_t)n_jobs);
  if (hipMemcpy(h.data(), d_status, sizeof(int32_t) * (size_t)n_jobs, hipMemcpyDeviceToHost) != hipSuccess)
    return PQG_ERR_HIP;
  for (int j = 0; j < n_jobs; j++)
    if (h[(size_t)j]) {
      set_status(st, h[(size_t)j], j, -1, "gzip block");
      return h[(size_t)j];
    }
  return PQG_OK;
}

int pqg_zstd_decompress(pqg_ctx* ctx, const uint8_t* d_src, uint64_t src_bytes, uint8_t* d_dst, uint64_t dst_bytes,
                        const pqg_zstd_job* d_jobs, int n_jobs, int32_t* d_status) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (n_jobs == 0) return PQG_OK;
  if (!d_src || !d_dst || !d_jobs) return PQG_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  // the scratch may be in use by a previous call still queued on the stream: grow only after it
  // one literal buffer per wave of the (bounded) grid, not per job
  const uint64_t slots = (uint64_t)std::min<int>(n_jobs, (int)pqg::ZSTD_GRID);
  if (ctx->zstd_scratch.cap < pqg::ZSTD_LIT_SCRATCH * slots) {
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
    if (ctx->zstd_scratch.ensure(pqg::ZSTD_LIT_SCRATCH * slots) != hipSuccess) return PQG_ERR_HIP;
  }
  // sequence pre-pass scratch: dst_bytes / 5 + 1 eight-byte records (a job's records start at its
  // dst_offset / 5) and one mode word per job; without it every job takes the inline decoder
  uint64_t* seqs = nullptr;
  int32_t* mode = nullptr;
  {
    const size_t need_s = 8u * (size_t)(dst_bytes / 5u + 2u), need_m = 4u * (size_t)n_jobs;
    if (ctx->zstd_seqs.cap < need_s || ctx->zstd_mode.cap < need_m) {
      if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
      if (ctx->zstd_seqs.ensure(need_s) != hipSuccess || ctx->zstd_mode.ensure(need_m) != hipSuccess) {
        (void)hipGetLastError();
        ctx->zstd_seqs.release();
        ctx->zstd_mode.release();
      }
    }
    if (ctx->zstd_seqs.cap >= need_s && ctx->zstd_mode.cap >= need_m) {
      seqs = (uint64_t*)ctx->zstd_seqs.p;
      mode = (int32_t*)ctx->zstd_mode.p;
    }
  }
  const hipError_t e = pqg::launch_zstd(ctx->stream, d_src, src_bytes, d_dst, dst_bytes, d_jobs, n_jobs, d_status,
                                        (uint8_t*)ctx->zstd_scratch.p, seqs, mode);
  return e == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

int pqg_zstd_sync(pqg_ctx* ctx, const int32_t* d_status, int n_jobs, pqg_status* st) {
  if (!ctx || n_jobs < 0) return PQG_ERR_INVALID_ARG;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return PQG_ERR_HIP;
  if (st) set_status(st, PQG_OK, -1, -1, "zstd");
  if (!d_status || n_jobs == 0) return PQG_OK;
  std::vector<int32_t> h((size_t)n_jobs);
  if (hipMemcpy(h.data(), d_status, sizeof(int32_t) * (size_t)n_jobs, hipMemcpyDeviceToHost) != hipSuccess)
    return PQG_ERR_HIP;
  for (int j = 0; j < n_jobs; j++)
    if (h[(size_t)j]) {
      set_status(st, h[(size_t)j], j, -1, "zstd frame");
      return h[(size_t)j];
    }
  return PQG_OK;
}

int pqg_router_read(pqg_ctx* ctx, int bit_width, const uint8_t* in, size_t in_len, int count, int32_t* out) {
  if (!ctx || bit_width < 0 || bit_width > 32 || count < 0 || (count && (!in || !out))) return PQG_ERR_INVALID_ARG;
  if (count % 8 != 0) return PQG_ERR_INVALID_ARG;  // currentCount of a bit-packed run is a multiple of 8
  const uint64_t need = (uint64_t)count * (uint64_t)bit_width / 8u;
  if (need > in_len) return PQG_ERR_EOF;  // in.slice(count * bitWidth / 8) -> EOFException
  if (count == 0) return PQG_OK;
  ctx->staged.clear();  // pin_in / pin_out are reused: an earlier staged decode's outputs are gone
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  hipStream_t s = ctx->stream;
  const uint64_t in_al = (need + 16 + 255) & ~uint64_t(255);
  const uint64_t tail = 32;  // [in_off, counts, out_off]
  if (ctx->host_runs.ensure(in_al + (uint64_t)count * 4 + 256 + tail) != hipSuccess ||
      ctx->pin_in.ensure(in_al + tail) != hipSuccess || ctx->pin_out.ensure((uint64_t)count * 4) != hipSuccess)
    return PQG_ERR_HIP;
  uint8_t* pin = (uint8_t*)ctx->pin_in.p;
  std::memcpy(pin, in, need);
  std::memset(pin + need, 0, in_al - need);
  uint64_t* meta = (uint64_t*)(pin + in_al);
  meta[0] = 0;                               // in offset
  ((uint32_t*)&meta[1])[0] = (uint32_t)count; // count
  meta[2] = 0;                               // out offset
  uint8_t* d = (uint8_t*)ctx->host_runs.p;
  int32_t* dout = (int32_t*)(d + in_al + tail + 256 - ((uintptr_t)(d + in_al + tail) & 255));
  if (hipMemcpyAsync(d, pin, in_al + tail, hipMemcpyHostToDevice, s) != hipSuccess) return PQG_ERR_HIP;
  hipError_t e = pqg::launch_unpack_runs(s, bit_width, d, need + 16, (const uint64_t*)(d + in_al),
                                         (const uint32_t*)(d + in_al + 8), (const uint64_t*)(d + in_al + 16), dout, 1,
                                         (uint32_t)count);
  if (e != hipSuccess) return PQG_ERR_HIP;
  if (hipMemcpyAsync(ctx->pin_out.p, dout, (size_t)count * 4, hipMemcpyDeviceToHost, s) != hipSuccess) return PQG_ERR_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return PQG_ERR_HIP;
  std::memcpy(out, ctx->pin_out.p, (size_t)count * 4);
  return PQG_OK;
}

int pqg_router_read_runs(pqg_ctx* ctx, int bit_width, const uint8_t* in, size_t in_len, const uint64_t* in_offsets,
                         const uint32_t* counts, int n_runs, int32_t* out) {
  if (!ctx || bit_width < 0 || bit_width > 32 || n_runs < 0) return PQG_ERR_INVALID_ARG;
  if (n_runs == 0) return PQG_OK;
  if (!in_offsets || !counts || !out) return PQG_ERR_INVALID_ARG;
  // every run's slice first (SingleBufferInputStream.slice throws before any unpack)
  uint64_t n_bytes = 0, n_vals = 0;
  uint32_t max_count = 0;
  for (int r = 0; r < n_runs; r++) {
    if (counts[r] % 8u != 0) return PQG_ERR_INVALID_ARG;
    const uint64_t need = (uint64_t)counts[r] * (uint64_t)bit_width / 8u;
    if (in_offsets[r] > in_len || need > in_len - in_offsets[r]) return PQG_ERR_EOF;
    if (need && !in) return PQG_ERR_INVALID_ARG;
    n_bytes += (need + 15) & ~uint64_t(15);
    n_vals += counts[r];
    max_count = std::max(max_count, counts[r]);
  }
  if (n_vals == 0) return PQG_OK;
  ctx->staged.clear();  // pin_in / pin_out are reused: an earlier staged decode's outputs are gone
  if (hipSetDevice(ctx->device) != hipSuccess) return PQG_ERR_HIP;
  hipStream_t s = ctx->stream;
  // pinned image: [run bytes, each 16-B aligned][in_off u64 x n][out_off u64 x n][counts u32 x n]
  auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  const uint64_t o_in = al(n_bytes + 16), o_out = o_in + 8ull * (uint64_t)n_runs, o_cnt = o_out + 8ull * (uint64_t)n_runs;
  const uint64_t img = al(o_cnt + 4ull * (uint64_t)n_runs);
  if (ctx->pin_in.ensure(img) != hipSuccess || ctx->pin_out.ensure(4 * n_vals) != hipSuccess ||
      ctx->host_runs.ensure(img + 4 * n_vals + 256) != hipSuccess)
    return PQG_ERR_HIP;
  uint8_t* pin = (uint8_t*)ctx->pin_in.p;
  uint64_t* pin_in_off = (uint64_t*)(pin + o_in);
  uint64_t* pin_out_off = (uint64_t*)(pin + o_out);
  uint32_t* pin_cnt = (uint32_t*)(pin + o_cnt);
  uint64_t b = 0, v = 0;
  for (int r = 0; r < n_runs; r++) {
    const uint64_t need = (uint64_t)counts[r] * (uint64_t)bit_width / 8u;
    if (need) std::memcpy(pin + b, in + in_offsets[r], need);
    const uint64_t padded = (need + 15) & ~uint64_t(15);
    std::memset(pin + b + need, 0, padded - need);
    pin_in_off[r] = b;
    pin_out_off[r] = v;
    pin_cnt[r] = counts[r];
    b += padded;
    v += counts[r];
  }
  std::memset(pin + n_bytes, 0, o_in - n_bytes);
  uint8_t* d = (uint8_t*)ctx->host_runs.p;
  int32_t* dout = (int32_t*)(d + img);
  if (hipMemcpyAsync(d, pin, img, hipMemcpyHostToDevice, s) != hipSuccess) return PQG_ERR_HIP;
  for (int r0 = 0; r0 < n_runs; r0 += 65535) {  // grid.y holds the run index
    const int nr = std::min(n_runs - r0, 65535);
    const hipError_t e = pqg::launch_unpack_runs(s, bit_width, d, n_bytes + 16, (const uint64_t*)(d + o_in) + r0,
                                                 (const uint32_t*)(d + o_cnt) + r0, (const uint64_t*)(d + o_out) + r0,
                                                 dout, nr, max_count);
    if (e != hipSuccess) return PQG_ERR_HIP;
  }
  if (hipMemcpyAsync(ctx->pin_out.p, dout, (size_t)(4 * n_vals), hipMemcpyDeviceToHost, s) != hipSuccess) return PQG_ERR_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) return PQG_ERR_HIP;
  std::memcpy(out, ctx->pin_out.p, (size_t)(4 * n_vals));
  return PQG_OK;
}

}  // extern "C"

// ---- ParquetReadRouter.read with the page's runs cached --------------------------------------------

namespace {

// Bounds of one walk: what a miss decodes in its single round trip.
constexpr uint64_t ROUTER_MAX_VALUES = 1u << 22;
constexpr size_t ROUTER_MAX_RUNS = 1u << 16;

// Served from the cache when the run at this stream position (stream_left bytes before the end) was
// walked, with the same width and count, and its bytes are the ones unpacked then.
bool router_hit(RouterCache& c, int w, const uint8_t* in, uint64_t need, uint64_t stream_left, int count,
                int32_t* out) {
  if (c.w != w || stream_left > c.tail_len || c.off.empty()) return false;
  const uint64_t pos = c.tail_len - stream_left;
  const auto it = std::lower_bound(c.off.begin(), c.off.end(), pos);
  if (it == c.off.end() || *it != pos) return false;
  const size_t r = (size_t)(it - c.off.begin());
  if (c.cnt[r] != (uint32_t)count) return false;
  if (need && std::memcmp(in, c.bytes.data() + pos, need) != 0) return false;
  std::memcpy(out, c.vals.data() + c.vo[r], (size_t)count * 4);
  c.hits++;
  return true;
}

}  // namespace

extern "C" {

int pqg_router_cache_lookup(pqg_ctx* ctx, int bit_width, const uint8_t* run, size_t stream_left, int count,
                            int32_t* out, int* hit) {
  if (!ctx || !hit || bit_width < 0 || bit_width > 32 || count < 0 || count % 8 != 0 || (count && !out))
    return PQG_ERR_INVALID_ARG;
  *hit = 0;
  const uint64_t need = (uint64_t)count * (uint64_t)bit_width / 8u;
  if (need > stream_left) return PQG_ERR_EOF;
  if (need && !run) return PQG_ERR_INVALID_ARG;
  if (count == 0) {
    *hit = 1;
    return PQG_OK;
  }
  *hit = router_hit(ctx->router, bit_width, run, need, stream_left, count, out) ? 1 : 0;
  return PQG_OK;
}

int pqg_router_read_page(pqg_ctx* ctx, int bit_width, const uint8_t* in, size_t stream_left, int count, int32_t* out) {
  int hit = 0;
  const int lrc = pqg_router_cache_lookup(ctx, bit_width, in, stream_left, count, out, &hit);
  if (lrc != PQG_OK || hit) return lrc;
  if (!in) return PQG_ERR_INVALID_ARG;
  RouterCache& c = ctx->router;
  const uint64_t L = stream_left, need = (uint64_t)count * (uint64_t)bit_width / 8u;
  // Walk the hybrid stream after this run (RunLengthBitPackingHybridDecoder.readNext :80-109 header
  // forms; BytesUtils.readUnsignedVarInt :202-211) and list every bit-packed run whose bytes are in the
  // stream. The walk is a prediction of the caller's next reads: bytes past the hybrid stream (data the
  // caller reads otherwise) may parse as runs, which are decoded and never served; a header that cannot
  // be a run ends the walk. Runs the walk missed are served by a later miss.
  c.w = -1;
  c.off.clear();
  c.cnt.clear();
  c.vo.clear();
  c.off.push_back(0);
  c.cnt.push_back((uint32_t)count);
  c.vo.push_back(0);
  uint64_t total = (uint64_t)count, q = need;
  const uint32_t nb_rle = ((uint32_t)bit_width + 7u) / 8u;
  while (q < L && c.off.size() < ROUTER_MAX_RUNS) {
    uint32_t hdr = 0, sh = 0, b = 0;
    uint64_t k = q;
    bool ok = true;
    while (true) {
      if (k >= L || sh > 28) { ok = false; break; }
      b = in[k++];
      if (!(b & 0x80u)) break;
      hdr |= (b & 0x7Fu) << sh;
      sh += 7;
    }
    if (!ok) break;
    hdr |= b << sh;
    if (!(hdr & 1u)) {  // RLE run: count, then the value in ceil(w / 8) bytes
      q = k + nb_rle;
      continue;
    }
    const uint64_t groups = hdr >> 1, vals = groups * 8u, bytes = groups * (uint64_t)bit_width;
    if (vals > 0x7FFFFFF8u || k + bytes > L || total + vals > ROUTER_MAX_VALUES) break;
    if (vals) {
      c.off.push_back(k);
      c.cnt.push_back((uint32_t)vals);
      c.vo.push_back(total);
      total += vals;
    }
    q = k + bytes;
  }
  c.vals.resize(total);
  const uint64_t keep = c.off.size() > 1 ? c.off.back() + (uint64_t)c.cnt.back() * (uint64_t)bit_width / 8u : need;
  c.bytes.assign(in, in + keep);
  c.tail_len = L;
  c.misses++;
  const int rc = pqg_router_read_runs(ctx, bit_width, in, (size_t)L, c.off.data(), c.cnt.data(), (int)c.off.size(),
                                      c.vals.data());
  if (rc != PQG_OK) {
    c.off.clear();
    return rc;
  }
  c.w = bit_width;
  std::memcpy(out, c.vals.data(), (size_t)count * 4);
  return PQG_OK;
}

int pqg_router_cache_stats(pqg_ctx* ctx, uint64_t* hits, uint64_t* misses) {
  if (!ctx) return PQG_ERR_INVALID_ARG;
  if (hits) *hits = ctx->router.hits;
  if (misses) *misses = ctx->router.misses;
  return PQG_OK;
}

}  // extern "C"

