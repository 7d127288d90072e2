// pqgpu_internal.h — device-side tables shared by the kernels and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pqgpu.h"

namespace pqg {

// Per output column, on the device.
struct ColumnDev {
  int32_t physical_type;
  int32_t type_length;
  int32_t max_rep;
  int32_t max_def;
  int32_t elem_width;   // bytes per dense value
  uint32_t dict_n;      // dictionary entries (0 if none)
  uint64_t dict_offset; // dictionary page body offset in the batch
  uint64_t dict_bytes;  // dictionary page body bytes
  void* values;
  uint8_t* def_levels;
  uint8_t* rep_levels;
  // BYTE_ARRAY columns: `values` = int64 offsets[n_slots + 1] into binary_data; per value
  // scratch: blen (length; dictionary ids of RLE_DICTIONARY pages until k_bin_dict_map) and
  // bsrc (source byte offset relative to the page body, or to the dictionary page body)
  uint8_t* binary_data;
  uint64_t binary_capacity;
  uint32_t* blen;
  uint32_t* bsrc;
  // BYTE_ARRAY dictionary entries (PlainBinaryDictionary): length and offset in the dictionary page
  uint32_t* dict_len;
  uint32_t* dict_src;
  uint64_t n_slots;        // level slots of the column in the batch (offsets span n_slots + 1)
  uint64_t* block_sums;    // BYTE_ARRAY offset scan: per 4096-value block
  uint64_t* bin_total;     // BYTE_ARRAY: bytes of the decoded values (device, one u64)
  // A required BYTE_ARRAY column whose data pages are all dictionary-encoded and whose dictionary page
  // fits DD_DICT_MAX: its pages take launch_dict_dd (compact ids + chunk byte sums, scan, offsets and
  // bytes); dict_direct = the bytes of its ids in blen (1: u8, 2: u16), 0 for every other column.
  // dd_global: a dictionary too large to stage in LDS (over DD_DICT_MAX bytes or 2,048 entries, at most
  // 65,536 entries: u16 ids): entries and value bytes are gathered from HBM (k_dd_gsums, k_dd_gstr)
  uint32_t dict_direct;
  uint32_t dd_global;
  uint64_t* dict_ent;  // dd_global: entry i = source << 32 | length (k_dent_scatter), one gather per value
};

// Per page, on the device. The host fills the descriptor facts; for nullable
// columns k_levels fills data_begin / n_values and k_scan_offsets fills out_offset (or, in a plan
// running on V2 header null counts, the host fills them too and k_levels verifies them).
struct PageWork {
  uint64_t base;        // page body offset in the batch
  uint32_t size;        // page body bytes
  uint32_t num_slots;   // header num_values
  uint32_t data_begin;  // data section start (page-relative)
  uint32_t n_values;    // non-null values to decode
  uint64_t out_offset;  // first dense value index of the page in its column
  uint64_t slot_offset; // first level slot of the page in its column
  int32_t column;
  int32_t version;
  int32_t rl_encoding;
  int32_t dl_encoding;
  uint32_t rl_len;      // V2
  uint32_t dl_len;      // V2
  // dictionary pages: run records (walk -> tiles)
  uint64_t rec_base;    // first run record of the page
  uint32_t chunk_base;  // first output chunk of the page
  uint32_t aux;         // DELTA_LENGTH_BYTE_ARRAY: start of the value bytes (end of the length stream)
  uint32_t bin_kind;    // BYTE_ARRAY pages: BIN_PLAIN / BIN_DLBA / BIN_DICT (source of the value bytes)
  uint32_t reserved;    // DELTA_BYTE_ARRAY (set by k_delta): 0 chunk-parallel copy, 1 serial copy, 2 carry chain
  uint32_t pflags;      // pqg_page_desc.flags (PQG_PAGE_DBA_CARRY)
  uint32_t pad0;
  uint64_t bin_base;    // PLAIN-only BYTE_ARRAY columns (k_bin_bases): value bytes of the column's earlier pages
};

// Error counter handle passed to every kernel. Error words and the counter are tagged with the
// plan's launch epoch (1..ERR_EPOCH_MAX) instead of being re-initialised each launch: a word
// holds (epoch << 48) | (~key & ERR_KEY_MASK) and is raised with atomicMax, so the newest epoch
// wins and, inside one epoch, the smallest key (index << 8 | code); the counter holds the epoch
// of the last launch that reported. The region is zeroed only when the epoch wraps.
struct ErrCount {
  uint32_t* p;
  uint32_t epoch;
};
constexpr uint32_t ERR_EPOCH_MAX = 0xFFFFu;
constexpr uint64_t ERR_KEY_MASK = (1ull << 48) - 1;

enum BinKind : uint32_t { BIN_PLAIN = 0, BIN_DLBA = 1, BIN_DICT = 2, BIN_DBA = 3 };

// Output chunk of k_dict_expand: CH_TILES x 64 lanes x 16 bytes.
constexpr uint32_t DICT_CHUNK_TILES = 16;
inline uint32_t dict_chunk_values(int elem_width) { return DICT_CHUNK_TILES * 64u * (16u / (uint32_t)elem_width); }
// output chunks of a dictionary page of n slots (slots shifted by up to 16 / width - 1 for 16-B alignment)
inline uint32_t dict_page_chunks(uint32_t n, int elem_width) {
  const uint32_t ch = dict_chunk_values(elem_width);
  return (uint32_t)(((uint64_t)n + (uint32_t)(16 / elem_width) - 1 + ch - 1) / ch);
}
constexpr int DICT_WPB = 4;  // pages (walkers) / chunks (tiles) per workgroup of the dictionary kernels

hipError_t launch_dict(int width, hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                       const ColumnDev* cols, const int32_t* list, int n, uint64_t* rec, uint32_t* chunk_run,
                       const uint64_t* chunks, uint32_t n_chunks, uint64_t* pstat, uint32_t* flags, uint32_t epoch,
                       bool fused, uint64_t* err,
                       ErrCount err_count);
// hint_bad: non-null when the plan runs on V2 header null counts (PQG_PAGE_NULL_COUNT): the host filled
// every listed page's n_values / data_begin / out_offset, k_levels only verifies them and stores
// err_count.epoch to *hint_bad on a mismatch or a level error (no PageWork write); null: level-first
hipError_t launch_levels(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work, const ColumnDev* cols,
                         const int32_t* list, int n, uint64_t* err, ErrCount err_count, uint32_t* hint_bad);
hipError_t launch_scan(hipStream_t st, PageWork* work, const int32_t* col_pages, const int32_t* col_page_start,
                       int n_cols);
hipError_t launch_plain(int kind, hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                        const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count);
hipError_t launch_delta(int width, hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                        const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count);
// dictionary kernels: MODE 0 = values of a 4/8-byte dictionary; MODE 1 = the ids themselves
// (u32, into ColumnDev::blen) for BYTE_ARRAY / FIXED_LEN_BYTE_ARRAY / INT96 dictionaries
hipError_t launch_dict_ids(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const int32_t* list, int n, uint64_t* rec, uint32_t* chunk_run,
                           const uint64_t* chunks, uint32_t n_chunks, uint64_t* pstat, uint32_t* flags,
                           uint32_t epoch, bool fused,
                           uint64_t* err, ErrCount err_count);
// dictionary-direct BYTE_ARRAY columns (ColumnDev::dict_direct): the walk + per-chunk byte sums
// (k_dict_fused_dd, or k_dict_runs + k_dict_tiles_dd in split mode), the per-column scan of the sums
// (k_dd_bases: chunks of column i are sums[dd_start[2i] .. dd_start[2i + 1])), then offsets and value
// bytes (k_dd_str; dd_region = LDS bytes of the staged dictionary page + its u32 entry table)
// global: the columns' dictionaries are gathered from HBM (ColumnDev::dd_global): ids only in the walk's
// expansion, then k_dd_gsums, k_dd_bases, k_dd_gstr
hipError_t launch_dict_dd(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                          const ColumnDev* cols, const int32_t* list, int n, uint64_t* rec, uint32_t* chunk_run,
                          const uint64_t* chunks, uint32_t n_chunks, uint64_t* pstat, uint32_t* flags,
                          uint32_t epoch, bool fused, uint64_t* err, ErrCount err_count, uint64_t* sums,
                          const int32_t* dd_cols, const int32_t* dd_start, int n_dd_cols, uint32_t dd_region,
                          bool global, hipEvent_t entries_ready = nullptr);
// DELTA_LENGTH_BYTE_ARRAY lengths (k_delta into blen, records PageWork::aux)
hipError_t launch_dlba_lengths(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                               const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count);
// pqgpu_snappy.hip: one wave per raw Snappy block (jobs: pqg_snappy_job, device array)
// ZSTD frames per job (pqgpu_zstd.hip): a grid of at most ZSTD_GRID one-wave workgroups loops over
// the jobs; scratch = min(n_jobs, ZSTD_GRID) x ZSTD_LIT_SCRATCH bytes of literal buffers (<= 512 MiB)
constexpr uint64_t ZSTD_LIT_SCRATCH = 131072;
constexpr uint32_t ZSTD_GRID = 4096;
// With seqs / mode (both non-null) the sequences are first decoded one lane per job by k_zstd_seq into
// seqs (8-byte records; job j at dst_offset / 5, so seqs holds dst_bytes / 5 + 1 records) and
// replayed by k_zstd; mode[j] (n_jobs int32) says which jobs the pre-pass left to the inline decoder.
hipError_t launch_zstd(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                       const pqg_snappy_job* jobs, int n_jobs, int32_t* status, uint8_t* scratch, uint64_t* seqs,
                       int32_t* mode);
hipError_t launch_snappy(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                         const void* jobs, int n_jobs, int32_t* status);
hipError_t launch_lz4raw(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                         const void* jobs, int n_jobs, int32_t* status);
// With recs / mode (both non-null) the DEFLATE tokens are first decoded one lane per job by k_gzip_seq
// (literals stored in place, back-references as 8-byte records at dst_offset / 3: recs holds
// dst_bytes / 3 + 2 of them) and replayed by k_gzip_replay; mode[j] (n_jobs int32) = the job's record
// count, or -1 for the jobs left to k_gzip.
// Pages of fewer output bytes than prepass_min skip the token pre-pass (one lane builds a dynamic block's
// Huffman tables serially there; k_gzip's wave builds them in parallel, which small pages, with few
// tokens to share the cost, need): PQG_DISPATCH_GZIP_PREPASS_MIN, default GZ_PREPASS_MIN.
constexpr uint32_t GZ_PREPASS_MIN = 16384;
hipError_t launch_gzip(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                       const void* jobs, int n_jobs, int32_t* status, uint64_t* recs, int32_t* mode,
                       uint32_t prepass_min = GZ_PREPASS_MIN);
// DELTA_BYTE_ARRAY prefix / suffix lengths (k_delta MODE 2: bsrc = prefix, blen = value length, aux;
// dba_meta: per BIN_CHUNK-value chunk {suffix bytes before it, smallest prefix in it};
// PageWork::reserved = 1 when a value is longer than DBA_VB: that page takes the serial copy)
constexpr uint32_t DBA_VB = 2048;  // LDS bytes of one value buffer of the DELTA_BYTE_ARRAY copy
hipError_t launch_dba_lengths(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                              const ColumnDev* cols, const int32_t* list, int n, uint64_t* err, ErrCount err_count,
                              uint32_t* dba_meta);
// DELTA_BYTE_ARRAY value bytes: chunk tails, per-page chain of chunk tails, chunk copies, serial
// copy of the pages with long values, and (carry_cols: one wave per column) the PQG_PAGE_DBA_CARRY
// pages of each column in page order. FIXED_LEN_BYTE_ARRAY columns write value i at i * type_length
// of `values` (dba_off).
hipError_t launch_dba_copy(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const int32_t* list, int n, const uint64_t* chunks,
                           uint32_t n_chunks, const uint32_t* dba_meta, const int32_t* carry_cols, int n_carry_cols,
                           uint64_t* err, ErrCount err_count);
// pqgpu_binary.hip
constexpr uint32_t BIN_CHUNK = 256;     // values per DELTA_BYTE_ARRAY copy chunk
// values per k_bin_copy chunk (one workgroup); A/B on C3 / str_plain / str_dict / C4 (profiles/r03/copy_ab):
// 512 beats 256 (C3 copy 3.65 vs 4.21 ms) and 1,024 (C3 5.73 ms, str_dict 0.80 vs 0.44 ms)
constexpr uint32_t CP_CHUNK_VALUES = 512;
// PLAIN BYTE_ARRAY pages walked in segments of BW_SEG_BYTES (k_bin_walk_seg) when a plan has fewer
// than BW_SEG_MAX_PAGES such pages; BW_SEG_CAP values of scratch per segment (len + src)
constexpr uint32_t BW_SEG_BYTES = 16384;
constexpr uint32_t BW_SEG_CAP = BW_SEG_BYTES / 4 + 2;
constexpr uint32_t BW_SEG_MAX_PAGES = 4096;
constexpr uint32_t SCAN_BLOCK = 4096;   // values per offset-scan block
// dictionary page bytes staged by k_dd_str (dict_direct): 32 KiB since round 5 (8 KiB before; the suite's
// str_dict dictionary, 1,000 entries of 4-32 bytes in 22 KB, then took the per-value path: 0.667 ms, now
// 0.347 ms, profiles/r05/dd32k; k_dd_str's LDS at 32 KiB + the entry table: 4 workgroups per CU)
constexpr uint32_t DD_DICT_MAX = 32768;
hipError_t launch_bss(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work, const ColumnDev* cols,
                      const int32_t* list, int n, uint64_t* err, ErrCount err_count);
// BYTE_ARRAY dictionary pages of at least DENT_MIN bytes: entries walked per 2 KiB tile in parallel
// (k_dent_walk, k_dent_resolve, k_dent_scatter) instead of one wave per page. tiles: column | tile << 32
// (in column order; dictionary dcols[i]'s tiles are [dstart[i], dstart[i + 1])); scratch per tile: rec
// 16 bytes, scr BW_CAP u16, tb 8 bytes
constexpr uint32_t DENT_MIN = 16384;
constexpr uint32_t DENT_TILE = 2048;
constexpr uint32_t DENT_CAP = DENT_TILE / 4;
hipError_t launch_dict_entries(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, const ColumnDev* cols,
                               const uint64_t* tiles, uint32_t n_tiles, const int32_t* dcols, const int32_t* dstart,
                               int n_dcols, uint64_t* rec, uint16_t* scr, uint64_t* tb, int n_pages, uint64_t* err,
                               ErrCount err_count);
hipError_t launch_bin_walk(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const int32_t* list, int n, int dict_walk, int n_pages,
                           uint64_t* err, ErrCount err_count);
// PLAIN-only BYTE_ARRAY columns in one pass: k_bin_bases (one workgroup per column, pages in column
// order in col_pages[col_start[c], col_start[c + 1])) then k_bin_plain over the 2 KiB tiles `segs`
// (page | tile << 32, in column / page / tile order). aggw / incw: per tile, tagged with `epoch`
// (1..255; zeroed when it wraps); ticket: zeroed before the launch; inexact: set to flag_epoch when a
// page's values do not end at its section end (the plan is then re-run on the per-value path).
// per_page (plans with BW_SEG_MAX_PAGES or more PLAIN pages): k_bin_plain_pg, one wave per page of
// col_pages[0, n_pages_total), instead of the tiles.
constexpr uint32_t BP_TILE = 2048;
hipError_t launch_bin_plain(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work, const ColumnDev* cols,
                            const int32_t* col_pages, const int32_t* col_start, int n_cols, const uint64_t* segs,
                            uint32_t n_segs, uint64_t* aggw, uint64_t* incw, uint32_t* ticket, uint32_t epoch,
                            uint32_t* inexact, uint32_t flag_epoch, uint64_t* err, ErrCount err_count,
                            bool per_page, int n_pages_total);
hipError_t launch_bin_walk_seg(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                               const ColumnDev* cols, const uint64_t* segs, uint32_t n_segs, uint64_t* status,
                               uint32_t* ticket, uint32_t* tmp, uint64_t* err, ErrCount err_count);
hipError_t launch_bin_dict_map(hipStream_t st, PageWork* work, const ColumnDev* cols, const int32_t* list, int n);
hipError_t launch_gather_fixed(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                               const ColumnDev* cols, const int32_t* list, int n);
hipError_t launch_bin_scan(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, const ColumnDev* cols,
                           const int32_t* bin_cols, int n_bin_cols,
                           const uint64_t* blocks, uint32_t n_blocks);
hipError_t launch_bin_copy(hipStream_t st, const uint8_t* bytes, uint64_t n_bytes, PageWork* work,
                           const ColumnDev* cols, const uint64_t* chunks, uint32_t n_chunks, uint64_t* err,
                           ErrCount err_count);
// pqgpu_assembly.hip: levels -> offsets / validity of one leaf column's path
constexpr uint32_t ASM_MAX_DEPTHS = 8;  // repetition depths 0..7 (max_rep <= 7)
constexpr uint32_t ASM_MAX_NODES = 16;  // path length
struct AsmParams {
  uint32_t n_nodes;
  uint32_t max_rep;
  uint32_t DR[ASM_MAX_DEPTHS];          // definition level of the r-th REPEATED node (DR[0] = 0)
  int32_t kind[ASM_MAX_NODES];          // pqg_repetition
  uint32_t depth[ASM_MAX_NODES];        // repetition depth of the node's entries
  uint32_t D[ASM_MAX_NODES];            // definition level of the node
  uint8_t* validity[ASM_MAX_NODES];
  int64_t* offsets[ASM_MAX_NODES];
};
hipError_t launch_assemble(hipStream_t st, const uint8_t* def, const uint8_t* rep, uint64_t n, const AsmParams& P,
                           uint64_t* block_counts, uint32_t n_blocks, uint64_t* totals, uint32_t* ticket, int phase);
hipError_t launch_unpack_runs(hipStream_t st, int w, const uint8_t* in, uint64_t in_bytes, const uint64_t* in_off,
                              const uint32_t* counts, const uint64_t* out_off, int32_t* out, int n_runs,
                              uint32_t max_count);

}  // namespace pqg
