// pqgpu_lz4.hip — page decompression, codec LZ4_RAW, on gfx950.
//
// Replaces the decompression step of parquet-mr's page reader for LZ4_RAW column chunks:
// ColumnChunkPageReadStore.readPage (parquet-hadoop/.../hadoop/ColumnChunkPageReadStore.java:144-172
// V1, :218-247 V2 data section) -> Lz4RawDecompressor (parquet-hadoop/.../hadoop/codec/
// Lz4RawDecompressor.java:26-50; aircompressor's Lz4Decompressor underneath): one raw LZ4 block per
// page into a buffer of the header's uncompressed size. Format (lz4 doc/lz4_Block_format.md):
// sequences of a token (literal length in the high nibble, match length - 4 in the low one; 15
// continues with bytes added while they are 255), the literals, a 2-byte offset and the match, which
// may overlap its own output; the block ends with literals only. CPU restatement: pqr_lz4_raw_decompress
// (oracle/pqref.c).
//
// One wave per block. The scalar unit parses sequences from an LDS segment of the block into a batch
// of at most 64 elements and 256 output bytes (a literal run or a match, each cut into pieces of at
// most 64 bytes); the batch is then resolved byte by byte as in k_snappy: every output byte gets its
// source (a literal byte in the segment, or the output position it copies), pointer jumping follows
// in-batch copies of copies in log2(depth) rounds, and the bytes come from the segment, a 4 KiB LDS
// ring of the most recent output, or (older) HBM. The ring goes to HBM as aligned dwords.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"
#include "pqgpu_lzexec.h"

namespace pqg {

struct Lz4JobDev {  // = pqg_snappy_job
  uint64_t src_offset;
  uint64_t dst_offset;
  uint32_t src_size;
  uint32_t dst_size;
};

__global__ __launch_bounds__(WAVE) void k_lz4raw(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                                 uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                                 const Lz4JobDev* __restrict__ jobs, int n_jobs,
                                                 int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[LZ_RING];
  __shared__ __attribute__((aligned(16))) uint8_t seg[LZ_SEG];
  __shared__ uint32_t e_src[LZ_EL], e_len[LZ_EL];  // element: source (LZ_LIT | segment offset, or output position), bytes
  __shared__ uint32_t sS[LZ_CAP];                  // source of every output byte of the batch
  const int jb = (int)blockIdx.x;
  if (jb >= n_jobs) return;
  const uint32_t lane = lane_id();
  const Lz4JobDev J = jobs[jb];
  const uint32_t n = uni(J.src_size), ulen = uni(J.dst_size);
  if (J.src_offset + n > src_bytes || J.dst_offset + ulen > dst_bytes || ulen >= LZ_LIT) {
    if (lane == 0 && status) status[jb] = PQG_ERR_INVALID_ARG;
    return;
  }
  const rsrc_t rs = make_rsrc(src + J.src_offset, src_bytes - J.src_offset);
  const rsrc_t ro = make_rsrc(dst + J.dst_offset, dst_bytes - J.dst_offset);  // far matches read the output back
  uint8_t* out = dst + J.dst_offset;
  uint32_t lo = 0x80000000u;  // segment = block bytes [lo, lo + LZ_SEG)
  auto fill = [&](uint32_t q) {
    lo = uni(q & ~15u);
#pragma unroll
    for (uint32_t i = 0; i < LZ_SEG; i += 16u * WAVE) {
      const uint32_t o = i + 16u * lane;
      *(u32x4*)(seg + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + o), 0, 0);
    }
    wave_sync();
  };
  auto in_seg = [&](uint32_t q) { return q >= lo && q < lo + LZ_SEG; };
  int code = n == 0u ? PQG_ERR_CORRUPT : 0;  // an empty output is the single byte 0, never no bytes
  // byte q of the block (uniform q): from the segment, else a buffer load (rare: header bytes past the
  // segment inside a batch, whose literal elements still point into the segment)
  auto byte_at = [&](uint32_t q) -> uint32_t {
    if (in_seg(q)) return uni((uint32_t)seg[q - lo]);
    return uni((ld32(rs, q & ~3u) >> ((q & 3u) * 8u)) & 0xFFu);
  };
  // sequence state (uniform): next header position p; the current sequence's literals still to emit
  // (lit_left at lit_p) and its match (match_left at offset moff; hdr_match: its offset / length not
  // read yet, mnib: the token's match nibble); done: the block's literals-only last sequence was read
  uint32_t p = 0, op = 0, lit_left = 0, lit_p = 0, match_left = 0, moff = 0, mnib = 0;
  bool hdr_match = false, done = false;
  while (!code) {
    // the segment follows the stream between batches (literal elements point into it)
    {
      const uint32_t q = uni(lit_left ? lit_p : p);
      if (q < lo || q + 64u > lo + LZ_SEG) fill(q);
    }
    // ---- a batch of elements (scalar unit): output [op, op + T)
    uint32_t m = 0, T = 0;
    while (m < LZ_EL && T < LZ_CAP) {
      p = uni(p);
      if (lit_left) {
        if (!in_seg(lit_p)) break;  // the next batch refills the segment at lit_p
        uint32_t take = lit_left < LZ_PIECE ? lit_left : LZ_PIECE;
        take = take < LZ_CAP - T ? take : LZ_CAP - T;
        take = take < lo + LZ_SEG - lit_p ? take : lo + LZ_SEG - lit_p;
        if (lane == 0) {
          e_src[m] = LZ_LIT | (lit_p - lo);
          e_len[m] = take;
        }
        lit_p += take;
        lit_left -= take;
        T += take;
        m++;
        continue;
      }
      if (hdr_match) {  // the offset and match length after the literals
        if (p == n) {   // the last sequence: literals only
          done = true;
          hdr_match = false;
          break;
        }
        if (p + 2u > n) { code = PQG_ERR_CORRUPT; break; }
        moff = byte_at(p) | (byte_at(p + 1u) << 8);
        p += 2u;
        uint32_t ml = mnib;
        if (ml == 15u) {
          uint32_t b;
          do {
            if (p >= n) { code = PQG_ERR_CORRUPT; break; }
            b = byte_at(p);
            p++;
            ml += b;
          } while (b == 255u && ml < LZ_LIT);
          if (code) break;
        }
        ml += 4u;
        const uint32_t at = op + T;  // output position of the match
        if (moff == 0u || moff > at || ml >= LZ_LIT || (uint64_t)at + ml > ulen) { code = PQG_ERR_CORRUPT; break; }
        match_left = ml;
        hdr_match = false;
        continue;
      }
      if (match_left) {
        uint32_t take = match_left < LZ_PIECE ? match_left : LZ_PIECE;
        take = take < LZ_CAP - T ? take : LZ_CAP - T;
        if (lane == 0) {
          e_src[m] = op + T - moff;
          e_len[m] = take;
        }
        match_left -= take;
        T += take;
        m++;
        continue;
      }
      // the next sequence: token and literal length
      if (p >= n) { code = PQG_ERR_CORRUPT; break; }
      const uint32_t token = byte_at(p);
      p++;
      uint32_t ll = token >> 4;
      if (ll == 15u) {
        uint32_t b;
        do {
          if (p >= n) { code = PQG_ERR_CORRUPT; break; }
          b = byte_at(p);
          p++;
          ll += b;
        } while (b == 255u && ll < LZ_LIT);
        if (code) break;
      }
      if (ll >= LZ_LIT || (uint64_t)p + ll > n || (uint64_t)op + T + ll > ulen) { code = PQG_ERR_CORRUPT; break; }
      lit_left = ll;
      lit_p = p;
      p += ll;
      mnib = token & 15u;
      hdr_match = true;
    }
    if (code) break;
    m = uni(m);
    T = uni(T);
    wave_sync();
    if (m) {
      lz_exec_batch(ring, seg, sS, e_src, e_len, m, T, op, out, ro);
      op += T;
    }
    if (done && !lit_left && !match_left) break;
  }
  if (!code && op != ulen) code = PQG_ERR_CORRUPT;
  if (lane == 0 && status) status[jb] = code;
}

hipError_t launch_lz4raw(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                         const void* jobs, int n_jobs, int32_t* status) {
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_lz4raw, dim3(n_jobs), dim3(WAVE), 0, st, src, src_bytes, dst, dst_bytes,
                     (const Lz4JobDev*)jobs, n_jobs, status);
  return hipGetLastError();
}

}  // namespace pqg
