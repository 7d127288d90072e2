// pqgpu_snappy.hip — page decompression, codec SNAPPY, on gfx950.
//
// Replaces the decompression step of parquet-mr's page reader: ColumnChunkPageReadStore.readPage
// (parquet-hadoop/.../hadoop/ColumnChunkPageReadStore.java:144-172 V1, :218-247 V2 data section)
// -> SnappyDecompressor (parquet-hadoop/.../hadoop/codec/SnappyDecompressor.java) -> xerial
// Snappy.uncompress: one raw Snappy block per page into a buffer of the header's uncompressed
// size. Format (google/snappy format_description.txt): varint length, then elements — literal
// (tag & 3 == 0) or copy (1-, 2-, 4-byte offset, length 1..64) that may overlap its own output.
//
// One wave per block. The element stream is serial, so the wave parses tags as uniform scalars
// from an LDS segment of the compressed bytes and moves each element's bytes with all lanes:
// literals from the segment, copies from an 8 KiB LDS ring of the most recent output (older
// offsets are read back from the output after a store drain). Each element's tag and its
// length / offset bytes come from ONE 8-byte LDS read. Output bytes go to HBM as produced.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

// LDS per wave (one-wave workgroups): 8 KiB ring + 2 KiB segment -> 16 blocks in flight per CU
constexpr uint32_t SN_RING = 8192;   // LDS window of the most recent output bytes
constexpr uint32_t SN_RMASK = SN_RING - 1;
constexpr uint32_t SN_SEG = 2048;    // LDS segment of the compressed block

struct SnappyJobDev {  // = pqg_snappy_job
  uint64_t src_offset;
  uint64_t dst_offset;
  uint32_t src_size;
  uint32_t dst_size;
};

__global__ __launch_bounds__(WAVE) void k_snappy(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                                 uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                                 const SnappyJobDev* __restrict__ jobs, int n_jobs,
                                                 int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[SN_RING];
  __shared__ __attribute__((aligned(16))) uint8_t seg[SN_SEG];
  const int jb = (int)blockIdx.x;
  if (jb >= n_jobs) return;
  const uint32_t lane = lane_id();
  const SnappyJobDev J = jobs[jb];
  const uint32_t n = uni(J.src_size), ulen_exp = uni(J.dst_size);
  int code = 0;
  if (J.src_offset + n > src_bytes || J.dst_offset + ulen_exp > dst_bytes) {
    if (lane == 0 && status) status[jb] = PQG_ERR_INVALID_ARG;
    return;
  }
  // range-checked views from the job's start to the end of the buffers (a 16-byte load that
  // straddles the end of a range returns 0 as a whole, so the ranges are not cut at the block end;
  // the parser itself never uses bytes past src_size)
  const rsrc_t rs = make_rsrc(src + J.src_offset, src_bytes - J.src_offset);
  const rsrc_t ro = make_rsrc(dst + J.dst_offset, dst_bytes - J.dst_offset);  // far copies read the output back
  uint8_t* out = dst + J.dst_offset;
  uint32_t lo = 0x80000000u;  // segment = block bytes [lo, lo + SN_SEG)
  auto fill = [&](uint32_t p) {
    lo = uni(p & ~15u);
#pragma unroll
    for (uint32_t i = 0; i < SN_SEG; i += 16u * WAVE) {
      const uint32_t o = i + 16u * lane;
      *(u32x4*)(seg + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + o), 0, 0);
    }
    wave_sync();
  };
  // byte p of the block (uniform p)
  auto byte_at = [&](uint32_t p) -> uint32_t {
    if (p < lo || p >= lo + SN_SEG) fill(p);
    return uni(seg[p - lo]);
  };
  typedef uint32_t __attribute__((may_alias)) u32a;
  // bytes p .. p + 7 of the block (uniform p), one LDS round trip
  auto peek8 = [&](uint32_t p) -> uint64_t {
    if (p < lo || p + 12u > lo + SN_SEG) fill(p);
    const uint32_t a = (p - lo) & ~3u, sb = p & 3u;  // lo is 16-aligned
    const uint32_t x0 = *(const u32a*)(seg + a), x1 = *(const u32a*)(seg + a + 4), x2 = *(const u32a*)(seg + a + 8);
    return ((uint64_t)uni(__builtin_amdgcn_alignbyte(x2, x1, sb)) << 32) | uni(__builtin_amdgcn_alignbyte(x1, x0, sb));
  };
  // uncompressed length (varint, <= 32 bits)
  uint32_t p = 0, ulen = 0;
  {
    uint32_t k = 0, b = 0x80u;
    while (k < 5u && (b & 0x80u)) {
      if (p >= n) break;
      b = byte_at(p);
      ulen |= (b & 0x7Fu) << (7u * k);
      p++;
      k++;
    }
    if ((b & 0x80u) || (k == 5u && b > 15u)) code = PQG_ERR_CORRUPT;
  }
  if (!code && ulen != ulen_exp) code = PQG_ERR_CORRUPT;
  uint32_t op = 0;
  while (!code && op < ulen) {
    op = uni(op);
    p = uni(p);
    if (p >= n) { code = PQG_ERR_CORRUPT; break; }
    const uint64_t w8 = peek8(p);  // tag + up to 4 length / offset bytes
    const uint32_t tag = (uint32_t)w8 & 0xFFu;
    const uint32_t x = (uint32_t)(w8 >> 8);  // the 4 bytes after the tag
    p++;
    if ((tag & 3u) == 0u) {  // literal
      uint64_t len = tag >> 2;
      if (len >= 60u) {
        const uint32_t nb = (uint32_t)len - 59u;
        if ((uint64_t)p + nb > n) { code = PQG_ERR_CORRUPT; break; }
        len = nb == 4u ? x : (x & ((1u << (8u * nb)) - 1u));
        p += nb;
      }
      len += 1;
      if ((uint64_t)p + len > n || (uint64_t)op + len > ulen) { code = PQG_ERR_CORRUPT; break; }
      const uint32_t L = (uint32_t)len;
      for (uint32_t done = 0; done < L;) {
        const uint32_t q = uni(p + done);
        if (q < lo || q + 16u > lo + SN_SEG) fill(q);
        uint32_t piece = lo + SN_SEG - q;
        piece = uni(piece < L - done ? piece : L - done);
        for (uint32_t i = lane; i < piece; i += WAVE) {
          const uint8_t b = seg[q - lo + i];
          ring[(op + done + i) & SN_RMASK] = b;
          gst(out + op + done + i, b);
        }
        done += piece;
        __builtin_amdgcn_wave_barrier();
      }
      p += L;
      op += L;
    } else {  // copy
      uint32_t len, off;
      if ((tag & 3u) == 1u) {
        if (p + 1u > n) { code = PQG_ERR_CORRUPT; break; }
        len = 4u + ((tag >> 2) & 7u);
        off = ((tag >> 5) << 8) | (x & 0xFFu);
        p += 1;
      } else if ((tag & 3u) == 2u) {
        if (p + 2u > n) { code = PQG_ERR_CORRUPT; break; }
        len = 1u + (tag >> 2);
        off = x & 0xFFFFu;
        p += 2;
      } else {
        if (p + 4u > n) { code = PQG_ERR_CORRUPT; break; }
        len = 1u + (tag >> 2);
        off = x;
        p += 4;
      }
      if (off == 0u || off > op || (uint64_t)op + len > ulen) { code = PQG_ERR_CORRUPT; break; }
      uint32_t b = 0;
      if (off <= SN_RING - WAVE) {
        // byte op + i = byte op - off + (i mod off): the pattern of the last `off` bytes repeats
        if (lane < len) b = ring[(op - off + (off >= len ? lane : lane % off)) & SN_RMASK];
      } else {
        // older than the ring (off > len here): this wave's own stores, drained, read back
        __builtin_amdgcn_s_waitcnt(0);
        const uint32_t a = op - off + lane;
        const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(a & ~3u), 0, 0);
        b = lane < len ? (w >> ((a & 3u) * 8u)) & 0xFFu : 0u;
      }
      // (the ring positions read, < op, and written, >= op, never alias: off <= SN_RING - 64;
      // LDS operations of one wave complete in order, so the next element reads these writes)
      __builtin_amdgcn_wave_barrier();
      if (lane < len) {
        ring[(op + lane) & SN_RMASK] = (uint8_t)b;
        gst(out + op + lane, (uint8_t)b);
      }
      __builtin_amdgcn_wave_barrier();
      op += len;
    }
  }
  if (lane == 0 && status) status[jb] = code;
}

hipError_t launch_snappy(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                         const void* jobs, int n_jobs, int32_t* status) {
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_snappy, dim3(n_jobs), dim3(WAVE), 0, st, src, src_bytes, dst, dst_bytes,
                     (const SnappyJobDev*)jobs, n_jobs, status);
  return hipGetLastError();
}

}  // namespace pqg
