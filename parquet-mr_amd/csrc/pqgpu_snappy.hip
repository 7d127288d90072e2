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
constexpr uint32_t SN_W = 128;       // window of element starts per batch (<= 64 elements)

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
  __shared__ uint8_t sJ[SN_W], sM[SN_W];  // window successor table, chain marks
  __shared__ uint32_t elist[WAVE];          // the batch's element starts
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
  // Elements are taken a 256-byte window of the compressed block at a time: every lane parses
  // an element header at each of its 4 byte positions (as if an element started there), the
  // true chain of element starts is then followed from the current position with one
  // v_readlane per element, and the batch (<= 64 elements, <= SN_OB output bytes) is executed:
  // literals by their own lanes in parallel (long ones cooperatively), then the copies in order,
  // each by all lanes from the LDS ring.
  uint32_t op = 0;
  auto read8 = [&](uint32_t q) -> uint64_t {  // bytes q .. q + 7 from the segment (per lane)
    const uint32_t a = (q - lo) & ~3u, sb = q & 3u;
    const uint32_t x0 = *(const u32a*)(seg + a), x1 = *(const u32a*)(seg + a + 4), x2 = *(const u32a*)(seg + a + 8);
    return ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sb) << 32) | __builtin_amdgcn_alignbyte(x1, x0, sb);
  };
  // element header at q: header bytes, output length, and (literals) data length
  auto header = [](uint64_t x, uint32_t& hl, uint32_t& olen, uint32_t& off, uint32_t& type) {
    const uint32_t tag = (uint32_t)x & 0xFFu, y = (uint32_t)(x >> 8);
    type = tag & 3u;
    off = 0;
    if (type == 0u) {
      const uint32_t lf = tag >> 2;
      if (lf < 60u) {
        hl = 1u;
        olen = lf + 1u;
      } else {
        const uint32_t nb = lf - 59u;
        hl = 1u + nb;
        const uint32_t v = nb == 4u ? y : (y & ((1u << (8u * nb)) - 1u));
        olen = v == 0xFFFFFFFFu ? 0xFFFFFFFFu : v + 1u;  // (a 2^32-byte literal cannot fit: invalid below)
      }
    } else if (type == 1u) {
      hl = 2u;
      olen = 4u + ((tag >> 2) & 7u);
      off = ((tag >> 5) << 8) | (y & 0xFFu);
    } else if (type == 2u) {
      hl = 3u;
      olen = 1u + (tag >> 2);
      off = y & 0xFFFFu;
    } else {
      hl = 5u;
      olen = 1u + (tag >> 2);
      off = y;
    }
  };
  while (!code && op < ulen) {
    op = uni(op);
    p = uni(p);
    if (p >= n) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t B = p & ~1u;  // window [B, B + SN_W): 2 byte positions per lane
    if (B < lo || B + SN_W + 80u > lo + SN_SEG) fill(B);
    // ---- every position of the window as an element start: its successor's window offset
    uint32_t jv[2];
#pragma unroll
    for (uint32_t b = 0; b < 2; b++) {
      const uint32_t q = B + 2u * lane + b;
      uint32_t hl, olen, off, type;
      header(read8(q), hl, olen, off, type);
      const uint64_t e = (uint64_t)q + hl + (type == 0u ? olen : 0u) - B;
      jv[b] = e < SN_W ? (uint32_t)e : SN_W;
      sJ[2u * lane + b] = (uint8_t)jv[b];
      sM[2u * lane + b] = q == p ? 1u : 0u;
    }
    wave_sync();
    // ---- pointer doubling marks the chain of element starts from p (list ranking: <= 7 rounds
    // of LDS work per window instead of one scalar step per element)
#pragma unroll 1
    for (uint32_t r = 0; r < 7; r++) {
      uint32_t jn[2];
      bool more = false;
#pragma unroll
      for (uint32_t b = 0; b < 2; b++)
        if (sM[2u * lane + b] && jv[b] < SN_W) sM[jv[b]] = 1u;
#pragma unroll
      for (uint32_t b = 0; b < 2; b++) jn[b] = jv[b] < SN_W ? sJ[jv[b]] : SN_W;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t b = 0; b < 2; b++) {
        jv[b] = jn[b];
        sJ[2u * lane + b] = (uint8_t)jn[b];
      }
      wave_sync();
#pragma unroll
      for (uint32_t b = 0; b < 2; b++) more |= sM[2u * lane + b] && jv[b] < SN_W;
      if (!__ballot(more)) break;
    }
    // ---- marked positions in order = the batch's elements (<= 64: an element has >= 2 bytes)
    const uint32_t mk0 = sM[2u * lane], mk1 = sM[2u * lane + 1u];
    uint32_t m;
    const uint32_t eb = wave_excl_scan_u32(mk0 + mk1, &m);
    if (mk0) elist[eb] = B + 2u * lane;
    if (mk1) elist[eb + mk0] = B + 2u * lane + 1u;
    wave_sync();
    m = uni(m);
    // ---- the batch: lane k < m holds element k
    const uint32_t q = lane < m ? elist[lane] : B;
    uint32_t hl, len, off, type;
    header(read8(q), hl, len, off, type);
    if (lane >= m) len = 0;
    uint32_t btot;
    const uint32_t ox = wave_excl_scan_u32(len < 0x80000000u ? len : 0x80000000u, &btot);
    const uint64_t ok = (uint64_t)op + ox;  // output position of the element
    // the stream ends at the element that completes the output (trailing input is ignored) or at
    // the end of the input
    {
      const uint64_t stop = __ballot(lane < m && (q >= n || ok >= ulen));
      if (stop) m = (uint32_t)__builtin_ctzll(stop);
    }
    const bool in = lane < m;
    if (!in) len = 0;
    btot = m ? uni(rdl(ox, m - 1) + rdl(len, m - 1)) : 0u;
    bool valid = true;
    if (in) {
      if (type == 0u) valid = (uint64_t)q + hl + len <= n && ok + len <= ulen;
      else valid = (uint64_t)q + hl <= n && off != 0u && off <= ok && ok + len <= ulen;
    }
    if (__ballot(!valid)) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t cur = m ? uni(rdl(q + hl + (type == 0u ? len : 0u), m - 1)) : p;  // next element start
    const uint64_t bend = (uint64_t)op + btot;  // the ring holds output [bend - SN_RING, bend) once the literals are in
    const uint32_t o32 = (uint32_t)ok;
    uint64_t lm = __ballot(in && type == 0u && len > (uint32_t)WAVE);  // literals over 64 bytes
    // literals of <= 64 bytes: each by its own lane (the data lies inside the segment)
    if (in && type == 0u && len <= (uint32_t)WAVE) {
      const uint32_t s0 = q + hl - lo;
      for (uint32_t i = 0; i < len; i++) {
        const uint8_t v = seg[s0 + i];
        ring[(o32 + i) & SN_RMASK] = v;
        gst(out + o32 + i, v);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // longer literals: all lanes, from refilled segments
    while (lm) {
      const uint32_t k = (uint32_t)__builtin_ctzll(lm);
      lm &= lm - 1;
      const uint32_t L = rdl(len, k), ls = rdl(q + hl, k), lo_out = rdl(o32, k);
      for (uint32_t done = 0; done < L;) {
        const uint32_t qq = uni(ls + done);
        if (qq < lo || qq + 16u > lo + SN_SEG) fill(qq);
        uint32_t piece = lo + SN_SEG - qq;
        piece = uni(piece < L - done ? piece : L - done);
        for (uint32_t i = lane; i < piece; i += WAVE) {
          const uint8_t v = seg[qq - lo + i];
          ring[(lo_out + done + i) & SN_RMASK] = v;
          gst(out + lo_out + done + i, v);
        }
        done += piece;
        __builtin_amdgcn_wave_barrier();
      }
    }
    // copies whose source starts at or after the end of every earlier copy's output read only
    // literal bytes and bytes from before the batch (all in the ring now): each by its own lane,
    // in parallel (an overlapping copy re-reads its own earlier bytes, in order)
    const bool is_copy = in && type != 0u;
    uint32_t pend;
    {
      uint32_t x = is_copy ? o32 + len : 0u;  // inclusive prefix max of the copies' output ends
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d);
        if ((int)lane >= d) x = y > x ? y : x;
      }
      pend = (uint32_t)__shfl_up((int)x, 1);
      if (lane == 0) pend = 0;
    }
    const bool indep = is_copy && (uint64_t)(o32 - off) + SN_RING >= bend + WAVE && o32 - off >= pend;
    if (indep) {
      for (uint32_t i = 0; i < len; i++) {
        const uint8_t v = ring[(o32 - off + i) & SN_RMASK];
        ring[(o32 + i) & SN_RMASK] = v;
        gst(out + o32 + i, v);
      }
    }
    __builtin_amdgcn_wave_barrier();
    // the other copies, in element order, all lanes (ring positions read < o, written >= o: no
    // aliasing while off <= SN_RING - SN_OB - 64; older offsets read the drained output back)
    uint64_t cm = __ballot(is_copy && !indep);
    while (cm) {
      const uint32_t k = (uint32_t)__builtin_ctzll(cm);
      cm &= cm - 1;
      const uint32_t L = rdl(len, k), F = rdl(off, k), O = rdl(o32, k);
      uint32_t v = 0;
      if ((uint64_t)(O - F) + SN_RING >= bend + WAVE) {
        if (lane < L) v = ring[(O - F + (F >= L ? lane : lane % F)) & SN_RMASK];
      } else {
        __builtin_amdgcn_s_waitcnt(0);
        const uint32_t a = O - F + lane;
        const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(a & ~3u), 0, 0);
        v = lane < L ? (w >> ((a & 3u) * 8u)) & 0xFFu : 0u;
      }
      __builtin_amdgcn_wave_barrier();
      if (lane < L) {
        ring[(O + lane) & SN_RMASK] = (uint8_t)v;
        gst(out + O + lane, (uint8_t)v);
      }
      __builtin_amdgcn_wave_barrier();
    }
    op += btot;
    p = cur;
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
