// pqgpu_snappy.hip — page decompression, codec SNAPPY, on gfx950.
//
// Replaces the decompression step of parquet-mr's page reader: ColumnChunkPageReadStore.readPage
// (parquet-hadoop/.../hadoop/ColumnChunkPageReadStore.java:144-172 V1, :218-247 V2 data section)
// -> SnappyDecompressor (parquet-hadoop/.../hadoop/codec/SnappyDecompressor.java) -> xerial
// Snappy.uncompress: one raw Snappy block per page into a buffer of the header's uncompressed
// size. Format (google/snappy format_description.txt): varint length, then elements — literal
// (tag & 3 == 0) or copy (1-, 2-, 4-byte offset, length 1..64) that may overlap its own output.
//
// One wave per block, elements taken a 128-byte window of the compressed bytes (staged in an LDS
// segment) at a time: every lane parses an element header at its 2 byte positions as if an
// element started there, and pointer doubling over the window's successor table marks the true
// chain of element starts. The batch (<= 64 elements, <= 256 output bytes) is then resolved byte
// by byte: every output byte gets its source (a literal byte in the segment, or the output
// position it copies), and pointer jumping follows chains of dependent copies in log2(depth)
// rounds until each source is a literal byte or lies before the batch (in an 4 KiB LDS ring of
// the most recent output, or, older, in HBM). The batch's bytes go to the ring and from there to
// HBM with aligned dword stores; a long literal that ends a batch is streamed to HBM directly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

// LDS per wave (one-wave workgroups): 4 KiB ring + 2 KiB segment + 1 KiB byte sources + 0.5 KiB
// chain tables = 7.7 KiB -> 20 blocks per CU: all 5,000 pages of a 100 M-value chunk at once
constexpr uint32_t SN_RING = 4096;   // LDS window of the most recent output bytes
constexpr uint32_t SN_RMASK = SN_RING - 1;
constexpr uint32_t SN_SEG = 2048;    // LDS segment of the compressed block
constexpr uint32_t SN_W = 128;       // window of element starts per batch (<= 64 elements)
constexpr uint32_t SN_CAP = 256;     // output bytes per batch (a longer first element: a literal, streamed)
constexpr uint32_t SN_LIT = 0x80000000u;  // source tag of a literal byte (| its segment offset)

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
  __shared__ uint32_t sS[SN_CAP];           // source of every output byte of the batch
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
  if (!code && ulen >= SN_LIT) code = PQG_ERR_INVALID_ARG;  // page sizes are int32 (PageHeader)
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
  const u32a* ring32 = (const u32a*)ring;
  // ring bytes of output positions t .. t + 3 (per lane; the ring wraps)
  auto ring4 = [&](uint32_t t) -> uint32_t {
    const uint32_t r = t & SN_RMASK & ~3u;
    return __builtin_amdgcn_alignbyte(ring32[((r + 4u) & SN_RMASK) >> 2], ring32[r >> 2], t & 3u);
  };
  // output [a, e) (uniform, e - a <= SN_RING, all in the ring) to HBM: aligned dwords, bytes at the ends
  const uint32_t oal = (uint32_t)(uintptr_t)out & 3u;
  auto flush = [&](uint32_t a, uint32_t e) {
    const uint32_t base = ((a + oal) & ~3u) - oal;  // out + base is dword aligned (base <= a, may wrap)
    const uint32_t skip = a - base, span = e - base;
    for (uint32_t d0 = 0; d0 < span; d0 += 4u * WAVE) {
      const uint32_t d = d0 + 4u * lane;
      if (d < span) {
        const uint32_t t = base + d, v = ring4(t);
        if (d >= skip && d + 4u <= span) {
          gst((uint32_t*)(out + t), v);
        } else {
#pragma unroll
          for (uint32_t j = 0; j < 4u; j++)
            if (d + j >= skip && d + j < span) gst(out + (t + j), (uint8_t)(v >> (8u * j)));
        }
      }
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
      // at most SN_CAP output bytes (an element longer than that is a literal: a batch of its own)
      const uint64_t over = __ballot(lane < m && lane > 0u && (uint64_t)ox + len > SN_CAP);
      if (over) m = (uint32_t)__builtin_ctzll(over);
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
    const uint32_t o32 = (uint32_t)ok;
    // a literal of over 64 bytes that ends the batch (it may be longer than the ring) goes to HBM
    // straight from the segment; the batch's other output, [op, fend), goes via the ring
    const bool tail_lit = m && rdl(type, m - 1) == 0u && rdl(len, m - 1) > (uint32_t)WAVE;
    const uint32_t fend = tail_lit ? uni(rdl(o32, m - 1)) : uni(op + btot);
    const uint32_t T = fend - op;  // <= SN_CAP
    // ---- the source of every output byte: its literal byte in the segment, or the output position
    // it copies (an overlapping copy's later bytes copy its own earlier ones)
    if (in && !(tail_lit && lane == m - 1)) {
      const uint32_t s0 = type == 0u ? SN_LIT | (q + hl - lo) : o32 - off, b0 = o32 - op;
      for (uint32_t i = 0; i < len; i++) sS[b0 + i] = s0 + i;
    }
    wave_sync();
    // ---- pointer jumping until every source is a literal byte or a byte from before the batch
    // (chains of dependent copies resolve in log2(depth) rounds instead of one copy at a time)
    constexpr uint32_t NB = SN_CAP / WAVE;
    uint32_t sv[NB];
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const uint32_t b = lane + WAVE * j;
      sv[j] = b < T ? sS[b] : SN_LIT;
    }
#pragma unroll 1
    for (uint32_t r = 0; r < 12u; r++) {  // branch-free rounds (the index is clamped to the table)
      bool more = false, hop = false;
#pragma unroll
      for (uint32_t j = 0; j < NB; j++) {
        const bool inb = !(sv[j] & SN_LIT) && sv[j] >= op;
        const uint32_t nv = sS[(sv[j] - op) & (SN_CAP - 1u)];
        sv[j] = inb ? nv : sv[j];
        hop |= inb;
        more |= inb && !(nv & SN_LIT) && nv >= op;
      }
      if (!__ballot(hop)) break;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t j = 0; j < NB; j++) sS[lane + WAVE * j] = sv[j];  // entries >= T hold SN_LIT
      wave_sync();
      if (!__ballot(more)) break;
    }
    // ---- the bytes: literal bytes from the segment, earlier output from the ring, or (older than
    // the ring) from HBM after the earlier batches' stores have drained
    uint32_t bv[NB];
    bool far = false;
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const uint32_t v = sv[j];
      const uint32_t lit = seg[v & (SN_SEG - 1u)], rg = ring[v & SN_RMASK];
      bv[j] = (v & SN_LIT) ? lit : rg;
      far |= !(v & SN_LIT) && (uint64_t)v + SN_RING < (uint64_t)fend + WAVE;
    }
    if (__ballot(far)) {
      __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
      for (uint32_t j = 0; j < NB; j++) {
        const uint32_t v = sv[j];
        if (!(v & SN_LIT) && (uint64_t)v + SN_RING < (uint64_t)fend + WAVE) {
          const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(v & ~3u), 0, 0);
          bv[j] = (w >> ((v & 3u) * 8u)) & 0xFFu;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const uint32_t b = lane + WAVE * j;
      if (b < T) ring[(op + b) & SN_RMASK] = (uint8_t)bv[j];
    }
    wave_sync();
    flush(op, fend);
    if (tail_lit) {  // all lanes, from refilled segments, to the ring and to HBM
      const uint32_t k = m - 1u, L = rdl(len, k), ls = rdl(q + hl, k);
      for (uint32_t done = 0; done < L;) {
        const uint32_t qq = uni(ls + done);
        if (qq < lo || qq + 16u > lo + SN_SEG) fill(qq);
        uint32_t piece = lo + SN_SEG - qq;
        piece = uni(piece < L - done ? piece : L - done);
        for (uint32_t i = lane; i < piece; i += WAVE) {
          const uint8_t v = seg[qq - lo + i];
          ring[(fend + done + i) & SN_RMASK] = v;
          gst(out + fend + done + i, v);
        }
        done += piece;
        __builtin_amdgcn_wave_barrier();
      }
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
