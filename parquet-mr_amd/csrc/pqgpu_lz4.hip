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
// One wave per block, sequences taken a 128-byte window of token candidates at a time (the SNAPPY
// kernel's scheme): every lane parses a sequence at each of its 2 byte positions as if a token
// started there (literal-length extension, literals, offset, match-length extension: up to 6
// extension bytes each) and records its successor's window offset; pointer doubling over that
// successor table marks the true chain from the current token; the marked sequences that fit a batch
// of 256 output bytes get their output positions by a wave scan, every output byte its source (a
// literal byte in the 4 KiB LDS segment of the block, or the output position it copies), and the
// batch is resolved as in pqgpu_lzexec.h (pointer jumping over copies of copies, a 4 KiB output ring,
// far matches read back from HBM). A sequence the window path does not take — longer extensions,
// more than 256 output bytes, bytes outside the segment, a malformed header — is decoded on its own
// by the scalar unit and emitted in 64-byte pieces, which also raises every error (all of them
// PQG_ERR_CORRUPT, as aircompressor's MalformedInputException).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"
#include "pqgpu_lzexec.h"

namespace pqg {

constexpr uint32_t L4_SEG = 4096;     // LDS segment of the block
constexpr uint32_t L4_W = 128;        // token candidates per window (2 per lane)
constexpr uint32_t L4_REACH = 2048;   // segment bytes kept past a window for its sequences' literals

struct Lz4JobDev {  // = pqg_snappy_job
  uint64_t src_offset;
  uint64_t dst_offset;
  uint32_t src_size;
  uint32_t dst_size;
};

struct L4Seq {
  uint32_t ls, ll, ml, off, succ;
  bool fast, last;
};

__global__ __launch_bounds__(WAVE) void k_lz4raw(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                                 uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                                 const Lz4JobDev* __restrict__ jobs, int n_jobs,
                                                 int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[LZ_RING];
  __shared__ __attribute__((aligned(16))) uint8_t seg[L4_SEG + 16];
  __shared__ uint8_t sJ[L4_W], sM[L4_W];        // window successor table, chain marks
  __shared__ uint32_t elist[WAVE];               // the window's chain of tokens
  __shared__ uint32_t sS[LZ_CAP];                // source of every output byte of the batch
  __shared__ uint32_t e_src[LZ_EL], e_len[LZ_EL];  // elements of a sequence taken on its own
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
  typedef uint32_t __attribute__((may_alias)) u32a;
  uint32_t lo = 0x80000000u;  // segment = block bytes [lo, lo + L4_SEG)
  auto fill = [&](uint32_t q) {
    lo = uni(q & ~15u);
#pragma unroll
    for (uint32_t i = 0; i < L4_SEG; i += 16u * WAVE) {
      const uint32_t o = i + 16u * lane;
      *(u32x4*)(seg + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + o), 0, 0);
    }
    wave_sync();
  };
  auto read8 = [&](uint32_t q) -> uint64_t {  // block bytes q .. q + 7 from the segment (per lane)
    const uint32_t a = (q - lo) & ~3u, sb = q & 3u;
    const uint32_t x0 = *(const u32a*)(seg + a), x1 = *(const u32a*)(seg + a + 4), x2 = *(const u32a*)(seg + a + 8);
    return ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sb) << 32) | __builtin_amdgcn_alignbyte(x1, x0, sb);
  };
  auto byte_at = [&](uint32_t q) -> uint32_t {  // byte q of the block (uniform q)
    if (q >= lo && q < lo + L4_SEG) return uni((uint32_t)seg[q - lo]);
    return uni((ld32(rs, q & ~3u) >> ((q & 3u) * 8u)) & 0xFFu);
  };
  // length extension in bytes 0..5 of y (LZ4: bytes added while they are 255): count, value
  auto ext6 = [](uint64_t y, uint32_t& nb, uint32_t& add) -> bool {
    const uint64_t ny = ~y & 0x0000FFFFFFFFFFFFull;  // a zero byte: an extension byte of 255
    if (!ny) return false;
    const uint32_t k = (uint32_t)__builtin_ctzll(ny) >> 3;
    nb = k + 1u;
    add = 255u * k + (uint32_t)((y >> (8u * k)) & 0xFFu);
    return true;
  };
  // a sequence at q (per lane, from the segment); fast: the window path takes it
  auto parse = [&](uint32_t q) -> L4Seq {
    L4Seq r;
    const uint64_t x = read8(q);
    const uint32_t t = (uint32_t)x & 0xFFu;
    uint32_t nll = 0, ll = t >> 4;
    bool fast = q < n;
    if (ll == 15u) {
      uint32_t add = 0;
      fast &= ext6(x >> 8, nll, add);
      ll += add;
    }
    r.ls = q + 1u + nll;
    r.ll = ll;
    const uint32_t le = r.ls + ll;
    fast &= r.ls <= n && le <= lo + L4_SEG;
    r.last = fast && le == n;
    r.ml = 0;
    r.off = 0;
    r.succ = le;
    if (!r.last) {
      const bool in = le + 12u <= lo + L4_SEG;
      fast &= in;
      const uint64_t z = read8(in ? le : lo);
      r.off = (uint32_t)z & 0xFFFFu;
      uint32_t nml = 0, ml = t & 15u;
      if (ml == 15u) {
        uint32_t add = 0;
        fast &= ext6(z >> 16, nml, add);
        ml += add;
      }
      r.ml = ml + 4u;
      r.succ = le + 2u + nml;
      fast &= r.succ <= n;
    }
    r.fast = fast;
    return r;
  };
  int code = n == 0u ? PQG_ERR_CORRUPT : 0;  // an empty output is the single byte 0, never no bytes
  uint32_t p = 0, op = 0;
  bool done = false;
  // one sequence at p on its own (any lengths; the reference's checks): literal pieces, then the match
  auto serial_one = [&]() {
    uint32_t q = p;
    const uint32_t token = byte_at(q);
    q++;
    uint32_t ll = token >> 4;
    if (ll == 15u) {
      uint32_t b;
      do {
        if (q >= n) { code = PQG_ERR_CORRUPT; return; }
        b = byte_at(q);
        q++;
        ll += b;
      } while (b == 255u && ll < LZ_LIT);
    }
    if (ll >= LZ_LIT || (uint64_t)q + ll > n || (uint64_t)op + ll > ulen) { code = PQG_ERR_CORRUPT; return; }
    uint32_t lp = q, left = ll;
    q += ll;
    const bool last = q == n;
    uint32_t moff = 0, ml = 0;
    if (!last) {
      if (q + 2u > n) { code = PQG_ERR_CORRUPT; return; }
      moff = byte_at(q) | (byte_at(q + 1u) << 8);
      q += 2u;
      ml = token & 15u;
      if (ml == 15u) {
        uint32_t b;
        do {
          if (q >= n) { code = PQG_ERR_CORRUPT; return; }
          b = byte_at(q);
          q++;
          ml += b;
        } while (b == 255u && ml < LZ_LIT);
      }
      ml += 4u;
      const uint32_t at = op + ll;
      if (moff == 0u || moff > at || ml >= LZ_LIT || (uint64_t)at + ml > ulen) { code = PQG_ERR_CORRUPT; return; }
    }
    uint32_t mleft = ml;
    while (left || mleft) {
      if (left && (lp < lo || lp + LZ_PIECE > lo + L4_SEG)) fill(lp);
      uint32_t m = 0, T = 0;
      while (m < LZ_EL && T < LZ_CAP && (left || mleft)) {
        uint32_t take;
        if (left) {
          take = left < LZ_PIECE ? left : LZ_PIECE;
          take = take < LZ_CAP - T ? take : LZ_CAP - T;
          take = take < lo + L4_SEG - lp ? take : lo + L4_SEG - lp;
          if (take == 0u) break;  // the next round refills the segment at lp
          if (lane == 0) {
            e_src[m] = LZ_LIT | (lp - lo);
            e_len[m] = take;
          }
          lp += take;
          left -= take;
        } else {
          take = mleft < LZ_PIECE ? mleft : LZ_PIECE;
          take = take < LZ_CAP - T ? take : LZ_CAP - T;
          if (lane == 0) {
            e_src[m] = op + T - moff;
            e_len[m] = take;
          }
          mleft -= take;
        }
        T += take;
        m++;
      }
      wave_sync();
      if (m) {
        lz_exec_batch<L4_SEG - 1u>(ring, seg, sS, e_src, e_len, m, T, op, out, ro);
        op += T;
      }
    }
    p = q;
    done = last;
  };
  while (!code && !done) {
    p = uni(p);
    op = uni(op);
    if (p >= n) { code = PQG_ERR_CORRUPT; break; }  // (the block ends with a literals-only sequence)
    const uint32_t B = p & ~1u;  // window [B, B + L4_W): 2 candidates per lane
    if (B < lo || B + L4_W + L4_REACH > lo + L4_SEG) fill(B);
    // ---- every candidate as a token: its successor's window offset (L4_W: leaves the window or ends)
#pragma unroll
    for (uint32_t b = 0; b < 2; b++) {
      const uint32_t q = B + 2u * lane + b;
      const L4Seq r = parse(q);
      const uint32_t j = (!r.fast || r.last || r.succ - B >= L4_W) ? L4_W : r.succ - B;
      sJ[2u * lane + b] = (uint8_t)j;
      sM[2u * lane + b] = q == p ? 1u : 0u;
    }
    wave_sync();
    // ---- pointer doubling marks the chain of tokens from p
    uint32_t jv[2] = {sJ[2u * lane], sJ[2u * lane + 1u]};
#pragma unroll 1
    for (uint32_t r = 0; r < 7; r++) {
      uint32_t jn[2];
      bool more = false;
#pragma unroll
      for (uint32_t b = 0; b < 2; b++)
        if (sM[2u * lane + b] && jv[b] < L4_W) sM[jv[b]] = 1u;
#pragma unroll
      for (uint32_t b = 0; b < 2; b++) jn[b] = jv[b] < L4_W ? sJ[jv[b]] : L4_W;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (uint32_t b = 0; b < 2; b++) {
        jv[b] = jn[b];
        sJ[2u * lane + b] = (uint8_t)jn[b];
      }
      wave_sync();
#pragma unroll
      for (uint32_t b = 0; b < 2; b++) more |= sM[2u * lane + b] && jv[b] < L4_W;
      if (!__ballot(more)) break;
    }
    const uint32_t mk0 = sM[2u * lane], mk1 = sM[2u * lane + 1u];
    uint32_t m;
    const uint32_t eb = wave_excl_scan_u32(mk0 + mk1, &m);
    if (mk0) elist[eb] = B + 2u * lane;
    if (mk1) elist[eb + mk0] = B + 2u * lane + 1u;
    wave_sync();
    m = uni(m);  // >= 1 (p itself); <= 43 (a sequence has >= 3 bytes)
    // ---- the batch: the prefix of fast sequences within LZ_CAP output bytes (lane k: sequence k)
    const uint32_t q = lane < m ? elist[lane] : B;
    const L4Seq r = parse(q);
    const uint32_t tot = r.ll + r.ml;
    const uint64_t cum =
        wave_incl_scan_u64(lane < m && r.fast ? (tot < LZ_CAP + 1u ? tot : LZ_CAP + 1u) : (uint64_t)LZ_CAP + 1u);
    const uint64_t stop = __ballot(lane >= m || !r.fast || cum > LZ_CAP);
    const uint32_t mb = stop ? (uint32_t)__builtin_ctzll(stop) : WAVE;
    if (mb == 0u) {  // the sequence at p on its own
      serial_one();
      continue;
    }
    const bool in = lane < mb;
    uint32_t T;
    const uint32_t ob = wave_excl_scan_u32(in ? tot : 0u, &T);
    T = uni(T);
    const uint32_t at = op + ob + r.ll;  // output position of the match
    const bool valid = !in || ((uint64_t)r.ls + r.ll <= n && (uint64_t)op + ob + tot <= ulen &&
                               (r.last || (r.off != 0u && r.off <= at)));
    if (__ballot(!valid)) { code = PQG_ERR_CORRUPT; break; }
    if (in) {
      const uint32_t l0 = LZ_LIT | (r.ls - lo);
      for (uint32_t i = 0; i < r.ll; i++) sS[ob + i] = l0 + i;
      for (uint32_t i = 0; i < r.ml; i++) sS[ob + r.ll + i] = at + i - r.off;
    }
    wave_sync();
    lz_exec_sources<L4_SEG - 1u>(ring, seg, sS, T, op, out, ro);
    op += T;
    p = uni(rdl(r.succ, mb - 1u));
    done = rdl(r.last ? 1u : 0u, mb - 1u) != 0u;
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
