// pqgpu_gzip.hip — page decompression, codec GZIP, on gfx950.
//
// Replaces the decompression step of parquet-mr's page reader for GZIP column chunks:
// ColumnChunkPageReadStore.readPage (parquet-hadoop/.../hadoop/ColumnChunkPageReadStore.java:144-172
// V1, :218-247 V2 data section) -> CodecFactory.HeapBytesDecompressor.decompress
// (parquet-hadoop/.../hadoop/CodecFactory.java:155-182: Hadoop GzipCodec's input stream, read for
// exactly the header's uncompressed size). Format: gzip members (RFC 1952) of DEFLATE data (RFC 1951:
// stored, fixed-Huffman and dynamic-Huffman blocks, back-references up to 32 KiB). CPU restatement:
// pqr_gzip_decompress (oracle/gzip_ref.c), whose semantics this follows: members one after the other,
// reading stops once the page's bytes are produced (the trailer of the member that completes the page
// is not read), a member that ends earlier has its ISIZE checked before the next header.
// A non-final member's CRC-32 is recomputed from the output (gz_member_crc; the token pre-pass hands
// multi-member pages to k_gzip).
//
// One wave per page. The scalar unit runs the bit reader (a 64-bit container refilled 4 bytes at a
// time from an LDS segment of the member) and decodes symbols through 512-entry first-level tables in
// LDS (codes of up to 9 bits in one lookup; longer ones bit by bit from the canonical tables). The
// lanes build the tables of every block (ballots rank the symbols of each code length) and execute the
// output in batches of at most 64 elements / 256 bytes (pqgpu_lzexec.h: literal runs from an LDS
// literal buffer, back-references resolved byte by byte, a 4 KiB output ring, far references read
// back from HBM).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"
#include "pqgpu_lzexec.h"

namespace pqg {

constexpr uint32_t GZ_FAST = 9;  // first-level table bits
constexpr uint32_t GZ_SLOW = 0xFFFFFFFFu;

// First-level table entry (codes of <= 9 bits; longer: GZ_SLOW): symbol | code length << 9, and for a
// length symbol its base << 13 | extra bits << 22, for a distance symbol base << 13 | extra bits << 28
// (no dependent table lookup between a symbol and its extra bits).
__device__ __forceinline__ uint32_t gz_ent_sym(uint32_t e) { return e & 511u; }
__device__ __forceinline__ uint32_t gz_ent_len(uint32_t e) { return (e >> 9) & 15u; }

// Symbol-loop state between calls of gz_symbols (LDS; SGPRs inside the call)
struct GzState {
  uint64_t src, src_len;  // the job's input
  uint64_t bb;            // bit container: bc bits, LSB first; p = next input byte to load
  uint32_t bc, p, lo, n;  // lo: the LDS segment holds input [lo, lo + LZ_SEG)
  uint32_t at, ulen, mstart;  // output position of the batch, page size, member's first output byte
  uint32_t cdist, clen, cfull;  // a match carried into the next batch (cfull: it completes the page)
  uint32_t m, T, res;     // result: elements, bytes; 0 batch full, 1 end of block, 2 page complete, 3 corrupt
};

struct GzLds {
  uint8_t ring[LZ_RING];
  uint8_t lits[LZ_SEG];
  uint8_t seg[LZ_SEG + 16];  // compressed bytes [lo, lo + LZ_SEG)
  uint32_t sS[LZ_CAP];
  uint32_t e_src[LZ_EL], e_len[LZ_EL];
  uint32_t lfast[1u << GZ_FAST], dfast[1u << GZ_FAST];
  uint32_t lentab[32], disttab[32];  // base | extra bits << 16 (length symbols 257.., distance symbols)
  int16_t lcount[16], lsym[320], dcount[16], dsym[32], ccount[16], csym[32];
  uint8_t lens[320 + 32];
  uint8_t ord[20];
  GzState st;
};

__constant__ uint16_t GZ_LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t GZ_LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t GZ_DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                      1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t GZ_DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t GZ_ORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Canonical Huffman tables of lens[0 .. n) (RFC 1951 3.2.2): counts, symbols in canonical order and,
// when `fast`, the first-level table (bit-reversed codes of <= 9 bits). kind 0: literal / length
// table (ext = lentab), 1: distance table (ext = disttab). Returns left (0: complete, > 0: incomplete)
// or -1 (over-subscribed). All lanes.
__device__ int gz_build(const uint8_t* lens, int n, int16_t* count, int16_t* sym, uint32_t* fast, int kind,
                        const uint32_t* ext) {
  const uint32_t lane = lane_id();
  uint32_t cnt[16];
#pragma unroll
  for (int l = 0; l < 16; l++) cnt[l] = 0;
  for (int s0 = 0; s0 < n; s0 += WAVE) {
    const int s = s0 + (int)lane;
    const uint32_t l = s < n ? lens[s] : 0u;
#pragma unroll
    for (int k = 1; k < 16; k++) cnt[k] += (uint32_t)__builtin_popcountll(__ballot(s < n && l == (uint32_t)k));
  }
  int left = 1;
  uint32_t offs[16], code[16];
  offs[1] = 0;
  code[1] = 0;
#pragma unroll
  for (int l = 1; l < 16; l++) {
    left = (left << 1) - (int)cnt[l];
    if (l < 15) {
      offs[l + 1] = offs[l] + cnt[l];
      code[l + 1] = (code[l] + cnt[l]) << 1;
    }
  }
  uint32_t mine = 0;
#pragma unroll
  for (int l = 1; l < 16; l++) mine = lane == (uint32_t)l ? cnt[l] : mine;
  if (lane < 16u) count[lane] = (int16_t)mine;
  if (left < 0) return -1;
  if (fast)
    for (uint32_t i = lane; i < (1u << GZ_FAST); i += WAVE) fast[i] = GZ_SLOW;
  wave_sync();
  uint32_t run[16];
#pragma unroll
  for (int l = 0; l < 16; l++) run[l] = 0;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int s0 = 0; s0 < n; s0 += WAVE) {
    const int s = s0 + (int)lane;
    const uint32_t l = s < n ? lens[s] : 0u;
    uint32_t rank = 0, base_o = 0, base_c = 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
      const uint64_t b = __ballot(s < n && l == (uint32_t)k);
      if (l == (uint32_t)k) {
        rank = run[k] + (uint32_t)__builtin_popcountll(b & lt);
        base_o = offs[k];
        base_c = code[k];
      }
      run[k] += (uint32_t)__builtin_popcountll(b);
    }
    if (s < n && l) {
      sym[base_o + rank] = (int16_t)s;
      if (fast && l <= GZ_FAST) {
        uint32_t e = (uint32_t)s | (l << 9);
        if (kind == 0 && s > 256 && s < 286) {
          const uint32_t t = ext[s - 257];
          e |= ((t & 0x1FFu) << 13) | ((t >> 16) << 22);
        } else if (kind == 1 && s < 30) {
          const uint32_t t = ext[s];
          e |= ((t & 0x7FFFu) << 13) | ((t >> 16) << 28);
        }
        const uint32_t c = base_c + rank;                            // MSB-first code
        const uint32_t rv = __builtin_bitreverse32(c) >> (32u - l);  // as the LSB-first reader sees it
        for (uint32_t k = 0; k < (1u << (GZ_FAST - l)); k++) fast[rv | (k << l)] = e;
      }
    }
  }
  wave_sync();
  return left;
}

// Input segment: bytes [q & ~15, + LZ_SEG) of the job's input into LDS (all lanes).
__device__ __forceinline__ uint32_t gz_fill(GzLds& L, rsrc_t rs, uint32_t q) {
  const uint32_t lo = uni(q & ~15u);
#pragma unroll
  for (uint32_t i = 0; i < LZ_SEG; i += 16u * WAVE) {
    const uint32_t o = i + 16u * lane_id();
    *(u32x4*)(L.seg + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + o), 0, 0);
  }
  wave_sync();
  return lo;
}

// The symbols of a Huffman block, one batch (<= LZ_EL elements, <= LZ_CAP bytes) per call, into
// L.e_src / e_len / lits; L.st.res says why it returned. A function of its own so that its state
// stays in SGPRs (the ZSTD sequence loop's lesson: inlined into the job's code, the uniform state
// was spilled to VGPR lanes). Elements and literal bytes are staged in VGPRs (lane k: element k,
// literal byte k + 64 j) and written to LDS once per batch.
__device__ __attribute__((noinline)) void gz_symbols(GzLds& L) {
  GzState& S = L.st;
  const uint32_t lane = lane_id();
  const rsrc_t rs = make_rsrc((const uint8_t*)uni64(S.src), uni64(S.src_len));
  uint64_t bb = uni64(S.bb);
  uint32_t bc = uni(S.bc), p = uni(S.p), lo = uni(S.lo);
  const uint32_t n = uni(S.n), ulen = uni(S.ulen), mstart = uni(S.mstart), op = uni(S.at);
  const uint64_t nbits = (uint64_t)n * 8u;
  typedef uint32_t __attribute__((aligned(1), may_alias)) u32u;
  uint32_t m = 0, T = 0, res = 0, run = 0;  // run: bytes of the open literal element
  uint32_t es = 0, el = 0, lv0 = 0, lv1 = 0, lv2 = 0, lv3 = 0;
  uint32_t cdist = 0, clen = 0, cfull = 0;
  auto refill = [&]() {
    if (bc <= 32u) {
      if (p < lo || p + 4u > lo + LZ_SEG) lo = gz_fill(L, rs, p);
      uint32_t w = uni(*(const u32u*)(L.seg + (p - lo)));
      if (p + 4u > n) w = p >= n ? 0u : w & (0xFFFFFFFFu >> (8u * (p + 4u - n)));
      bb |= (uint64_t)w << bc;
      bc += 32u;
      p += 4u;
    }
  };
  auto take_bits = [&](uint32_t k) -> uint32_t {  // k <= 15, after a refill
    const uint32_t v = (uint32_t)bb & ((1u << k) - 1u);
    bb >>= k;
    bc -= k;
    return v;
  };
  auto slow = [&](const int16_t* count, const int16_t* sym) -> int {  // codes of 10-15 bits
    int c = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
      c |= (int)take_bits(1);
      const int k = (int)uni((uint32_t)(int32_t)count[l]);
      if (c - k < first) return (int)uni((uint32_t)(int32_t)sym[index + (c - first)]);
      index += k;
      first = (first + k) << 1;
      c <<= 1;
    }
    return -1;
  };
  auto close = [&]() {
    if (run) {
      es = lane == m ? (LZ_LIT | (T - run)) : es;
      el = lane == m ? run : el;
      m++;
      run = 0;
    }
  };
  // a back-reference in pieces of <= LZ_PIECE bytes, as many as the batch holds; returns the rest
  auto put_match = [&](uint32_t dist, uint32_t len) -> uint32_t {
    close();
    while (len && m < LZ_EL && T < LZ_CAP) {
      uint32_t t = len < LZ_PIECE ? len : LZ_PIECE;
      t = t < LZ_CAP - T ? t : LZ_CAP - T;
      es = lane == m ? op + T - dist : es;
      el = lane == m ? t : el;
      m++;
      T += t;
      len -= t;
    }
    return len;
  };
  // (literal bytes sit at their batch offset: lits[T] for the byte of output op + T)
  if (uni(S.clen)) {
    const uint32_t d = uni(S.cdist), f = uni(S.cfull);
    const uint32_t rest = put_match(d, uni(S.clen));
    if (rest) {
      cdist = d;
      clen = rest;
      cfull = f;
    } else if (f) {
      res = 2;
    }
  }
  if (!clen && res == 0) {
    while (true) {
      if (m + (run ? 1u : 0u) >= LZ_EL || T >= LZ_CAP) break;  // batch full
      refill();
      uint32_t e = uni(L.lfast[(uint32_t)bb & ((1u << GZ_FAST) - 1u)]);
      uint32_t sym;
      if (e != GZ_SLOW) {
        const uint32_t l = gz_ent_len(e);
        bb >>= l;
        bc -= l;
        sym = gz_ent_sym(e);
      } else {
        refill();
        const int s = slow(L.lcount, L.lsym);
        if (s < 0) { res = 3; break; }
        sym = (uint32_t)s;
        e = sym < 257u || sym > 285u ? sym : sym | ((uni(L.lentab[sym - 257u]) & 0x1FFu) << 13) |
                                                   ((uni(L.lentab[sym - 257u]) >> 16) << 22);
      }
      if ((uint64_t)p * 8u - bc > nbits) { res = 3; break; }
      if (sym < 256u) {
        if (op + T >= ulen) { res = 2; break; }
        if (run == LZ_PIECE) close();
        const uint32_t j = T >> 6;
        const bool me = lane == (T & 63u);
        lv0 = me && j == 0 ? sym : lv0;
        lv1 = me && j == 1 ? sym : lv1;
        lv2 = me && j == 2 ? sym : lv2;
        lv3 = me && j == 3 ? sym : lv3;
        T++;
        run++;
        continue;
      }
      if (sym == 256u) { res = 1; break; }
      if (sym > 285u) { res = 3; break; }
      refill();
      uint32_t len = ((e >> 13) & 0x1FFu) + take_bits((e >> 22) & 7u);
      uint32_t d = uni(L.dfast[(uint32_t)bb & ((1u << GZ_FAST) - 1u)]);
      if (d != GZ_SLOW) {
        const uint32_t l = gz_ent_len(d);
        bb >>= l;
        bc -= l;
      } else {
        const int s = slow(L.dcount, L.dsym);
        if (s < 0 || s >= 30) { res = 3; break; }
        const uint32_t t = uni(L.disttab[s]);
        d = (uint32_t)s | ((t & 0x7FFFu) << 13) | ((t >> 16) << 28);
      }
      if (gz_ent_sym(d) >= 30u) { res = 3; break; }
      refill();
      const uint32_t dist = ((d >> 13) & 0x7FFFu) + take_bits(d >> 28);
      if ((uint64_t)p * 8u - bc > nbits) { res = 3; break; }
      const uint32_t at = op + T;
      if (dist > at - mstart) { res = 3; break; }
      uint32_t full = 0;
      if (len > ulen - at) {  // the page completes inside this match
        len = ulen - at;
        full = 1;
      }
      const uint32_t rest = len ? put_match(dist, len) : 0u;
      if (rest) {
        cdist = dist;
        clen = rest;
        cfull = full;
        break;
      }
      if (full) { res = 2; break; }
    }
  }
  close();
  // literal bytes at their batch offsets, elements in lanes
  if (lane < T) L.lits[lane] = (uint8_t)lv0;
  if (lane + 64u < T) L.lits[lane + 64u] = (uint8_t)lv1;
  if (lane + 128u < T) L.lits[lane + 128u] = (uint8_t)lv2;
  if (lane + 192u < T) L.lits[lane + 192u] = (uint8_t)lv3;
  if (lane < m) {
    L.e_src[lane] = es;
    L.e_len[lane] = el;
  }
  if (lane == 0) {
    S.bb = bb; S.bc = bc; S.p = p; S.lo = lo;
    S.cdist = cdist; S.clen = clen; S.cfull = cfull;
    S.m = m; S.T = T; S.res = res;
  }
  wave_sync();
}

struct GzJobDev {  // = pqg_snappy_job
  uint64_t src_offset;
  uint64_t dst_offset;
  uint32_t src_size;
  uint32_t dst_size;
};

// CRC-32 (RFC 1952 8; reflected polynomial 0xEDB88320) of output bytes [b, e) through `ro`, after this
// wave's stores: lane l takes a contiguous piece bit by bit, the pieces are joined in order with
// crc(A B) = (crc(A) * x^(8|B|) mod P) ^ crc(B) (GF(2) arithmetic of zlib's crc32_combine). Only for
// members that end before the page (rare: multi-member pages), so plain loops.
__device__ __forceinline__ uint32_t gz_mulmodp(uint32_t a, uint32_t b) {
  uint32_t pr = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) pr ^= b;
    b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return pr;
}
__device__ __forceinline__ uint32_t gz_x8n(uint32_t n) {  // x^(8n) mod P
  uint32_t r = 1u << 31, pw = 1u << 23;                    // x^0, x^8
  for (; n; n >>= 1) {
    if (n & 1u) r = gz_mulmodp(pw, r);
    pw = gz_mulmodp(pw, pw);
  }
  return r;
}
__device__ uint32_t gz_member_crc(rsrc_t ro, uint32_t b, uint32_t e) {
  __builtin_amdgcn_s_waitcnt(0);
  const uint32_t lane = lane_id(), len = e - b, S = (len + WAVE - 1u) / WAVE;
  const uint32_t lb = b + (lane * S < len ? lane * S : len), le = b + ((lane + 1u) * S < len ? (lane + 1u) * S : len);
  uint32_t c = 0xFFFFFFFFu;
  for (uint32_t q = lb; q < le; q++) {
    c ^= (__builtin_amdgcn_raw_buffer_load_b32(ro, (int)(q & ~3u), 0, 0) >> ((q & 3u) * 8u)) & 0xFFu;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
  }
  c ^= 0xFFFFFFFFu;
  uint32_t tot = 0;
  const uint32_t xs = gz_x8n(S);
  for (uint32_t l = 0; l < WAVE; l++) {
    const uint32_t cl = uni(__builtin_amdgcn_readlane(c, l));
    const uint32_t n_l = l * S < len ? ((l + 1u) * S < len ? S : len - l * S) : 0u;
    if (n_l) tot = gz_mulmodp(n_l == S ? xs : gz_x8n(n_l), tot) ^ cl;
  }
  return tot;
}

__global__ __launch_bounds__(WAVE) void k_gzip(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                               uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                               const GzJobDev* __restrict__ jobs, int n_jobs,
                                               int32_t* __restrict__ status, const int32_t* __restrict__ mode) {
  __shared__ __attribute__((aligned(16))) GzLds L;
  const int jb = (int)blockIdx.x;
  if (jb >= n_jobs) return;
  if (mode && mode[jb] >= 0) return;  // decoded by the token pre-pass (k_gzip_seq + k_gzip_replay)
  const uint32_t lane = lane_id();
  const GzJobDev J = jobs[jb];
  const uint32_t n = uni(J.src_size), ulen = uni(J.dst_size);
  if (J.src_offset + n > src_bytes || J.dst_offset + ulen > dst_bytes || ulen >= LZ_LIT) {
    if (lane == 0 && status) status[jb] = PQG_ERR_INVALID_ARG;
    return;
  }
  const rsrc_t rs = make_rsrc(src + J.src_offset, src_bytes - J.src_offset);
  const rsrc_t ro = make_rsrc(dst + J.dst_offset, dst_bytes - J.dst_offset);
  uint8_t* out = dst + J.dst_offset;
  const uint64_t nbits = (uint64_t)n * 8u;
  // length / distance bases and extra bits, and the code-length order, in LDS (a __constant__
  // table indexed per symbol is a vector memory load whose wait also waits for the output stores)
  if (lane < 29u) L.lentab[lane] = GZ_LBASE[lane] | ((uint32_t)GZ_LEXT[lane] << 16);
  if (lane < 30u) L.disttab[lane] = GZ_DBASE[lane] | ((uint32_t)GZ_DEXT[lane] << 16);
  if (lane < 19u) L.ord[lane] = GZ_ORD[lane];
  if (lane == 0) {
    L.st.src = (uint64_t)(uintptr_t)(src + J.src_offset);
    L.st.src_len = src_bytes - J.src_offset;
    L.st.n = n;
    L.st.ulen = ulen;
  }
  wave_sync();
  uint32_t lo = 0x80000000u;  // segment = input bytes [lo, lo + LZ_SEG)
  auto byte_at = [&](uint32_t q) -> uint32_t {  // byte q of the input (0 past its end)
    return q < n ? uni((ld32(rs, q & ~3u) >> ((q & 3u) * 8u)) & 0xFFu) : 0u;
  };
  // bit reader of the block headers and code lengths (the symbol loop has its own, in gz_symbols):
  // bytes past n read as 0; reading past the input shows as consumed() > nbits
  uint32_t p = 0, bc = 0;
  uint64_t bb = 0;
  typedef uint32_t __attribute__((aligned(1), may_alias)) u32u;
  auto refill = [&]() {
    while (bc <= 32u) {
      if (p < lo || p + 4u > lo + LZ_SEG) lo = gz_fill(L, rs, p);
      uint32_t w = uni(*(const u32u*)(L.seg + (p - lo)));
      if (p + 4u > n) w = p >= n ? 0u : w & (0xFFFFFFFFu >> (8u * (p + 4u - n)));
      bb |= (uint64_t)w << bc;
      bc += 32u;
      p += 4u;
    }
  };
  auto consumed = [&]() -> uint64_t { return (uint64_t)p * 8u - bc; };
  auto bits = [&](uint32_t k) -> uint32_t {  // k <= 32
    refill();
    const uint32_t v = (uint32_t)(bb & ((1ull << k) - 1ull));
    bb >>= k;
    bc -= k;
    return v;
  };
  auto restart = [&](uint32_t q) {  // the reader continues at byte q
    p = q;
    bb = 0;
    bc = 0;
  };
  auto decode_slow = [&](const int16_t* count, const int16_t* sym) -> int {
    int c = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
      c |= (int)bits(1);
      const int k = (int)uni((uint32_t)(int32_t)count[l]);
      if (c - k < first) return (int)uni((uint32_t)(int32_t)sym[index + (c - first)]);
      index += k;
      first = (first + k) << 1;
      c <<= 1;
    }
    return -1;
  };

  uint32_t op = 0;  // output bytes written
  auto exec = [&](uint32_t m, uint32_t T) {
    if (m) {
      lz_exec_batch(L.ring, L.lits, L.sS, L.e_src, L.e_len, m, T, op, out, ro);
      op += T;
    }
  };
  int code = 0;
  bool full = false;  // a symbol past the page's size was decoded: reading stops there
  uint32_t q = 0;     // byte position of the next member
  while (!code && op < ulen) {
    // ---- member header (RFC 1952 2.3)
    if (q >= n) { code = PQG_ERR_EOF; break; }  // the stream ends before the page's size
    if (q + 10u > n) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t flg = byte_at(q + 3u);
    if (byte_at(q) != 0x1fu || byte_at(q + 1u) != 0x8bu || byte_at(q + 2u) != 8u || (flg & 0xE0u)) {
      code = PQG_ERR_CORRUPT;
      break;
    }
    q += 10u;
    if (flg & 4u) {
      if (q + 2u > n) { code = PQG_ERR_CORRUPT; break; }
      q += 2u + (byte_at(q) | (byte_at(q + 1u) << 8));
    }
    if (flg & 8u) { while (q < n && byte_at(q)) q++; q++; }
    if (flg & 16u) { while (q < n && byte_at(q)) q++; q++; }
    if (flg & 2u) q += 2u;
    if (q > n) { code = PQG_ERR_CORRUPT; break; }
    restart(q);
    const uint32_t member_start = op;
    // ---- DEFLATE blocks (RFC 1951 3.2.3)
    uint32_t last = 0;
    do {
      last = bits(1);
      const uint32_t type = bits(2);
      if (consumed() > nbits) { code = PQG_ERR_CORRUPT; break; }
      if (type == 0u) {  // stored: LEN, NLEN at the next byte boundary, then LEN bytes
        const uint32_t at = (uint32_t)((consumed() + 7u) >> 3);
        if (at + 4u > n) { code = PQG_ERR_CORRUPT; break; }
        const uint32_t len = byte_at(at) | (byte_at(at + 1u) << 8), nlen = byte_at(at + 2u) | (byte_at(at + 3u) << 8);
        if (len != (~nlen & 0xFFFFu) || at + 4u + len > n) { code = PQG_ERR_CORRUPT; break; }
        uint32_t s = at + 4u, left = len;
        while (left) {  // up to 256 bytes a batch, straight into the literal buffer
          if (op >= ulen) { full = true; break; }
          uint32_t take = left < LZ_CAP ? left : LZ_CAP;
          take = take < ulen - op ? take : ulen - op;
          for (uint32_t i = lane; i < take; i += WAVE) {
            const uint32_t b = s + i;
            L.lits[i] = (uint8_t)(ld32(rs, b & ~3u) >> ((b & 3u) * 8u));
          }
          const uint32_t m = (take + LZ_PIECE - 1u) / LZ_PIECE;
          if (lane < m) {
            L.e_src[lane] = LZ_LIT | (lane * LZ_PIECE);
            L.e_len[lane] = take - lane * LZ_PIECE < LZ_PIECE ? take - lane * LZ_PIECE : LZ_PIECE;
          }
          wave_sync();
          exec(m, take);
          s += take;
          left -= take;
        }
        restart(at + 4u + len);
        continue;
      }
      if (type == 3u) { code = PQG_ERR_CORRUPT; break; }
      if (type == 1u) {  // fixed codes (RFC 1951 3.2.6)
        for (uint32_t s = lane; s < 288u + 30u; s += WAVE)
          L.lens[s] = s < 144u ? 8 : s < 256u ? 9 : s < 280u ? 7 : s < 288u ? 8 : 5;
        wave_sync();
        gz_build(L.lens, 288, L.lcount, L.lsym, L.lfast, 0, L.lentab);
        gz_build(L.lens + 288, 30, L.dcount, L.dsym, L.dfast, 1, L.disttab);
      } else {  // dynamic codes (RFC 1951 3.2.7)
        const uint32_t nlen = bits(5) + 257u, ndist = bits(5) + 1u, ncode = bits(4) + 4u;
        if (nlen > 286u || ndist > 30u) { code = PQG_ERR_CORRUPT; break; }
        if (lane < 19u) L.lens[lane] = 0;
        wave_sync();
        for (uint32_t i = 0; i < ncode; i++) {
          const uint32_t v = bits(3);
          if (lane == 0) L.lens[L.ord[i]] = (uint8_t)v;
        }
        wave_sync();
        if (consumed() > nbits || gz_build(L.lens, 19, L.ccount, L.csym, nullptr, 0, nullptr) != 0) {
          code = PQG_ERR_CORRUPT;
          break;
        }
        // the literal / length and distance code lengths (lens[0 .. 19) is free again: the
        // code-length code lives in ccount / csym)
        uint32_t idx = 0;
        while (idx < nlen + ndist) {
          const int sym = decode_slow(L.ccount, L.csym);
          if (sym < 0) { code = PQG_ERR_CORRUPT; break; }
          if (sym < 16) {
            if (lane == 0) L.lens[idx] = (uint8_t)sym;
            idx++;
          } else {
            uint32_t rep, val = 0;
            if (sym == 16) {
              if (idx == 0) { code = PQG_ERR_CORRUPT; break; }
              val = uni((uint32_t)L.lens[idx - 1u]);
              rep = 3u + bits(2);
            } else if (sym == 17) {
              rep = 3u + bits(3);
            } else {
              rep = 11u + bits(7);
            }
            if (idx + rep > nlen + ndist) { code = PQG_ERR_CORRUPT; break; }
            for (uint32_t k = lane; k < rep; k += WAVE) L.lens[idx + k] = (uint8_t)val;
            idx += rep;
          }
          wave_sync();
        }
        if (!code && consumed() > nbits) code = PQG_ERR_CORRUPT;
        if (code) break;
        wave_sync();
        if (uni((uint32_t)L.lens[256]) == 0u) { code = PQG_ERR_CORRUPT; break; }  // no end-of-block code
        // the distance lengths move from nlen to 288 (both tables built from lens)
        const uint32_t dl = lane < ndist ? L.lens[nlen + lane] : 0u;
        wave_sync();
        if (lane < 32u) L.lens[288u + lane] = (uint8_t)dl;
        wave_sync();
        // incomplete codes only when a single symbol is used (zlib's rule; pqr_gzip_decompress)
        const int e1 = gz_build(L.lens, (int)nlen, L.lcount, L.lsym, L.lfast, 0, L.lentab);
        uint32_t used = 0;
        for (int l = 1; l < 16; l++) used += uni((uint32_t)(int32_t)L.lcount[l]);
        if (e1 < 0 || (e1 > 0 && used != 1u)) { code = PQG_ERR_CORRUPT; break; }
        const int e2 = gz_build(L.lens + 288, (int)ndist, L.dcount, L.dsym, L.dfast, 1, L.disttab);
        used = 0;
        for (int l = 1; l < 16; l++) used += uni((uint32_t)(int32_t)L.dcount[l]);
        if (e2 < 0 || (e2 > 0 && used > 1u)) { code = PQG_ERR_CORRUPT; break; }
      }
      // ---- the block's symbols, a batch per gz_symbols call
      if (lane == 0) {
        L.st.bb = bb; L.st.bc = bc; L.st.p = p; L.st.lo = lo;
        L.st.mstart = member_start; L.st.clen = 0;
      }
      uint32_t res = 0;
      do {
        if (lane == 0) L.st.at = op;
        wave_sync();
        gz_symbols(L);
        res = uni(L.st.res);
        if (res == 3u) { code = PQG_ERR_CORRUPT; break; }
        exec(uni(L.st.m), uni(L.st.T));
      } while (res == 0u);
      bb = uni64(L.st.bb);
      bc = uni(L.st.bc);
      p = uni(L.st.p);
      lo = uni(L.st.lo);
      if (res == 2u) full = true;
    } while (!code && !full && !last);
    if (code || full || op >= ulen) break;  // complete: the trailer is not read
    // ---- trailer of a member that ends before the page is complete: CRC-32 and ISIZE
    const uint32_t at = (uint32_t)((consumed() + 7u) >> 3);
    if (at + 8u > n) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t crc = byte_at(at) | (byte_at(at + 1u) << 8) | (byte_at(at + 2u) << 16) | (byte_at(at + 3u) << 24);
    const uint32_t isz = byte_at(at + 4u) | (byte_at(at + 5u) << 8) | (byte_at(at + 6u) << 16) | (byte_at(at + 7u) << 24);
    if (isz != op - member_start) { code = PQG_ERR_CORRUPT; break; }
    if (gz_member_crc(ro, member_start, op) != crc) { code = PQG_ERR_CORRUPT; break; }
    q = at + 8u;
  }
  if (!code && op != ulen) code = PQG_ERR_EOF;
  if (lane == 0 && status) status[jb] = code;
}

// ---- Token pre-pass (k_gzip_seq): one LANE per page ------------------------------------------------
// The symbol loop above is a serial scalar chain per page whose issue the CU's one scalar unit shares
// among its waves (the round-3 ZSTD diagnosis). Here every lane decodes the DEFLATE tokens of its own
// page with vector instructions (12 pages per workgroup): Huffman tables per block in the lane's LDS
// slice (first-level table of 512 entries carrying length / distance bases and extra bits, canonical
// counts for longer codes), the input through a 512-byte LDS window re-centred collectively (all lanes
// of the token loop together), literal bytes stored straight to their output positions, and each
// back-reference as an 8-byte record {output position:32, distance:16, length:16} (job j's records at
// dst_offset / 3). k_gzip_replay then executes the records in 189-byte output windows with the shared
// executor (literal bytes read back from the output). Anything else — a malformed stream, a page that
// completes inside a member, more records than the job's range, a stream past 4 GiB — is left to
// k_gzip, which reports exactly what it always did.
constexpr uint32_t GQ_JOBS = 12;
constexpr uint32_t GQ_WIN = 512;
constexpr int32_t GQ_INLINE = -1;  // mode[j]: -1 = k_gzip decodes job j, else its record count


struct GqLane {
  uint8_t win[GQ_WIN + 16];  // input bytes [wlo, wlo + GQ_WIN) (offsets into src)
  uint32_t lfast[1u << GZ_FAST], dfast[1u << GZ_FAST];
  int16_t lcount[16], lsym[288], dcount[16], dsym[32];
  uint16_t offs[16], next[16];
  uint8_t lens[320 + 32];
};
struct GqLds {
  GqLane l[GQ_JOBS];
  uint32_t lentab[32], disttab[32];
  uint8_t ord[20];
};

// Canonical tables of lens[0 .. n) for one lane (serial): as gz_build, returns left (0 complete,
// > 0 incomplete) or -1 (over-subscribed)
__device__ int gq_build(GqLane& T, const uint8_t* lens, int n, int16_t* count, int16_t* sym, uint32_t* fast, int kind,
                        const uint32_t* ext) {
  for (int l = 0; l < 16; l++) count[l] = 0;
  for (int s = 0; s < n; s++) count[lens[s]]++;
  count[0] = 0;
  int left = 1;
  T.offs[1] = 0;
  T.next[1] = 0;
  for (int l = 1; l < 16; l++) {
    left = (left << 1) - count[l];
    if (left < 0) return -1;
    if (l < 15) {
      T.offs[l + 1] = (uint16_t)(T.offs[l] + count[l]);
      T.next[l + 1] = (uint16_t)((T.next[l] + count[l]) << 1);
    }
  }
  for (uint32_t i = 0; i < (1u << GZ_FAST); i++) fast[i] = GZ_SLOW;
  for (int s = 0; s < n; s++) {
    const uint32_t l = lens[s];
    if (!l) continue;
    sym[T.offs[l]++] = (int16_t)s;
    const uint32_t c = T.next[l]++;
    if (l <= GZ_FAST) {
      uint32_t e = (uint32_t)s | (l << 9);
      if (kind == 0 && s > 256 && s < 286) {
        const uint32_t t = ext[s - 257];
        e |= ((t & 0x1FFu) << 13) | ((t >> 16) << 22);
      } else if (kind == 1 && s < 30) {
        const uint32_t t = ext[s];
        e |= ((t & 0x7FFFu) << 13) | ((t >> 16) << 28);
      }
      const uint32_t rv = __builtin_bitreverse32(c) >> (32u - l);
      for (uint32_t k = 0; k < (1u << (GZ_FAST - l)); k++) fast[rv | (k << l)] = e;
    }
  }
  return left;
}

// canonical decode of the code at the bottom of x (LSB first, MSB-first code); returns the symbol
// (its length in *len) or -1
__device__ __forceinline__ int gq_slow(uint64_t x, const int16_t* count, const int16_t* sym, uint32_t* len) {
  int c = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    c |= (int)((x >> (l - 1)) & 1u);
    const int k = count[l];
    if (c - k < first) {
      *len = (uint32_t)l;
      return sym[index + (c - first)];
    }
    index += k;
    first = (first + k) << 1;
    c <<= 1;
  }
  return -1;
}

__device__ int32_t gq_job(GqLds& L, GqLane& T, rsrc_t rs, const GzJobDev& J, uint8_t* dst, uint64_t* recs) {
  if (J.src_offset + J.src_size + 16u >= 0xFFFFFF00ull || J.dst_size == 0u || J.dst_size >= (1u << 31))
    return GQ_INLINE;
  const uint32_t so = (uint32_t)J.src_offset, n = J.src_size, ulen = J.dst_size;
  const uint64_t endbit = ((uint64_t)so + n) * 8u;
  uint8_t* out = dst + J.dst_offset;
  const uint64_t rbase = J.dst_offset / 3u;
  const uint32_t rcap = (uint32_t)((J.dst_offset + J.dst_size) / 3u - rbase);
  uint64_t* rec = recs + rbase;
  typedef uint32_t __attribute__((may_alias)) u32a;
  uint32_t wlo = 0xFFFFFFFFu;
  // the token loop re-centres once bp >= rthr (fewer than 24 window bytes left above bp; bp only
  // grows and every window starts at or below the position it was centred for)
  uint64_t rthr = 0;
  auto recenter = [&](uint32_t byte) {
    wlo = byte & ~15u;
    rthr = ((uint64_t)wlo + GQ_WIN - 23u) * 8u;
#pragma unroll
    for (uint32_t o = 0; o < GQ_WIN; o += 16)
      *(u32x4*)(T.win + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(wlo + o), 0, 0);
  };
  auto peek = [&](uint64_t b) -> uint64_t {  // 64 input bits from bit b (window must hold them)
    const uint32_t byte = (uint32_t)(b >> 3);
    const uint32_t rel = byte - wlo, r4 = rel & ~3u, sh = (rel & 3u) * 8u + (uint32_t)(b & 7u);
    const uint32_t d0 = *(const u32a*)(T.win + r4), d1 = *(const u32a*)(T.win + r4 + 4), d2 = *(const u32a*)(T.win + r4 + 8);
    return (uint64_t)__builtin_amdgcn_alignbit(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32);
  };
  auto ensure = [&](uint64_t b) {  // the window holds the 8 bytes from bit b (single lane)
    const uint32_t byte = (uint32_t)(b >> 3);
    if (wlo == 0xFFFFFFFFu || byte < wlo || byte + 12u > wlo + GQ_WIN) recenter(byte);
  };
  uint64_t bp = 0;
  auto bits = [&](uint32_t k) -> uint32_t {  // k <= 32
    ensure(bp);
    const uint32_t v = (uint32_t)(peek(bp) & ((1ull << k) - 1ull));
    bp += k;
    return v;
  };
  auto byte_at = [&](uint32_t q) -> uint32_t {  // byte q of the job's input (absolute offset so + q)
    return (ld32(rs, (so + q) & ~3u) >> (((so + q) & 3u) * 8u)) & 0xFFu;
  };
  uint32_t op = 0, cnt = 0, q = 0;
  while (op < ulen) {
    // member header (RFC 1952 2.3)
    if (q + 10u > n) return GQ_INLINE;
    const uint32_t flg = byte_at(q + 3u);
    if (byte_at(q) != 0x1fu || byte_at(q + 1u) != 0x8bu || byte_at(q + 2u) != 8u || (flg & 0xE0u)) return GQ_INLINE;
    q += 10u;
    if (flg & 4u) {
      if (q + 2u > n) return GQ_INLINE;
      q += 2u + (byte_at(q) | (byte_at(q + 1u) << 8));
    }
    if (flg & 8u) { while (q < n && byte_at(q)) q++; q++; }
    if (flg & 16u) { while (q < n && byte_at(q)) q++; q++; }
    if (flg & 2u) q += 2u;
    if (q > n) return GQ_INLINE;
    bp = ((uint64_t)so + q) * 8u;
    const uint32_t mstart = op;
    uint32_t last = 0;
    do {
      last = bits(1);
      const uint32_t type = bits(2);
      if (bp > endbit || type == 3u) return GQ_INLINE;
      if (type == 0u) {  // stored
        bp = (bp + 7u) & ~7ull;
        const uint32_t len = bits(16), nlen = bits(16);
        const uint32_t at = (uint32_t)(bp >> 3) - so;
        if (len != (~nlen & 0xFFFFu) || at + len > n || op + len > ulen) return GQ_INLINE;
        for (uint32_t i = 0; i < len; i++) gst(out + op + i, (uint8_t)byte_at(at + i));
        op += len;
        bp += 8ull * len;
        continue;
      }
      if (type == 1u) {
        for (uint32_t s = 0; s < 288u + 30u; s++) T.lens[s] = s < 144u ? 8 : s < 256u ? 9 : s < 280u ? 7 : s < 288u ? 8 : 5;
        gq_build(T, T.lens, 288, T.lcount, T.lsym, T.lfast, 0, L.lentab);
        gq_build(T, T.lens + 288, 30, T.dcount, T.dsym, T.dfast, 1, L.disttab);
      } else {
        const uint32_t nlen = bits(5) + 257u, ndist = bits(5) + 1u, ncode = bits(4) + 4u;
        if (nlen > 286u || ndist > 30u) return GQ_INLINE;
        for (uint32_t s = 0; s < 19u; s++) T.lens[s] = 0;
        for (uint32_t i = 0; i < ncode; i++) T.lens[L.ord[i]] = (uint8_t)bits(3);
        // the code-length code: canonical tables in dcount / dsym (rebuilt below)
        if (gq_build(T, T.lens, 19, T.dcount, T.dsym, T.dfast, 2, nullptr) != 0) return GQ_INLINE;
        uint32_t idx = 0;
        while (idx < nlen + ndist) {
          ensure(bp);
          // the code-length code is complete with codes of <= 7 bits: one first-level lookup
          const uint32_t ce = T.dfast[(uint32_t)peek(bp) & ((1u << GZ_FAST) - 1u)];
          if (ce == GZ_SLOW) return GQ_INLINE;
          const int sym = (int)gz_ent_sym(ce);
          bp += gz_ent_len(ce);
          if (sym < 16) {
            T.lens[idx++] = (uint8_t)sym;
          } else {
            uint32_t rep, val = 0;
            if (sym == 16) {
              if (idx == 0) return GQ_INLINE;
              val = T.lens[idx - 1u];
              rep = 3u + bits(2);
            } else if (sym == 17) {
              rep = 3u + bits(3);
            } else {
              rep = 11u + bits(7);
            }
            if (idx + rep > nlen + ndist) return GQ_INLINE;
            for (uint32_t k = 0; k < rep; k++) T.lens[idx + k] = (uint8_t)val;
            idx += rep;
          }
        }
        if (bp > endbit || T.lens[256] == 0u) return GQ_INLINE;
        // (descending: position 288 + k is read as nlen + k' for a larger k' when nlen > 258)
        for (int k = 31; k >= 0; k--) T.lens[288 + k] = (uint32_t)k < ndist ? T.lens[nlen + (uint32_t)k] : 0;
        const int e1 = gq_build(T, T.lens, (int)nlen, T.lcount, T.lsym, T.lfast, 0, L.lentab);
        if (e1 != 0) return GQ_INLINE;  // (incomplete single-code tables: the inline path)
        const int e2 = gq_build(T, T.lens + 288, (int)ndist, T.dcount, T.dsym, T.dfast, 1, L.disttab);
        if (e2 != 0) return GQ_INLINE;
      }
      // ---- the block's tokens: one step per token with the literal and back-reference forms
      // computed side by side (selects, both table reads issued together) and one exit test; codes
      // longer than the first-level tables take a rare branch
      while (true) {
        {  // re-centre every window of the loop together when one could leave its window
          const bool want = bp >= rthr;
          if (__ballot(want)) recenter((uint32_t)(bp >> 3));
        }
        const uint64_t x = peek(bp);
        uint32_t e = T.lfast[(uint32_t)x & ((1u << GZ_FAST) - 1u)];
        bool bad = false;
        uint32_t l = gz_ent_len(e);
        if (e == GZ_SLOW) {
          const int s2 = gq_slow(x, T.lcount, T.lsym, &l);
          bad = s2 < 0;
          e = s2 < 0 ? 0u : (uint32_t)s2;
          if (s2 > 256 && s2 < 286) {
            const uint32_t t = L.lentab[s2 - 257];
            e |= ((t & 0x1FFu) << 13) | ((t >> 16) << 22);
          }
        }
        const uint32_t sym = gz_ent_sym(e);
        const bool lit = sym < 256u, eob = sym == 256u;
        const uint32_t lext = lit || eob ? 0u : (e >> 22) & 7u;
        const uint32_t len = lit ? 1u : ((e >> 13) & 0x1FFu) + (uint32_t)((x >> l) & ((1u << lext) - 1u));
        const uint64_t y = x >> (l + lext);
        uint32_t d = T.dfast[(uint32_t)y & ((1u << GZ_FAST) - 1u)];
        uint32_t dl = gz_ent_len(d);
        if (!lit && !eob && d == GZ_SLOW) {
          const int s3 = gq_slow(y, T.dcount, T.dsym, &dl);
          bad |= s3 < 0 || s3 >= 30;
          const uint32_t t = L.disttab[s3 < 0 || s3 >= 30 ? 0 : s3];
          d = (uint32_t)(s3 < 0 ? 0 : s3) | ((t & 0x7FFFu) << 13) | ((t >> 16) << 28);
        }
        const uint32_t dext = d >> 28;
        const uint32_t dist = ((d >> 13) & 0x7FFFu) + (uint32_t)((y >> dl) & ((1u << dext) - 1u));
        const uint32_t tb = lit || eob ? l : l + lext + dl + dext;
        bad |= bp + tb > endbit || sym > 285u;
        if (!lit && !eob) bad |= gz_ent_sym(d) >= 30u || dist > op - mstart || cnt >= rcap;
        if (!eob) bad |= op + len > ulen;  // (a page completing inside the member: the scalar decoder)
        if (bad) return GQ_INLINE;
        bp += tb;
        if (eob) break;
        if (lit) {
          gst(out + op, (uint8_t)sym);
        } else {
          gst(rec + cnt, (uint64_t)op | ((uint64_t)dist << 32) | ((uint64_t)len << 48));
          cnt++;
        }
        op += len;
      }
    } while (!last);
    if (op >= ulen) break;  // complete: the trailer is not read
    // a member that ends before the page (its CRC-32 is checked by k_gzip)
    return GQ_INLINE;
  }
  // pages of long back-references (over 48 output bytes per record on average: few tokens, mostly
  // copying) are cheaper for the scalar decoder than for 189-byte replay windows
  return op == ulen && (cnt == 0u || ulen / cnt <= 48u) ? (int32_t)cnt : GQ_INLINE;
}

__global__ __launch_bounds__(64) void k_gzip_seq(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                                 uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                                 const GzJobDev* __restrict__ jobs, int n_jobs,
                                                 uint64_t* __restrict__ recs, int32_t* __restrict__ mode,
                                                 uint32_t min_out) {
  __shared__ __attribute__((aligned(16))) GqLds L;
  const uint32_t lane = lane_id();
  if (lane < 29u) L.lentab[lane] = GZ_LBASE[lane] | ((uint32_t)GZ_LEXT[lane] << 16);
  if (lane < 30u) L.disttab[lane] = GZ_DBASE[lane] | ((uint32_t)GZ_DEXT[lane] << 16);
  if (lane < 19u) L.ord[lane] = GZ_ORD[lane];
  wave_sync();
  const int j = (int)(blockIdx.x * GQ_JOBS + lane);
  if (lane >= GQ_JOBS || j >= n_jobs) return;  // (no cross-lane operation follows)
  const GzJobDev J = jobs[j];
  if (J.src_offset + J.src_size > src_bytes || J.dst_offset + J.dst_size > dst_bytes || J.dst_size < min_out) {  // (small pages: k_gzip)
    mode[j] = GQ_INLINE;
    return;
  }
  const rsrc_t rs = make_rsrc(src, src_bytes);
  mode[j] = gq_job(L, L.l[lane], rs, J, dst, recs);
}

// Replay: the records of a pre-passed page in 189-byte output windows. Every byte of a window gets its
// source — itself (a literal the pre-pass stored, read back into LDS) or the output position its
// back-reference copies — and the window is resolved by the shared executor.
__global__ __launch_bounds__(WAVE) void k_gzip_replay(uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                                      const GzJobDev* __restrict__ jobs, int n_jobs,
                                                      const uint64_t* __restrict__ recs,
                                                      const int32_t* __restrict__ mode, int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[LZ_RING];
  __shared__ __attribute__((aligned(16))) uint8_t lits[256];
  __shared__ uint32_t sS[LZ_CAP];
  __shared__ uint64_t rq[256];  // records [rq0, rq0 + 256)
  const int jb = (int)blockIdx.x;
  if (jb >= n_jobs || mode[jb] < 0) return;
  const uint32_t nrec = (uint32_t)mode[jb];
  if (nrec == 0u) {  // literals only: the pre-pass wrote the whole page
    if (lane_id() == 0 && status) status[jb] = 0;
    return;
  }
  const uint32_t lane = lane_id();
  const GzJobDev J = jobs[jb];
  const uint32_t ulen = uni(J.dst_size);
  uint8_t* out = dst + J.dst_offset;
  const rsrc_t ro = make_rsrc(out, dst_bytes - J.dst_offset);
  const uint64_t* rec = recs + J.dst_offset / 3u;
  uint32_t ri = 0, rq0 = 0, rqn = 0;  // next record; queue [rq0, rq0 + rqn)
  bool more = true;                   // records past the queue may exist
  for (uint32_t A = 0; A < ulen;) {
    if (more && ri + WAVE > rq0 + rqn) {  // refill the queue from ri
      rq0 = ri;
      for (uint32_t k = lane; k < 256u; k += WAVE) {
        const uint32_t i = rq0 + k;
        rq[k] = i < nrec ? rec[i] : ~0ull;
      }
      rqn = rq0 + 256u <= nrec ? 256u : nrec - rq0;
      more = rq0 + rqn < nrec;
      wave_sync();
    }
    // the window: up to LZ_CAP bytes, ending where the 64th record from ri starts (records are
    // disjoint and ascending and record ri ends past A, so that start lies past A and at most 63
    // records reach into the window, one per lane)
    uint32_t T = ulen - A < LZ_CAP ? ulen - A : LZ_CAP;
    if (ri + (WAVE - 1u) < rq0 + rqn) {
      const uint32_t at63 = uni((uint32_t)rq[ri + (WAVE - 1u) - rq0]);
      T = at63 - A < T ? at63 - A : T;
    }
    const uint32_t Bend = A + T;
    // the literal bytes of the window, and every byte's default source: itself
    for (uint32_t i = lane; i < T; i += WAVE) {
      const uint32_t a = A + i;
      lits[i] = (uint8_t)(__builtin_amdgcn_raw_buffer_load_b32(ro, (int)(a & ~3u), 0, 0) >> ((a & 3u) * 8u));
      sS[i] = LZ_LIT | i;
    }
    // records overlapping the window: a prefix of the queue from ri (output positions ascending)
    const uint32_t k = ri + lane;
    const uint64_t r = k < rq0 + rqn ? rq[k - rq0] : ~0ull;
    const uint32_t at = (uint32_t)r, dist = (uint32_t)(r >> 32) & 0xFFFFu, len = (uint32_t)(r >> 48);
    const bool valid = k < rq0 + rqn && at < Bend;  // (a queued record ends past A: ri moves past finished ones)
    const uint64_t stop = __ballot(!valid);
    const uint32_t m = stop ? (uint32_t)__builtin_ctzll(stop) : WAVE;
    wave_sync();
    if (lane < m) {
      const uint32_t b0 = at > A ? at : A, b1 = at + len < Bend ? at + len : Bend;
      for (uint32_t q = b0; q < b1; q++) sS[q - A] = q - dist;
    }
    wave_sync();
    lz_exec_sources<255u>(ring, lits, sS, T, A, out, ro);
    // records that end inside the window are done
    const uint64_t done = __ballot(lane < m && at + len <= Bend);
    ri += (uint32_t)__builtin_popcountll(done);
    A += T;
  }
  if (lane == 0 && status) status[jb] = 0;
}

hipError_t launch_gzip(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                       const void* jobs, int n_jobs, int32_t* status, uint64_t* recs, int32_t* mode,
                       uint32_t prepass_min) {
  if (n_jobs <= 0) return hipSuccess;
  if (!(recs && mode)) mode = nullptr;
  if (mode) {
    hipLaunchKernelGGL(k_gzip_seq, dim3((n_jobs + (int)GQ_JOBS - 1) / (int)GQ_JOBS), dim3(64), 0, st, src, src_bytes,
                       dst, dst_bytes, (const GzJobDev*)jobs, n_jobs, recs, mode, prepass_min);
    hipLaunchKernelGGL(k_gzip_replay, dim3(n_jobs), dim3(WAVE), 0, st, dst, dst_bytes, (const GzJobDev*)jobs, n_jobs,
                       (const uint64_t*)recs, (const int32_t*)mode, status);
  }
  hipLaunchKernelGGL(k_gzip, dim3(n_jobs), dim3(WAVE), 0, st, src, src_bytes, dst, dst_bytes,
                     (const GzJobDev*)jobs, n_jobs, status, (const int32_t*)mode);
  return hipGetLastError();
}

}  // namespace pqg
