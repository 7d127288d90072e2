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
// (Its CRC-32 is not recomputed on the device: a corrupted non-final member whose DEFLATE data still
// decodes to its ISIZE is accepted here and rejected by the oracle.)
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
constexpr uint16_t GZ_SLOW = 0xFFFFu;

struct GzLds {
  uint8_t ring[LZ_RING];
  uint8_t lits[LZ_SEG];
  uint8_t seg[LZ_SEG];  // compressed bytes [lo, lo + LZ_SEG)
  uint32_t sS[LZ_CAP];
  uint32_t e_src[LZ_EL], e_len[LZ_EL];
  uint16_t lfast[1u << GZ_FAST], dfast[1u << GZ_FAST];  // symbol | length << 9
  int16_t lcount[16], lsym[320], dcount[16], dsym[32], ccount[16], csym[32];
  uint8_t lens[320 + 32];
};

__constant__ uint16_t GZ_LBASE[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t GZ_LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t GZ_DBASE[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                      1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t GZ_DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t GZ_ORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Canonical Huffman tables of lens[0 .. n) (RFC 1951 3.2.2): counts, symbols in canonical order and,
// when `fast`, the first-level table (bit-reversed codes of <= 9 bits -> symbol | length << 9).
// Returns left (0: complete, > 0: incomplete) or -1 (over-subscribed). All lanes.
__device__ int gz_build(const uint8_t* lens, int n, int16_t* count, int16_t* sym, uint16_t* fast) {
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
        const uint32_t c = base_c + rank;                    // MSB-first code
        const uint32_t rv = __builtin_bitreverse32(c) >> (32u - l);  // as the LSB-first reader sees it
        for (uint32_t k = 0; k < (1u << (GZ_FAST - l)); k++) fast[rv | (k << l)] = (uint16_t)(s | (l << 9));
      }
    }
  }
  wave_sync();
  return left;
}

struct GzJobDev {  // = pqg_snappy_job
  uint64_t src_offset;
  uint64_t dst_offset;
  uint32_t src_size;
  uint32_t dst_size;
};

__global__ __launch_bounds__(WAVE) void k_gzip(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                               uint8_t* __restrict__ dst, uint64_t dst_bytes,
                                               const GzJobDev* __restrict__ jobs, int n_jobs,
                                               int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) GzLds L;
  const int jb = (int)blockIdx.x;
  if (jb >= n_jobs) return;
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
  typedef uint32_t __attribute__((aligned(1), may_alias)) u32u;
  const uint64_t nbits = (uint64_t)n * 8u;
  uint32_t lo = 0x80000000u;  // segment = member bytes [lo, lo + LZ_SEG)
  auto fill = [&](uint32_t q) {
    lo = uni(q & ~15u);
#pragma unroll
    for (uint32_t i = 0; i < LZ_SEG; i += 16u * WAVE) {
      const uint32_t o = i + 16u * lane;
      *(u32x4*)(L.seg + o) = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + o), 0, 0);
    }
    wave_sync();
  };
  auto byte_at = [&](uint32_t q) -> uint32_t {  // byte q of the input (0 past its end)
    return q < n ? uni((ld32(rs, q & ~3u) >> ((q & 3u) * 8u)) & 0xFFu) : 0u;
  };
  // bit reader: the container bb holds bc bits; p = next byte to load. Bytes past n read as 0 (the
  // buffer resource returns 0 past the job's range only at the end of `src`, so they are masked):
  // reading past the input shows as consumed() > nbits, checked after every symbol.
  uint32_t p = 0, bc = 0;
  uint64_t bb = 0;
  auto refill = [&]() {
    while (bc <= 32u) {
      if (p < lo || p + 4u > lo + LZ_SEG) fill(p);
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
  // canonical decode (RFC 1951 3.2.2 order): the code read bit by bit, MSB first
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
  auto decode = [&](const uint16_t* fast, const int16_t* count, const int16_t* sym) -> int {
    refill();
    const uint32_t e = uni((uint32_t)fast[bb & ((1u << GZ_FAST) - 1u)]);
    if (e != GZ_SLOW) {
      const uint32_t l = e >> 9;
      bb >>= l;
      bc -= l;
      return (int)(e & 511u);
    }
    return decode_slow(count, sym);
  };

  // ---- output batches (pqgpu_lzexec.h)
  uint32_t op = 0;                // output bytes executed
  uint32_t m = 0, T = 0, nl = 0;  // batch: elements, output bytes, literal bytes
  bool open = false;              // the batch's last element is a literal run still growing
  auto exec = [&]() {
    if (m) {
      wave_sync();
      lz_exec_batch(L.ring, L.lits, L.sS, L.e_src, L.e_len, m, T, op, out, ro);
      op += T;
    }
    m = 0;
    T = 0;
    nl = 0;
    open = false;
  };
  auto put_lit = [&](uint32_t b) {
    if (m >= LZ_EL || T >= LZ_CAP) exec();
    if (lane == 0) {
      L.lits[nl] = (uint8_t)b;
      if (open) {
        L.e_len[m - 1u] += 1u;
      } else {
        L.e_src[m] = LZ_LIT | nl;
        L.e_len[m] = 1u;
      }
    }
    if (!open) m++;
    nl++;
    T++;
    open = (T & (LZ_PIECE - 1u)) != 0u;  // literal elements end at 64-byte steps of the batch
  };
  auto put_match = [&](uint32_t dist, uint32_t len) {
    open = false;
    while (len) {
      if (m >= LZ_EL || T >= LZ_CAP) exec();
      uint32_t take = len < LZ_PIECE ? len : LZ_PIECE;
      take = take < LZ_CAP - T ? take : LZ_CAP - T;
      if (lane == 0) {
        L.e_src[m] = op + T - dist;
        L.e_len[m] = take;
      }
      m++;
      T += take;
      len -= take;
    }
  };

  int code = 0;
  bool full = false;  // a symbol past the page's size was decoded: reading stops there
  uint32_t q = 0;     // byte position of the next member
  while (!code && op + T < ulen) {
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
    const uint32_t member_start = op + T;
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
          exec();
          if (op >= ulen) { full = true; break; }
          uint32_t take = left < LZ_CAP ? left : LZ_CAP;
          take = take < ulen - op ? take : ulen - op;
          for (uint32_t i = lane; i < take; i += WAVE) {
            const uint32_t b = s + i;
            L.lits[i] = (uint8_t)(ld32(rs, b & ~3u) >> ((b & 3u) * 8u));
          }
          if (lane < (take + LZ_PIECE - 1u) / LZ_PIECE) {
            L.e_src[lane] = LZ_LIT | (lane * LZ_PIECE);
            L.e_len[lane] = take - lane * LZ_PIECE < LZ_PIECE ? take - lane * LZ_PIECE : LZ_PIECE;
          }
          m = (take + LZ_PIECE - 1u) / LZ_PIECE;
          T = take;
          exec();
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
        gz_build(L.lens, 288, L.lcount, L.lsym, L.lfast);
        gz_build(L.lens + 288, 30, L.dcount, L.dsym, L.dfast);
      } else {  // dynamic codes (RFC 1951 3.2.7)
        const uint32_t nlen = bits(5) + 257u, ndist = bits(5) + 1u, ncode = bits(4) + 4u;
        if (nlen > 286u || ndist > 30u) { code = PQG_ERR_CORRUPT; break; }
        if (lane < 19u) L.lens[lane] = 0;
        wave_sync();
        for (uint32_t i = 0; i < ncode; i++) {
          const uint32_t v = bits(3);
          if (lane == 0) L.lens[GZ_ORD[i]] = (uint8_t)v;
        }
        wave_sync();
        if (consumed() > nbits || gz_build(L.lens, 19, L.ccount, L.csym, nullptr) != 0) { code = PQG_ERR_CORRUPT; break; }
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
        const int e1 = gz_build(L.lens, (int)nlen, L.lcount, L.lsym, L.lfast);
        uint32_t used = 0;
        for (int l = 1; l < 16; l++) used += uni((uint32_t)(int32_t)L.lcount[l]);
        if (e1 < 0 || (e1 > 0 && used != 1u)) { code = PQG_ERR_CORRUPT; break; }
        const int e2 = gz_build(L.lens + 288, (int)ndist, L.dcount, L.dsym, L.dfast);
        used = 0;
        for (int l = 1; l < 16; l++) used += uni((uint32_t)(int32_t)L.dcount[l]);
        if (e2 < 0 || (e2 > 0 && used > 1u)) { code = PQG_ERR_CORRUPT; break; }
      }
      // ---- the block's symbols
      while (true) {
        const int sym = decode(L.lfast, L.lcount, L.lsym);
        if (sym < 0 || consumed() > nbits) { code = PQG_ERR_CORRUPT; break; }
        if (sym < 256) {
          if (op + T >= ulen) { full = true; break; }
          put_lit((uint32_t)sym);
        } else if (sym == 256) {
          break;
        } else {
          const uint32_t li = (uint32_t)sym - 257u;
          if (li >= 29u) { code = PQG_ERR_CORRUPT; break; }
          uint32_t len = GZ_LBASE[li] + bits(GZ_LEXT[li]);
          const int ds = decode(L.dfast, L.dcount, L.dsym);
          if (ds < 0 || ds >= 30) { code = PQG_ERR_CORRUPT; break; }
          const uint32_t dist = GZ_DBASE[ds] + bits(GZ_DEXT[ds]);
          if (consumed() > nbits) { code = PQG_ERR_CORRUPT; break; }
          const uint32_t at = op + T;
          if (dist > at - member_start) { code = PQG_ERR_CORRUPT; break; }
          if (len > ulen - at) {  // the page completes inside this match
            len = ulen - at;
            full = true;
          }
          if (len) put_match(dist, len);
          if (full) break;
        }
      }
    } while (!code && !full && !last);
    if (code || full || op + T >= ulen) break;  // complete: the trailer is not read
    // ---- trailer of a member that ends before the page is complete: ISIZE (CRC-32 not recomputed)
    const uint32_t at = (uint32_t)((consumed() + 7u) >> 3);
    if (at + 8u > n) { code = PQG_ERR_CORRUPT; break; }
    const uint32_t isz = byte_at(at + 4u) | (byte_at(at + 5u) << 8) | (byte_at(at + 6u) << 16) | (byte_at(at + 7u) << 24);
    if (isz != op + T - member_start) { code = PQG_ERR_CORRUPT; break; }
    q = at + 8u;
  }
  if (!code) exec();
  if (!code && op != ulen) code = PQG_ERR_EOF;
  if (lane == 0 && status) status[jb] = code;
}

hipError_t launch_gzip(hipStream_t st, const uint8_t* src, uint64_t src_bytes, uint8_t* dst, uint64_t dst_bytes,
                       const void* jobs, int n_jobs, int32_t* status) {
  if (n_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gzip, dim3(n_jobs), dim3(WAVE), 0, st, src, src_bytes, dst, dst_bytes,
                     (const GzJobDev*)jobs, n_jobs, status);
  return hipGetLastError();
}

}  // namespace pqg
