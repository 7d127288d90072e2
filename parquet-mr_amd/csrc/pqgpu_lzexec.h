// pqgpu_lzexec.h — execution of a batch of LZ77 elements (literal runs and back-references) by one
// wave, shared by the LZ4_RAW (pqgpu_lz4.hip) and GZIP (pqgpu_gzip.hip) page decoders.
//
// A batch is at most LZ_EL elements and LZ_CAP output bytes: element k is a run of e_len[k] bytes
// whose source is either literal bytes in an LDS buffer (e_src[k] = LZ_LIT | offset) or earlier output
// (e_src[k] = the output position it copies from). Every output byte gets its
// source, pointer jumping follows copies of bytes copied inside the same batch in log2(depth)
// rounds, and the bytes come from the literal buffer, a 4 KiB LDS ring of the most recent output, or
// (older) the output in HBM after this wave's stores completed. The batch's bytes go to the ring and
// from there to HBM as aligned dwords (bytes at the ends).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pqgpu_device.h"

namespace pqg {

constexpr uint32_t LZ_RING = 4096;  // LDS window of the most recent output bytes
constexpr uint32_t LZ_RMASK = LZ_RING - 1;
constexpr uint32_t LZ_SEG = 2048;   // LDS segment of the compressed block / literal buffer
constexpr uint32_t LZ_CAP = 256;    // output bytes per batch
constexpr uint32_t LZ_EL = 64;      // elements per batch
constexpr uint32_t LZ_PIECE = 64;   // bytes per element at most
constexpr uint32_t LZ_LIT = 0x80000000u;  // source tag of a literal byte (| its offset in the literal buffer)

// ring bytes of output positions t .. t + 3 (the ring wraps)
__device__ __forceinline__ uint32_t lz_ring4(const uint8_t* ring, uint32_t t) {
  typedef uint32_t __attribute__((may_alias)) u32a;
  const u32a* ring32 = (const u32a*)ring;
  const uint32_t r = t & LZ_RMASK & ~3u;
  return __builtin_amdgcn_alignbyte(ring32[((r + 4u) & LZ_RMASK) >> 2], ring32[r >> 2], t & 3u);
}

// output [a, e) (all in the ring) to HBM: aligned dwords, bytes at the ends
__device__ __forceinline__ void lz_flush(const uint8_t* ring, uint8_t* out, uint32_t a, uint32_t e) {
  const uint32_t oal = (uint32_t)(uintptr_t)out & 3u;
  const uint32_t base = ((a + oal) & ~3u) - oal;
  const uint32_t skip = a - base, span = e - base;
  for (uint32_t d0 = 0; d0 < span; d0 += 4u * WAVE) {
    const uint32_t d = d0 + 4u * lane_id();
    if (d < span) {
      const uint32_t t = base + d, v = lz_ring4(ring, t);
      if (d >= skip && d + 4u <= span) {
        gst((uint32_t*)(out + t), v);
      } else {
#pragma unroll
        for (uint32_t j = 0; j < 4u; j++)
          if (d + j >= skip && d + j < span) gst(out + (t + j), (uint8_t)(v >> (8u * j)));
      }
    }
  }
}

// Output [op, op + T) from its byte sources sS[0, T) (LZ_LIT | offset in the literal buffer `lits`
// of LMASK + 1 bytes, or the output position copied): ring + HBM. ro: a buffer resource over the
// output (far copies read it back).
template <uint32_t LMASK = LZ_SEG - 1u>
__device__ __forceinline__ void lz_exec_sources(uint8_t* ring, const uint8_t* lits, uint32_t* sS, uint32_t T,
                                                uint32_t op, uint8_t* out, rsrc_t ro) {
  const uint32_t lane = lane_id();
  constexpr uint32_t NB = LZ_CAP / WAVE;
  uint32_t sv[NB];
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint32_t b = lane + WAVE * j;
    sv[j] = b < T ? sS[b] : LZ_LIT;
  }
#pragma unroll 1
  for (uint32_t r = 0; r < 12u; r++) {  // copies of copies inside the batch
    bool more = false, hop = false;
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const bool inb = !(sv[j] & LZ_LIT) && sv[j] >= op;
      const uint32_t nv = sS[(sv[j] - op) & (LZ_CAP - 1u)];
      sv[j] = inb ? nv : sv[j];
      hop |= inb;
      more |= inb && !(nv & LZ_LIT) && nv >= op;
    }
    if (!__ballot(hop)) break;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) sS[lane + WAVE * j] = sv[j];
    wave_sync();
    if (!__ballot(more)) break;
  }
  uint32_t bv[NB];
  bool far = false;
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint32_t v = sv[j];
    const uint32_t lit = lits[v & LMASK], rg = ring[v & LZ_RMASK];
    bv[j] = (v & LZ_LIT) ? lit : rg;
    far |= lane + WAVE * j < T && !(v & LZ_LIT) && v + LZ_RING < op + T + WAVE;
  }
  if (__ballot(far)) {  // older than the ring: from HBM, after this wave's stores completed
    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const uint32_t v = sv[j];
      if (lane + WAVE * j < T && !(v & LZ_LIT) && v + LZ_RING < op + T + WAVE) {
        const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(ro, (int)(v & ~3u), 0, 0);
        bv[j] = (w >> ((v & 3u) * 8u)) & 0xFFu;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint32_t b = lane + WAVE * j;
    if (b < T) ring[(op + b) & LZ_RMASK] = (uint8_t)bv[j];
  }
  wave_sync();
  lz_flush(ring, out, op, op + T);
}

// Execute elements [0, m) producing output [op, op + T): ring + HBM. `lits` is the literal buffer
// (LZ_SEG bytes).
template <uint32_t LMASK = LZ_SEG - 1u>
__device__ __forceinline__ void lz_exec_batch(uint8_t* ring, const uint8_t* lits, uint32_t* sS, const uint32_t* e_src,
                                              const uint32_t* e_len, uint32_t m, uint32_t T, uint32_t op,
                                              uint8_t* out, rsrc_t ro) {
  const uint32_t lane = lane_id();
  const uint32_t es = lane < m ? e_src[lane] : 0u, el = lane < m ? e_len[lane] : 0u;
  uint32_t tot;
  const uint32_t eo = wave_excl_scan_u32(el, &tot);
  for (uint32_t i = 0; i < el; i++) sS[eo + i] = es + i;  // literal: buffer byte; copy: output position
  wave_sync();
  lz_exec_sources<LMASK>(ring, lits, sS, T, op, out, ro);
}

}  // namespace pqg
