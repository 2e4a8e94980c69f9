// Fused rANS decode (+ float join) kernel for gfx950.
//
// Restates ansDecodeTable + ansDecodeKernel (ans/GpuANSDecode.cuh:34-476)
// and the float join (JoinFloatWriter / joinFloat,
// float/GpuFloatDecompress.cuh:39-841) in one pass, fp64 included.
//
// MI355X design:
//  * 128-thread workgroups (2 waves).  A wave decodes K block *pairs*: lanes
//    0-31 one block, lanes 32-63 the next (the reference's 32-state
//    interleaving).  K = 2 independent pairs (fp64: one pair with two
//    streams) give every step two independent state chains, and the step
//    body is branch-free so hipcc interleaves them.
//  * Per-half block bookkeeping (read pointer, ring window, data pointer)
//    is wave-uniform and lives in SGPRs; per step the VALU does only the
//    table lookup, state update, one v_mbcnt pair and the LDS word read.
//  * The compressed words of each block are staged in an LDS ring (1024 u16
//    per block, refilled 512 words at a time with one 16 B load per lane), so
//    the reference's dependent read in[-prefix] is an LDS read.
//  * Decoded symbols of a 1024-symbol segment go to LDS (1 byte / step); the
//    segment is then joined with the raw float bytes (prefetched 16 B loads)
//    and written with 16 B stores.
#pragma once

#include "device.h"

namespace dietgpu {
namespace dec {
constexpr int kThreads = 128;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kRing = 1024;    // u16 words per block ring
constexpr uint32_t kRefill = 512;   // words per refill (64 lanes x 16 B)
constexpr uint32_t kSegSteps = 32;  // decode steps per output segment
constexpr uint32_t kSegWords = kSegSteps * 32;
constexpr uint32_t kUnroll = 4;     // steps between ring checks
}  // namespace dec

#define DG_L __attribute__((address_space(3)))
template <typename T>
using lp = DG_L T*;

template <int FT>
struct DecCfg {
  static constexpr int S = FloatTraits<FT>::kSegs;  // ANS streams per word
  static constexpr int K = S == 2 ? 1 : 2;          // block pairs per wave
  static constexpr int kBlocksPerWave = 2 * K;
  static constexpr int kBlocksPerWG = dec::kWaves * kBlocksPerWave;
  // 16-byte raw vectors per 16-word chunk
  static constexpr int kRawVecs = FT == 0 ? 0 : (FT <= 2 ? 1 : (FT == 3 ? 3 : 6));
};

// One stream of one block pair.  Everything but x / ringLane is wave-uniform.
struct DPair {
  uint32_t x;                   // this lane's rANS state
  lp<const uint16_t> ringLane;  // this lane's half ring
  int32_t ptr[2];               // per half: next read is below ptr
  int32_t lo[2];                // per half: ring holds stream words >= lo
  gp<const uint16_t> data[2];   // per half: block's compressed words (HBM)
  lp<uint16_t> ring[2];         // per half: LDS ring
};

// Copy stream words [a, b) (a multiple of 8, b - a <= 512) of one half into
// its ring with the whole wave (one 16 B load per lane).  May read up to 7
// words past b: the block padding every archive has.
__device__ __forceinline__ void ringFill(gp<const uint16_t> data, lp<uint16_t> ring, int32_t a,
                                         int32_t b, uint32_t lane, bool vec) {
  if (vec) {
    const int32_t j = int32_t(lane);
    if (j < ((b - a + 7) >> 3)) {
      const uint4 v = ld16((gp<const uint4>)(data + a) + j);
      *(lp<u32x4>)(ring + ((a + 8 * j) & int32_t(dec::kRing - 1))) = u32x4{v.x, v.y, v.z, v.w};
    }
  } else {
    for (int32_t k = a + int32_t(lane); k < b; k += 64) ring[k & int32_t(dec::kRing - 1)] = data[k];
  }
}

// Ensure the next kUnroll steps of both halves find their words in the ring.
__device__ __forceinline__ void ringEnsure(DPair& p, uint32_t lane, bool vec) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (p.lo[hh] > 0 && p.ptr[hh] - int32_t(32 * dec::kUnroll) < p.lo[hh]) {
      const int32_t nlo = max(0, p.lo[hh] - int32_t(dec::kRefill));
      ringFill(p.data[hh], p.ring[hh], nlo, p.lo[hh], lane, vec);
      p.lo[hh] = nlo;
    }
  }
}

// One LIFO decode step (decodeOneWarp, ans/GpuANSDecode.cuh:55-105) of one
// stream of a block pair.  hv: all-ones on lanes 32-63.  Returns the LUT
// entry (symbol in bits 0-7).  kMask: lanes with !valid keep their state and
// do not read.
template <bool kMask>
__device__ __forceinline__ uint32_t decStep(DPair& p, bool valid, lp<const uint32_t> lut,
                                            uint32_t mask, int pb, uint32_t hv) {
  const uint32_t e = lut[p.x & mask];
  uint32_t xn = __umul24((e >> 8) & 0xfffu, p.x >> pb) + (e >> 20);
  if (kMask) xn = valid ? xn : p.x;
  const bool rd = kMask ? (valid && xn < kMinState) : (xn < kMinState);
  const uint64_t vote = ballot(rd);
  const int32_t cLo = __popc(uint32_t(vote));
  const int32_t cHi = __popc(uint32_t(vote >> 32));
  // read index = ptr' + (#readers of my half below me); mbcnt over 64 lanes
  // already counts all low-half readers for lanes 32-63.
  const int32_t baseLo = p.ptr[0] - cLo;
  const int32_t baseHi = p.ptr[1] - cHi - cLo;
  p.ptr[0] = baseLo;
  p.ptr[1] -= cHi;
  const uint32_t vbase = uint32_t(baseLo) + (hv & uint32_t(baseHi - baseLo));
  const uint32_t idx = __builtin_amdgcn_mbcnt_hi(uint32_t(vote >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(uint32_t(vote), vbase));
  const uint32_t v = p.ringLane[idx & (dec::kRing - 1)];  // harmless for non-readers
  // x = rd ? (xn << 16 | v) : xn as one v_perm.  Feeding the word through an
  // intrinsic (not a select) keeps the LDS read unconditional: a branch
  // around it would split the step and serialise the independent chains.
  p.x = __builtin_amdgcn_perm(xn, v, rd ? 0x05040100u : 0x07060504u);
  return e;
}

// Join 16 decoded symbols (LDS) with their raw bytes into output words.
template <int FT>
struct Join {
  using WordT = typename FloatTraits<FT>::WordT;
  static constexpr int kRawVecs = DecCfg<FT>::kRawVecs;
  static constexpr int kR = kRawVecs > 0 ? kRawVecs : 1;

  // prefetch the raw vectors of the chunk starting at word i0
  static __device__ __forceinline__ void load(uint4 (&r)[kR], gp<const uint8_t> raw, uint32_t n,
                                              uint32_t i0) {
    if constexpr (FT == 1 || FT == 2) {
      r[0] = ld16(raw + i0);
    } else if constexpr (FT == 3) {
      r[0] = ld16(raw + 2 * i0);
      r[1] = ld16(raw + 2 * i0 + 16);
      r[2] = ld16(raw + 2 * roundUp(n, 8) + i0);
    } else if constexpr (FT == 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = ld16(raw + 4 * i0 + 16 * k);
      const uint32_t hb = 4 * roundUp(n, 4);
      r[4] = ld16(raw + hb + 2 * i0);
      r[5] = ld16(raw + hb + 2 * i0 + 16);
    }
  }

  static __device__ __forceinline__ WordT one(uint32_t s0, uint32_t s1, gp<const uint8_t> raw,
                                              uint32_t n, uint32_t i) {
    if constexpr (FT == 0) {
      return WordT(s0);
    } else if constexpr (FT == 1) {
      return WordT((s0 << 8) | raw[i]);
    } else if constexpr (FT == 2) {
      const uint32_t r = raw[i];
      return WordT((s0 << 7) | (r >> 1) | ((r & 1u) << 15));
    } else if constexpr (FT == 3) {
      const uint32_t lo = ((gp<const uint16_t>)raw)[i];
      const uint32_t hb = raw[2 * roundUp(n, 8) + i];
      return rotr32((s0 << 24) | (hb << 16) | lo, 1);
    } else {
      const uint64_t lo = ((gp<const uint32_t>)raw)[i];
      const uint64_t hb = ((gp<const uint16_t>)(raw + 4 * roundUp(n, 4)))[i];
      const uint64_t v = (uint64_t(s0) << 56) | (uint64_t(s1) << 48) | (hb << 32) | lo;
      return (v >> 1) | (v << 63);
    }
  }

  // vector join of a full chunk: out[i0 .. i0+16)
  static __device__ __forceinline__ void vec(gp<uint8_t> outB, uint32_t i0, uint4 sv, uint4 sv1,
                                             const uint4 (&r)[kR]) {
    const uint32_t sw[4] = {sv.x, sv.y, sv.z, sv.w};
    if constexpr (FT == 0) {
      st16(outB + i0, sv);
    } else if constexpr (FT == 1 || FT == 2) {
      const uint32_t rw[4] = {r[0].x, r[0].y, r[0].z, r[0].w};
      uint32_t o[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // words 4k..4k+3: bytes of sw[k] / rw[k] spread into 16-bit lanes
        const uint32_t s01 = __builtin_amdgcn_perm(0u, sw[k], 0x0c010c00u);
        const uint32_t s23 = __builtin_amdgcn_perm(0u, sw[k], 0x0c030c02u);
        const uint32_t r01 = __builtin_amdgcn_perm(0u, rw[k], 0x0c010c00u);
        const uint32_t r23 = __builtin_amdgcn_perm(0u, rw[k], 0x0c030c02u);
        if constexpr (FT == 1) {
          o[2 * k] = (s01 << 8) | r01;
          o[2 * k + 1] = (s23 << 8) | r23;
        } else {
          o[2 * k] = (s01 << 7) | ((r01 >> 1) & 0x007f007fu) | ((r01 & 0x00010001u) << 15);
          o[2 * k + 1] = (s23 << 7) | ((r23 >> 1) & 0x007f007fu) | ((r23 & 0x00010001u) << 15);
        }
      }
      gp<uint4> d = (gp<uint4>)(outB + 2 * i0);
      st16(d, make_uint4(o[0], o[1], o[2], o[3]));
      st16(d + 1, make_uint4(o[4], o[5], o[6], o[7]));
    } else if constexpr (FT == 3) {
      const uint32_t lo[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
      const uint32_t hb[4] = {r[2].x, r[2].y, r[2].z, r[2].w};
      uint32_t o[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t s = (sw[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const uint32_t h8 = (hb[k >> 2] >> (8 * (k & 3))) & 0xffu;
        const uint32_t l16 = (lo[k >> 1] >> (16 * (k & 1))) & 0xffffu;
        o[k] = rotr32((s << 24) | (h8 << 16) | l16, 1);
      }
      gp<uint4> d = (gp<uint4>)(outB + 4 * i0);
#pragma unroll
      for (int k = 0; k < 4; ++k) st16(d + k, make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]));
    } else {
      const uint32_t sw1[4] = {sv1.x, sv1.y, sv1.z, sv1.w};
      const uint32_t lo[16] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w,
                               r[2].x, r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w};
      const uint32_t hw[8] = {r[4].x, r[4].y, r[4].z, r[4].w, r[5].x, r[5].y, r[5].z, r[5].w};
      gp<uint4> d = (gp<uint4>)(outB + 8 * i0);
#pragma unroll
      for (int k = 0; k < 16; k += 2) {
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int kk = k + q;
          const uint32_t s0 = (sw[kk >> 2] >> (8 * (kk & 3))) & 0xffu;
          const uint32_t s1 = (sw1[kk >> 2] >> (8 * (kk & 3))) & 0xffu;
          const uint32_t h16 = (hw[kk >> 1] >> (16 * (kk & 1))) & 0xffffu;
          // v = s0:s1:h16:lo (64 bits); w = rotr64(v, 1)
          const uint32_t vhi = (s0 << 24) | (s1 << 16) | h16;
          const uint32_t vlo = lo[kk];
          o[2 * q] = (vlo >> 1) | (vhi << 31);
          o[2 * q + 1] = (vhi >> 1) | (vlo << 31);
        }
        st16(d + (k >> 1), make_uint4(o[0], o[1], o[2], o[3]));
      }
    }
  }
};

// grid (ceil(maxBlocks / kBlocksPerWG), batch).  out.size(b) = capacity
// (bytes for raw ANS, words for floats).
template <int FT>
__global__ __launch_bounds__(dec::kThreads) void k_decode(BatchDesc in, BatchDesc out,
                                                          uint32_t batchOffset, int pb,
                                                          uint8_t* __restrict__ outSuccess,
                                                          uint32_t* __restrict__ outSize) {
  using Cfg = DecCfg<FT>;
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr int S = Cfg::S, K = Cfg::K, R = Join<FT>::kR;
  __shared__ uint32_t lutS[S][1u << 11];
  __shared__ __attribute__((aligned(16))) uint16_t ringS[dec::kWaves][K][S][2][dec::kRing];
  __shared__ __attribute__((aligned(16))) uint8_t segS[dec::kWaves][K][S][2][dec::kSegWords];
  __shared__ uint32_t red[dec::kWaves];
  __shared__ uint32_t cdfS[kNumSymbols];
  __shared__ uint32_t pdfS[kNumSymbols];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t tid = threadIdx.x;
  gp<const uint8_t> base = startOf(in, b);
  gp<const uint32_t> fh = (gp<const uint32_t>)base;

  gp<const uint8_t> arch[S];
  uint32_t n;
  bool ok;
  if constexpr (FT == 0) {
    arch[0] = base;
    n = fh[2];
    ok = fh[0] == kANSMagicVersion;
  } else {
    n = fh[1];
    ok = fh[0] == kFloatMagicVersion && (fh[2] & 0xfu) == uint32_t(FT);
    arch[0] = base + 32 + floatRawBytes(FT, n);
    if constexpr (S == 2) arch[S - 1] = arch[0] + fh[4];
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    gp<const uint32_t> ah = (gp<const uint32_t>)arch[s];
    ok = ok && ah[0] == kANSMagicVersion && (ah[4] & 0xfu) == uint32_t(pb) && ah[2] == n;
  }
  const bool success = ok && out.size(b) >= n;
  if (blockIdx.x == 0 && tid == 0) {
    if (outSuccess) outSuccess[b] = success ? 1 : 0;
    if (outSize) outSize[b] = ok ? n : 0u;
  }
  const uint32_t nBlocks = divUp(n, kBlockSize);
  if (!success || blockIdx.x * Cfg::kBlocksPerWG >= nBlocks) return;

#pragma unroll
  for (int s = 0; s < S; ++s) {
    buildLut<dec::kThreads>((gp<const uint16_t>)(arch[s] + kANSHeaderBytes), lutS[s], red, cdfS,
                            pdfS);
    __syncthreads();
  }

  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, l = lane & 31;
  const uint32_t hv = lane >= 32 ? ~0u : 0u;
  const uint32_t blk0 = blockIdx.x * Cfg::kBlocksPerWG + w * Cfg::kBlocksPerWave;
  if (blk0 >= nBlocks) return;

  const bool vecIn = (reinterpret_cast<uintptr_t>(base) & 15) == 0;
  gp<uint8_t> outB = startOf(out, b);
  const bool vecOut = (reinterpret_cast<uintptr_t>(outB) & 15) == 0;
  gp<const uint8_t> raw = base + 32;
  const uint32_t mask = (1u << pb) - 1;

  // per pair c: blocks blk0 + 2c (lanes 0-31) and blk0 + 2c + 1 (lanes 32-63)
  uint32_t uwH[K][2];  // wave-uniform
  DPair st[K][S];
#pragma unroll
  for (int c = 0; c < K; ++c) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      gp<const uint8_t> states = arch[s] + kANSHeaderBytes + kPdfBytes;
      gp<const uint2> bw = (gp<const uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
      gp<const uint16_t> data = (gp<const uint16_t>)(bw + roundUp(nBlocks, 2));
      DPair& d = st[c][s];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const uint32_t bk = blk0 + 2 * c + hh;
        d.ring[hh] = (lp<uint16_t>)&ringS[w][c][s][hh][0];
        if (bk < nBlocks) {
          const uint2 e = ld8(bw + bk);
          uwH[c][hh] = e.x >> 16;
          d.ptr[hh] = int32_t(e.x & 0xffffu);
          d.data[hh] = data + e.y;
          d.lo[hh] = d.ptr[hh] > int32_t(dec::kRing)
                         ? int32_t(roundUp(uint32_t(d.ptr[hh]) - dec::kRing, 8))
                         : 0;
          // initial fill of [lo, cw) (<= 1024 words: two wave-wide passes)
          ringFill(d.data[hh], d.ring[hh], d.lo[hh], min(d.ptr[hh], d.lo[hh] + 512), lane, vecIn);
          if (d.ptr[hh] > d.lo[hh] + 512)
            ringFill(d.data[hh], d.ring[hh], d.lo[hh] + 512, d.ptr[hh], lane, vecIn);
        } else {
          uwH[c][hh] = 0;
          d.ptr[hh] = 0;
          d.lo[hh] = 0;
          d.data[hh] = data;
        }
      }
      d.ringLane = lane >= 32 ? (lp<const uint16_t>)d.ring[1] : (lp<const uint16_t>)d.ring[0];
      const uint32_t bkMine = blk0 + 2 * c + (lane >> 5);
      d.x = bkMine < nBlocks
                ? ((gp<const uint32_t>)(states + uint64_t(kStateBytesPerBlock) * bkMine))[l]
                : kMinState;
    }
  }

  uint32_t T = 0;
#pragma unroll
  for (int c = 0; c < K; ++c) T = max(T, max(divUp(uwH[c][0], 32), divUp(uwH[c][1], 32)));

  for (int32_t g = int32_t(T - 1) / int32_t(dec::kSegSteps); g >= 0; --g) {
    const uint32_t segW0 = uint32_t(g) * dec::kSegWords;  // first word of segment in block
    // prefetch the raw bytes of this segment's full chunks
    uint4 rv[K][2][R];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
      const uint32_t bk = blk0 + 2 * c + (lane >> 5);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t off = segW0 + 16 * (l + 32 * q);
        if (FT != 0 && vecIn && off + 16 <= uw) Join<FT>::load(rv[c][q], raw, n, bk * kBlockSize + off);
      }
    }

    bool full = true;
#pragma unroll
    for (int c = 0; c < K; ++c)
      full = full && uwH[c][0] >= segW0 + dec::kSegWords && uwH[c][1] >= segW0 + dec::kSegWords;

    const int32_t tTop = min(int32_t(T) - 1, g * int32_t(dec::kSegSteps) + int32_t(dec::kSegSteps) - 1);
    const int32_t tBot = g * int32_t(dec::kSegSteps);
    if (full) {
      for (int32_t t0 = tTop; t0 >= tBot; t0 -= int32_t(dec::kUnroll)) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, vecIn);
#pragma unroll
        for (uint32_t u = 0; u < dec::kUnroll; ++u) {
          const uint32_t si = uint32_t(t0 - int32_t(u) - tBot) * 32 + l;
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) {
              const uint32_t e = decStep<false>(st[c][s], true, (lp<const uint32_t>)lutS[s], mask, pb, hv);
              segS[w][c][s][lane >> 5][si] = uint8_t(e);
            }
        }
      }
    } else {
      for (int32_t t = tTop; t >= tBot; --t) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, vecIn);
        const uint32_t si = uint32_t(t - tBot) * 32 + l;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
          const bool valid = uint32_t(t) * 32 + l < uw;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const uint32_t e = decStep<true>(st[c][s], valid, (lp<const uint32_t>)lutS[s], mask, pb, hv);
            if (valid) segS[w][c][s][lane >> 5][si] = uint8_t(e);
          }
        }
      }
    }

    // join + store this segment
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
      const uint32_t bk = blk0 + 2 * c + (lane >> 5);
      if (uw <= segW0) continue;
      const uint32_t segCnt = min(dec::kSegWords, uw - segW0);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t off = 16 * (l + 32 * q);  // word offset inside the segment
        if (off >= segCnt) continue;
        const uint32_t i0 = bk * kBlockSize + segW0 + off;
        lp<const uint8_t> s0 = (lp<const uint8_t>)&segS[w][c][0][lane >> 5][off];
        lp<const uint8_t> s1 = (lp<const uint8_t>)&segS[w][c][S - 1][lane >> 5][off];
        if ((FT == 0 || vecIn) && vecOut && off + 16 <= segCnt) {
          const u32x4 p0 = *(lp<const u32x4>)s0;
          const u32x4 p1 = *(lp<const u32x4>)s1;
          const uint4 a = make_uint4(p0.x, p0.y, p0.z, p0.w);
          const uint4 a1 = make_uint4(p1.x, p1.y, p1.z, p1.w);
          Join<FT>::vec(outB, i0, a, a1, rv[c][q]);
        } else {
          const uint32_t cnt = min(16u, segCnt - off);
          gp<WordT> o = (gp<WordT>)outB;
          for (uint32_t k = 0; k < cnt; ++k) o[i0 + k] = Join<FT>::one(s0[k], s1[k], raw, n, i0 + k);
        }
      }
    }
  }
}

}  // namespace dietgpu
