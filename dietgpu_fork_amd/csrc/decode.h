// Fused rANS decode (+ float join) kernel for gfx950.
//
// Restates ansDecodeTable + ansDecodeKernel (ans/GpuANSDecode.cuh:34-476)
// and the float join (JoinFloatWriter / joinFloat,
// float/GpuFloatDecompress.cuh:39-841) in one pass, fp64 included.
//
// MI355X design:
//  * 256-thread workgroups (4 waves), 4 waves / SIMD.  A wave decodes K block
//    *pairs*: lanes 0-31 one block, lanes 32-63 the next (the reference's
//    32-state interleaving).  K = 2 independent pairs (fp64: one pair with
//    two streams) give every step two independent state chains; the step is
//    branch-free so they interleave.
//  * 64-bit decode table {pdf | sym << 24, slot - cdf}: the state update is
//    one v_mad_u32_u24 (u24 ignores the symbol byte), and `entry >> 16` =
//    sym << 8 is stored with ds_write_b16_d16_hi -- already the high byte of
//    an fp16 / bf16 word.  ds_read_b64 costs the same LDS cycles as b32.
//  * Per-half block bookkeeping (read pointer, ring window, data pointer) is
//    wave-uniform (SGPRs).  Compressed words are staged in a 512-word LDS
//    ring per block stream; the next 256-word refill is prefetched into
//    registers as soon as the previous one lands, so refills rarely wait on
//    HBM.
//  * 16-step segments are fully unrolled (constant LDS offsets); the
//    decoded 512-word segment is joined with its raw float bytes (16 B loads
//    issued before the segment) and written with 16 B stores.
#pragma once

#include <type_traits>

#include "device.h"

#ifndef DG_EXP
#define DG_EXP 0  // timing experiments only (make exp): 0 = the real decoder
#endif

namespace dietgpu {
#if DG_EXP == 7
// experiment 7: per-wave s_memtime stamps (lane 0), 24 slots per wave
__device__ uint64_t g_dbgT[16384 * 24];
#define DG_STAMP(slot)                                                                \
  do {                                                                                \
    if (lane == 0 && blockIdx.y * gridDim.x * 4 < 16384)                              \
      g_dbgT[((blockIdx.y * gridDim.x + blockIdx.x) * 4 + w) * 24 + (slot)] =         \
          __builtin_amdgcn_s_memtime();                                               \
  } while (0)
#else
#define DG_STAMP(slot) \
  do {                 \
  } while (0)
#endif
namespace dec {
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kRing = 512;      // u16 words per block-stream ring
constexpr uint32_t kRefill = 256;    // words per refill (64 lanes x 8 B)
constexpr uint32_t kSegSteps = 16;   // decode steps per output segment
constexpr uint32_t kSegWords = kSegSteps * 32;
constexpr uint32_t kUnroll = 4;      // steps between ring checks
}  // namespace dec

template <int FT>
struct DecCfg {
  static constexpr int S = FloatTraits<FT>::kSegs;  // ANS streams per word
  static constexpr int K = S == 2 ? 1 : 2;          // block pairs per wave
  static constexpr int kBlocksPerWave = 2 * K;
  static constexpr int kBlocksPerWG = dec::kWaves * kBlocksPerWave;
  static constexpr uint32_t kHalfStreams = dec::kWaves * K * S * 2;
  static constexpr uint32_t kRingBytes = kHalfStreams * dec::kRing * 2;
  static constexpr uint32_t kSegBytes = kHalfStreams * dec::kSegWords * 2;
  // dynamic LDS: S tables of 8 << pb bytes, rings, segment buffers
  __host__ __device__ static constexpr uint32_t lutBytes(int pb) { return S * (8u << pb); }
  __host__ __device__ static constexpr uint32_t ldsBytes(int pb) {
    return lutBytes(pb) + kRingBytes + kSegBytes;
  }
};

// One ANS stream of one block pair.  All but x / pf are wave-uniform.
struct DStream {
  uint32_t x;                   // this lane's rANS state
  lp<uint16_t> ring;            // LDS ring of half 0 (half 1 follows)
  lp<const uint16_t> ringLane;  // this lane's half ring
  int32_t ptr[2];               // per half: next read is below ptr
  int32_t lo[2];                // per half: ring holds stream words >= lo
  gp<const uint16_t> data[2];   // per half: block's compressed words (HBM)
  u32x2 pf[2];                  // per half: prefetched words [lo - 256, lo)
};

// 4 compressed words at p (8 B load when aligned)
__device__ __forceinline__ u32x2 ld4w(gp<const uint16_t> p, bool vec) {
  if (vec) return *(gp<const u32x2>)p;
  return u32x2{uint32_t(p[0]) | (uint32_t(p[1]) << 16), uint32_t(p[2]) | (uint32_t(p[3]) << 16)};
}

// Prefetch words [max(0, lo - 256), lo) of one half (lane j: 4 words).
// May read up to 3 words past lo: inside the block's 8-word padding.
__device__ __forceinline__ void ringPrefetch(DStream& p, int hh, uint32_t lane, bool vec) {
  const int32_t nlo = max(0, p.lo[hh] - int32_t(dec::kRefill));
  if (p.lo[hh] > 0 && int32_t(4 * lane) < p.lo[hh] - nlo)
    p.pf[hh] = ld4w(p.data[hh] + nlo + 4 * lane, vec);
}

// Refill [lo - 256, lo) of each half from its prefetch registers when fewer
// than kAt words are buffered below ptr (the refill overwrites words
// >= lo + 256, all consumed since ptr < lo + kAt <= lo + 256).  kAt = 256 at
// segment boundaries; kAt = 32 * kUnroll every kUnroll steps as the
// emergency path for dense data (then the next prefetch is issued at once).
template <int kAt, bool kPrefetchNow>
__device__ __forceinline__ void ringRefill(DStream& p, uint32_t lane, bool vec) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (DG_EXP != 3 && p.lo[hh] > 0 && p.ptr[hh] - kAt < p.lo[hh]) {
      const int32_t nlo = max(0, p.lo[hh] - int32_t(dec::kRefill));
      if (int32_t(4 * lane) < p.lo[hh] - nlo)
        *(lp<u32x2>)(p.ring + hh * dec::kRing + ((nlo + 4 * lane) & (dec::kRing - 1))) = p.pf[hh];
      p.lo[hh] = nlo;
      if (kPrefetchNow) ringPrefetch(p, hh, lane, vec);
    }
  }
}

// One LIFO decode step (decodeOneWarp, ans/GpuANSDecode.cuh:55-105) of one
// stream of a block pair.  hv: all-ones on lanes 32-63 (opaque to the
// compiler).  Returns the table entry's low word (sym in bits 24-31).
// kMask: lanes with !valid keep their state and do not read.
template <bool kMask>
__device__ __forceinline__ uint32_t decStep(DStream& p, bool valid, lp<const u32x2> lut,
                                            uint32_t mask, int pb, uint32_t hv) {
  const u32x2 e = lut[p.x & mask];
  uint32_t xn = __umul24(e.x, p.x >> pb) + e.y;
  if (kMask) xn = valid ? xn : p.x;
  const bool rd = kMask ? (valid && xn < kMinState) : (xn < kMinState);
  const uint64_t vote = ballot(rd);
  const int32_t cLo = __popc(uint32_t(vote));
  const int32_t cHi = __popc(uint32_t(vote >> 32));
  // read index = ptr' + (#readers of my half below me); v_mbcnt over 64
  // lanes already counts every low-half reader for lanes 32-63.
  const int32_t baseLo = p.ptr[0] - cLo;
  const int32_t diff = p.ptr[1] - p.ptr[0] - cHi;  // (ptr1 - cHi - cLo) - baseLo
  p.ptr[0] = baseLo;
  p.ptr[1] -= cHi;
  const uint32_t vbase = uint32_t(baseLo) + (hv & uint32_t(diff));
  const uint32_t idx = __builtin_amdgcn_mbcnt_hi(uint32_t(vote >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(uint32_t(vote), vbase));
#if DG_EXP == 2
  const uint32_t v = idx;  // experiment: no ring read
#else
  const uint32_t v = p.ringLane[idx & (dec::kRing - 1)];  // harmless for non-readers
#endif
  // x = rd ? (xn << 16 | v) : xn as one v_perm.  Feeding the word through an
  // intrinsic (not a select) keeps the LDS read unconditional: a branch
  // around it would split the step and serialise the independent chains.
  p.x = __builtin_amdgcn_perm(xn, v, rd ? 0x05040100u : 0x07060504u);
  return e.x;
}

// Join 16 decoded symbols (u16 sym << 8 in LDS) with their raw bytes.
template <int FT>
struct Join {
  using WordT = typename FloatTraits<FT>::WordT;
  static constexpr int kR = FT == 0 ? 1 : (FT <= 2 ? 1 : (FT == 3 ? 3 : 6));

  // raw vectors of the chunk starting at word i0 (16 B loads)
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

  // scalar join of word i (s0, s1: symbols)
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

  // [raw_a, sym0, raw_b, sym1] from a symbol pair (syms at bytes 1, 3) and
  // raw bytes a, b = bytes 2*odd, 2*odd + 1 of rw
  static __device__ __forceinline__ uint32_t pair16(uint32_t sp, uint32_t rw, int odd) {
    return __builtin_amdgcn_perm(sp, rw, odd ? 0x07030502u : 0x07010500u);
  }

  // vector join of a full chunk: out words [i0, i0 + 16).  s / s1: 8 dwords
  // of u16 (sym << 8) of stream 0 / 1.
  static __device__ __forceinline__ void vec(gp<uint8_t> outB, uint32_t i0, const uint32_t (&s)[8],
                                             const uint32_t (&s1)[8], const uint4 (&r)[kR]) {
    if constexpr (FT == 0) {
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __builtin_amdgcn_perm(s[2 * k + 1], s[2 * k], 0x07050301u);
      st16(outB + i0, make_uint4(o[0], o[1], o[2], o[3]));
    } else if constexpr (FT == 1 || FT == 2) {
      const uint32_t rw[4] = {r[0].x, r[0].y, r[0].z, r[0].w};
      uint32_t o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t t = pair16(s[k], rw[k >> 1], k & 1);  // exp << 8 | raw per half
        // bf16: rotate each 16-bit half right by one (raw = mant << 1 | sign)
        o[k] = FT == 1 ? t : (((t >> 1) & 0x7fff7fffu) | ((t << 15) & 0x80008000u));
      }
      gp<uint4> d = (gp<uint4>)(outB + 2 * i0);
      st16(d, make_uint4(o[0], o[1], o[2], o[3]));
      st16(d + 1, make_uint4(o[4], o[5], o[6], o[7]));
    } else if constexpr (FT == 3) {
      const uint32_t lw[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
      const uint32_t hw[4] = {r[2].x, r[2].y, r[2].z, r[2].w};
      uint32_t o[16];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t h = pair16(s[k], hw[k >> 1], k & 1);  // [hb, sym] x 2
        const uint32_t w0 = __builtin_amdgcn_perm(h, lw[k], 0x05040100u);
        const uint32_t w1 = __builtin_amdgcn_perm(h, lw[k], 0x07060302u);
        o[2 * k] = __builtin_amdgcn_alignbit(w0, w0, 1);
        o[2 * k + 1] = __builtin_amdgcn_alignbit(w1, w1, 1);
      }
      gp<uint4> d = (gp<uint4>)(outB + 4 * i0);
#pragma unroll
      for (int k = 0; k < 4; ++k) st16(d + k, make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]));
    } else {
      const uint32_t lw[16] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w,
                               r[2].x, r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w};
      const uint32_t hw[8] = {r[4].x, r[4].y, r[4].z, r[4].w, r[5].x, r[5].y, r[5].z, r[5].w};
      gp<uint4> d = (gp<uint4>)(outB + 8 * i0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        // [s1, s0] pairs, then vhi = [h16, s1, s0] per word; w = rotr64(vhi:lo, 1)
        const uint32_t p = __builtin_amdgcn_perm(s[k], s1[k], 0x07030501u);
        const uint32_t vh0 = __builtin_amdgcn_perm(p, hw[k], 0x05040100u);
        const uint32_t vh1 = __builtin_amdgcn_perm(p, hw[k], 0x07060302u);
        const uint32_t l0 = lw[2 * k], l1 = lw[2 * k + 1];
        st16(d + k, make_uint4(__builtin_amdgcn_alignbit(vh0, l0, 1), __builtin_amdgcn_alignbit(l0, vh0, 1),
                               __builtin_amdgcn_alignbit(vh1, l1, 1), __builtin_amdgcn_alignbit(l1, vh1, 1)));
      }
    }
  }
};

// 64-bit decode table of one archive: entry[slot] = {pdf | sym << 24,
// slot - cdf[sym]} (packDecodeLookup, ans/GpuANSDecode.cuh:34-44, re-laid
// out for v_mad_u32_u24).  scratch: >= 2 * 256 + 4 dwords of LDS.
__device__ __forceinline__ void buildLut64(gp<const uint16_t> pdfIn, lp<u32x2> lut,
                                           uint32_t* scratch) {
  static_assert(dec::kThreads == kNumSymbols, "one symbol per thread");
  uint32_t* cdfS = scratch;
  uint32_t* pdfS = scratch + kNumSymbols;
  uint32_t* red = scratch + 2 * kNumSymbols;
  const uint32_t tid = threadIdx.x;
  const uint32_t p = pdfIn[tid];
  const uint32_t c = blockExclusiveScan<dec::kThreads>(p, red, nullptr);
  pdfS[tid] = p;
  cdfS[tid] = c;
  __syncthreads();
  const uint32_t lane = tid & 63;
  for (uint32_t s = tid >> 6; s < kNumSymbols; s += dec::kWaves) {
    const uint32_t ps = pdfS[s], cs = cdfS[s];
    for (uint32_t j = lane; j < ps; j += 64) lut[cs + j] = u32x2{ps | (s << 24), j};
  }
}

// grid (ceil(maxBlocks / (kBlocksPerWG * chunksPerWG)), batch), dynamic LDS
// DecCfg<FT>::ldsBytes(pb).  out.size(b) = capacity (bytes for raw ANS,
// words for floats).
template <int FT>
__global__ __launch_bounds__(dec::kThreads) void k_decode(BatchDesc in, BatchDesc out,
                                                          uint32_t batchOffset, int pb,
                                                          uint32_t chunksPerWG,
                                                          uint8_t* __restrict__ outSuccess,
                                                          uint32_t* __restrict__ outSize) {
  using Cfg = DecCfg<FT>;
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr int S = Cfg::S, K = Cfg::K, R = Join<FT>::kR;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  lp<uint8_t> L = (lp<uint8_t>)smem;
  const uint32_t lutBytes = Cfg::lutBytes(pb);
  lp<uint16_t> ringAll = (lp<uint16_t>)(L + lutBytes);
  lp<uint16_t> segAll = (lp<uint16_t>)(L + lutBytes + Cfg::kRingBytes);

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
  if (!success || blockIdx.x * chunksPerWG * Cfg::kBlocksPerWG >= nBlocks) return;

#pragma unroll
  for (int s = 0; s < S; ++s) {
    buildLut64((gp<const uint16_t>)(arch[s] + kANSHeaderBytes),
               (lp<u32x2>)(L + s * (lutBytes / S)), (uint32_t*)segAll);
    __syncthreads();
  }

  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, l = lane & 31;
  uint32_t hv = lane >= 32 ? ~0u : 0u;
  asm volatile("" : "+v"(hv));  // keep `hv & x` a v_and (not a v_cndmask pair)
  DG_STAMP(0);
#if DG_EXP == 7
  if (lane == 0 && blockIdx.y * gridDim.x * 4 < 16384)
    g_dbgT[((blockIdx.y * gridDim.x + blockIdx.x) * 4 + w) * 24 + 23] =
        __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) |
        (uint64_t(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11))) << 32);
  if (lane == 0 && blockIdx.y * gridDim.x * 4 < 16384)
    g_dbgT[((blockIdx.y * gridDim.x + blockIdx.x) * 4 + w) * 24 + 22] = __builtin_amdgcn_s_memrealtime();
#endif

  const bool vecIn = (reinterpret_cast<uintptr_t>(base) & 15) == 0;
  gp<uint8_t> outB = startOf(out, b);
  const bool vecOut = (reinterpret_cast<uintptr_t>(outB) & 15) == 0;
  gp<const uint8_t> raw = base + 32;
  const uint32_t mask = (1u << pb) - 1;

  // Persistent over chunksPerWG consecutive 16-block chunks of this element
  // (the grid is sized to one generation of resident workgroups, so no
  // second-generation dip and one table build per workgroup).
  for (uint32_t pass = 0; pass < chunksPerWG; ++pass) {
    const uint32_t blk0 = (blockIdx.x * chunksPerWG + pass) * Cfg::kBlocksPerWG + w * Cfg::kBlocksPerWave;
    if (blk0 >= nBlocks) break;
    // per pair c: blocks blk0 + 2c (lanes 0-31) and blk0 + 2c + 1 (lanes 32-63)
    uint32_t uwH[K][2];  // wave-uniform
    DStream st[K][S];
    lp<uint16_t> segLane[K][S];
  #pragma unroll
    for (int c = 0; c < K; ++c) {
  #pragma unroll
      for (int s = 0; s < S; ++s) {
        gp<const uint8_t> states = arch[s] + kANSHeaderBytes + kPdfBytes;
        gp<const uint2> bw = (gp<const uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
        gp<const uint16_t> data = (gp<const uint16_t>)(bw + roundUp(nBlocks, 2));
        DStream& d = st[c][s];
        const uint32_t hs = (w * K + c) * S + s;  // half-stream pair index
        d.ring = ringAll + hs * 2 * dec::kRing;
        d.ringLane = d.ring + (hv & dec::kRing);
        segLane[c][s] = segAll + hs * 2 * dec::kSegWords + (hv & dec::kSegWords) + l;
  #pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const uint32_t bk = blk0 + 2 * c + hh;
          uwH[c][hh] = 0;
          d.ptr[hh] = 0;
          d.lo[hh] = 0;
          d.data[hh] = data;
          d.pf[hh] = u32x2{0, 0};
          if (bk < nBlocks) {
            const uint2 e = ld8(bw + bk);
            const uint32_t ex = readfirst(e.x), ey = readfirst(e.y);  // wave-uniform: SGPRs
            uwH[c][hh] = ex >> 16;
            const int32_t cw = int32_t(ex & 0xffffu);
            d.ptr[hh] = cw;
            d.data[hh] = data + ey;
            const int32_t lo = cw > int32_t(dec::kRing) ? int32_t(roundUp(uint32_t(cw) - dec::kRing, 4)) : 0;
            d.lo[hh] = lo;
            // initial fill of [lo, cw) (<= 512 words: two wave-wide passes)
  #pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int32_t a = lo + q * int32_t(dec::kRefill) + int32_t(4 * lane);
              if (a < cw)
                *(lp<u32x2>)(d.ring + hh * dec::kRing + (a & (dec::kRing - 1))) = ld4w(d.data[hh] + a, vecIn);
            }
            ringPrefetch(d, hh, lane, vecIn);
          }
        }
        const uint32_t bkMine = blk0 + 2 * c + (lane >> 5);
        d.x = bkMine < nBlocks
                  ? ((gp<const uint32_t>)(states + uint64_t(kStateBytesPerBlock) * bkMine))[l]
                  : kMinState;
      }
    }

    uint32_t T = 0;
  #pragma unroll
    for (int c = 0; c < K; ++c) T = max(T, max(divUp(uwH[c][0], 32), divUp(uwH[c][1], 32)));

    lp<const u32x2> lut[S];
  #pragma unroll
    for (int s = 0; s < S; ++s) lut[s] = (lp<const u32x2>)(L + s * (lutBytes / S));

    // segments [0, nFull) are full for every block of the wave; the partial
    // top segments (element tail / odd block count) are decoded first, masked
    uint32_t nFull = ~0u;
  #pragma unroll
    for (int c = 0; c < K; ++c) nFull = min(nFull, min(uwH[c][0], uwH[c][1]) / dec::kSegWords);
    const int32_t nSeg = int32_t(divUp(T, dec::kSegSteps));
    const uint32_t off = 16 * l;  // this lane's chunk in a segment

    // Per segment the VMEM order is: [steps: LDS only] [boundary refill from
    // the prefetch registers] [join: raw bytes loaded a segment earlier,
    // 16 B stores] [issue the next segment's raw loads and ring prefetches].
    // Every s_waitcnt vmcnt then finds only operations issued a whole step
    // phase earlier.  kVec: 16 B aligned input and output (once per wave).
    auto run = [&](auto vecTag) {
      constexpr bool kVec = decltype(vecTag)::value;
      uint4 rv[K][R];
      auto i0x = [&](int k) { return uint32_t(k) + lane; };
      auto loadRaw = [&](int32_t g, bool fullSeg) {
        const uint32_t segW0 = uint32_t(g) * dec::kSegWords;
  #pragma unroll
        for (int c = 0; c < K; ++c) {
          const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
          const uint32_t bk = blk0 + 2 * c + (lane >> 5);
          if (FT != 0 && kVec && (fullSeg || segW0 + off + 16 <= uw)) {
            if (DG_EXP == 4) {
  #pragma unroll
              for (int k = 0; k < R; ++k) rv[c][k] = make_uint4(i0x(k), 0, 0, 0);
            } else {
              Join<FT>::load(rv[c], raw, n, bk * kBlockSize + segW0 + off);
            }
          }
        }
      };
      auto join = [&](int32_t g, bool fullSeg) {
        const uint32_t segW0 = uint32_t(g) * dec::kSegWords;
  #pragma unroll
        for (int c = 0; c < K && DG_EXP != 1; ++c) {
          const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
          const uint32_t bk = blk0 + 2 * c + (lane >> 5);
          if (!fullSeg && segW0 + off >= uw) continue;
          const uint32_t cnt = fullSeg ? 16u : min(16u, uw - segW0 - off);
          const uint32_t i0 = bk * kBlockSize + segW0 + off;
          lp<const uint16_t> q0 = segLane[c][0] - l + off;
          lp<const uint16_t> q1 = segLane[c][S - 1] - l + off;
          if (kVec && cnt == 16) {
            uint32_t sv[8], sv1[8];
            const u32x4 a0 = *(lp<const u32x4>)q0, a1 = *(lp<const u32x4>)(q0 + 8);
            sv[0] = a0.x; sv[1] = a0.y; sv[2] = a0.z; sv[3] = a0.w;
            sv[4] = a1.x; sv[5] = a1.y; sv[6] = a1.z; sv[7] = a1.w;
            if constexpr (S == 2) {
              const u32x4 b0 = *(lp<const u32x4>)q1, b1 = *(lp<const u32x4>)(q1 + 8);
              sv1[0] = b0.x; sv1[1] = b0.y; sv1[2] = b0.z; sv1[3] = b0.w;
              sv1[4] = b1.x; sv1[5] = b1.y; sv1[6] = b1.z; sv1[7] = b1.w;
            } else {
  #pragma unroll
              for (int k = 0; k < 8; ++k) sv1[k] = 0;
            }
            Join<FT>::vec(outB, i0, sv, sv1, rv[c]);
          } else {
            gp<WordT> o = (gp<WordT>)outB;
            for (uint32_t k = 0; k < cnt; ++k)
              o[i0 + k] = Join<FT>::one(q0[k] >> 8, q1[k] >> 8, raw, n, i0 + k);
          }
        }
      };
      auto boundary = [&]() {
  #pragma unroll
        for (int c = 0; c < K; ++c)
  #pragma unroll
          for (int s = 0; s < S; ++s) ringRefill<int(dec::kRefill), false>(st[c][s], lane, kVec);
      };
      auto reissue = [&]() {
  #pragma unroll
        for (int c = 0; c < K; ++c)
  #pragma unroll
          for (int s = 0; s < S; ++s)
  #pragma unroll
            for (int hh = 0; hh < 2; ++hh) ringPrefetch(st[c][s], hh, lane, kVec);
      };

      if (nSeg > 0) loadRaw(nSeg - 1, uint32_t(nSeg - 1) < nFull);
      // partial segments: masked steps
      for (int32_t g = nSeg - 1; g >= int32_t(nFull); --g) {
        const int32_t tTop = min(int32_t(T) - 1, g * int32_t(dec::kSegSteps) + int32_t(dec::kSegSteps) - 1);
        const int32_t tBot = g * int32_t(dec::kSegSteps);
        for (int32_t t = tTop; t >= tBot; --t) {
  #pragma unroll
          for (int c = 0; c < K; ++c)
  #pragma unroll
            for (int s = 0; s < S; ++s) ringRefill<32, true>(st[c][s], lane, kVec);
  #pragma unroll
          for (int c = 0; c < K; ++c) {
            const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
            const bool valid = uint32_t(t) * 32 + l < uw;
  #pragma unroll
            for (int s = 0; s < S; ++s) {
              const uint32_t e = decStep<true>(st[c][s], valid, lut[s], mask, pb, hv);
              if (valid) segLane[c][s][(t - tBot) * 32] = uint16_t(e >> 16);
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        boundary();
        join(g, false);
        __builtin_amdgcn_wave_barrier();
        if (g > 0) loadRaw(g - 1, uint32_t(g - 1) < nFull);
        reissue();
      }
      // full segments: unrolled, unmasked
      DG_STAMP(1);
      for (int32_t g = min(nSeg, int32_t(nFull)) - 1; g >= 0; --g) {
  #pragma unroll
        for (int grp = int(dec::kSegSteps / dec::kUnroll) - 1; grp >= 0 && DG_EXP != 6; --grp) {
  #pragma unroll
          for (int c = 0; c < K; ++c)
  #pragma unroll
            for (int s = 0; s < S; ++s)
              ringRefill<int(32 * dec::kUnroll), true>(st[c][s], lane, kVec);
  #pragma unroll
          for (int u = int(dec::kUnroll) - 1; u >= 0; --u) {
            const int tr = grp * int(dec::kUnroll) + u;  // step within segment
  #pragma unroll
            for (int c = 0; c < K; ++c)
  #pragma unroll
              for (int s = 0; s < S; ++s) {
                const uint32_t e = decStep<false>(st[c][s], true, lut[s], mask, pb, hv);
                segLane[c][s][tr * 32] = uint16_t(e >> 16);
              }
          }
        }
        __builtin_amdgcn_wave_barrier();
        DG_STAMP(2 + 2 * (g & 7));
        boundary();
        join(g, true);
        __builtin_amdgcn_wave_barrier();
        if (g > 0) loadRaw(g - 1, true);
        reissue();
        DG_STAMP(3 + 2 * (g & 7));
  #if DG_EXP == 7
        if (g == 0 && lane == 0 && blockIdx.y * gridDim.x * 4 < 16384)
          g_dbgT[((blockIdx.y * gridDim.x + blockIdx.x) * 4 + w) * 24 + 21] = __builtin_amdgcn_s_memrealtime();
  #endif
      }
    };
    if (vecIn && vecOut)
      run(std::true_type{});
    else
      run(std::false_type{});
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace dietgpu
