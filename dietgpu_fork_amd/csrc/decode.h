// Fused rANS decode (+ float join) kernel for gfx950.
//
// Restates ansDecodeTable + ansDecodeKernel (ans/GpuANSDecode.cuh:34-476)
// and the float join (JoinFloatWriter / joinFloat,
// float/GpuFloatDecompress.cuh:39-841) in one pass, fp64 included.
//
// MI355X design:
//  * The step is a chain of two dependent LDS round trips (table entry, then
//    the renormalisation word), so throughput comes from independent chains:
//    256-thread workgroups (4 waves), every wave one block pair (K = 1; fp64:
//    the pair's 2 streams) -- lanes 0-31 one block, lanes 32-63 the next (the
//    reference's 32-state interleaving) -- and many resident waves (more,
//    smaller waves beat 2-4 interleaved pairs per wave, DecCfg below).
//  * 64-bit decode table {pdf | sym << 24, slot - cdf}: the state update is
//    one v_mad_u32_u24 (u24 ignores the symbol byte); `entry >> 16` =
//    sym << 8 is stored with ds_write_b16_d16_hi, already the high byte of an
//    fp16 / bf16 word.  ds_read_b64 costs the LDS cycles of b32.
//  * The step is branch-free: per-half read pointers are SGPRs, the reader
//    index is v_mbcnt over the ballot, the ring read is unconditional and
//    the state update one v_perm.
//  * Compressed words are staged in a 512-word LDS ring per block stream,
//    refilled 256 words at a time (8 B per lane) from registers prefetched
//    at the previous refill; the initial fill holds a typical bf16 block's
//    whole stream.
//  * 8-step segments are unrolled (constant LDS offsets); each lane joins 8
//    words of the segment with their raw float bytes (loaded a segment
//    earlier) and writes them with 16 B stores.
#pragma once

#include <type_traits>

#include "device.h"

namespace dietgpu {

namespace dec {
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kRing = 512;      // u16 words per block-stream ring
constexpr uint32_t kRefill = 256;    // words per refill (64 lanes x 8 B)
constexpr uint32_t kWPL = kRefill / 64;  // words per lane per refill
constexpr uint32_t kSegSteps = 8;    // decode steps per output segment
constexpr uint32_t kSegWords = kSegSteps * 32;
constexpr uint32_t kUnroll = 4;      // steps between ring checks
constexpr uint32_t kChunk = kSegWords / 32;  // words joined per lane per segment
}  // namespace dec

// KK: block pairs per wave (0 = the default, 1).  One pair per wave beats
// 2-4 interleaved pairs per wave at every batch size measured (c2 decode
// 125 -> 102 us, c3 3.0 -> 2.3 ms): more, smaller waves hide the step's
// latency better and fill the chip without generation quantisation.
template <int FT, int KK = 0>
struct DecCfg {
  static constexpr int S = FloatTraits<FT>::kSegs;  // ANS streams per word
  static constexpr int K = KK ? KK : 1;             // block pairs per wave
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

// 4 compressed words at p (one 8 B load when aligned)
__device__ __forceinline__ u32x2 ld4w(gp<const uint16_t> p, bool vec) {
  if (vec) return *(gp<const u32x2>)p;
  return u32x2{uint32_t(p[0]) | (uint32_t(p[1]) << 16), uint32_t(p[2]) | (uint32_t(p[3]) << 16)};
}

// Prefetch words [max(0, lo - 256), lo) of one half (lane j: 4 words).  lo
// stays a multiple of 4, so the lanes cover the range exactly.
__device__ __forceinline__ void ringPrefetch(DStream& p, int hh, uint32_t lane, bool vec) {
  const int32_t nlo = max(0, p.lo[hh] - int32_t(dec::kRefill));
  if (p.lo[hh] > 0 && int32_t(dec::kWPL * lane) < p.lo[hh] - nlo)
    p.pf[hh] = ld4w(p.data[hh] + nlo + dec::kWPL * lane, vec);
}

// Before kUnroll steps: if fewer than 32 * kUnroll words are buffered below
// ptr, refill [lo - 256, lo) from the prefetch registers (the refill
// overwrites words >= lo + 256, all consumed since ptr < lo + 256) and
// prefetch the next 256 words.
__device__ __forceinline__ void ringEnsure(DStream& p, uint32_t lane, bool vec) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (p.lo[hh] > 0 && p.ptr[hh] - int32_t(32 * dec::kUnroll) < p.lo[hh]) {
      const int32_t nlo = max(0, p.lo[hh] - int32_t(dec::kRefill));
      if (int32_t(dec::kWPL * lane) < p.lo[hh] - nlo)
        *(lp<u32x2>)(p.ring + hh * dec::kRing + ((nlo + dec::kWPL * lane) & (dec::kRing - 1))) = p.pf[hh];
      p.lo[hh] = nlo;
      ringPrefetch(p, hh, lane, vec);
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
  const uint32_t v = p.ringLane[idx & (dec::kRing - 1)];  // harmless for non-readers
  // x = rd ? (xn << 16 | v) : xn as one v_perm.  Feeding the word through an
  // intrinsic (not a select) keeps the LDS read unconditional: a branch
  // around it would split the step and serialise the independent chains.
  p.x = __builtin_amdgcn_perm(xn, v, rd ? 0x05040100u : 0x07060504u);
  return e.x;
}

// All chains of a wave, one step each, in three phases separated by
// scheduling barriers: (A) every chain's table read, (B) every chain's state
// update, ballot and ring read, (C) every chain's v_perm.  Without the
// barriers the scheduler serialises the chains (one LDS round trip exposed
// per chain-step); with them the LDS latencies of the chains overlap.
// Returns the table entries' low words (sym in bits 24-31) in e0[].
template <bool kMask, int NC>
__device__ __forceinline__ void decStepAll(DStream* const (&p)[NC], const bool (&valid)[NC],
                                           lp<const u32x2> const (&lut)[NC], uint32_t mask, int pb,
                                           uint32_t hv, uint32_t (&e0)[NC]) {
  u32x2 e[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) e[c] = lut[c][p[c]->x & mask];
  __builtin_amdgcn_sched_barrier(0);
  uint32_t xn[NC], v[NC];
  bool rd[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    DStream& q = *p[c];
    xn[c] = __umul24(e[c].x, q.x >> pb) + e[c].y;
    if (kMask) xn[c] = valid[c] ? xn[c] : q.x;
    rd[c] = kMask ? (valid[c] && xn[c] < kMinState) : (xn[c] < kMinState);
    const uint64_t vote = ballot(rd[c]);
    const int32_t cLo = __popc(uint32_t(vote));
    const int32_t cHi = __popc(uint32_t(vote >> 32));
    const int32_t baseLo = q.ptr[0] - cLo;
    const int32_t diff = q.ptr[1] - q.ptr[0] - cHi;
    q.ptr[0] = baseLo;
    q.ptr[1] -= cHi;
    const uint32_t vbase = uint32_t(baseLo) + (hv & uint32_t(diff));
    const uint32_t idx = __builtin_amdgcn_mbcnt_hi(uint32_t(vote >> 32),
                                                   __builtin_amdgcn_mbcnt_lo(uint32_t(vote), vbase));
    v[c] = q.ringLane[idx & (dec::kRing - 1)];
    e0[c] = e[c].x;
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < NC; ++c)
    p[c]->x = __builtin_amdgcn_perm(xn[c], v[c], rd[c] ? 0x05040100u : 0x07060504u);
}

// Wave priority from the share of the wave's work still ahead (wave-uniform
// q in [0, 3]): the SIMD arbiter otherwise favours the oldest waves, so waves
// that started together finish up to ~35 % apart and the kernel ends on a
// tail with too few waves left to hide latency.
__device__ __forceinline__ void setPrioRemaining(uint32_t left, uint32_t total) {
  const uint32_t q = total ? min(3u, (4u * left) / total) : 0u;
  if (q == 3) __builtin_amdgcn_s_setprio(3);
  else if (q == 2) __builtin_amdgcn_s_setprio(2);
  else if (q == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// Join 8 decoded symbols (u16 sym << 8 in LDS) with their raw bytes.
template <int FT>
struct Join {
  using WordT = typename FloatTraits<FT>::WordT;
  // raw dwords per 8-word chunk
  static constexpr int kR = FT == 0 ? 1 : (FT <= 2 ? 2 : (FT == 3 ? 6 : 12));

  // raw bytes of the chunk starting at word i0 (i0 a multiple of 8)
  static __device__ __forceinline__ void load(uint32_t (&r)[kR], gp<const uint8_t> raw, uint32_t n,
                                              uint32_t i0) {
    if constexpr (FT == 1 || FT == 2) {
      const uint2 a = ld8(raw + i0);
      r[0] = a.x; r[1] = a.y;
    } else if constexpr (FT == 3) {
      const uint4 a = ld16(raw + 2 * i0);
      const uint2 h = ld8(raw + 2 * roundUp(n, 8) + i0);
      r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w; r[4] = h.x; r[5] = h.y;
    } else if constexpr (FT == 4) {
      const uint4 a = ld16(raw + 4 * i0), b = ld16(raw + 4 * i0 + 16);
      const uint4 h = ld16(raw + 4 * roundUp(n, 4) + 2 * i0);
      r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
      r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
      r[8] = h.x; r[9] = h.y; r[10] = h.z; r[11] = h.w;
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

  // vector join of a full chunk: out words [i0, i0 + 8).  nt: streaming
  // stores (the decoded output is not read again by the codec; not for fp64,
  // whose lanes write 64 B each in four stores: streaming partial lines
  // measured 2.5x slower).  s / s1: 4 dwords of
  // u16 (sym << 8) of stream 0 / 1.
  // NT: streaming (non-temporal) stores.  A compile-time choice: with a
  // runtime flag LLVM sinks the two stores of each branch into one and drops
  // the nontemporal hint.
  template <bool nt>
  static __device__ __forceinline__ void vec(gp<uint8_t> outB, uint32_t i0, const uint32_t (&s)[4],
                                             const uint32_t (&s1)[4], const uint32_t (&r)[kR]) {
    if constexpr (FT == 0) {
      const uint2 v = make_uint2(__builtin_amdgcn_perm(s[1], s[0], 0x07050301u),
                                 __builtin_amdgcn_perm(s[3], s[2], 0x07050301u));
      if constexpr (nt) st8nt(outB + i0, v);
      else st8(outB + i0, v);
    } else if constexpr (FT == 1 || FT == 2) {
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t t = pair16(s[k], r[k >> 1], k & 1);  // exp << 8 | raw per half
        // bf16: rotate each 16-bit half right by one (raw = mant << 1 | sign)
        o[k] = FT == 1 ? t : (((t >> 1) & 0x7fff7fffu) | ((t << 15) & 0x80008000u));
      }
      if constexpr (nt) st16nt(outB + 2 * i0, make_uint4(o[0], o[1], o[2], o[3]));
      else st16(outB + 2 * i0, make_uint4(o[0], o[1], o[2], o[3]));
    } else if constexpr (FT == 3) {
      uint32_t o[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t h = pair16(s[k], r[4 + (k >> 1)], k & 1);  // [hb, sym] x 2
        const uint32_t w0 = __builtin_amdgcn_perm(h, r[k], 0x05040100u);
        const uint32_t w1 = __builtin_amdgcn_perm(h, r[k], 0x07060302u);
        o[2 * k] = __builtin_amdgcn_alignbit(w0, w0, 1);
        o[2 * k + 1] = __builtin_amdgcn_alignbit(w1, w1, 1);
      }
      gp<uint4> d = (gp<uint4>)(outB + 4 * i0);
      if constexpr (nt) {
        st16nt(d, make_uint4(o[0], o[1], o[2], o[3]));
        st16nt(d + 1, make_uint4(o[4], o[5], o[6], o[7]));
      } else {
        st16(d, make_uint4(o[0], o[1], o[2], o[3]));
        st16(d + 1, make_uint4(o[4], o[5], o[6], o[7]));
      }
    } else {
      gp<uint4> d = (gp<uint4>)(outB + 8 * i0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // [s1, s0] pairs, then vhi = [h16, s1, s0] per word; w = rotr64(vhi:lo, 1)
        const uint32_t p = __builtin_amdgcn_perm(s[k], s1[k], 0x07030501u);
        const uint32_t vh0 = __builtin_amdgcn_perm(p, r[8 + k], 0x05040100u);
        const uint32_t vh1 = __builtin_amdgcn_perm(p, r[8 + k], 0x07060302u);
        const uint32_t l0 = r[2 * k], l1 = r[2 * k + 1];
        st16(d + k, make_uint4(__builtin_amdgcn_alignbit(vh0, l0, 1), __builtin_amdgcn_alignbit(l0, vh0, 1),
                               __builtin_amdgcn_alignbit(vh1, l1, 1), __builtin_amdgcn_alignbit(l1, vh1, 1)));
      }
    }
  }
};

// 64-bit decode table of one archive: entry[slot] = {pdf | sym << 24,
// slot - cdf[sym]} (packDecodeLookup, ans/GpuANSDecode.cuh:34-44, re-laid
// out for v_mad_u32_u24).  scratch: >= 2 * 256 + 4 dwords of LDS.
// Slot-parallel: each thread finds the symbol of its 2^pb / 256 slots by a
// binary search over the exclusive cdf (the largest s with cdf[s] <= slot,
// which always has pdf > 0), all of its slots' searches interleaved.  The
// symbol-parallel fill it replaces (each wave walking 64 symbols in turn)
// was a chain of 64 dependent LDS round trips: 5.5 of a one-block decode's
// 25 us.  Slots a corrupt table (pdf sum != 2^pb) leaves uncovered get a
// neighbouring symbol; none is written outside the table.
__device__ __forceinline__ void buildLut64(gp<const uint16_t> pdfIn, lp<u32x2> lut, int pb,
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
  constexpr int kG = 4;  // slots searched together
  const uint32_t total = 1u << pb;
#pragma unroll 1
  for (uint32_t g0 = tid; g0 < total; g0 += kG * dec::kThreads) {
    uint32_t s[kG], cs[kG];
#pragma unroll
    for (int j = 0; j < kG; ++j) s[j] = 0, cs[j] = 0;
#pragma unroll
    for (uint32_t bit = kNumSymbols / 2; bit; bit >>= 1) {
#pragma unroll
      for (int j = 0; j < kG; ++j) {
        const uint32_t cv = cdfS[s[j] + bit];
        const bool up = cv <= g0 + j * dec::kThreads;
        s[j] = up ? s[j] + bit : s[j];
        cs[j] = up ? cv : cs[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kG; ++j) {
      const uint32_t slot = g0 + j * dec::kThreads;
      if (slot < total) lut[slot] = u32x2{pdfS[s[j]] | (s[j] << 24), slot - cs[j]};
    }
  }
}

// grid (ceil(maxBlocks / (kBlocksPerWG * chunksPerWG)), batch), dynamic LDS
// DecCfg<FT>::ldsBytes(pb).  out.size(b) = capacity (bytes for raw ANS,
// words for floats).  Pointer tables may ride in the first (InlineTable) argument
// (BatchDesc::field).
// BAL: remaining-work wave priorities (single-generation grids).
// At most 80 SGPRs: a 256-thread workgroup of 82-96 SGPRs is admitted 7 times
// per CU, not 8, while the occupancy API still answers 8
// (MI355X_MICROARCH.md, Residency) -- the byte decoder's BAL instance had
// 82: the raw-ANS decodes of benchmark.py's shapes took 113-261 us instead
// of 77-180, their single-generation grids (sized by the API's answer) ran a
// second generation.  (fp64, VGPR-bound at four workgroups per CU, spills a
// few SGPRs to VGPR lanes instead: its decode time is unchanged.)
template <int FT, int KK, bool NT, bool BAL>
__global__ __launch_bounds__(dec::kThreads) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(4))) void k_decode(const InlineTable,
                                                          BatchDesc in, BatchDesc out,
                                                          uint32_t batchOffset, int pb,
                                                          uint32_t chunksPerWG,
                                                          uint8_t* __restrict__ outSuccess,
                                                          uint32_t* __restrict__ outSize) {
  using Cfg = DecCfg<FT, KK>;
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

  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, l = lane & 31;
  uint32_t hv = lane >= 32 ? ~0u : 0u;
  asm volatile("" : "+v"(hv));  // keep `hv & x` a v_and (not a v_cndmask pair)

  const bool vecIn = (reinterpret_cast<uintptr_t>(base) & 15) == 0;
  gp<uint8_t> outB = startOf(out, b);
  const bool vecOut = (reinterpret_cast<uintptr_t>(outB) & 15) == 0;
  gp<const uint8_t> raw = base + 32;
  const uint32_t mask = (1u << pb) - 1;
  lp<const u32x2> lut[S];
#pragma unroll
  for (int s = 0; s < S; ++s) lut[s] = (lp<const u32x2>)(L + s * (lutBytes / S));

  // A pass's loads that do not depend on its blockWords -- the initial states
  // and the raw float bytes of the first segment decoded (16 B-aligned full
  // segments; block sizes follow from n) -- go out together with the
  // blockWords, so that the blockWords -> ring fill chain no longer precedes
  // them (cold archives: three dependent HBM round trips per pass became
  // two).  The first pass's are issued before the decode-table build, whose
  // pdf load and LDS passes they then overlap.
  const bool vecIO = vecIn && vecOut;
  uint32_t x0[K][S];
  uint2 bwE[K][S][2];
  uint32_t rvA[K][R], rvB[K][R];
  auto issue = [&](uint32_t blk0) __attribute__((always_inline)) {
    const uint32_t off = dec::kChunk * l;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const uint32_t bkMine = blk0 + 2 * c + (lane >> 5);
      // the first segment decoded is the block pair's top one; full (and so
      // loadable unmasked) when both blocks of every pair are whole
      const uint32_t uwMin = min(blk0 + 2 * c + 1 < nBlocks ? min(kBlockSize, n - (blk0 + 2 * c + 1) * kBlockSize) : 0u,
                                 blk0 + 2 * c < nBlocks ? min(kBlockSize, n - (blk0 + 2 * c) * kBlockSize) : 0u);
      if (FT != 0 && vecIO && uwMin == kBlockSize)
        Join<FT>::load(rvA[c], raw, n, bkMine * kBlockSize + (kBlockSize / 32 / dec::kSegSteps - 1) * dec::kSegWords + off);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        gp<const uint8_t> states = arch[s] + kANSHeaderBytes + kPdfBytes;
        gp<const uint2> bw = (gp<const uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
        x0[c][s] = bkMine < nBlocks ? ((gp<const uint32_t>)(states + uint64_t(kStateBytesPerBlock) * bkMine))[l]
                                    : kMinState;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const uint32_t bk = blk0 + 2 * c + hh;
          bwE[c][s][hh] = bk < nBlocks ? ld8(bw + bk) : make_uint2(0, 0);
        }
      }
    }
  };
  {
    const uint32_t blk00 = blockIdx.x * chunksPerWG * Cfg::kBlocksPerWG + w * Cfg::kBlocksPerWave;
    if (blk00 < nBlocks) issue(blk00);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    buildLut64((gp<const uint16_t>)(arch[s] + kANSHeaderBytes),
               (lp<u32x2>)(L + s * (lutBytes / S)), pb, (uint32_t*)segAll);
    __syncthreads();
  }

  // Persistent over chunksPerWG consecutive chunks of this element (the grid
  // is one generation of resident workgroups; one table build per WG).
  for (uint32_t pass = 0; pass < chunksPerWG; ++pass) {
    const uint32_t blk0 = (blockIdx.x * chunksPerWG + pass) * Cfg::kBlocksPerWG + w * Cfg::kBlocksPerWave;
    if (blk0 >= nBlocks) break;
    if (pass > 0) issue(blk0);

    // per pair c: blocks blk0 + 2c (lanes 0-31) and blk0 + 2c + 1 (lanes 32-63)
    uint32_t uwH[K][2];  // wave-uniform: block sizes follow from n alone
    DStream st[K][S];
    lp<uint16_t> segLane[K][S];
#pragma unroll
    for (int c = 0; c < K; ++c)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const uint32_t bk = blk0 + 2 * c + hh;
        uwH[c][hh] = bk < nBlocks ? min(kBlockSize, n - bk * kBlockSize) : 0u;
      }
    uint32_t T = 0;
#pragma unroll
    for (int c = 0; c < K; ++c) T = max(T, max(divUp(uwH[c][0], 32), divUp(uwH[c][1], 32)));
    // segments [0, nFull) are full for every block of the wave; the partial
    // top segments (element tail / odd block count) are decoded first, masked
    uint32_t nFull = ~0u;
#pragma unroll
    for (int c = 0; c < K; ++c) nFull = min(nFull, min(uwH[c][0], uwH[c][1]) / dec::kSegWords);
    const int32_t nSeg = int32_t(divUp(T, dec::kSegSteps));
    const uint32_t off = dec::kChunk * l;  // this lane's chunk in a segment

    const bool rawEarly = FT != 0 && vecIO && nSeg > 0 && uint32_t(nSeg - 1) < nFull;
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
          d.ptr[hh] = 0;
          d.lo[hh] = 0;
          d.data[hh] = data;
          d.pf[hh] = u32x2{0, 0};
          if (bk < nBlocks) {
            const uint2 e = bwE[c][s][hh];
            const uint32_t ex = readfirst(e.x), ey = readfirst(e.y);  // wave-uniform: SGPRs
            const int32_t cw = int32_t(ex & 0xffffu);
            d.ptr[hh] = cw;
            d.data[hh] = data + ey;
            const int32_t lo =
                cw > int32_t(dec::kRing) ? int32_t(roundUp(uint32_t(cw) - dec::kRing, dec::kWPL)) : 0;
            d.lo[hh] = lo;
            // initial fill of [lo, cw) (<= 512 words: two wave-wide passes).
            // The last lane may copy up to 3 words past cw (the block's
            // 8-word padding) into slots below lo + 512: never a live slot.
#pragma unroll
            for (int q = 0; q < int(dec::kRing / dec::kRefill); ++q) {
              const int32_t a = lo + q * int32_t(dec::kRefill) + int32_t(dec::kWPL * lane);
              if (a < cw)
                *(lp<u32x2>)(d.ring + hh * dec::kRing + (a & (dec::kRing - 1))) = ld4w(d.data[hh] + a, vecIn);
            }
            ringPrefetch(d, hh, lane, vecIn);
          }
        }
        d.x = x0[c][s];
      }
    }

    DStream* chains[K * S];
    lp<const u32x2> lutC[K * S];
    bool allValid[K * S];
#pragma unroll
    for (int c = 0; c < K; ++c)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        chains[c * S + s] = &st[c][s];
        lutC[c * S + s] = lut[s];
        allValid[c * S + s] = true;
      }

    // kVec: 16 B aligned input and output (once per wave): full segments
    // then load and join unconditionally.
    auto run = [&](auto vecTag) {
      constexpr bool kVec = decltype(vecTag)::value;
      // raw float bytes, double-buffered: a full segment's bytes are loaded
      // before the previous segment's steps, a whole segment ahead of use
      auto loadRaw = [&](int32_t g, bool fullSeg, uint32_t (&rv)[K][R]) {
        const uint32_t segW0 = uint32_t(g) * dec::kSegWords;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
          const uint32_t bk = blk0 + 2 * c + (lane >> 5);
          if (FT != 0 && kVec && (fullSeg || segW0 + off + dec::kChunk <= uw))
            Join<FT>::load(rv[c], raw, n, bk * kBlockSize + segW0 + off);
        }
      };
      auto join = [&](int32_t g, bool fullSeg, const uint32_t (&rv)[K][R]) {
        const uint32_t segW0 = uint32_t(g) * dec::kSegWords;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
          const uint32_t bk = blk0 + 2 * c + (lane >> 5);
          if (!fullSeg && segW0 + off >= uw) continue;
          const uint32_t cnt = fullSeg ? dec::kChunk : min(dec::kChunk, uw - segW0 - off);
          const uint32_t i0 = bk * kBlockSize + segW0 + off;
          lp<const uint16_t> q0 = segLane[c][0] - l + off;
          lp<const uint16_t> q1 = segLane[c][S - 1] - l + off;
          if (kVec && cnt == dec::kChunk) {
            uint32_t sv[4], sv1[4];
            const u32x4 a0 = *(lp<const u32x4>)q0;
            sv[0] = a0.x; sv[1] = a0.y; sv[2] = a0.z; sv[3] = a0.w;
            if constexpr (S == 2) {
              const u32x4 b0 = *(lp<const u32x4>)q1;
              sv1[0] = b0.x; sv1[1] = b0.y; sv1[2] = b0.z; sv1[3] = b0.w;
            } else {
#pragma unroll
              for (int k = 0; k < 4; ++k) sv1[k] = 0;
            }
            Join<FT>::template vec<NT>(outB, i0, sv, sv1, rv[c]);
          } else {
            gp<WordT> o = (gp<WordT>)outB;
            for (uint32_t k = 0; k < cnt; ++k)
              o[i0 + k] = Join<FT>::one(q0[k] >> 8, q1[k] >> 8, raw, n, i0 + k);
          }
        }
      };

      if (nSeg > 0 && !(kVec && rawEarly)) loadRaw(nSeg - 1, uint32_t(nSeg - 1) < nFull, rvA);
      // partial segments (a pair with an element's tail block, or with no
      // second block at all): masked steps, unrolled like the full segments
      // (constant LDS offsets, the ring checked every kUnroll steps); steps
      // past a block's end are no-ops of the masked step.  A per-step loop
      // here cost such pairs 7-8 us (1 x 4096 words: decode 33.6 -> 25.7 us)
      for (int32_t g = nSeg - 1; g >= int32_t(nFull); --g) {
        const int32_t tBot = g * int32_t(dec::kSegSteps);
#pragma unroll
        for (int grp = int(dec::kSegSteps / dec::kUnroll) - 1; grp >= 0; --grp) {
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, kVec);
#pragma unroll
          for (int u = int(dec::kUnroll) - 1; u >= 0; --u) {
            const int tr = grp * int(dec::kUnroll) + u;
            const uint32_t t = uint32_t(tBot + tr);
            bool vld[K * S];
#pragma unroll
            for (int c = 0; c < K; ++c) {
              const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
#pragma unroll
              for (int s = 0; s < S; ++s) vld[c * S + s] = t * 32 + l < uw;
            }
            uint32_t e0[K * S];
            decStepAll<true, K * S>(chains, vld, lutC, mask, pb, hv, e0);
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
              for (int s = 0; s < S; ++s)
                if (vld[c * S + s]) segLane[c][s][tr * 32] = uint16_t(e0[c * S + s] >> 16);
          }
        }
        __builtin_amdgcn_wave_barrier();
        join(g, false, rvA);
        __builtin_amdgcn_wave_barrier();
        if (g > 0) loadRaw(g - 1, uint32_t(g - 1) < nFull, rvA);
      }
      // full segments: unrolled, unmasked
      auto fullSeg = [&](int32_t g, const uint32_t (&cur)[K][R], uint32_t (&nxt)[K][R]) {
        if constexpr (BAL)
          setPrioRemaining((chunksPerWG - 1 - pass) * uint32_t(nSeg) + uint32_t(g), chunksPerWG * uint32_t(nSeg));
        if (g > 0) loadRaw(g - 1, true, nxt);
#pragma unroll
        for (int grp = int(dec::kSegSteps / dec::kUnroll) - 1; grp >= 0; --grp) {
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, kVec);
#pragma unroll
          for (int u = int(dec::kUnroll) - 1; u >= 0; --u) {
            const int tr = grp * int(dec::kUnroll) + u;  // step within segment
            uint32_t e0[K * S];
            decStepAll<false, K * S>(chains, allValid, lutC, mask, pb, hv, e0);
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
              for (int s = 0; s < S; ++s) segLane[c][s][tr * 32] = uint16_t(e0[c * S + s] >> 16);
          }
        }
        __builtin_amdgcn_wave_barrier();
        join(g, true, cur);
        __builtin_amdgcn_wave_barrier();
      };
      int32_t g = min(nSeg, int32_t(nFull)) - 1;  // rvA holds segment g's bytes
      for (; g >= 1; g -= 2) {
        fullSeg(g, rvA, rvB);
        fullSeg(g - 1, rvB, rvA);
      }
      if (g == 0) fullSeg(0, rvA, rvB);
    };
    if (vecIn && vecOut)
      run(std::true_type{});
    else
      run(std::false_type{});
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace dietgpu
