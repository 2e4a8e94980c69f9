// Compression kernels for gfx950: histogram, table normalisation, fused
// float-split + rANS encode, and archive coalescing.
//
//   k_hist<FT>      histogramBatch (ans/GpuANSStatistics.cuh:21-143) and the
//                   histogram half of splitFloat (float/GpuFloatCompress.cuh:
//                   423-551)
//   k_normalize     quantizeWeights / normalizeProbabilitiesFromHistogram
//                   (ans/GpuANSStatistics.cuh:178-430)
//   k_encode<FT>    ansEncodeBatchFull/Partial (ans/GpuANSEncode.cuh:49-495)
//                   fused with the split half of splitFloat
//   k_coalesce<FT>  batchExclusivePrefixSum + ansEncodeCoalesceBatch
//                   (ans/BatchPrefixSum.cuh, ans/GpuANSEncode.cuh:497-668) +
//                   incOutputSizes / setHeaderAndANSOutOffset
//                   (float/GpuFloatCompress.cuh:557-667)
#pragma once

#include <type_traits>

#include "device.h"
#include "sync_arena.h"

namespace dietgpu {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kSlotBytes = kStateBytesPerBlock + kSlotDataBytes;

// Bit-exact restatement of normalizeProbabilitiesFromHistogram
// (ans/GpuANSStatistics.cuh:178-366) -- float32 quantisation, the diff > 0
// bump of symbol ids < diff, the diff < 0 decrement rounds over the
// descending (q << 16) | sym order -- by ONE wave, lane l holding symbols
// 4l + j (j < 4), in registers only: no workgroup barrier (the other waves of a
// workgroup work meanwhile) and no LDS round trip (queued behind the other
// workgroups' traffic, a dozen of them took microseconds).  c[j]: the
// counts in, the pdfs out; cdf[j]: the exclusive cumulative pdfs (symbol
// order).  total > 0.
//   Ranks: the keys (q << 16) | s of the g0 entries with q > 1 (the only ones
// ever decremented) are broadcast one at a time with v_readlane (g0 is a few
// dozen); rank = number of larger keys, i.e. the position in the
// reference's descending sort.  Rounds: the reference decrements ranks
// [g - k, g) of the g entries still > 1; those always form a prefix of the
// ranks (values stay in descending rank order: only the lowest-ranked are
// ever lowered), so an entry tests its own rank against g in place.
__device__ __forceinline__ void normalizeWave(uint32_t (&c)[4], uint32_t (&cdf)[4], uint32_t total, int pb) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t W = 1u << pb;
  uint32_t q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float r = __fdiv_rn(float(c[j]), float(total));
    q[j] = uint32_t(__fmul_rn(float(W), r));
    if (c[j] > 0 && q[j] == 0) q[j] = 1;
  }
  const int diff = int(W) - int(waveSum(q[0] + q[1] + q[2] + q[3]));
  if (diff > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      q[j] += uint32_t(diff) / kNumSymbols + (4 * lane + j < uint32_t(diff) % kNumSymbols ? 1u : 0u);
  } else if (diff < 0) {
    uint32_t key[4], rank[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) key[j] = (q[j] << 16) | (4 * lane + j);
    auto countAbove = [&](uint32_t kj, uint64_t m) __attribute__((always_inline)) {
      while (m) {
        const uint32_t src = uint32_t(__builtin_ctzll(m));
        m &= m - 1;
        const uint32_t kb = uint32_t(__builtin_amdgcn_readlane(int(kj), int(src)));
#pragma unroll
        for (int j = 0; j < 4; ++j) rank[j] += kb > key[j] ? 1u : 0u;
      }
    };
    countAbove(key[0], ballot(q[0] > 1));
    countAbove(key[1], ballot(q[1] > 1));
    countAbove(key[2], ballot(q[2] > 1));
    countAbove(key[3], ballot(q[3] > 1));
    int d = -diff;
    while (d > 0) {
      int g = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) g += __popcll(ballot(q[j] > 1));
      if (g == 0) break;  // reference asserts; unreachable for real tables
      const int k = d < g ? d : g;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (q[j] > 1 && int(rank[j]) >= g - k) q[j] -= 1;
      d -= k;
    }
  }
  const uint32_t lsum = q[0] + q[1] + q[2] + q[3];
  const uint32_t base = waveInclusiveScan(lsum) - lsum;
  cdf[0] = base;
  cdf[1] = base + q[0];
  cdf[2] = cdf[1] + q[1];
  cdf[3] = cdf[2] + q[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) c[j] = q[j];
}

// Encode table entry (internal, never archived) of a symbol with pdf q and
// cumulative frequency cdf:
//   x = pdf << (31 - pb)              renormalisation threshold
//   y = magic m                       x / pdf == umulhi(x, m) >> shift
//   z = cdf (+ 2^pb - 1 for pdf 1)
//   w = (2^pb - pdf) | shift << 24    x' = x + z + (x / pdf) * (2^pb - pdf)
// The dividend is the state after renormalisation, x < pdf << (31 - pb) <=
// 2^31, so a 32-bit magic suffices (Granlund-Montgomery, N = 31): with
// l = ceil(log2 q) >= 1, m = ceil(2^(31+l) / q) < 2^32 satisfies
// 2^(31+l) <= m q <= 2^(31+l) + 2^l, hence floor(x / q) =
// floor(x m / 2^(31+l)) = umulhi(x, m) >> (l - 1) for every x < 2^31: two
// VALU operations, not the three of the 33-bit magic ((umulhi + x) >> l).
// pdf 1 has no such magic; it takes m = 2^32 - 1, shift 0, i.e. the
// quotient x - 1 (x >= 16 there: renormalised states of a pdf-1 symbol are
// >= 2^15 or >= 2^(31-pb) >> 16), and the one missing (2^pb - 1) goes into
// z: x' = x 2^pb + cdf as the reference computes (ans/GpuANSEncode.cuh:63-89).
// Computed at compile time for every pdf 1 <= q <= 2^11 (a 64-bit division
// per symbol is ~100 VALU instructions).
__host__ __device__ constexpr uint32_t encMagic(uint32_t q, uint32_t* shift) {
  if (q <= 1) {
    *shift = 0;
    return q ? 0xffffffffu : 0u;
  }
  uint32_t l = 0;
  while ((1u << l) < q) ++l;
  *shift = l - 1;
  return uint32_t(((1ull << (31 + l)) + q - 1) / q);
}
struct MagicTable {
  uint32_t m[(1u << 11) + 1];
  constexpr MagicTable() : m() {
    for (uint32_t q = 1; q <= (1u << 11); ++q) {
      uint32_t sh = 0;
      m[q] = encMagic(q, &sh);
    }
  }
};
__device__ constexpr MagicTable kMagic{};

__device__ __forceinline__ uint4 encEntryPack(uint32_t q, uint32_t cdf, uint32_t magic, uint32_t shift,
                                              int pb) {
  const uint32_t z = cdf + (q == 1 ? (1u << pb) - 1 : 0u);
  return make_uint4(q << (kStateBits - pb), magic, z, ((1u << pb) - q) | (shift << 24));
}

__device__ __forceinline__ uint4 encTableEntry(uint32_t q, uint32_t cdf, int pb) {
  uint32_t shift = 0, magic = 0;
  if (q > 1) {
    shift = 31 - __clz(q - 1);  // ceil(log2 q) - 1
    magic = kMagic.m[q];
  } else if (q == 1) {
    magic = 0xffffffffu;
  }
  return encEntryPack(q, cdf, magic, shift, pb);
}

// The magic of pdf q >= 2 computed in registers (no dependent global load of
// kMagic on a latency-bound path): ceil(2^(32+shift) / q) from v_rcp_f64 and
// two Newton steps (any seed better than 2^-8 relative then lands within one
// of the quotient: it is below 2^32), and an exact fix-up -- the remainder
// 2^(32+shift) - m q is an integer below 2^13 in magnitude, so one fma yields
// it exactly.  About a quarter of the IEEE double division it replaced
// (v_div_scale / v_div_fmas / v_div_fixup and three 64-bit integer products
// per entry), which sat on the compressor's hand-off window.  Exhaustively
// checked against encMagic (dietgpu_test_enc_magic, tests/test_gpu_kat.py).
__device__ __forceinline__ uint32_t encMagicReg(uint32_t q, uint32_t shift) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double qd = double(q);
  double r = __builtin_amdgcn_rcp(qd);
  r = __builtin_fma(r, __builtin_fma(-qd, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-qd, r, 1.0), r);
  const int e = int(32 + shift);
  double m = __builtin_floor(__builtin_amdgcn_ldexp(r, e));
  double rem = __builtin_fma(-m, qd, __builtin_amdgcn_ldexp(1.0, e));
  if (rem < 0.0) {
    m -= 1.0;
    rem += qd;
  } else if (rem >= qd) {
    m += 1.0;
    rem -= qd;
  }
  return uint32_t(m) + (rem != 0.0 ? 1u : 0u);
#else
  uint32_t sh = 0;
  (void)shift;
  return encMagic(q, &sh);
#endif
}

__device__ __forceinline__ uint4 encTableEntryReg(uint32_t q, uint32_t cdf, int pb) {
  uint32_t shift = 0, magic = 0;
  if (q > 1) {
    shift = 31 - __clz(q - 1);
    magic = encMagicReg(q, shift);
  } else if (q == 1) {
    magic = 0xffffffffu;
  }
  return encEntryPack(q, cdf, magic, shift, pb);
}

// ---------------------------------------------------------------------------
// Normalisation of one (element, segment): sums the partial histograms,
// normalises (normalizeWave) and stores the encode table rows
// (encTableEntry) and the u16 pdf.  Run by k_normalize, or -- one launch
// fewer -- by the last workgroup to finish an element in the kernel that
// writes its final partial rows (k_hist or k_histReduce: NormArgs::arrive,
// the classic last-block reduction: every workgroup counts itself in after
// a release fence; the one that takes the count to its total, having
// acquired, sees every row).
// ---------------------------------------------------------------------------
// Column sums of `rows` rows of 256 u32 (row stride 256) by one workgroup:
// thread t loads 16 B (bins 4(t & 63) .. +3) of every fourth row (rows
// congruent to t >> 6), eight rows in flight, and the four row streams meet
// in LDS (`red4`: 256 x 16 B).  Returns bin t's sum.  A row per thread
// per load would expose one memory round trip per eight rows; this takes
// one per 32.
// kSc1: the rows were handed off inside this launch (sc1 stores, last
// arrival): every load of them is an sc1 load.
template <bool kSc1>
__device__ __forceinline__ uint32_t sumRows256(gp<const uint32_t> base, uint32_t rows, u32x4* red4) {
  const uint32_t t = threadIdx.x, q = t & 63, st = t >> 6;
  gp<const u32x4> p = (gp<const u32x4>)base + q;
  auto ld = [&](uint32_t r) { return kSc1 ? ldSc1x4(p + uint64_t(r) * (kNumSymbols / 4)) : p[uint64_t(r) * (kNumSymbols / 4)]; };
  u32x4 acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = u32x4{0, 0, 0, 0};
  uint32_t r = st;
  for (; r + 28 < rows; r += 32) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += ld(r + 4 * k);
  }
  for (; r < rows; r += 4) acc[0] += ld(r);
#pragma unroll
  for (int k = 1; k < 8; ++k) acc[0] += acc[k];
  __syncthreads();  // red4 free
  red4[st * 64 + q] = acc[0];
  __syncthreads();
  const uint32_t qq = t >> 2, j = t & 3;
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const u32x4 v = red4[k * 64 + qq];
    sum += j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
  }
  __syncthreads();  // red4 reusable
  return sum;
}

struct NormArgs {
  BatchDesc in;                 // symbol totals (element sizes)
  const uint32_t* hist;         // [segs][nb][rows][256] rows to sum
  uint32_t rows;
  int pb;
  uint4* table;                 // [segs][nb][256]
  uint16_t* pdf;                // [segs][nb][256]
  const uint32_t* partCk;       // [nb][ckRows] byte-checksum partials, or null
  uint32_t ckRows;
  uint32_t* ckOut;
  uint32_t* arrive;             // [nb] last-arrival counters (self-resetting), or null
  bool totalFromHist = false;   // the symbol total is the rows' sum (in.size unknown yet: sparse lists)
};

__device__ __forceinline__ void normalizeElement(const NormArgs& a, uint32_t numInBatch, uint32_t b,
                                                 uint32_t seg, uint32_t* keys, uint32_t* red, u32x4* red4) {
  const uint32_t s = threadIdx.x;
  const uint64_t row = uint64_t(seg) * numInBatch + b;
  // (arrive set: the last arrival of this launch, rows and checksum
  // partials handed off with sc1 stores, read with sc1 loads)
  const bool sc1 = a.arrive != nullptr;
  if (a.partCk && seg == 0 && s == 0) {
    uint32_t ck = 0;
    for (uint32_t c = 0; c < a.ckRows; ++c) {
      gp<const uint32_t> pc = G(a.partCk) + uint64_t(b) * a.ckRows + c;
      ck ^= sc1 ? ldSc1(pc) : *pc;
    }
    G(a.ckOut)[b] = ck;
  }
  gp<const uint32_t> rowsBase = G(a.hist) + row * a.rows * kNumSymbols;
  const uint32_t count = sc1 ? sumRows256<true>(rowsBase, a.rows, red4) : sumRows256<false>(rowsBase, a.rows, red4);

  const uint32_t total = a.totalFromHist ? blockSum<kThreads>(count, red) : a.in.size(b);
  if (total == 0) {  // :193-195 (the reference leaves the table untouched)
    st16(G(a.table) + row * kNumSymbols + s, make_uint4(0, 0, 0, 0));
    G(a.pdf)[row * kNumSymbols + s] = 0;
    return;
  }
  // one wave normalises in registers (normalizeWave: no workgroup barriers,
  // no LDS rank sort) and computes the table entries' magics in registers
  // (no dependent load of kMagic): on these latency-bound single-workgroup
  // tails that is most of the kernel
  keys[s] = count;
  __syncthreads();
  if (s < 64) {
    uint32_t c[4], cdf[4];
    const u32x4 kv = *(lp<const u32x4>)&keys[4 * s];
    c[0] = kv.x;
    c[1] = kv.y;
    c[2] = kv.z;
    c[3] = kv.w;
    normalizeWave(c, cdf, total, a.pb);
    gp<uint4> trow = G(a.table) + row * kNumSymbols + 4 * s;
#pragma unroll
    for (int j = 0; j < 4; ++j) st16(trow + j, encTableEntryReg(c[j], cdf[j], a.pb));
    st8((gp<uint8_t>)(G(a.pdf) + row * kNumSymbols + 4 * s), make_uint2(c[0] | (c[1] << 16), c[2] | (c[3] << 16)));
  }
  __syncthreads();  // keys reusable
}

// After this workgroup's rows of element b are stored -- with sc1 stores --
// true in the one workgroup that completes the element's `arrivals`.  The
// hand-off is MI355X_MICROARCH.md's counter form without fences: every
// storing wave waits for its sc1 stores, a barrier, then one lane's counter
// add; the last arrival reads the rows with sc1 loads only (an agent fence
// per workgroup writes back and invalidates the XCD's L2: 3.5 us each, c3's
// 1024 workgroups took 15 ms).  The counter wraps to 0 on the last arrival,
// ready for the next call.  Whole workgroup; `flag`: one LDS word.
__device__ __forceinline__ bool lastArrival(uint32_t* counter, uint32_t arrivals, uint32_t* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 row stores are done
  __syncthreads();
  if (threadIdx.x == 0) *flag = atomicInc(counter, arrivals - 1) == arrivals - 1 ? 1u : 0u;
  __syncthreads();
  return *flag != 0;
}

static __global__ __launch_bounds__(kThreads) void k_normalize(NormArgs a, uint32_t batchOffset,
                                                               uint32_t numInBatch) {
  __shared__ __attribute__((aligned(16))) uint32_t keys[kNumSymbols];
  __shared__ uint32_t red[kWaves];
  __shared__ u32x4 red4[kThreads];
  normalizeElement(a, numInBatch, batchOffset + blockIdx.x, blockIdx.y, keys, red, red4);
}

// ---------------------------------------------------------------------------
// k_hist: per-chunk symbol histogram(s) (+ byte-XOR checksum for raw bytes).
// grid (chunksPerElem, batch).  Each workgroup writes its 256 (x segs)
// partial counts without atomics; k_normalize sums them.  LDS counters are
// laid out bin-major with one column per lane of a 32-lane group
// (hs[sym * 32 + (lane & 31)]): every ds_add of a wave half hits 32
// distinct banks and never the same address, however skewed the symbol
// distribution (float exponents concentrate on a handful of values).
// fp64's two segments take 16 columns each (32 KB instead of 64: four
// workgroups per CU instead of two; c4 fp64 compress 128 -> 124 us), where
// lanes l and l + 16 of a wave half share a column.
// ---------------------------------------------------------------------------
constexpr int kHistCols = 32;
// kRows (small three-kernel grids, k_encode's prologue normalisation):
// chunk c adds its counts with atomics into row c % P of [segs][nb][P][256],
// P = proRowsOf(chunks) = min(chunks, kProRows) (this call's zeroed buffer of
// the sync arena), so the encoder sums P rows instead of a k_histReduce /
// k_normalize launch summing thousands; zero bins add nothing.  Sized by the
// chunk count, so a batch of many one-chunk elements holds one row per
// element and segment, not 64.  `zeroNext`: the same layout in the other
// buffer, zeroed here for the next call (SyncLease::rows).
constexpr uint32_t kProRows = 64;
__host__ __device__ constexpr uint32_t proRowsOf(uint32_t chunks) { return chunks < kProRows ? chunks : kProRows; }

template <int FT, bool kChecksum, bool kRows = false>
__global__ __launch_bounds__(kThreads) void k_hist(BatchDesc in, uint32_t batchOffset,
                                                   uint32_t numInBatch, uint32_t chunkWords,
                                                   uint32_t chunksPerElem,
                                                   uint32_t* __restrict__ partHist,
                                                   uint32_t* __restrict__ partCk, NormArgs na,
                                                   uint32_t* __restrict__ zeroNext = nullptr) {
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  // two segments (fp64): 16 columns each, so the counters take 32 KB and
  // four workgroups fit a CU (64 KB allowed two)
  constexpr int kHistCols = kSegs == 2 ? 16 : dietgpu::kHistCols;
  __shared__ __attribute__((aligned(16))) uint32_t hs[kSegs][kNumSymbols * kHistCols];
  __shared__ uint32_t red[kWaves];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t c = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  for (int s = 0; s < kSegs; ++s)
    for (uint32_t i = tid; i < kNumSymbols * kHistCols / 4; i += kThreads)
      *(lp<u32x4>)&hs[s][4 * i] = u32x4{0, 0, 0, 0};
  __syncthreads();

  const uint32_t size = in.size(b);
  const uint64_t begin = uint64_t(c) * chunkWords;
  uint32_t ck = 0;
  uint32_t* h0 = &hs[0][tid & (kHistCols - 1)];
  uint32_t* h1 = &hs[kSegs - 1][tid & (kHistCols - 1)];
  auto addWord = [&](WordT w) {
    atomicAdd(&h0[compOf<FT>(w, 0) * kHistCols], 1u);
    if constexpr (kSegs == 2) atomicAdd(&h1[compOf<FT>(w, 1) * kHistCols], 1u);
  };

  if (begin < size) {
    const uint32_t n = uint32_t(min(uint64_t(chunkWords), uint64_t(size) - begin));
    gp<const WordT> q = (gp<const WordT>)startOf(in, b) + begin;
    constexpr uint32_t kPerVec = 16 / sizeof(WordT);
    const uintptr_t qa = reinterpret_cast<uintptr_t>(q);
    uint32_t head = uint32_t(((16 - (qa & 15)) & 15) / sizeof(WordT));
    if ((qa & (sizeof(WordT) - 1)) != 0) head = n;
    head = min(head, n);
    for (uint32_t i = tid; i < head; i += kThreads) {
      const WordT w = q[i];
      addWord(w);
      if constexpr (kChecksum) ck ^= uint32_t(w);
    }
    gp<const uint4> q4 = (gp<const uint4>)(q + head);
    const uint32_t n4 = (n - head) / kPerVec;
    // software-pipelined main part: the next 4-vector batch is in flight
    // while the current one is counted (uniform trip count, so the loads
    // are unconditional and each wait is a counted vmcnt)
    constexpr uint32_t kB = 4 * kThreads;
    const uint32_t nIt = n4 / kB;
    uint32_t i = tid;
    auto count4 = [&](const uint4 (&v)[4]) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const WordT* ws = reinterpret_cast<const WordT*>(&v[k]);
#pragma unroll
        for (uint32_t j = 0; j < kPerVec; ++j) addWord(ws[j]);
        if constexpr (kChecksum) ck ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      }
    };
    if (nIt > 0) {
      uint4 cur[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) cur[k] = ld16(q4 + i + k * kThreads);
      for (uint32_t it = 1; it < nIt; ++it) {
        uint4 nxt[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) nxt[k] = ld16(q4 + i + kB + k * kThreads);
        count4(cur);
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
        i += kB;
      }
      count4(cur);
      i += kB;
    }
    for (; i < n4; i += kThreads) {
      const uint4 v = ld16(q4 + i);
      const WordT* ws = reinterpret_cast<const WordT*>(&v);
#pragma unroll
      for (uint32_t j = 0; j < kPerVec; ++j) addWord(ws[j]);
      if constexpr (kChecksum) ck ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    for (uint32_t t = head + n4 * kPerVec + tid; t < n; t += kThreads) {
      const WordT w = q[t];
      addWord(w);
      if constexpr (kChecksum) ck ^= uint32_t(w);
    }
  }
  __syncthreads();
  for (int s = 0; s < kSegs; ++s) {
    // bin tid: sum its 32 columns, rotated so the wave's reads spread banks
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kHistCols; ++k) sum += hs[s][tid * kHistCols + ((k + tid) & (kHistCols - 1))];
    if constexpr (kRows) {
      const uint32_t P = proRowsOf(chunksPerElem);
      const uint64_t row = (uint64_t(s) * numInBatch + b) * P + c % P;
      if (sum) __hip_atomic_fetch_add(G(partHist) + row * kNumSymbols + tid, sum, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
      if (c < P) G(zeroNext)[row * kNumSymbols + tid] = 0;
    } else {
      gp<uint32_t> dst = G(partHist) + ((uint64_t(s) * numInBatch + b) * chunksPerElem + c) * kNumSymbols + tid;
      if (na.arrive) stSc1(dst, sum);  // read by this launch's last arrival
      else *dst = sum;
    }
  }
  if constexpr (kChecksum) {
    ck = (ck ^ (ck >> 8) ^ (ck >> 16) ^ (ck >> 24)) & 0xffu;
    ck = waveXor(ck);
    if ((tid & 63) == 0) red[tid >> 6] = ck;
    __syncthreads();
    if (tid == 0) {
      gp<uint32_t> dst = G(partCk) + uint64_t(b) * chunksPerElem + c;
      if (na.arrive) stSc1(dst, red[0] ^ red[1] ^ red[2] ^ red[3]);
      else *dst = red[0] ^ red[1] ^ red[2] ^ red[3];
    }
  }
  // the element's last workgroup normalises it (hs is free: keys there)
  if (na.arrive && lastArrival(na.arrive + b, chunksPerElem, &red[0])) {
    for (int s = 0; s < kSegs; ++s) {
      normalizeElement(na, numInBatch, b, s, &hs[0][0], &hs[0][kNumSymbols],
                       reinterpret_cast<u32x4*>(&hs[0][2 * kNumSymbols]));
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// k_histReduce: first level of the partial-histogram sum when an element has
// many chunks (few large elements: one 128 MiB fp64 tensor is 2048 chunks,
// which k_normalize's single workgroup would sum serially for ~0.3 ms).
// grid (groups, batch, segments): workgroup g sums chunks [64g, 64g + 64) of
// its (element, segment) row, and the byte-checksum partials likewise.
// ---------------------------------------------------------------------------
constexpr uint32_t kReduceRows = 64;

static __global__ __launch_bounds__(kThreads) void k_histReduce(
    uint32_t batchOffset, uint32_t numInBatch, uint32_t chunksPerElem, uint32_t groups,
    const uint32_t* __restrict__ part, const uint32_t* __restrict__ partCk,
    uint32_t* __restrict__ outHist, uint32_t* __restrict__ outCk, NormArgs na, uint32_t segs) {
  __shared__ __attribute__((aligned(16))) uint32_t keys[kNumSymbols];
  __shared__ uint32_t red[kWaves + 1];
  __shared__ u32x4 red4[kThreads];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t g = blockIdx.x;
  const uint64_t row = uint64_t(blockIdx.z) * numInBatch + b;
  const uint32_t c0 = g * kReduceRows;
  const uint32_t c1 = min(chunksPerElem, c0 + kReduceRows);
  const uint32_t sum = sumRows256<false>(G(part) + (row * chunksPerElem + c0) * kNumSymbols, c1 - c0, red4);
  stSc1(G(outHist) + (row * groups + g) * kNumSymbols + threadIdx.x, sum);
  if (partCk && blockIdx.z == 0 && threadIdx.x < 64) {
    uint32_t ck = 0;
    for (uint32_t k = c0 + threadIdx.x; k < c1; k += 64) ck ^= G(partCk)[uint64_t(b) * chunksPerElem + k];
    ck = waveXor(ck);
    if (threadIdx.x == 0) stSc1(G(outCk) + uint64_t(b) * groups + g, ck);
  }
  // the (element, segment)'s last workgroup normalises that segment: fp64's
  // two segments are normalised by two workgroups side by side
  if (na.arrive && lastArrival(na.arrive + uint64_t(b) * segs + blockIdx.z, groups, &red[kWaves]))
    normalizeElement(na, numInBatch, b, blockIdx.z, keys, red, red4);
}

// ---------------------------------------------------------------------------
// k_encode: fused split + rANS encode.
//   * 256-thread workgroups (4 waves).  Lanes 0-31 / 32-63 of a wave code
//     one 4 KiB block each; each wave runs one block pair (fp64: with its
//     two streams) as independent chains.
//   * Per 512-symbol segment the wave splits 16 B input vectors (loaded one
//     segment ahead): float raw bytes go straight to the archive's raw
//     section, ANS symbols to LDS.  It then runs 16 branch-free encode steps
//     per block from LDS (fully unrolled).
//   * Emitted u16 words go to an LDS ring per block stream (writers at
//     ascending lane order, stored under an exec mask so
//     the step has no branch).  fp64 (512-word rings): flushed to the block's
//     scratch slot 256 words at a time with one 8 B store per lane, and
//     k_coalesce packs the slots into the archive.  Single-segment formats
//     (1024-word rings): only overflow is flushed; after the look-back the
//     workgroup copies its blocks from the rings (and slots) to the archive.
// ---------------------------------------------------------------------------
namespace enc {
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kSegSteps = 16;
constexpr uint32_t kSegWords = kSegSteps * 32;
constexpr uint32_t kRing = 512;    // u16 words per block-stream output ring
// Single-segment formats keep a block's whole typical output in LDS (a 4 KiB
// block at 4 bit/symbol is ~1.1 K words): only overflow beyond the ring goes
// through the slot, the rest is copied from LDS straight to its final place
constexpr uint32_t kRingFused = 1024;
constexpr uint32_t kFlush = 256;   // words per flush (64 lanes x 8 B)
constexpr uint32_t kUnroll = 4;    // steps between flush checks
}  // namespace enc

// KK: block pairs per wave (0 = the default, 1; see decode.h DecCfg: c2
// encode 111 -> 97 us against 2 pairs per wave).
template <int FT, int KK = 0>
struct EncCfg {
  using WordT = typename FloatTraits<FT>::WordT;
  static constexpr int S = FloatTraits<FT>::kSegs;
  static constexpr int K = KK ? KK : 1;
  static constexpr int kBlocksPerWave = 2 * K;
  static constexpr int kBlocksPerWG = enc::kWaves * kBlocksPerWave;
  // 16-byte input vectors per lane per block per segment (32 lanes x V x 16 B
  // = 512 words)
  static constexpr int V = int(enc::kSegWords * sizeof(WordT) / (32 * 16));
  static constexpr uint32_t kWordsPerVec = 16 / sizeof(WordT);
  static constexpr uint32_t kHalfStreams = enc::kWaves * K * S * 2;
};

// One ANS stream of one block pair.  All but x are wave-uniform.
struct EStream {
  uint32_t x;              // this lane's state
  lp<uint16_t> ring;       // output ring of half 0 (half 1 follows)
  lp<uint16_t> ringLane;   // this lane's half ring
  int32_t nout[2];         // per half: words emitted so far
  int32_t flushed[2];      // per half: words already in the slot
  gp<uint16_t> out[2];     // per half: slot data
};

// Flush 256 ring words of each half with >= kAt words pending.  Called with
// kAt = 256 at segment boundaries (before the next segment's loads are
// issued, so waits for those loads never drain fresh stores) and with
// kAt = 384 every kUnroll steps (only dense data gets there; it keeps the
// ring from overflowing: pending <= 383 + 128 < 512).
template <int kAt, uint32_t kRing = enc::kRing>
__device__ __forceinline__ void ringFlush(EStream& p, uint32_t lane) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (p.nout[hh] - p.flushed[hh] >= kAt) {
      const int32_t a = p.flushed[hh] + int32_t(4 * lane);
      *(gp<u32x2>)(p.out[hh] + a) = *(lp<const u32x2>)(p.ring + hh * kRing + (a & (kRing - 1)));
      p.flushed[hh] += enc::kFlush;
    }
  }
}

// Flush everything left (whole 4-word groups; the slot has room for them).
__device__ __forceinline__ void ringFlushAll(EStream& p, uint32_t lane) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    for (int32_t a0 = p.flushed[hh]; a0 < p.nout[hh]; a0 += int32_t(enc::kFlush)) {
      const int32_t a = a0 + int32_t(4 * lane);
      if (a < p.nout[hh])
        *(gp<u32x2>)(p.out[hh] + a) = *(lp<const u32x2>)(p.ring + hh * enc::kRing + (a & (enc::kRing - 1)));
    }
    p.flushed[hh] = p.nout[hh];
  }
}

// One rANS encode step (encodeOneWarp, ans/GpuANSEncode.cuh:49-90) of one
// stream of a block pair, given the symbol's table entry e; writers emit in
// ascending lane order.  hv: all-ones on lanes 32-63 (opaque to the
// compiler).  Masked (!valid) lanes neither write nor change state.
template <bool kMask, uint32_t kRing = enc::kRing>
__device__ __forceinline__ void encStep(EStream& p, bool valid, const u32x4& e, uint32_t hv) {
  bool wr = true;
  uint64_t vote;
  uint32_t x;  // the state after renormalisation
  if constexpr (kMask) {
    wr = valid && p.x >= e.x;
    vote = ballot(wr);
    x = wr ? (p.x >> kEncodedBits) : p.x;
  } else {
    // compare into VCC so the select is one v_cndmask with SDWA WORD_1 (x >> 16)
    static_assert(kEncodedBits == 16, "WORD_1 select");
    asm("v_cmp_ge_u32_e32 vcc, %2, %3\n\t"
        "v_cndmask_b32_sdwa %0, %2, %2, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
        "src1_sel:WORD_1\n\t"
        "s_mov_b64 %1, vcc"
        : "=v"(x), "=s"(vote)
        : "v"(p.x), "v"(e.x)
        : "vcc");
  }
  const int32_t cLo = __popc(uint32_t(vote));
  const int32_t cHi = __popc(uint32_t(vote >> 32));
  // write index = nout + (#writers of my half below me); v_mbcnt over 64
  // lanes counts every low-half writer for lanes 32-63.
  const int32_t diff = p.nout[1] - cLo - p.nout[0];
  const uint32_t vbase = uint32_t(p.nout[0]) + (hv & uint32_t(diff));
  p.nout[0] += cLo;
  p.nout[1] += cHi;
  const uint32_t idx = __builtin_amdgcn_mbcnt_hi(uint32_t(vote >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(uint32_t(vote), vbase));
  const uint32_t ringAddr = uint32_t(size_t(p.ringLane + (idx & (kRing - 1))));
  // writers store under an exec mask set in the asm itself: two SALU
  // instructions, no VALU select and no split of the step's control flow
  // (the LDS ops of a wave complete in order,
  // so the compiler's later lgkmcnt waits stay conservative; "memory" keeps
  // the ring reads of the flushes after it)
  uint64_t sav;
  asm volatile("s_and_saveexec_b64 %0, %1\n\tds_write_b16 %2, %3\n\ts_mov_b64 exec, %0"
               : "=&s"(sav)
               : "s"(vote), "v"(ringAddr), "v"(p.x)
               : "memory", "scc");
  (void)wr;
  const uint32_t q = __umulhi(x, e.y) >> (e.w >> 24);
  const uint32_t xn = __umul24(q, e.w) + x + e.z;  // u24 ignores the shift byte
  p.x = (!kMask || valid) ? xn : x;
}

// Split 16 B of input words: ANS symbols -> LDS (sym0 / sym1), raw remainder
// -> the archive raw section at word index i0 (splitFloat's per-word split,
// float/GpuFloatCompress.cuh:423-551; FloatTypeInfo::split,
// float/GpuFloatUtils.cuh:190-370).
// (store = false: symbols only, no raw-section store)
template <int FT>
__device__ __forceinline__ void splitVec(const uint4& v, uint32_t i0, uint32_t n,
                                         gp<uint8_t> raw, lp<uint8_t> sym0, lp<uint8_t> sym1,
                                         bool store = true) {
  using WordT = typename FloatTraits<FT>::WordT;
  const WordT* ws = reinterpret_cast<const WordT*>(&v);
  if constexpr (FT == 0) {
    *(lp<u32x4>)sym0 = u32x4{v.x, v.y, v.z, v.w};
  } else if constexpr (FT == 1 || FT == 2) {
    // words (lo, hi) of each dword; exponent / raw bytes gathered with v_perm
    const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
    uint32_t t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // bf16: rotate each half left by one so that [exp | raw] are the bytes
      t[k] = FT == 1 ? dw[k] : (((dw[k] << 1) & 0xfffefffeu) | ((dw[k] >> 15) & 0x00010001u));
    }
    const uint32_t e0 = __builtin_amdgcn_perm(t[1], t[0], 0x07050301u);
    const uint32_t e1 = __builtin_amdgcn_perm(t[3], t[2], 0x07050301u);
    const uint32_t r0 = __builtin_amdgcn_perm(t[1], t[0], 0x06040200u);
    const uint32_t r1 = __builtin_amdgcn_perm(t[3], t[2], 0x06040200u);
    *(lp<u32x2>)sym0 = u32x2{e0, e1};
    if (store) st8(raw + i0, make_uint2(r0, r1));
  } else if constexpr (FT == 3) {
    uint32_t r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = rotl32(ws[k], 1);
    *(lp<uint32_t>)sym0 = (__builtin_amdgcn_perm(r[1], r[0], 0x07030703u) & 0xffffu) |
                          (__builtin_amdgcn_perm(r[3], r[2], 0x07030703u) << 16);
    if (store) {
      st8(raw + 2 * i0, make_uint2(__builtin_amdgcn_perm(r[1], r[0], 0x05040100u),
                                   __builtin_amdgcn_perm(r[3], r[2], 0x05040100u)));
      *(gp<uint32_t>)(raw + 2 * roundUp(n, 8) + i0) =
          (__builtin_amdgcn_perm(r[1], r[0], 0x06020602u) & 0xffffu) |
          (__builtin_amdgcn_perm(r[3], r[2], 0x06020602u) << 16);
    }
  } else {
    const uint64_t r0 = rotl64(ws[0], 1), r1 = rotl64(ws[1], 1);
    *(lp<uint16_t>)sym0 = uint16_t((r0 >> 56) | ((r1 >> 56) << 8));
    *(lp<uint16_t>)sym1 = uint16_t(((r0 >> 48) & 0xffu) | (((r1 >> 48) & 0xffu) << 8));
    st8(raw + 4 * i0, make_uint2(uint32_t(r0), uint32_t(r1)));
    *(gp<uint32_t>)(raw + 4 * roundUp(n, 4) + 2 * i0) =
        uint32_t((r0 >> 32) & 0xffffu) | (uint32_t((r1 >> 32) & 0xffffu) << 16);
  }
}

// scalar split of one word (unaligned input or element tail)
template <int FT>
__device__ __forceinline__ void splitOne(typename FloatTraits<FT>::WordT w, uint32_t i, uint32_t n,
                                         gp<uint8_t> raw, lp<uint8_t> sym0, lp<uint8_t> sym1) {
  if constexpr (FT == 0) {
    *sym0 = w;
  } else if constexpr (FT == 1) {
    *sym0 = uint8_t(w >> 8);
    raw[i] = uint8_t(w);
  } else if constexpr (FT == 2) {
    *sym0 = uint8_t(w >> 7);
    raw[i] = uint8_t((w << 1) | (w >> 15));
  } else if constexpr (FT == 3) {
    const uint32_t v = rotl32(w, 1);
    *sym0 = uint8_t(v >> 24);
    ((gp<uint16_t>)raw)[i] = uint16_t(v);
    raw[2 * roundUp(n, 8) + i] = uint8_t(v >> 16);
  } else {
    const uint64_t v = rotl64(w, 1);
    *sym0 = uint8_t(v >> 56);
    *sym1 = uint8_t(v >> 48);
    ((gp<uint32_t>)raw)[i] = uint32_t(v);
    ((gp<uint16_t>)(raw + 4 * roundUp(n, 4)))[i] = uint16_t(v >> 32);
  }
}

// Payload copy of a run of nk consecutive blocks: the blocks are contiguous
// in the archive (block k at word pre[k], pre in LDS; cwL[k] words), so
// every thread copies 16 B vectors (8 words) across the whole range, the
// source slot found by binary search over pre; 4 vectors in flight per
// thread.  Words past a block's count are written as 0.
// With rings (k_encode, single-segment formats): words at or past flushed[k]
// are still in block k's LDS ring (rings + k * kR, index mod kR; flushed is a
// multiple of 256 and the vectors 8-word aligned, so a vector never straddles).
template <uint32_t kR = 0>
__device__ __forceinline__ void copyPayload(const uint32_t* pre, const uint32_t* cwL, uint32_t nk,
                                            gp<const uint8_t> slot0, gp<uint8_t> data,
                                            const uint16_t* rings = nullptr,
                                            const uint32_t* flushed = nullptr) {
  if (nk == 0) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t w0 = pre[0];
  const uint32_t nv = (pre[nk - 1] + roundUp(cwL[nk - 1], 8) - w0) / 8;
  gp<uint4> dst = (gp<uint4>)(data + 2ull * w0);
  constexpr int kIn = 4;
  for (uint32_t v0 = tid; v0 < nv; v0 += kIn * kThreads) {
    uint4 val[kIn];
    uint32_t valid[kIn];
#pragma unroll
    for (int q = 0; q < kIn; ++q) {
      const uint32_t v = v0 + q * kThreads;
      valid[q] = 0;
      if (v < nv) {
        const uint32_t w = w0 + 8 * v;
        uint32_t lo = 0, hi = nk;  // last k with pre[k] <= w
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pre[mid] <= w) lo = mid; else hi = mid;
        }
        const uint32_t off = w - pre[lo];
        valid[q] = cwL[lo] > off ? cwL[lo] - off : 0;
        if (kR && off >= flushed[lo]) {
          const u32x4 r = *(lp<const u32x4>)(rings + lo * kR + (off & (kR - 1)));
          val[q] = make_uint4(r[0], r[1], r[2], r[3]);
        } else {
          val[q] = ld16((gp<const uint4>)(slot0 + uint64_t(lo) * kSlotBytes + 2ull * off));
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kIn; ++q) {
      const uint32_t v = v0 + q * kThreads;
      if (v >= nv) continue;
      uint4 x = val[q];
      if (valid[q] < 8) {
        uint32_t* vw = reinterpret_cast<uint32_t*>(&x);
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
          if (2 * r + 1 >= valid[q]) vw[r] &= (2 * r < valid[q]) ? 0xffffu : 0u;
        }
      }
      st16(dst + v, x);
    }
  }
}

// ---------------------------------------------------------------------------
// Fused coalesce (single-segment formats).  Each encode workgroup publishes
// its blocks' word total and finds its archive offset by a decoupled
// look-back over the element's earlier workgroups (lower blockIdx.x: with
// the hardware's in-order dispatch within an XCD already running; any other
// order can only delay the wait, which is bounded and poisons instead of
// hanging), then writes its own blocks' blockWords and payload.  One 8 B
// flag per (element, workgroup), epoch-tagged in the sync arena: bits 63:62
// = 1 aggregate / 2 inclusive prefix, low 32 bits the value.  The value lives in the flag word itself, so a relaxed
// agent-scope 8 B store/load (sc1: written through, read past L1) is the
// whole hand-off.
// ---------------------------------------------------------------------------
struct EncTail {
  const uint16_t* pdf;  // normalised pdf rows (k_normalize)
  const uint32_t* ck;   // per-element checksum (k_normalize / k_checksum)
  uint32_t* outSize;
  uint64_t* flags;      // nW per element
  uint32_t nW;
  int pb;
  bool useChecksum;
  uint32_t spinCap = 1u << 24;  // look-back polls before the element is poisoned
  uint32_t* err = nullptr;      // device error word (poisoned elements)
  // sparse archives: element sizes whose header + bitmap precede this dense
  // archive (sparseOverhead), added to outSize; null otherwise
  const uint32_t* sparseN = nullptr;
  uint32_t skew = 0;  // test hook: emulated out-of-order start (skewDelay, device.h)
  uint32_t epoch = 0;  // this call's epoch: the flags are epoch-tagged (sync arena), never zeroed
  // prologue normalisation (k_encode<.., kPro>): k_hist's rowsPer
  // (proRowsOf(chunks)) rows per (segment, element), and (fp64) where
  // workgroup 0 leaves the pdf rows for k_coalesce
  const uint32_t* rows = nullptr;
  uint32_t rowsPer = kProRows;
  uint16_t* pdfOut = nullptr;
};

// Prologue normalisation of k_encode (small grids): every workgroup sums its
// element's P <= kProRows histogram rows per segment (k_hist<.., kRows>) and
// normalises them itself -- wave s segment s, in registers (normalizeWave)
// -- into its LDS encode table and pdf row.  The redundant work is a few
// microseconds at the start of a one-generation grid; the k_histReduce /
// k_normalize launch it replaces (a chain of dependent round trips over
// thousands of rows, plus its launch) cost ~10 us per call (c4 fp64,
// batch-1 float tensors).  red4: S * 256 16 B scratch.  Whole workgroup;
// the caller synchronises before reading tblS / pdfS.
template <int S>
__device__ __forceinline__ void proNormalize(gp<const uint32_t> rows, uint32_t P, uint32_t nb, uint32_t b,
                                             uint32_t n, int pb, lp<u32x4> red4,
                                             uint32_t (*tblS)[kNumSymbols * 4], uint16_t (*pdfS)[kNumSymbols]) {
  const uint32_t t = threadIdx.x, q = t & 63, st = t >> 6;
  constexpr uint32_t kPer = kProRows / 4;  // rows per thread (rows congruent to st mod 4)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    gp<const u32x4> p = (gp<const u32x4>)(rows + (uint64_t(s) * nb + b) * P * kNumSymbols) + q;
    // every row of this thread in flight at once (one round trip); rows past
    // P (wave-uniform) are not loaded
    u32x4 v[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      v[k] = st + 4 * k < P ? p[uint64_t(st + 4 * k) * (kNumSymbols / 4)] : u32x4{0, 0, 0, 0};
    u32x4 acc = u32x4{0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) acc += v[k];
    red4[s * kThreads + st * 64 + q] = acc;
  }
  __syncthreads();
  const uint32_t w = t >> 6;
  if (w < uint32_t(S)) {
    u32x4 a = red4[w * kThreads + q];
#pragma unroll
    for (uint32_t k = 1; k < 4; ++k) a += red4[w * kThreads + k * 64 + q];
    uint32_t c[4] = {a.x, a.y, a.z, a.w}, cdf[4] = {0, 0, 0, 0};
    if (n != 0) {
      normalizeWave(c, cdf, n, pb);
    } else {  // (ans/GpuANSStatistics.cuh:193-195: an empty element's table is zero)
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 e = n != 0 ? encTableEntryReg(c[j], cdf[j], pb) : make_uint4(0, 0, 0, 0);
      *(lp<u32x4>)&tblS[w][4 * (4 * q + j)] = u32x4{e.x, e.y, e.z, e.w};
    }
    *(lp<u32x2>)&pdfS[w][4 * q] = u32x2{c[0] | (c[1] << 16), c[2] | (c[3] << 16)};
  }
}

// bytes of a sparse archive before its dense part: 16 B header, bitmap
// padded to 16 (float/GpuSparseFloatCompress.cuh)
__device__ __forceinline__ uint64_t sparseOverhead(const uint32_t* sparseN, uint32_t b) {
  return sparseN ? 16ull + roundUp64((uint64_t(sparseN[b]) + 7) / 8, 16) : 0ull;
}

constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPrefix = 2ull << 62;
constexpr uint64_t kFlagPoisonE = 1ull << 61;

// Decoupled look-back over earlier members [0, x) of
// an element, with epoch-tagged, poison-carrying flags: bits 63:62 status (1 aggregate, 2
// inclusive prefix), 61 poison, 47:32 epoch, 31:0 value.  A flag of another
// epoch reads as "not yet published".  Whole wave; returns the sum of the
// values of members [0, x); `poison` in: this member's own, out: whether any
// member [0, x] is poisoned (or the wait ran out of polls).
// (storeOwn = false: this member's aggregate flag is already published)
__device__ __forceinline__ uint32_t lookBackPoison(gp<uint64_t> f, uint32_t x, uint32_t agg,
                                                   uint32_t epoch, uint32_t cap, bool& poison,
                                                   bool storeOwn = true) {
  const uint32_t lane = laneId();
  const uint64_t tag = uint64_t(epoch) << 32;
  const uint64_t own = poison ? kFlagPoisonE : 0ull;
  if (storeOwn && lane == 0)
    __hip_atomic_store(f + x, (x == 0 ? kFlagPrefix : kFlagAgg) | own | tag | agg, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (x == 0) return 0;
  uint32_t excl = 0;
  uint64_t pz = 0;
  bool done = false;
  int32_t j = int32_t(x);
  for (uint32_t spins = 0; spins < cap;) {
    const int32_t k = j - 1 - int32_t(lane);
    const uint64_t v = k >= 0 ? __hip_atomic_load(f + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : (kFlagPrefix | tag);
    const uint32_t hi = uint32_t(v >> 32);
    const uint32_t status = (hi & kEpochMask) == epoch ? hi >> 30 : 0u;
    const uint64_t isPre = ballot(status == 2);
    const uint64_t isZero = ballot(status == 0);
    const uint32_t firstPre = isPre ? uint32_t(__builtin_ctzll(isPre)) : 64u;
    const uint64_t need = firstPre >= 63 ? ~0ull : (2ull << firstPre) - 1;
    if (isZero & need) {
      __builtin_amdgcn_s_sleep(2);
      ++spins;
      continue;
    }
    excl += waveSum(lane <= firstPre ? uint32_t(v) : 0u);
    pz |= ballot(lane <= firstPre && (v & kFlagPoisonE) != 0);
    if (firstPre < 64) {
      done = true;
      break;
    }
    j -= 64;
  }
  poison = poison || pz != 0 || !done;
  if (lane == 0)
    __hip_atomic_store(f + x, kFlagPrefix | (poison ? kFlagPoisonE : 0ull) | tag | uint64_t(excl + agg),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// Header fields known before encoding (all but the word totals): ANS header
// words 0-2 and 4-7, the pdf table, float header words 0-3 and 5-7, and the
// raw section's rounding tails.  Whole workgroup.
template <int FT>
__device__ __forceinline__ void writeHeadFixed(gp<uint8_t> base, gp<uint8_t> o, uint32_t n, uint32_t nBlocks,
                               const EncTail& t, uint32_t b, uint16_t pdfOfTid) {
  const uint32_t tid = threadIdx.x;
  const bool ansCk = FT == 0 && t.useChecksum;
  if (tid == 0) {
    gp<uint32_t> hdr = (gp<uint32_t>)o;
    hdr[0] = kANSMagicVersion;
    hdr[1] = nBlocks;
    hdr[2] = n;
    hdr[4] = uint32_t(t.pb) | (ansCk ? 0x10u : 0u);
    hdr[5] = ansCk ? G(t.ck)[b] : 0u;
    hdr[6] = 0;
    hdr[7] = 0;
    if constexpr (FT != 0) {
      gp<uint32_t> fh = (gp<uint32_t>)base;
      fh[0] = kFloatMagicVersion;
      fh[1] = n;
      fh[2] = uint32_t(FT) | (t.useChecksum ? 0x10u : 0u);
      fh[3] = t.useChecksum ? G(t.ck)[b] : 0u;
      fh[5] = 0;
      fh[6] = 0;
      fh[7] = 0;
    }
  }
  ((gp<uint16_t>)(o + kANSHeaderBytes))[tid] = pdfOfTid;
  if constexpr (FT != 0) {
    if (tid < 16) {
      gp<uint8_t> raw = base + 32;
      if constexpr (FT == 1 || FT == 2) {
        if (n + tid < roundUp(n, 16)) raw[n + tid] = 0;
      } else {
        static_assert(FT == 3, "single-segment float formats only");
        if (n + tid < roundUp(n, 8)) ((gp<uint16_t>)raw)[n + tid] = 0;
        if (n + tid < roundUp(n, 16)) raw[2 * roundUp(n, 8) + n + tid] = 0;
      }
    }
  }
}

// The fields that need the element's word total (last workgroup, one lane).
template <int FT>
__device__ __forceinline__ void writeHeadTotal(gp<uint8_t> base, gp<uint8_t> o, uint32_t n, uint32_t nBlocks,
                               uint32_t totalWords, gp<uint2> bwords, const EncTail& t, uint32_t b) {
  ((gp<uint32_t>)o)[3] = totalWords;
  if (nBlocks & 1) st8(bwords + nBlocks, make_uint2(0, 0));
  const uint64_t ansBytes = ansOverhead(nBlocks) + 2ull * totalWords;
  uint64_t sz = ansBytes;
  if constexpr (FT != 0) {
    ((gp<uint32_t>)base)[4] = uint32_t(roundUp64(ansBytes, 16));  // GpuFloatHeader2
    sz += 32ull + floatRawBytes(FT, n);
  }
  sz += sparseOverhead(t.sparseN, b);
  if (t.outSize) G(t.outSize)[b] = uint32_t(sz);
}

// grid (max(1, ceil(MB / kBlocksPerWG)), batch).  Single-segment formats
// (kFused): writes the whole archive (states straight to it, words via the
// slots, see EncTail).  fp64: writes per block slot states, slot words and
// cw[] (word count) for k_coalesce.
template <int FT, int KK, bool kPro = false>
__global__ __launch_bounds__(enc::kThreads) void k_encode(BatchDesc in, BatchDesc out,
                                                          uint32_t batchOffset,
                                                          uint32_t numInBatch, uint32_t MB,
                                                          const uint4* __restrict__ table,
                                                          uint8_t* __restrict__ slots,
                                                          uint32_t* __restrict__ cw, EncTail tail) {
  using Cfg = EncCfg<FT, KK>;
  using WordT = typename Cfg::WordT;
  constexpr int S = Cfg::S, K = Cfg::K, V = Cfg::V;
  constexpr bool kFused = S == 1;
  constexpr uint32_t R = kFused ? enc::kRingFused : enc::kRing;
  static_assert(!kFused || K == 1, "fused copy addresses block k's ring at k * R");
  __shared__ __attribute__((aligned(16))) uint32_t tblS[S][kNumSymbols * 4];
  __shared__ __attribute__((aligned(16))) uint8_t symS[Cfg::kHalfStreams][enc::kSegWords];
  __shared__ __attribute__((aligned(16))) uint16_t ringS[Cfg::kHalfStreams / 2][2 * R];
  __shared__ uint32_t cwE[Cfg::kBlocksPerWG];
  __shared__ uint32_t flE[Cfg::kBlocksPerWG];
  __shared__ uint32_t preE[Cfg::kBlocksPerWG];
  __shared__ uint32_t cwSeg[kFused ? 1 : S][Cfg::kBlocksPerWG];  // fp64: word counts per segment
  __shared__ __attribute__((aligned(16))) uint16_t pdfS[kPro ? S : 1][kNumSymbols];
  static_assert(sizeof(ringS) >= S * kThreads * 16, "prologue scratch in the rings");

  const uint32_t tid = threadIdx.x;
  // (chunk, element) = blockIdx: the fused look-back waits on lower chunks of
  // the same element (see lookBackPoison's caller below).  A start ticket
  // here (one atomic per workgroup on a shared counter) serialised the
  // starts of the big grids: c3 encode 2.35 -> 2.68 ms, batch-1 bf16
  // 62 -> 80 us.
  const uint32_t wx = blockIdx.x, wy = blockIdx.y;
  if (kFused && tail.skew && tid == 0) skewDelay(tail.skew);  // test hook (dietgpu_set_dispatch_skew)
  const uint32_t b = batchOffset + wy;
  const uint32_t n = in.size(b);
  const uint32_t nBlocks = divUp(n, kBlockSize);
  const uint32_t first = wx * Cfg::kBlocksPerWG;
  // workgroup 0 of an element always runs (headers, empty elements; with
  // kPro also the pdf rows k_coalesce reads)
  if (first >= nBlocks && ((!kFused && !kPro) || wx != 0)) return;
  gp<uint8_t> base = startOf(out, b);
  gp<uint8_t> o = base + (FT == 0 ? 0u : 32u + floatRawBytes(FT, n));  // ANS archive
  gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
  gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
  if constexpr (kPro) {
    proNormalize<S>(G(tail.rows), tail.rowsPer, numInBatch, b, n, tail.pb, (lp<u32x4>)&ringS[0][0], tblS, pdfS);
    __syncthreads();
    if (!kFused && wx == 0) {
#pragma unroll
      for (int s = 0; s < S; ++s) G(tail.pdfOut)[(uint64_t(s) * numInBatch + b) * kNumSymbols + tid] = pdfS[s][tid];
    }
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint4 t = ld16(G(table) + (uint64_t(s) * numInBatch + b) * kNumSymbols + tid);
      *(lp<u32x4>)&tblS[s][4 * tid] = u32x4{t.x, t.y, t.z, t.w};
    }
    __syncthreads();
  }

  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, h = lane >> 5, l = lane & 31;
  const uint32_t blk0 = first + w * Cfg::kBlocksPerWave;
  if (blk0 < nBlocks) {
  uint32_t hv = h ? ~0u : 0u;
  asm volatile("" : "+v"(hv));  // keep `hv & x` a v_and

  gp<const WordT> src = (gp<const WordT>)startOf(in, b);
  gp<uint8_t> raw = FT == 0 ? gp<uint8_t>(nullptr) : startOf(out, b) + 32;
  const bool vecIn = (reinterpret_cast<uintptr_t>(src) & 15) == 0;

  uint32_t uwH[K][2];  // wave-uniform
  uint32_t blk[K], uw[K];
  EStream st[K][S];
  lp<uint8_t> symLane[K][S];
#pragma unroll
  for (int c = 0; c < K; ++c) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint32_t bk = blk0 + 2 * c + hh;
      uwH[c][hh] = bk < nBlocks ? min(kBlockSize, n - bk * kBlockSize) : 0u;
    }
    blk[c] = blk0 + 2 * c + h;
    uw[c] = h ? uwH[c][1] : uwH[c][0];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      EStream& p = st[c][s];
      const uint32_t hs = (w * K + c) * S + s;
      p.x = kStartState;
      p.ring = (lp<uint16_t>)&ringS[hs][0];
      p.ringLane = p.ring + (hv & R);
      symLane[c][s] = (lp<uint8_t>)&symS[2 * hs][0] + (hv & enc::kSegWords) + l;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const uint32_t bk = blk0 + 2 * c + hh;
        const uint32_t sb = bk < nBlocks ? bk : blk0;
        p.nout[hh] = 0;
        p.flushed[hh] = 0;
        p.out[hh] = (gp<uint16_t>)(G(slots) + ((uint64_t(s) * numInBatch + b) * MB + sb) * kSlotBytes +
                                   kStateBytesPerBlock);
      }
    }
  }
  uint32_t T = 0;
#pragma unroll
  for (int c = 0; c < K; ++c) T = max(T, max(divUp(uwH[c][0], 32), divUp(uwH[c][1], 32)));
  const uint32_t nSeg = divUp(T, enc::kSegSteps);

  lp<const u32x4> tbl[S];
#pragma unroll
  for (int s = 0; s < S; ++s) tbl[s] = (lp<const u32x4>)&tblS[s][0];

  // segments [0, nFull) are full for every block of the wave
  uint32_t nFull = ~0u;
#pragma unroll
  for (int c = 0; c < K; ++c)
    nFull = min(nFull, min(uwH[c][0], uwH[c][1]) / enc::kSegWords);

  // kVec: 16 B aligned input (chosen once per wave).  With it, full
  // segments split unconditionally, so the prefetch registers are always
  // consumed before they are reloaded (no vmcnt(0) drain of the stores).
  auto run = [&](auto vecTag) {
    constexpr bool kVec = decltype(vecTag)::value;
    uint4 pv[K][V];  // input vectors, one segment ahead
    auto loadSeg = [&](uint32_t g) {
#pragma unroll
      for (int c = 0; c < K; ++c) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const uint32_t j0 = g * enc::kSegWords + (k * 32 + l) * Cfg::kWordsPerVec;
          if (kVec && (g < nFull || j0 + Cfg::kWordsPerVec <= uw[c]))
            pv[c][k] = ld16(src + blk[c] * kBlockSize + j0);
        }
      }
    };
    // split segment g: symbols -> LDS, raw -> archive
    auto split = [&](uint32_t g, bool fullSeg) {
      const uint32_t segW0 = g * enc::kSegWords;
#pragma unroll
      for (int c = 0; c < K; ++c) {
        if (!fullSeg && uw[c] <= segW0) continue;
        const uint32_t segCnt = fullSeg ? enc::kSegWords : min(enc::kSegWords, uw[c] - segW0);
#pragma unroll
        for (int k = 0; k < V; ++k) {
          const uint32_t off = (k * 32 + l) * Cfg::kWordsPerVec;  // word offset in segment
          lp<uint8_t> s0 = symLane[c][0] - l + off;
          lp<uint8_t> s1 = symLane[c][S - 1] - l + off;
          const uint32_t i0 = blk[c] * kBlockSize + segW0 + off;
          if (kVec && (fullSeg || off + Cfg::kWordsPerVec <= segCnt)) {
            splitVec<FT>(pv[c][k], i0, n, raw, s0, s1);
          } else {
            for (uint32_t q = 0; q < Cfg::kWordsPerVec && off + q < segCnt; ++q)
              splitOne<FT>(src[i0 + q], i0 + q, n, raw, s0 + q, s1 + q);
          }
        }
      }
    };

    if (nSeg > 0) loadSeg(0);
    for (uint32_t g = 0; g < nFull; ++g) {
      split(g, true);
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int s = 0; s < S; ++s) ringFlush<int(R - 256), R>(st[c][s], lane);
      if (g + 1 < nSeg) loadSeg(g + 1);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int grp = 0; grp < int(enc::kSegSteps / enc::kUnroll); ++grp) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) ringFlush<int(R - 128), R>(st[c][s], lane);
        // the group's symbols and table entries first: their LDS reads
        // cannot be hoisted over the ring stores of earlier steps
        u32x4 E[enc::kUnroll][K][S];
#pragma unroll
        for (int u = 0; u < int(enc::kUnroll); ++u)
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s)
              E[u][c][s] = tbl[s][symLane[c][s][(grp * int(enc::kUnroll) + u) * 32]];
#pragma unroll
        for (int u = 0; u < int(enc::kUnroll); ++u)
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) encStep<false, R>(st[c][s], true, E[u][c][s], hv);
      }
      __builtin_amdgcn_wave_barrier();
    }
    // partial segments (element tail / odd block counts): masked steps,
    // unrolled like the full segments (groups of kUnroll steps, the ring
    // checked once per group, table reads ahead); steps past a block's end
    // are no-ops of the masked step
    for (uint32_t g = nFull; g < nSeg; ++g) {
      split(g, false);
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int s = 0; s < S; ++s) ringFlush<int(R - 256), R>(st[c][s], lane);
      if (g + 1 < nSeg) loadSeg(g + 1);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int grp = 0; grp < int(enc::kSegSteps / enc::kUnroll); ++grp) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) ringFlush<int(R - 128), R>(st[c][s], lane);
        u32x4 E[enc::kUnroll][K][S];
        bool vd[enc::kUnroll][K];
#pragma unroll
        for (int u = 0; u < int(enc::kUnroll); ++u) {
          const uint32_t tr = uint32_t(grp * int(enc::kUnroll) + u);
          const uint32_t t = g * enc::kSegSteps + tr;
#pragma unroll
          for (int c = 0; c < K; ++c) {
            vd[u][c] = t * 32 + l < uw[c];
#pragma unroll
            for (int s = 0; s < S; ++s)
              E[u][c][s] = tbl[s][vd[u][c] ? uint32_t(symLane[c][s][tr * 32]) : 0u];
          }
        }
#pragma unroll
        for (int u = 0; u < int(enc::kUnroll); ++u)
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) encStep<true, R>(st[c][s], vd[u][c], E[u][c][s], hv);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_wave_barrier();
    }
  };
  if (vecIn)
    run(std::true_type{});
  else
    run(std::false_type{});

#pragma unroll
  for (int c = 0; c < K; ++c) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      EStream& p = st[c][s];
      if constexpr (!kFused) ringFlushAll(p, lane);  // fused: the rest stays in LDS
      if (uw[c]) {
        const uint32_t words = uint32_t(h ? p.nout[1] : p.nout[0]);
        if constexpr (kFused) {
          ((gp<uint32_t>)(states + uint64_t(kStateBytesPerBlock) * blk[c]))[l] = p.x;
          if (l == 0) {
            cwE[blk[c] - first] = words;
            flE[blk[c] - first] = uint32_t(h ? p.flushed[1] : p.flushed[0]);
          }
        } else {
          gp<uint8_t> slot = G(slots) + ((uint64_t(s) * numInBatch + b) * MB + blk[c]) * kSlotBytes;
          ((gp<uint32_t>)slot)[l] = p.x;
          if (l == 0) {
            G(cw)[(uint64_t(s) * numInBatch + b) * MB + blk[c]] = words;
            cwSeg[kFused ? 0 : s][blk[c] - first] = words;
          }
        }
      }
    }
  }
  }  // blk0 < nBlocks
  if constexpr (!kFused) {
    // fp64: one decoupled look-back per segment over the element's
    // workgroups (wave s: segment s, side by side), so that k_coalesce reads
    // each block range's prefix from the look-back flags instead of summing
    // every earlier block's word count (quadratic in the blocks: a 1e8-word
    // fp64 element's coalesce took 129 us for 211 MB).  The flags end as
    // inclusive prefixes, per (segment, element, workgroup).
    if (tail.flags) {
      __syncthreads();
      const uint32_t nk = first < nBlocks ? min(uint32_t(Cfg::kBlocksPerWG), nBlocks - first) : 0u;
      if (w < uint32_t(S) && nk > 0) {
        const uint32_t r = lane < nk ? roundUp(cwSeg[w][lane], 8) : 0u;
        const uint32_t agg = readfirst(__shfl(waveInclusiveScan(r), 63));
        bool pz = false;
        (void)lookBackPoison(G(tail.flags) + (uint64_t(w) * numInBatch + b) * tail.nW, wx, agg, tail.epoch,
                             tail.spinCap, pz);
      }
    }
  }
  if constexpr (kFused) {
    // every wave's slot stores are complete before other waves copy them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t nk = first < nBlocks ? min(uint32_t(Cfg::kBlocksPerWG), nBlocks - first) : 0u;
    if (w == 0) {
      const uint32_t r = lane < nk ? roundUp(cwE[lane], 8) : 0u;
      const uint32_t inc = waveInclusiveScan(r);
      const uint32_t agg = readfirst(__shfl(inc, 63));
      bool pz = false;
      const uint32_t excl = lookBackPoison(G(tail.flags) + uint64_t(b) * tail.nW, wx, agg, tail.epoch, tail.spinCap, pz);
      if (lane < nk) preE[lane] = excl + inc - r;
      if (lane == 0 && (first + Cfg::kBlocksPerWG >= nBlocks)) {
        if (pz) {
          if (tail.outSize) G(tail.outSize)[b] = 0u;
          __hip_atomic_fetch_add(G(tail.err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          writeHeadTotal<FT>(base, o, n, nBlocks, excl + agg, bwords, tail, b);
        }
      }
    }
    if (wx == 0)
      writeHeadFixed<FT>(base, o, n, nBlocks, tail, b,
                         kPro ? pdfS[0][tid] : G(tail.pdf)[uint64_t(b) * kNumSymbols + tid]);
    __syncthreads();
    if (tid < nk) {
      const uint32_t k = first + tid;
      const uint32_t uwk = min(kBlockSize, n - k * kBlockSize);
      st8(bwords + k, make_uint2((uwk << 16) | cwE[tid], preE[tid]));
    }
    copyPayload<R>(preE, cwE, nk, G(slots) + (uint64_t(b) * MB + first) * kSlotBytes + kStateBytesPerBlock,
                   (gp<uint8_t>)(bwords + roundUp(nBlocks, 2)), &ringS[0][0], flE);
  }
}

// ---------------------------------------------------------------------------
// k_coalesce: grid (ceil(maxBlocks / blocksPerWG), batch, segments).  Each
// workgroup recomputes its element's block prefix (sum of roundUp(cw, 8)
// before its range + a block scan of its own range), copies its blocks'
// states and words into the final archive; workgroup 0 writes the header(s),
// the pdf table and the output size.  Pad words are written as 0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sumRoundedWords(gp<const uint32_t> cw, uint32_t n,
                                                    uint32_t* red) {
  uint32_t v = 0;
  for (uint32_t i = threadIdx.x; i < n; i += kThreads) v += roundUp(cw[i], 8);
  return blockSum<kThreads>(v, red);
}

// CoalPrefix: the encoder's per-(segment, element) look-back flags (fp64:
// k_encode<4> leaves each workgroup's inclusive prefix of rounded words in
// its flag), so a block range's prefix and the segment totals are a few
// loads instead of sums over every earlier block.  Null: sum the word counts.
struct CoalPrefix {
  const uint64_t* flags = nullptr;
  uint32_t nW = 0;          // encode workgroups per element
  uint32_t encBlocks = 0;   // blocks per encode workgroup
  uint32_t epoch = 0;
  uint32_t* err = nullptr;  // device error word (an element whose look-back poisoned)
};

template <int FT>
__global__ __launch_bounds__(kThreads) void k_coalesce(
    BatchDesc in, BatchDesc out, uint32_t batchOffset, uint32_t numInBatch, uint32_t MB,
    uint32_t blocksPerWG, const uint8_t* __restrict__ slots, const uint32_t* __restrict__ cw,
    const uint16_t* __restrict__ pdf, int pb, bool useChecksum,
    const uint32_t* __restrict__ ck, uint32_t* __restrict__ outSize, const uint32_t* __restrict__ sparseN,
    CoalPrefix cp) {
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  __shared__ uint32_t red[kWaves];
  __shared__ uint32_t pre[kThreads];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t seg = blockIdx.z;
  const uint32_t tid = threadIdx.x;
  const uint32_t n = in.size(b);
  const uint32_t nBlocks = divUp(n, kBlockSize);
  const uint32_t first = blockIdx.x * blocksPerWG;
  if (first >= nBlocks && blockIdx.x != 0) return;

  gp<const uint32_t> cw0 = G(cw) + uint64_t(b) * MB;
  gp<const uint32_t> cwS = G(cw) + (uint64_t(seg) * numInBatch + b) * MB;

  // segment totals (inclusive prefix of the last encode workgroup) and the
  // prefix before this range, from the encoder's flags
  const bool fromFlags = cp.flags != nullptr && nBlocks > 0;
  uint32_t segTotal[2] = {0, 0};
  uint32_t flagBefore = 0, base = first;
  if (fromFlags) {
    const uint32_t eLast = (nBlocks - 1) / cp.encBlocks;
    bool bad = false;
    auto flagOf = [&](uint32_t s, uint32_t e) -> uint32_t {
      const uint64_t v = G(cp.flags)[(uint64_t(s) * numInBatch + b) * cp.nW + e];
      const uint32_t hi = uint32_t(v >> 32);
      bad = bad || (v & kFlagPoisonE) != 0 || (hi >> 30) != 2u || (hi & kEpochMask) != cp.epoch;
      return uint32_t(v);
    };
#pragma unroll
    for (int s = 0; s < kSegs; ++s) segTotal[s] = flagOf(uint32_t(s), eLast);
    const uint32_t e = min(first, nBlocks) / cp.encBlocks;
    base = e * cp.encBlocks;
    if (e > 0) flagBefore = flagOf(seg, e - 1);
    if (bad) {  // an encoder look-back gave up: the element is abandoned
      if (blockIdx.x == 0 && seg == 0 && tid == 0) {
        if (outSize) G(outSize)[b] = 0u;
        __hip_atomic_fetch_add(G(cp.err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }

  gp<uint8_t> o = startOf(out, b);
  uint32_t total0Words = 0;
  if constexpr (FT != 0) {
    o += 32 + floatRawBytes(FT, n);
    if (kSegs == 2 && (seg == 1 || blockIdx.x == 0)) {
      total0Words = fromFlags ? segTotal[0] : sumRoundedWords(cw0, nBlocks, red);
      if (seg == 1) o += roundUp64(ansOverhead(nBlocks) + 2ull * total0Words, 16);
    }
  }
  gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
  gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
  gp<uint8_t> data = (gp<uint8_t>)(bwords + roundUp(nBlocks, 2));

  // exclusive scan over [base, last): base is this range's first block, or
  // (flags) the first block of its encode workgroup, whose prefix the flag
  // holds
  const uint32_t sumBefore = fromFlags ? flagBefore : sumRoundedWords(cwS, min(first, nBlocks), red);
  const uint32_t last = min(first + blocksPerWG, nBlocks);
  const uint32_t j = base + tid;
  const uint32_t cwj = j < last ? cwS[j] : 0u;
  const uint32_t ex = blockExclusiveScan<kThreads>(roundUp(cwj, 8), red, nullptr) + sumBefore;
  if (j >= first && j < first + kThreads) pre[j - first] = ex;
  __syncthreads();

  if (blockIdx.x == 0) {
    const uint32_t totalWords = fromFlags ? segTotal[seg] : sumRoundedWords(cwS, nBlocks, red);
    uint32_t total1Words = 0;
    if (kSegs == 2 && seg == 0)
      total1Words = fromFlags ? segTotal[1] : sumRoundedWords(cwS + uint64_t(numInBatch) * MB, nBlocks, red);
    const uint64_t ansBytes = ansOverhead(nBlocks) + 2ull * totalWords;
    if (tid == 0) {
      gp<uint32_t> hdr = (gp<uint32_t>)o;
      const bool ansCk = FT == 0 && useChecksum;
      hdr[0] = kANSMagicVersion;
      hdr[1] = nBlocks;
      hdr[2] = n;
      hdr[3] = totalWords;
      hdr[4] = uint32_t(pb) | (ansCk ? 0x10u : 0u);
      hdr[5] = ansCk ? G(ck)[b] : 0u;
      hdr[6] = 0;
      hdr[7] = 0;
      if (nBlocks & 1) st8(bwords + nBlocks, make_uint2(0, 0));
      if constexpr (FT == 0) {
        if (outSize) G(outSize)[b] = uint32_t(ansBytes);
      } else if (seg == 0) {
        gp<uint32_t> fh = (gp<uint32_t>)startOf(out, b);
        fh[0] = kFloatMagicVersion;
        fh[1] = n;
        fh[2] = uint32_t(FT) | (useChecksum ? 0x10u : 0u);
        fh[3] = useChecksum ? G(ck)[b] : 0u;
        fh[4] = uint32_t(roundUp64(ansBytes, 16));  // GpuFloatHeader2
        fh[5] = 0;
        fh[6] = 0;
        fh[7] = 0;
        uint64_t sz = 32ull + floatRawBytes(FT, n) + ansBytes;
        if (kSegs == 2) sz += ansOverhead(nBlocks) + 2ull * total1Words;
        sz += sparseOverhead(sparseN, b);
        if (outSize) G(outSize)[b] = uint32_t(sz);
      }
    }
    ((gp<uint16_t>)(o + kANSHeaderBytes))[tid] = G(pdf)[(uint64_t(seg) * numInBatch + b) * kNumSymbols + tid];
    // zero the raw section's rounding tails (reference: uninitialised)
    if constexpr (FT != 0) {
      if (seg == 0 && tid < 16) {
        gp<uint8_t> raw = startOf(out, b) + 32;
        if constexpr (FT == 1 || FT == 2) {
          if (n + tid < roundUp(n, 16)) raw[n + tid] = 0;
        } else if constexpr (FT == 3) {
          if (n + tid < roundUp(n, 8)) ((gp<uint16_t>)raw)[n + tid] = 0;
          if (n + tid < roundUp(n, 16)) raw[2 * roundUp(n, 8) + n + tid] = 0;
        } else {
          if (n + tid < roundUp(n, 4)) ((gp<uint32_t>)raw)[n + tid] = 0;
          if (n + tid < roundUp(n, 8)) ((gp<uint16_t>)(raw + 4 * roundUp(n, 4)))[n + tid] = 0;
        }
      }
    }
  }

  // per block: states (32 lanes) and the blockWords entry
  const uint32_t lane = tid & 63;
  __shared__ uint32_t cwL[kThreads];
  if (j >= first && j < first + kThreads) cwL[j - first] = cwj;
  for (uint32_t k = first + (tid >> 6); k < last; k += kWaves) {
    gp<const uint8_t> slot = G(slots) + ((uint64_t(seg) * numInBatch + b) * MB + k) * kSlotBytes;
    if (lane < 32)
      ((gp<uint32_t>)(states + uint64_t(kStateBytesPerBlock) * k))[lane] = ((gp<const uint32_t>)slot)[lane];
    if (lane == 32) {
      const uint32_t uwk = (k + 1 < nBlocks || n % kBlockSize == 0) ? kBlockSize : n % kBlockSize;
      st8(bwords + k, make_uint2((uwk << 16) | cwS[k], pre[k - first]));
    }
  }
  __syncthreads();
  const uint32_t nk = last > first ? last - first : 0;
  copyPayload(pre, cwL, nk, G(slots) + ((uint64_t(seg) * numInBatch + b) * MB + first) * kSlotBytes +
                                kStateBytesPerBlock, data);
}

// ---------------------------------------------------------------------------
// utility kernels
// ---------------------------------------------------------------------------
// XOR-of-bytes checksum of size(b) * unitBytes bytes (checksumBatch,
// ans/GpuChecksum.cuh:26-133).  grid (chunks, batch); out pre-zeroed.
static __global__ __launch_bounds__(kThreads) void k_checksum(BatchDesc in, uint32_t batchOffset,
                                                              uint32_t unitBytes, uint32_t chunkBytes,
                                                              uint32_t* __restrict__ out) {
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint64_t size = uint64_t(in.size(b)) * unitBytes;
  const uint64_t begin = uint64_t(blockIdx.x) * chunkBytes;
  uint32_t ck = 0;
  if (begin < size) {
    gp<const uint8_t> p = startOf(in, b) + begin;
    const uint32_t nb = uint32_t(min(uint64_t(chunkBytes), size - begin));
    for (uint32_t i = threadIdx.x; i < nb; i += kThreads) ck ^= p[i];
  }
  ck = waveXor(ck);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ck;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t v = red[0] ^ red[1] ^ red[2] ^ red[3];
    if (v) atomicXor(&out[b], v);
  }
}

// header readout (ansGetCompressedInfoKernel, ans/GpuANSInfo.cuh:16-37;
// floatGetCompressedInfoKernel, float/GpuFloatInfo.cuh:18-36)
static __global__ void k_info(BatchDesc in, uint32_t numInBatch, bool isFloat,
                              uint32_t* __restrict__ sizes, uint32_t* __restrict__ types,
                              uint32_t* __restrict__ checksums) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= numInBatch) return;
  gp<const uint32_t> h = (gp<const uint32_t>)startOf(in, b);
  const bool ok = h[0] == (isFloat ? kFloatMagicVersion : kANSMagicVersion);
  if (isFloat) {
    if (sizes) G(sizes)[b] = ok ? h[1] : 0u;
    if (types) G(types)[b] = ok ? (h[2] & 0xfu) : 0u;
    if (checksums) G(checksums)[b] = h[3];
  } else {
    if (sizes) G(sizes)[b] = ok ? h[2] : 0u;
    if (checksums) G(checksums)[b] = h[5];
  }
}

}  // namespace dietgpu
