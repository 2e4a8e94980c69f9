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

#include "device.h"

namespace dietgpu {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kSlotBytes = kStateBytesPerBlock + kSlotDataBytes;
constexpr int kHistCopies = 16;
constexpr int kHistPitch = kNumSymbols + 1;

// ---------------------------------------------------------------------------
// k_hist: per-chunk symbol histogram(s) (+ byte-XOR checksum for raw bytes).
// grid (chunksPerElem, batch).  Each workgroup writes its 256 (x segs)
// partial counts without atomics; k_normalize sums them.  LDS counters are
// privatised 16 ways (lane & 15, pitch 257) so the few hot exponent values of
// float data do not serialise on one LDS address / bank.
// ---------------------------------------------------------------------------
template <int FT, bool kChecksum>
__global__ __launch_bounds__(kThreads) void k_hist(BatchDesc in, uint32_t batchOffset,
                                                   uint32_t numInBatch, uint32_t chunkWords,
                                                   uint32_t chunksPerElem,
                                                   uint32_t* __restrict__ partHist,
                                                   uint32_t* __restrict__ partCk) {
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  __shared__ uint32_t hs[kSegs][kHistCopies * kHistPitch];
  __shared__ uint32_t red[kWaves];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t c = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  for (int s = 0; s < kSegs; ++s)
    for (uint32_t i = tid; i < kHistCopies * kHistPitch; i += kThreads) hs[s][i] = 0;
  __syncthreads();

  const uint32_t size = in.size(b);
  const uint64_t begin = uint64_t(c) * chunkWords;
  uint32_t ck = 0;
  uint32_t* h0 = &hs[0][(tid & (kHistCopies - 1)) * kHistPitch];
  uint32_t* h1 = &hs[kSegs - 1][(tid & (kHistCopies - 1)) * kHistPitch];
  auto addWord = [&](WordT w) {
    atomicAdd(&h0[compOf<FT>(w, 0)], 1u);
    if constexpr (kSegs == 2) atomicAdd(&h1[compOf<FT>(w, 1)], 1u);
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
    uint32_t i = tid;
    for (; i + 3 * kThreads < n4; i += 4 * kThreads) {
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = ld16(q4 + i + k * kThreads);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const WordT* ws = reinterpret_cast<const WordT*>(&v[k]);
#pragma unroll
        for (uint32_t j = 0; j < kPerVec; ++j) addWord(ws[j]);
        if constexpr (kChecksum) ck ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      }
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
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kHistCopies; ++k) sum += hs[s][k * kHistPitch + tid];
    G(partHist)[((uint64_t(s) * numInBatch + b) * chunksPerElem + c) * kNumSymbols + tid] = sum;
  }
  if constexpr (kChecksum) {
    ck = (ck ^ (ck >> 8) ^ (ck >> 16) ^ (ck >> 24)) & 0xffu;
    ck = waveXor(ck);
    if ((tid & 63) == 0) red[tid >> 6] = ck;
    __syncthreads();
    if (tid == 0) G(partCk)[uint64_t(b) * chunksPerElem + c] = red[0] ^ red[1] ^ red[2] ^ red[3];
  }
}

// ---------------------------------------------------------------------------
// k_normalize: one workgroup per (element, segment).  Bit-exact restatement of
// normalizeProbabilitiesFromHistogram (ans/GpuANSStatistics.cuh:178-366):
// float32 quantisation, descending order of the unique keys (q << 16) | sym
// by rank counting (in place of cub::BlockRadixSort), the diff > 0 bump of
// *symbol ids* < diff, the diff < 0 decrement of sorted ranks [g-k, g), and
// the exclusive cdf.  Encode table entry (internal, never archived):
//   x = pdf << (31 - pb)              renormalisation threshold
//   y = magic                         x / pdf == (umulhi(x, magic) + x) >> shift
//   z = cdf
//   w = (2^pb - pdf) | shift << 24    x' = x + cdf + (x / pdf) * (2^pb - pdf)
// ---------------------------------------------------------------------------
static __global__ __launch_bounds__(kThreads) void k_normalize(
    BatchDesc in, uint32_t batchOffset, uint32_t numInBatch, const uint32_t* __restrict__ hist,
    uint32_t chunksPerElem, int pb, uint4* __restrict__ table, uint16_t* __restrict__ pdfOut,
    const uint32_t* __restrict__ partCk, uint32_t* __restrict__ ckOut) {
  __shared__ uint32_t keys[kNumSymbols];
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.x;
  const uint32_t seg = blockIdx.y;
  const uint32_t s = threadIdx.x;
  const uint64_t row = uint64_t(seg) * numInBatch + b;

  if (partCk && seg == 0 && s == 0) {
    uint32_t ck = 0;
    for (uint32_t c = 0; c < chunksPerElem; ++c) ck ^= G(partCk)[uint64_t(b) * chunksPerElem + c];
    G(ckOut)[b] = ck;
  }
  uint32_t count = 0;
  gp<const uint32_t> hp = G(hist) + row * chunksPerElem * kNumSymbols + s;
  for (uint32_t c = 0; c < chunksPerElem; ++c) count += hp[uint64_t(c) * kNumSymbols];

  const uint32_t total = in.size(b);
  if (total == 0) {  // :193-195 (the reference leaves the table untouched)
    st16(G(table) + row * kNumSymbols + s, make_uint4(0, 0, 0, 0));
    G(pdfOut)[row * kNumSymbols + s] = 0;
    return;
  }
  const uint32_t W = 1u << pb;
  const float r = __fdiv_rn(float(count), float(total));
  const float f = __fmul_rn(float(W), r);
  uint32_t q = uint32_t(f);
  if (count > 0 && q == 0) q = 1;
  const uint32_t qsum = blockSum<kThreads>(q, red);

  const uint32_t key = (q << 16) | s;
  keys[s] = key;
  __syncthreads();
  uint32_t rank = 0;
#pragma unroll 8
  for (uint32_t t = 0; t < kNumSymbols; ++t) rank += keys[t] > key ? 1u : 0u;

  const int diff = int(W) - int(qsum);
  if (diff > 0) {
    q += uint32_t(diff) / kNumSymbols + (s < uint32_t(diff) % kNumSymbols ? 1u : 0u);
  } else if (diff < 0) {
    int d = -diff;
    while (d > 0) {
      const int g = int(blockSum<kThreads>(q > 1 ? 1u : 0u, red));
      if (g == 0) break;  // reference asserts; unreachable for real tables
      const int k = d < g ? d : g;
      if (int(rank) >= g - k && int(rank) < g) q -= 1;
      d -= k;
    }
  }
  const uint32_t cdf = blockExclusiveScan<kThreads>(q, red, nullptr);
  uint32_t shift = 0, magic = 0;
  if (q > 0) {
    shift = 32 - __clz(q - 1);
    magic = uint32_t(((1ull << 32) * ((1ull << shift) - q)) / q + 1);
  }
  st16(G(table) + row * kNumSymbols + s,
       make_uint4(q << (kStateBits - pb), magic, cdf, (W - q) | (shift << 24)));
  G(pdfOut)[row * kNumSymbols + s] = uint16_t(q);
}

// ---------------------------------------------------------------------------
// k_encode: fused split + rANS encode.
//   * 128-thread workgroups; a half-wave codes one 4 KiB block; each lane
//     runs K blocks (K = 2, fp64: K = 1 with its two streams) for ILP.
//   * Per 1024-symbol segment the wave loads the block's words with 16 B
//     loads (issued one segment ahead), writes the float raw bytes straight
//     into the archive's raw section and the ANS symbols into LDS, then runs
//     32 encode steps per block from LDS.
//   * Emitted u16 words go to a per-block scratch slot; k_coalesce packs the
//     slots into the archive.
// ---------------------------------------------------------------------------
namespace enc {
constexpr int kThreads = 128;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kSegWords = 1024;
}  // namespace enc

template <int FT>
struct EncCfg {
  using WordT = typename FloatTraits<FT>::WordT;
  static constexpr int S = FloatTraits<FT>::kSegs;
  static constexpr int K = S == 2 ? 1 : 2;
  static constexpr int kBlocksPerWave = 2 * K;
  static constexpr int kBlocksPerWG = enc::kWaves * kBlocksPerWave;
  // 16-byte input vectors per lane per block per segment (32 lanes x V x 16 B
  // = 1024 words)
  static constexpr int V = int(enc::kSegWords * sizeof(WordT) / (32 * 16));
  static constexpr uint32_t kWordsPerVec = 16 / sizeof(WordT);
};

struct EStream {
  uint32_t x;             // state
  uint32_t nout;          // half-uniform: words emitted so far
  gp<uint16_t> out;       // slot data of this half's block
};

// One rANS encode step (encodeOneWarp, ans/GpuANSEncode.cuh:49-90) of one
// stream for both half-waves; writers emit in ascending lane order.
template <bool kMask>
__device__ __forceinline__ void encStep(EStream& s, bool valid, uint32_t sym,
                                        const uint4* __restrict__ tbl, uint32_t h) {
  const uint4 e = tbl[sym];
  bool wr = s.x >= e.x;
  if (kMask) wr = wr && valid;
  const uint64_t vote = ballot(wr);
  const uint32_t cLo = uint32_t(__popc(uint32_t(vote)));
  const uint32_t cHi = uint32_t(__popc(uint32_t(vote >> 32)));
  uint32_t x = s.x;
  if (wr) {
    const uint32_t base = s.nout - (h ? cLo : 0u);
    s.out[base + mbcnt(vote)] = uint16_t(x);
    x >>= kEncodedBits;
  }
  s.nout += h ? cHi : cLo;
  uint32_t q = __umulhi(x, e.y);
  q = (q + x) >> (e.w >> 24);
  const uint32_t xn = __umul24(q, e.w) + x + e.z;
  s.x = (!kMask || valid) ? xn : x;
}

// Split 16 B of input words: ANS symbols -> LDS (sym0 / sym1), raw remainder
// -> the archive raw section at word index i0.
template <int FT>
__device__ __forceinline__ void splitVec(const uint4& v, uint32_t i0, uint32_t n,
                                         gp<uint8_t> raw, uint8_t* sym0, uint8_t* sym1) {
  using WordT = typename FloatTraits<FT>::WordT;
  const WordT* ws = reinterpret_cast<const WordT*>(&v);
  if constexpr (FT == 0) {
    *reinterpret_cast<uint4*>(sym0) = v;
  } else if constexpr (FT == 1 || FT == 2) {
    uint32_t e0 = 0, e1 = 0, r0 = 0, r1 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = ws[k], c = ws[k + 4];
      if constexpr (FT == 1) {
        e0 |= (a >> 8) << (8 * k);
        e1 |= (c >> 8) << (8 * k);
        r0 |= (a & 0xffu) << (8 * k);
        r1 |= (c & 0xffu) << (8 * k);
      } else {
        e0 |= ((a >> 7) & 0xffu) << (8 * k);
        e1 |= ((c >> 7) & 0xffu) << (8 * k);
        r0 |= (((a << 1) | (a >> 15)) & 0xffu) << (8 * k);
        r1 |= (((c << 1) | (c >> 15)) & 0xffu) << (8 * k);
      }
    }
    *reinterpret_cast<uint2*>(sym0) = make_uint2(e0, e1);
    st8(raw + i0, make_uint2(r0, r1));
  } else if constexpr (FT == 3) {
    uint32_t e = 0, hb = 0, lo[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t r = rotl32(ws[k], 1);
      e |= (r >> 24) << (8 * k);
      hb |= ((r >> 16) & 0xffu) << (8 * k);
      lo[k] = r & 0xffffu;
    }
    *reinterpret_cast<uint32_t*>(sym0) = e;
    st8(raw + 2 * i0, make_uint2(lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16)));
    *(gp<uint32_t>)(raw + 2 * roundUp(n, 8) + i0) = hb;
  } else {
    const uint64_t r0 = rotl64(ws[0], 1), r1 = rotl64(ws[1], 1);
    *reinterpret_cast<uint16_t*>(sym0) = uint16_t((r0 >> 56) | ((r1 >> 56) << 8));
    *reinterpret_cast<uint16_t*>(sym1) = uint16_t(((r0 >> 48) & 0xffu) | (((r1 >> 48) & 0xffu) << 8));
    st8(raw + 4 * i0, make_uint2(uint32_t(r0), uint32_t(r1)));
    *(gp<uint32_t>)(raw + 4 * roundUp(n, 4) + 2 * i0) =
        uint32_t((r0 >> 32) & 0xffffu) | (uint32_t((r1 >> 32) & 0xffffu) << 16);
  }
}

// scalar split of one word (unaligned input or element tail)
template <int FT>
__device__ __forceinline__ void splitOne(typename FloatTraits<FT>::WordT w, uint32_t i, uint32_t n,
                                         gp<uint8_t> raw, uint8_t* sym0, uint8_t* sym1) {
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

template <int FT>
__global__ __launch_bounds__(enc::kThreads) void k_encode(BatchDesc in, BatchDesc out,
                                                          uint32_t batchOffset,
                                                          uint32_t numInBatch, uint32_t MB,
                                                          const uint4* __restrict__ table,
                                                          uint8_t* __restrict__ slots,
                                                          uint32_t* __restrict__ cw) {
  using Cfg = EncCfg<FT>;
  using WordT = typename Cfg::WordT;
  constexpr int S = Cfg::S, K = Cfg::K, V = Cfg::V;
  __shared__ uint4 tbl[S][kNumSymbols];
  __shared__ __attribute__((aligned(16))) uint8_t symBuf[enc::kWaves][K][S][2][enc::kSegWords];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t tid = threadIdx.x;
  for (int s = 0; s < S; ++s) {
    for (uint32_t i = tid; i < kNumSymbols; i += enc::kThreads)
      tbl[s][i] = ld16(G(table) + (uint64_t(s) * numInBatch + b) * kNumSymbols + i);
  }
  __syncthreads();

  const uint32_t n = in.size(b);
  const uint32_t nBlocks = divUp(n, kBlockSize);
  const uint32_t w = tid >> 6, lane = tid & 63, h = lane >> 5, l = lane & 31;
  const uint32_t blk0 = blockIdx.x * Cfg::kBlocksPerWG + w * Cfg::kBlocksPerWave;
  if (blk0 >= nBlocks) return;

  gp<const WordT> src = (gp<const WordT>)startOf(in, b);
  gp<uint8_t> raw = FT == 0 ? gp<uint8_t>(nullptr) : startOf(out, b) + 32;
  const bool vecIn = (reinterpret_cast<uintptr_t>(src) & 15) == 0;

  uint32_t blk[K], uw[K];
  EStream st[K][S];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    blk[c] = blk0 + 2 * c + h;
    uw[c] = blk[c] < nBlocks ? min(kBlockSize, n - blk[c] * kBlockSize) : 0u;
    const uint32_t sb = blk[c] < nBlocks ? blk[c] : blk0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      st[c][s].x = kStartState;
      st[c][s].nout = 0;
      st[c][s].out = (gp<uint16_t>)(G(slots) + ((uint64_t(s) * numInBatch + b) * MB + sb) * kSlotBytes +
                                    kStateBytesPerBlock);
    }
  }
  uint32_t T = 0;
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const uint32_t tc = divUp(uw[c], 32);
    T = max(T, max(__builtin_amdgcn_readlane(tc, 0), __builtin_amdgcn_readlane(tc, 32)));
  }
  const uint32_t nSeg = divUp(T, 32);

  // prefetch segment 0
  uint4 pv[K][V];
  auto loadSeg = [&](uint32_t g) {
#pragma unroll
    for (int c = 0; c < K; ++c) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const uint32_t j0 = g * enc::kSegWords + (k * 32 + l) * Cfg::kWordsPerVec;
        if (vecIn && j0 + Cfg::kWordsPerVec <= uw[c])
          pv[c][k] = ld16(src + blk[c] * kBlockSize + j0);
      }
    }
  };
  loadSeg(0);

  for (uint32_t g = 0; g < nSeg; ++g) {
    const uint32_t segW0 = g * enc::kSegWords;
    // split this segment: symbols -> LDS, raw -> archive
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (uw[c] <= segW0) continue;
      const uint32_t segCnt = min(enc::kSegWords, uw[c] - segW0);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const uint32_t off = (k * 32 + l) * Cfg::kWordsPerVec;  // word offset in segment
        uint8_t* s0 = &symBuf[w][c][0][h][off];
        uint8_t* s1 = &symBuf[w][c][S - 1][h][off];
        const uint32_t i0 = blk[c] * kBlockSize + segW0 + off;
        if (vecIn && off + Cfg::kWordsPerVec <= segCnt) {
          splitVec<FT>(pv[c][k], i0, n, raw, s0, s1);
        } else {
          for (uint32_t q = 0; q < Cfg::kWordsPerVec && off + q < segCnt; ++q)
            splitOne<FT>(src[i0 + q], i0 + q, n, raw, s0 + q, s1 + q);
        }
      }
    }
    if (g + 1 < nSeg) loadSeg(g + 1);

    bool full = true;
#pragma unroll
    for (int c = 0; c < K; ++c) full = full && uw[c] >= segW0 + enc::kSegWords;
    full = ballot(full) == ~0ull;
    const uint32_t tEnd = min(T, (g + 1) * 32);
    if (full) {
#pragma unroll 4
      for (uint32_t t = g * 32; t < tEnd; ++t) {
        const uint32_t si = (t - g * 32) * 32 + l;
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) encStep<false>(st[c][s], true, symBuf[w][c][s][h][si], tbl[s], h);
      }
    } else {
      for (uint32_t t = g * 32; t < tEnd; ++t) {
        const uint32_t si = (t - g * 32) * 32 + l;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const bool valid = t * 32 + l < uw[c];
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const uint32_t sym = valid ? uint32_t(symBuf[w][c][s][h][si]) : 0u;
            encStep<true>(st[c][s], valid, sym, tbl[s], h);
          }
        }
      }
    }
  }

#pragma unroll
  for (int c = 0; c < K; ++c) {
    if (!uw[c]) continue;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      gp<uint8_t> slot = G(slots) + ((uint64_t(s) * numInBatch + b) * MB + blk[c]) * kSlotBytes;
      ((gp<uint32_t>)slot)[l] = st[c][s].x;
      if (l == 0) G(cw)[(uint64_t(s) * numInBatch + b) * MB + blk[c]] = st[c][s].nout;
    }
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

template <int FT>
__global__ __launch_bounds__(kThreads) void k_coalesce(
    BatchDesc in, BatchDesc out, uint32_t batchOffset, uint32_t numInBatch, uint32_t MB,
    uint32_t blocksPerWG, const uint8_t* __restrict__ slots, const uint32_t* __restrict__ cw,
    const uint16_t* __restrict__ pdf, int pb, bool useChecksum,
    const uint32_t* __restrict__ ck, uint32_t* __restrict__ outSize) {
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

  gp<uint8_t> o = startOf(out, b);
  uint32_t total0Words = 0;
  if constexpr (FT != 0) {
    o += 32 + floatRawBytes(FT, n);
    if (kSegs == 2 && (seg == 1 || blockIdx.x == 0)) {
      total0Words = sumRoundedWords(cw0, nBlocks, red);
      if (seg == 1) o += roundUp64(ansOverhead(nBlocks) + 2ull * total0Words, 16);
    }
  }
  gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
  gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
  gp<uint8_t> data = (gp<uint8_t>)(bwords + roundUp(nBlocks, 2));

  const uint32_t sumBefore = sumRoundedWords(cwS, min(first, nBlocks), red);
  const uint32_t last = min(first + blocksPerWG, nBlocks);
  const uint32_t j = first + tid;
  const uint32_t cwj = (tid < blocksPerWG && j < last) ? cwS[j] : 0u;
  const uint32_t ex = blockExclusiveScan<kThreads>(roundUp(cwj, 8), red, nullptr) + sumBefore;
  pre[tid] = ex;
  __syncthreads();

  if (blockIdx.x == 0) {
    const uint32_t totalWords = sumRoundedWords(cwS, nBlocks, red);
    uint32_t total1Words = 0;
    if (kSegs == 2 && seg == 0) total1Words = sumRoundedWords(cwS + uint64_t(numInBatch) * MB, nBlocks, red);
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

  // copy this workgroup's blocks: one wave per block
  const uint32_t lane = tid & 63;
  for (uint32_t k = first + (tid >> 6); k < last; k += kWaves) {
    const uint32_t c = cwS[k];
    const uint32_t p = pre[k - first];
    gp<const uint8_t> slot = G(slots) + ((uint64_t(seg) * numInBatch + b) * MB + k) * kSlotBytes;
    if (lane < 32) {
      ((gp<uint32_t>)(states + uint64_t(kStateBytesPerBlock) * k))[lane] = ((gp<const uint32_t>)slot)[lane];
    }
    if (lane == 0) {
      const uint32_t uwk = (k + 1 < nBlocks || n % kBlockSize == 0) ? kBlockSize : n % kBlockSize;
      st8(bwords + k, make_uint2((uwk << 16) | c, p));
    }
    gp<const uint4> src = (gp<const uint4>)(slot + kStateBytesPerBlock);
    gp<uint4> dst = (gp<uint4>)(data + 2ull * p);
    const uint32_t nv = divUp(c, 8);
    for (uint32_t i = lane; i < nv; i += 64) {
      uint4 v = ld16(src + i);
      const uint32_t valid = c - i * 8;
      if (valid < 8) {
        uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          if (2 * q + 1 >= valid) vw[q] &= (2 * q < valid) ? 0xffffu : 0u;
        }
      }
      st16(dst + i, v);
    }
  }
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
