// HIP kernels of the MI355X-native rANS byte codec and exponent-split float
// codec (gfx950 / CDNA4, wave64).
//
// Wire format = reference: one ANS block is 4096
// symbols coded by 32 interleaved rANS states, symbol 32t+l on lane l.
// MI355X mapping: one 64-lane wavefront owns TWO blocks, lanes 0-31 block 2k
// and lanes 32-63 block 2k+1; 64-bit ballots are split per half-wave and the
// emission prefix is v_mbcnt of the half's bits.  A 256-thread workgroup owns
// 8 consecutive blocks of one batch element.
//
// Kernel <-> reference map (paths relative to /root/reference/dietgpu):
//   k_hist<FT>          histogramBatch (ans/GpuANSStatistics.cuh:21-143) and
//                       the histogram half of splitFloat
//                       (float/GpuFloatCompress.cuh:423-551)
//   k_normalize         quantizeWeights / normalizeProbabilitiesFromHistogram
//                       (ans/GpuANSStatistics.cuh:178-430)
//   k_encode<FT>        ansEncodeBatchFull/Partial (ans/GpuANSEncode.cuh:
//                       49-495) fused with the split half of splitFloat
//   k_coalesce<FT>      batchExclusivePrefixSum + ansEncodeCoalesceBatch
//                       (ans/BatchPrefixSum.cuh, ans/GpuANSEncode.cuh:497-668)
//                       + incOutputSizes / setHeaderAndANSOutOffset
//                       (float/GpuFloatCompress.cuh:557-667)
//   k_decode<FT>        ansDecodeTable + ansDecodeKernel
//                       (ans/GpuANSDecode.cuh:34-476) fused with joinFloat /
//                       JoinFloatWriter (float/GpuFloatDecompress.cuh:39-841),
//                       fp64 included (the reference runs fp64 in two passes)
//
// FT template parameter: 0 = raw bytes, 1 fp16, 2 bf16, 3 fp32, 4 fp64.
#pragma once

#include "batch.h"
#include "common.h"

namespace dietgpu {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kBlocksPerWG = 2 * kWaves;
constexpr uint32_t kSlotBytes = kStateBytesPerBlock + kSlotDataBytes;
constexpr int kHistCopies = 16;
constexpr int kHistPitch = kNumSymbols + 1;

template <int FT>
struct FloatTraits;
template <>
struct FloatTraits<0> {  // raw bytes
  using WordT = uint8_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<1> {
  using WordT = uint16_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<2> {
  using WordT = uint16_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<3> {
  using WordT = uint32_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<4> {
  using WordT = uint64_t;
  static constexpr int kSegs = 2;
};

// ---------------------------------------------------------------------------
// split / join of one float word (float/GpuFloatUtils.cuh:190-370)
// comp0/comp1: ANS symbols; raw layout per getUncompDataSize
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl32(uint32_t v, int s) {
  return (v << s) | (v >> (32 - s));
}
__device__ __forceinline__ uint32_t rotr32(uint32_t v, int s) {
  return (v >> s) | (v << (32 - s));
}

// symbol byte(s) of a word
template <int FT>
__device__ __forceinline__ uint32_t compOf(typename FloatTraits<FT>::WordT w, int seg) {
  if constexpr (FT == 0) {
    return w;
  } else if constexpr (FT == 1) {
    return uint32_t(w) >> 8;
  } else if constexpr (FT == 2) {
    return (uint32_t(w) >> 7) & 0xffu;  // exponent
  } else if constexpr (FT == 3) {
    return rotl32(w, 1) >> 24;
  } else {
    uint64_t v = (w << 1) | (w >> 63);
    return seg == 0 ? uint32_t(v >> 56) : uint32_t(v >> 48) & 0xffu;
  }
}

// ---------------------------------------------------------------------------
// wave / block reductions
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t waveSum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t waveXor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  return v;
}
// inclusive scan within the wave
__device__ __forceinline__ uint32_t waveInclusiveScan(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(v, o);
    if (lane >= uint32_t(o)) v += u;
  }
  return v;
}
// all 256 threads must call; smem >= kWaves words
__device__ __forceinline__ uint32_t blockSum(uint32_t v, uint32_t* smem) {
  v = waveSum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) smem[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) t += smem[i];
  return t;
}
// exclusive scan over the 256 threads; returns the block total in *total
__device__ __forceinline__ uint32_t blockExclusiveScan(uint32_t v, uint32_t* smem,
                                                       uint32_t* total) {
  uint32_t inc = waveInclusiveScan(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 63) smem[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    uint32_t s = smem[i];
    before += (i < int(threadIdx.x >> 6)) ? s : 0;
    all += s;
  }
  if (total) *total = all;
  return before + inc - v;
}

// ---------------------------------------------------------------------------
// k_hist: per-chunk symbol histogram(s) (+ byte-XOR checksum for raw bytes)
// grid (chunksPerElem, batch).  Each workgroup writes its 256 (x segs) partial
// counts without atomics; k_normalize sums them.  LDS counts are privatised
// 16 ways (lane & 15) so skewed data (a few hot exponents) does not serialise
// on one LDS address.
// ---------------------------------------------------------------------------
template <int FT, bool kChecksum>
__global__ __launch_bounds__(kThreads) void k_hist(BatchDesc in, uint32_t batchOffset,
                                                   uint32_t numInBatch,
                                                   uint32_t chunkWords,
                                                   uint32_t chunksPerElem,
                                                   uint32_t* __restrict__ partHist,
                                                   uint32_t* __restrict__ partCk) {
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  __shared__ uint32_t h[kSegs][kHistCopies * kHistPitch];
  __shared__ uint32_t red[kWaves];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t c = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  for (int s = 0; s < kSegs; ++s)
    for (uint32_t i = tid; i < kHistCopies * kHistPitch; i += kThreads) h[s][i] = 0;
  __syncthreads();

  const uint32_t size = in.size(b);
  const uint64_t begin = uint64_t(c) * chunkWords;
  uint32_t ck = 0;
  uint32_t* h0 = &h[0][(tid & (kHistCopies - 1)) * kHistPitch];
  uint32_t* h1 = &h[kSegs - 1][(tid & (kHistCopies - 1)) * kHistPitch];

  auto addWord = [&](WordT w) {
    atomicAdd(&h0[compOf<FT>(w, 0)], 1u);
    if constexpr (kSegs == 2) atomicAdd(&h1[compOf<FT>(w, 1)], 1u);
  };

  if (begin < size) {
    const uint32_t n = uint32_t(min(uint64_t(chunkWords), uint64_t(size) - begin));
    const WordT* q = reinterpret_cast<const WordT*>(in.start(b)) + begin;
    constexpr uint32_t kPerVec = 16 / sizeof(WordT);
    // words before the first 16 B boundary
    uint32_t head = uint32_t(((16 - (reinterpret_cast<uintptr_t>(q) & 15)) & 15) / sizeof(WordT));
    if ((reinterpret_cast<uintptr_t>(q) & (sizeof(WordT) - 1)) != 0) head = n;  // misaligned words
    head = min(head, n);
    for (uint32_t i = tid; i < head; i += kThreads) {
      WordT w = q[i];
      addWord(w);
      if constexpr (kChecksum) ck ^= uint32_t(w);
    }
    const uint4* q4 = reinterpret_cast<const uint4*>(q + head);
    const uint32_t n4 = (n - head) / kPerVec;
    uint32_t i = tid;
    for (; i + 3 * kThreads < n4; i += 4 * kThreads) {
      uint4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = q4[i + k * kThreads];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const WordT* ws = reinterpret_cast<const WordT*>(&v[k]);
#pragma unroll
        for (uint32_t j = 0; j < kPerVec; ++j) addWord(ws[j]);
        if constexpr (kChecksum) ck ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
      }
    }
    for (; i < n4; i += kThreads) {
      uint4 v = q4[i];
      const WordT* ws = reinterpret_cast<const WordT*>(&v);
#pragma unroll
      for (uint32_t j = 0; j < kPerVec; ++j) addWord(ws[j]);
      if constexpr (kChecksum) ck ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    for (uint32_t t = head + n4 * kPerVec + tid; t < n; t += kThreads) {
      WordT w = q[t];
      addWord(w);
      if constexpr (kChecksum) ck ^= uint32_t(w);
    }
  }
  __syncthreads();
  for (int s = 0; s < kSegs; ++s) {
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kHistCopies; ++k) sum += h[s][k * kHistPitch + tid];
    partHist[((uint64_t(s) * numInBatch + b) * chunksPerElem + c) * kNumSymbols + tid] = sum;
  }
  if constexpr (kChecksum) {
    ck = (ck ^ (ck >> 8) ^ (ck >> 16) ^ (ck >> 24)) & 0xffu;
    ck = waveXor(ck);
    if ((tid & 63) == 0) red[tid >> 6] = ck;
    __syncthreads();
    if (tid == 0) partCk[uint64_t(b) * chunksPerElem + c] = red[0] ^ red[1] ^ red[2] ^ red[3];
  }
}

// ---------------------------------------------------------------------------
// k_normalize: one workgroup per (element, segment).  Bit-exact restatement of
// normalizeProbabilitiesFromHistogram (ans/GpuANSStatistics.cuh:178-366):
// float32 quantisation, descending order of unique keys (q << 16) | sym by
// rank counting (replaces cub::BlockRadixSort), the diff>0 bump of *symbol
// ids* < diff, the diff<0 decrement of sorted ranks [g-k, g), exclusive cdf.
// Output table entry (internal, never archived):
//   x = pdf << (31 - pb)      renormalisation threshold
//   y = magic                 x / pdf == (umulhi(x, magic) + x) >> shift
//   z = cdf
//   w = (2^pb - pdf) | shift << 24   so  x' = x + cdf + q * (2^pb - pdf)
// ---------------------------------------------------------------------------
static __global__ __launch_bounds__(kThreads) void k_normalize(
    BatchDesc in, uint32_t batchOffset, uint32_t numInBatch,
    const uint32_t* __restrict__ hist, uint32_t chunksPerElem, int pb,
    uint4* __restrict__ table, uint16_t* __restrict__ pdfOut,
    const uint32_t* __restrict__ partCk, uint32_t* __restrict__ ckOut) {
  __shared__ uint32_t keys[kNumSymbols];
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.x;
  const uint32_t seg = blockIdx.y;
  const uint32_t s = threadIdx.x;
  const uint64_t row = uint64_t(seg) * numInBatch + b;

  if (partCk && seg == 0 && s == 0) {
    uint32_t ck = 0;
    for (uint32_t c = 0; c < chunksPerElem; ++c) ck ^= partCk[uint64_t(b) * chunksPerElem + c];
    ckOut[b] = ck;
  }

  uint32_t count = 0;
  const uint32_t* hp = hist + row * chunksPerElem * kNumSymbols + s;
  for (uint32_t c = 0; c < chunksPerElem; ++c) count += hp[uint64_t(c) * kNumSymbols];

  const uint32_t total = in.size(b);
  if (total == 0) {  // :193-195 (reference leaves the table untouched)
    table[row * kNumSymbols + s] = make_uint4(0, 0, 0, 0);
    pdfOut[row * kNumSymbols + s] = 0;
    return;
  }
  const uint32_t W = 1u << pb;
  // :212-218: uint32 * float -> float, truncated to uint32 (IEEE, no FMA)
  float r = __fdiv_rn(float(count), float(total));
  float f = __fmul_rn(float(W), r);
  uint32_t q = uint32_t(f);
  if (count > 0 && q == 0) q = 1;
  const uint32_t qsum = blockSum(q, red);

  const uint32_t key = (q << 16) | s;
  keys[s] = key;
  __syncthreads();
  uint32_t rank = 0;
#pragma unroll 8
  for (uint32_t t = 0; t < kNumSymbols; ++t) rank += keys[t] > key ? 1u : 0u;

  int diff = int(W) - int(qsum);
  if (diff > 0) {
    // while (diff > 0) { +1 for every symbol id < min(diff, 256) }
    q += uint32_t(diff) / kNumSymbols + (s < uint32_t(diff) % kNumSymbols ? 1u : 0u);
  } else if (diff < 0) {
    int d = -diff;
    while (d > 0) {
      int g = int(blockSum(q > 1 ? 1u : 0u, red));
      if (g == 0) break;  // reference asserts (unreachable for real tables)
      int k = d < g ? d : g;
      if (int(rank) >= g - k && int(rank) < g) q -= 1;
      d -= k;
    }
  }

  uint32_t cdf = blockExclusiveScan(q, red, nullptr);
  uint32_t shift = 0, magic = 0;
  if (q > 0) {
    shift = 32 - __clz(q - 1);
    uint64_t m = ((1ull << 32) * ((1ull << shift) - q)) / q + 1;
    magic = uint32_t(m);
  }
  table[row * kNumSymbols + s] =
      make_uint4(q << (kStateBits - pb), magic, cdf, (W - q) | (shift << 24));
  pdfOut[row * kNumSymbols + s] = uint16_t(q);
}

// ---------------------------------------------------------------------------
// encode one 4 KiB block per half-wave from LDS symbols
// ---------------------------------------------------------------------------
struct EncStream {
  uint32_t state;
  uint32_t nout;
};

// One rANS encode step for all 64 lanes (two blocks).  Emission order within
// the half = ascending lane among writers (encodeOneWarp :63-75).
__device__ __forceinline__ void encodeStep(EncStream& st, bool valid, uint32_t sym,
                                           const uint4* __restrict__ tbl,
                                           uint16_t* __restrict__ outHalf,
                                           uint32_t h) {
  const uint4 e = tbl[sym];
  const bool write = valid && st.state >= e.x;
  const uint64_t vote = ballot(write);
  const uint32_t lo = uint32_t(vote);
  const uint32_t hi = uint32_t(vote >> 32);
  const uint32_t prefix = mbcnt(vote) - (h ? uint32_t(__popc(lo)) : 0u);
  if (write) {
    outHalf[st.nout + prefix] = uint16_t(st.state);
    st.state >>= kEncodedBits;
  }
  st.nout += uint32_t(__popc(h ? hi : lo));
  if (valid) {
    const uint32_t x = st.state;
    uint32_t q = __umulhi(x, e.y);
    q = (q + x) >> (e.w >> 24);
    st.state = __umul24(q, e.w & 0xffffffu) + x + e.z;
  }
}

// Copy `count` bytes global -> LDS (dst 16 B aligned) with the whole wave.
__device__ __forceinline__ void stageBytes(const uint8_t* __restrict__ src, uint32_t count,
                                           uint8_t* __restrict__ dst, uint32_t lane) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(src);
  uint32_t done = 0;
  if ((a & 15) == 0) {
    const uint32_t n16 = count / 16;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll 8
    for (uint32_t i = lane; i < n16; i += 64) d4[i] = s4[i];
    done = n16 * 16;
  } else if ((a & 3) == 0) {
    const uint32_t n4 = count / 4;
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(dst);
#pragma unroll 8
    for (uint32_t i = lane; i < n4; i += 64) d1[i] = s1[i];
    done = n4 * 4;
  }
  for (uint32_t i = done + lane; i < count; i += 64) dst[i] = src[i];
}

// Stage the words [w0, w0 + count) of one element: symbol bytes -> LDS
// (symsOut[seg][j]), raw remainder -> the archive's raw section.
template <int FT>
__device__ __forceinline__ void stageFloat(const typename FloatTraits<FT>::WordT* __restrict__ src,
                                           uint32_t w0, uint32_t count, uint32_t n,
                                           uint8_t* __restrict__ raw, uint8_t* sym0,
                                           uint8_t* sym1, uint32_t lane) {
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr uint32_t kPerVec = 16 / sizeof(WordT);
  const WordT* s = src + w0;
  auto one = [&](uint32_t j, WordT w) {
    const uint32_t i = w0 + j;
    if constexpr (FT == 1) {
      sym0[j] = uint8_t(w >> 8);
      raw[i] = uint8_t(w);
    } else if constexpr (FT == 2) {
      sym0[j] = uint8_t(w >> 7);
      raw[i] = uint8_t((w << 1) | (w >> 15));
    } else if constexpr (FT == 3) {
      uint32_t v = rotl32(w, 1);
      sym0[j] = uint8_t(v >> 24);
      reinterpret_cast<uint16_t*>(raw)[i] = uint16_t(v);
      raw[2 * roundUp(n, 8) + i] = uint8_t(v >> 16);
    } else {
      uint64_t v = (w << 1) | (w >> 63);
      sym0[j] = uint8_t(v >> 56);
      sym1[j] = uint8_t(v >> 48);
      reinterpret_cast<uint32_t*>(raw)[i] = uint32_t(v);
      reinterpret_cast<uint16_t*>(raw + 4 * roundUp(n, 4))[i] = uint16_t(v >> 32);
    }
  };
  // vector path needs 16 B aligned source and a 16 B aligned group start
  if ((reinterpret_cast<uintptr_t>(s) & 15) == 0) {
    const uint32_t nv = count / kPerVec;
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
#pragma unroll 4
    for (uint32_t v = lane; v < nv; v += 64) {
      uint4 x = s4[v];
      const WordT* ws = reinterpret_cast<const WordT*>(&x);
      const uint32_t j0 = v * kPerVec;
      const uint32_t i0 = w0 + j0;
      if constexpr (FT == 1 || FT == 2) {
        uint32_t e0 = 0, e1 = 0, r0 = 0, r1 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t a = ws[k], c = ws[k + 4];
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
        *reinterpret_cast<uint2*>(sym0 + j0) = make_uint2(e0, e1);
        *reinterpret_cast<uint2*>(raw + i0) = make_uint2(r0, r1);
      } else if constexpr (FT == 3) {
        uint32_t e = 0, hb = 0;
        uint32_t lo[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t r = rotl32(ws[k], 1);
          e |= (r >> 24) << (8 * k);
          hb |= ((r >> 16) & 0xffu) << (8 * k);
          lo[k] = r & 0xffffu;
        }
        *reinterpret_cast<uint32_t*>(sym0 + j0) = e;
        *reinterpret_cast<uint2*>(raw + 2 * i0) =
            make_uint2(lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16));
        *reinterpret_cast<uint32_t*>(raw + 2 * roundUp(n, 8) + i0) = hb;
      } else {
        uint64_t r0 = (ws[0] << 1) | (ws[0] >> 63);
        uint64_t r1 = (ws[1] << 1) | (ws[1] >> 63);
        *reinterpret_cast<uint16_t*>(sym0 + j0) = uint16_t((r0 >> 56) | ((r1 >> 56) << 8));
        *reinterpret_cast<uint16_t*>(sym1 + j0) =
            uint16_t(((r0 >> 48) & 0xffu) | (((r1 >> 48) & 0xffu) << 8));
        *reinterpret_cast<uint2*>(raw + 4 * i0) = make_uint2(uint32_t(r0), uint32_t(r1));
        *reinterpret_cast<uint32_t*>(raw + 4 * roundUp(n, 4) + 2 * i0) =
            uint32_t((r0 >> 32) & 0xffffu) | (uint32_t((r1 >> 32) & 0xffffu) << 16);
      }
    }
    for (uint32_t j = nv * kPerVec + lane; j < count; j += 64) one(j, s[j]);
  } else {
    for (uint32_t j = lane; j < count; j += 64) one(j, s[j]);
  }
}

// ---------------------------------------------------------------------------
// k_encode: grid (ceil(maxBlocks / 8), batch).  Per wave: stage two blocks of
// input (symbols to LDS, float raw bytes straight to the archive), then run
// the interleaved rANS coder with both half-waves in lockstep; emitted words
// go to a per-block scratch slot, compacted later by k_coalesce.
// ---------------------------------------------------------------------------
template <int FT>
__global__ __launch_bounds__(kThreads) void k_encode(BatchDesc in, BatchDesc out,
                                                     uint32_t batchOffset,
                                                     uint32_t numInBatch, uint32_t MB,
                                                     const uint4* __restrict__ table,
                                                     uint8_t* __restrict__ slots,
                                                     uint32_t* __restrict__ cw) {
  using WordT = typename FloatTraits<FT>::WordT;
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  __shared__ uint4 tbl[kSegs][kNumSymbols];
  __shared__ __attribute__((aligned(16))) uint8_t syms[kSegs][kWaves][2 * kBlockSize];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t w = tid >> 6;
  const uint32_t h = lane >> 5;
  const uint32_t l = lane & 31;
#pragma unroll
  for (int s = 0; s < kSegs; ++s)
    tbl[s][tid] = table[(uint64_t(s) * numInBatch + b) * kNumSymbols + tid];

  const uint32_t size = in.size(b);
  const uint32_t nBlocks = divUp(size, kBlockSize);
  const uint32_t blk0 = blockIdx.x * kBlocksPerWG + 2 * w;
  if (blk0 < nBlocks) {
    const uint32_t begin = blk0 * kBlockSize;
    const uint32_t count = min(2 * kBlockSize, size - begin);
    if constexpr (FT == 0) {
      stageBytes(in.start(b) + begin, count, syms[0][w], lane);
    } else {
      uint8_t* raw = out.start(b) + 32;
      stageFloat<FT>(reinterpret_cast<const WordT*>(in.start(b)), begin, count, size, raw,
                     syms[0][w], syms[kSegs - 1][w], lane);
    }
  }
  __syncthreads();
  if (blk0 >= nBlocks) return;

  const uint32_t blk = blk0 + h;
  const uint32_t uw = blk < nBlocks ? min(kBlockSize, size - blk * kBlockSize) : 0u;
  const uint32_t steps0 = divUp(__builtin_amdgcn_readlane(uw, 0), 32);
  const uint32_t steps1 = divUp(__builtin_amdgcn_readlane(uw, 32), 32);
  const uint32_t steps = max(steps0, steps1);

  EncStream st[kSegs];
  uint16_t* outData[kSegs];
  const uint8_t* mySyms[kSegs];
#pragma unroll
  for (int s = 0; s < kSegs; ++s) {
    st[s].state = kStartState;
    st[s].nout = 0;
    uint8_t* slot =
        slots + ((uint64_t(s) * numInBatch + b) * MB + (blk < nBlocks ? blk : blk0)) * kSlotBytes;
    outData[s] = reinterpret_cast<uint16_t*>(slot + kStateBytesPerBlock);
    mySyms[s] = syms[s][w] + h * kBlockSize;
  }

#pragma unroll 4
  for (uint32_t t = 0; t < steps; ++t) {
    const uint32_t idx = t * 32 + l;
    const bool valid = idx < uw;
#pragma unroll
    for (int s = 0; s < kSegs; ++s) {
      const uint32_t sym = valid ? uint32_t(mySyms[s][idx]) : 0u;
      encodeStep(st[s], valid, sym, tbl[s], outData[s], h);
    }
  }

  if (uw) {
#pragma unroll
    for (int s = 0; s < kSegs; ++s) {
      uint8_t* slot = slots + ((uint64_t(s) * numInBatch + b) * MB + blk) * kSlotBytes;
      reinterpret_cast<uint32_t*>(slot)[l] = st[s].state;
      if (l == 0) cw[(uint64_t(s) * numInBatch + b) * MB + blk] = st[s].nout;
    }
  }
}

// ---------------------------------------------------------------------------
// k_coalesce: grid (ceil(maxBlocks / blocksPerWG), batch, segments).
// Each workgroup recomputes its element's block prefix (sum of roundUp(cw, 8)
// before its range + a block scan of its own range), copies its blocks'
// states and words into the final archive, and workgroup 0 writes the
// header(s), pdf table and output size.  Pad words are written as 0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sumRoundedWords(const uint32_t* __restrict__ cw, uint32_t n,
                                                    uint32_t* red) {
  uint32_t v = 0;
  for (uint32_t i = threadIdx.x; i < n; i += kThreads) v += roundUp(cw[i], 8);
  return blockSum(v, red);
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
  __shared__ uint32_t totals[2];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t seg = blockIdx.z;
  const uint32_t tid = threadIdx.x;
  const uint32_t n = in.size(b);
  const uint32_t nBlocks = divUp(n, kBlockSize);
  const uint32_t first = blockIdx.x * blocksPerWG;
  if (first >= nBlocks && blockIdx.x != 0) return;

  const uint32_t* cw0 = cw + uint64_t(b) * MB;
  const uint32_t* cwS = cw + (uint64_t(seg) * numInBatch + b) * MB;

  // archive base of this segment
  uint8_t* o = out.start(b);
  uint32_t total0Words = 0;
  if constexpr (FT != 0) {
    o += 32 + floatRawBytes(FT, n);
    if (kSegs == 2 && (seg == 1 || blockIdx.x == 0)) {
      total0Words = sumRoundedWords(cw0, nBlocks, red);
      if (seg == 1) o += roundUp64(ansOverhead(nBlocks) + 2ull * total0Words, 16);
    }
  }
  uint8_t* states = o + kANSHeaderBytes + kPdfBytes;
  uint2* bwords = reinterpret_cast<uint2*>(states + uint64_t(kStateBytesPerBlock) * nBlocks);
  uint8_t* data = reinterpret_cast<uint8_t*>(bwords + roundUp(nBlocks, 2));

  // prefix of rounded word counts
  const uint32_t sumBefore = sumRoundedWords(cwS, min(first, nBlocks), red);
  const uint32_t last = min(first + blocksPerWG, nBlocks);
  const uint32_t j = first + tid;
  const uint32_t cwj = (tid < blocksPerWG && j < last) ? cwS[j] : 0u;
  const uint32_t ex = blockExclusiveScan(roundUp(cwj, 8), red, nullptr) + sumBefore;
  pre[tid] = ex;
  __syncthreads();

  if (blockIdx.x == 0) {
    uint32_t totalWords = sumRoundedWords(cwS, nBlocks, red);
    uint32_t total1Words = 0;
    if (kSegs == 2 && seg == 0) total1Words = sumRoundedWords(cwS + uint64_t(numInBatch) * MB, nBlocks, red);
    const uint64_t ansBytes = ansOverhead(nBlocks) + 2ull * totalWords;
    if (tid == 0) {
      uint32_t* hdr = reinterpret_cast<uint32_t*>(o);
      const bool ansCk = FT == 0 && useChecksum;
      hdr[0] = kANSMagicVersion;
      hdr[1] = nBlocks;
      hdr[2] = n;
      hdr[3] = totalWords;
      hdr[4] = uint32_t(pb) | (ansCk ? 0x10u : 0u);
      hdr[5] = ansCk ? ck[b] : 0u;
      hdr[6] = 0;
      hdr[7] = 0;
      if (nBlocks & 1) bwords[nBlocks] = make_uint2(0, 0);
      if constexpr (FT == 0) {
        if (outSize) outSize[b] = uint32_t(ansBytes);
      } else if (seg == 0) {
        uint32_t* fh = reinterpret_cast<uint32_t*>(out.start(b));
        fh[0] = kFloatMagicVersion;
        fh[1] = n;
        fh[2] = uint32_t(FT) | (useChecksum ? 0x10u : 0u);
        fh[3] = useChecksum ? ck[b] : 0u;
        fh[4] = uint32_t(roundUp64(ansBytes, 16));  // GpuFloatHeader2
        fh[5] = 0;
        fh[6] = 0;
        fh[7] = 0;
        uint64_t sz = 32ull + floatRawBytes(FT, n) + ansBytes;
        if (kSegs == 2) sz += ansOverhead(nBlocks) + 2ull * total1Words;
        if (outSize) outSize[b] = uint32_t(sz);
      }
    }
    reinterpret_cast<uint16_t*>(o + kANSHeaderBytes)[tid] =
        pdf[(uint64_t(seg) * numInBatch + b) * kNumSymbols + tid];
    // zero the raw section's rounding tails (reference: uninitialised)
    if constexpr (FT != 0) {
      if (seg == 0 && tid < 16) {
        uint8_t* raw = out.start(b) + 32;
        if constexpr (FT == 1 || FT == 2) {
          if (n + tid < roundUp(n, 16)) raw[n + tid] = 0;
        } else if constexpr (FT == 3) {
          if (n + tid < roundUp(n, 8)) reinterpret_cast<uint16_t*>(raw)[n + tid] = 0;
          if (n + tid < roundUp(n, 16)) raw[2 * roundUp(n, 8) + n + tid] = 0;
        } else {
          if (n + tid < roundUp(n, 4)) reinterpret_cast<uint32_t*>(raw)[n + tid] = 0;
          if (n + tid < roundUp(n, 8))
            reinterpret_cast<uint16_t*>(raw + 4 * roundUp(n, 4))[n + tid] = 0;
        }
      }
    }
  }

  // copy this workgroup's blocks: one wave per block
  const uint32_t lane = tid & 63;
  for (uint32_t k = first + (tid >> 6); k < last; k += kWaves) {
    const uint32_t c = cwS[k];
    const uint32_t p = pre[k - first];
    const uint8_t* slot = slots + ((uint64_t(seg) * numInBatch + b) * MB + k) * kSlotBytes;
    if (lane < 32) {
      reinterpret_cast<uint32_t*>(states + uint64_t(kStateBytesPerBlock) * k)[lane] =
          reinterpret_cast<const uint32_t*>(slot)[lane];
    }
    if (lane == 0) {
      const uint32_t uwk = (k + 1 < nBlocks || n % kBlockSize == 0) ? kBlockSize : n % kBlockSize;
      bwords[k] = make_uint2((uwk << 16) | c, p);
    }
    const uint4* src = reinterpret_cast<const uint4*>(slot + kStateBytesPerBlock);
    uint4* dst = reinterpret_cast<uint4*>(data + 2ull * p);
    const uint32_t nv = divUp(c, 8);
    for (uint32_t i = lane; i < nv; i += 64) {
      uint4 v = src[i];
      const uint32_t valid = c - i * 8;  // words of this vector that are real
      if (valid < 8) {
        uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          if (2 * q + 1 >= valid) vw[q] &= (2 * q < valid) ? 0xffffu : 0u;
        }
      }
      dst[i] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
// LUT[s] = (s - cdf[sym]) << 20 | pdf << 8 | sym   (packDecodeLookup :34-44)
// Built by the whole workgroup from the archive's pdf table.
__device__ __forceinline__ void buildLut(const uint16_t* __restrict__ pdfIn, uint32_t* lut,
                                         uint32_t* red, uint32_t* cdfS, uint32_t* pdfS) {
  const uint32_t tid = threadIdx.x;
  const uint32_t p = pdfIn[tid];
  const uint32_t c = blockExclusiveScan(p, red, nullptr);
  pdfS[tid] = p;
  cdfS[tid] = c;
  __syncthreads();
  const uint32_t lane = tid & 63;
  for (uint32_t s = tid >> 6; s < kNumSymbols; s += kWaves) {
    const uint32_t ps = pdfS[s], cs = cdfS[s];
    for (uint32_t j = lane; j < ps; j += 64) lut[cs + j] = (j << 20) | (ps << 8) | s;
  }
}

struct DecStream {
  uint32_t state;
  int32_t ptr;  // one past the next word to read (half-uniform)
  const uint16_t* in;
};

// One LIFO decode step (decodeOneWarp :55-105) for both half-waves.
__device__ __forceinline__ uint32_t decodeStep(DecStream& st, bool valid, const uint32_t* lut,
                                               int pb, uint32_t h) {
  const uint32_t e = lut[st.state & ((1u << pb) - 1)];
  if (valid) st.state = __umul24((e >> 8) & 0xfffu, st.state >> pb) + (e >> 20);
  const bool read = valid && st.state < kMinState;
  const uint64_t vote = ballot(read);
  const uint32_t lo = uint32_t(vote);
  const uint32_t hi = uint32_t(vote >> 32);
  const uint32_t cnt = uint32_t(__popc(h ? hi : lo));
  const uint32_t lt = mbcnt(vote) - (h ? uint32_t(__popc(lo)) : 0u);
  if (read) {
    const uint32_t v = st.in[st.ptr - int32_t(cnt - lt)];
    st.state = (st.state << 16) | v;
  }
  st.ptr -= int32_t(cnt);
  return e & 0xffu;
}

template <int FT>
__device__ __forceinline__ void writeJoined(uint8_t* __restrict__ outB, const uint8_t* __restrict__ raw,
                                            uint32_t n, uint32_t i, uint32_t s0, uint32_t s1) {
  if constexpr (FT == 0) {
    outB[i] = uint8_t(s0);
  } else if constexpr (FT == 1) {
    reinterpret_cast<uint16_t*>(outB)[i] = uint16_t((s0 << 8) | raw[i]);
  } else if constexpr (FT == 2) {
    const uint32_t r = raw[i];
    reinterpret_cast<uint16_t*>(outB)[i] = uint16_t((s0 << 7) | (r >> 1) | ((r & 1u) << 15));
  } else if constexpr (FT == 3) {
    const uint32_t lo = reinterpret_cast<const uint16_t*>(raw)[i];
    const uint32_t hb = raw[2 * roundUp(n, 8) + i];
    reinterpret_cast<uint32_t*>(outB)[i] = rotr32((s0 << 24) | (hb << 16) | lo, 1);
  } else {
    const uint64_t lo = reinterpret_cast<const uint32_t*>(raw)[i];
    const uint64_t hb = reinterpret_cast<const uint16_t*>(raw + 4 * roundUp(n, 4))[i];
    const uint64_t v = (uint64_t(s0) << 56) | (uint64_t(s1) << 48) | (hb << 32) | lo;
    reinterpret_cast<uint64_t*>(outB)[i] = (v >> 1) | (v << 63);
  }
}

// grid (ceil(maxBlocks / 8), batch).  out.size(b) = capacity (bytes for raw,
// words for floats).
template <int FT>
__global__ __launch_bounds__(kThreads) void k_decode(BatchDesc in, BatchDesc out,
                                                     uint32_t batchOffset, int pb,
                                                     uint8_t* __restrict__ outSuccess,
                                                     uint32_t* __restrict__ outSize) {
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  __shared__ uint32_t lut[kSegs][1u << 11];
  __shared__ uint32_t red[kWaves];
  __shared__ uint32_t cdfS[kNumSymbols];
  __shared__ uint32_t pdfS[kNumSymbols];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t tid = threadIdx.x;
  const uint8_t* base = in.start(b);
  const uint32_t* fh = reinterpret_cast<const uint32_t*>(base);

  const uint8_t* arch[kSegs];
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
    if constexpr (kSegs == 2) arch[1] = arch[0] + fh[4];
  }
#pragma unroll
  for (int s = 0; s < kSegs; ++s) {
    const uint32_t* ah = reinterpret_cast<const uint32_t*>(arch[s]);
    ok = ok && ah[0] == kANSMagicVersion && (ah[4] & 0xfu) == uint32_t(pb) && ah[2] == n;
  }
  const bool success = ok && out.size(b) >= n;
  if (blockIdx.x == 0 && tid == 0) {
    if (outSuccess) outSuccess[b] = success ? 1 : 0;
    if (outSize) outSize[b] = ok ? n : 0u;
  }
  const uint32_t nBlocks = divUp(n, kBlockSize);
  if (!success || blockIdx.x * kBlocksPerWG >= nBlocks) return;

#pragma unroll
  for (int s = 0; s < kSegs; ++s) {
    buildLut(reinterpret_cast<const uint16_t*>(arch[s] + kANSHeaderBytes), lut[s], red, cdfS, pdfS);
    __syncthreads();
  }

  const uint32_t lane = tid & 63;
  const uint32_t h = lane >> 5;
  const uint32_t l = lane & 31;
  const uint32_t blk = blockIdx.x * kBlocksPerWG + 2 * (tid >> 6) + h;
  if (blockIdx.x * kBlocksPerWG + 2 * (tid >> 6) >= nBlocks) return;

  uint32_t uw = 0;
  DecStream st[kSegs];
#pragma unroll
  for (int s = 0; s < kSegs; ++s) {
    const uint8_t* states = arch[s] + kANSHeaderBytes + kPdfBytes;
    const uint2* bwords = reinterpret_cast<const uint2*>(states + uint64_t(kStateBytesPerBlock) * nBlocks);
    const uint16_t* data = reinterpret_cast<const uint16_t*>(bwords + roundUp(nBlocks, 2));
    if (blk < nBlocks) {
      st[s].state = reinterpret_cast<const uint32_t*>(states + uint64_t(kStateBytesPerBlock) * blk)[l];
      const uint2 bw = bwords[blk];
      uw = bw.x >> 16;
      st[s].ptr = int32_t(bw.x & 0xffffu);
      st[s].in = data + bw.y;
    } else {
      st[s].state = kMinState;
      st[s].ptr = 0;
      st[s].in = data;
    }
  }
  const uint32_t steps0 = divUp(__builtin_amdgcn_readlane(uw, 0), 32);
  const uint32_t steps1 = divUp(__builtin_amdgcn_readlane(uw, 32), 32);
  const uint32_t steps = max(steps0, steps1);

  uint8_t* outB = out.start(b);
  const uint8_t* raw = base + 32;
  const uint32_t blockBase = blk * kBlockSize;

#pragma unroll 4
  for (int32_t t = int32_t(steps) - 1; t >= 0; --t) {
    const uint32_t idx = uint32_t(t) * 32 + l;
    const bool valid = idx < uw;
    const uint32_t s0 = decodeStep(st[0], valid, lut[0], pb, h);
    uint32_t s1 = 0;
    if constexpr (kSegs == 2) s1 = decodeStep(st[1], valid, lut[1], pb, h);
    if (valid) writeJoined<FT>(outB, raw, n, blockBase + idx, s0, s1);
  }
}

// ---------------------------------------------------------------------------
// small utility kernels
// ---------------------------------------------------------------------------
// XOR-of-bytes checksum of `size(b) * unitBytes` bytes (checksumBatch,
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
    const uint8_t* p = in.start(b) + begin;
    const uint32_t n = uint32_t(min(uint64_t(chunkBytes), size - begin));
    for (uint32_t i = threadIdx.x; i < n; i += kThreads) ck ^= p[i];
  }
  ck = waveXor(ck);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ck;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t v = red[0] ^ red[1] ^ red[2] ^ red[3];
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
  const uint32_t* h = reinterpret_cast<const uint32_t*>(in.start(b));
  const bool ok = h[0] == (isFloat ? kFloatMagicVersion : kANSMagicVersion);
  if (isFloat) {
    if (sizes) sizes[b] = ok ? h[1] : 0u;
    if (types) types[b] = ok ? (h[2] & 0xfu) : 0u;
    if (checksums) checksums[b] = h[3];
  } else {
    if (sizes) sizes[b] = ok ? h[2] : 0u;
    if (checksums) checksums[b] = h[5];
  }
}

} // namespace dietgpu
