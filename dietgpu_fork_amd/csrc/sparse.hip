// Sparse float codec: nonzero bitmap + per-element exclusive scan +
// compaction, wrapped around the dense float codec.
//
// Reference: float/GpuSparseFloatCompress.{cu,cuh},
// float/GpuSparseFloatDecompress.{cu,cuh}.  The reference scans with one
// thrust::exclusive_scan per batch element on the legacy default stream
// between two cudaDeviceSynchronize calls (GpuSparseFloatCompress.cuh:360-369);
// here the scan is a batched two-level scan over 4096-word tiles, fully
// stream-ordered (no host or device-wide sync).
//
// Wire format: 16 B header {u32 N, 12 B zero}, bitmap
// ceil(N/8) bytes (bit 7 of byte k <-> element 8k) padded to 16, then a dense
// float archive of the compacted list.  The compacted list reproduces the
// reference's n-2 quirk (fill_comp_input :162-184): when x[N-2] == 0 one extra
// slot (written as 0 here, uninitialised in the reference) precedes x[N-1].
#include <algorithm>
#include <cstring>
#include <vector>

#include "codec_internal.h"
#include "common.h"
#include "dietgpu/GpuFloatCodec.h"
#include "decode.h"
#include "encode.h"
#include "profile.h"

namespace dietgpu {

namespace {

constexpr uint32_t kTileWords = 4096;   // 4 waves x 16 steps x 64 lanes
constexpr uint32_t kMaxGridY = 65535;

template <int FT>
using WordOf = typename FloatTraits<FT>::WordT;

// flags of words [base, base + 64) as a lane mask <-> packed bitmap u64
__device__ __forceinline__ uint64_t maskToBitmap(uint64_t m) {
  return __builtin_bswap64(__builtin_bitreverse64(m));
}

template <int FT>
__device__ __forceinline__ bool isNonzero(WordOf<FT> w) {
  return w != 0;  // bitwise: -0.0 is "nonzero" (generate_bitmap :56)
}

// s1: bitmap + per-tile nonzero count.  grid (tiles, batch)
template <int FT>
__global__ __launch_bounds__(kThreads) void k_sparseBitmap(BatchDesc in, const uint64_t* outPtrs,
                                                           uint32_t batchOffset,
                                                           uint32_t tilesPerElem,
                                                           uint32_t* __restrict__ tileCounts) {
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = in.size(b);
  const uint32_t tile = blockIdx.x;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const WordOf<FT>* x = reinterpret_cast<const WordOf<FT>*>(in.start(b));
  uint8_t* o = reinterpret_cast<uint8_t*>(outPtrs[b]);
  const uint32_t bmBytes = (n + 7) / 8, bmPad = roundUp(bmBytes, 16);
  if (tile == 0 && threadIdx.x == 0) {
    reinterpret_cast<uint4*>(o)[0] = make_uint4(n, 0, 0, 0);
  }
  uint32_t cnt = 0;
  const uint32_t base = tile * kTileWords + w * (kTileWords / kWaves);
  if (base < n) {
#pragma unroll 4
    for (uint32_t j = 0; j < kTileWords / kWaves / 64; ++j) {
      const uint32_t i0 = base + 64 * j;
      if (i0 >= n) break;
      const uint32_t i = i0 + lane;
      const bool f = i < n && isNonzero<FT>(x[i]);
      const uint64_t m = ballot(f);
      cnt += uint32_t(__popcll(m));
      if (lane == 0) {
        uint64_t* dst = reinterpret_cast<uint64_t*>(o + 16 + i0 / 8);
        dst[0] = maskToBitmap(m);
        // zero the 16-byte padding after the last bitmap word
        const uint32_t end = i0 / 8 + 8;
        if (i0 + 64 >= n && end < bmPad) dst[1] = 0;
      }
    }
  }
  cnt = blockSum<kThreads>(lane == 0 ? cnt : 0u, red);
  if (threadIdx.x == 0) tileCounts[uint64_t(b) * tilesPerElem + tile] = cnt;
}

// s2 / d2: exclusive scan of tile counts per element (in place); optional
// compacted-list length with the n-2 quirk.  grid (batch)
template <int FT>
__global__ __launch_bounds__(kThreads) void k_sparseScan(BatchDesc in, uint32_t batchOffset,
                                                         uint32_t tilesPerElem,
                                                         const uint32_t* __restrict__ sizes,
                                                         uint32_t* __restrict__ tileCounts,
                                                         uint32_t* __restrict__ listLen) {
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.x;
  const uint32_t n = sizes ? sizes[b] : in.size(b);
  const uint32_t tiles = min(divUp(n, kTileWords), tilesPerElem);
  uint32_t* tc = tileCounts + uint64_t(b) * tilesPerElem;
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < tiles; t0 += kThreads) {
    const uint32_t t = t0 + threadIdx.x;
    const uint32_t v = t < tiles ? tc[t] : 0u;
    uint32_t total = 0;
    const uint32_t ex = blockExclusiveScan<kThreads>(v, red, &total);
    if (t < tiles) tc[t] = carry + ex;
    carry += total;
    __syncthreads();
  }
  if (listLen && threadIdx.x == 0) {
    const WordOf<FT>* x = reinterpret_cast<const WordOf<FT>*>(in.start(b));
    uint32_t len = 0;
    if (n == 1) {
      len = isNonzero<FT>(x[0]) ? 1u : 0u;
    } else if (n >= 2) {
      // idx[n-2] + flag[n-1] + 1 == nnz - flag[n-2] + 1
      len = carry - (isNonzero<FT>(x[n - 2]) ? 1u : 0u) + 1u;
    }
    listLen[b] = len;
  }
}

// s3: scatter nonzeros into the compacted list.  grid (tiles, batch)
template <int FT>
__global__ __launch_bounds__(kThreads) void k_sparseCompact(BatchDesc in, uint32_t batchOffset,
                                                            uint32_t tilesPerElem,
                                                            const uint32_t* __restrict__ tileOff,
                                                            const uint64_t* __restrict__ listPtrs) {
  constexpr uint32_t kSteps = kTileWords / kWaves / 64;
  __shared__ uint32_t waveCnt[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = in.size(b);
  const uint32_t tile = blockIdx.x;
  if (tile * kTileWords >= n) return;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const WordOf<FT>* x = reinterpret_cast<const WordOf<FT>*>(in.start(b));
  WordOf<FT>* list = reinterpret_cast<WordOf<FT>*>(listPtrs[b]);
  const uint32_t base = tile * kTileWords + w * (kTileWords / kWaves);
  WordOf<FT> v[kSteps];
  uint64_t m[kSteps];
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t i = base + 64 * j + lane;
    v[j] = i < n ? x[i] : WordOf<FT>(0);
    m[j] = ballot(v[j] != 0);
    cnt += uint32_t(__popcll(m[j]));
  }
  if (lane == 0) waveCnt[w] = cnt;
  __syncthreads();
  uint32_t pos = tileOff[uint64_t(b) * tilesPerElem + tile];
  for (uint32_t k = 0; k < w; ++k) pos += waveCnt[k];
  // the n-2 quirk: x[n-1] goes to idx[n-2] + 1 and, when x[n-2] == 0, the
  // skipped slot idx[n-2] is part of the list (written as 0)
  const bool gap = n >= 2 && x[n - 2] == 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t i = base + 64 * j + lane;
    const uint32_t dst = pos + mbcnt(m[j]);
    if (i + 1 == n && gap) {
      list[dst] = WordOf<FT>(0);
      if (v[j] != 0) list[dst + 1] = v[j];
    } else if (v[j] != 0) {
      list[dst] = v[j];
    }
    pos += uint32_t(__popcll(m[j]));
  }
}

__global__ void k_sparseAddSizes(BatchDesc in, uint32_t numInBatch, uint32_t* __restrict__ outSize) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < numInBatch && outSize) outSize[b] += 16 + roundUp((in.size(b) + 7) / 8, 16);
}

// d1: headers -> dense-archive pointers + per-tile popcounts of the bitmap.
// grid (tiles, batch)
__global__ __launch_bounds__(kThreads) void k_sparseHeaders(BatchDesc in, uint32_t batchOffset,
                                                            uint32_t tilesPerElem,
                                                            uint64_t* __restrict__ densePtrs,
                                                            uint32_t* __restrict__ sizes,
                                                            uint32_t* __restrict__ tileCounts) {
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint8_t* a = in.start(b);
  const uint32_t n = reinterpret_cast<const uint32_t*>(a)[0];
  const uint32_t tile = blockIdx.x;
  if (tile == 0 && threadIdx.x == 0) {
    densePtrs[b] = reinterpret_cast<uint64_t>(a + 16 + roundUp((n + 7) / 8, 16));
    sizes[b] = n;
  }
  if (tile >= tilesPerElem) return;
  uint32_t c = 0;
  const uint32_t bytes0 = tile * (kTileWords / 8);
  const uint32_t bmBytes = (n + 7) / 8;
  for (uint32_t k = threadIdx.x; k < kTileWords / 8; k += kThreads) {
    if (bytes0 + k < bmBytes) c += __popc(a[16 + bytes0 + k]);
  }
  c = blockSum<kThreads>(c, red);
  if (threadIdx.x == 0) tileCounts[uint64_t(b) * tilesPerElem + tile] = c;
}

// d3: expand the decoded nonzero list into the output.  grid (tiles, batch)
template <int FT>
__global__ __launch_bounds__(kThreads) void k_sparseExpand(BatchDesc in, BatchDesc out,
                                                           uint32_t batchOffset,
                                                           uint32_t tilesPerElem,
                                                           const uint32_t* __restrict__ sizes,
                                                           const uint32_t* __restrict__ tileOff,
                                                           const uint64_t* __restrict__ listPtrs,
                                                           const uint8_t* __restrict__ denseOk,
                                                           uint8_t* __restrict__ outSuccess,
                                                           uint32_t* __restrict__ outSize) {
  constexpr uint32_t kSteps = kTileWords / kWaves / 64;
  __shared__ uint32_t waveCnt[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = sizes[b];
  const bool ok = denseOk[b] != 0 && out.size(b) >= n;
  const uint32_t tile = blockIdx.x;
  if (tile == 0 && threadIdx.x == 0) {
    if (outSuccess) outSuccess[b] = ok ? 1 : 0;
    if (outSize) outSize[b] = n;  // fill_in_nonzeros :107-109
  }
  if (!ok || tile * kTileWords >= n) return;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint8_t* bm = in.start(b) + 16;
  const WordOf<FT>* list = reinterpret_cast<const WordOf<FT>*>(listPtrs[b]);
  WordOf<FT>* y = reinterpret_cast<WordOf<FT>*>(out.start(b));
  const uint32_t base = tile * kTileWords + w * (kTileWords / kWaves);
  uint64_t m[kSteps];
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t i0 = base + 64 * j;
    m[j] = i0 < n ? maskToBitmap(*reinterpret_cast<const uint64_t*>(bm + i0 / 8)) : 0ull;
    if (i0 < n && n - i0 < 64) m[j] &= (1ull << (n - i0)) - 1;
    cnt += uint32_t(__popcll(m[j]));
  }
  if (lane == 0) waveCnt[w] = cnt;
  __syncthreads();
  uint32_t pos = tileOff[uint64_t(b) * tilesPerElem + tile];
  for (uint32_t k = 0; k < w; ++k) pos += waveCnt[k];
  // x[n-1] is read from idx[n-2] + 1 (fill_in_nonzeros :139-144)
  const bool gap = n >= 2 && ((bm[(n - 2) / 8] >> (7 - (n - 2) % 8)) & 1) == 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t i = base + 64 * j + lane;
    if (i < n) {
      const bool f = (m[j] >> lane) & 1;
      uint32_t src = pos + mbcnt(m[j]);
      if (i + 1 == n && gap) src += 1;
      y[i] = f ? list[src] : WordOf<FT>(0);
    }
    pos += uint32_t(__popcll(m[j]));
  }
}

template <int FT>
void sparseCompressT(StackDeviceMemory& res, const FloatCompressConfig& config, uint32_t nb,
                     const BatchDesc& in, uint32_t maxN, const uint64_t* outPtrs_dev,
                     const BatchDesc& denseOut, uint32_t* outSize_dev, hipStream_t s) {
  const uint32_t tiles = std::max(1u, divUp(maxN, kTileWords));
  auto tileCounts = res.alloc<uint32_t>(s, size_t(nb) * tiles);
  auto listLen = res.alloc<uint32_t>(s, nb);
  auto list = res.alloc<uint8_t>(s, size_t(nb) * (roundUp(maxN, 16) + 16) * sizeof(WordOf<FT>));
  std::vector<uint64_t> listPtrs(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    listPtrs[i] = reinterpret_cast<uint64_t>(list.data()) +
                  uint64_t(i) * (roundUp(maxN, 16) + 16) * sizeof(WordOf<FT>);
  }
  auto listPtrsDev = res.alloc<uint64_t>(s, nb);
  StackDeviceMemory::copyToDevice(listPtrsDev.data(), listPtrs.data(), nb * 8, s);
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    {
      prof::Scope p("sparse", s);
      k_sparseBitmap<FT><<<dim3(tiles, ny), kThreads, 0, s>>>(in, outPtrs_dev, y0, tiles,
                                                               tileCounts.data());
      HIP_LAUNCH_CHECK();
      k_sparseScan<FT><<<ny, kThreads, 0, s>>>(in, y0, tiles, nullptr, tileCounts.data(),
                                               listLen.data());
      HIP_LAUNCH_CHECK();
      k_sparseCompact<FT><<<dim3(tiles, ny), kThreads, 0, s>>>(in, y0, tiles, tileCounts.data(),
                                                                listPtrsDev.data());
      HIP_LAUNCH_CHECK();
    }
  }
  // (the compacted lists are 16 B-aligned slices of one arena allocation)
  floatCompressDescs(res, config, nb, BatchDesc::pointers(listPtrsDev.data(), listLen.data()),
                     maxN, denseOut, outSize_dev, s, nullptr, true);
  if (outSize_dev) {
    k_sparseAddSizes<<<divUp(nb, 128), 128, 0, s>>>(in, nb, outSize_dev);
    HIP_LAUNCH_CHECK();
  }
}

template <int FT>
FloatDecompressStatus sparseDecompressT(StackDeviceMemory& res,
                                        const FloatDecompressConfig& config, uint32_t nb,
                                        const BatchDesc& in, const BatchDesc& out,
                                        uint32_t maxCap, uint8_t* outSuccess_dev,
                                        uint32_t* outSize_dev, hipStream_t s) {
  const uint32_t tiles = std::max(1u, divUp(maxCap, kTileWords));
  auto densePtrs = res.alloc<uint64_t>(s, nb);
  auto sizes = res.alloc<uint32_t>(s, nb);
  auto tileCounts = res.alloc<uint32_t>(s, size_t(nb) * tiles);
  auto denseOk = res.alloc<uint8_t>(s, nb);
  auto list = res.alloc<uint8_t>(s, size_t(nb) * (roundUp(maxCap, 16) + 16) * sizeof(WordOf<FT>));
  std::vector<uint64_t> listPtrs(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    listPtrs[i] = reinterpret_cast<uint64_t>(list.data()) +
                  uint64_t(i) * (roundUp(maxCap, 16) + 16) * sizeof(WordOf<FT>);
  }
  auto listPtrsDev = res.alloc<uint64_t>(s, nb);
  StackDeviceMemory::copyToDevice(listPtrsDev.data(), listPtrs.data(), nb * 8, s);
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    prof::Scope p("sparse", s);
    k_sparseHeaders<<<dim3(tiles, ny), kThreads, 0, s>>>(in, y0, tiles, densePtrs.data(),
                                                          sizes.data(), tileCounts.data());
    HIP_LAUNCH_CHECK();
    k_sparseScan<FT><<<ny, kThreads, 0, s>>>(in, y0, tiles, sizes.data(), tileCounts.data(),
                                             nullptr);
    HIP_LAUNCH_CHECK();
  }
  // dense decode of the nonzero list (capacity: the largest output)
  auto cfg = config;
  cfg.useChecksum = false;
  floatDecompressDescs(res, cfg, nb, BatchDesc::pointers(densePtrs.data(), nullptr),
                       BatchDesc::pointers(listPtrsDev.data(), nullptr, maxCap + 1), maxCap + 1,
                       denseOk.data(), nullptr, s);
  FloatDecompressStatus status;
  if (config.useChecksum) {
    // verify the dense archive's checksum over the bytes it was computed on
    // (the first listLen bytes of the nonzero list)
    auto denseLen = res.alloc<uint32_t>(s, nb);
    k_info<<<divUp(nb, 128), 128, 0, s>>>(BatchDesc::pointers(densePtrs.data(), nullptr), nb, true,
                                          denseLen.data(), nullptr, nullptr);
    HIP_LAUNCH_CHECK();
    status.errorInfo = verifyChecksums(res, nb, BatchDesc::pointers(densePtrs.data(), nullptr), true,
                                       BatchDesc::pointers(listPtrsDev.data(), denseLen.data()),
                                       maxCap + 1, s);
    if (!status.errorInfo.empty()) status.error = FloatDecompressError::ChecksumMismatch;
  }
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    prof::Scope p("sparse", s);
    k_sparseExpand<FT><<<dim3(tiles, ny), kThreads, 0, s>>>(
        in, out, y0, tiles, sizes.data(), tileCounts.data(), listPtrsDev.data(), denseOk.data(),
        outSuccess_dev, outSize_dev);
    HIP_LAUNCH_CHECK();
  }
  return status;
}

}  // namespace

uint32_t getMaxSparseFloatCompressedSize(FloatType ft, uint32_t size) {
  const uint64_t v = 16ull + roundUp64((uint64_t(size) + 7) / 8, 16) + getMaxFloatCompressedSize(ft, size);
  DG_CHECK(v <= uint64_t(INT32_MAX), "input too large: " << size << " float words");
  return uint32_t(v);
}

void floatCompressSparse(StackDeviceMemory& res, const FloatCompressConfig& config,
                         uint32_t numInBatch, const void** in, const uint32_t* inSize, void** out,
                         uint32_t* outSize_dev, hipStream_t stream) {
  if (numInBatch == 0) return;
  DG_CHECK(!config.ansConfig.useChecksum, "ANS-level checksum not allowed in float mode");
  const int ft = int(config.floatType);
  DG_CHECK(ft >= 1 && ft <= 4, "bad float type");
  const uint32_t ws = floatWordBytes(ft);
  std::vector<uint64_t> ip(numInBatch), op(numInBatch), dp(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint32_t maxN = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    op[i] = reinterpret_cast<uint64_t>(out[i]);
    DG_CHECK(op[i] % 16 == 0, "out[i] must be 16-byte aligned");
    DG_CHECK(ip[i] % ws == 0, "input not word aligned");
    sz[i] = inSize[i];
    dp[i] = op[i] + 16 + roundUp((sz[i] + 7) / 8, 16);
    maxN = std::max(maxN, sz[i]);
  }
  std::vector<uint64_t> ptrs(ip);
  ptrs.insert(ptrs.end(), op.begin(), op.end());
  ptrs.insert(ptrs.end(), dp.begin(), dp.end());
  auto tbl = res.alloc<uint8_t>(stream, ptrs.size() * 8 + sz.size() * 4);
  std::vector<uint8_t> host(ptrs.size() * 8 + sz.size() * 4);
  std::memcpy(host.data(), ptrs.data(), ptrs.size() * 8);
  std::memcpy(host.data() + ptrs.size() * 8, sz.data(), sz.size() * 4);
  StackDeviceMemory::copyToDevice(tbl.data(), host.data(), host.size(), stream);
  const uint64_t* ipD = reinterpret_cast<const uint64_t*>(tbl.data());
  const uint64_t* opD = ipD + numInBatch;
  const uint64_t* dpD = opD + numInBatch;
  const uint32_t* szD = reinterpret_cast<const uint32_t*>(dpD + numInBatch);
  auto inD = BatchDesc::pointers(ipD, szD);
  auto denseOut = BatchDesc::pointers(dpD, nullptr);
  switch (ft) {
    case 1: sparseCompressT<1>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream); break;
    case 2: sparseCompressT<2>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream); break;
    case 3: sparseCompressT<3>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream); break;
    default: sparseCompressT<4>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream); break;
  }
}

FloatDecompressStatus floatDecompressSparse(StackDeviceMemory& res,
                                            const FloatDecompressConfig& config,
                                            uint32_t numInBatch, const void** in, void** out,
                                            const uint32_t* outCapacity, uint8_t* outSuccess_dev,
                                            uint32_t* outSize_dev, hipStream_t stream) {
  if (numInBatch == 0) return FloatDecompressStatus();
  DG_CHECK(!config.ansConfig.useChecksum, "ANS-level checksum not allowed in float mode");
  const int ft = int(config.floatType);
  DG_CHECK(ft >= 1 && ft <= 4, "bad float type");
  std::vector<uint64_t> ptrs(2 * numInBatch);
  std::vector<uint32_t> cap(numInBatch);
  uint32_t maxCap = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ptrs[i] = reinterpret_cast<uint64_t>(in[i]);
    ptrs[numInBatch + i] = reinterpret_cast<uint64_t>(out[i]);
    cap[i] = outCapacity[i];
    maxCap = std::max(maxCap, cap[i]);
  }
  auto tbl = res.alloc<uint8_t>(stream, ptrs.size() * 8 + cap.size() * 4);
  std::vector<uint8_t> host(ptrs.size() * 8 + cap.size() * 4);
  std::memcpy(host.data(), ptrs.data(), ptrs.size() * 8);
  std::memcpy(host.data() + ptrs.size() * 8, cap.data(), cap.size() * 4);
  StackDeviceMemory::copyToDevice(tbl.data(), host.data(), host.size(), stream);
  const uint64_t* ipD = reinterpret_cast<const uint64_t*>(tbl.data());
  const uint64_t* opD = ipD + numInBatch;
  const uint32_t* capD = reinterpret_cast<const uint32_t*>(opD + numInBatch);
  auto inD = BatchDesc::pointers(ipD, nullptr);
  auto outD = BatchDesc::pointers(opD, capD);
  switch (ft) {
    case 1: return sparseDecompressT<1>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
    case 2: return sparseDecompressT<2>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
    case 3: return sparseDecompressT<3>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
    default: return sparseDecompressT<4>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
  }
}

}  // namespace dietgpu
