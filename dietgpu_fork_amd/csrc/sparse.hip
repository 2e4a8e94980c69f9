// Sparse float codec: nonzero bitmap + per-element exclusive scan +
// compaction, wrapped around the dense float codec.
//
// Reference: float/GpuSparseFloatCompress.{cu,cuh},
// float/GpuSparseFloatDecompress.{cu,cuh}.  The reference scans with one
// thrust::exclusive_scan per batch element on the legacy default stream
// between two cudaDeviceSynchronize calls (GpuSparseFloatCompress.cuh:360-369);
// here compression is ONE pass over the input (k_sparseCompress: bitmap, tile
// counts, decoupled look-back over the tiles of an element, compaction), and
// decompression scans the bitmap's tile popcounts, fully stream-ordered (no
// host or device-wide sync).
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
#include "lookback.h"
#include "profile.h"
#include "sync_arena.h"

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

// Compression in one pass.  grid (tiles, batch); a workgroup takes one
// 4096-word tile of one element: it loads the tile (16 B vectors when the
// element is 16 B aligned, coalesced) into LDS, then each wave takes 1024
// consecutive words as 16 steps of 64 lanes: the ballot of nonzero flags is
// the step's 64 bitmap bits (generate_bitmap :40-71) and its nonzeros'
// ranks (v_mbcnt).  The tile's nonzero count goes through a decoupled
// look-back over the element's earlier tiles (epoch-tagged flags, lookback.h);
// then the nonzeros are scattered into the compacted list (fill_comp_input
// :119-185, n-2 quirk included).  A look-back that runs out of polls marks the
// element (its final outSize becomes 0) instead of guessing.
template <int FT, bool kVec>
__global__ __launch_bounds__(kThreads) void k_sparseCompress(BatchDesc in, const uint64_t* outPtrs,
                                                             uint32_t batchOffset, uint32_t tilesPerElem,
                                                             const uint64_t* __restrict__ listPtrs,
                                                             uint32_t* __restrict__ listLen,
                                                             uint64_t* __restrict__ flags, uint32_t epoch,
                                                             uint32_t spinCap, uint8_t* __restrict__ poisoned,
                                                             uint32_t* __restrict__ err) {
  using W = WordOf<FT>;
  constexpr uint32_t kSteps = kTileWords / kWaves / 64;
  constexpr uint32_t kVecs = kTileWords * sizeof(W) / 16 / kThreads;  // 16 B vectors per thread
  __shared__ __attribute__((aligned(16))) W buf[kTileWords];
  __shared__ uint32_t waveCnt[kWaves];
  __shared__ uint32_t exclS;
  __shared__ uint32_t poisonS;
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = in.size(b);
  const uint32_t tile = blockIdx.x;
  if (tile * kTileWords >= n && !(n == 0 && tile == 0)) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  gp<const W> x = (gp<const W>)in.start(b);
  gp<uint8_t> o = (gp<uint8_t>)outPtrs[b];
  if (tile == 0 && tid == 0) st16(o, make_uint4(n, 0, 0, 0));
  const uint32_t t0 = tile * kTileWords;
  const uint32_t tileN = min(kTileWords, n - min(n, t0));
  // tile -> LDS (words past the element read as 0)
  if (kVec) {
    constexpr uint32_t kWPV = 16 / sizeof(W);
#pragma unroll
    for (uint32_t v = 0; v < kVecs; ++v) {
      const uint32_t wi = (v * kThreads + tid) * kWPV;  // first word of the vector
      uint4 val = make_uint4(0, 0, 0, 0);
      if (wi + kWPV <= tileN) {
        val = ld16((gp<const uint4>)(x + t0 + wi));
      } else if (wi < tileN) {
        W tmp[kWPV];
#pragma unroll
        for (uint32_t k = 0; k < kWPV; ++k) tmp[k] = wi + k < tileN ? x[t0 + wi + k] : W(0);
        __builtin_memcpy(&val, tmp, 16);
      }
      *(lp<u32x4>)&buf[wi] = u32x4{val.x, val.y, val.z, val.w};
    }
  } else {
#pragma unroll 4
    for (uint32_t i = tid; i < kTileWords; i += kThreads) buf[i] = i < tileN ? x[t0 + i] : W(0);
  }
  __syncthreads();
  // bitmap bits and counts, wave w: words [w * 1024, (w + 1) * 1024) of the tile
  const uint32_t bmBytes = (n + 7) / 8, bmPad = roundUp(bmBytes, 16);
  uint64_t m[kSteps];
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t q = w * (kTileWords / kWaves) + 64 * j;  // step's first word in the tile
    m[j] = ballot(buf[q + lane] != W(0));  // bitwise: -0.0 is "nonzero" (generate_bitmap :56)
    cnt += uint32_t(__popcll(m[j]));
    const uint32_t i0 = t0 + q;
    if (lane == 0 && i0 < n) {
      gp<uint64_t> dst = (gp<uint64_t>)(o + 16 + i0 / 8);
      dst[0] = maskToBitmap(m[j]);
      // zero the 16-byte padding after the last bitmap word
      const uint32_t end = i0 / 8 + 8;
      if (i0 + 64 >= n && end < bmPad) dst[1] = 0;
    }
  }
  if (lane == 0) waveCnt[w] = cnt;
  __syncthreads();
  if (w == 0) {
    const uint32_t total = waveCnt[0] + waveCnt[1] + waveCnt[2] + waveCnt[3];
    bool pz = false;
    const uint32_t excl =
        lookBackPoison(G(flags) + uint64_t(b) * tilesPerElem, tile, total, epoch, spinCap, pz);
    if (lane == 0) {
      exclS = excl;
      poisonS = pz ? 1u : 0u;
      if ((tile + 1) * kTileWords >= n) {  // the element's last tile
        uint32_t len = 0;
        if (n == 1) {
          len = buf[0] != W(0) ? 1u : 0u;
        } else if (n >= 2) {
          // idx[n-2] + flag[n-1] + 1 == nnz - flag[n-2] + 1
          len = excl + total - (x[n - 2] != W(0) ? 1u : 0u) + 1u;
        }
        listLen[b] = pz ? 0u : len;
        poisoned[b] = pz ? 1 : 0;
        if (pz) __hip_atomic_fetch_add(G(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  __syncthreads();
  if (poisonS) return;
  uint32_t pos = exclS;
  for (uint32_t k = 0; k < w; ++k) pos += waveCnt[k];
  gp<W> list = (gp<W>)listPtrs[b];
  // the n-2 quirk: x[n-1] goes to idx[n-2] + 1 and, when x[n-2] == 0, the
  // skipped slot idx[n-2] is part of the list (written as 0)
  const bool gap = n >= 2 && x[n - 2] == W(0);
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t q = w * (kTileWords / kWaves) + 64 * j + lane;
    const uint32_t i = t0 + q;
    const W v = buf[q];
    const uint32_t dst = pos + mbcnt(m[j]);
    if (i + 1 == n && gap) {
      list[dst] = W(0);
      if (v != W(0)) list[dst + 1] = v;
    } else if (v != W(0)) {
      list[dst] = v;
    }
    pos += uint32_t(__popcll(m[j]));
  }
}

// outSize of the sparse archive: header + padded bitmap + dense archive; 0 for
// an element whose compaction was abandoned (k_sparseCompress)
__global__ void k_sparseAddSizes(BatchDesc in, uint32_t numInBatch, const uint8_t* __restrict__ poisoned,
                                 uint32_t* __restrict__ outSize) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < numInBatch && outSize)
    outSize[b] = poisoned[b] ? 0u : outSize[b] + 16 + roundUp((in.size(b) + 7) / 8, 16);
}

// d1: headers -> dense-archive pointers and sizes.  One thread per element.
__global__ void k_sparseHeaders(BatchDesc in, uint32_t numInBatch, uint64_t* __restrict__ densePtrs,
                                uint32_t* __restrict__ sizes) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= numInBatch) return;
  const uint8_t* a = in.start(b);
  const uint32_t n = reinterpret_cast<const uint32_t*>(a)[0];
  densePtrs[b] = reinterpret_cast<uint64_t>(a + 16 + roundUp((n + 7) / 8, 16));
  sizes[b] = n;
}

// d3: expand the decoded nonzero list into the output (fill_in_nonzeros
// :95-144).  grid (tiles, batch); per 4096-word tile: the bitmap's popcount,
// a decoupled look-back over the element's earlier tiles for the tile's
// first list index, the expansion into LDS, and 16 B stores when the output
// is 16 B aligned.  The element's last tile reports success and size (a
// look-back that runs out of polls reports failure).
template <int FT, bool kVec>
__global__ __launch_bounds__(kThreads) void k_sparseExpand(BatchDesc in, BatchDesc out, uint32_t batchOffset,
                                                           uint32_t tilesPerElem, const uint32_t* __restrict__ sizes,
                                                           const uint64_t* __restrict__ listPtrs,
                                                           const uint8_t* __restrict__ denseOk,
                                                           uint8_t* __restrict__ outSuccess,
                                                           uint32_t* __restrict__ outSize, uint64_t* __restrict__ flags,
                                                           uint32_t epoch, uint32_t spinCap,
                                                           uint32_t* __restrict__ err) {
  using W = WordOf<FT>;
  constexpr uint32_t kSteps = kTileWords / kWaves / 64;
  constexpr uint32_t kVecs = kTileWords * sizeof(W) / 16 / kThreads;
  __shared__ __attribute__((aligned(16))) W buf[kTileWords];
  __shared__ uint32_t waveCnt[kWaves];
  __shared__ uint32_t exclS, poisonS;
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = sizes[b];
  const bool ok = denseOk[b] != 0 && out.size(b) >= n;
  const uint32_t tile = blockIdx.x;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (n == 0) {
    if (tile == 0 && tid == 0) {
      if (outSuccess) outSuccess[b] = ok ? 1 : 0;
      if (outSize) outSize[b] = 0;
    }
    return;
  }
  if (tile * kTileWords >= n) return;
  const bool last = (tile + 1) * kTileWords >= n;
  if (!ok) {
    if (last && tid == 0) {
      if (outSuccess) outSuccess[b] = 0;
      if (outSize) outSize[b] = n;  // fill_in_nonzeros :107-109
    }
    return;
  }
  gp<const uint8_t> bm = (gp<const uint8_t>)in.start(b) + 16;
  const uint32_t t0 = tile * kTileWords;
  uint64_t m[kSteps];
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t i0 = t0 + w * (kTileWords / kWaves) + 64 * j;
    m[j] = i0 < n ? maskToBitmap(*(gp<const uint64_t>)(bm + i0 / 8)) : 0ull;
    if (i0 < n && n - i0 < 64) m[j] &= (1ull << (n - i0)) - 1;
    cnt += uint32_t(__popcll(m[j]));
  }
  if (lane == 0) waveCnt[w] = cnt;
  __syncthreads();
  if (w == 0) {
    bool pz = false;
    const uint32_t total = waveCnt[0] + waveCnt[1] + waveCnt[2] + waveCnt[3];
    const uint32_t excl =
        lookBackPoison(G(flags) + uint64_t(b) * tilesPerElem, tile, total, epoch, spinCap, pz);
    if (lane == 0) {
      exclS = excl;
      poisonS = pz ? 1u : 0u;
      if (last) {
        if (outSuccess) outSuccess[b] = pz ? 0 : 1;
        if (outSize) outSize[b] = n;
        if (pz) __hip_atomic_fetch_add(G(err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  __syncthreads();
  if (poisonS) return;
  uint32_t pos = exclS;
  for (uint32_t k = 0; k < w; ++k) pos += waveCnt[k];
  gp<const W> list = (gp<const W>)listPtrs[b];
  // x[n-1] is read from idx[n-2] + 1 (fill_in_nonzeros :139-144)
  const bool gap = n >= 2 && ((bm[(n - 2) / 8] >> (7 - (n - 2) % 8)) & 1) == 0;
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t q = w * (kTileWords / kWaves) + 64 * j + lane;
    const uint32_t i = t0 + q;
    const bool f = (m[j] >> lane) & 1;
    uint32_t src = pos + mbcnt(m[j]);
    if (i + 1 == n && gap) src += 1;
    buf[q] = f ? list[src] : W(0);
    pos += uint32_t(__popcll(m[j]));
  }
  __syncthreads();
  gp<W> y = (gp<W>)out.start(b);
  const uint32_t tileN = min(kTileWords, n - t0);
  if (kVec) {
    constexpr uint32_t kWPV = 16 / sizeof(W);
#pragma unroll
    for (uint32_t v = 0; v < kVecs; ++v) {
      const uint32_t wi = (v * kThreads + tid) * kWPV;
      if (wi + kWPV <= tileN) {
        const u32x4 val = *(lp<const u32x4>)&buf[wi];
        st16((gp<void>)(y + t0 + wi), make_uint4(val.x, val.y, val.z, val.w));
      } else {
        for (uint32_t k = wi; k < tileN && k < wi + kWPV; ++k) y[t0 + k] = buf[k];
      }
    }
  } else {
    for (uint32_t i = tid; i < tileN; i += kThreads) y[t0 + i] = buf[i];
  }
}

template <int FT>
void sparseCompressT(StackDeviceMemory& res, const FloatCompressConfig& config, uint32_t nb,
                     const BatchDesc& in, uint32_t maxN, const uint64_t* outPtrs_dev,
                     const BatchDesc& denseOut, uint32_t* outSize_dev, hipStream_t s, bool inAligned16) {
  const uint32_t tiles = std::max(1u, divUp(maxN, kTileWords));
  auto listLen = res.alloc<uint32_t>(s, nb);
  auto poisoned = res.alloc<uint8_t>(s, nb);
  auto list = res.alloc<uint8_t>(s, size_t(nb) * (roundUp(maxN, 16) + 16) * sizeof(WordOf<FT>));
  std::vector<uint64_t> listPtrs(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    listPtrs[i] = reinterpret_cast<uint64_t>(list.data()) +
                  uint64_t(i) * (roundUp(maxN, 16) + 16) * sizeof(WordOf<FT>);
  }
  auto listPtrsDev = res.alloc<uint64_t>(s, nb);
  StackDeviceMemory::copyToDevice(listPtrsDev.data(), listPtrs.data(), nb * 8, s);
  {
    // epoch-tagged look-back flags, one per (element, tile)
    SyncLease lease(res, s, size_t(nb) * tiles * 8);
    for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
      const uint32_t ny = std::min(kMaxGridY, nb - y0);
      prof::Scope p("sparse", s);
      auto* f = reinterpret_cast<uint64_t*>(lease.base);
      if (inAligned16) {
        k_sparseCompress<FT, true><<<dim3(tiles, ny), kThreads, 0, s>>>(
            in, outPtrs_dev, y0, tiles, listPtrsDev.data(), listLen.data(), f, lease.epoch, spinCap(),
            poisoned.data(), deviceErrorWord());
      } else {
        k_sparseCompress<FT, false><<<dim3(tiles, ny), kThreads, 0, s>>>(
            in, outPtrs_dev, y0, tiles, listPtrsDev.data(), listLen.data(), f, lease.epoch, spinCap(),
            poisoned.data(), deviceErrorWord());
      }
      HIP_LAUNCH_CHECK();
    }
  }
  // (the compacted lists are 16 B-aligned slices of one arena allocation)
  floatCompressDescs(res, config, nb, BatchDesc::pointers(listPtrsDev.data(), listLen.data()),
                     maxN, denseOut, outSize_dev, s, nullptr, true);
  if (outSize_dev) {
    k_sparseAddSizes<<<divUp(nb, 128), 128, 0, s>>>(in, nb, poisoned.data(), outSize_dev);
    HIP_LAUNCH_CHECK();
  }
}

template <int FT>
FloatDecompressStatus sparseDecompressT(StackDeviceMemory& res,
                                        const FloatDecompressConfig& config, uint32_t nb,
                                        const BatchDesc& in, const BatchDesc& out,
                                        uint32_t maxCap, uint8_t* outSuccess_dev,
                                        uint32_t* outSize_dev, hipStream_t s, bool outAligned16) {
  const uint32_t tiles = std::max(1u, divUp(maxCap, kTileWords));
  auto densePtrs = res.alloc<uint64_t>(s, nb);
  auto sizes = res.alloc<uint32_t>(s, nb);
  auto denseOk = res.alloc<uint8_t>(s, nb);
  auto list = res.alloc<uint8_t>(s, size_t(nb) * (roundUp(maxCap, 16) + 16) * sizeof(WordOf<FT>));
  std::vector<uint64_t> listPtrs(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    listPtrs[i] = reinterpret_cast<uint64_t>(list.data()) +
                  uint64_t(i) * (roundUp(maxCap, 16) + 16) * sizeof(WordOf<FT>);
  }
  auto listPtrsDev = res.alloc<uint64_t>(s, nb);
  StackDeviceMemory::copyToDevice(listPtrsDev.data(), listPtrs.data(), nb * 8, s);
  {
    prof::Scope p("sparse", s);
    k_sparseHeaders<<<divUp(nb, 128), 128, 0, s>>>(in, nb, densePtrs.data(), sizes.data());
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
  SyncLease lease(res, s, size_t(nb) * tiles * 8);
  auto* f = reinterpret_cast<uint64_t*>(lease.base);
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    prof::Scope p("sparse", s);
    if (outAligned16) {
      k_sparseExpand<FT, true><<<dim3(tiles, ny), kThreads, 0, s>>>(
          in, out, y0, tiles, sizes.data(), listPtrsDev.data(), denseOk.data(), outSuccess_dev, outSize_dev, f,
          lease.epoch, spinCap(), deviceErrorWord());
    } else {
      k_sparseExpand<FT, false><<<dim3(tiles, ny), kThreads, 0, s>>>(
          in, out, y0, tiles, sizes.data(), listPtrsDev.data(), denseOk.data(), outSuccess_dev, outSize_dev, f,
          lease.epoch, spinCap(), deviceErrorWord());
    }
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
  bool aligned = true;
  for (uint32_t i = 0; i < numInBatch; ++i) aligned = aligned && ip[i] % 16 == 0;
  switch (ft) {
    case 1: sparseCompressT<1>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream, aligned); break;
    case 2: sparseCompressT<2>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream, aligned); break;
    case 3: sparseCompressT<3>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream, aligned); break;
    default: sparseCompressT<4>(res, config, numInBatch, inD, maxN, opD, denseOut, outSize_dev, stream, aligned); break;
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
  bool aligned = true;
  for (uint32_t i = 0; i < numInBatch; ++i) aligned = aligned && ptrs[numInBatch + i] % 16 == 0;
  switch (ft) {
    case 1: return sparseDecompressT<1>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream, aligned);
    case 2: return sparseDecompressT<2>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream, aligned);
    case 3: return sparseDecompressT<3>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream, aligned);
    default: return sparseDecompressT<4>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream, aligned);
  }
}

}  // namespace dietgpu
