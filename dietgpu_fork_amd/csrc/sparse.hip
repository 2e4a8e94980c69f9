// Sparse float codec: nonzero bitmap + per-element exclusive scan +
// compaction, wrapped around the dense float codec.
//
// Reference: float/GpuSparseFloatCompress.{cu,cuh},
// float/GpuSparseFloatDecompress.{cu,cuh}.  The reference scans with one
// thrust::exclusive_scan per batch element on the legacy default stream
// between two cudaDeviceSynchronize calls (GpuSparseFloatCompress.cuh:360-369);
// here both directions are reduce-then-scan over 4096-word tiles, fully
// stream-ordered (no host or device-wide sync): compression reads the input
// ONCE (k_sparseCount: bitmap, tile counts, nonzeros compacted within the
// tile into a staging area; k_sparseGather: each tile sums its element's
// earlier tile counts and moves its staged nonzeros to their list
// positions); decompression counts the bitmap per 1024-word chunk and scans
// the counts within each workgroup of 256 chunks (k_sparseChunks), then
// expands one chunk per wave, adding the element's earlier workgroups' totals
// (k_sparseExpand).  (A decoupled look-back across
// the tiles of one element measured slower: with thousands of tiles its
// chain dominates.)
//
// Wire format: 16 B header {u32 N, 12 B zero}, bitmap
// ceil(N/8) bytes (bit 7 of byte k <-> element 8k) padded to 16, then a dense
// float archive of the compacted list.  The compacted list reproduces the
// reference's n-2 quirk (fill_comp_input :162-184): when x[N-2] == 0 one extra
// slot (written as 0 here, uninitialised in the reference) precedes x[N-1].
#include <algorithm>
#include <cstring>
#include <optional>
#include <vector>

#include "codec_internal.h"
#include "common.h"
#include "dietgpu/GpuFloatCodec.h"
#include "decode.h"
#include "encode.h"
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

// Load tile `tile` of an element (words past n read as 0) into LDS: 16 B
// vectors when the element is 16 B aligned (coalesced), else words.
template <typename W, bool kVec>
__device__ __forceinline__ void loadTile(gp<const W> x, uint32_t t0, uint32_t tileN, W* buf) {
  const uint32_t tid = threadIdx.x;
  if (kVec) {
    constexpr uint32_t kWPV = 16 / sizeof(W);
    constexpr uint32_t kVecs = kTileWords * sizeof(W) / 16 / kThreads;
#pragma unroll
    for (uint32_t v = 0; v < kVecs; ++v) {
      const uint32_t wi = (v * kThreads + tid) * kWPV;  // first word of the vector
      uint4 val = make_uint4(0, 0, 0, 0);
      if (wi + kWPV <= tileN) {
        val = ld16nt((gp<const uint4>)(x + t0 + wi));  // read once: stream it
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
}

// One tile of k_sparseCount (t0 < n).
template <int FT, bool kVec, bool kHist, typename W, typename HS>
__device__ __forceinline__ void sparseCountTile(const BatchDesc& in, gp<uint8_t> o, uint32_t b, uint32_t n,
                                                uint32_t tile, uint32_t numInBatch, uint32_t tilesPerElem,
                                                uint32_t* __restrict__ tileCounts, W* __restrict__ staging,
                                                uint32_t* __restrict__ histRows, uint32_t* __restrict__ zeroNext,
                                                uint32_t nRows, W* buf, HS& hs, uint32_t* waveCnt) {
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  constexpr uint32_t kSteps = kTileWords / kWaves / 64;
  constexpr uint32_t kCols = 4;  // LDS counter columns per bin (lane & 3)
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t t0 = tile * kTileWords;
  if constexpr (kHist) {
    for (int sg = 0; sg < kSegs; ++sg)
      for (uint32_t i = tid; i < kNumSymbols * kCols / 4; i += kThreads)
        *(lp<u32x4>)&hs[sg][4 * i] = u32x4{0, 0, 0, 0};
  }
  gp<const W> x = (gp<const W>)in.start(b);
  // bitwise: -0.0 is "nonzero" (generate_bitmap :56); loaded with the tile
  const W xn2 = n >= 2 ? x[n - 2] : W(1);
  loadTile<W, kVec>(x, t0, min(kTileWords, n - t0), buf);
  __syncthreads();
  const uint32_t bmBytes = (n + 7) / 8, bmPad = roundUp(bmBytes, 16);
  const bool gap = xn2 == W(0);
  // (the step ballots are taken again in the compaction below: sixteen
  // 64-bit masks held across the barrier cost registers, i.e. occupancy)
  uint32_t cnt = 0;
  uint64_t bmLane = 0;  // lane j < kSteps: the bitmap word of step j
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t q = w * (kTileWords / kWaves) + 64 * j;  // step's first word in the tile
    const uint64_t mj = ballot(buf[q + lane] != W(0));
    cnt += uint32_t(__popcll(mj));
    bmLane = lane == j ? maskToBitmap(mj) : bmLane;
    const uint32_t i0 = t0 + q;
    if (gap && i0 <= n - 1 && n - 1 < i0 + 64) cnt += 1;  // the extra slot
  }
  {
    // the wave's kSteps bitmap words in one store; then zero the 16-byte
    // padding after the element's last bitmap word
    const uint32_t i0 = t0 + w * (kTileWords / kWaves) + 64 * lane;
    gp<uint64_t> dst = (gp<uint64_t>)(o + 16 + i0 / 8);
    if (lane < kSteps && i0 < n) {
      dst[0] = bmLane;
      if (i0 + 64 >= n && i0 / 8 + 8 < bmPad) dst[1] = 0;
    }
  }
  if (lane == 0) waveCnt[w] = cnt;
  __syncthreads();
  uint32_t pos = 0;
  for (uint32_t k = 0; k < w; ++k) pos += waveCnt[k];
  if (tid == 0) tileCounts[uint64_t(b) * tilesPerElem + tile] = waveCnt[0] + waveCnt[1] + waveCnt[2] + waveCnt[3];
  W* st = staging + (uint64_t(b) * tilesPerElem + tile) * (kTileWords + 1);
#pragma unroll
  for (uint32_t j = 0; j < kSteps; ++j) {
    const uint32_t q = w * (kTileWords / kWaves) + 64 * j;
    const uint32_t i = t0 + q + lane;
    const W v = buf[q + lane];
    const uint64_t mj = ballot(v != W(0));
    const uint32_t dst = pos + mbcnt(mj);
    if (i + 1 == n && gap) {
      st[dst] = W(0);
      if (v != W(0)) st[dst + 1] = v;
    } else if (v != W(0)) {
      st[dst] = v;
    }
    if constexpr (kHist) {
      auto count = [&](W y) {
#pragma unroll
        for (int sg = 0; sg < kSegs; ++sg)
          atomicAdd(&hs[sg][compOf<FT>(y, sg) * kCols + (lane & (kCols - 1))], 1u);
      };
      if (i + 1 == n && gap) count(W(0));
      if (v != W(0)) count(v);
    }
    pos += uint32_t(__popcll(mj)) + ((gap && t0 + q <= n - 1 && n - 1 < t0 + q + 64) ? 1u : 0u);
  }
  if constexpr (kHist) {
    __syncthreads();
    for (int sg = 0; sg < kSegs; ++sg) {
      uint32_t sum = 0;
#pragma unroll
      for (uint32_t k = 0; k < kCols; ++k) sum += hs[sg][tid * kCols + ((k + tid) & (kCols - 1))];
      // few adds per address: the tiles of an element spread over nRows rows
      const uint64_t row = (uint64_t(sg) * numInBatch + b) * nRows + tile % nRows;
      if (sum)
        __hip_atomic_fetch_add(G(histRows) + row * kNumSymbols + tid, sum, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      // the same row of the arena's other buffer, zeroed for the next call
      if (tile < nRows) G(zeroNext)[row * kNumSymbols + tid] = 0;
    }
  }
}

// s1: bitmap + tile count + tile-local compaction.  grid (tiles, batch); a
// workgroup takes one 4096-word tile of one element into LDS, then each wave
// takes 1024 consecutive words as 16 steps of 64 lanes: the ballot of nonzero
// flags is the step's 64 bitmap bits (generate_bitmap :40-71) and its
// nonzeros' ranks (v_mbcnt).  The nonzeros go, in order, to the tile's slice
// of a staging area; the n-2 quirk (fill_comp_input :162-184) is one extra
// staged slot: when x[n-2] == 0, a 0 precedes x[n-1]'s slot.  (A persistent
// grid streaming several tiles per workgroup measured slower: its live state
// halves the occupancy, and a wave's wait for its next tile's loads also
// drains its stores.)
//
// kHist: the staged words are also counted into the dense codec's symbol
// histogram(s) (the compacted list's symbols, the n-2 slot included) and
// added into row tile % nRows of [segments][nb][nRows][256] (PartialHist),
// so the dense codec skips its histogram pass over the list.  The rows are
// the stream's sync-arena row buffer (SyncLease::rows, zero on entry); the
// first nRows tiles zero the same rows of the other buffer for the next call
// (`zeroNext`), so no zeroing launch precedes this one (1 x 15M fp32: a
// 4.7 us k_zero of 64 KB before).  (Normalising in the element's last-arriving tile instead of the
// dense codec's k_normalize launch made every tile pay a store drain and a
// counter round trip: c4 1 x 15M fp32 compress 70 -> 95 us.)
// (at most 80 SGPRs: 86-94 admit 7 workgroups per CU instead of 8,
// MI355X_MICROARCH.md, Residency)
template <int FT, bool kVec, bool kHist>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_num_sgpr(80))) void k_sparseCount(BatchDesc in, BatchDesc outD,
                                                          uint32_t batchOffset, uint32_t numInBatch,
                                                          uint32_t tilesPerElem,
                                                          uint32_t* __restrict__ tileCounts,
                                                          WordOf<FT>* __restrict__ staging,
                                                          uint32_t* __restrict__ histRows,
                                                          uint32_t* __restrict__ zeroNext, uint32_t nRows) {
  using W = WordOf<FT>;
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  constexpr uint32_t kCols = 4;  // LDS counter columns per bin (lane & 3)
  __shared__ __attribute__((aligned(16))) W buf[kTileWords];
  __shared__ __attribute__((aligned(16))) uint32_t hs[kHist ? kSegs : 1][kHist ? kNumSymbols * kCols : 4];
  __shared__ uint32_t waveCnt[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = in.size(b);
  const uint32_t tile = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  gp<uint8_t> o = startOf(outD, b);
  if (tile == 0 && tid == 0) st16(o, make_uint4(n, 0, 0, 0));
  const uint32_t t0 = tile * kTileWords;
  if (t0 >= n) {
    if (tid == 0) tileCounts[uint64_t(b) * tilesPerElem + tile] = 0;
  } else {
    sparseCountTile<FT, kVec, kHist>(in, o, b, n, tile, numInBatch, tilesPerElem, tileCounts, staging, histRows,
                                     zeroNext, nRows, buf, hs, waveCnt);
  }
}

// Sum of counts[0, k) by the whole workgroup: 16 loads in flight per thread
// (4,096 counts per memory round trip; an element of 16 M words has 4,096
// tiles).  Every workgroup of an element sums its own prefix of the tile
// counts, which stay in L2 (a 15 M-word element: 14.6 KB of counts, 27 MB of
// L2 reads over its 3,662 workgroups), instead of a separate scan launch
// (each launch of this chain costs ~5 us, however little it does).
__device__ __forceinline__ uint32_t tilePrefix(gp<const uint32_t> counts, uint32_t k, uint32_t* red) {
  constexpr uint32_t kR = 16;
  uint32_t sum = 0;
  for (uint32_t base = 0; base < k; base += kR * kThreads) {
    uint32_t v[kR];
#pragma unroll
    for (uint32_t j = 0; j < kR; ++j) {
      const uint32_t i = base + j * kThreads + threadIdx.x;
      v[j] = i < k ? counts[i] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kR; ++j) sum += v[j];
  }
  return blockSum<kThreads>(sum, red);
}

// s2: staged nonzeros -> their list positions.  grid (tiles [+ 1], batch).
// The tile's list offset is the sum of the element's earlier tile counts
// (tilePrefix); the last tile also stores the list's length.  With
// na.hist set (k_sparseCount counted the list's histogram), one extra
// workgroup per element normalises it meanwhile, into the dense codec's
// encode table and pdf: the dense codec then skips its k_normalize launch
// (c4 1 x 15M fp32 compress -6 us).
template <int FT>
__global__ __launch_bounds__(kThreads) void k_sparseGather(BatchDesc in, uint32_t batchOffset,
                                                           uint32_t numInBatch, uint32_t tilesPerElem,
                                                           const uint32_t* __restrict__ tileCounts,
                                                           uint32_t* __restrict__ listLen,
                                                           const WordOf<FT>* __restrict__ staging,
                                                           BatchDesc lists, NormArgs na) {
  using W = WordOf<FT>;
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t tile = blockIdx.x;
  if (tile == tilesPerElem) {  // (grid.x = tiles + 1 only with na.hist)
    __shared__ __attribute__((aligned(16))) uint32_t keys[kNumSymbols];
    __shared__ u32x4 red4[kThreads];
    for (int sg = 0; sg < FloatTraits<FT>::kSegs; ++sg) {
      normalizeElement(na, numInBatch, b, sg, keys, red, red4);
      __syncthreads();
    }
    return;
  }
  const uint32_t n = in.size(b);
  if (tile * kTileWords >= n) {
    // an empty element has no last tile: its (empty) list length is written here
    if (n == 0 && tile == 0 && threadIdx.x == 0) listLen[b] = 0;
    return;
  }
  const uint64_t row = uint64_t(b) * tilesPerElem + tile;
  const uint32_t cnt = tileCounts[row];
  const uint32_t off = tilePrefix(G(tileCounts) + uint64_t(b) * tilesPerElem, tile, red);
  if ((tile + 1) * kTileWords >= n && threadIdx.x == 0) listLen[b] = off + cnt;
  const W* st = staging + row * (kTileWords + 1);
  gp<W> list = (gp<W>)lists.start(b);
  // every staged word of the tile in flight at once, then the stores (a
  // load -> store loop took one memory round trip per 256 words: 5 x 15M
  // fp32 at 50 % zeros, 2,048 nonzeros a tile, 92 us for this kernel)
  constexpr uint32_t kPer = (kTileWords + 1 + kThreads - 1) / kThreads;
  W v[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kThreads;
    if (i < cnt) v[k] = st[i];
  }
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = threadIdx.x + k * kThreads;
    if (i < cnt) list[off + i] = v[k];
  }
}

// Decompression works on 1024-word chunks (16 bitmap words, one wave).
constexpr uint32_t kChunkWords = 1024;

// d1: one thread per chunk: the popcount of its 128 bitmap bytes (bits past
// N masked: the bitmap's padding is the reference's uninitialised bytes),
// then the workgroup's exclusive scan of its 256 chunk counts: chunkPre[c] =
// the count of the earlier chunks of c's workgroup, blockTot[g] = workgroup
// g's total; (chunk 0) the dense archive's address and N.  grid
// (ceil(chunks / 256), batch).  The expansion adds the earlier workgroups'
// totals itself (k_sparseExpand), so no scan launch or cross-workgroup
// hand-off follows (a separate one-workgroup-per-element scan launch: 1 x 15M
// fp32 decompress 5.8 us more).  A chunk's 128 B read may run past the padded
// bitmap into the dense archive that follows it (>= 576 B), never past the
// archive.
__global__ __launch_bounds__(kThreads) void k_sparseChunks(BatchDesc in, uint32_t batchOffset,
                                                           uint32_t chunksPerElem, uint32_t blocksPerElem,
                                                           uint64_t* __restrict__ densePtrs,
                                                           uint32_t* __restrict__ sizes,
                                                           uint32_t* __restrict__ chunkPre,
                                                           uint32_t* __restrict__ blockTot) {
  __shared__ uint32_t red[kWaves];
  const uint32_t b = batchOffset + blockIdx.y;
  gp<const uint8_t> a = (gp<const uint8_t>)in.start(b);
  const uint32_t n = ((gp<const uint32_t>)a)[0];
  const uint32_t c = blockIdx.x * kThreads + threadIdx.x;
  if (c == 0) {
    densePtrs[b] = reinterpret_cast<uint64_t>(in.start(b) + 16 + roundUp((n + 7) / 8, 16));
    sizes[b] = n;
  }
  uint32_t cnt = 0;
  const uint32_t i0 = c * kChunkWords;
  if (c < chunksPerElem && i0 < n) {
    gp<const uint64_t> bm = (gp<const uint64_t>)(a + 16) + uint64_t(c) * (kChunkWords / 64);
    uint64_t v[kChunkWords / 64];
#pragma unroll
    for (uint32_t k = 0; k < kChunkWords / 64; ++k) v[k] = i0 + 64 * k < n ? bm[k] : 0ull;
#pragma unroll
    for (uint32_t k = 0; k < kChunkWords / 64; ++k) {
      const uint32_t e = i0 + 64 * k;
      uint64_t m = v[k];
      if (e < n && n - e < 64) m = maskToBitmap(m) & ((1ull << (n - e)) - 1);  // element order, tail cut
      cnt += uint32_t(__popcll(m));
    }
  }
  uint32_t total = 0;
  const uint32_t excl = blockExclusiveScan<kThreads>(cnt, red, &total);
  if (c < chunksPerElem) chunkPre[uint64_t(b) * chunksPerElem + c] = excl;
  if (threadIdx.x == 0) blockTot[uint64_t(b) * blocksPerElem + blockIdx.x] = total;
}

// d3: expand the decoded nonzero list into the output (fill_in_nonzeros
// :95-144).  One wave per 1024-word chunk (grid (ceil(chunks / 4), batch)),
// no LDS and no barrier: lanes 0-15 load the chunk's 16 bitmap words
// beside its list offset (the scanned chunk count), then for each 64-word
// row the row's mask comes to SGPRs (readlane), each lane's list index is
// offset + v_mbcnt of the mask, and all 16 rows' list gathers are issued
// back to back (their addresses depend only on the bitmap) before the 16
// row stores.  (The tile-per-workgroup kernel it replaces summed every
// earlier tile's count per tile and staged through LDS: 5 x 15M fp32 at
// 50 % zeros 176 us, fp64 430 us.)
template <int FT>
__global__ __launch_bounds__(kThreads) void k_sparseExpand(BatchDesc in, BatchDesc out, uint32_t batchOffset,
                                                           uint32_t chunksPerElem, uint32_t blocksPerElem,
                                                           const uint32_t* __restrict__ sizes,
                                                           const uint32_t* __restrict__ chunkPre,
                                                           const uint32_t* __restrict__ blockTot, BatchDesc lists,
                                                           const uint8_t* __restrict__ denseOk,
                                                           uint8_t* __restrict__ outSuccess,
                                                           uint32_t* __restrict__ outSize) {
  using W = WordOf<FT>;
  constexpr uint32_t kRows = kChunkWords / 64;
  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t n = sizes[b];
  const bool ok = denseOk[b] != 0 && out.size(b) >= n;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (outSuccess) outSuccess[b] = ok ? 1 : 0;
    if (outSize) outSize[b] = n;  // fill_in_nonzeros :107-109
  }
  const uint32_t lane = threadIdx.x & 63, w = readfirst(threadIdx.x >> 6);
  const uint32_t c = blockIdx.x * kWaves + w;
  const uint32_t i0 = c * kChunkWords;
  if (!ok || c >= chunksPerElem || i0 >= n) return;
  gp<const uint8_t> bm = (gp<const uint8_t>)in.start(b) + 16;
  uint64_t mv = 0;
  if (lane < kRows && i0 + 64 * lane < n) {
    mv = maskToBitmap(*(gp<const uint64_t>)(bm + i0 / 8 + 8 * lane));
    const uint32_t rem = n - (i0 + 64 * lane);
    if (rem < 64) mv &= (1ull << rem) - 1;
  }
  // the chunk's list offset: its count prefix within its k_sparseChunks
  // workgroup plus the totals of the element's earlier workgroups, loaded
  // in the bitmap's round trip (one load per lane up to 64 workgroups, i.e.
  // 16 M words)
  const uint32_t g = c / kThreads;
  uint32_t part = 0;
  for (uint32_t k0 = 0; k0 < g; k0 += 64)
    part += k0 + lane < g ? G(blockTot)[uint64_t(b) * blocksPerElem + k0 + lane] : 0u;
  uint32_t base = readfirst(G(chunkPre)[uint64_t(b) * chunksPerElem + c]) + waveSum(part);
  // x[n-1] is read from idx[n-2] + 1 (fill_in_nonzeros :139-144): only the
  // chunk holding word n-1 looks
  const bool gap = n >= 2 && n - 1 - i0 < kChunkWords && ((bm[(n - 2) / 8] >> (7 - (n - 2) % 8)) & 1) == 0;
  gp<const W> list = (gp<const W>)lists.start(b);
  W v[kRows];
#pragma unroll
  for (uint32_t j = 0; j < kRows; ++j) {
    const uint64_t m = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(mv >> 32)), int(j)))) << 32) |
                       uint32_t(__builtin_amdgcn_readlane(int(uint32_t(mv)), int(j)));
    const uint32_t i = i0 + 64 * j + lane;
    uint32_t src = base + mbcnt(m);
    if (gap && i + 1 == n) src += 1;
    v[j] = (m >> lane) & 1 ? list[src] : W(0);
    base += uint32_t(__popcll(m));
  }
  gp<W> y = (gp<W>)out.start(b);
#pragma unroll
  for (uint32_t j = 0; j < kRows; ++j) {
    const uint32_t i = i0 + 64 * j + lane;
    // streaming: nothing here re-reads the output
    if (i < n) __builtin_nontemporal_store(v[j], y + i);
  }
}

// in: the sparse inputs (sizes = N); outD: the sparse archives; denseOut:
// where each dense archive starts; sparseN: a device array holding each
// element's N (the dense archive's size writer adds the sparse header and
// bitmap to outSize, EncTail::sparseN).
template <int FT>
void sparseCompressT(StackDeviceMemory& res, const FloatCompressConfig& config, uint32_t nb,
                     const BatchDesc& in, uint32_t maxN, const BatchDesc& outD,
                     const BatchDesc& denseOut, const uint32_t* sparseN, uint32_t* outSize_dev, hipStream_t s,
                     bool inAligned16) {
  const uint32_t tiles = std::max(1u, divUp(maxN, kTileWords));
  auto tileCounts = res.alloc<uint32_t>(s, size_t(nb) * tiles);
  auto listLen = res.alloc<uint32_t>(s, nb);
  // per tile: its nonzeros in order, plus the n-2 quirk's slot
  auto staging = res.alloc<WordOf<FT>>(s, size_t(nb) * tiles * (kTileWords + 1));
  // the compacted lists: 16 B-aligned rows of one arena allocation, lengths
  // on the device
  const uint64_t listStride = uint64_t(roundUp(maxN, 16) + 16) * sizeof(WordOf<FT>);
  auto list = res.alloc<uint8_t>(s, size_t(nb) * listStride);
  BatchDesc lists = BatchDesc::strided(list.data(), listStride, 0);
  lists.sizes = listLen.data();
  // the list's symbol histogram, counted here for a single element when the
  // three-kernel dense path follows (the single-pass compressor counts as it
  // loads): the dense codec then skips its histogram pass (c4 1 x 15M fp32:
  // compress 85 -> 75 us).  It lengthens every tile's workgroup, so with
  // more elements the separate k_hist over the compacted lists is faster
  // (5 x 15M: 155 us against 170).
  bool countHist = nb == 1;
  if constexpr (FT != 4) countHist = countHist && !persistentPreferred<FT>(nb, maxN);
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  // histogram rows: up to 64 per element, accumulated with atomics into this
  // stream's sync-arena row buffer (zero on entry; k_sparseCount zeroes the
  // other buffer for the next call).  The lease is released before the dense
  // codec takes its own.
  const uint32_t G = tiles;
  const uint32_t R = std::min(tiles, kReduceRows);
  const size_t rowsBytes = countHist ? size_t(kSegs) * nb * R * kNumSymbols * 4 : 0;
  std::optional<SyncLease> lease;
  if (countHist) lease.emplace(res, s, kNoSyncRegions, false, rowsBytes);
  uint32_t* const histRows = countHist ? static_cast<uint32_t*>(lease->rows[0]) : nullptr;
  uint32_t* const zeroNext = countHist ? static_cast<uint32_t*>(lease->rows[1]) : nullptr;
  auto table = res.alloc<uint4>(s, countHist ? size_t(kSegs) * nb * kNumSymbols : 1);
  auto pdf = res.alloc<uint16_t>(s, countHist ? size_t(kSegs) * nb * kNumSymbols : 1);
  NormArgs na{};
  na.in = in;
  na.hist = histRows;
  na.rows = R;
  na.pb = config.ansConfig.probBits;
  na.table = table.data();
  na.pdf = pdf.data();
  na.totalFromHist = true;  // the list length is written by this same launch
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    prof::Scope p("sparse", s);
    auto launch = [&](auto vecTag, auto histTag) {
      k_sparseCount<FT, decltype(vecTag)::value, decltype(histTag)::value><<<dim3(G, ny), kThreads, 0, s>>>(
          in, outD, y0, nb, tiles, tileCounts.data(), staging.data(), histRows, zeroNext, R);
    };
    if (inAligned16) {
      if (countHist) launch(std::true_type{}, std::true_type{});
      else launch(std::true_type{}, std::false_type{});
    } else {
      if (countHist) launch(std::false_type{}, std::true_type{});
      else launch(std::false_type{}, std::false_type{});
    }
    HIP_LAUNCH_CHECK();
    k_sparseGather<FT><<<dim3(tiles + (countHist ? 1 : 0), ny), kThreads, 0, s>>>(
        in, y0, nb, tiles, tileCounts.data(), listLen.data(), staging.data(), lists, na);
    HIP_LAUNCH_CHECK();
  }
  lease.reset();
  PartialHist pre{histRows, R};
  pre.table = table.data();
  pre.pdf = pdf.data();
  floatCompressDescs(res, config, nb, lists, maxN, denseOut, outSize_dev, s, nullptr, true,
                     countHist ? &pre : nullptr, sparseN);
}

template <int FT>
FloatDecompressStatus sparseDecompressT(StackDeviceMemory& res,
                                        const FloatDecompressConfig& config, uint32_t nb,
                                        const BatchDesc& in, const BatchDesc& out,
                                        uint32_t maxCap, uint8_t* outSuccess_dev,
                                        uint32_t* outSize_dev, hipStream_t s) {
  const uint32_t chunks = std::max(1u, divUp(maxCap, kChunkWords));
  const uint32_t cblocks = divUp(chunks, kThreads);  // k_sparseChunks workgroups per element
  auto densePtrs = res.alloc<uint64_t>(s, nb);
  auto sizes = res.alloc<uint32_t>(s, nb);
  auto denseOk = res.alloc<uint8_t>(s, nb);
  const uint64_t listStride = uint64_t(roundUp(maxCap, 16) + 16) * sizeof(WordOf<FT>);
  auto list = res.alloc<uint8_t>(s, size_t(nb) * listStride);
  const BatchDesc lists = BatchDesc::strided(list.data(), listStride, maxCap + 1);
  auto chunkPre = res.alloc<uint32_t>(s, size_t(nb) * chunks);
  auto blockTot = res.alloc<uint32_t>(s, size_t(nb) * cblocks);
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    prof::Scope p("sparse", s);
    k_sparseChunks<<<dim3(cblocks, ny), kThreads, 0, s>>>(in, y0, chunks, cblocks, densePtrs.data(), sizes.data(),
                                                          chunkPre.data(), blockTot.data());
    HIP_LAUNCH_CHECK();
  }
  // dense decode of the nonzero list (capacity: the largest output)
  auto cfg = config;
  cfg.useChecksum = false;
  floatDecompressDescs(res, cfg, nb, BatchDesc::pointers(densePtrs.data(), nullptr),
                       lists, maxCap + 1,
                       denseOk.data(), nullptr, s, nullptr, /*streamOut=*/false,  // the expansion reads it
                       /*capacityOnly=*/true);
  FloatDecompressStatus status;
  if (config.useChecksum) {
    // verify the dense archive's checksum over the bytes it was computed on
    // (the first listLen bytes of the nonzero list)
    auto denseLen = res.alloc<uint32_t>(s, nb);
    k_info<<<divUp(nb, 128), 128, 0, s>>>(BatchDesc::pointers(densePtrs.data(), nullptr), nb, true,
                                          denseLen.data(), nullptr, nullptr);
    HIP_LAUNCH_CHECK();
    status.errorInfo = verifyChecksums(res, nb, BatchDesc::pointers(densePtrs.data(), nullptr), true,
                                       [&] {
                                         BatchDesc d = lists;
                                         d.sizes = denseLen.data();
                                         return d;
                                       }(),
                                       maxCap + 1, s);
    if (!status.errorInfo.empty()) status.error = FloatDecompressError::ChecksumMismatch;
  }
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    prof::Scope p("sparse", s);
    k_sparseExpand<FT><<<dim3(divUp(chunks, kWaves), ny), kThreads, 0, s>>>(
        in, out, y0, chunks, cblocks, sizes.data(), chunkPre.data(), blockTot.data(), lists, denseOk.data(),
        outSuccess_dev, outSize_dev);
    HIP_LAUNCH_CHECK();
  }
  return status;
}

}  // namespace

uint32_t getMaxSparseFloatCompressedSize(FloatType ft, uint32_t size) {
  const uint64_t v = 16ull + roundUp64((uint64_t(size) + 7) / 8, 16) + getMaxFloatCompressedSize(ft, size);
  DG_CHECK(v <= uint64_t(UINT32_MAX), "input too large: " << size << " float words");
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
  bool aligned = true;
  for (uint32_t i = 0; i < numInBatch; ++i) aligned = aligned && ip[i] % 16 == 0;
  GpuMemoryReservation<uint8_t> tbl;
  BatchDesc inD, outD, denseOut;
  const uint32_t* sparseN;
  if (numInBatch == 1) {
    // one element (the reference's SparseFloatBenchmark shape): stride
    // descriptors, no table upload; the dense archive's size writer reads N
    // from the sparse header k_sparseCount writes first (word 0 of the archive)
    inD = BatchDesc::strided(in[0], 0, sz[0]);
    outD = BatchDesc::strided(out[0], 0, 0);
    denseOut = BatchDesc::strided(reinterpret_cast<void*>(dp[0]), 0, 0);
    sparseN = reinterpret_cast<const uint32_t*>(out[0]);
  } else {
    std::vector<uint64_t> ptrs(ip);
    ptrs.insert(ptrs.end(), op.begin(), op.end());
    ptrs.insert(ptrs.end(), dp.begin(), dp.end());
    tbl = res.alloc<uint8_t>(stream, ptrs.size() * 8 + sz.size() * 4);
    std::vector<uint8_t> host(ptrs.size() * 8 + sz.size() * 4);
    std::memcpy(host.data(), ptrs.data(), ptrs.size() * 8);
    std::memcpy(host.data() + ptrs.size() * 8, sz.data(), sz.size() * 4);
    StackDeviceMemory::copyToDevice(tbl.data(), host.data(), host.size(), stream);
    const uint64_t* ipD = reinterpret_cast<const uint64_t*>(tbl.data());
    const uint64_t* opD = ipD + numInBatch;
    const uint64_t* dpD = opD + numInBatch;
    const uint32_t* szD = reinterpret_cast<const uint32_t*>(dpD + numInBatch);
    inD = BatchDesc::pointers(ipD, szD);
    outD = BatchDesc::pointers(opD, nullptr);
    denseOut = BatchDesc::pointers(dpD, nullptr);
    sparseN = szD;
  }
  switch (ft) {
    case 1: sparseCompressT<1>(res, config, numInBatch, inD, maxN, outD, denseOut, sparseN, outSize_dev, stream, aligned); break;
    case 2: sparseCompressT<2>(res, config, numInBatch, inD, maxN, outD, denseOut, sparseN, outSize_dev, stream, aligned); break;
    case 3: sparseCompressT<3>(res, config, numInBatch, inD, maxN, outD, denseOut, sparseN, outSize_dev, stream, aligned); break;
    default: sparseCompressT<4>(res, config, numInBatch, inD, maxN, outD, denseOut, sparseN, outSize_dev, stream, aligned); break;
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
  GpuMemoryReservation<uint8_t> tbl;
  BatchDesc inD, outD;
  if (numInBatch == 1) {  // stride descriptors, no table upload
    inD = BatchDesc::strided(in[0], 0, 0);
    outD = BatchDesc::strided(out[0], 0, cap[0]);
  } else {
    tbl = res.alloc<uint8_t>(stream, ptrs.size() * 8 + cap.size() * 4);
    std::vector<uint8_t> host(ptrs.size() * 8 + cap.size() * 4);
    std::memcpy(host.data(), ptrs.data(), ptrs.size() * 8);
    std::memcpy(host.data() + ptrs.size() * 8, cap.data(), cap.size() * 4);
    StackDeviceMemory::copyToDevice(tbl.data(), host.data(), host.size(), stream);
    const uint64_t* ipD = reinterpret_cast<const uint64_t*>(tbl.data());
    const uint64_t* opD = ipD + numInBatch;
    const uint32_t* capD = reinterpret_cast<const uint32_t*>(opD + numInBatch);
    inD = BatchDesc::pointers(ipD, nullptr);
    outD = BatchDesc::pointers(opD, capD);
  }
  switch (ft) {
    case 1: return sparseDecompressT<1>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
    case 2: return sparseDecompressT<2>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
    case 3: return sparseDecompressT<3>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
    default: return sparseDecompressT<4>(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev, stream);
  }
}

}  // namespace dietgpu
