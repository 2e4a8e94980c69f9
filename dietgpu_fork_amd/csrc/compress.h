// Single-pass compression for single-segment formats (bytes, fp16, bf16,
// fp32): one launch reads every input byte exactly once from HBM.
//
//   k_compress<FT, kCk>   histogramBatch + normalizeProbabilitiesFromHistogram
//                         + ansEncodeBatch + ansEncodeCoalesceBatch
//                         (ans/GpuANSStatistics.cuh:21-430,
//                         ans/GpuANSEncode.cuh:49-668) and, for floats, the
//                         split / size bookkeeping of floatCompressDevice
//                         (float/GpuFloatCompress.cuh:423-874)
//
// The reference (and k_hist -> k_normalize -> k_encode here) reads the input
// twice: once for the histogram, once to encode.  Here the workgroups of one
// element form a team.  Phase 1: each workgroup streams its 8 blocks once,
// writes the float raw bytes to the archive, keeps the ANS symbols in
// registers (lane l of a block holds symbols l, l+32, ... : exactly the ones
// it encodes) and counts them in LDS.  Team barrier: the partial histograms
// are published; once all have arrived every workgroup sums them and
// normalises.  Phase 2: every workgroup builds the encode table and
// encodes from registers; emitted words stay in 1024-word LDS rings (only
// dense blocks spill to a scratch slot), then the decoupled look-back of
// k_encode places them in the archive.
//
// Cross-workgroup hand-offs follow MI355X_MICROARCH.md's sc1 protocol (row 1
// of its hand-off table): payloads are stored with agent-scope relaxed
// (sc1) stores, every storing wave waits vmcnt(0), a workgroup barrier, then
// one lane signals (agent-scope atomic add / sc1 flag store); the consumer
// polls with sc1 loads, passes a workgroup barrier, and reads the payload
// with sc1 loads only.
//
// Forward progress: a workgroup waits only for workgroups of its own team
// (the team barrier) or for lower blockIdx.x of its team (look-back).  Teams
// are contiguous in dispatch order, so with in-order dispatch a team always
// completes once each XCD can hold ceil(team / 8) of its workgroups; the host
// takes this path only when a team fits in half the resident slots
// (compressSinglePassFits), and every wait has a spin cap.
#pragma once

#include "encode.h"
#include "sync_arena.h"

namespace dietgpu {

namespace cmp {
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kBlocksPerWG = 2 * kWaves;           // one block pair per wave
constexpr uint32_t kSteps = kBlockSize / kLanesPerBlock;  // 128 steps per block
constexpr uint32_t kSegSteps = 16;
constexpr uint32_t kSegWords = kSegSteps * kLanesPerBlock;  // 512 symbols
constexpr uint32_t kSegs = kSteps / kSegSteps;               // 8
constexpr uint32_t kRing = 1024;  // u16 words per block ring (a typical block's whole output)
constexpr uint32_t kSpill = 768;  // pending words that trigger a 256-word spill to the slot
constexpr uint32_t kSpinCap = 1u << 24;
// Largest team (workgroups per element, i.e. up to 1 MiB of symbols): larger
// teams wait longer at the barrier than a second read of the input costs, so
// the host sends them down the three-kernel path.
constexpr uint32_t kMaxTeam = 32;
// phase-1 histogram: u32 counters, 16 columns (lane & 15) per bin, bin rows
// padded to 17 dwords so lanes l and l + 16 (one column) rarely share a bank
constexpr uint32_t kHistCols = 16;
constexpr uint32_t kHistStride = kHistCols + 1;
constexpr uint32_t kHistWords = 256 * kHistStride;
constexpr uint32_t kPoolWords = kHistWords > kBlocksPerWG * kRing / 2 ? kHistWords : kBlocksPerWG * kRing / 2;
}  // namespace cmp

struct CompScratch {
  uint32_t* part;     // [nb][nW][256] partial histograms (sc1)
  uint32_t* partCk;   // [nb][nW] partial byte checksums (FT 0 with checksum)
  uint32_t* arrive;   // [nb][nW] team arrival flags = epoch (sync arena)
  uint64_t* flags;    // [nb][nW] look-back flags {status:2, epoch:30, value:32} (sync arena)
  uint8_t* slots;     // [nb][MB][kSlotDataBytes] spill space for dense blocks
  const uint32_t* ckIn;  // float checksum per element (k_checksum) or null
  uint32_t* outSize;
  uint32_t nW;        // workgroups per element row of the grid
  uint32_t MB;        // max blocks per element
  int pb;
  uint32_t epoch;     // this call's epoch (SyncLease)
  // Cross-generation prefetch: while it encodes, a workgroup pulls the input
  // of the workgroup `prefetchDist` linear ids ahead (the one that will take
  // over a slot about when this one exits) into the caches.  0: off.
  uint32_t prefetchDist;
  // Staggered start: odd element rows below staggerRows (the first
  // generation) wait staggerTicks (100 MHz) before phase 1.  0: off.
  uint32_t staggerTicks;
  uint32_t staggerRows;
  bool useChecksum;
};

__device__ __forceinline__ uint32_t ldSc1(gp<const uint32_t> p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stSc1(gp<uint32_t> p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back over the element's earlier workgroups (lookBack in
// encode.h) with epoch-tagged flags: bits 63:62 status (1 aggregate, 2
// inclusive prefix), 61:32 epoch, 31:0 value; a flag of another epoch reads
// as "not yet published".  Called by one whole wave; returns the sum of the
// values of workgroups [0, x).
__device__ __forceinline__ uint32_t lookBackEpoch(gp<uint64_t> f, uint32_t x, uint32_t agg,
                                                  uint32_t epoch) {
  const uint32_t lane = laneId();
  const uint64_t tag = uint64_t(epoch) << 32;
  if (lane == 0)
    __hip_atomic_store(f + x, (x == 0 ? kFlagPrefix : kFlagAgg) | tag | agg, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (x == 0) return 0;
  uint32_t excl = 0;
  int32_t j = int32_t(x);
  for (uint32_t spins = 0; spins < cmp::kSpinCap;) {
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
    if (firstPre < 64) break;
    j -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(f + x, kFlagPrefix | tag | uint64_t(excl + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// grid (nW, batch), 256 threads.  Workgroup x of element b owns blocks
// [8x, 8x + 8); wave w codes blocks 8x + 2w (lanes 0-31) and 8x + 2w + 1
// (lanes 32-63).  Pointer tables may ride in the first (InlineTable) argument (BatchDesc::field).  5 waves per SIMD (96 VGPRs, 32 of them the symbols; 27 KB
// of LDS per workgroup).
#if DG_EXP == 90 || DG_EXP == 91
#define DG_CMP_WPE 4  // experiment: 4 waves / SIMD (c2: exactly 4 generations)
#else
#define DG_CMP_WPE 5
#endif
template <int FT, bool kCk>
__global__ __launch_bounds__(cmp::kThreads) __attribute__((amdgpu_waves_per_eu(DG_CMP_WPE, 8))) void k_compress(const InlineTable, BatchDesc in,
                                                            BatchDesc out, uint32_t batchOffset,
                                                            CompScratch sc) {
  using WordT = typename FloatTraits<FT>::WordT;
  static_assert(FloatTraits<FT>::kSegs == 1, "single-segment formats only");
  constexpr uint32_t kWPV = 16 / sizeof(WordT);                       // words per 16 B vector
  constexpr int V = int(cmp::kSegWords * sizeof(WordT) / (32 * 16));  // vectors / lane / segment
  constexpr int kRegs = int(cmp::kSteps / 4);                         // symbol registers

  // hist (phase 1: bin-major u32 counters, cmp::kHistCols columns) and the
  // output rings (phase 2) share `pool`
  __shared__ __attribute__((aligned(16))) uint32_t pool[cmp::kPoolWords];
  __shared__ __attribute__((aligned(16))) uint32_t tblS[kNumSymbols * 4];
  __shared__ __attribute__((aligned(16))) uint8_t symT[cmp::kBlocksPerWG][cmp::kSegWords];
  __shared__ uint32_t trashS[cmp::kWaves][64];
  __shared__ uint32_t keys[kNumSymbols];
  __shared__ uint32_t red[cmp::kWaves];
  __shared__ uint32_t cwE[cmp::kBlocksPerWG], flE[cmp::kBlocksPerWG], preE[cmp::kBlocksPerWG];

  const uint32_t b = batchOffset + blockIdx.y;
  const uint32_t x = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const uint32_t n = in.size(b);
  const uint32_t nBlocks = divUp(n, kBlockSize);
  const uint32_t team = max(1u, divUp(nBlocks, cmp::kBlocksPerWG));
  if (x >= team) return;
  const uint32_t first = x * cmp::kBlocksPerWG;
  if (sc.staggerTicks && (blockIdx.y & 1u) && blockIdx.y < sc.staggerRows) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < sc.staggerTicks) __builtin_amdgcn_s_sleep(16);
  }

  for (uint32_t i = tid; i < cmp::kHistWords / 4; i += cmp::kThreads)
    *(lp<u32x4>)&pool[4 * i] = u32x4{0, 0, 0, 0};
  static_assert(cmp::kHistWords % 4 == 0, "16 B zeroing");
  __syncthreads();

  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, h = lane >> 5, l = lane & 31;
  DG_STAMP_RT(22);
  uint32_t uwH[2];  // wave-uniform block sizes of the pair
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const uint32_t bk = first + 2 * w + hh;
    uwH[hh] = bk < nBlocks ? min(kBlockSize, n - bk * kBlockSize) : 0u;
  }
  const uint32_t blk = first + 2 * w + h;
  const uint32_t uw = h ? uwH[1] : uwH[0];

  // ---------------- phase 1: split + symbol registers + histogram ----------
  gp<const WordT> src = (gp<const WordT>)startOf(in, b);
  gp<uint8_t> raw = FT == 0 ? gp<uint8_t>(nullptr) : startOf(out, b) + 32;
  const bool vecIn = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  lp<uint8_t> myT = (lp<uint8_t>)&symT[2 * w + h][0];
  lp<uint32_t> hcol = (lp<uint32_t>)&pool[l & (cmp::kHistCols - 1)];
  // quad byte transpose of the symbols (phase 1): lane l = 4 qm + qr
  const uint32_t qr = l & 3, qm = l >> 2;
  const uint32_t sel1 = (qr & 2) ? 0x03020706u : 0x05040100u;
  const uint32_t sel2 = (qr & 1) ? 0x03070105u : 0x06020400u;
  uint32_t symR[kRegs];
#pragma unroll
  for (int i = 0; i < kRegs; ++i) symR[i] = 0;
  uint32_t ck = 0;
  const uint32_t nSeg = divUp(max(uwH[0], uwH[1]), cmp::kSegWords);
  gp<const WordT> blkSrc = src + uint64_t(blk) * kBlockSize;

  // every segment's loads are issued D segments ahead (D = 4 for up to 2
  // vectors per lane, 2 for fp32): about two HBM latencies per workgroup, not
  // eight, within the 96 VGPRs of 5 waves per SIMD
  constexpr int D = DG_EXP == 90 ? (V <= 2 ? 8 : 4) : (V <= 2 ? 4 : 2);
  auto phase1 = [&](auto vecTag) {
    constexpr bool kVec = decltype(vecTag)::value;
    uint4 pv[D][V];
    auto load = [&](uint32_t g) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const uint32_t j0 = g * cmp::kSegWords + (k * 32 + l) * kWPV;
        if (kVec && j0 + kWPV <= uw) pv[g % D][k] = ld16(blkSrc + j0);
      }
    };
    auto split = [&](uint32_t g) {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const uint32_t off = (k * 32 + l) * kWPV;  // word offset in the segment
        const uint32_t j0 = g * cmp::kSegWords + off;
        const uint32_t i0 = blk * kBlockSize + j0;
        if (kVec && j0 + kWPV <= uw) {
          const uint4 v = pv[g % D][k];
          splitVec<FT>(v, i0, n, raw, myT + off, myT + off);
          if constexpr (kCk) ck ^= v.x ^ v.y ^ v.z ^ v.w;
        } else {
          for (uint32_t q = 0; q < kWPV && j0 + q < uw; ++q) {
            const WordT wd = blkSrc[j0 + q];
            splitOne<FT>(wd, i0 + q, n, raw, myT + off + q, myT + off + q);
            if constexpr (kCk) ck ^= uint32_t(wd);
          }
        }
      }
    };
#pragma unroll
    for (uint32_t g = 0; g < uint32_t(D); ++g)
      if (g < nSeg) load(g);
#pragma unroll
    for (uint32_t g = 0; g < cmp::kSegs; ++g) {
      if (g >= nSeg) break;
      split(g);
      DG_STAMP_RT(6 + g);
      if (g + D < nSeg) load(g + D);
      __builtin_amdgcn_wave_barrier();
      if (DG_EXP == 51) continue;  // counting experiment: no symbols / histogram
      // Transpose: lane l = 4m + r reads the dwords of rows 4q + r (q < 4),
      // columns 4m..4m+3, and a 4 x 4 byte transpose inside its quad (two
      // DPP exchanges + v_perm) leaves it column l, steps 4q..4q+3, packed
      // as phase 2 wants: 4 ds_read_b32 instead of 16 ds_read_u8.
      uint32_t W[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q)
        W[q] = *(lp<const uint32_t>)(myT + (4 * q + qr) * 32 + 4 * qm);
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        // (mov_dpp, not update_dpp: no zeroed `old` register per exchange)
        uint32_t p2 = uint32_t(__builtin_amdgcn_mov_dpp(int(W[q]), 0x4E, 0xF, 0xF, true));
        W[q] = __builtin_amdgcn_perm(p2, W[q], sel1);  // 16-bit halves with lane r ^ 2
        uint32_t p1 = uint32_t(__builtin_amdgcn_mov_dpp(int(W[q]), 0xB1, 0xF, 0xF, true));
        W[q] = __builtin_amdgcn_perm(p1, W[q], sel2);  // bytes with lane r ^ 1
        // opaque: otherwise phase 2's byte extractions would be folded back
        // into 128 unpacked symbol registers
        asm volatile("" : "+v"(W[q]));
        symR[g * 4 + q] = W[q];
      }
      // count: +1 at row sym (bfe + mad_u24 address, constant increment);
      // segments full for both blocks of the wave skip the per-symbol bounds
      // select (a wave-uniform branch)
      auto count = [&](auto maskTag) {
        constexpr bool kMasked = decltype(maskTag)::value;
#pragma unroll
        for (uint32_t t = 0; t < cmp::kSegSteps; ++t) {
          const uint32_t sym = __builtin_amdgcn_ubfe(W[t / 4], 8 * (t & 3), 8);
          uint32_t add = 1u;
          if (kMasked) add = g * cmp::kSegWords + t * 32 + l < uw ? 1u : 0u;
          __hip_atomic_fetch_add(hcol + __umul24(sym, cmp::kHistStride), add, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      };
      if ((g + 1) * cmp::kSegWords <= min(uwH[0], uwH[1]))
        count(std::false_type{});
      else
        count(std::true_type{});
      __builtin_amdgcn_wave_barrier();
    }
  };
  if (DG_EXP == 92) __builtin_amdgcn_s_setprio(1);
  if (vecIn)
    phase1(std::true_type{});
  else
    phase1(std::false_type{});
  if (DG_EXP == 92) __builtin_amdgcn_s_setprio(0);
  DG_STAMP_RT(1);
  __syncthreads();

  // partial histogram of this workgroup: bin tid, sum of its columns (the
  // padded rows make the 32 lanes' reads of one column conflict free)
  {
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < cmp::kHistCols; ++k) cnt += pool[tid * cmp::kHistStride + k];
    stSc1(G(sc.part) + (uint64_t(b) * sc.nW + x) * kNumSymbols + tid, cnt);
    if constexpr (kCk) {
      ck = (ck ^ (ck >> 8) ^ (ck >> 16) ^ (ck >> 24)) & 0xffu;
      ck = waveXor(ck);
      if (lane == 0) red[w] = ck;
      __syncthreads();
      if (tid == 0) stSc1(G(sc.partCk) + uint64_t(b) * sc.nW + x, red[0] ^ red[1] ^ red[2] ^ red[3]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // Arrival: one sc1 flag store (= this call's epoch) after every wave's
  // partial-histogram stores have completed.  Wave 0 then polls the team's
  // flags (lane j: member j); every workgroup sums the team's partials itself
  // (one hop; the host keeps teams small, kMaxTeam).
  gp<uint32_t> arrive = G(sc.arrive) + uint64_t(b) * sc.nW;
  if (tid == 0) stSc1(arrive + x, sc.epoch);
  DG_STAMP_RT(2);
  if (w == 0) {
    for (uint32_t spins = 0; spins < cmp::kSpinCap; ++spins) {
      const bool in = lane >= team || ldSc1(arrive + lane) == sc.epoch;
      if (ballot(!in) == 0) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  uint32_t q, ckE = 0;
  {
    gp<const uint32_t> hp = G(sc.part) + uint64_t(b) * sc.nW * kNumSymbols + tid;
    uint32_t acc[cmp::kMaxTeam];
#pragma unroll
    for (uint32_t k = 0; k < cmp::kMaxTeam; ++k)
      acc[k] = k < team ? ldSc1(hp + uint64_t(k) * kNumSymbols) : 0u;
    uint32_t count = 0;
#pragma unroll
    for (uint32_t k = 0; k < cmp::kMaxTeam; ++k) count += acc[k];
    q = n == 0 ? 0u : normalizeCount(count, n, sc.pb, keys, red);
    if constexpr (kCk) {
      uint32_t c = tid < team ? ldSc1(G(sc.partCk) + uint64_t(b) * sc.nW + tid) : 0u;
      c = waveXor(c);
      __syncthreads();
      if (lane == 0) red[w] = c;
      __syncthreads();
      ckE = red[0] ^ red[1] ^ red[2] ^ red[3];
    }
  }
  {
    const uint32_t cdf = blockExclusiveScan<cmp::kThreads>(q, red, nullptr);
    const uint4 e = encTableEntry(q, cdf, sc.pb);
    *(lp<u32x4>)&tblS[4 * tid] = u32x4{e.x, e.y, e.z, e.w};
  }
  __syncthreads();  // table visible; the histogram is dead, `pool` becomes the rings
  DG_STAMP_RT(3);

  // Prefetch for the next generation (CompScratch::prefetchDist): LDS-DMA
  // loads of that workgroup's input into this wave's dead transpose buffer
  // (never read; drained by the vmcnt(0) after phase 2), so its phase 1
  // reads from the caches and HBM streams while this workgroup encodes.
  if (sc.prefetchDist) {
    const uint32_t lin = blockIdx.y * gridDim.x + x + sc.prefetchDist;
    const uint32_t y2 = lin / gridDim.x, x2 = lin - (lin / gridDim.x) * gridDim.x;
    if (y2 < gridDim.y) {
      const uint32_t b2 = batchOffset + y2;
      const uint32_t n2 = in.size(b2);
      const uint32_t w0 = x2 * cmp::kBlocksPerWG * kBlockSize;
      gp<const uint8_t> s2 = (gp<const uint8_t>)((gp<const WordT>)startOf(in, b2) + w0);
      if (w0 < n2 && (reinterpret_cast<uintptr_t>(s2) & 15) == 0) {
        const uint32_t bytes = min(n2 - w0, cmp::kBlocksPerWG * kBlockSize) * uint32_t(sizeof(WordT));
        for (uint32_t off = 16 * tid; off + 16 <= bytes; off += 16 * cmp::kThreads)
          __builtin_amdgcn_global_load_lds((gp<void>)(s2 + off), (lp<void>)&symT[2 * w][0], 16, 0, 0);
      }
    }
  }

  // ---------------- phase 2: rANS encode from registers ---------------------
  gp<uint8_t> base = startOf(out, b);
  gp<uint8_t> o = base + (FT == 0 ? 0u : 32u + floatRawBytes(FT, n));  // ANS archive
  gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
  gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * nBlocks);
  lp<uint16_t> rings = (lp<uint16_t>)&pool[0];
  if (first + 2 * w < nBlocks) {
    uint32_t hv = h ? ~0u : 0u;
    asm volatile("" : "+v"(hv));  // keep `hv & x` a v_and
    const uint32_t trashAddr = uint32_t(size_t((lp<uint32_t>)&trashS[w][lane]));
    EStream p;
    p.x = kStartState;
    p.ring = rings + 2 * w * cmp::kRing;
    p.ringLane = p.ring + (hv & cmp::kRing);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint32_t bk = min(first + 2 * w + hh, nBlocks - 1);
      p.nout[hh] = 0;
      p.flushed[hh] = 0;
      p.out[hh] = (gp<uint16_t>)(G(sc.slots) + (uint64_t(b) * sc.MB + bk) * kSlotDataBytes);
    }
    lp<const u32x4> tbl = (lp<const u32x4>)&tblS[0];
    auto encode = [&](auto fullTag) {
      constexpr bool kFull = decltype(fullTag)::value;
#pragma unroll
      for (uint32_t t0 = 0; t0 < cmp::kSteps; t0 += enc::kUnroll) {
        ringFlush<int(cmp::kSpill), cmp::kRing>(p, lane);
        u32x4 E[enc::kUnroll];
#pragma unroll
        for (uint32_t u = 0; u < enc::kUnroll; ++u) {
          const uint32_t t = t0 + u;
          E[u] = tbl[(symR[t / 4] >> (8 * (t & 3))) & 0xffu];
        }
#pragma unroll
        for (uint32_t u = 0; u < enc::kUnroll; ++u) {
          const uint32_t t = t0 + u;
          encStep<!kFull, cmp::kRing>(p, kFull || t * 32 + l < uw, E[u], hv, trashAddr);
        }
        // keep the scheduler from hoisting later groups' table reads (the
        // rings and the table are distinct arrays): registers, not latency,
        // bound this loop
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (DG_EXP == 93) __builtin_amdgcn_s_setprio(1);
    if (DG_EXP == 50) {  // counting experiment: no encode
    } else if (uwH[0] == kBlockSize && uwH[1] == kBlockSize)
      encode(std::true_type{});
    else
      encode(std::false_type{});
    if (uw) {
      ((gp<uint32_t>)(states + uint64_t(kStateBytesPerBlock) * blk))[l] = p.x;
      if (l == 0) {
        cwE[2 * w + h] = uint32_t(h ? p.nout[1] : p.nout[0]);
        flE[2 * w + h] = uint32_t(h ? p.flushed[1] : p.flushed[0]);
      }
    }
  }
  if (DG_EXP == 93) __builtin_amdgcn_s_setprio(0);
  DG_STAMP_RT(4);
  // spilled words are read back by other waves of this workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---------------- placement: decoupled look-back + copy-out --------------
  const uint32_t nk = first < nBlocks ? min(cmp::kBlocksPerWG, nBlocks - first) : 0u;
  if (w == 0) {
    const uint32_t r = lane < nk ? roundUp(cwE[lane], 8) : 0u;
    const uint32_t inc = waveInclusiveScan(r);
    const uint32_t agg = readfirst(__shfl(inc, 63));
    const uint32_t excl = lookBackEpoch(G(sc.flags) + uint64_t(b) * sc.nW, x, agg, sc.epoch);
    if (lane < nk) preE[lane] = excl + inc - r;
    if (lane == 0 && x == team - 1) {
      const EncTail t{nullptr, nullptr, sc.outSize, nullptr, 0, sc.pb, sc.useChecksum};
      writeHeadTotal<FT>(base, o, n, nBlocks, excl + agg, bwords, t, b);
    }
  }
  if (x == 0) {
    // header fields known before encoding, the pdf table, raw-section tails
    if (tid == 0) {
      const bool ansCk = FT == 0 && sc.useChecksum;
      const uint32_t ckv = FT == 0 ? ckE : (sc.ckIn ? G(sc.ckIn)[b] : 0u);
      gp<uint32_t> hdr = (gp<uint32_t>)o;
      hdr[0] = kANSMagicVersion;
      hdr[1] = nBlocks;
      hdr[2] = n;
      hdr[4] = uint32_t(sc.pb) | (ansCk ? 0x10u : 0u);
      hdr[5] = ansCk ? ckv : 0u;
      hdr[6] = 0;
      hdr[7] = 0;
      if constexpr (FT != 0) {
        gp<uint32_t> fh = (gp<uint32_t>)base;
        fh[0] = kFloatMagicVersion;
        fh[1] = n;
        fh[2] = uint32_t(FT) | (sc.useChecksum ? 0x10u : 0u);
        fh[3] = sc.useChecksum ? ckv : 0u;
        fh[5] = 0;
        fh[6] = 0;
        fh[7] = 0;
      }
    }
    ((gp<uint16_t>)(o + kANSHeaderBytes))[tid] = uint16_t(q);
    if constexpr (FT != 0) {
      if (tid < 16) {
        if constexpr (FT == 1 || FT == 2) {
          if (n + tid < roundUp(n, 16)) raw[n + tid] = 0;
        } else {
          if (n + tid < roundUp(n, 8)) ((gp<uint16_t>)raw)[n + tid] = 0;
          if (n + tid < roundUp(n, 16)) raw[2 * roundUp(n, 8) + n + tid] = 0;
        }
      }
    }
  }
  __syncthreads();
  DG_STAMP_RT(5);
  if (tid < nk) {
    const uint32_t k = first + tid;
    const uint32_t uwk = min(kBlockSize, n - k * kBlockSize);
    st8(bwords + k, make_uint2((uwk << 16) | cwE[tid], preE[tid]));
  }
  if (nk == 0) return;
  // payload: 16 B vectors over the workgroup's contiguous archive range; the
  // source is the block's ring, or its slot for words spilled before the end
  gp<uint4> dst = (gp<uint4>)((gp<uint8_t>)(bwords + roundUp(nBlocks, 2)) + 2ull * preE[0]);
  const uint32_t nv = (preE[nk - 1] + roundUp(cwE[nk - 1], 8) - preE[0]) / 8;
  for (uint32_t v = tid; v < nv; v += cmp::kThreads) {
    const uint32_t wd = preE[0] + 8 * v;
    uint32_t k = 0;
#pragma unroll
    for (uint32_t s = 1; s < cmp::kBlocksPerWG; ++s) k += (s < nk && preE[s] <= wd) ? 1u : 0u;
    const uint32_t off = wd - preE[k];
    uint4 val;
    if (off < flE[k]) {
      val = ld16((gp<const uint4>)(G(sc.slots) + (uint64_t(b) * sc.MB + first + k) * kSlotDataBytes + 2ull * off));
    } else {
      const u32x4 r = *(lp<const u32x4>)(rings + k * cmp::kRing + (off & (cmp::kRing - 1)));
      val = make_uint4(r.x, r.y, r.z, r.w);
    }
    const uint32_t valid = cwE[k] > off ? cwE[k] - off : 0u;
    if (valid < 8) {
      uint32_t* vw = reinterpret_cast<uint32_t*>(&val);
#pragma unroll
      for (uint32_t r = 0; r < 4; ++r)
        if (2 * r + 1 >= valid) vw[r] &= (2 * r < valid) ? 0xffffu : 0u;
    }
    st16(dst + v, val);
  }
  DG_STAMP_RT(21);
}

}  // namespace dietgpu
