// Persistent, software-pipelined single-pass compression for single-segment
// formats (bytes, fp16, bf16, fp32): one launch reads every input byte once.
//
//   k_pcompress<FT, kCk>  histogramBatch + normalizeProbabilitiesFromHistogram
//                         + ansEncodeBatch + batchExclusivePrefixSum +
//                         ansEncodeCoalesceBatch (ans/GpuANSStatistics.cuh:
//                         21-430, ans/GpuANSEncode.cuh:49-845,
//                         ans/BatchPrefixSum.cuh) and, for floats, splitFloat
//                         + the size bookkeeping of floatCompressDevice
//                         (float/GpuFloatCompress.cuh:423-874)
//
// Work items.  An item is 8 consecutive 4 KiB blocks of one element (one
// block pair per wave); the items of an element form its team.  The grid is
// at most one generation of resident workgroups, a whole number of teams, and
// the items are dealt out in rounds of one grid: workgroup w takes item
// r * grid + j(w) in round r.  j(w) keeps each team on one XCD (workgroups
// w, w + 8, ... share one under the observed round-robin placement), so the
// team's hand-offs stay in one L2 (speed only, never correctness).  No
// atomics hand out work: a shared work-queue counter serialises at ~90
// dequeues per microsecond, 11 us per round of 1024 workgroups.
//
// Pipeline.  A workgroup holds two items: E, whose table is known and which it
// encodes, and L (its next round's item), which it loads.  Per iteration,
// segment by segment (512 symbols per block), it encodes 16 steps of E from
// registers and then splits the same segment of L (16 B loads issued two
// segments ahead, raw float bytes straight to the archive, ANS symbols
// transposed into the registers E's segment just freed, counted in an LDS
// histogram), so the HBM stream of L overlaps the VALU-bound encode of E
// inside every wave.  Then it publishes L's partial histogram, places E
// (decoupled look-back, headers, payload copy from the LDS rings), waits at
// L's team barrier and normalises L (every member sums the team's partials
// itself: one hop).

// Cross-workgroup hand-offs follow MI355X_MICROARCH.md's sc1 protocol (row 1
// of its hand-off table): payloads are stored with agent-scope relaxed (sc1)
// stores, every storing wave waits vmcnt(0), a workgroup barrier, then one
// lane signals; consumers poll with sc1 loads and read the payload with sc1
// loads only.
//
// Forward progress.  Waits are on the team barrier of L (all members loaded)
// and on the look-back of E (lower members placed).  A team's items all
// belong to one round, and a workgroup reaches round r's barrier only after
// publishing every earlier round's item, so (by induction over rounds) every
// wait ends once the grid is resident: the host launches at most the
// occupancy-reported number of workgroups.  Each wait is bounded by a poll
// cap (a kernel argument); a wait that runs out POISONS the element instead
// of guessing: the poison bit rides in the look-back flag to the element's
// last member, which writes outSize = 0 and counts the element in the device
// error word.
#pragma once

#include <utility>

#include "encode.h"
#include "lookback.h"
#include "sync_arena.h"

namespace dietgpu {

namespace pc {
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kBlocksPerItem = 2 * kWaves;           // one block pair per wave
constexpr uint32_t kSteps = kBlockSize / kLanesPerBlock;  // 128 steps per block
constexpr uint32_t kSegSteps = 16;
constexpr uint32_t kSegWords = kSegSteps * kLanesPerBlock;  // 512 symbols
constexpr uint32_t kSegs = kSteps / kSegSteps;               // 8
constexpr uint32_t kRing = 1024;  // u16 words per block ring (a typical block's whole output)
// pending words that trigger a 256-word spill to the slot: checked every
// enc::kUnroll steps (<= 128 new words per block), so a block holds at most
// kSpill + 127 < kRing unflushed words; most blocks never spill
constexpr uint32_t kSpill = kRing - 128;
// Largest team summed by every member (a 1 MiB-symbol element): its partials
// are one sc1 load per member and bin.
constexpr uint32_t kMaxTeam = 32;
// histogram: u32 counters, 8 columns (lane & 7) per bin, rows padded to 9
constexpr uint32_t kHistCols = 8;
constexpr uint32_t kHistStride = kHistCols + 1;
constexpr uint32_t kHistWords = 256 * kHistStride;
}  // namespace pc

struct PCompArgs {
  uint32_t* part;        // [items][256] partial histograms (sc1)
  uint32_t* partCk;      // [items] partial byte checksums (FT 0 with checksum)
  uint32_t* arrive;      // [items] team arrival flags = epoch (sync arena)
  uint64_t* flags;       // [items] look-back flags (sync arena)
  uint32_t* err;         // device error word (elements poisoned)
  uint8_t* slots;        // [grid][8][kSlotDataBytes] spill space of each workgroup
  const uint32_t* teamStart;  // [nb + 1] first item of each element, or null: uniform teams
  const uint32_t* ckIn;  // float checksum per element (k_checksum) or null
  uint32_t* outSize;
  uint32_t items;        // total items
  uint32_t team;         // items per element when uniform
  uint32_t nb;
  uint32_t grid;         // workgroups = items per round (a whole number of teams)
  uint32_t xcdTeams;     // 1: team members share w % 8 (teams per round % 8 == 0)
  uint32_t epoch;
  uint32_t spinCap;      // polls per wait before poisoning
  int pb;
  bool useChecksum;
};

// One item: element b, member x of a team of `team` items starting at item tb.
struct PItem {
  uint32_t i;  // item index, or >= items: none
  uint32_t b, x, team, tb, n, nBlocks;
};

__device__ __forceinline__ PItem itemOf(uint32_t i, const PCompArgs& a, const BatchDesc& in) {
  PItem it;
  it.i = i;
  it.b = it.x = it.team = it.tb = it.n = it.nBlocks = 0;
  if (i >= a.items) return it;
  if (a.teamStart == nullptr) {
    it.b = i / a.team;
    it.team = a.team;
    it.tb = it.b * a.team;
  } else {  // largest b with teamStart[b] <= i (scalar loads)
    uint32_t lo = 0, hi = a.nb;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (BatchDesc::tableAt(a.teamStart, mid) <= i) lo = mid; else hi = mid;
    }
    it.b = lo;
    it.tb = BatchDesc::tableAt(a.teamStart, lo);
    it.team = BatchDesc::tableAt(a.teamStart, lo + 1) - it.tb;
  }
  it.x = i - it.tb;
  it.n = in.size(it.b);
  it.nBlocks = divUp(it.n, kBlockSize);
  return it;
}

// Kernel-argument layout of k_pcompress (explicit arguments in order, each at
// its natural alignment).  The kernel re-reads its arguments from the kernarg
// segment where it needs them, through a pointer the compiler cannot see
// through: otherwise it keeps both descriptors and the argument block (~50
// SGPRs) live across the pipelined loop and spills SGPRs to scratch inside
// the encode steps, where every reload's vmcnt wait drains the prefetched
// input loads.
constexpr size_t kArgIn = sizeof(InlineTable);
constexpr size_t kArgOut = (kArgIn + sizeof(BatchDesc) + alignof(BatchDesc) - 1) / alignof(BatchDesc) * alignof(BatchDesc);
constexpr size_t kArgA = (kArgOut + sizeof(BatchDesc) + alignof(PCompArgs) - 1) / alignof(PCompArgs) * alignof(PCompArgs);

// f(std::integral_constant<uint32_t, I>{}) for I = 0 .. N-1, expanded at
// compile time (the segment loop's body is too large for #pragma unroll,
// and a loop index left dynamic would put the symbol registers in scratch)
template <typename F, uint32_t... I>
__device__ __forceinline__ void staticForImpl(F&& f, std::integer_sequence<uint32_t, I...>) {
  (f(std::integral_constant<uint32_t, I>{}), ...);
}
template <uint32_t N, typename F>
__device__ __forceinline__ void staticFor(F&& f) {
  staticForImpl(f, std::make_integer_sequence<uint32_t, N>{});
}

template <typename T>
__device__ __forceinline__ T kernArg(size_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  const DG_CONST uint8_t* k = (const DG_CONST uint8_t*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(k));  // opaque: a fresh scalar load at every use
  return *(const DG_CONST T*)(k + off);
#else
  (void)off;
  return T();
#endif
}

// Grid: one generation of resident workgroups (1-D), 256 threads.  Pointer
// tables may ride in the first (InlineTable) argument (BatchDesc::inl).  4
// waves per SIMD (<= 128 VGPRs, ~36 KB of LDS per workgroup).
template <int FT, bool kCk>
__global__ __launch_bounds__(pc::kThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_pcompress(
    const InlineTable, BatchDesc, BatchDesc, PCompArgs) {
  auto IN = [] { return kernArg<BatchDesc>(kArgIn); };
  auto OUT = [] { return kernArg<BatchDesc>(kArgOut); };
  auto A = [] { return kernArg<PCompArgs>(kArgA); };
  using WordT = typename FloatTraits<FT>::WordT;
  static_assert(FloatTraits<FT>::kSegs == 1, "single-segment formats only");
  constexpr uint32_t kWPV = 16 / sizeof(WordT);                      // words per 16 B vector
  constexpr int V = int(pc::kSegWords * sizeof(WordT) / (32 * 16));  // vectors / lane / segment
  constexpr int kRegs = int(pc::kSteps / 4);                         // symbol registers
  // segments of loads in flight ahead of the split: two (the 16 encode steps
  // of each segment in between cover an HBM latency; four spill the 128-VGPR
  // budget of 4 waves per SIMD)
  constexpr int D = 2;

  __shared__ __attribute__((aligned(16))) uint32_t hist[pc::kHistWords];
  __shared__ __attribute__((aligned(16))) uint16_t rings[pc::kBlocksPerItem * pc::kRing];
  __shared__ __attribute__((aligned(16))) uint32_t tblS[kNumSymbols * 4];
  __shared__ __attribute__((aligned(16))) uint8_t symT[pc::kBlocksPerItem][pc::kSegWords];
  __shared__ uint32_t trashS[pc::kWaves][64];
  __shared__ uint32_t keys[kNumSymbols];
  __shared__ uint16_t pdfS[kNumSymbols];
  __shared__ uint32_t red[pc::kWaves];
  __shared__ uint32_t cwE[pc::kBlocksPerItem], flE[pc::kBlocksPerItem], preE[pc::kBlocksPerItem];
  __shared__ uint32_t stateS;

  const uint32_t tid = threadIdx.x;
  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, h = lane >> 5, l = lane & 31;
  uint32_t hv = h ? ~0u : 0u;
  asm volatile("" : "+v"(hv));  // keep `hv & x` a v_and
  const uint32_t trashAddr = uint32_t(size_t((lp<uint32_t>)&trashS[w][lane]));
  lp<uint8_t> myT = (lp<uint8_t>)&symT[2 * w + h][0];
  lp<uint32_t> hcol = (lp<uint32_t>)&hist[l & (pc::kHistCols - 1)];
  // quad byte transpose of the symbols (phase 1): lane l = 4 qm + qr
  const uint32_t qr = l & 3, qm = l >> 2;
  const uint32_t sel1 = (qr & 2) ? 0x03020706u : 0x05040100u;
  const uint32_t sel2 = (qr & 1) ? 0x03070105u : 0x06020400u;
  lp<const u32x4> tbl = (lp<const u32x4>)&tblS[0];
  gp<uint8_t> slotBase = G(A().slots) + uint64_t(blockIdx.x) * pc::kBlocksPerItem * kSlotDataBytes;

  for (uint32_t i = tid; i < pc::kHistWords / 4; i += pc::kThreads)
    *(lp<u32x4>)&hist[4 * i] = u32x4{0, 0, 0, 0};
  static_assert(pc::kHistWords % 4 == 0, "16 B zeroing");
  static_assert(pc::kSpill + 32 * enc::kUnroll <= pc::kRing, "ring overflow between spill checks");

  // ---- per-item state (wave-uniform; E: encoding, L: loading) ----
  uint32_t symR[kRegs];
#pragma unroll
  for (int i = 0; i < kRegs; ++i) symR[i] = 0;
  uint4 pv[D][V];
  static_assert(sizeof(WordT) <= 4, "single-segment formats have words of at most 4 bytes");
  uint32_t ck = 0;

  // this workgroup's item of round r (>= items: none)
  auto itemAt = [&](uint32_t r) __attribute__((always_inline)) -> uint32_t {
    const PCompArgs ka = A();
    uint32_t j = blockIdx.x;
    if (ka.xcdTeams) {  // w = xcd + 8 (group * team + x), team slot = group * 8 + xcd
      const uint32_t xcd = blockIdx.x & 7u, q = blockIdx.x >> 3;
      const uint32_t grp = q / ka.team, x = q - grp * ka.team;
      j = (grp * 8 + xcd) * ka.team + x;
    }
    const uint64_t i = uint64_t(r) * ka.grid + j;
    return i < ka.items ? uint32_t(i) : ka.items;
  };
  auto pairSize = [&](const PItem& it, int hh) __attribute__((always_inline)) -> uint32_t {
    const uint32_t bk = it.x * pc::kBlocksPerItem + 2 * w + hh;
    return bk < it.nBlocks ? min(kBlockSize, it.n - bk * kBlockSize) : 0u;
  };
  auto srcOf = [&](const PItem& it) __attribute__((always_inline)) -> gp<const WordT> {
    return (gp<const WordT>)startOf(IN(), it.b) +
           uint64_t(it.x * pc::kBlocksPerItem + 2 * w + h) * kBlockSize;
  };

  // 16 B streaming loads of segment g of this lane's block (the input is read
  // once; non-temporal, so the caches keep the archives for the decoder:
  // c2 step 267 -> 239 us together with the decoder's streaming stores,
  // same-box A/B), issued unconditionally (an
  // item's load schedule is then branch-free, so the compiler's wait counts
  // stay exact instead of draining every load in flight at a branch merge):
  // a vector with no word of the block reads the element's first vector
  // instead.  16 B-aligned input only (the host sends anything else down the
  // three-kernel path): a vector holding the last valid word is then a whole
  // 16 B chunk of the same page.
  auto load = [&](gp<const WordT> elem, gp<const WordT> src, uint32_t uw, uint32_t g)
                  __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const uint32_t j0 = g * pc::kSegWords + (k * 32 + l) * kWPV;
      pv[g % D][k] = ld16nt(j0 < uw ? src + j0 : elem);
    }
  };

  // ---- phase-1 pieces for segment g of item L ----
  // split: raw bytes -> archive, symbols -> myT.  kFull: both blocks of the
  // pair whole; otherwise words at or past the block's end are zeroed (their
  // raw bytes are the archive's zero padding, their symbols are never
  // counted or encoded) and vectors wholly past it store nothing.
  auto split = [&](const PItem& it, gp<uint8_t> raw, uint32_t uw, uint32_t g, auto fullTag)
                   __attribute__((always_inline)) {
    constexpr bool kFull = decltype(fullTag)::value;
    const uint32_t blk = it.x * pc::kBlocksPerItem + 2 * w + h;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const uint32_t off = (k * 32 + l) * kWPV;  // word offset in the segment
      const uint32_t j0 = g * pc::kSegWords + off;
      const uint32_t i0 = blk * kBlockSize + j0;
      uint4 v = pv[g % D][k];
      bool store = true;
      if (!kFull) {
        const uint32_t valid = j0 < uw ? min(uw - j0, kWPV) : 0u;  // words
        constexpr uint32_t kWPD = 4 / sizeof(WordT);                // words per dword
        uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
          const uint32_t cnt = valid > d * kWPD ? min(valid - d * kWPD, kWPD) : 0u;
          vw[d] &= cnt >= kWPD ? ~0u : (1u << (cnt * 8 * sizeof(WordT))) - 1u;
        }
        store = valid != 0;
      }
      splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, store);
      if constexpr (kCk) ck ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  };
  // transpose: lane l = 4m + r reads the dwords of rows 4q + r (q < 4),
  // columns 4m..4m+3; a 4 x 4 byte transpose inside its quad (two DPP
  // exchanges + v_perm) leaves it column l, steps 4q..4q+3, packed for the
  // encoder: 4 ds_read_b32 instead of 16 ds_read_u8.  Then count.
  auto transposeCount = [&](uint32_t g, uint32_t uw, bool masked) __attribute__((always_inline)) {
    uint32_t W[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) W[q] = *(lp<const uint32_t>)(myT + (4 * q + qr) * 32 + 4 * qm);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      uint32_t p2 = uint32_t(__builtin_amdgcn_mov_dpp(int(W[q]), 0x4E, 0xF, 0xF, true));
      W[q] = __builtin_amdgcn_perm(p2, W[q], sel1);  // 16-bit halves with lane r ^ 2
      uint32_t p1 = uint32_t(__builtin_amdgcn_mov_dpp(int(W[q]), 0xB1, 0xF, 0xF, true));
      W[q] = __builtin_amdgcn_perm(p1, W[q], sel2);  // bytes with lane r ^ 1
      // opaque: otherwise the encoder's byte extractions would be folded
      // back into 128 unpacked symbol registers
      asm volatile("" : "+v"(W[q]));
      symR[g * 4 + q] = W[q];
    }
    if (!masked) {
#pragma unroll
      for (uint32_t t = 0; t < pc::kSegSteps; ++t) {
        const uint32_t sym = __builtin_amdgcn_ubfe(W[t / 4], 8 * (t & 3), 8);
        __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
#pragma unroll
      for (uint32_t t = 0; t < pc::kSegSteps; ++t) {
        const uint32_t sym = __builtin_amdgcn_ubfe(W[t / 4], 8 * (t & 3), 8);
        const uint32_t add = g * pc::kSegWords + t * 32 + l < uw ? 1u : 0u;
        __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), add, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  };
  // ---- encode pieces for item E ----
  EStream p;
  auto encInit = [&]() __attribute__((always_inline)) {
    p.x = kStartState;
    p.ring = (lp<uint16_t>)&rings[2 * w * pc::kRing];
    p.ringLane = p.ring + (hv & pc::kRing);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      p.nout[hh] = 0;
      p.flushed[hh] = 0;
      p.out[hh] = (gp<uint16_t>)(slotBase + (2 * w + hh) * kSlotDataBytes);
    }
  };
  auto encSegFull = [&](uint32_t g) __attribute__((always_inline)) {
#pragma unroll
    for (uint32_t t0 = g * pc::kSegSteps; t0 < (g + 1) * pc::kSegSteps; t0 += enc::kUnroll) {
      ringFlush<int(pc::kSpill), pc::kRing>(p, lane);
      u32x4 Ev[enc::kUnroll];
#pragma unroll
      for (uint32_t u = 0; u < enc::kUnroll; ++u) {
        const uint32_t t = t0 + u;
        Ev[u] = tbl[(symR[t / 4] >> (8 * (t & 3))) & 0xffu];
      }
#pragma unroll
      for (uint32_t u = 0; u < enc::kUnroll; ++u) encStep<false, pc::kRing>(p, true, Ev[u], hv, trashAddr);
      // keep the scheduler from hoisting later groups' table reads over the
      // ring stores (registers, not latency, bound this loop)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto encSegMasked = [&](uint32_t g, uint32_t uw) __attribute__((always_inline)) {
#pragma unroll
    for (uint32_t t0 = g * pc::kSegSteps; t0 < (g + 1) * pc::kSegSteps; t0 += enc::kUnroll) {
      ringFlush<int(pc::kSpill), pc::kRing>(p, lane);
      u32x4 Ev[enc::kUnroll];
#pragma unroll
      for (uint32_t u = 0; u < enc::kUnroll; ++u) {
        const uint32_t t = t0 + u;
        Ev[u] = tbl[(symR[t / 4] >> (8 * (t & 3))) & 0xffu];
      }
#pragma unroll
      for (uint32_t u = 0; u < enc::kUnroll; ++u) {
        const uint32_t t = t0 + u;
        encStep<true, pc::kRing>(p, t * 32 + l < uw, Ev[u], hv, trashAddr);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- publish L's partial histogram, arrive ----
  // (after a workgroup barrier: every wave's counts are in)
  auto publish = [&](const PItem& it) __attribute__((always_inline)) {
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < pc::kHistCols; ++k) {
      cnt += hist[tid * pc::kHistStride + k];
      hist[tid * pc::kHistStride + k] = 0;
    }
    stSc1(G(A().part) + uint64_t(it.i) * kNumSymbols + tid, cnt);
    if constexpr (kCk) {
      uint32_t c = (ck ^ (ck >> 8) ^ (ck >> 16) ^ (ck >> 24)) & 0xffu;
      c = waveXor(c);
      if (lane == 0) red[w] = c;
      __syncthreads();
      if (tid == 0) stSc1(G(A().partCk) + it.i, red[0] ^ red[1] ^ red[2] ^ red[3]);
      ck = 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) stSc1(G(A().arrive) + it.i, A().epoch);
  };

  // ---- team barrier + normalisation of L: table in tblS, pdf in pdfS ----
  // Returns (uniform) whether the wait ran out of polls; ckOut: the element's
  // byte checksum (kCk).
  auto barrierNormalize = [&](const PItem& it, uint32_t& ckOut) __attribute__((always_inline)) -> bool {
    if (w == 0) {
      bool ok = it.team == 1;  // a team of one waits for nobody
      for (uint32_t spins = 0; !ok && spins < A().spinCap; ++spins) {
        const bool inT = lane >= it.team || ldSc1(G(A().arrive) + it.tb + lane) == A().epoch;
        if (ballot(!inT) == 0) {
          ok = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) stateS = ok ? 0u : 1u;
    }
    __syncthreads();
    const bool timedOut = readfirst(stateS) != 0;
    gp<const uint32_t> hp = G(A().part) + uint64_t(it.tb) * kNumSymbols + tid;
    // (16 loads in flight at a time: L's symbols hold 32 VGPRs meanwhile)
    uint32_t count = 0;
    for (uint32_t k0 = 0; k0 < it.team; k0 += 16) {
      uint32_t acc[16];
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k)
        acc[k] = k0 + k < it.team ? ldSc1(hp + uint64_t(k0 + k) * kNumSymbols) : 0u;
#pragma unroll
      for (uint32_t k = 0; k < 16; ++k) count += acc[k];
    }
    const uint32_t q = it.n == 0 ? 0u : normalizeCount(count, it.n, A().pb, keys, red);
    if constexpr (kCk) {
      uint32_t c = tid < it.team ? ldSc1(G(A().partCk) + it.tb + tid) : 0u;
      c = waveXor(c);
      __syncthreads();
      if (lane == 0) red[w] = c;
      __syncthreads();
      ckOut = red[0] ^ red[1] ^ red[2] ^ red[3];
    }
    const uint32_t cdf = blockExclusiveScan<pc::kThreads>(q, red, nullptr);
    const uint4 e = encTableEntryReg(q, cdf, A().pb);
    *(lp<u32x4>)&tblS[4 * tid] = u32x4{e.x, e.y, e.z, e.w};
    pdfS[tid] = uint16_t(q);
    __syncthreads();
    return timedOut;
  };

  // ---- E's aggregate (its words, rounded to 8 per block) -> its look-back flag ----
  auto publishAgg = [&](const PItem& it, bool poison) __attribute__((always_inline)) {
    const uint32_t first = it.x * pc::kBlocksPerItem;
    const uint32_t nk = first < it.nBlocks ? min(pc::kBlocksPerItem, it.nBlocks - first) : 0u;
    const uint32_t r = lane < nk ? roundUp(cwE[lane], 8) : 0u;
    const uint32_t agg = readfirst(__shfl(waveInclusiveScan(r), 63));
    if (lane == 0)
      __hip_atomic_store(G(A().flags) + it.tb + it.x,
                         (it.x == 0 ? kFlagPrefix : kFlagAgg) | (poison ? kFlagPoison : 0ull) |
                             (uint64_t(A().epoch) << 32) | agg,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // ---- placement of E: look-back, headers, payload copy-out ----
  auto place = [&](const PItem& it, bool poison, uint32_t ckE) __attribute__((always_inline)) {
    // spilled words are read back by other waves of this workgroup: a wave
    // that spilled waits for its stores (the others need not drain the
    // raw-section stores of the split)
    if (p.flushed[0] | p.flushed[1]) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t first = it.x * pc::kBlocksPerItem;
    const uint32_t nk = first < it.nBlocks ? min(pc::kBlocksPerItem, it.nBlocks - first) : 0u;
    gp<uint8_t> base = startOf(OUT(), it.b);
    gp<uint8_t> o = base + (FT == 0 ? 0u : 32u + floatRawBytes(FT, it.n));  // ANS archive
    gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
    gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * it.nBlocks);
    if (w == 0) {
      const uint32_t r = lane < nk ? roundUp(cwE[lane], 8) : 0u;
      const uint32_t inc = waveInclusiveScan(r);
      const uint32_t agg = readfirst(__shfl(inc, 63));
      bool pz = poison;
      const uint32_t excl = lookBackPoison(G(A().flags) + it.tb, it.x, agg, A().epoch, A().spinCap, pz, false);
      if (lane < nk) preE[lane] = excl + inc - r;
      if (lane == 0 && it.x == it.team - 1) {
        if (pz) {
          if (A().outSize) G(A().outSize)[it.b] = 0u;
          __hip_atomic_fetch_add(G(A().err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          const EncTail t{nullptr, nullptr, A().outSize, nullptr, 0, A().pb, A().useChecksum};
          writeHeadTotal<FT>(base, o, it.n, it.nBlocks, excl + agg, bwords, t, it.b);
        }
      }
    }
    if (it.x == 0) {
      // header fields known before encoding, the pdf table, raw-section tails
      if (tid == 0) {
        const bool ansCk = FT == 0 && A().useChecksum;
        const uint32_t ckv = FT == 0 ? ckE : (A().ckIn ? G(A().ckIn)[it.b] : 0u);
        gp<uint32_t> hdr = (gp<uint32_t>)o;
        hdr[0] = kANSMagicVersion;
        hdr[1] = it.nBlocks;
        hdr[2] = it.n;
        hdr[4] = uint32_t(A().pb) | (ansCk ? 0x10u : 0u);
        hdr[5] = ansCk ? ckv : 0u;
        hdr[6] = 0;
        hdr[7] = 0;
        if constexpr (FT != 0) {
          gp<uint32_t> fh = (gp<uint32_t>)base;
          fh[0] = kFloatMagicVersion;
          fh[1] = it.n;
          fh[2] = uint32_t(FT) | (A().useChecksum ? 0x10u : 0u);
          fh[3] = A().useChecksum ? ckv : 0u;
          fh[5] = 0;
          fh[6] = 0;
          fh[7] = 0;
        }
      }
      ((gp<uint16_t>)(o + kANSHeaderBytes))[tid] = pdfS[tid];
      if constexpr (FT != 0) {
        gp<uint8_t> raw = base + 32;
        const uint32_t n = it.n;
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
    if (tid < nk) {
      const uint32_t k = first + tid;
      const uint32_t uwk = min(kBlockSize, it.n - k * kBlockSize);
      st8(bwords + k, make_uint2((uwk << 16) | cwE[tid], preE[tid]));
    }
    if (nk == 0) return;
    // payload: 16 B vectors over the item's contiguous archive range; the
    // source is the block's ring, or its slot for words spilled before the end
    gp<uint4> dst = (gp<uint4>)((gp<uint8_t>)(bwords + roundUp(it.nBlocks, 2)) + 2ull * preE[0]);
    const uint32_t nv = (preE[nk - 1] + roundUp(cwE[nk - 1], 8) - preE[0]) / 8;
    for (uint32_t v = tid; v < nv; v += pc::kThreads) {
      const uint32_t wd = preE[0] + 8 * v;
      uint32_t k = 0;
#pragma unroll
      for (uint32_t s = 1; s < pc::kBlocksPerItem; ++s) k += (s < nk && preE[s] <= wd) ? 1u : 0u;
      const uint32_t off = wd - preE[k];
      uint4 val;
      if (off < flE[k]) {
        val = ld16((gp<const uint4>)(slotBase + k * kSlotDataBytes + 2ull * off));
      } else {
        const u32x4 r = *(lp<const u32x4>)(rings + k * pc::kRing + (off & (pc::kRing - 1)));
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
  };

  // ---- encode E's pair (and store its states / word counts) ----
  auto encodeDone = [&](const PItem& it) __attribute__((always_inline)) {
    const uint32_t uw = h ? pairSize(it, 1) : pairSize(it, 0);
    if (uw) {
      gp<uint8_t> o = startOf(OUT(), it.b) + (FT == 0 ? 0u : 32u + floatRawBytes(FT, it.n));
      gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
      const uint32_t blk = it.x * pc::kBlocksPerItem + 2 * w + h;
      ((gp<uint32_t>)(states + uint64_t(kStateBytesPerBlock) * blk))[l] = p.x;
    }
    if (l == 0) {
      cwE[2 * w + h] = uw ? uint32_t(h ? p.nout[1] : p.nout[0]) : 0u;
      flE[2 * w + h] = uw ? uint32_t(h ? p.flushed[1] : p.flushed[0]) : 0u;
    }
  };

  // ================= the pipeline =================
  // Only item indices live across iterations; everything else is recomputed
  // (scalar work) where it is needed.
  __syncthreads();  // histogram zeroed
  uint32_t iE = A().items, iL = itemAt(0), round = 0;
  if (iL >= A().items) return;
  uint32_t ckE = 0;
  bool poisonE = false;
  while (true) {
    const bool hasE = iE < A().items, hasL = iL < A().items;
    if (!hasE && !hasL) break;
    __builtin_amdgcn_s_setprio(0);
    {
      const PItem E = itemOf(iE, A(), IN()), L = itemOf(iL, A(), IN());
      const uint32_t uwE0 = pairSize(E, 0), uwE1 = pairSize(E, 1);
      const uint32_t uwL0 = pairSize(L, 0), uwL1 = pairSize(L, 1);
      // encode: the full-step variant when both blocks of the pair are whole
      // (uwE0 >= uwE1); a poisoned item encodes nothing (uw 0: every step masked)
      const bool encOn = hasE && uwE0 != 0 && !poisonE;
      const bool fastE = uwE1 == kBlockSize;
      const uint32_t uwEnc = h ? uwE1 : uwE0;
      // split: the unmasked variant when both blocks of the pair are whole
      const bool loadOn = hasL && uwL0 != 0;
      const bool fullL = uwL1 == kBlockSize;
      const uint32_t uwL = h ? uwL1 : uwL0;
      const gp<const WordT> elemL = (gp<const WordT>)startOf(IN(), L.b);
      const gp<const WordT> srcL = srcOf(L);
      gp<uint8_t> rawL = FT == 0 ? gp<uint8_t>(nullptr) : startOf(OUT(), L.b) + 32;
      if (hasE) encInit();
      auto encSeg = [&](uint32_t g) __attribute__((always_inline)) {
        if (encOn) {
          if (fastE) encSegFull(g);
          else encSegMasked(g, uwEnc);
        }
      };
      if (loadOn) {
        // segment by segment: encode 16 steps of E, then split the same
        // segment of L into the symbol registers those steps freed; loads
        // run D segments ahead of the split
#pragma unroll
        for (uint32_t g = 0; g < uint32_t(D); ++g) load(elemL, srcL, uwL, g);
        staticFor<pc::kSegs>([&](auto gTag) __attribute__((always_inline)) {
          constexpr uint32_t g = decltype(gTag)::value;
          encSeg(g);
          if (fullL) split(L, rawL, uwL, g, std::true_type{});
          else split(L, rawL, uwL, g, std::false_type{});
          if (g + D < pc::kSegs) load(elemL, srcL, uwL, g + D);
          __builtin_amdgcn_wave_barrier();
          transposeCount(g, uwL, (g + 1) * pc::kSegWords > uwL1);
          __builtin_amdgcn_wave_barrier();
        });
      } else {
        staticFor<pc::kSegs>([&](auto gTag) __attribute__((always_inline)) {
          encSeg(decltype(gTag)::value);
        });
      }
      if (hasE) encodeDone(E);
    }
    // The hand-offs below are on the team's critical path while the other
    // workgroups of this CU stream: they issue at raised priority (3 % of
    // the c2 launch, same-box A/B).
    __builtin_amdgcn_s_setprio(2);
    // E's word counts and L's histogram counts are in; E's aggregate goes out
    // at once, so that the team's look-backs in place() rarely wait
    __syncthreads();
    if (hasE && w == 0) publishAgg(itemOf(iE, A(), IN()), poisonE);
    if (hasL) publish(itemOf(iL, A(), IN()));
    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);
    uint32_t iN = A().items;
    if (hasL) {
      poisonE = barrierNormalize(itemOf(iL, A(), IN()), ckE);
      iN = itemAt(++round);
    }
    iE = iL;
    iL = iN;
  }
}

}  // namespace dietgpu
