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
// at most one generation of resident workgroups, a whole number of teams of
// workgroups, and a workgroup team takes one element per round: member x of
// team T works item x of the team's element.  Team membership (kXcd) keeps
// each team on one XCD (workgroups w, w + 8, ... share one under the
// observed round-robin placement), so the team's hand-offs stay in one L2
// (speed only, never correctness), and gives the members increasing
// workgroup indices.  Elements of rounds 0 and 1 are static (r * teams + T); from
// round 2 on, member 0 takes the team's element two rounds ahead with one
// returning add on a per-call counter and logs it (epoch-tagged) for the
// other members, so teams that ran fast take more elements.  One add per
// team and round (not per workgroup: a shared counter serialises at ~90
// dequeues per microsecond), issued in one round's hand-off window and read
// a round later, off every critical path.
//
// Pipeline.  A workgroup holds two items: E, whose table is known and which it
// encodes, and L (its next round's item), which it loads.  Per iteration,
// segment by segment (512 symbols per block), it encodes 16 steps of E from
// registers and then splits the same segment of L (16 B loads issued two
// segments ahead, raw float bytes straight to the archive, ANS symbols
// transposed into the registers E's segment just freed, counted in an LDS
// histogram), so the HBM stream of L overlaps the VALU-bound encode of E
// inside every wave.  The hand-off window then publishes L's partial
// histogram and E's look-back aggregate, loads the team's partials of L while
// wave 0 runs E's look-back, and after one workgroup barrier wave 0
// normalises L (every member sums the team's partials itself: one hop) while
// waves 1-3 copy E's payload out of the LDS rings.
//
// Cross-workgroup hand-offs follow MI355X_MICROARCH.md's tagged-granule form:
// a partial histogram word is {epoch << 16 | count}, read with sc1 loads, so
// its consumer needs no arrival flag (no drain of the producer's stores, no
// barrier, one memory round trip per hop); the look-back flags carry their
// value and epoch in one 8 B word.  Where the host could lay the teams out
// XCD-aligned (kXcd: every batch whose teams per round round up to a multiple
// of 8 within the resident grid, small batches padded with idle teams) the
// partials are stored plain (sc0): the line stays in the XCD's L2, where the
// team's other members -- the same XCD under round-robin placement -- read it
// at L2 latency (an sc1 store drops the line and every read goes to the
// fabric: c2 compress 141.5 -> 138.5 us).  Other grids store them sc1
// (write-through), which a member on any XCD reads fresh.  Were a member
// ever placed elsewhere and served a stale line, the team barrier's time
// budget counts the element from the input (below) and the device's fallback
// word counts the event (dietgpu_barrier_fallback_count), so placement is
// speed only.  The flags and the log keep sc1 stores: their waits have no
// such fallback.
//
// Forward progress does not depend on the grid being co-resident.  The only
// wait on workgroups that may not have been dispatched is L's team barrier
// (its members have higher as well as lower indices); it is bounded by a time
// budget (PCompArgs::fallbackTicks), after which the workgroup counts L's
// element itself from the input (an extra read on this slow path only) and
// goes on.  Every other wait is the look-back on LOWER members of E's team
// and the log read (written by member 0), i.e. on lower workgroup indices.
// That cannot deadlock as long as each XCD dispatches its own workgroups in
// index order (observed; not a HIP contract): the lowest unfinished
// workgroup then waits on nothing unfinished, and its XCD dispatched every
// lower workgroup of its own before it, so it holds or will get a slot --
// whatever the timing across XCDs and whatever another kernel holds.
// Members numbered by a per-team start ticket instead (a wait is then only
// ever on a workgroup that has started, under any dispatch order) measured
// c2 compress +10 us, same box, in every form tried (DESIGN.md section 7,
// round 4), so the kernel keeps the index order and bounds the waits
// instead.  Another kernel holding CUs
// (a second compress on another stream, an RCCL collective) therefore delays
// the call but cannot stall it.  The look-back is still bounded by a poll cap
// (a kernel argument); a look-back that runs out POISONS the element instead
// of guessing: the poison bit rides in the look-back flag to the element's
// last member, which writes outSize = 0 and counts the element in the device
// error word (a poisoned element's output bytes are undefined).
#pragma once

#include <utility>

#include "encode.h"
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
// histogram: u32 counters, 12 columns (l % 12 of a 32-lane half) per bin,
// rows padded to 13: two or three lanes of a half share a column where 8
// columns had four, so hot bins serialise less (c2 compress 143.5 -> 141.5
// us same-box; 13.3 KB, the most that keeps four workgroups per CU)
constexpr uint32_t kHistCols = 12;
constexpr uint32_t kHistStride = kHistCols + 1;
constexpr uint32_t kHistWords = 256 * kHistStride;
}  // namespace pc

struct PCompArgs {
  uint32_t* part;        // [items][256] partial histograms, epoch << 16 | count (sync arena)
  uint32_t* partCk;      // [items] partial byte checksums, epoch << 16 | xor (FT 0 with checksum)
  uint64_t* flags;       // [items] look-back flags (sync arena)
  uint32_t* err;         // device error words: [0] elements poisoned, [1] team-barrier fallbacks
  uint8_t* slots;        // [grid][8][kSlotDataBytes] spill space of each workgroup
  const uint32_t* ckIn;  // float checksum per element (k_checksum) or null
  uint32_t* outSize;
  const uint32_t* sparseN;  // EncTail::sparseN
  uint32_t items;        // total items
  uint32_t team;         // items per element
  uint32_t nb;
  uint32_t grid;         // workgroups = items per round (a whole number of teams)
  uint64_t* ctr;         // [2] element dequeue counters, this call's at epoch & 1 (sync arena)
  uint64_t* elog;        // [teams][maxR] element of each team's round, epoch << 32 | element (sync arena)
  uint32_t maxR;         // rounds a team may take
  uint32_t slotSpan;     // workgroups per dispatch slot (the CU count): slot = blockIdx / slotSpan
  uint32_t epoch;
  uint32_t spinCap;      // polls per look-back before poisoning
  uint32_t fallbackTicks;  // team-barrier wait (100 MHz ticks) before counting the element itself
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
  it.b = i / a.team;
  it.team = a.team;
  it.tb = it.b * a.team;
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

__device__ __forceinline__ uint64_t realtime() {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_s_memrealtime();  // 100 MHz
#else
  return 0;
#endif
}

// Grid: one generation of resident workgroups (1-D), 256 threads.  Pointer
// tables may ride in the first (InlineTable) argument (BatchDesc::inl).  4
// waves per SIMD (<= 128 VGPRs, ~40 KB of LDS per workgroup).
// kXcd: the grid is a whole number of 8-team groups and member x of team
// T = 8 g + c is workgroup c + 8 (g team + x), so a team's workgroups share
// blockIdx % 8, i.e. one XCD under round-robin placement (speed only); the
// partial histograms then go out as plain stores that stay in that L2.
// Otherwise (teams per round not a multiple of 8 within the resident grid)
// a team's workgroups are consecutive and spread over the XCDs, and the
// partials are stored write-through (sc1), which every XCD reads fresh.
template <int FT, bool kCk, bool kXcd>
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
  __shared__ __attribute__((aligned(16))) uint16_t pdfS[kNumSymbols];
  __shared__ uint32_t ckS[pc::kWaves];
  __shared__ __attribute__((aligned(16))) uint32_t cwE[pc::kBlocksPerItem];
  __shared__ __attribute__((aligned(16))) uint32_t flE[pc::kBlocksPerItem];
  __shared__ __attribute__((aligned(16))) uint32_t preE[pc::kBlocksPerItem];
  __shared__ uint32_t poisonS, sigS, fbS;

  const uint32_t tid = threadIdx.x;
  // the lane's half (0: lanes 0-31, 1: lanes 32-63), recomputed at each use
  // by three VALU instructions: held live across the pipeline it spills, and
  // a reload's vmcnt wait drains the input loads in flight
  auto halfNow = []() __attribute__((always_inline)) -> uint32_t {
    uint32_t hh;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshrrev_b32 %0, 5, %0"
                 : "=v"(hh));
    return hh;
  };
  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, l = lane & 31;
  // lane / thread index recomputed at each use (the hand-off code's LDS and
  // global addresses derive from them: hoisted to the kernel entry they are
  // spilled, and each scratch reload is a memory round trip -- microseconds
  // while the other workgroups stream)
  auto laneNow = []() __attribute__((always_inline)) -> uint32_t {
    uint32_t v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
  };
  auto tidNow = [&]() __attribute__((always_inline)) -> uint32_t { return (w << 6) + laneNow(); };
  uint32_t hv = halfNow() ? ~0u : 0u;
  asm volatile("" : "+v"(hv));  // keep `hv & x` a v_and
  lp<uint32_t> hcol = (lp<uint32_t>)&hist[l % pc::kHistCols];
  // quad byte transpose of the symbols (phase 1): lane l = 4 qm + qr
  const uint32_t qr = l & 3, qm = l >> 2;
  const uint32_t sel1 = (qr & 2) ? 0x03020706u : 0x05040100u;
  const uint32_t sel2 = (qr & 1) ? 0x03070105u : 0x06020400u;
  lp<const u32x4> tbl = (lp<const u32x4>)&tblS[0];
  gp<uint8_t> slotBase = G(A().slots) + uint64_t(blockIdx.x) * pc::kBlocksPerItem * kSlotDataBytes;

  for (uint32_t i = tid; i < pc::kHistWords / 4; i += pc::kThreads)
    *(lp<u32x4>)&hist[4 * i] = u32x4{0, 0, 0, 0};
  if (tid == 0) sigS = fbS = 0;
  static_assert(pc::kHistWords % 4 == 0, "16 B zeroing");
  static_assert(pc::kSpill + 32 * enc::kUnroll <= pc::kRing, "ring overflow between spill checks");

  // ---- per-item state (wave-uniform; E: encoding, L: loading) ----
  uint32_t symR[kRegs];
#pragma unroll
  for (int i = 0; i < kRegs; ++i) symR[i] = 0;
  uint4 pv[D][V];
  static_assert(sizeof(WordT) <= 4, "single-segment formats have words of at most 4 bytes");
  uint32_t ck = 0;

  // Teams and elements.  Team T (members x = 0 .. team-1, increasing
  // workgroup indices) takes element T in round 0 and teams + T in round 1;
  // later rounds' elements come from a dequeue counter, taken by member 0 two
  // rounds ahead and logged per team (elog[T][r]), so teams that run ahead
  // take more elements (the SIMD arbiter favours the earlier-dispatched
  // workgroups of a CU: with a static deal their teams finished rounds of
  // work ahead of the last ones).
  auto teamX = [&](uint32_t& T, uint32_t& X) __attribute__((always_inline)) {
    const PCompArgs ka = A();
    if constexpr (kXcd) {  // w = xcd + 8 (group * team + x), team T = group * 8 + xcd
      const uint32_t xcd = blockIdx.x & 7u, q = blockIdx.x >> 3;
      const uint32_t grp = q / ka.team;
      X = q - grp * ka.team;
      T = grp * 8 + xcd;
    } else {
      T = blockIdx.x / ka.team;
      X = blockIdx.x - T * ka.team;
    }
  };
  // item of element e (>= nb: none) for this member
  auto itemOfElem = [&](uint32_t e) __attribute__((always_inline)) -> uint32_t {
    uint32_t T, X;
    teamX(T, X);
    const PCompArgs ka = A();
    return e < ka.nb ? e * ka.team + X : ka.items;
  };
  // element of this team's round r (r >= 2: from the log, written by member
  // 0 a round earlier; a lower workgroup index, so the wait always ends)
  auto elemOfRound = [&](uint32_t r) __attribute__((always_inline)) -> uint32_t {
    uint32_t T, X;
    teamX(T, X);
    const PCompArgs ka = A();
    const uint32_t teams = ka.grid / ka.team;
    if (r < 2) return min(r * teams + T, ka.nb);
    if (r >= ka.maxR) return ka.nb;
    gp<const uint64_t> slot = G(ka.elog) + uint64_t(T) * ka.maxR + r;
    uint64_t v = 0;
    // (not bounded by spinCap: no element's archive depends on this wait,
    // whose writer is never blocked; the bound only guards logic errors)
    for (uint32_t spins = 0; spins < (1u << 26); ++spins) {
      v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (uint32_t(v >> 32) == ka.epoch) return min(uint32_t(v), ka.nb);
      __builtin_amdgcn_s_sleep(2);
    }
    // (unreachable: member 0 never waits unboundedly) count it as abandoned
    __hip_atomic_fetch_add(G(ka.err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ka.nb;
  };
  // member 0: take the element of round r (>= 2) and log it
  auto dequeueRound = [&](uint32_t r) __attribute__((always_inline)) {
    uint32_t T, X;
    teamX(T, X);
    const PCompArgs ka = A();
    if (X != 0 || r >= ka.maxR) return;
    const uint32_t teams = ka.grid / ka.team;
    const uint64_t tag = uint64_t(ka.epoch) << 32;
    // one returning add on this call's counter (zeroed by the previous call
    // on this stream, see below): a compare-and-swap loop under 64
    // contenders took 17 us
    const uint32_t e = 2 * teams + uint32_t(__hip_atomic_fetch_add(G(ka.ctr) + (ka.epoch & 1u), 1ull,
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __hip_atomic_store(G(ka.elog) + uint64_t(T) * ka.maxR + r, tag | min(e, ka.nb), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  };
  auto pairSize = [&](const PItem& it, int hh) __attribute__((always_inline)) -> uint32_t {
    const uint32_t bk = it.x * pc::kBlocksPerItem + 2 * w + hh;
    return bk < it.nBlocks ? min(kBlockSize, it.n - bk * kBlockSize) : 0u;
  };
  // this lane's block size of an item (h ? pairSize(it, 1) : pairSize(it, 0))
  auto laneSize = [&](const PItem& it) __attribute__((always_inline)) -> uint32_t {
    const uint32_t bk = it.x * pc::kBlocksPerItem + 2 * w + halfNow();
    return bk < it.nBlocks ? min(kBlockSize, it.n - bk * kBlockSize) : 0u;
  };
  auto srcOf = [&](const PItem& it) __attribute__((always_inline)) -> gp<const WordT> {
    const uint32_t hh = halfNow();
    return (gp<const WordT>)startOf(IN(), it.b) +
           uint64_t(it.x * pc::kBlocksPerItem + 2 * w + hh) * kBlockSize;
  };

  // 16 B streaming loads of segment g of this lane's block into load slot
  // g % D (the input is read once; non-temporal, so the caches keep the
  // archives for the decoder: c2 step 267 -> 239 us together with the
  // decoder's streaming stores, same-box A/B), issued unconditionally (an
  // item's load schedule is then branch-free, so the compiler's wait counts
  // stay exact instead of draining every load in flight at a branch merge):
  // a vector with no word of the block (or of no item at all) reads a dummy
  // vector of this workgroup's slot space instead.  16 B-aligned input only
  // (the host sends anything else down the three-kernel path): a vector
  // holding the last valid word is then a whole 16 B chunk of the same page.
  auto load = [&](gp<const WordT> dummy, gp<const WordT> src, uint32_t uw, uint32_t g)
                  __attribute__((always_inline)) {
    // (opaque lane: the per-segment offsets are recomputed here, never
    // hoisted out of the loop -- 16 of them held live spill to scratch)
    uint32_t ll = l;
    asm volatile("" : "+v"(ll));
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const uint32_t j0 = g * pc::kSegWords + (k * 32 + ll) * kWPV;
      pv[g % D][k] = ld16nt(j0 < uw ? src + j0 : dummy);
    }
  };

  // ---- split segment g of an item from load slot g % D: raw bytes ->
  // archive, symbols -> this half-wave's symbol buffer.  kFull: both blocks of the pair
  // whole; otherwise words at or past the block's end are zeroed (their raw
  // bytes are the archive's zero padding, their symbols are never counted or
  // encoded) and vectors wholly past it store nothing.
  auto split = [&](const PItem& it, gp<uint8_t> raw, uint32_t uw, uint32_t g, auto fullTag)
                   __attribute__((always_inline)) {
    constexpr bool kFull = decltype(fullTag)::value;
    const uint32_t hh = halfNow();
    const uint32_t blk = it.x * pc::kBlocksPerItem + 2 * w + hh;
    lp<uint8_t> myT = (lp<uint8_t>)&symT[2 * w + hh][0];
    uint32_t ll = l;
    asm volatile("" : "+v"(ll));
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const uint32_t off = (k * 32 + ll) * kWPV;  // word offset in the segment
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
  // transpose segment g from the symbol buffer: lane l = 4m + r reads the
  // dwords of rows 4q + r (q < 4), columns 4m..4m+3; a 4 x 4 byte transpose
  // inside its quad (two DPP exchanges + v_perm) leaves it column l, steps
  // 4q..4q+3, packed for the encoder: 4 ds_read_b32 instead of 16
  // ds_read_u8.  Then count.
  auto transposeCount = [&](uint32_t g, uint32_t uw, bool masked) __attribute__((always_inline)) {
    lp<const uint8_t> myT = (lp<const uint8_t>)&symT[2 * w + halfNow()][0];
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
      for (uint32_t u = 0; u < enc::kUnroll; ++u) encStep<false, pc::kRing>(p, true, Ev[u], hv);
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
        encStep<true, pc::kRing>(p, t * 32 + l < uw, Ev[u], hv);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- publish L's partial histogram (and byte checksum): one tagged word
  // per bin, epoch << 16 | count (an item counts at most 32768 symbols) ----
  // (after a workgroup barrier: every wave's counts and ckS are in).  The
  // data carries its own epoch, so the consumer needs no separate arrival
  // flag: no drain of the stores, no barrier, one memory round trip per hop
  // (MI355X_MICROARCH.md: a tagged granule).  kXcd: plain (sc0) stores keep
  // the line in this XCD's L2 for the team's sc1 loads (header comment);
  // otherwise sc1 (write-through) stores, since members on other XCDs read
  // from memory.  The words live in the persistent epoch-tagged sync arena,
  // never in scratch a stale value could come from.
  auto publishHist = [&](const PItem& it) __attribute__((always_inline)) {
    const uint32_t tid = tidNow(), lane = laneNow();
    (void)tid;
    (void)lane;
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < pc::kHistCols; ++k) {
      cnt += hist[tid * pc::kHistStride + k];
      hist[tid * pc::kHistStride + k] = 0;
    }
    const uint32_t tag = A().epoch << 16;
    if constexpr (kXcd)
      __hip_atomic_store(G(A().part) + uint64_t(it.i) * kNumSymbols + tid, tag | cnt, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
    else
      stSc1(G(A().part) + uint64_t(it.i) * kNumSymbols + tid, tag | cnt);
    if constexpr (kCk) {
      if (tid == 0) stSc1(G(A().partCk) + it.i, tag | (ckS[0] ^ ckS[1] ^ ckS[2] ^ ckS[3]));
    }
  };

  // ---- slow path (wave 0 alone): L's element counted from its input, the
  // team having not completed within the budget.  c[j]: the count of symbol
  // 4 lane + j; ckOut: the element's byte checksum (kCk).  The histogram's
  // LDS is zero on entry and on exit (no other wave touches it meanwhile).
  auto countElementWave = [&](const PItem& it, uint32_t (&c)[4], uint32_t& ckOut) __attribute__((always_inline)) {
    const uint32_t lane = laneNow();
    const gp<const WordT> src = (gp<const WordT>)startOf(IN(), it.b);
    const uint32_t nv = divUp(it.n, kWPV);
    lp<uint32_t> col = (lp<uint32_t>)&hist[lane % pc::kHistCols];
    uint32_t x = 0;
    for (uint32_t v = lane; v < nv; v += 64) {
      const uint4 q = ld16(src + uint64_t(v) * kWPV);
      const WordT* ws = reinterpret_cast<const WordT*>(&q);
#pragma unroll
      for (uint32_t k = 0; k < kWPV; ++k) {
        if (v * kWPV + k < it.n) {
          __hip_atomic_fetch_add(col + __umul24(compOf<FT>(ws[k], 0), pc::kHistStride), 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
          if constexpr (kCk) x ^= uint32_t(ws[k]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t bin = 4 * lane + j;
      c[j] = 0;
#pragma unroll
      for (uint32_t k = 0; k < pc::kHistCols; ++k) {
        c[j] += hist[bin * pc::kHistStride + k];
        hist[bin * pc::kHistStride + k] = 0;
      }
    }
    if constexpr (kCk) ckOut = waveXor(x);
  };

  // ---- E's aggregate (its words, rounded to 8 per block) -> its look-back flag ----
  auto publishAgg = [&](const PItem& it) __attribute__((always_inline)) {
    const uint32_t tid = tidNow(), lane = laneNow();
    (void)tid;
    (void)lane;
    const uint32_t first = it.x * pc::kBlocksPerItem;
    const uint32_t nk = first < it.nBlocks ? min(pc::kBlocksPerItem, it.nBlocks - first) : 0u;
    const uint32_t r = lane < nk ? roundUp(cwE[lane], 8) : 0u;
    const uint32_t agg = readfirst(__shfl(waveInclusiveScan(r), 63));
    if (lane == 0)
      __hip_atomic_store(G(A().flags) + it.tb + it.x,
                         (it.x == 0 ? kFlagPrefix : kFlagAgg) | (uint64_t(A().epoch) << 32) | agg,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // ---- wave 0: E's look-back -> preE, the last member's header total ----
  auto lookBackE = [&](const PItem& it) __attribute__((always_inline)) {
    const uint32_t tid = tidNow(), lane = laneNow();
    (void)tid;
    (void)lane;
    const uint32_t first = it.x * pc::kBlocksPerItem;
    const uint32_t nk = first < it.nBlocks ? min(pc::kBlocksPerItem, it.nBlocks - first) : 0u;
    gp<uint8_t> base = startOf(OUT(), it.b);
    gp<uint8_t> o = base + (FT == 0 ? 0u : 32u + floatRawBytes(FT, it.n));  // ANS archive
    gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
    gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * it.nBlocks);
    const uint32_t r = lane < nk ? roundUp(cwE[lane], 8) : 0u;
    const uint32_t inc = waveInclusiveScan(r);
    const uint32_t agg = readfirst(__shfl(inc, 63));
    bool pz = false;
    const uint32_t excl = lookBackPoison(G(A().flags) + it.tb, it.x, agg, A().epoch, A().spinCap, pz, false);
    if (lane < nk) preE[lane] = excl + inc - r;
    if (lane == 0) {
      poisonS = pz ? 1u : 0u;
      if (it.x == it.team - 1) {
        if (pz) {
          if (A().outSize) G(A().outSize)[it.b] = 0u;
          __hip_atomic_fetch_add(G(A().err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          EncTail t{nullptr, nullptr, A().outSize, nullptr, 0, A().pb, A().useChecksum};
          t.sparseN = A().sparseN;
          writeHeadTotal<FT>(base, o, it.n, it.nBlocks, excl + agg, bwords, t, it.b);
        }
      }
    }
  };

  // ---- wave 0, after L's normalisation: L's header fields known before
  // encoding (all but the word totals), its pdf table and the raw section's
  // rounding tails, by the team's first member ----
  auto writeHeadFixedL = [&](const PItem& it, uint32_t ckv) __attribute__((always_inline)) {
    const uint32_t tid = tidNow(), lane = laneNow();
    (void)tid;
    (void)lane;
    gp<uint8_t> base = startOf(OUT(), it.b);
    gp<uint8_t> o = base + (FT == 0 ? 0u : 32u + floatRawBytes(FT, it.n));  // ANS archive
    if (lane == 0) {
      const bool ansCk = FT == 0 && A().useChecksum;
      if (FT != 0) ckv = A().ckIn ? G(A().ckIn)[it.b] : 0u;
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
    // pdf: 4 symbols per lane, one 8 B store
    {
      const u32x2 pd = *(lp<const u32x2>)&pdfS[4 * lane];
      *(gp<u32x2>)((gp<uint8_t>)(o + kANSHeaderBytes) + 8 * lane) = pd;
    }
    if constexpr (FT != 0) {
      gp<uint8_t> raw = base + 32;
      const uint32_t n = it.n;
      if (lane < 16) {
        if constexpr (FT == 1 || FT == 2) {
          if (n + lane < roundUp(n, 16)) raw[n + lane] = 0;
        } else {
          if (n + lane < roundUp(n, 8)) ((gp<uint16_t>)raw)[n + lane] = 0;
          if (n + lane < roundUp(n, 16)) raw[2 * roundUp(n, 8) + n + lane] = 0;
        }
      }
    }
  };

  // ---- placement of E by waves 1-3 (t = tid - 64 of 192), after the
  // look-back: blockWords and the payload copy-out ----
  auto place = [&](const PItem& it) __attribute__((always_inline)) {
    const uint32_t tid = tidNow(), lane = laneNow();
    (void)tid;
    (void)lane;
    constexpr uint32_t kPT = pc::kThreads - 64;
    const uint32_t t = tid - 64;
    const uint32_t first = it.x * pc::kBlocksPerItem;
    const uint32_t nk = first < it.nBlocks ? min(pc::kBlocksPerItem, it.nBlocks - first) : 0u;
    gp<uint8_t> o = startOf(OUT(), it.b) + (FT == 0 ? 0u : 32u + floatRawBytes(FT, it.n));  // ANS archive
    gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
    gp<uint2> bwords = (gp<uint2>)(states + uint64_t(kStateBytesPerBlock) * it.nBlocks);
    // a poisoned element's archive is abandoned (outSize 0): its payload
    // range is not known, so nothing more is written
    if (nk == 0 || poisonS) return;
    if (t < nk) {
      const uint32_t k = first + t;
      const uint32_t uwk = min(kBlockSize, it.n - k * kBlockSize);
      st8(bwords + k, make_uint2((uwk << 16) | cwE[t], preE[t]));
    }
    // payload: 16 B vectors over the item's contiguous archive range; the
    // source is the block's ring, or its slot for words spilled before the end
    // (per-wave block lists with wave-uniform block parameters measured +1
    // us)
    gp<uint4> dst = (gp<uint4>)((gp<uint8_t>)(bwords + roundUp(it.nBlocks, 2)) + 2ull * preE[0]);
    const uint32_t nv = (preE[nk - 1] + roundUp(cwE[nk - 1], 8) - preE[0]) / 8;
    for (uint32_t v = t; v < nv; v += kPT) {
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

  // ---- encode E's pair done: states to the archive, word counts to LDS ----
  auto encodeDone = [&](const PItem& it) __attribute__((always_inline)) {
    const uint32_t hh = halfNow();
    const uint32_t uw = laneSize(it);
    if (uw) {
      gp<uint8_t> o = startOf(OUT(), it.b) + (FT == 0 ? 0u : 32u + floatRawBytes(FT, it.n));
      gp<uint8_t> states = o + kANSHeaderBytes + kPdfBytes;
      const uint32_t blk = it.x * pc::kBlocksPerItem + 2 * w + hh;
      ((gp<uint32_t>)(states + uint64_t(kStateBytesPerBlock) * blk))[l] = p.x;
    }
    if (l == 0) {
      cwE[2 * w + hh] = uw ? uint32_t(hh ? p.nout[1] : p.nout[0]) : 0u;
      flE[2 * w + hh] = uw ? uint32_t(hh ? p.flushed[1] : p.flushed[0]) : 0u;
    }
  };

  // a vector with no word of the block loads from this workgroup's slot space
  const gp<const WordT> dummy = (gp<const WordT>)slotBase;

  // ================= the pipeline =================
  // Only item indices live across iterations; everything else is recomputed
  // (scalar work) where it is needed.
  // the next call on this stream (epoch + 1) counts from zero: calls on one
  // stream run one after another, so nothing reads that counter now
  if (blockIdx.x == 0 && tid == 0)
    __hip_atomic_store(G(A().ctr) + ((A().epoch + 1) & 1u), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();  // histogram zeroed
  uint32_t round = 0;
  uint32_t iE = A().items, iL = itemOfElem(elemOfRound(0));
  if (iL >= A().items) return;
  while (true) {
    const bool hasE = iE < A().items, hasL = iL < A().items;
    if (!hasE && !hasL) break;
    // Segment-phase wave priority rotates over the CU's dispatch slots
    // round by round.  At equal priority the SIMD arbiter favours the older
    // waves: the last-dispatched slot's teams ran a quarter slower and set
    // the kernel's end (slot medians 140 / 146 / 152 / 160 us of a 169 us
    // launch); rotating gives each slot each level in turn.  (The hand-off
    // window runs above all of them.)
    {
      const uint32_t pr = (blockIdx.x / A().slotSpan + round) % 3u;
      if (pr == 0) __builtin_amdgcn_s_setprio(0);
      else if (pr == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(2);
    }
    {
      const PItem E = itemOf(iE, A(), IN()), L = itemOf(iL, A(), IN());
      const uint32_t uwE0 = pairSize(E, 0), uwE1 = pairSize(E, 1);
      const uint32_t uwL0 = pairSize(L, 0), uwL1 = pairSize(L, 1);
      // encode: the full-step variant when both blocks of the pair are whole
      // (uwE0 >= uwE1)
      const bool encOn = hasE && uwE0 != 0;
      const bool fastE = uwE1 == kBlockSize;
      const uint32_t uwEnc = halfNow() ? uwE1 : uwE0;
      // split: the unmasked variant when both blocks of the pair are whole
      const bool loadOn = hasL && uwL0 != 0;
      const bool fullL = uwL1 == kBlockSize;
      const uint32_t uwL = halfNow() ? uwL1 : uwL0;
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
        for (uint32_t g = 0; g < uint32_t(D); ++g) load(dummy, srcL, uwL, g);
        staticFor<pc::kSegs>([&](auto gTag) __attribute__((always_inline)) {
          constexpr uint32_t g = decltype(gTag)::value;
          encSeg(g);
          if (fullL) split(L, rawL, uwL, g, std::true_type{});
          else split(L, rawL, uwL, g, std::false_type{});
          if constexpr (g + D < pc::kSegs) load(dummy, srcL, uwL, g + D);
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
    __builtin_amdgcn_s_setprio(3);
    if constexpr (kCk) {
      if (hasL) {
        const uint32_t c = waveXor((ck ^ (ck >> 8) ^ (ck >> 16) ^ (ck >> 24)) & 0xffu);
        if (lane == 0) ckS[w] = c;
      }
      ck = 0;
    }
    // E's word counts and L's histogram counts are in
    __syncthreads();
    if (hasL) publishHist(itemOf(iL, A(), IN()));
    if (hasE && w == 0) publishAgg(itemOf(iE, A(), IN()));
    // L's team partials: wave w gathers members w, w + 4, ... (16 B = four
    // bins per lane: a lane holds bins 4l .. 4l + 3, the layout the one-wave
    // normalisation takes); the first four of each wave's members are loaded
    // now, in flight over E's look-back; their tags say who is in
    constexpr uint32_t kPer = pc::kMaxTeam / pc::kWaves;  // members per wave
    constexpr uint32_t kFirst = 4;                         // loaded before the barrier
    u32x4 pa[kFirst];
    uint32_t ckv = 0;
    if (hasL) {
      const uint32_t lane = laneNow();
      const PItem L = itemOf(iL, A(), IN());
      const BufRsrc hb = bufOf(G(A().part) + uint64_t(L.tb) * kNumSymbols);
#pragma unroll
      for (uint32_t m = 0; m < kFirst; ++m) {
        const uint32_t k = w + pc::kWaves * m;
        pa[m] = k < L.team ? ldSc1x4(hb, (k * 64 + lane) * 16) : u32x4{0, 0, 0, 0};
      }
      if constexpr (kCk) {
        if (w == 0) ckv = lane < L.team ? ldSc1(G(A().partCk) + L.tb + lane) : 0u;
      }
    }
    // (member 0, wave 0) this team's element of round + 2, taken now, if
    // round + 1 has one
    if (hasL && w == 0 && lane == 0) {
      uint32_t T, X;
      teamX(T, X);
      if (X == 0 && elemOfRound(round + 1) < A().nb) dequeueRound(round + 2);
    }
    // the next round's element: its log entry (written a round ago) read
    // now, by lane 0 of each wave, in flight over the rest of the window
    uint64_t nextRaw = 0;
    if (hasL && lane == 0 && round + 1 >= 2 && round + 1 < A().maxR) {
      uint32_t T, X;
      teamX(T, X);
      nextRaw = __hip_atomic_load(G(A().elog) + uint64_t(T) * A().maxR + round + 1, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    if (hasE && w == 0) lookBackE(itemOf(iE, A(), IN()));
    // spilled words of E are read back by other waves in place(): a wave
    // that spilled waits for its slot stores
    if (hasE && (p.flushed[0] | p.flushed[1])) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // L's team partials -> per-wave sums (LDS, the zeroed histogram's first
    // 4 KB); wave 0 adds them and normalises L while waves 1-3 place E
    if (hasL) {
      const uint32_t lane = laneNow();
      const PItem L = itemOf(iL, A(), IN());
      const uint32_t ep = A().epoch;
      const BufRsrc hb = bufOf(G(A().part) + uint64_t(L.tb) * kNumSymbols);
      auto tagged = [&](const u32x4& v) __attribute__((always_inline)) -> bool {
        return (v.x >> 16) == ep && (v.y >> 16) == ep && (v.z >> 16) == ep && (v.w >> 16) == ep;
      };
      uint32_t c[4] = {0, 0, 0, 0};
      uint32_t miss = 0;  // bit m: member w + 4 m not yet summed (this lane)
      auto take = [&](const u32x4& v) __attribute__((always_inline)) {
        c[0] += v.x & 0xffffu;
        c[1] += v.y & 0xffffu;
        c[2] += v.z & 0xffffu;
        c[3] += v.w & 0xffffu;
      };
#pragma unroll
      for (uint32_t m = 0; m < kPer; ++m) {
        const uint32_t k = w + pc::kWaves * m;
        if (k >= L.team) continue;
        if (m < kFirst && tagged(pa[m])) take(pa[m]);
        else miss |= 1u << m;
      }
      bool ckMissing = kCk && w == 0 && lane < L.team;
      uint32_t ckAcc = 0;
      if (ckMissing && (ckv >> 16) == ep) {
        ckAcc = ckv & 0xffu;
        ckMissing = false;
      }
      // the rest (members >= 16, late members), polled with backoff; after
      // the time budget (or spinCap polls) this wave gives up and the element
      // is counted from its input instead
      bool giveUp = false;
      const uint64_t t0 = realtime();
      for (uint32_t spins = 0; ballot(miss != 0 || ckMissing) != 0; ++spins) {
        if (spins >= A().spinCap || realtime() - t0 >= A().fallbackTicks) {
          giveUp = true;
          break;
        }
        if (spins) __builtin_amdgcn_s_sleep(2);
#pragma unroll
        for (uint32_t m = 0; m < kPer; ++m) {
          if ((miss >> m) & 1u) {
            const u32x4 v = ldSc1x4(hb, ((w + pc::kWaves * m) * 64 + lane) * 16);
            if (tagged(v)) {
              take(v);
              miss &= ~(1u << m);
            }
          }
        }
        if (ckMissing) {
          ckv = ldSc1(G(A().partCk) + L.tb + lane);
          if ((ckv >> 16) == ep) {
            ckAcc = ckv & 0xffu;
            ckMissing = false;
          }
        }
      }
      lp<u32x4> red4 = (lp<u32x4>)&hist[0];  // [wave][64 lanes] (the histogram is zero here)
      if (w != 0) {
        red4[w * 64 + lane] = u32x4{c[0], c[1], c[2], c[3]};
        if (giveUp && lane == 0) __hip_atomic_store(&fbS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // (one add per wave: the LDS counter reaches kWaves - 1)
        if (lane == 0) __hip_atomic_fetch_add(&sigS, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        while (__hip_atomic_load(&sigS, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != pc::kWaves - 1)
          __builtin_amdgcn_s_sleep(1);
        sigS = 0;
        uint32_t ckL = kCk ? waveXor(ckAcc) : 0u;
        const bool fb = giveUp || __hip_atomic_load(&fbS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
#pragma unroll
        for (uint32_t v = 1; v < pc::kWaves; ++v) {
          const u32x4 o = red4[v * 64 + lane];
          c[0] += o.x;
          c[1] += o.y;
          c[2] += o.z;
          c[3] += o.w;
          red4[v * 64 + lane] = u32x4{0, 0, 0, 0};
        }
        if (fb) {
          fbS = 0;
          // counted per call (dietgpu_barrier_fallback_count): a nonzero
          // count on an uncontended chip means a hand-off that never lands
          if (lane == 0)
            __hip_atomic_fetch_add(G(A().err) + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          countElementWave(L, c, ckL);
        }
        uint32_t cdf[4];
        if (L.n != 0) {
          normalizeWave(c, cdf, L.n, A().pb);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) c[j] = cdf[j] = 0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4 e = encTableEntryReg(c[j], cdf[j], A().pb);
          *(lp<u32x4>)&tblS[4 * (4 * lane + j)] = u32x4{e.x, e.y, e.z, e.w};
        }
        *(lp<u32x2>)&pdfS[4 * lane] = u32x2{c[0] | (c[1] << 16), c[2] | (c[3] << 16)};
        if (L.x == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          writeHeadFixedL(L, ckL);
        }
      }
    }
    if (hasE && w != 0) place(itemOf(iE, A(), IN()));
    // the next round's element (logged a round ago): lane 0 of each wave
    uint32_t iN = A().items;
    if (hasL) {
      uint32_t e = 0;
      if (lane == 0) {
        e = uint32_t(nextRaw >> 32) == A().epoch ? min(uint32_t(nextRaw), A().nb) : elemOfRound(round + 1);
      }
      iN = itemOfElem(readfirst(e));
    }
    __syncthreads();
    iE = iL;
    iL = iN;
    ++round;
  }
}

}  // namespace dietgpu
