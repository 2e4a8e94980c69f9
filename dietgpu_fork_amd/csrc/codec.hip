// Host orchestration of the MI355X rANS byte codec and float codec.
// Implements the C++ API of include/dietgpu/GpuANSCodec.h and
// include/dietgpu/GpuFloatCodec.h (reference: ans/GpuANSEncode.cu,
// ans/GpuANSDecode.cu, ans/GpuANSInfo.cu, float/GpuFloatCompress.cu,
// float/GpuFloatDecompress.cu, float/GpuFloatInfo.cu).
//
// Launch sequence per call (all stream-ordered, no host sync unless a
// checksum has to be verified):
//   compress:   k_hist -> k_normalize -> k_encode (+ k_coalesce for fp64)
//   decompress: k_decode (table build + rANS decode + float join fused)
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <tuple>
#include <type_traits>
#include <vector>

#include "codec_internal.h"
#include "dietgpu/GpuANSCodec.h"
#include "dietgpu/GpuFloatCodec.h"
#include "pcompress.h"
#include "decode.h"
#include "encode.h"
#include "profile.h"

namespace dietgpu {

namespace {
constexpr uint32_t kMaxGridY = 65535;

// k_hist chunk (words): 4 K .. 64 K words, halved while the batch has fewer
// than 2,048 chunks -- for single-segment formats only down to 16 K words
// once there are 512: a k_hist workgroup zeroes and sums 32 KB of LDS
// counters, which 4 K- or 8 K-word chunks do not amortise (1 x 16M bf16
// compress 41.6 -> 37.0 us, fp32 48.2 -> 46.3 us, same box; 1e8-word
// elements keep their 32 K-word chunks, 64 K measured slower).  fp64's two
// 16-column counter sets keep the 2,048 rule.
uint32_t histChunkWords(uint32_t nb, uint32_t maxSize, int segs) {
  uint32_t chunk = 64 * 1024;
  auto enough = [&](uint32_t c) {
    const uint64_t total = uint64_t(nb) * divUp(std::max(maxSize, 1u), c);
    return total >= 2048 || (segs == 1 && c <= 16 * 1024 && total >= 512);
  };
  while (chunk > 4096 && !enough(chunk)) chunk /= 2;
  while (divUp(maxSize, chunk) > 4096) chunk *= 2;
  return chunk;
}

// workgroups of `kernel` resident on the whole device at once (cached per
// device, kernel and LDS size: the queries cost host time on every call)
uint32_t residentSlots(const void* kernel, int threads, uint32_t dynLds) {
  static std::mutex m;
  static std::map<std::tuple<int, const void*, int, uint32_t>, uint32_t> cache;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  const auto key = std::make_tuple(dev, kernel, threads, dynLds);
  std::lock_guard<std::mutex> g(m);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 0, perCU = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kernel, threads, dynLds));
  const uint32_t v = uint32_t(std::max(1, cus) * std::max(1, perCU));
  cache[key] = v;
  return v;
}

uint32_t residentCUs() {
  static std::mutex m;
  static std::map<int, uint32_t> cache;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(m);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  cache[dev] = uint32_t(std::max(1, cus));
  return cache[dev];
}

void checkProbBits(int pb) {
  DG_CHECK(pb >= 9 && pb <= 11, "unhandled pdf precision " << pb << " (must be 9, 10 or 11)");
}

}  // namespace

// ---------------------------------------------------------------------------
// parameter tables (the reference's BatchProvider pointer / size arrays)
// ---------------------------------------------------------------------------
// Small tables (allowInline, <= 8 KB) ride in the InlineTable kernel argument
// of k_pcompress / k_decode: the BatchDesc fields then hold byte offsets into
// it (biased by 8, so none is 0) and BatchDesc::inl says which.  Any other
// kernel gets a device copy made in its driver's scope (DeviceDescs).  Larger
// tables, or callers that need device pointers, get one upload here.
struct DeviceTables {
  GpuMemoryReservation<uint8_t> mem;
  std::vector<uint8_t> host;
  std::unique_ptr<InlineTable> image;  // kernarg image when inline
  bool inl = false;
  const uint64_t* u64a = nullptr;
  const uint64_t* u64b = nullptr;
  const uint32_t* u32a = nullptr;

  // mark the table-backed fields of a descriptor built from u64a/u64b/u32a
  BatchDesc tag(BatchDesc d) const {
    if (!inl) return d;
    if (d.ptrs) d.inl |= BatchDesc::kInlPtrs;
    if (d.sizes) d.inl |= BatchDesc::kInlSizes;
    if (d.offsets) d.inl |= BatchDesc::kInlOffsets;
    return d;
  }
};
constexpr size_t kInlineBias = 8;

const InlineTable& kernargTable(const DeviceTables* t) {
  static const InlineTable kEmpty{};
  return t && t->inl ? *t->image : kEmpty;
}

DeviceTables uploadTables(StackDeviceMemory& res, hipStream_t s, uint32_t nb,
                          const std::vector<uint64_t>& a, const std::vector<uint64_t>& b,
                          const std::vector<uint32_t>& c, bool allowInline = false) {
  const size_t bytesA = a.size() * 8, bytesB = b.size() * 8, bytesC = c.size() * 4;
  DeviceTables t;
  t.host.resize(bytesA + bytesB + bytesC);
  if (bytesA) std::memcpy(t.host.data(), a.data(), bytesA);
  if (bytesB) std::memcpy(t.host.data() + bytesA, b.data(), bytesB);
  if (bytesC) std::memcpy(t.host.data() + bytesA + bytesB, c.data(), bytesC);
  t.inl = allowInline && kInlineBias + t.host.size() <= sizeof(InlineTable);
  uintptr_t base;
  if (t.inl) {
    t.image.reset(new InlineTable());
    std::memcpy(reinterpret_cast<uint8_t*>(t.image->w) + kInlineBias, t.host.data(), t.host.size());
    base = kInlineBias;
  } else {
    t.mem = res.alloc<uint8_t>(s, std::max<size_t>(t.host.size(), 1));
    StackDeviceMemory::copyToDevice(t.mem.data(), t.host.data(), t.host.size(), s);
    base = reinterpret_cast<uintptr_t>(t.mem.data());
  }
  t.u64a = reinterpret_cast<const uint64_t*>(base);
  t.u64b = reinterpret_cast<const uint64_t*>(base + bytesA);
  t.u32a = reinterpret_cast<const uint32_t*>(base + bytesA + bytesB);
  (void)nb;
  return t;
}

// Device copy of inline tables for kernels without an InlineTable argument,
// allocated in the calling driver's scope (the arena is LIFO) and only when
// the tables are inline.  A one-element batch needs no copy at all: its
// descriptors become stride descriptors of that element (its address, and
// its size as the fixed size), so the three-kernel path of a batch-1
// pointer / split-size call launches no upload kernel (fp64 1 x 16M words
// and the float_benchmark's batch-1 grid: a 4.7 us k_table launch before
// k_hist).
struct DeviceDescs {
  GpuMemoryReservation<uint8_t> mem;
  uintptr_t base = 0;
  const InlineTable* single = nullptr;  // nb == 1: entries read from the kernarg image
  DeviceDescs(StackDeviceMemory& res, hipStream_t s, const DeviceTables* t, uint32_t nb) {
    if (!t || !t->inl) return;
    if (nb == 1) {
      single = t->image.get();
      return;
    }
    mem = res.alloc<uint8_t>(s, std::max<size_t>(t->host.size(), 1));
    StackDeviceMemory::copyToDevice(mem.data(), t->host.data(), t->host.size(), s);
    base = reinterpret_cast<uintptr_t>(mem.data()) - kInlineBias;
  }
  BatchDesc map(BatchDesc d) const {
    if (!d.inl) return d;
    if (single) {
      auto entry = [&](auto p) {
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(p)>>;
        T v;
        std::memcpy(&v, reinterpret_cast<const uint8_t*>(single->w) + reinterpret_cast<uintptr_t>(p), sizeof(T));
        return v;
      };
      uint8_t* start = d.mode == BatchDesc::kPointer ? reinterpret_cast<uint8_t*>(entry(d.ptrs))
                       : d.mode == BatchDesc::kSplit ? d.base + entry(d.offsets)
                                                     : d.base;
      DG_CHECK(!d.sizes || (d.inl & BatchDesc::kInlSizes), "mixed inline / device size table");
      const uint32_t size = d.sizes ? entry(d.sizes) : d.fixedSize;
      return BatchDesc::strided(start, 0, size);
    }
    auto rebase = [&](auto p) { return reinterpret_cast<decltype(p)>(base + reinterpret_cast<uintptr_t>(p)); };
    if (d.inl & BatchDesc::kInlPtrs) d.ptrs = rebase(d.ptrs);
    if (d.inl & BatchDesc::kInlSizes) d.sizes = rebase(d.sizes);
    if (d.inl & BatchDesc::kInlOffsets) d.offsets = rebase(d.offsets);
    d.inl = 0;
    return d;
  }
};

// ---------------------------------------------------------------------------
// generic drivers
// ---------------------------------------------------------------------------
// Device error words (one pair per device, code object global): [0] elements
// the compressor poisoned (a bounded wait ran out, pcompress.h; their outSize
// is 0), [1] k_pcompress team-barrier fallbacks (a workgroup that counted its
// element from the input after the time budget; archives stay exact).
__device__ uint32_t g_dgErrors[2];

uint32_t* deviceErrorWord() {
  static std::mutex m;
  static std::map<int, uint32_t*> addr;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(m);
  auto it = addr.find(dev);
  if (it != addr.end()) return it->second;
  void* p = nullptr;
  HIP_CHECK(hipGetSymbolAddress(&p, HIP_SYMBOL(g_dgErrors)));
  addr[dev] = static_cast<uint32_t*>(p);
  return static_cast<uint32_t*>(p);
}

static uint32_t readErrorWord(uint32_t k, bool reset) {
  uint32_t* p = deviceErrorWord() + k;
  HIP_CHECK(hipDeviceSynchronize());
  uint32_t v = 0;
  HIP_CHECK(hipMemcpy(&v, p, sizeof(v), hipMemcpyDeviceToHost));
  if (reset && v) HIP_CHECK(hipMemset(p, 0, sizeof(v)));
  return v;
}

uint32_t deviceErrorCount(bool reset) { return readErrorWord(0, reset); }
uint32_t barrierFallbackCount(bool reset) { return readErrorWord(1, reset); }

// Single-pass compression (k_pcompress, pcompress.h) for single-segment
// formats without a caller-supplied histogram, elements of at most
// pc::kMaxTeam items (1 MiB of symbols).  One generation of resident
// workgroups pulls items off the work queue.
// Teams of k_pcompress for nb elements of maxWords: team size, teams per
// round (XCD-aligned when that fits, see compressPersistent) and whether
// they are XCD-aligned.  team == 0: the elements are too large.
struct PersistentPlan {
  uint32_t team = 0, teamsPerRound = 0, rounds = 0;
  bool xcd = false;
};

template <int FT>
PersistentPlan planPersistent(uint32_t nb, uint32_t maxWords) {
  PersistentPlan p;
  const uint32_t team = std::max(1u, divUp(divUp(maxWords, kBlockSize), pc::kBlocksPerItem));
  if (team > pc::kMaxTeam || nb == 0) return p;
  // (the instances have the same resources: one occupancy query)
  const uint32_t slots = residentSlots(reinterpret_cast<const void*>(&k_pcompress<FT, false, true>), pc::kThreads, 0);
  // rounds of whole teams, balanced: R rounds of ceil(nb / R) teams
  const uint32_t maxTeams = std::max(1u, slots / team);
  p.team = team;
  p.rounds = divUp(nb, maxTeams);
  p.teamsPerRound = divUp(nb, p.rounds);
  // XCD-aligned teams (kXcd, pcompress.h) whenever the teams per round round
  // up to a multiple of 8 within the resident grid (never more rounds; a
  // batch of fewer than 8 elements gets idle teams that exit at once), so
  // the partial histograms stay in one L2.  Otherwise (e.g. 33 elements of
  // 31 items in 1,024 slots) the team members span XCDs and the partials go
  // out write-through.
  p.xcd = roundUp(p.teamsPerRound, 8) <= maxTeams;
  if (p.xcd) p.teamsPerRound = roundUp(p.teamsPerRound, 8);
  return p;
}

// Whether the single-pass compressor beats the three-kernel path (k_hist ->
// k_encode with prologue normalisation) for a batch.  At most 256 items, or
// one round whose teams cannot be XCD-aligned, leave most of the chip idle
// while a team's members wait on each other's partial histograms; there the
// chip-wide histogram pass plus the encoder are faster (round 5, bf16:
// 1 x 1e6 words 30.7 -> 22.9 us, 8 x 524288 26.9 -> 25.1 us, 33 x 1e6
// 48.9 -> 46.9 us; 16 x 1e6, 496 items, stays single-pass: 33.5 against
// 37.1 us).
// (dietgpu_set_compress_path overrides the rule: test hook.)
template <int FT>
bool persistentPreferred(uint32_t nb, uint32_t maxWords) {
  const int mode = compressPath();
  if (mode == 2) return false;
  const PersistentPlan p = planPersistent<FT>(nb, maxWords);
  if (p.team == 0) return false;
  if (mode == 1) return true;
  if (uint64_t(p.team) * nb <= 256) return false;
  return !(p.rounds == 1 && !p.xcd);
}
template bool persistentPreferred<1>(uint32_t, uint32_t);
template bool persistentPreferred<2>(uint32_t, uint32_t);
template bool persistentPreferred<3>(uint32_t, uint32_t);

template <int FT, bool kCk, bool kXcd>
void launchPersistent(uint32_t grid, hipStream_t s, const DeviceTables* tabs, const BatchDesc& in,
                      const BatchDesc& out, const PCompArgs& a) {
  k_pcompress<FT, kCk, kXcd><<<grid, pc::kThreads, 0, s>>>(kernargTable(tabs), in, out, a);
  HIP_LAUNCH_CHECK();
}

template <int FT, bool kCk>
bool compressPersistent(StackDeviceMemory& res, int pb, bool useChecksum, uint32_t nb,
                        const BatchDesc& in, uint32_t maxSize, const BatchDesc& out,
                        uint32_t* outSize_dev, hipStream_t s, const DeviceTables* tabs,
                        const uint32_t* sparseN) {
  const PersistentPlan plan = planPersistent<FT>(nb, maxSize);
  const uint32_t team = plan.team;
  if (team == 0) return false;
  const uint64_t items64 = uint64_t(team) * nb;
  DG_CHECK(items64 < (1ull << 30), "batch too large for one compress call");
  const uint32_t items = uint32_t(items64);
  const bool xcdTeams = plan.xcd;
  const uint32_t grid = plan.teamsPerRound * team;

  auto slotMem = res.alloc<uint8_t>(s, size_t(grid) * pc::kBlocksPerItem * kSlotDataBytes);
  auto ck = res.alloc<uint32_t>(s, FT != 0 && useChecksum ? nb : 1);
  DeviceDescs dd(res, s, FT != 0 && useChecksum ? tabs : nullptr, nb);  // k_checksum's view
  // epoch-tagged state in this stream's persistent arena (no per-call
  // zeroing), one region per kind of word: the dequeue counters (at a fixed
  // place: a call zeroes the next call's), the look-back flags, the tagged
  // partial histograms then the tagged partial byte checksums, the per-team
  // element log.  A team takes at most maxR rounds (pcompress.h, "Teams and
  // elements"): twice the static share bounds the log while leaving the
  // teams below it room for every element.
  const size_t partBytes = size_t(items) * kNumSymbols * 4;
  const uint32_t teams = grid / team;
  const uint32_t maxR = 2 * divUp(nb, teams) + 2;
  const size_t regions[kSyncRegions] = {16, size_t(items) * 8, partBytes + (kCk ? size_t(items) * 4 : 0),
                                        size_t(teams) * maxR * 8, 0};
  SyncLease lease(res, s, regions, /*dequeue=*/true);
  if (FT != 0 && useChecksum) {
    zeroAsync(ck.data(), sizeof(uint32_t) * nb, s);
    // float checksum: the reference passes float-word counts as byte counts
    // (float/GpuFloatCompress.cuh:709)
    const uint32_t ckChunk = 1u << 20;
    for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
      const uint32_t ny = std::min(kMaxGridY, nb - y0);
      dim3 g(std::max(1u, divUp(maxSize, ckChunk)), ny);
      k_checksum<<<g, kThreads, 0, s>>>(dd.map(in), y0, 1, ckChunk, ck.data());
      HIP_LAUNCH_CHECK();
    }
  }
  PCompArgs a;
  a.ctr = static_cast<uint64_t*>(lease.base[kSyncCounters]);
  a.flags = static_cast<uint64_t*>(lease.base[kSyncFlags]);
  a.part = static_cast<uint32_t*>(lease.base[kSyncPartials]);
  a.partCk = kCk ? a.part + size_t(items) * kNumSymbols : nullptr;
  a.elog = static_cast<uint64_t*>(lease.base[kSyncLog]);
  a.maxR = maxR;
  a.slotSpan = std::max(1u, residentCUs());
  a.err = deviceErrorWord();
  a.slots = slotMem.data();
  a.ckIn = FT != 0 && useChecksum ? ck.data() : nullptr;
  a.outSize = outSize_dev;
  a.sparseN = sparseN;
  a.items = items;
  a.team = team;
  a.nb = nb;
  a.grid = grid;
  a.epoch = lease.epoch;
  a.spinCap = spinCap();
  a.fallbackTicks = barrierBudgetTicks();
  a.pb = pb;
  a.useChecksum = useChecksum;
  prof::Scope p("compress", s);
  if (xcdTeams) launchPersistent<FT, kCk, true>(grid, s, tabs, in, out, a);
  else launchPersistent<FT, kCk, false>(grid, s, tabs, in, out, a);
  return true;
}

// inAligned16: every element's input starts 16 B-aligned (the single-pass
// compressor reads whole 16 B vectors; anything else takes three kernels)
template <int FT>
void encodeBatchDevice(StackDeviceMemory& res, int pb, bool useChecksum, uint32_t nb,
                       const BatchDesc& inArg, uint32_t maxSize, const uint32_t* hist_dev,
                       const BatchDesc& outArg, uint32_t* outSize_dev, hipStream_t s,
                       const DeviceTables* tabs, bool inAligned16, const PartialHist* pre = nullptr,
                       const uint32_t* sparseN = nullptr) {
  checkProbBits(pb);
  if (nb == 0) return;
  constexpr int kSegs = FloatTraits<FT>::kSegs;
  constexpr bool kFused = kSegs == 1;  // k_encode writes the archive itself
  const uint32_t MB = divUp(maxSize, kBlockSize);
  const bool userHist = FT == 0 && hist_dev != nullptr;
  const bool preHist = FT != 0 && pre != nullptr;  // partial rows counted by the caller
  const bool preNorm = preHist && pre->table != nullptr;  // ... and normalised
  const uint32_t chunkWords = histChunkWords(nb, maxSize, kSegs);
  const uint32_t chunks = preHist ? std::max(1u, pre->nRows) : std::max(1u, divUp(maxSize, chunkWords));
  const bool runHist = !preHist && (!userHist || useChecksum);
  const bool rawCk = FT == 0 && useChecksum;
  const uint32_t nW = std::max(1u, divUp(MB, EncCfg<FT>::kBlocksPerWG));
  if constexpr (kFused) {
    // (byte archives with a checksum stay single-pass: the three-kernel path
    // has no prologue normalisation for them)
    if (!userHist && inAligned16 && ((rawCk && compressPath() != 2) || persistentPreferred<FT>(nb, maxSize))) {
      const bool done = rawCk ? compressPersistent<FT, FT == 0>(res, pb, useChecksum, nb, inArg,
                                                                 maxSize, outArg, outSize_dev, s, tabs, sparseN)
                              : compressPersistent<FT, false>(res, pb, useChecksum, nb, inArg, maxSize,
                                                              outArg, outSize_dev, s, tabs, sparseN);
      if (done) return;
    }
  }
  // three-kernel path: plain device tables
  DeviceDescs dd(res, s, tabs, nb);
  const BatchDesc in = dd.map(inArg), out = dd.map(outArg);

  // Prologue normalisation (k_encode<.., kPro>, encode.h proNormalize):
  // when the encode grid is at most two generations of resident workgroups,
  // k_hist accumulates P = proRowsOf(chunks) rows per (segment, element) with
  // atomics (in the sync arena) and every encode workgroup normalises its
  // element itself, instead of a k_histReduce / k_normalize launch.  Not for
  // byte archives with a checksum (their partial checksums are summed by the
  // normalisation kernels) nor for caller-supplied histograms, and only while
  // the rows (double-buffered in the stream's arena, which never shrinks)
  // stay within kProRowsBudget.
  constexpr size_t kProRowsBudget = 32ull << 20;
  const size_t proRowsBytes = size_t(kSegs) * nb * proRowsOf(chunks) * kNumSymbols * 4;
  const bool pro = runHist && !userHist && !rawCk && MB > 0 && proRowsBytes <= kProRowsBudget &&
                   uint64_t(nb) * nW <= 2ull * residentSlots(reinterpret_cast<const void*>(&k_encode<FT, 0, true>),
                                                             enc::kThreads, 0);
  auto partHist = res.alloc<uint32_t>(s, runHist && !pro ? size_t(kSegs) * nb * chunks * kNumSymbols : 1);
  auto partCk = res.alloc<uint32_t>(s, rawCk ? size_t(nb) * chunks : 1);
  const uint32_t* chunkRows = preHist ? pre->rows : partHist.data();
  // first-level sums when elements have many chunks (k_histReduce)
  const uint32_t groups = divUp(chunks, kReduceRows);
  const bool reduce2 = (runHist || preHist) && !preNorm && !pro && chunks > kReduceRows;
  auto groupHist = res.alloc<uint32_t>(s, reduce2 ? size_t(kSegs) * nb * groups * kNumSymbols : 1);
  auto groupCk = res.alloc<uint32_t>(s, reduce2 && rawCk ? size_t(nb) * groups : 1);
  auto ck = res.alloc<uint32_t>(s, nb);
  auto tableMem = res.alloc<uint4>(s, preNorm ? 1 : size_t(kSegs) * nb * kNumSymbols);
  auto pdfMem = res.alloc<uint16_t>(s, preNorm ? 1 : size_t(kSegs) * nb * kNumSymbols);
  const uint4* table = preNorm ? pre->table : tableMem.data();
  const uint16_t* pdf = preNorm ? pre->pdf : pdfMem.data();
  auto slots = res.alloc<uint8_t>(s, size_t(kSegs) * nb * std::max(MB, 1u) * kSlotBytes);
  auto cw = res.alloc<uint32_t>(s, kFused ? 1 : size_t(kSegs) * nb * std::max(MB, 1u));
  // the normalisation runs in the last workgroup of the kernel that writes
  // an element's final partial rows (k_histReduce, or a k_hist of at most
  // 4096 workgroups), saving the k_normalize launch.  Each of those
  // workgroups pays a wait for its rows' write-through stores and a counter
  // round trip: with many (c3's k_hist: 65,536) that costs more than the
  // launch (c3 hist 0.74 -> 1.09 ms), so k_normalize runs there.
  const bool finalInReduce = reduce2;
  const bool finalInHist = !reduce2 && !pro && runHist && uint64_t(chunks) * nb <= 4096;
  // k_encode's look-back flags (one per segment, element and encode
  // workgroup, epoch-tagged, never zeroed; fp64's end as the prefixes
  // k_coalesce reads), the last-arrival counters and (pro) the histogram
  // rows, in this stream's sync arena
  const size_t regions[kSyncRegions] = {0, size_t(kSegs) * nb * nW * 8, 0, 0, size_t(nb) * kSegs * 4, 0};
  SyncLease lease(res, s, regions, false, pro ? proRowsBytes : 0);
  // fp64 (two segments): k_encode's per-segment look-back leaves each
  // workgroup's prefix in its flag for k_coalesce, whose per-workgroup sums
  // over every earlier block are otherwise quadratic in the blocks (1e8
  // words: coalesce 129 us).  Below kCoalFlagBlocks blocks per element the
  // sums are cheaper than the look-back's hand-offs (16.7M words: compress
  // +1.5 us with it).
  constexpr uint32_t kCoalFlagBlocks = 8192;
  uint64_t* const flagsFor = (kFused || MB > kCoalFlagBlocks) ? static_cast<uint64_t*>(lease.base[kSyncFlags])
                                                                : nullptr;
  NormArgs na;
  na.in = in;
  na.hist = userHist ? hist_dev : (reduce2 ? groupHist.data() : chunkRows);
  na.rows = userHist ? 1u : (reduce2 ? groups : chunks);
  na.pb = pb;
  na.table = tableMem.data();
  na.pdf = pdfMem.data();
  na.partCk = rawCk ? (reduce2 ? groupCk.data() : partCk.data()) : nullptr;
  na.ckRows = reduce2 ? groups : chunks;
  na.ckOut = ck.data();
  na.arrive = nullptr;
  NormArgs naFinal = na;
  naFinal.arrive = static_cast<uint32_t*>(lease.base[kSyncArrive]);

  if (FT != 0 && useChecksum) {
    zeroAsync(ck.data(), sizeof(uint32_t) * nb, s);
  }
  // launch groups: histogram -> (normalise) -> encode per group of elements
  // (kMallSliceBytes > 0: groups of about that many input bytes, so that the
  // encoder re-reads its input from the 256 MiB Infinity Cache; 0: one group
  // up to the grid limit)
  constexpr size_t kMallSliceBytes = 0;
  uint32_t slice = kMaxGridY;
  if (kMallSliceBytes && runHist && !pro)
    slice = uint32_t(std::max<size_t>(1, std::min<size_t>(kMaxGridY, kMallSliceBytes / std::max<size_t>(
                                                                            1, size_t(maxSize) * sizeof(typename FloatTraits<FT>::WordT)))));
  for (uint32_t y0 = 0; y0 < nb; y0 += slice) {
    const uint32_t ny = std::min(slice, nb - y0);
    if (runHist) {
      prof::Scope p("hist", s);
      dim3 g(chunks, ny);
      const NormArgs& nh = finalInHist ? naFinal : na;
      if (pro) {
        k_hist<FT, false, true><<<g, kThreads, 0, s>>>(in, y0, nb, chunkWords, chunks,
                                                       static_cast<uint32_t*>(lease.rows[0]), nullptr, na,
                                                       static_cast<uint32_t*>(lease.rows[1]));
      } else if (rawCk) {
        k_hist<FT, true><<<g, kThreads, 0, s>>>(in, y0, nb, chunkWords, chunks, partHist.data(),
                                                partCk.data(), nh);
      } else {
        k_hist<FT, false><<<g, kThreads, 0, s>>>(in, y0, nb, chunkWords, chunks, partHist.data(),
                                                 nullptr, nh);
      }
      HIP_LAUNCH_CHECK();
    }
    if (FT != 0 && useChecksum) {
      // float checksum: the reference passes float-word counts as byte counts
      // (float/GpuFloatCompress.cuh:709)
      const uint32_t ckChunk = 1u << 20;
      dim3 g(std::max(1u, divUp(maxSize, ckChunk)), ny);
      k_checksum<<<g, kThreads, 0, s>>>(in, y0, 1, ckChunk, ck.data());
      HIP_LAUNCH_CHECK();
    }
    if (reduce2) {
      prof::Scope p("normalize", s);
      dim3 g(groups, ny, kSegs);
      k_histReduce<<<g, kThreads, 0, s>>>(y0, nb, chunks, groups, chunkRows, rawCk ? partCk.data() : nullptr,
                                          groupHist.data(), rawCk ? groupCk.data() : nullptr,
                                          finalInReduce ? naFinal : na, kSegs);
      HIP_LAUNCH_CHECK();
    }
    if (!finalInReduce && !finalInHist && !preNorm && !pro) {
      prof::Scope p("normalize", s);
      dim3 g(ny, kSegs);
      k_normalize<<<g, kThreads, 0, s>>>(na, y0, nb);
      HIP_LAUNCH_CHECK();
    }
    if (MB > 0 || kFused) {
      prof::Scope p("encode", s);
      dim3 g(nW, ny);
      EncTail tail{pdf, ck.data(), outSize_dev, flagsFor, nW, pb, useChecksum, spinCap(), deviceErrorWord(),
                   sparseN};
      tail.epoch = lease.epoch;
      tail.skew = dispatchSkew();
      if (pro) {
        tail.rows = static_cast<const uint32_t*>(lease.rows[0]);
        tail.rowsPer = proRowsOf(chunks);
        tail.pdfOut = pdfMem.data();
        k_encode<FT, 0, true><<<g, enc::kThreads, 0, s>>>(in, out, y0, nb, std::max(MB, 1u), table,
                                                          slots.data(), cw.data(), tail);
      } else {
        k_encode<FT, 0><<<g, enc::kThreads, 0, s>>>(in, out, y0, nb, std::max(MB, 1u), table,
                                                 slots.data(), cw.data(), tail);
      }
      HIP_LAUNCH_CHECK();
    }
    if (!kFused) {
      prof::Scope p("coalesce", s);
      // blocks per workgroup: 4 (c4 fp64: 2,048 workgroups for the two
      // segments' 4,096 blocks each; 32 gave 256 and a latency-bound copy:
      // coalesce 28.4 -> 16 us at 8, 15.0 at 4, 19.2 at 16, same box)
      const uint32_t bpw = 4;
      dim3 g(std::max(1u, divUp(MB, bpw)), ny, kSegs);
      CoalPrefix cp;
      cp.flags = flagsFor;
      cp.nW = nW;
      cp.encBlocks = EncCfg<FT>::kBlocksPerWG;
      cp.epoch = lease.epoch;
      cp.err = deviceErrorWord();
      k_coalesce<FT><<<g, kThreads, 0, s>>>(in, out, y0, nb, std::max(MB, 1u), bpw, slots.data(),
                                            cw.data(), pdf, pb, useChecksum, ck.data(),
                                            outSize_dev, sparseN, cp);
      HIP_LAUNCH_CHECK();
    }
  }
}

template <int FT>
void decodeBatchDevice(StackDeviceMemory& res, int pb, uint32_t nb, const BatchDesc& in,
                       const BatchDesc& out, uint32_t maxCapacity, uint8_t* outSuccess_dev,
                       uint32_t* outSize_dev, hipStream_t s, const DeviceTables* tabs = nullptr,
                       bool streamOut = true, bool capacityOnly = false) {
  checkProbBits(pb);
  if (nb == 0) return;
  const uint32_t maxBlocks = divUp(maxCapacity, kBlockSize);
  auto launch = [&](auto kTag, auto ntTag) {
    constexpr int KK = decltype(kTag)::value;
    constexpr bool NT = decltype(ntTag)::value;
    using Cfg = DecCfg<FT, KK>;
    for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
      const uint32_t ny = std::min(kMaxGridY, nb - y0);
      prof::Scope p("decode", s);
      // about one generation of resident workgroups; each decodes P chunks
      // (one table build per P chunks).  P is capped at kMaxDecodeChunks:
      // large batches then run several generations, which measured faster
      // than long persistent loops (c3: 3.02 ms at P = 64, 2.31 ms at P = 8,
      // 2.60 ms at P = 1; c2's P = 2 is unaffected)
      constexpr uint32_t kMaxDecodeChunks = 8;
      const uint32_t lds = Cfg::ldsBytes(pb);
      const uint32_t chunks = std::max(1u, divUp(maxBlocks, Cfg::kBlocksPerWG));
      const uint32_t slots =
          residentSlots(reinterpret_cast<const void*>(&k_decode<FT, KK, NT, true>), dec::kThreads, lds);
      // capacityOnly: the capacity is all the host knows and may far exceed
      // the archives' sizes (the sparse codec's nonzero lists): one chunk per
      // workgroup, so the chunks that exist run side by side instead of P
      // passes of a workgroup while the grid's upper part exits at once
      // (5 x 15M fp32 at 50 % zeros: the list decode 77 -> see DESIGN)
      const uint32_t P = capacityOnly ? 1u
                                      : std::min(kMaxDecodeChunks,
                                                 std::max(1u, uint32_t((uint64_t(chunks) * ny + slots / 2) / slots)));
      dim3 g(divUp(chunks, P), ny);
      // remaining-work wave priorities balance the finish of a single
      // generation (c2 decode −2 %); across several generations they cost
      // (c3 decode 2.02 ms without, 2.32 ms with, same-box A/B).  A template
      // parameter: a runtime flag changed the step loop's code (c2 +25 %)
      if (uint64_t(g.x) * ny <= slots)
        k_decode<FT, KK, NT, true><<<g, dec::kThreads, lds, s>>>(kernargTable(tabs), in, out, y0, pb, P,
                                                                 outSuccess_dev, outSize_dev);
      else
        k_decode<FT, KK, NT, false><<<g, dec::kThreads, lds, s>>>(kernargTable(tabs), in, out, y0, pb, P,
                                                                  outSuccess_dev, outSize_dev);
      HIP_LAUNCH_CHECK();
    }
  };
  // streaming stores when nobody re-reads the output right away (fp64's
  // 8-dword rows measured slower with them)
  if constexpr (FT != 4) {
    if (streamOut) return launch(std::integral_constant<int, 0>{}, std::true_type{});
  }
  launch(std::integral_constant<int, 0>{}, std::false_type{});
}

// Verify stored checksums against `unitBytes * out.size(b)` decoded bytes
// (ansDecodeBatch :557-591 / floatDecompressDevice :1077-1112).  Host sync.
std::vector<std::pair<int, std::string>> verifyChecksums(StackDeviceMemory& res, uint32_t nb,
                                                         const BatchDesc& archivesArg, bool isFloat,
                                                         const BatchDesc& decodedArg,
                                                         uint32_t maxBytes, hipStream_t s,
                                                         const DeviceTables* tabs) {
  std::vector<std::pair<int, std::string>> errs;
  if (nb == 0) return errs;
  DeviceDescs dd(res, s, tabs, nb);
  const BatchDesc archives = dd.map(archivesArg), decoded = dd.map(decodedArg);
  auto now = res.alloc<uint32_t>(s, nb);
  auto old = res.alloc<uint32_t>(s, nb);
  zeroAsync(now.data(), sizeof(uint32_t) * nb, s);
  const uint32_t ckChunk = 1u << 20;
  for (uint32_t y0 = 0; y0 < nb; y0 += kMaxGridY) {
    const uint32_t ny = std::min(kMaxGridY, nb - y0);
    dim3 g(std::max(1u, divUp(maxBytes, ckChunk)), ny);
    k_checksum<<<g, kThreads, 0, s>>>(decoded, y0, 1, ckChunk, now.data());
    HIP_LAUNCH_CHECK();
  }
  k_info<<<divUp(nb, 128), 128, 0, s>>>(archives, nb, isFloat, nullptr, nullptr, old.data());
  HIP_LAUNCH_CHECK();
  auto a = now.copyToHost(s);
  auto o = old.copyToHost(s);
  for (uint32_t i = 0; i < nb; ++i) {
    if (a[i] != o[i]) {
      std::ostringstream e;
      e << "Checksum mismatch in batch member " << i << ": expected checksum " << std::hex << o[i]
        << " got " << a[i] << "\n";
      errs.emplace_back(int(i), e.str());
    }
  }
  return errs;
}

static bool allAligned16(const std::vector<uint64_t>& addrs) {
  for (uint64_t a : addrs)
    if (a % 16) return false;
  return true;
}

static void checkOutAligned(const void* p, const char* what) {
  DG_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0,
           what << " must be 16-byte aligned (archives are written with 16 B stores)");
}

// ---------------------------------------------------------------------------
// ANS byte codec API
// ---------------------------------------------------------------------------
uint32_t getMaxCompressedSize(uint32_t bytes) {
  // ans/GpuANSEncode.cu:13-25 (overhead term evaluated for 4096 *blocks*)
  uint64_t raw = ansOverhead(kBlockSize);
  raw += uint64_t(roundUp(kBlockSize + kBlockSize / 4, 16)) * ((uint64_t(bytes) + kBlockSize - 1) / kBlockSize);
  raw = roundUp64(raw, 16);
  DG_CHECK(raw <= uint64_t(INT32_MAX), "input too large: " << bytes << " bytes");
  return uint32_t(raw);
}

void ansEncodeBatchStride(StackDeviceMemory& res, const ANSCodecConfig& config,
                          uint32_t numInBatch, const void* in_dev, uint32_t inPerBatchSize,
                          uint32_t inPerBatchStride, const uint32_t* histogram_dev,
                          void* out_dev, uint32_t outPerBatchStride,
                          uint32_t* outBatchSize_dev, hipStream_t stream) {
  if (numInBatch == 0) return;
  checkOutAligned(out_dev, "out_dev");
  DG_CHECK(outPerBatchStride % 16 == 0, "outPerBatchStride must be a multiple of 16");
  auto in = BatchDesc::strided(in_dev, inPerBatchStride, inPerBatchSize);
  auto out = BatchDesc::strided(out_dev, outPerBatchStride, 0);
  const bool al = reinterpret_cast<uintptr_t>(in_dev) % 16 == 0 && inPerBatchStride % 16 == 0;
  encodeBatchDevice<0>(res, config.probBits, config.useChecksum, numInBatch, in, inPerBatchSize,
                       histogram_dev, out, outBatchSize_dev, stream, nullptr, al);
}

void ansEncodeBatchPointer(StackDeviceMemory& res, const ANSCodecConfig& config,
                           uint32_t numInBatch, const void** in, const uint32_t* inSize,
                           const uint32_t* histogram_dev, void** out, uint32_t* outSize_dev,
                           hipStream_t stream) {
  if (numInBatch == 0) return;
  std::vector<uint64_t> ip(numInBatch), op(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint32_t maxSize = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    op[i] = reinterpret_cast<uint64_t>(out[i]);
    checkOutAligned(out[i], "out[i]");
    sz[i] = inSize[i];
    maxSize = std::max(maxSize, inSize[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, ip, op, sz, true);
  auto inD = t.tag(BatchDesc::pointers(t.u64a, t.u32a));
  auto outD = t.tag(BatchDesc::pointers(t.u64b, nullptr));
  encodeBatchDevice<0>(res, config.probBits, config.useChecksum, numInBatch, inD, maxSize,
                       histogram_dev, outD, outSize_dev, stream, &t, allAligned16(ip));
}

void ansEncodeBatchSplitSize(StackDeviceMemory& res, const ANSCodecConfig& config,
                             uint32_t numInBatch, const void* in_dev,
                             const uint32_t* inSplitSizes, const uint32_t* histogram_dev,
                             void* out_dev, uint32_t outStride, uint32_t* outSize_dev,
                             hipStream_t stream) {
  if (numInBatch == 0) return;
  DG_CHECK(reinterpret_cast<uintptr_t>(in_dev) % kANSRequiredAlignment == 0,
           "in_dev must be " << kANSRequiredAlignment << "-byte aligned");
  checkOutAligned(out_dev, "out_dev");
  DG_CHECK(outStride % 16 == 0, "outStride must be a multiple of 16");
  std::vector<uint64_t> off(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint64_t run = 0;
  uint32_t maxSize = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    if (i + 1 != numInBatch) {
      DG_CHECK(inSplitSizes[i] % kANSRequiredAlignment == 0,
               "interior split sizes must be multiples of " << kANSRequiredAlignment);
    }
    off[i] = run;
    sz[i] = inSplitSizes[i];
    run += inSplitSizes[i];
    maxSize = std::max(maxSize, inSplitSizes[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, off, {}, sz, true);
  auto inD = t.tag(BatchDesc::split(in_dev, t.u64a, t.u32a));
  auto outD = BatchDesc::strided(out_dev, outStride, 0);
  const bool al = reinterpret_cast<uintptr_t>(in_dev) % 16 == 0 && allAligned16(off);
  encodeBatchDevice<0>(res, config.probBits, config.useChecksum, numInBatch, inD, maxSize,
                       histogram_dev, outD, outSize_dev, stream, &t, al);
}

static ANSDecodeStatus ansDecodeCommon(StackDeviceMemory& res, const ANSCodecConfig& config,
                                       uint32_t nb, const BatchDesc& in, const BatchDesc& out,
                                       uint32_t maxCap, uint8_t* succ, uint32_t* sizes,
                                       hipStream_t s, const DeviceTables* tabs = nullptr) {
  ANSDecodeStatus status;
  decodeBatchDevice<0>(res, config.probBits, nb, in, out, maxCap, succ, sizes, s, tabs, !config.useChecksum);
  if (config.useChecksum) {
    status.errorInfo = verifyChecksums(res, nb, in, false, out, maxCap, s, tabs);
    if (!status.errorInfo.empty()) status.error = ANSDecodeError::ChecksumMismatch;
  }
  return status;
}

ANSDecodeStatus ansDecodeBatchStride(StackDeviceMemory& res, const ANSCodecConfig& config,
                                     uint32_t numInBatch, const void* in_dev,
                                     uint32_t inPerBatchStride, void* out_dev,
                                     uint32_t outPerBatchStride, uint32_t outPerBatchCapacity,
                                     uint8_t* outSuccess_dev, uint32_t* outSize_dev,
                                     hipStream_t stream) {
  if (numInBatch == 0) return ANSDecodeStatus();
  auto in = BatchDesc::strided(in_dev, inPerBatchStride, 0);
  auto out = BatchDesc::strided(out_dev, outPerBatchStride, outPerBatchCapacity);
  return ansDecodeCommon(res, config, numInBatch, in, out, outPerBatchCapacity, outSuccess_dev,
                         outSize_dev, stream);
}

ANSDecodeStatus ansDecodeBatchPointer(StackDeviceMemory& res, const ANSCodecConfig& config,
                                      uint32_t numInBatch, const void** in, void** out,
                                      const uint32_t* outCapacity, uint8_t* outSuccess_dev,
                                      uint32_t* outSize_dev, hipStream_t stream) {
  if (numInBatch == 0) return ANSDecodeStatus();
  std::vector<uint64_t> ip(numInBatch), op(numInBatch);
  std::vector<uint32_t> cap(numInBatch);
  uint32_t maxCap = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    op[i] = reinterpret_cast<uint64_t>(out[i]);
    cap[i] = outCapacity[i];
    maxCap = std::max(maxCap, cap[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, ip, op, cap, true);
  auto inD = t.tag(BatchDesc::pointers(t.u64a, nullptr));
  auto outD = t.tag(BatchDesc::pointers(t.u64b, t.u32a));
  return ansDecodeCommon(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev,
                         stream, &t);
}

ANSDecodeStatus ansDecodeBatchSplitSize(StackDeviceMemory& res, const ANSCodecConfig& config,
                                        uint32_t numInBatch, const void** in, void* out_dev,
                                        const uint32_t* outSplitSizes, uint8_t* outSuccess_dev,
                                        uint32_t* outSize_dev, hipStream_t stream) {
  if (numInBatch == 0) return ANSDecodeStatus();
  DG_CHECK(reinterpret_cast<uintptr_t>(out_dev) % kANSRequiredAlignment == 0,
           "out_dev must be " << kANSRequiredAlignment << "-byte aligned");
  std::vector<uint64_t> ip(numInBatch), off(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint64_t run = 0;
  uint32_t maxCap = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    if (i + 1 != numInBatch) {
      DG_CHECK(outSplitSizes[i] % kANSRequiredAlignment == 0,
               "interior split sizes must be multiples of " << kANSRequiredAlignment);
    }
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    off[i] = run;
    sz[i] = outSplitSizes[i];
    run += outSplitSizes[i];
    maxCap = std::max(maxCap, sz[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, ip, off, sz, true);
  auto inD = t.tag(BatchDesc::pointers(t.u64a, nullptr));
  auto outD = t.tag(BatchDesc::split(out_dev, t.u64b, t.u32a));
  return ansDecodeCommon(res, config, numInBatch, inD, outD, maxCap, outSuccess_dev, outSize_dev,
                         stream, &t);
}

void ansGetCompressedInfoDevice(StackDeviceMemory& res, const void** in_dev, uint32_t numInBatch,
                                uint32_t* outSizes_dev, uint32_t* outChecksum_dev,
                                hipStream_t stream) {
  if (numInBatch == 0 || (!outSizes_dev && !outChecksum_dev)) return;
  auto inD = BatchDesc::pointers(reinterpret_cast<const uint64_t*>(in_dev), nullptr);
  k_info<<<divUp(numInBatch, 128), 128, 0, stream>>>(inD, numInBatch, false, outSizes_dev,
                                                      nullptr, outChecksum_dev);
  HIP_LAUNCH_CHECK();
}

void ansGetCompressedInfo(StackDeviceMemory& res, const void** in, uint32_t numInBatch,
                          uint32_t* outSizes_dev, uint32_t* outChecksum_dev, hipStream_t stream) {
  if (numInBatch == 0 || (!outSizes_dev && !outChecksum_dev)) return;
  std::vector<uint64_t> ip(numInBatch);
  for (uint32_t i = 0; i < numInBatch; ++i) ip[i] = reinterpret_cast<uint64_t>(in[i]);
  auto t = uploadTables(res, stream, numInBatch, ip, {}, {});
  ansGetCompressedInfoDevice(res, reinterpret_cast<const void**>(const_cast<uint64_t*>(t.u64a)),
                             numInBatch, outSizes_dev, outChecksum_dev, stream);
}

// ---------------------------------------------------------------------------
// float codec API
// ---------------------------------------------------------------------------
// float/GpuFloatCompress.cu:23-47.  The result is a u32 there too and may
// exceed INT32_MAX (the reference's published batch-1 sweep compresses
// 1.07e9 bf16 words, README.md:118: 2.41e9 bytes of capacity); every archive
// offset is unsigned 32-bit, so anything up to UINT32_MAX is accepted.  The
// raw section is sized in 64 bits here so that an fp32 / fp64 size past the
// u32 range is refused instead of wrapping.
uint32_t getMaxFloatCompressedSize(FloatType ft, uint32_t size) {
  DG_CHECK(ft != FloatType::kUndefined && uint32_t(ft) <= 4, "bad float type");
  const uint64_t n8 = roundUp64(size, 8), n16 = roundUp64(size, 16);
  const uint64_t raw = ft == FloatType::kFloat32 ? 2 * n8 + n16
                       : ft == FloatType::kFloat64 ? 4 * roundUp64(size, 4) + 2 * n8 : n16;
  uint64_t base = 32ull + getMaxCompressedSize(size) + raw;
  if (ft == FloatType::kFloat64) base += getMaxCompressedSize(size);
  DG_CHECK(base <= uint64_t(UINT32_MAX), "input too large: " << size << " float words");
  return uint32_t(base);
}

static void checkFloatConfig(const FloatCodecConfig& c) {
  DG_CHECK(!c.ansConfig.useChecksum,
           "ANS-level checksumming is not allowed in float mode (use FloatCodecConfig.useChecksum)");
  DG_CHECK(c.floatType != FloatType::kUndefined && uint32_t(c.floatType) <= 4, "bad float type");
}

void floatCompressDescs(StackDeviceMemory& res, const FloatCompressConfig& config, uint32_t nb,
                        const BatchDesc& in, uint32_t maxSize, const BatchDesc& out,
                        uint32_t* outSize_dev, hipStream_t s, const DeviceTables* tabs,
                        bool inAligned16, const PartialHist* pre, const uint32_t* sparseN) {
  checkFloatConfig(config);
  const int pb = config.ansConfig.probBits;
  switch (config.floatType) {
    case FloatType::kFloat16:
      encodeBatchDevice<1>(res, pb, config.useChecksum, nb, in, maxSize, nullptr, out, outSize_dev, s,
                             tabs, inAligned16, pre, sparseN);
      break;
    case FloatType::kBFloat16:
      encodeBatchDevice<2>(res, pb, config.useChecksum, nb, in, maxSize, nullptr, out, outSize_dev, s,
                             tabs, inAligned16, pre, sparseN);
      break;
    case FloatType::kFloat32:
      encodeBatchDevice<3>(res, pb, config.useChecksum, nb, in, maxSize, nullptr, out, outSize_dev, s,
                             tabs, inAligned16, pre, sparseN);
      break;
    default:
      encodeBatchDevice<4>(res, pb, config.useChecksum, nb, in, maxSize, nullptr, out, outSize_dev, s,
                             tabs, inAligned16, pre, sparseN);
      break;
  }
}

FloatDecompressStatus floatDecompressDescs(StackDeviceMemory& res,
                                           const FloatDecompressConfig& config, uint32_t nb,
                                           const BatchDesc& in, const BatchDesc& out,
                                           uint32_t maxCap, uint8_t* succ, uint32_t* sizes,
                                           hipStream_t s, const DeviceTables* tabs, bool streamOut,
                                           bool capacityOnly) {
  checkFloatConfig(config);
  const int pb = config.ansConfig.probBits;
  // streaming output stores unless the output is read back (checksum)
  const bool nt = streamOut && !config.useChecksum;
  switch (config.floatType) {
    case FloatType::kFloat16:
      decodeBatchDevice<1>(res, pb, nb, in, out, maxCap, succ, sizes, s, tabs, nt, capacityOnly);
      break;
    case FloatType::kBFloat16:
      decodeBatchDevice<2>(res, pb, nb, in, out, maxCap, succ, sizes, s, tabs, nt, capacityOnly);
      break;
    case FloatType::kFloat32:
      decodeBatchDevice<3>(res, pb, nb, in, out, maxCap, succ, sizes, s, tabs, nt, capacityOnly);
      break;
    default:
      decodeBatchDevice<4>(res, pb, nb, in, out, maxCap, succ, sizes, s, tabs, nt, capacityOnly);
      break;
  }
  FloatDecompressStatus status;
  if (config.useChecksum) {
    // checksums `capacity` bytes (float words treated as bytes), as the
    // reference does (float/GpuFloatDecompress.cuh:1077-1112)
    status.errorInfo = verifyChecksums(res, nb, in, true, out, maxCap, s, tabs);
    if (!status.errorInfo.empty()) status.error = FloatDecompressError::ChecksumMismatch;
  }
  return status;
}

void floatCompress(StackDeviceMemory& res, const FloatCompressConfig& config, uint32_t numInBatch,
                   const void** in, const uint32_t* inSize, void** out, uint32_t* outSize_dev,
                   hipStream_t stream) {
  if (numInBatch == 0) return;
  checkFloatConfig(config);
  const uint32_t ws = floatWordBytes(int(config.floatType));
  std::vector<uint64_t> ip(numInBatch), op(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint32_t maxSize = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    op[i] = reinterpret_cast<uint64_t>(out[i]);
    DG_CHECK(ip[i] % ws == 0, "float input " << i << " not aligned to its word size");
    checkOutAligned(out[i], "out[i]");
    sz[i] = inSize[i];
    maxSize = std::max(maxSize, inSize[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, ip, op, sz, true);
  floatCompressDescs(res, config, numInBatch, t.tag(BatchDesc::pointers(t.u64a, t.u32a)), maxSize,
                     t.tag(BatchDesc::pointers(t.u64b, nullptr)), outSize_dev, stream, &t,
                     allAligned16(ip));
}

void floatCompressSplitSize(StackDeviceMemory& res, const FloatCompressConfig& config,
                            uint32_t numInBatch, const void* in_dev, const uint32_t* inSplitSizes,
                            void* out_dev, uint32_t outStride, uint32_t* outSize_dev,
                            hipStream_t stream) {
  if (numInBatch == 0) return;
  checkFloatConfig(config);
  checkOutAligned(out_dev, "out_dev");
  DG_CHECK(outStride % 16 == 0, "outStride must be a multiple of 16");
  const uint32_t ws = floatWordBytes(int(config.floatType));
  DG_CHECK(reinterpret_cast<uintptr_t>(in_dev) % ws == 0, "in_dev not word aligned");
  std::vector<uint64_t> off(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint64_t run = 0;
  uint32_t maxSize = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    off[i] = run * ws;
    sz[i] = inSplitSizes[i];
    run += inSplitSizes[i];
    maxSize = std::max(maxSize, sz[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, off, {}, sz, true);
  floatCompressDescs(res, config, numInBatch, t.tag(BatchDesc::split(in_dev, t.u64a, t.u32a)),
                     maxSize, BatchDesc::strided(out_dev, outStride, 0), outSize_dev, stream, &t,
                     reinterpret_cast<uintptr_t>(in_dev) % 16 == 0 && allAligned16(off));
}

void floatCompressBatchStride(StackDeviceMemory& res, const FloatCompressConfig& config,
                              uint32_t numInBatch, const void* in_dev, uint32_t inPerBatchWords,
                              uint64_t inPerBatchStrideBytes, void* out_dev,
                              uint64_t outPerBatchStrideBytes, uint32_t* outSize_dev,
                              hipStream_t stream) {
  if (numInBatch == 0) return;
  checkOutAligned(out_dev, "out_dev");
  DG_CHECK(outPerBatchStrideBytes % 16 == 0, "out stride must be a multiple of 16");
  floatCompressDescs(res, config, numInBatch,
                     BatchDesc::strided(in_dev, inPerBatchStrideBytes, inPerBatchWords),
                     inPerBatchWords, BatchDesc::strided(out_dev, outPerBatchStrideBytes, 0),
                     outSize_dev, stream, nullptr,
                     reinterpret_cast<uintptr_t>(in_dev) % 16 == 0 && inPerBatchStrideBytes % 16 == 0);
}

FloatDecompressStatus floatDecompress(StackDeviceMemory& res, const FloatDecompressConfig& config,
                                      uint32_t numInBatch, const void** in, void** out,
                                      const uint32_t* outCapacity, uint8_t* outSuccess_dev,
                                      uint32_t* outSize_dev, hipStream_t stream) {
  if (numInBatch == 0) return FloatDecompressStatus();
  checkFloatConfig(config);
  const uint32_t ws = floatWordBytes(int(config.floatType));
  std::vector<uint64_t> ip(numInBatch), op(numInBatch);
  std::vector<uint32_t> cap(numInBatch);
  uint32_t maxCap = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    op[i] = reinterpret_cast<uint64_t>(out[i]);
    DG_CHECK(op[i] % ws == 0, "float output " << i << " not aligned to its word size");
    cap[i] = outCapacity[i];
    maxCap = std::max(maxCap, cap[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, ip, op, cap, true);
  return floatDecompressDescs(res, config, numInBatch, t.tag(BatchDesc::pointers(t.u64a, nullptr)),
                              t.tag(BatchDesc::pointers(t.u64b, t.u32a)), maxCap, outSuccess_dev,
                              outSize_dev, stream, &t);
}

FloatDecompressStatus floatDecompressSplitSize(StackDeviceMemory& res,
                                               const FloatDecompressConfig& config,
                                               uint32_t numInBatch, const void** in, void* out_dev,
                                               const uint32_t* outSplitSizes,
                                               uint8_t* outSuccess_dev, uint32_t* outSize_dev,
                                               hipStream_t stream) {
  if (numInBatch == 0) return FloatDecompressStatus();
  checkFloatConfig(config);
  const uint32_t ws = floatWordBytes(int(config.floatType));
  DG_CHECK(reinterpret_cast<uintptr_t>(out_dev) % ws == 0, "out_dev not word aligned");
  std::vector<uint64_t> ip(numInBatch), off(numInBatch);
  std::vector<uint32_t> sz(numInBatch);
  uint64_t run = 0;
  uint32_t maxCap = 0;
  for (uint32_t i = 0; i < numInBatch; ++i) {
    ip[i] = reinterpret_cast<uint64_t>(in[i]);
    off[i] = run * ws;
    sz[i] = outSplitSizes[i];
    run += outSplitSizes[i];
    maxCap = std::max(maxCap, sz[i]);
  }
  auto t = uploadTables(res, stream, numInBatch, ip, off, sz, true);
  return floatDecompressDescs(res, config, numInBatch, t.tag(BatchDesc::pointers(t.u64a, nullptr)),
                              t.tag(BatchDesc::split(out_dev, t.u64b, t.u32a)), maxCap,
                              outSuccess_dev, outSize_dev, stream, &t);
}

FloatDecompressStatus floatDecompressBatchStride(StackDeviceMemory& res,
                                                 const FloatDecompressConfig& config,
                                                 uint32_t numInBatch, const void* in_dev,
                                                 uint64_t inPerBatchStrideBytes, void* out_dev,
                                                 uint64_t outPerBatchStrideBytes,
                                                 uint32_t outPerBatchCapacityWords,
                                                 uint8_t* outSuccess_dev, uint32_t* outSize_dev,
                                                 hipStream_t stream) {
  if (numInBatch == 0) return FloatDecompressStatus();
  return floatDecompressDescs(
      res, config, numInBatch, BatchDesc::strided(in_dev, inPerBatchStrideBytes, 0),
      BatchDesc::strided(out_dev, outPerBatchStrideBytes, outPerBatchCapacityWords),
      outPerBatchCapacityWords, outSuccess_dev, outSize_dev, stream);
}

void floatGetCompressedInfoDevice(StackDeviceMemory& res, const void** in_dev, uint32_t numInBatch,
                                  uint32_t* outSizes_dev, uint32_t* outTypes_dev,
                                  uint32_t* outChecksum_dev, hipStream_t stream) {
  if (numInBatch == 0 || (!outSizes_dev && !outTypes_dev && !outChecksum_dev)) return;
  auto inD = BatchDesc::pointers(reinterpret_cast<const uint64_t*>(in_dev), nullptr);
  k_info<<<divUp(numInBatch, 128), 128, 0, stream>>>(inD, numInBatch, true, outSizes_dev,
                                                      outTypes_dev, outChecksum_dev);
  HIP_LAUNCH_CHECK();
}

void floatGetCompressedInfo(StackDeviceMemory& res, const void** in, uint32_t numInBatch,
                            uint32_t* outSizes_dev, uint32_t* outTypes_dev,
                            uint32_t* outChecksum_dev, hipStream_t stream) {
  if (numInBatch == 0 || (!outSizes_dev && !outTypes_dev && !outChecksum_dev)) return;
  std::vector<uint64_t> ip(numInBatch);
  for (uint32_t i = 0; i < numInBatch; ++i) ip[i] = reinterpret_cast<uint64_t>(in[i]);
  auto t = uploadTables(res, stream, numInBatch, ip, {}, {});
  floatGetCompressedInfoDevice(res, reinterpret_cast<const void**>(const_cast<uint64_t*>(t.u64a)),
                               numInBatch, outSizes_dev, outTypes_dev, outChecksum_dev, stream);
}

}  // namespace dietgpu
