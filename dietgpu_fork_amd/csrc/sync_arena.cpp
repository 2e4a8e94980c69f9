// Per-(device, stream) sync arenas of the compressors (k_pcompress, k_encode;
// see sync_arena.h).
#include "sync_arena.h"

#include <algorithm>
#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <thread>
#include <tuple>

#include "common.h"

namespace dietgpu {

namespace {

struct Arena {
  std::mutex m;
  void* ptr[kSyncRegions] = {};
  size_t bytes[kSyncRegions] = {};
  uint32_t epoch = 0;
  // k_pcompress's two dequeue counters (kSyncCounters, u64 each): bit k set
  // while counter k may hold an earlier call's count.  A k_pcompress call at
  // epoch e uses counter e & 1 and zeroes counter (e + 1) & 1 for the next
  // call; a call in between that does not run k_pcompress (the three-kernel
  // path) still takes an epoch, so the counter a later k_pcompress call uses
  // can be the dirty one: it is then zeroed here, stream-ordered.
  uint32_t ctrDirty = 0;
  // kSyncRows: bytes at the start of row buffer k (the region's halves)
  // known to be zero
  size_t rowsClean[2] = {0, 0};
};

using Key = std::tuple<int, hipStream_t, size_t>;
std::mutex gMapMutex;
std::map<Key, std::unique_ptr<Arena>>& arenas() {
  static auto* m = new std::map<Key, std::unique_ptr<Arena>>();
  return *m;  // never destroyed: the runtime may be gone at exit
}

std::atomic<uint32_t> gSpinCap{1u << 24};
std::atomic<uint32_t> gBarrierBudget{20000};
std::atomic<uint32_t> gDispatchSkew{0};
}  // namespace

void setSpinCap(uint32_t polls) { gSpinCap.store(polls); }
uint32_t spinCap() { return gSpinCap.load(); }
void setBarrierBudget(uint32_t ticks) { gBarrierBudget.store(ticks); }
uint32_t barrierBudgetTicks() { return gBarrierBudget.load(); }
void setDispatchSkew(uint32_t ticks) { gDispatchSkew.store(ticks); }
uint32_t dispatchSkew() { return gDispatchSkew.load(); }
std::atomic<int> gCompressPath{0};
void setCompressPath(int mode) { gCompressPath.store(mode); }
int compressPath() { return gCompressPath.load(); }

SyncLease::SyncLease(StackDeviceMemory& res, hipStream_t stream, const size_t (&bytesIn)[kSyncRegions],
                     bool dequeue, size_t rowsBytes) {
  size_t bytes[kSyncRegions];
  for (int k = 0; k < kSyncRegions; ++k) bytes[k] = bytesIn[k];
  bytes[kSyncCounters] = std::max(bytes[kSyncCounters], kSyncCounterBytes);
  rowsBytes = roundUp64(rowsBytes, 256);
  bytes[kSyncRows] = 2 * rowsBytes;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_CHECK(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone) {
    // graph capture: per-call state from the caller's arena, zeroed by a
    // captured zeroing kernel (zeroAsync) on every replay
    capturing = true;
    size_t total = 0;
    for (int k = 0; k < kSyncRegions; ++k) total += roundUp64(std::max<size_t>(bytes[k], 8), 256);
    capMem_ = res.alloc<uint8_t>(stream, total);
    zeroAsync(capMem_.data(), total, stream);
    size_t off = 0;
    for (int k = 0; k < kSyncRegions; ++k) {
      base[k] = capMem_.data() + off;
      off += roundUp64(std::max<size_t>(bytes[k], 8), 256);
    }
    epoch = 1;
    rows[0] = base[kSyncRows];
    rows[1] = static_cast<uint8_t*>(base[kSyncRows]) + rowsBytes;
    return;
  }
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  const size_t tkey = stream == hipStreamPerThread ? std::hash<std::thread::id>()(std::this_thread::get_id()) : 0;
  Arena* a;
  {
    std::lock_guard<std::mutex> g(gMapMutex);
    auto& slot = arenas()[Key{dev, stream, tkey}];
    if (!slot) slot.reset(new Arena());
    a = slot.get();
  }
  lock_ = std::unique_lock<std::mutex>(a->m);
  bool grow = false;
  for (int k = 0; k < kSyncRegions; ++k) grow = grow || a->bytes[k] < bytes[k];
  if (grow) {
    // earlier calls may still read the regions being replaced
    HIP_CHECK(hipStreamSynchronize(stream));
    for (int k = 0; k < kSyncRegions; ++k) {
      if (a->bytes[k] >= bytes[k] && a->ptr[k]) continue;
      size_t want = std::max<size_t>(64 << 10, a->bytes[k]);
      while (want < bytes[k]) want *= 2;
      if (a->ptr[k]) HIP_CHECK(hipFree(a->ptr[k]));
      HIP_CHECK(hipMalloc(&a->ptr[k], want));
      zeroAsync(a->ptr[k], want, stream);
      a->bytes[k] = want;
      if (k == kSyncCounters) a->ctrDirty = 0;
      if (k == kSyncRows) a->rowsClean[0] = a->rowsClean[1] = want / 2;
    }
  }
  a->epoch = (a->epoch + 1) & kEpochMask;
  if (a->epoch == 0) {  // wrapped: words of every older epoch must go
    for (int k = 0; k < kSyncRegions; ++k) zeroAsync(a->ptr[k], a->bytes[k], stream);
    a->epoch = 1;
    a->ctrDirty = 0;
    a->rowsClean[0] = a->rowsClean[1] = a->bytes[kSyncRows] / 2;
  }
  if (dequeue) {  // a k_pcompress call: its counter must start at zero
    const uint32_t mine = a->epoch & 1u;
    if (a->ctrDirty & (1u << mine))
      zeroAsync(static_cast<uint64_t*>(a->ptr[kSyncCounters]) + mine, sizeof(uint64_t), stream);
    a->ctrDirty = 1u << mine;  // the kernel zeroes the other one
  }
  for (int k = 0; k < kSyncRegions; ++k) base[k] = a->ptr[k];
  epoch = a->epoch;
  if (rowsBytes) {
    // the buffer already zeroed (by the previous such call) if there is one,
    // else buffer epoch & 1; the other one is zeroed for the next call
    uint32_t mine = a->epoch & 1u;
    if (a->rowsClean[mine] < rowsBytes && a->rowsClean[mine ^ 1u] >= rowsBytes) mine ^= 1u;
    const size_t half = a->bytes[kSyncRows] / 2;
    rows[0] = static_cast<uint8_t*>(a->ptr[kSyncRows]) + mine * half;
    rows[1] = static_cast<uint8_t*>(a->ptr[kSyncRows]) + (mine ^ 1u) * half;
    if (a->rowsClean[mine] < rowsBytes) zeroAsync(rows[0], rowsBytes, stream);
    a->rowsClean[mine] = 0;            // accumulated into by this call
    a->rowsClean[mine ^ 1u] = rowsBytes;  // zeroed by this call's k_hist
  }
}

}  // namespace dietgpu
