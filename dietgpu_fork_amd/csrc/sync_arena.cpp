// Per-(device, stream) flag arenas for k_compress (see sync_arena.h).
#include "sync_arena.h"

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
  void* ptr = nullptr;
  size_t bytes = 0;
  uint32_t epoch = 0;
};

using Key = std::tuple<int, hipStream_t, size_t>;
std::mutex gMapMutex;
std::map<Key, std::unique_ptr<Arena>>& arenas() {
  static auto* m = new std::map<Key, std::unique_ptr<Arena>>();
  return *m;  // never destroyed: the runtime may be gone at exit
}

std::atomic<uint32_t> gSpinCap{1u << 24};
}  // namespace

void setSpinCap(uint32_t polls) { gSpinCap.store(polls); }
uint32_t spinCap() { return gSpinCap.load(); }

SyncLease::SyncLease(StackDeviceMemory& res, hipStream_t stream, size_t bytes) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_CHECK(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone) {
    // graph capture: per-call state from the caller's arena, zeroed by a
    // captured memset on every replay
    capturing = true;
    capMem_ = res.alloc<uint8_t>(stream, bytes);
    HIP_CHECK(hipMemsetAsync(capMem_.data(), 0, bytes, stream));
    base = capMem_.data();
    epoch = 1;
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
  bool zero = false;
  if (a->bytes < bytes) {
    size_t want = std::max<size_t>(64 << 10, a->bytes);
    while (want < bytes) want *= 2;
    if (a->ptr) {
      HIP_CHECK(hipStreamSynchronize(stream));  // earlier calls may still read it
      HIP_CHECK(hipFree(a->ptr));
    }
    HIP_CHECK(hipMalloc(&a->ptr, want));
    a->bytes = want;
    zero = true;
  }
  a->epoch = (a->epoch + 1) & kEpochMask;
  if (a->epoch == 0) zero = true;  // wrapped: flags of every older epoch must go
  if (zero) {
    HIP_CHECK(hipMemsetAsync(a->ptr, 0, a->bytes, stream));
    a->epoch = 1;
  }
  base = a->ptr;
  epoch = a->epoch;
}

}  // namespace dietgpu
