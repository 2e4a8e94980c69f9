// Per-(device, stream) flag arenas for k_compress (see sync_arena.h).
#include "sync_arena.h"

#include <map>
#include <memory>
#include <utility>

#include "common.h"

namespace dietgpu {

namespace {
struct Arena {
  std::mutex m;
  void* ptr = nullptr;
  size_t bytes = 0;
  uint32_t epoch = 0;
};

std::mutex gMapMutex;
std::map<std::pair<int, hipStream_t>, std::unique_ptr<Arena>>& arenas() {
  static auto* m = new std::map<std::pair<int, hipStream_t>, std::unique_ptr<Arena>>();
  return *m;  // never destroyed: the runtime may be gone at exit
}
}  // namespace

SyncLease::SyncLease(hipStream_t stream, size_t bytes) {
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  Arena* a;
  {
    std::lock_guard<std::mutex> g(gMapMutex);
    auto& slot = arenas()[{dev, stream}];
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
  if (a->epoch == 0) {  // wrapped: flags of every older epoch must go
    a->epoch = 1;
    zero = true;
  }
  if (zero) HIP_CHECK(hipMemsetAsync(a->ptr, 0, a->bytes, stream));
  base = a->ptr;
  epoch = a->epoch;
}

}  // namespace dietgpu
