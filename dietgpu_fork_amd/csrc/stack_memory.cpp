// LIFO device arena + pinned H2D staging ring.
// Semantics follow dietgpu/utils/StackDeviceMemory.cpp:34-250 (LIFO frees,
// overflow to hipMalloc with a warning, high-water mark).
#include "dietgpu/StackDeviceMemory.h"

#include <algorithm>
#include <cstring>
#include <deque>
#include <iostream>
#include <mutex>
#include <sstream>

#include "common.h"

namespace dietgpu {

StackDeviceMemory::StackDeviceMemory(int device, size_t bytes) : device_(device) {
  if (bytes) {
    bytes = std::max(bytes, kSDMAlignment);
    int prev = 0;
    HIP_CHECK(hipGetDevice(&prev));
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&owned_), bytes));
    HIP_CHECK(hipSetDevice(prev));
    start_ = owned_;
    head_ = start_;
    end_ = owned_ + bytes;
  }
}

StackDeviceMemory::StackDeviceMemory(int device, void* p, size_t bytes)
    : device_(device) {
  DG_CHECK(p || bytes == 0, "null temp memory with nonzero size");
  if (p && bytes >= kSDMAlignment) {
    // the managed region must start 256-byte aligned; trim the front if not
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    uintptr_t aligned = (a + kSDMAlignment - 1) / kSDMAlignment * kSDMAlignment;
    size_t lost = aligned - a;
    if (bytes > lost) {
      start_ = reinterpret_cast<char*>(aligned);
      head_ = start_;
      end_ = start_ + (bytes - lost) / kSDMAlignment * kSDMAlignment;
    }
  }
}

StackDeviceMemory::~StackDeviceMemory() {
  for (auto& kv : overflow_) {
    (void)hipFree(kv.first);
  }
  if (owned_) {
    (void)hipFree(owned_);
  }
}

void* StackDeviceMemory::allocPointer(hipStream_t stream, size_t bytes, AllocType type) {
  DG_CHECK(bytes >= kSDMAlignment && bytes % kSDMAlignment == 0, "bad size " << bytes);
  void* out = nullptr;
  size_t used = size_t(head_ - start_);
  if (type == AllocType::Permanent || bytes > getSizeAvailable()) {
    // the reference warns on every overflow; we warn once per arena
    if (type == AllocType::Temporary && !warned_) {
      warned_ = true;
      std::cerr << "WARNING: StackDeviceMemory: attempting to allocate " << bytes
                << " bytes with " << getSizeAvailable()
                << " bytes available; calling hipMalloc. Resize temp memory to >= "
                << std::max(maxSeen_, used + overflowBytes_ + bytes)
                << " bytes to avoid performance problems.\n";
    }
    int prev = 0;
    HIP_CHECK(hipGetDevice(&prev));
    HIP_CHECK(hipSetDevice(device_));
    hipError_t e = hipMalloc(&out, bytes);
    HIP_CHECK(hipSetDevice(prev));
    HIP_CHECK(e);
    overflow_[out] = bytes;
    overflowBytes_ += bytes;
  } else {
    out = head_;
    head_ += bytes;
    used += bytes;
  }
  maxSeen_ = std::max(maxSeen_, used + overflowBytes_);
  return out;
}

void StackDeviceMemory::deallocPointer(int device, hipStream_t stream, size_t bytes, void* p) {
  DG_CHECK(p, "null free");
  DG_CHECK(device == device_, "device mismatch");
  auto it = overflow_.find(p);
  if (it != overflow_.end()) {
    DG_CHECK(it->second == bytes, "overflow size mismatch");
    // the block may still be in use by work queued on `stream`
    (void)hipStreamSynchronize(stream);
    (void)hipFree(p);
    overflowBytes_ -= bytes;
    overflow_.erase(it);
    return;
  }
  char* pc = static_cast<char*>(p);
  DG_CHECK(pc >= start_ && pc < end_, "pointer not owned by this arena");
  DG_CHECK(pc + bytes == head_, "allocations must be freed in LIFO order");
  head_ = pc;
}

std::string StackDeviceMemory::toString() const {
  std::ostringstream s;
  s << "SDM device " << device_ << ": total " << getSizeTotal() << " B, available "
    << getSizeAvailable() << " B, max seen " << maxSeen_ << " B, overflow "
    << overflowBytes_ << " B";
  return s.str();
}

// ---------------------------------------------------------------------------
// pinned staging ring for host->device parameter tables
// ---------------------------------------------------------------------------
namespace {
struct StagingRing {
  static constexpr size_t kBytes = 8u << 20;
  struct Use {
    size_t off, bytes;
    hipEvent_t ev;
  };
  std::mutex mu;
  char* host = nullptr;
  size_t head = 0;
  std::deque<Use> inflight;
  std::vector<hipEvent_t> freeEvents;

  hipEvent_t getEvent() {
    if (!freeEvents.empty()) {
      auto e = freeEvents.back();
      freeEvents.pop_back();
      return e;
    }
    hipEvent_t e;
    // completion of the copy is all the ring needs: no system-scope fence
    // (it would write back and invalidate L2 at every upload)
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    return e;
  }
  // Uses are allocated in address order around the ring, so the oldest use is
  // the only one the new region [off, off+bytes) can run into first.
  void retireOverlapping(size_t off, size_t bytes) {
    while (!inflight.empty()) {
      auto& u = inflight.front();
      bool overlap = u.off < off + bytes && off < u.off + u.bytes;
      if (overlap) {
        HIP_CHECK(hipEventSynchronize(u.ev));
      } else if (hipEventQuery(u.ev) != hipSuccess) {
        break;
      }
      freeEvents.push_back(u.ev);
      inflight.pop_front();
    }
  }
};
StagingRing& ring() {
  static StagingRing r;
  return r;
}
} // namespace

bool uploadViaKernargs(void* dst, const void* src, size_t bytes, hipStream_t s);  // upload.hip

void StackDeviceMemory::copyToDevice(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return;
  if (uploadViaKernargs(dst, src, bytes, s)) return;  // tables up to 64 KB: no blit
  auto& r = ring();
  if (bytes > StagingRing::kBytes / 4) {
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return;
  }
  std::lock_guard<std::mutex> g(r.mu);
  if (!r.host) {
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&r.host), StagingRing::kBytes,
                            hipHostMallocDefault));
  }
  size_t n = (bytes + 255) / 256 * 256;
  if (r.head + n > StagingRing::kBytes) r.head = 0;
  size_t off = r.head;
  r.retireOverlapping(off, n);
  std::memcpy(r.host + off, src, bytes);
  HIP_CHECK(hipMemcpyAsync(dst, r.host + off, bytes, hipMemcpyHostToDevice, s));
  hipEvent_t ev = r.getEvent();
  HIP_CHECK(hipEventRecord(ev, s));
  r.inflight.push_back({off, n, ev});
  r.head = off + n;
}

StackDeviceMemory makeStackMemory(size_t bytes) {
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  return StackDeviceMemory(dev, bytes);
}

} // namespace dietgpu
