// Persistent per-(device, stream) device memory for k_compress's
// cross-workgroup flags (team arrivals, look-back prefixes).
//
// The flags carry a per-call epoch instead of being zeroed before every call:
// a flag counts only if its epoch is the current call's, so stale values from
// earlier calls are simply ignored and no memset launch precedes k_compress.
// Calls on one stream are serial, so one arena per (device, stream) keeps
// concurrent calls on different streams apart; the lease holds the arena's
// lock from epoch assignment to kernel launch, so host threads sharing a
// stream enqueue epochs in order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>

namespace dietgpu {

constexpr uint32_t kEpochMask = 0x3fffffffu;  // 30-bit epochs (flag bits 61:32)

class SyncLease {
 public:
  // A zero-initialised-at-creation region of >= bytes for the current device
  // and `stream`, and this call's epoch (1 .. kEpochMask).
  SyncLease(hipStream_t stream, size_t bytes);
  SyncLease(const SyncLease&) = delete;
  SyncLease& operator=(const SyncLease&) = delete;

  void* base = nullptr;
  uint32_t epoch = 0;

 private:
  std::unique_lock<std::mutex> lock_;
};

}  // namespace dietgpu
