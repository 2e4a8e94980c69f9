// Optional per-kernel-family hipEvent timing (used by bench.py to price the
// dominant kernel against the HBM roofline).  Disabled by default: a disabled
// Scope costs one relaxed atomic load.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dietgpu {
namespace prof {

bool enabled();
void setEnabled(bool on);
// Restrict recording to one kernel family (nullptr / "" = all families), so a
// timed region can price its dominant kernel without an event pair around
// every launch of the call.
void setFilter(const char* family);
void reset();
// Returns false if the family has never been recorded.
bool query(const char* family, double* totalMs, uint64_t* launches);

class Scope {
 public:
  Scope(const char* family, hipStream_t s);
  ~Scope();
  Scope(const Scope&) = delete;
  Scope& operator=(const Scope&) = delete;

 private:
  const char* family_;
  hipStream_t stream_;
  hipEvent_t start_ = nullptr;
};

}  // namespace prof
}  // namespace dietgpu
