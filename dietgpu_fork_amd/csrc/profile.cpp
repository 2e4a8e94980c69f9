#include "profile.h"

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace dietgpu {
namespace prof {

namespace {
struct Family {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  double totalMs = 0;
  uint64_t launches = 0;
};
std::atomic<bool> gEnabled{false};
std::mutex gMu;
std::string gFilter;  // guarded by gMu
std::map<std::string, Family>& families() {
  static std::map<std::string, Family> m;
  return m;
}
std::vector<hipEvent_t>& eventPool() {
  static std::vector<hipEvent_t> p;
  return p;
}
hipEvent_t getEvent() {
  auto& p = eventPool();
  if (!p.empty()) {
    hipEvent_t e = p.back();
    p.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing only: skip the system-scope fence (an L2 writeback per record)
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}
void drain(Family& f) {
  for (auto& pr : f.pending) {
    float ms = 0;
    (void)hipEventSynchronize(pr.second);
    if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) f.totalMs += ms;
    eventPool().push_back(pr.first);
    eventPool().push_back(pr.second);
  }
  f.pending.clear();
}
}  // namespace

bool enabled() { return gEnabled.load(std::memory_order_relaxed); }
void setEnabled(bool on) { gEnabled.store(on); }
void setFilter(const char* family) {
  std::lock_guard<std::mutex> g(gMu);
  gFilter = family ? family : "";
}

void reset() {
  std::lock_guard<std::mutex> g(gMu);
  for (auto& kv : families()) {
    drain(kv.second);
    kv.second.totalMs = 0;
    kv.second.launches = 0;
  }
}

bool query(const char* family, double* totalMs, uint64_t* launches) {
  std::lock_guard<std::mutex> g(gMu);
  auto it = families().find(family);
  if (it == families().end()) {
    if (totalMs) *totalMs = 0;
    if (launches) *launches = 0;
    return false;
  }
  drain(it->second);
  if (totalMs) *totalMs = it->second.totalMs;
  if (launches) *launches = it->second.launches;
  return true;
}

Scope::Scope(const char* family, hipStream_t s) : family_(family), stream_(s) {
  if (!enabled()) return;
  std::lock_guard<std::mutex> g(gMu);
  if (!gFilter.empty() && gFilter != family) return;
  start_ = getEvent();
  (void)hipEventRecord(start_, stream_);
}

Scope::~Scope() {
  if (!start_) return;
  std::lock_guard<std::mutex> g(gMu);
  hipEvent_t stop = getEvent();
  (void)hipEventRecord(stop, stream_);
  auto& f = families()[family_];
  f.pending.emplace_back(start_, stop);
  f.launches += 1;
}

}  // namespace prof
}  // namespace dietgpu
