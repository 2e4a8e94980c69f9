// LIFO device-memory arena used for every temporary of the codec.
//
// Replaces dietgpu/utils/StackDeviceMemory.h:23-298 (same class / method
// names and semantics: 256-byte granules, Temporary vs Permanent, LIFO frees,
// hipMalloc overflow with a stderr warning, high-water mark returned by the
// torch ops).  Differences: hipStream_t instead of cudaStream_t; host errors
// throw dietgpu::DietGpuError instead of aborting; the high-water mark includes
// the allocation that set it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace dietgpu {

constexpr size_t kSDMAlignment = 256;

class StackDeviceMemory;

enum class AllocType {
  Temporary,
  Permanent,
};

template <typename T>
struct GpuMemoryReservation {
  GpuMemoryReservation() = default;
  GpuMemoryReservation(StackDeviceMemory* r, int dev, hipStream_t s, void* p,
                       size_t n, size_t bytes)
      : res(r), device(dev), stream(s), ptr(p), num(n), sizeAllocated(bytes) {}
  GpuMemoryReservation(GpuMemoryReservation&& m) noexcept { *this = std::move(m); }
  GpuMemoryReservation& operator=(GpuMemoryReservation&& m) noexcept {
    if (this != &m) {
      release();
      res = m.res;
      device = m.device;
      stream = m.stream;
      ptr = m.ptr;
      num = m.num;
      sizeAllocated = m.sizeAllocated;
      m.res = nullptr;
      m.ptr = nullptr;
      m.num = 0;
      m.sizeAllocated = 0;
    }
    return *this;
  }
  GpuMemoryReservation(const GpuMemoryReservation&) = delete;
  GpuMemoryReservation& operator=(const GpuMemoryReservation&) = delete;
  ~GpuMemoryReservation() { release(); }

  T* data() { return reinterpret_cast<T*>(ptr); }
  const T* data() const { return reinterpret_cast<const T*>(ptr); }

  // Ordered w.r.t. `s`; synchronises `s` so the vector is valid on return.
  std::vector<T> copyToHost(hipStream_t s) const;

  void release();

  StackDeviceMemory* res = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;
  void* ptr = nullptr;
  size_t num = 0;
  size_t sizeAllocated = 0;
};

class StackDeviceMemory {
 public:
  // Owns a hipMalloc'd region of `bytes` (0: every allocation overflows).
  StackDeviceMemory(int device, size_t bytes);
  // Manages a caller-owned region (e.g. a torch uint8 tensor), no ownership.
  StackDeviceMemory(int device, void* p, size_t bytes);
  ~StackDeviceMemory();
  StackDeviceMemory(const StackDeviceMemory&) = delete;
  StackDeviceMemory& operator=(const StackDeviceMemory&) = delete;

  int getDevice() const { return device_; }

  template <typename T>
  GpuMemoryReservation<T> alloc(hipStream_t stream, size_t num,
                                AllocType type = AllocType::Temporary) {
    size_t bytes = (num * sizeof(T) + kSDMAlignment - 1) / kSDMAlignment * kSDMAlignment;
    if (bytes < kSDMAlignment) bytes = kSDMAlignment;
    return GpuMemoryReservation<T>(this, device_, stream,
                                   allocPointer(stream, bytes, type), num, bytes);
  }

  template <typename T>
  GpuMemoryReservation<T> copyAlloc(hipStream_t stream, const T* p, size_t num,
                                    AllocType type = AllocType::Temporary) {
    auto m = alloc<T>(stream, num, type);
    copyToDevice(m.data(), p, num * sizeof(T), stream);
    return m;
  }

  template <typename T>
  GpuMemoryReservation<T> copyAlloc(hipStream_t stream, const std::vector<T>& v,
                                    AllocType type = AllocType::Temporary) {
    return copyAlloc<T>(stream, v.data(), v.size(), type);
  }

  void* allocPointer(hipStream_t stream, size_t bytes, AllocType type);
  void deallocPointer(int device, hipStream_t stream, size_t bytes, void* p);

  size_t getSizeAvailable() const { return size_t(end_ - head_); }
  size_t getSizeTotal() const { return size_t(end_ - start_); }
  size_t getMaxMemoryUsage() const { return maxSeen_; }
  void resetMaxMemoryUsage() { maxSeen_ = 0; }
  std::string toString() const;

  // Asynchronous host->device copy through a pinned staging ring, so pointer /
  // size tables never force a pageable (synchronous) copy.
  static void copyToDevice(void* dst, const void* src, size_t bytes, hipStream_t s);

 private:
  int device_;
  char* owned_ = nullptr;
  char* start_ = nullptr;
  char* end_ = nullptr;
  char* head_ = nullptr;
  std::unordered_map<void*, size_t> overflow_;
  size_t overflowBytes_ = 0;
  size_t maxSeen_ = 0;
  bool warned_ = false;
};

template <typename T>
void GpuMemoryReservation<T>::release() {
  if (ptr && res) {
    res->deallocPointer(device, stream, sizeAllocated, ptr);
  }
  res = nullptr;
  ptr = nullptr;
  num = 0;
  sizeAllocated = 0;
}

template <typename T>
std::vector<T> GpuMemoryReservation<T>::copyToHost(hipStream_t s) const {
  std::vector<T> out(num);
  if (num) {
    (void)hipMemcpyAsync(out.data(), ptr, num * sizeof(T), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
  }
  return out;
}

StackDeviceMemory makeStackMemory(size_t bytes = 256 * 1024 * 1024);

} // namespace dietgpu
