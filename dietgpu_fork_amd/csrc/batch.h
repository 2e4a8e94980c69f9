// Batch addressing for the codec kernels.
//
// The reference templates every kernel on a BatchProvider type
// (ans/BatchProvider.cuh:16-194: stride / split-size / pointer / inline
// pointer).  Here one POD descriptor with a wave-uniform mode switch covers all
// of them, so each kernel is compiled once per float type rather than once per
// provider combination.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dietgpu {

struct BatchDesc {
  enum : uint32_t { kStride = 0, kPointer = 1, kSplit = 2 };
  uint32_t mode = kStride;
  uint32_t fixedSize = 0;        // size (units) when `sizes` is null
  uint64_t stride = 0;           // bytes between elements (stride mode)
  uint8_t* base = nullptr;       // stride / split base
  const uint64_t* ptrs = nullptr;    // pointer mode: device array of addresses
  const uint32_t* sizes = nullptr;   // per-element sizes (units), optional
  const uint64_t* offsets = nullptr; // split mode: byte offset of element b

  __device__ __forceinline__ uint8_t* start(uint32_t b) const {
    if (mode == kPointer) return reinterpret_cast<uint8_t*>(ptrs[b]);
    if (mode == kSplit) return base + offsets[b];
    return base + stride * b;
  }
  __device__ __forceinline__ uint32_t size(uint32_t b) const {
    return sizes ? sizes[b] : fixedSize;
  }

  static BatchDesc strided(const void* p, uint64_t strideBytes, uint32_t size) {
    BatchDesc d;
    d.mode = kStride;
    d.base = (uint8_t*)p;
    d.stride = strideBytes;
    d.fixedSize = size;
    return d;
  }
  static BatchDesc pointers(const uint64_t* ptrs_dev, const uint32_t* sizes_dev,
                            uint32_t fixed = 0) {
    BatchDesc d;
    d.mode = kPointer;
    d.ptrs = ptrs_dev;
    d.sizes = sizes_dev;
    d.fixedSize = fixed;
    return d;
  }
  static BatchDesc split(const void* p, const uint64_t* offsets_dev,
                         const uint32_t* sizes_dev) {
    BatchDesc d;
    d.mode = kSplit;
    d.base = (uint8_t*)p;
    d.offsets = offsets_dev;
    d.sizes = sizes_dev;
    return d;
  }
};

} // namespace dietgpu
