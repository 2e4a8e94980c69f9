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

// constant address space (4): scalar (s_load) reads of read-only tables
#define DG_CONST __attribute__((address_space(4)))

// Per-call pointer / size / offset tables small enough to ride in the kernel
// arguments of the hot kernels (k_pcompress, k_decode): the reference inlines
// up to 128 pointers in its kernel parameters (BatchProviderInlinePointer,
// ans/BatchProvider.cuh:100-194); here up to 8 KB of table (about 400
// elements), so a pointer-API call launches no upload kernel at all.
constexpr uint32_t kInlineWords = 1024;
struct InlineTable {
  uint64_t w[kInlineWords];
};

struct BatchDesc {
  enum : uint32_t { kStride = 0, kPointer = 1, kSplit = 2 };
  uint32_t mode = kStride;
  uint32_t fixedSize = 0;        // size (units) when `sizes` is null
  uint64_t stride = 0;           // bytes between elements (stride mode)
  uint8_t* base = nullptr;       // stride / split base
  const uint64_t* ptrs = nullptr;    // pointer mode: device array of addresses
  const uint32_t* sizes = nullptr;   // per-element sizes (units), optional
  const uint64_t* offsets = nullptr; // split mode: byte offset of element b
  // fields whose value is a byte offset into the launch's InlineTable
  enum : uint32_t { kInlPtrs = 1, kInlSizes = 2, kInlOffsets = 4 };
  uint32_t inl = 0;

  // A field flagged in `inl` holds a byte offset into the launch's
  // InlineTable, which must be the kernel's FIRST parameter: it is read in
  // place at the start of the kernarg segment (naming the parameter would
  // make the compiler copy all 8 KB into scratch).  inlineAt reads element
  // b's entry (b uniform) at each use; readfirstlane keeps every value
  // derived from it in SGPRs, as with a plain descriptor (without it the
  // decoder's bookkeeping moved to VGPRs: 59 -> 84 VGPRs).  Only kernels
  // with an InlineTable first argument may see inline fields.
  template <typename T>
  __device__ __forceinline__ T inlineAt(const void* field, uint32_t b) const {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass only parses device code)
    const DG_CONST T* p = reinterpret_cast<const DG_CONST T*>(
        (const DG_CONST uint8_t*)__builtin_amdgcn_kernarg_segment_ptr() + reinterpret_cast<uintptr_t>(field));
    const T v = p[b];
    if constexpr (sizeof(T) == 8) {
      const uint64_t u = uint64_t(v);
      // (the builtin returns int: widen through uint32_t, never sign-extend)
      const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(u)));
      const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(u >> 32)));
      return T(uint64_t(lo) | (uint64_t(hi) << 32));
    } else {
      return T(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(v))));
    }
#else
    (void)field;
    (void)b;
    return T(0);
#endif
  }

  __device__ __forceinline__ uint8_t* start(uint32_t b) const {
    if (mode == kPointer) {
      if (inl & kInlPtrs) return reinterpret_cast<uint8_t*>(inlineAt<uint64_t>(ptrs, b));
      return reinterpret_cast<uint8_t*>(tableAt(ptrs, b));
    }
    if (mode == kSplit) {
      if (inl & kInlOffsets) return base + inlineAt<uint64_t>(offsets, b);
      return base + tableAt(offsets, b);
    }
    return base + stride * b;
  }
  __device__ __forceinline__ uint32_t size(uint32_t b) const {
    if (!sizes) return fixedSize;
    if (inl & kInlSizes) return inlineAt<uint32_t>(sizes, b);
    return tableAt(sizes, b);
  }

  // Entry b of a device table (read-only for every kernel): through the
  // constant address space, so a wave-uniform b becomes a scalar load that
  // waits on lgkmcnt, not a vector load whose vmcnt(0) would also drain the
  // kernel's streaming loads in flight.
  template <typename T>
  __device__ __forceinline__ static T tableAt(const T* table, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const DG_CONST T*)table)[b];
#else
    return table[b];
#endif
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
