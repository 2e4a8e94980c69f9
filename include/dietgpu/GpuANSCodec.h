// Public C++ API of the MI355X-native rANS byte codec.
//
// Drop-in for dietgpu/ans/GpuANSCodec.h:22-341 of NSagan271/dietgpu_fork: same
// namespace, function names, argument order, units and semantics.  The only
// signature change is the stream type (hipStream_t).  Host-side validation
// errors throw dietgpu::DietGpuError (the reference aborts via glog CHECK).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "dietgpu/StackDeviceMemory.h"

namespace dietgpu {

constexpr int kANSRequiredAlignment = 4;   // GpuANSCodec.h:16
constexpr int kANSDefaultProbBits = 10;    // GpuANSCodec.h:20

// Bound on one archive of `uncompressedBytes` input (ans/GpuANSEncode.cu:13-25)
uint32_t getMaxCompressedSize(uint32_t uncompressedBytes);

struct ANSCodecConfig {
  inline ANSCodecConfig() : probBits(kANSDefaultProbBits), useChecksum(false) {}
  explicit inline ANSCodecConfig(int pb, bool checksum = false)
      : probBits(pb), useChecksum(checksum) {}
  int probBits;      // 9, 10 or 11
  bool useChecksum;  // XOR-of-bytes stored in the header, verified on decode
};

enum class ANSDecodeError : uint32_t {
  None = 0,
  ChecksumMismatch = 1,
};

struct ANSDecodeStatus {
  inline ANSDecodeStatus() : error(ANSDecodeError::None) {}
  ANSDecodeError error;
  std::vector<std::pair<int, std::string>> errorInfo;
};

// GpuANSCodec.h:64-98
void ansEncodeBatchStride(StackDeviceMemory& res, const ANSCodecConfig& config,
                          uint32_t numInBatch, const void* in_dev,
                          uint32_t inPerBatchSize, uint32_t inPerBatchStride,
                          const uint32_t* histogram_dev, void* out_dev,
                          uint32_t outPerBatchStride, uint32_t* outBatchSize_dev,
                          hipStream_t stream);

// GpuANSCodec.h:100-131
void ansEncodeBatchPointer(StackDeviceMemory& res, const ANSCodecConfig& config,
                           uint32_t numInBatch, const void** in,
                           const uint32_t* inSize, const uint32_t* histogram_dev,
                           void** out, uint32_t* outSize_dev, hipStream_t stream);

// GpuANSCodec.h:133-167
void ansEncodeBatchSplitSize(StackDeviceMemory& res, const ANSCodecConfig& config,
                             uint32_t numInBatch, const void* in_dev,
                             const uint32_t* inSplitSizes,
                             const uint32_t* histogram_dev, void* out_dev,
                             uint32_t outStride, uint32_t* outSize_dev,
                             hipStream_t stream);

// GpuANSCodec.h:173-226
ANSDecodeStatus ansDecodeBatchStride(StackDeviceMemory& res,
                                     const ANSCodecConfig& config,
                                     uint32_t numInBatch, const void* in_dev,
                                     uint32_t inPerBatchStride, void* out_dev,
                                     uint32_t outPerBatchStride,
                                     uint32_t outPerBatchCapacity,
                                     uint8_t* outSuccess_dev,
                                     uint32_t* outSize_dev, hipStream_t stream);

// GpuANSCodec.h:228-262
ANSDecodeStatus ansDecodeBatchPointer(StackDeviceMemory& res,
                                      const ANSCodecConfig& config,
                                      uint32_t numInBatch, const void** in,
                                      void** out, const uint32_t* outCapacity,
                                      uint8_t* outSuccess_dev,
                                      uint32_t* outSize_dev, hipStream_t stream);

// GpuANSCodec.h:264-300
ANSDecodeStatus ansDecodeBatchSplitSize(StackDeviceMemory& res,
                                        const ANSCodecConfig& config,
                                        uint32_t numInBatch, const void** in,
                                        void* out_dev,
                                        const uint32_t* outSplitSizes,
                                        uint8_t* outSuccess_dev,
                                        uint32_t* outSize_dev,
                                        hipStream_t stream);

// GpuANSCodec.h:306-341: sizes reported are the *uncompressed* byte counts
void ansGetCompressedInfo(StackDeviceMemory& res, const void** in,
                          uint32_t numInBatch, uint32_t* outSizes_dev,
                          uint32_t* outChecksum_dev, hipStream_t stream);
void ansGetCompressedInfoDevice(StackDeviceMemory& res, const void** in_dev,
                                uint32_t numInBatch, uint32_t* outSizes_dev,
                                uint32_t* outChecksum_dev, hipStream_t stream);

} // namespace dietgpu
