// Public C++ API of the MI355X-native exponent-split float codec and the
// sparse-float codec.
//
// Drop-in for dietgpu/float/GpuFloatCodec.h:32-322 of NSagan271/dietgpu_fork:
// same names, argument order, units (float sizes/capacities in *words*,
// compressed sizes in bytes) and semantics; hipStream_t streams.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "dietgpu/GpuANSCodec.h"

namespace dietgpu {

class StackDeviceMemory;

enum class FloatType : uint32_t {
  kUndefined = 0,
  kFloat16 = 1,
  kBFloat16 = 2,
  kFloat32 = 3,
  kFloat64 = 4,
};

uint32_t getMaxFloatCompressedSize(FloatType floatType, uint32_t size);
uint32_t getMaxSparseFloatCompressedSize(FloatType floatType, uint32_t size);

struct FloatCodecConfig {
  inline FloatCodecConfig()
      : floatType(FloatType::kFloat16), useChecksum(false), is16ByteAligned(false) {}
  inline FloatCodecConfig(FloatType ft, const ANSCodecConfig& ansConf, bool align,
                          bool checksum = false)
      : floatType(ft), useChecksum(checksum), ansConfig(ansConf),
        is16ByteAligned(align) {}
  FloatType floatType;
  bool useChecksum;
  ANSCodecConfig ansConfig;  // ansConfig.useChecksum must be false
  // Kept for API compatibility.  The MI355X decoder is always the fused
  // single-pass kernel (fp64 included), so alignment only picks load widths.
  bool is16ByteAligned;
};

using FloatCompressConfig = FloatCodecConfig;
using FloatDecompressConfig = FloatCodecConfig;

enum class FloatDecompressError : uint32_t {
  None = 0,
  ChecksumMismatch = 1,
};

struct FloatDecompressStatus {
  inline FloatDecompressStatus() : error(FloatDecompressError::None) {}
  FloatDecompressError error;
  std::vector<std::pair<int, std::string>> errorInfo;
};

// GpuFloatCodec.h:118-158
void floatCompress(StackDeviceMemory& res, const FloatCompressConfig& config,
                   uint32_t numInBatch, const void** in, const uint32_t* inSize,
                   void** out, uint32_t* outSize_dev, hipStream_t stream);

// GpuFloatCodec.h:160-187
void floatCompressSplitSize(StackDeviceMemory& res,
                            const FloatCompressConfig& config,
                            uint32_t numInBatch, const void* in_dev,
                            const uint32_t* inSplitSizes, void* out_dev,
                            uint32_t outStride, uint32_t* outSize_dev,
                            hipStream_t stream);

// GpuFloatCodec.h:189-203
void floatCompressSparse(StackDeviceMemory& res, const FloatCompressConfig& config,
                         uint32_t numInBatch, const void** in,
                         const uint32_t* inSize, void** out,
                         uint32_t* outSize_dev, hipStream_t stream);

// GpuFloatCodec.h:209-242
FloatDecompressStatus floatDecompress(StackDeviceMemory& res,
                                      const FloatDecompressConfig& config,
                                      uint32_t numInBatch, const void** in,
                                      void** out, const uint32_t* outCapacity,
                                      uint8_t* outSuccess_dev,
                                      uint32_t* outSize_dev, hipStream_t stream);

// GpuFloatCodec.h:244-280
FloatDecompressStatus floatDecompressSplitSize(
    StackDeviceMemory& res, const FloatDecompressConfig& config,
    uint32_t numInBatch, const void** in, void* out_dev,
    const uint32_t* outSplitSizes, uint8_t* outSuccess_dev,
    uint32_t* outSize_dev, hipStream_t stream);

// GpuFloatCodec.h:282-293
FloatDecompressStatus floatDecompressSparse(StackDeviceMemory& res,
                                            const FloatDecompressConfig& config,
                                            uint32_t numInBatch, const void** in,
                                            void** out,
                                            const uint32_t* outCapacity,
                                            uint8_t* outSuccess_dev,
                                            uint32_t* outSize_dev,
                                            hipStream_t stream);

// GpuFloatCodec.h:299-322
void floatGetCompressedInfo(StackDeviceMemory& res, const void** in,
                            uint32_t numInBatch, uint32_t* outSizes_dev,
                            uint32_t* outTypes_dev, uint32_t* outChecksum_dev,
                            hipStream_t stream);
void floatGetCompressedInfoDevice(StackDeviceMemory& res, const void** in_dev,
                                  uint32_t numInBatch, uint32_t* outSizes_dev,
                                  uint32_t* outTypes_dev,
                                  uint32_t* outChecksum_dev, hipStream_t stream);

// ---- MI355X extensions (not in the reference API) ----
// Stride-addressed float batch: no host->device parameter copies at all.
void floatCompressBatchStride(StackDeviceMemory& res,
                              const FloatCompressConfig& config,
                              uint32_t numInBatch, const void* in_dev,
                              uint32_t inPerBatchWords, uint64_t inPerBatchStrideBytes,
                              void* out_dev, uint64_t outPerBatchStrideBytes,
                              uint32_t* outSize_dev, hipStream_t stream);
FloatDecompressStatus floatDecompressBatchStride(
    StackDeviceMemory& res, const FloatDecompressConfig& config,
    uint32_t numInBatch, const void* in_dev, uint64_t inPerBatchStrideBytes,
    void* out_dev, uint64_t outPerBatchStrideBytes, uint32_t outPerBatchCapacityWords,
    uint8_t* outSuccess_dev, uint32_t* outSize_dev, hipStream_t stream);

} // namespace dietgpu
