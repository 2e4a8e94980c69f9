// Internal entry points shared by the dense and sparse float drivers.
#pragma once

#include <string>
#include <utility>
#include <vector>

#include "batch.h"
#include "dietgpu/GpuFloatCodec.h"

namespace dietgpu {

struct DeviceTables;  // codec.hip: per-call pointer tables (maybe kernel-argument inline)

// Partial symbol histograms of the float words counted by the caller (the
// sparse compressor counts its nonzeros as it compacts them, so the dense
// codec's histogram pass is skipped): u32 rows [segments][nb][nRows][256],
// summed per element.  Ignored when the single-pass compressor takes the call.
// table / pdf non-null: the caller has normalised the rows too
// ([segments][nb][256] encode-table entries and u16 pdfs, NormArgs layout),
// so the dense codec goes straight to k_encode.
struct PartialHist {
  const uint32_t* rows;
  uint32_t nRows;
  const uint4* table = nullptr;
  const uint16_t* pdf = nullptr;
};

void floatCompressDescs(StackDeviceMemory& res, const FloatCompressConfig& config, uint32_t nb,
                        const BatchDesc& in, uint32_t maxSize, const BatchDesc& out,
                        uint32_t* outSize_dev, hipStream_t s, const DeviceTables* tabs = nullptr,
                        bool inAligned16 = false, const PartialHist* pre = nullptr,
                        const uint32_t* sparseN = nullptr);

// Whether encodeBatchDevice compresses nb 16 B-aligned elements of at most
// maxWords words of a single-segment format (FT 0-3) with the single-pass
// compressor (k_pcompress) rather than the three-kernel path.
template <int FT>
bool persistentPreferred(uint32_t nb, uint32_t maxWords);

FloatDecompressStatus floatDecompressDescs(StackDeviceMemory& res,
                                           const FloatDecompressConfig& config, uint32_t nb,
                                           const BatchDesc& in, const BatchDesc& out,
                                           uint32_t maxCap, uint8_t* succ, uint32_t* sizes,
                                           hipStream_t s, const DeviceTables* tabs = nullptr,
                                           bool streamOut = true, bool capacityOnly = false);

// Compare archive checksums with the XOR of `decoded.size(b)` bytes of each
// decoded element; synchronises `s`.
std::vector<std::pair<int, std::string>> verifyChecksums(StackDeviceMemory& res, uint32_t nb,
                                                         const BatchDesc& archives, bool isFloat,
                                                         const BatchDesc& decoded,
                                                         uint32_t maxBytes, hipStream_t s,
                                                         const DeviceTables* tabs = nullptr);

// The device error word (elements whose compression was abandoned after a
// bounded wait ran out; their outSize is 0), codec.hip.
uint32_t* deviceErrorWord();

}  // namespace dietgpu
