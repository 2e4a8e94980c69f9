// Shared constants, host error handling and gfx950 wave helpers for the
// MI355X-native rANS / float codec.  Constants restate the reference's wire
// format (ans/GpuANSUtils.cuh:33-60, float/GpuFloatUtils.cuh:15-19) so archives
// are interchangeable; everything else is designed for CDNA4 (wave64, LDS,
// 8 XCDs).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

namespace dietgpu {

// ---------------------------------------------------------------------------
// wire-format constants (ans/GpuANSUtils.cuh:33-60)
// ---------------------------------------------------------------------------
constexpr uint32_t kNumSymbols = 256;
constexpr uint32_t kBlockSize = 4096;         // uncompressed bytes per ANS block
constexpr int kStateBits = 31;                // state kept < 2^31
constexpr int kEncodedBits = 16;              // u16 renormalisation words
constexpr uint32_t kStartState = 1u << (kStateBits - kEncodedBits);
constexpr uint32_t kMinState = 1u << (kStateBits - kEncodedBits);
constexpr uint32_t kANSMagicVersion = 0xd00d0001u;
constexpr uint32_t kFloatMagicVersion = 0xf00f0001u;
constexpr uint32_t kLanesPerBlock = 32;       // interleaved states per block
constexpr uint32_t kANSHeaderBytes = 32;
constexpr uint32_t kPdfBytes = 2 * kNumSymbols;
constexpr uint32_t kStateBytesPerBlock = 4 * kLanesPerBlock;

// Scratch slot per encoded block.  The reference sizes it at
// getRawCompBlockMaxSize(4096) = 5120 B, which an adversarial 11-bit block can
// exceed (<= 4096 * 11 / 16 + 1 words = 5634 B); we size for the true maximum.
constexpr uint32_t kSlotDataBytes = 5760;     // >= 2 * roundUp(2817, 8)

__host__ __device__ constexpr inline uint32_t divUp(uint32_t a, uint32_t b) {
  return (a + b - 1) / b;
}
__host__ __device__ constexpr inline uint32_t roundUp(uint32_t a, uint32_t b) {
  return divUp(a, b) * b;
}
__host__ __device__ constexpr inline uint64_t roundUp64(uint64_t a, uint64_t b) {
  return (a + b - 1) / b * b;
}

// ANSCoalescedHeader::getCompressedOverhead (ans/GpuANSUtils.cuh:68-86)
__host__ __device__ inline uint64_t ansOverhead(uint32_t numBlocks) {
  return kANSHeaderBytes + kPdfBytes + uint64_t(kStateBytesPerBlock) * numBlocks +
      8ull * roundUp(numBlocks, 2);
}

// Float raw-section size, FloatTypeInfo<FT>::getUncompDataSize
// (float/GpuFloatUtils.cuh:200-391).  ft: 1 fp16, 2 bf16, 3 fp32, 4 fp64.
__host__ __device__ inline uint32_t floatRawBytes(int ft, uint32_t n) {
  switch (ft) {
    case 1:
    case 2:
      return roundUp(n, 16);
    case 3:
      return 2 * roundUp(n, 8) + roundUp(n, 16);
    default:
      return 4 * roundUp(n, 4) + 2 * roundUp(n, 8);
  }
}

__host__ __device__ inline uint32_t floatWordBytes(int ft) {
  return ft <= 2 ? 2 : (ft == 3 ? 4 : 8);
}

// ---------------------------------------------------------------------------
// host error handling: the C++ API throws, the C ABI converts to codes
// ---------------------------------------------------------------------------
struct DietGpuError : public std::runtime_error {
  explicit DietGpuError(const std::string& s) : std::runtime_error(s) {}
};

#define DG_CHECK(cond, msg)                                                  \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::ostringstream _s;                                                 \
      _s << __FILE__ << ":" << __LINE__ << ": check failed: " #cond ": "    \
         << msg;                                                             \
      throw ::dietgpu::DietGpuError(_s.str());                               \
    }                                                                        \
  } while (0)

#define HIP_CHECK(expr)                                                      \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      std::ostringstream _s;                                                 \
      _s << __FILE__ << ":" << __LINE__ << ": HIP error " << int(_e) << " (" \
         << hipGetErrorString(_e) << ") in " #expr;                          \
      throw ::dietgpu::DietGpuError(_s.str());                               \
    }                                                                        \
  } while (0)

#define HIP_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

// Zero `bytes` of device memory in stream order with a kernel (upload.hip).
// Used instead of hipMemsetAsync everywhere: a memset captured into a
// hipGraph was not re-run on every replay on this ROCm (256 B and 1 MiB
// nodes kept their first replay's effect, tools/debug/memset_probe.py),
// while a kernel node is.
void zeroAsync(void* dst, size_t bytes, hipStream_t s);

// ---------------------------------------------------------------------------
// device helpers (gfx950 wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t laneId() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// number of set bits of `mask` strictly below this lane (v_mbcnt_lo/hi)
__device__ __forceinline__ uint32_t mbcnt(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi(uint32_t(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo(uint32_t(mask), 0u));
}
// (HIP's __ballot(int) round-trips the predicate through a VGPR; the bool
// builtin maps straight onto the compare's SGPR-pair result)
__device__ __forceinline__ uint64_t ballot(bool p) {
  return __builtin_amdgcn_ballot_w64(p);
}
__device__ __forceinline__ uint32_t readfirst(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}

} // namespace dietgpu
