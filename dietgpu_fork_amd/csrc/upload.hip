// Host -> device upload of small parameter tables (batch pointer / size /
// offset arrays) through kernel arguments.
//
// The reference copies its pointer arrays with cudaMemcpyAsync before every
// batch call (ans/BatchProvider.cuh:100-194 via its callers).  On MI355X a
// small hipMemcpyAsync from pinned memory runs as a blit kernel that reads
// host memory over PCIe and leaves ~5-8 us idle gaps around it; two per
// compress+decompress step were ~7 % of the c2 step.  Instead the table
// rides in the kernarg segment of a one-workgroup kernel (HIP copies kernargs
// into device memory at launch) that stores it into the destination.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstring>

#include "common.h"

namespace dietgpu {

namespace {
constexpr uint32_t kTableWords = 2048;  // 8 KB per launch (16 KB kernargs verified on gfx950)
constexpr uint32_t kMaxLaunches = 8;

struct TableChunk {
  uint32_t n;
  uint32_t w[kTableWords];
};

__global__ __launch_bounds__(256) void k_table(uint32_t* __restrict__ dst, TableChunk c) {
  for (uint32_t i = threadIdx.x; i < c.n; i += 256) dst[i] = c.w[i];
}
__global__ __launch_bounds__(256) void k_zero(uint8_t* __restrict__ dst, size_t bytes) {
  const size_t stride = size_t(gridDim.x) * 256;
  const size_t i0 = size_t(blockIdx.x) * 256 + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(dst) | bytes) % 16 == 0) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (size_t i = i0; i < bytes / 16; i += stride) d[i] = make_uint4(0, 0, 0, 0);
  } else {
    for (size_t i = i0; i < bytes; i += stride) dst[i] = 0;
  }
}
}  // namespace

void zeroAsync(void* dst, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  const size_t units = (reinterpret_cast<uintptr_t>(dst) | bytes) % 16 == 0 ? bytes / 16 : bytes;
  const uint32_t grid = uint32_t(std::min<size_t>(1024, (units + 255) / 256));
  k_zero<<<grid, 256, 0, s>>>(static_cast<uint8_t*>(dst), bytes);
  HIP_LAUNCH_CHECK();
}

// Returns false (nothing enqueued) when the table is not a whole number of
// aligned 4 B words or is larger than kMaxLaunches chunks.
bool uploadViaKernargs(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0 || bytes % 4 || reinterpret_cast<uintptr_t>(dst) % 4 ||
      bytes > size_t(kMaxLaunches) * kTableWords * 4)
    return false;
  const uint32_t words = uint32_t(bytes / 4);
  TableChunk c;
  for (uint32_t w0 = 0; w0 < words; w0 += kTableWords) {
    c.n = std::min(kTableWords, words - w0);
    std::memcpy(c.w, static_cast<const uint32_t*>(src) + w0, size_t(c.n) * 4);
    k_table<<<1, 256, 0, s>>>(static_cast<uint32_t*>(dst) + w0, c);
    HIP_LAUNCH_CHECK();
  }
  return true;
}

}  // namespace dietgpu
