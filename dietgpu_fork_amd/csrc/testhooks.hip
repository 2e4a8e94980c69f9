// Test hooks (not part of the reference API): a bounded-duration kernel that
// holds compute units, so tests can run the compressor while another kernel
// occupies part of the chip (pcompress.h, "Forward progress").
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"

namespace dietgpu {

namespace {
// Each workgroup holds `ldsBytes` of LDS (dynamic) and one wave per SIMD for
// `ticks` of the 100 MHz real-time counter, then exits: every wave reaches
// the exit whatever the other workgroups do.
__global__ __launch_bounds__(256) void k_occupy(uint64_t ticks, uint32_t* sink) {
  extern __shared__ uint32_t lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  uint32_t acc = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    acc += lds[(threadIdx.x + acc) & 255];
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // never: keeps the loop
}
}  // namespace

void testOccupy(hipStream_t s, uint32_t micros, uint32_t workgroups, uint32_t ldsBytes) {
  DG_CHECK(ldsBytes >= 1024 && ldsBytes <= 160 * 1024, "ldsBytes out of range");
  DG_CHECK(micros <= 1000000, "at most 1 s");
  k_occupy<<<workgroups, 256, ldsBytes, s>>>(uint64_t(micros) * 100, nullptr);
  HIP_LAUNCH_CHECK();
}

}  // namespace dietgpu
