// Test-hook library libdietgpu_testhooks.so (include/dietgpu_testhooks.h; not
// linked into the product library).  Not part of the reference API: a
// bounded-duration kernel that
// holds compute units, so tests can run the compressor while another kernel
// occupies part of the chip (pcompress.h, "Forward progress"); and the byte
// histogram of the three-kernel compressor's first pass exposed on its own,
// as the reference's ANSStatisticsTest.cu:44-95 exercises ansHistogramBatch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include <exception>
#include <string>

#include "capi_internal.h"
#include "common.h"
#include "dietgpu/StackDeviceMemory.h"
#include "dietgpu_testhooks.h"
#include "encode.h"

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

// Sum of an element's per-chunk partial histograms (k_hist rows): grid nb.
__global__ __launch_bounds__(kThreads) void k_sumChunkRows(const uint32_t* part, uint32_t chunks,
                                                          uint32_t* out) {
  __shared__ u32x4 red4[kThreads];
  const uint32_t b = blockIdx.x;
  const uint32_t v = sumRows256<false>(G(part) + uint64_t(b) * chunks * kNumSymbols, chunks, red4);
  G(out)[uint64_t(b) * kNumSymbols + threadIdx.x] = v;
}
}  // namespace

// hist[b][256] = byte histogram of element b of a stride batch (elements of
// `size` bytes, `stride` bytes apart): k_hist<0> (the compressor's own
// histogram kernel, chunked exactly as encodeBatchDevice chunks it) and a row
// sum.  ansHistogramBatch (ans/GpuANSStatistics.cuh:113-143).
void testHistogram(StackDeviceMemory& res, hipStream_t s, uint32_t nb, const void* in_dev, uint32_t size,
                   uint32_t stride, uint32_t* hist_dev) {
  if (nb == 0) return;
  DG_CHECK(nb <= 65535, "at most 65535 elements");
  const auto in = BatchDesc::strided(in_dev, stride, size);
  uint32_t chunk = 64 * 1024;
  while (divUp(size, chunk) > 4096) chunk *= 2;
  const uint32_t chunks = std::max(1u, divUp(size, chunk));
  auto part = res.alloc<uint32_t>(s, size_t(nb) * chunks * kNumSymbols);
  NormArgs na{};
  k_hist<0, false><<<dim3(chunks, nb), kThreads, 0, s>>>(in, 0, nb, chunk, chunks, part.data(), nullptr, na);
  HIP_LAUNCH_CHECK();
  k_sumChunkRows<<<nb, kThreads, 0, s>>>(part.data(), chunks, hist_dev);
  HIP_LAUNCH_CHECK();
}

// magic[q] for q = 0 .. 2048 by the compressors' in-register computation
__global__ __launch_bounds__(256) void k_encMagic(uint32_t* magic) {
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  if (q > (1u << 11)) return;
  G(magic)[q] = q == 0 ? 0u : q == 1 ? 0xffffffffu : encMagicReg(q, 31 - __clz(q - 1));
}

void testEncMagic(hipStream_t s, uint32_t* magic) {
  k_encMagic<<<divUp((1u << 11) + 1, 256), 256, 0, s>>>(magic);
  HIP_LAUNCH_CHECK();
}

void testOccupy(hipStream_t s, uint32_t micros, uint32_t workgroups, uint32_t ldsBytes) {
  DG_CHECK(ldsBytes >= 1024 && ldsBytes <= 160 * 1024, "ldsBytes out of range");
  DG_CHECK(micros <= 1000000, "at most 1 s");
  k_occupy<<<workgroups, 256, ldsBytes, s>>>(uint64_t(micros) * 100, nullptr);
  HIP_LAUNCH_CHECK();
}

}  // namespace dietgpu

namespace {
thread_local std::string gTestError;

template <typename F>
int guardedTest(F&& f) {
  try {
    gTestError.clear();
    f();
    return DIETGPU_OK;
  } catch (const std::exception& e) {
    gTestError = e.what();
  } catch (...) {
    gTestError = "unknown error";
  }
  return DIETGPU_ERR_INVALID;
}
}  // namespace

extern "C" {

const char* dietgpu_test_last_error(void) { return gTestError.c_str(); }

int dietgpu_test_occupy(void* stream, uint32_t micros, uint32_t workgroups, uint32_t lds_bytes) {
  return guardedTest([&] { dietgpu::testOccupy(reinterpret_cast<hipStream_t>(stream), micros, workgroups, lds_bytes); });
}

int dietgpu_test_histogram(dietgpu_stack* res, uint32_t nb, const void* in_dev, uint32_t size,
                           uint32_t stride, uint32_t* hist_dev, void* stream) {
  return guardedTest([&] {
    DG_CHECK(res && res->mem, "null dietgpu_stack");
    dietgpu::testHistogram(*res->mem, reinterpret_cast<hipStream_t>(stream), nb, in_dev, size, stride, hist_dev);
  });
}

int dietgpu_test_enc_magic(uint32_t* magic_dev, void* stream) {
  return guardedTest([&] { dietgpu::testEncMagic(reinterpret_cast<hipStream_t>(stream), magic_dev); });
}

}  // extern "C"
