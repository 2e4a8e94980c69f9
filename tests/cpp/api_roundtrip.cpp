// C++ consumer of the drop-in API: includes only include/dietgpu/*.h and links
// libdietgpu_amd.so, the way a program written against the reference's
// dietgpu/ans/GpuANSCodec.h and dietgpu/float/GpuFloatCodec.h would after
// swapping cudaStream_t for hipStream_t.  Roundtrips byte and float batches
// through the pointer and split-size entry points, checks sizes and
// the compressed-info readouts, and prints "OK" (exit 0) or the first failure.
//   tests/test_gpu_api.py::test_cpp_api_program runs it on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "dietgpu/GpuANSCodec.h"
#include "dietgpu/GpuFloatCodec.h"
#include "dietgpu/StackDeviceMemory.h"

using namespace dietgpu;

#define EXPECT(c)                                                   \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                 \
    }                                                               \
  } while (0)
#define HIP(x) EXPECT((x) == hipSuccess)

template <typename T>
T* devAlloc(size_t n) {
  void* p = nullptr;
  HIP(hipMalloc(&p, n * sizeof(T) + 16));
  return static_cast<T*>(p);
}

static void ansPointerRoundtrip(StackDeviceMemory& res, hipStream_t s) {
  std::mt19937 rng(1);
  const std::vector<uint32_t> sizes = {1, 4095, 4096, 70001};
  const uint32_t nb = uint32_t(sizes.size());
  std::vector<std::vector<uint8_t>> host(nb);
  std::vector<uint8_t*> in(nb), out(nb), dec(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    host[i].resize(sizes[i]);
    for (auto& b : host[i]) b = uint8_t(std::min<uint32_t>(255, rng() % 97 % 13));
    in[i] = devAlloc<uint8_t>(sizes[i]);
    HIP(hipMemcpy(in[i], host[i].data(), sizes[i], hipMemcpyHostToDevice));
    out[i] = devAlloc<uint8_t>(getMaxCompressedSize(sizes[i]));
    dec[i] = devAlloc<uint8_t>(sizes[i]);
  }
  uint32_t* outSize = devAlloc<uint32_t>(nb);
  const ANSCodecConfig cfg(kANSDefaultProbBits, true);
  ansEncodeBatchPointer(res, cfg, nb, (const void**)in.data(), sizes.data(), nullptr, (void**)out.data(), outSize, s);
  std::vector<uint32_t> csz(nb), info(nb), ck(nb);
  HIP(hipMemcpyAsync(csz.data(), outSize, nb * 4, hipMemcpyDeviceToHost, s));
  HIP(hipStreamSynchronize(s));
  for (uint32_t i = 0; i < nb; ++i) EXPECT(csz[i] > 0 && csz[i] % 16 == 0 && csz[i] <= getMaxCompressedSize(sizes[i]));
  uint32_t* infoDev = devAlloc<uint32_t>(2 * nb);
  ansGetCompressedInfo(res, (const void**)out.data(), nb, infoDev, infoDev + nb, s);
  HIP(hipMemcpyAsync(info.data(), infoDev, nb * 4, hipMemcpyDeviceToHost, s));
  HIP(hipMemcpyAsync(ck.data(), infoDev + nb, nb * 4, hipMemcpyDeviceToHost, s));
  HIP(hipStreamSynchronize(s));
  for (uint32_t i = 0; i < nb; ++i) {
    EXPECT(info[i] == sizes[i]);
    uint32_t x = 0;
    for (auto b : host[i]) x ^= b;
    EXPECT(ck[i] == x);
  }
  uint8_t* ok = devAlloc<uint8_t>(nb);
  uint32_t* dsz = devAlloc<uint32_t>(nb);
  const auto st = ansDecodeBatchPointer(res, cfg, nb, (const void**)out.data(), (void**)dec.data(), sizes.data(),
                                        ok, dsz, s);
  EXPECT(st.error == ANSDecodeError::None);
  std::vector<uint8_t> okH(nb);
  std::vector<uint32_t> dszH(nb);
  HIP(hipMemcpyAsync(okH.data(), ok, nb, hipMemcpyDeviceToHost, s));
  HIP(hipMemcpyAsync(dszH.data(), dsz, nb * 4, hipMemcpyDeviceToHost, s));
  HIP(hipStreamSynchronize(s));
  for (uint32_t i = 0; i < nb; ++i) {
    EXPECT(okH[i] == 1 && dszH[i] == sizes[i]);
    std::vector<uint8_t> back(sizes[i]);
    HIP(hipMemcpy(back.data(), dec[i], sizes[i], hipMemcpyDeviceToHost));
    EXPECT(std::memcmp(back.data(), host[i].data(), sizes[i]) == 0);
    HIP(hipFree(in[i]));
    HIP(hipFree(out[i]));
    HIP(hipFree(dec[i]));
  }
  HIP(hipFree(outSize));
  HIP(hipFree(infoDev));
  HIP(hipFree(ok));
  HIP(hipFree(dsz));
  std::printf("ans pointer roundtrip: ok\n");
}

static void floatSplitRoundtrip(StackDeviceMemory& res, hipStream_t s, FloatType ft, uint32_t wordBytes) {
  std::mt19937 rng{uint32_t(ft)};
  std::normal_distribution<float> nd;
  const std::vector<uint32_t> split = {5, 524288, 4097, 1};
  uint32_t total = 0;
  for (auto v : split) total += v;
  std::vector<uint8_t> host(size_t(total) * wordBytes);
  for (uint32_t i = 0; i < total; ++i) {
    const float f = nd(rng);
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if (wordBytes == 2) {
      const uint16_t h = uint16_t(u >> 16);  // bf16 truncation (fine as fp16 bits too)
      std::memcpy(&host[size_t(i) * 2], &h, 2);
    } else if (wordBytes == 4) {
      std::memcpy(&host[size_t(i) * 4], &u, 4);
    } else {
      const double d = f;
      std::memcpy(&host[size_t(i) * 8], &d, 8);
    }
  }
  const uint32_t nb = uint32_t(split.size());
  uint8_t* in = devAlloc<uint8_t>(host.size());
  HIP(hipMemcpy(in, host.data(), host.size(), hipMemcpyHostToDevice));
  uint32_t maxWords = 0;
  for (auto v : split) maxWords = std::max(maxWords, v);
  const uint32_t stride = getMaxFloatCompressedSize(ft, maxWords);
  uint8_t* out = devAlloc<uint8_t>(size_t(stride) * nb);
  uint32_t* outSize = devAlloc<uint32_t>(nb);
  const FloatCompressConfig cfg(ft, ANSCodecConfig(kANSDefaultProbBits), false, true);
  floatCompressSplitSize(res, cfg, nb, in, split.data(), out, stride, outSize, s);
  std::vector<uint32_t> csz(nb);
  HIP(hipMemcpyAsync(csz.data(), outSize, nb * 4, hipMemcpyDeviceToHost, s));
  HIP(hipStreamSynchronize(s));
  std::vector<const void*> rows(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    EXPECT(csz[i] > 0 && csz[i] % 16 == 0 && csz[i] <= stride);
    rows[i] = out + size_t(i) * stride;
  }
  uint32_t* infoDev = devAlloc<uint32_t>(3 * nb);
  floatGetCompressedInfo(res, rows.data(), nb, infoDev, infoDev + nb, infoDev + 2 * nb, s);
  std::vector<uint32_t> info(3 * nb);
  HIP(hipMemcpyAsync(info.data(), infoDev, 3 * nb * 4, hipMemcpyDeviceToHost, s));
  HIP(hipStreamSynchronize(s));
  for (uint32_t i = 0; i < nb; ++i) EXPECT(info[i] == split[i] && info[nb + i] == uint32_t(ft));
  uint8_t* dec = devAlloc<uint8_t>(host.size());
  uint8_t* ok = devAlloc<uint8_t>(nb);
  uint32_t* dsz = devAlloc<uint32_t>(nb);
  const auto st = floatDecompressSplitSize(res, cfg, nb, rows.data(), dec, split.data(), ok, dsz, s);
  EXPECT(st.error == FloatDecompressError::None);
  std::vector<uint8_t> back(host.size()), okH(nb);
  HIP(hipMemcpyAsync(back.data(), dec, host.size(), hipMemcpyDeviceToHost, s));
  HIP(hipMemcpyAsync(okH.data(), ok, nb, hipMemcpyDeviceToHost, s));
  HIP(hipStreamSynchronize(s));
  for (uint32_t i = 0; i < nb; ++i) EXPECT(okH[i] == 1);
  EXPECT(std::memcmp(back.data(), host.data(), host.size()) == 0);
  for (void* p : {(void*)in, (void*)out, (void*)outSize, (void*)infoDev, (void*)dec, (void*)ok, (void*)dsz})
    HIP(hipFree(p));
  std::printf("float split-size roundtrip (type %u): ok\n", uint32_t(ft));
}

int main() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  HIP(hipSetDevice(0));
  hipStream_t s;
  HIP(hipStreamCreate(&s));
  {
    auto res = makeStackMemory(64 << 20);
    ansPointerRoundtrip(res, s);
    floatSplitRoundtrip(res, s, FloatType::kFloat16, 2);
    floatSplitRoundtrip(res, s, FloatType::kBFloat16, 2);
    floatSplitRoundtrip(res, s, FloatType::kFloat32, 4);
    floatSplitRoundtrip(res, s, FloatType::kFloat64, 8);
  }
  HIP(hipStreamDestroy(s));
  std::printf("OK\n");
  return 0;
}
