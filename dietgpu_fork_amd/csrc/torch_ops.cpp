// Native PyTorch-ROCm operator library: TORCH_LIBRARY(dietgpu), loadable with
// torch.ops.load_library("dietgpu_fork_amd/_lib/libdietgpu_torch.so").
//
// Mirror of the reference's operator surface (dietgpu/DietGpu.cpp:921-978):
// the same ten operators, schemas, argument meaning, validation (TORCH_CHECK
// -> RuntimeError) and return values.  Every op runs on the current HIP
// stream of the inputs' device and calls the C++ codec API of
// libdietgpu_amd.so (include/dietgpu/*.h); all compute is in its HIP kernels.
//
// Extensions over the reference: fp64 tensors are accepted on decompression
// too (the reference rejects them at DietGpu.cpp:569-573 / 742-746 although
// its compressor produces them), and an archive the compressor had to abandon
// (outSize 0, see dietgpu_device_error_count in include/dietgpu_c.h) raises
// instead of being returned as an empty tensor.
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstdint>
#include <limits>
#include <optional>
#include <string>
#include <tuple>
#include <vector>

#include "dietgpu/GpuANSCodec.h"
#include "dietgpu/GpuFloatCodec.h"
#include "dietgpu/StackDeviceMemory.h"
#include "dietgpu_c.h"

namespace dietgpu {
namespace {

constexpr int kDefaultPrecision = 10;  // DietGpu.cpp:119
constexpr uint64_t kU32Max = std::numeric_limits<uint32_t>::max();

FloatType floatTypeOf(at::ScalarType t) {
  switch (t) {
    case at::ScalarType::Half:
      return FloatType::kFloat16;
    case at::ScalarType::BFloat16:
      return FloatType::kBFloat16;
    case at::ScalarType::Float:
      return FloatType::kFloat32;
    case at::ScalarType::Double:
      return FloatType::kFloat64;
    default:
      TORCH_CHECK(false, "unsupported dtype ", t, " for float compression");
  }
}

at::ScalarType dtypeOf(uint32_t ft) {
  switch (ft) {
    case 1:
      return at::ScalarType::Half;
    case 2:
      return at::ScalarType::BFloat16;
    case 3:
      return at::ScalarType::Float;
    case 4:
      return at::ScalarType::Double;
    default:
      TORCH_CHECK(false, "not a float archive (float type ", ft, ")");
  }
}

hipStream_t currentStream(int dev) { return c10::hip::getCurrentHIPStream(dev).stream(); }

// getTotalAndMaxSize, DietGpu.cpp:63-80 (elements)
std::pair<uint64_t, uint64_t> totalAndMax(const std::vector<at::Tensor>& ts) {
  uint64_t total = 0, mx = 0;
  for (const auto& t : ts) {
    const uint64_t n = uint64_t(t.numel());
    TORCH_CHECK(n * uint64_t(t.element_size()) <= kU32Max, "tensor too large");
    total += n;
    mx = std::max(mx, n);
  }
  TORCH_CHECK(mx <= kU32Max);
  return {total, mx};
}

void checkGpuTensor(const at::Tensor& t, int dev) {
  TORCH_CHECK(t.device().type() == at::kCUDA, "inputs must be GPU tensors");
  TORCH_CHECK(t.is_contiguous(), "inputs must be contiguous");
  TORCH_CHECK(t.get_device() == dev, "inputs must be on one device");
}

// The arena over the caller's temp_mem tensor (DietGpu.cpp:303-315), or an
// empty one whose every allocation overflows to hipMalloc.
StackDeviceMemory makeStack(int dev, const std::optional<at::Tensor>& tempMem) {
  if (tempMem) {
    TORCH_CHECK(tempMem->device().type() == at::kCUDA, "temp_mem must be a GPU tensor");
    TORCH_CHECK(tempMem->is_contiguous(), "temp_mem must be contiguous");
    TORCH_CHECK(tempMem->get_device() == dev, "temp_mem must be on the input device");
    const size_t bytes = size_t(tempMem->numel()) * tempMem->element_size();
    return StackDeviceMemory(dev, bytes ? tempMem->data_ptr() : nullptr, bytes);
  }
  return StackDeviceMemory(dev, nullptr, 0);
}

// Sizes of archives the compressor could not finish are 0: never hand one out.
void checkArchiveSizes(const int32_t* sizes, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    if (sizes[i] <= 0) {
      // (read and reset, as _native.check_archive_sizes does: a later error
      // reports only the elements abandoned since this one)
      const uint32_t errs = dietgpu_device_error_count(1);
      TORCH_CHECK(false, "compression of batch element ", i,
                  " was abandoned (a cross-workgroup wait ran out of polls; ", errs,
                  " element(s) counted in the device error word since the last report)");
    }
  }
}

// ---------------------------------------------------------------- sizes ----

std::tuple<int64_t, int64_t> max_float_compressed_output_size(const std::vector<at::Tensor>& ts) {
  TORCH_CHECK(!ts.empty());
  const auto tm = totalAndMax(ts);
  return {int64_t(ts.size()), int64_t(getMaxFloatCompressedSize(floatTypeOf(ts.front().scalar_type()),
                                                                uint32_t(tm.second)))};
}

int64_t max_float_compressed_size(const at::Tensor& dtype, int64_t size) {
  TORCH_CHECK(size >= 0 && uint64_t(size) <= kU32Max, "size out of range");
  return int64_t(getMaxFloatCompressedSize(floatTypeOf(dtype.scalar_type()), uint32_t(size)));
}

std::tuple<int64_t, int64_t> max_any_compressed_output_size(const std::vector<at::Tensor>& ts) {
  TORCH_CHECK(!ts.empty());
  const auto tm = totalAndMax(ts);
  const uint64_t bytes = tm.second * uint64_t(ts.front().element_size());
  TORCH_CHECK(bytes <= kU32Max, "tensor too large");
  return {int64_t(ts.size()), int64_t(getMaxCompressedSize(uint32_t(bytes)))};
}

int64_t max_any_compressed_size(int64_t bytes) {
  TORCH_CHECK(bytes >= 0 && uint64_t(bytes) <= kU32Max, "size out of range");
  return int64_t(getMaxCompressedSize(uint32_t(bytes)));
}

// ------------------------------------------------------------- compress ----

// compress_data_res, DietGpu.cpp:161-287
std::tuple<at::Tensor, at::Tensor, int64_t> compressRes(bool asFloat, StackDeviceMemory& res,
                                                        const std::vector<at::Tensor>& ts, bool checksum,
                                                        const std::optional<at::Tensor>& outCompressed,
                                                        const std::optional<at::Tensor>& outSizes) {
  TORCH_CHECK(!ts.empty());
  const int dev = ts.front().get_device();
  const auto rc = asFloat ? max_float_compressed_output_size(ts) : max_any_compressed_output_size(ts);
  const int64_t cols = std::get<1>(rc);
  for (const auto& t : ts) {
    checkGpuTensor(t, dev);
    if (asFloat) {
      TORCH_CHECK(t.scalar_type() == ts.front().scalar_type(), "float inputs must share a dtype");
      floatTypeOf(t.scalar_type());
    }
  }
  const auto n = int64_t(ts.size());
  at::Tensor comp;
  if (outCompressed) {
    const auto& c = *outCompressed;
    TORCH_CHECK(c.scalar_type() == at::kByte && c.device().type() == at::kCUDA && c.is_contiguous());
    TORCH_CHECK(c.dim() == 2 && c.size(0) >= n && c.size(1) >= cols);
    TORCH_CHECK(c.get_device() == dev);
    comp = c;
  } else {
    comp = at::empty({n, cols}, ts.front().options().dtype(at::kByte));
  }
  at::Tensor sizes;
  if (outSizes) {
    const auto& s = *outSizes;
    TORCH_CHECK(s.scalar_type() == at::kInt && s.device().type() == at::kCUDA && s.dim() == 1);
    TORCH_CHECK(s.is_contiguous() && s.size(0) >= n && s.get_device() == dev);
    sizes = s;
  } else {
    sizes = at::empty({n}, ts.front().options().dtype(at::kInt));
  }
  std::vector<const void*> in(ts.size());
  std::vector<uint32_t> inSize(ts.size());
  std::vector<void*> out(ts.size());
  auto* base = static_cast<uint8_t*>(comp.data_ptr());
  for (size_t i = 0; i < ts.size(); ++i) {
    in[i] = ts[i].data_ptr();
    inSize[i] = uint32_t(asFloat ? ts[i].numel() : ts[i].numel() * ts[i].element_size());
    out[i] = base + int64_t(i) * comp.size(1);
  }
  const hipStream_t s = currentStream(dev);
  if (asFloat) {
    const FloatCompressConfig cfg(floatTypeOf(ts.front().scalar_type()), ANSCodecConfig(kDefaultPrecision), false,
                                  checksum);
    floatCompress(res, cfg, uint32_t(n), in.data(), inSize.data(), out.data(),
                  reinterpret_cast<uint32_t*>(sizes.data_ptr<int32_t>()), s);
  } else {
    const ANSCodecConfig cfg(kDefaultPrecision, checksum);
    ansEncodeBatchPointer(res, cfg, uint32_t(n), in.data(), inSize.data(), nullptr, out.data(),
                          reinterpret_cast<uint32_t*>(sizes.data_ptr<int32_t>()), s);
  }
  return {comp, sizes, int64_t(res.getMaxMemoryUsage())};
}

std::tuple<at::Tensor, at::Tensor, int64_t> compress_data(bool asFloat, const std::vector<at::Tensor>& tsIn,
                                                          bool checksum, const std::optional<at::Tensor>& tempMem,
                                                          const std::optional<at::Tensor>& outCompressed,
                                                          const std::optional<at::Tensor>& outSizes) {
  TORCH_CHECK(!tsIn.empty());
  const int dev = tsIn.front().get_device();
  TORCH_CHECK(dev >= 0, "inputs must be GPU tensors");
  c10::hip::HIPGuard guard(dev);
  auto res = makeStack(dev, tempMem);
  return compressRes(asFloat, res, tsIn, checksum, outCompressed, outSizes);
}

// compressedMatrixToTensors, DietGpu.cpp:84-108
std::vector<at::Tensor> matrixToTensors(int64_t n, const at::Tensor& matrix, const at::Tensor& sizes) {
  const at::Tensor host = sizes.narrow(0, 0, n).to(at::kCPU);
  const int32_t* h = host.data_ptr<int32_t>();
  checkArchiveSizes(h, n);
  const at::Tensor flat = matrix.view({-1});
  const int64_t cols = matrix.size(1);
  std::vector<at::Tensor> out;
  out.reserve(size_t(n));
  for (int64_t i = 0; i < n; ++i) out.push_back(flat.narrow(0, i * cols, h[i]));
  return out;
}

// DietGpu.cpp:322-470
std::tuple<std::vector<at::Tensor>, at::Tensor, int64_t> compress_data_split_size(
    bool asFloat, const at::Tensor& tIn, const at::Tensor& tSplit, bool checksum,
    const std::optional<at::Tensor>& tempMem, const std::optional<at::Tensor>& outCompressed,
    const std::optional<at::Tensor>& outSizes) {
  TORCH_CHECK(tIn.device().type() == at::kCUDA && tIn.is_contiguous(), "t_in must be a contiguous GPU tensor");
  const int dev = tIn.get_device();
  c10::hip::HIPGuard guard(dev);
  const FloatType ft = asFloat ? floatTypeOf(tIn.scalar_type()) : FloatType::kUndefined;
  if (!asFloat) {
    TORCH_CHECK(reinterpret_cast<uintptr_t>(tIn.data_ptr()) % 4 == 0,
                "All splits should start on a 16 byte boundary; start pointer is not aligned");
  }
  TORCH_CHECK(tSplit.is_contiguous() && tSplit.device().type() == at::kCPU && tSplit.scalar_type() == at::kInt);
  const int64_t n = tSplit.numel();
  const int32_t* sp = tSplit.data_ptr<int32_t>();
  std::vector<uint32_t> split(static_cast<size_t>(n));
  uint32_t mx = 0;
  for (int64_t i = 0; i < n; ++i) {
    TORCH_CHECK(sp[i] > 0, "split sizes must be > 0");
    split[size_t(i)] = uint32_t(sp[i]);
    mx = std::max(mx, split[size_t(i)]);
    if (!asFloat && i != n - 1) {
      TORCH_CHECK(sp[i] % 4 == 0,
                  "All splits should start on a 16 byte boundary; the size of an interior split is not a "
                  "multiple of 16 bytes");
    }
  }
  const int64_t cols = asFloat ? int64_t(getMaxFloatCompressedSize(ft, mx)) : int64_t(getMaxCompressedSize(mx));
  at::Tensor comp;
  if (outCompressed) {
    const auto& c = *outCompressed;
    TORCH_CHECK(c.scalar_type() == at::kByte && c.device().type() == at::kCUDA && c.is_contiguous());
    TORCH_CHECK(c.dim() == 2 && c.size(0) >= n && c.size(1) >= cols && c.get_device() == dev);
    comp = c;
  } else {
    comp = at::empty({n, cols}, tIn.options().dtype(at::kByte));
  }
  at::Tensor sizes;
  if (outSizes) {
    const auto& s = *outSizes;
    TORCH_CHECK(s.scalar_type() == at::kInt && s.device().type() == at::kCUDA && s.dim() == 1);
    TORCH_CHECK(s.is_contiguous() && s.size(0) >= n && s.get_device() == dev);
    sizes = s;
  } else {
    sizes = at::empty({n}, tIn.options().dtype(at::kInt));
  }
  auto res = makeStack(dev, tempMem);
  const hipStream_t s = currentStream(dev);
  auto* osz = reinterpret_cast<uint32_t*>(sizes.data_ptr<int32_t>());
  if (asFloat) {
    const FloatCompressConfig cfg(ft, ANSCodecConfig(kDefaultPrecision), false, checksum);
    floatCompressSplitSize(res, cfg, uint32_t(n), tIn.data_ptr(), split.data(), comp.data_ptr(),
                           uint32_t(comp.size(1)), osz, s);
  } else {
    const ANSCodecConfig cfg(kDefaultPrecision, checksum);
    ansEncodeBatchSplitSize(res, cfg, uint32_t(n), tIn.data_ptr(), split.data(), nullptr, comp.data_ptr(),
                            uint32_t(comp.size(1)), osz, s);
  }
  auto lst = matrixToTensors(n, comp, sizes);
  return {lst, sizes, int64_t(res.getMaxMemoryUsage())};
}

// DietGpu.cpp:472-526
std::vector<at::Tensor> compress_data_simple(bool asFloat, const std::vector<at::Tensor>& tsIn, bool checksum,
                                             std::optional<int64_t> tempMem) {
  TORCH_CHECK(!tsIn.empty());
  const int dev = tsIn.front().get_device();
  TORCH_CHECK(dev >= 0, "inputs must be GPU tensors");
  c10::hip::HIPGuard guard(dev);
  std::optional<at::Tensor> scratch;
  if (tempMem && *tempMem > 0) scratch = at::empty({*tempMem}, tsIn.front().options().dtype(at::kByte));
  auto out = compress_data(asFloat, tsIn, checksum, scratch, std::nullopt, std::nullopt);
  const at::Tensor& comp = std::get<0>(out);
  const at::Tensor host = std::get<1>(out).to(at::kCPU);
  TORCH_CHECK(host.size(0) == int64_t(tsIn.size()));
  const int32_t* h = host.data_ptr<int32_t>();
  checkArchiveSizes(h, host.size(0));
  const at::Tensor flat = comp.view({-1});
  const int64_t cols = comp.size(1);
  std::vector<at::Tensor> lst;
  lst.reserve(tsIn.size());
  for (int64_t i = 0; i < int64_t(tsIn.size()); ++i) lst.push_back(flat.narrow(0, i * cols, h[i]).clone());
  return lst;
}

// ----------------------------------------------------------- decompress ----

void checkOutDtype(const at::Tensor& t) {
  const auto d = t.scalar_type();
  TORCH_CHECK(d == at::kHalf || d == at::kBFloat16 || d == at::kFloat || d == at::kDouble,
              "float outputs must be float16, bfloat16, float32 or float64");
}

void checkStatusTensors(const std::optional<at::Tensor>& status, const std::optional<at::Tensor>& sizes, int64_t n,
                        int dev) {
  if (status) {
    TORCH_CHECK(status->is_contiguous() && status->device().type() == at::kCUDA && status->scalar_type() == at::kByte);
    TORCH_CHECK(status->numel() == n && status->get_device() == dev);
  }
  if (sizes) {
    TORCH_CHECK(sizes->is_contiguous() && sizes->device().type() == at::kCUDA && sizes->scalar_type() == at::kInt);
    TORCH_CHECK(sizes->numel() == n && sizes->get_device() == dev);
  }
}

void raiseOnChecksum(bool asFloat, bool mismatch) {
  if (!mismatch) return;
  if (asFloat) TORCH_CHECK(false, "floatDecompress: checksum mismatch seen on decoded data; archive cannot be unpacked");
  TORCH_CHECK(false, "ANSDecode: checksum mismatch seen on decoded data; archive cannot be unpacked");
}

// decompress_data_res, DietGpu.cpp:536-650
int64_t decompressRes(bool asFloat, StackDeviceMemory& res, const std::vector<at::Tensor>& tsIn,
                      const std::vector<at::Tensor>& tsOut, bool checksum, const std::optional<at::Tensor>& status,
                      const std::optional<at::Tensor>& sizes) {
  TORCH_CHECK(!tsIn.empty() && tsIn.size() == tsOut.size());
  const int dev = tsIn.front().get_device();
  std::vector<const void*> in(tsIn.size());
  std::vector<void*> out(tsIn.size());
  std::vector<uint32_t> cap(tsIn.size());
  for (size_t i = 0; i < tsIn.size(); ++i) {
    const auto& ti = tsIn[i];
    const auto& to = tsOut[i];
    TORCH_CHECK(ti.device().type() == at::kCUDA && ti.get_device() == dev && ti.is_contiguous());
    TORCH_CHECK(to.device().type() == at::kCUDA && to.get_device() == dev && to.is_contiguous());
    TORCH_CHECK(ti.scalar_type() == at::kByte, "compressed inputs must be uint8");
    if (asFloat) checkOutDtype(to);
    const uint64_t c = asFloat ? uint64_t(to.numel()) : uint64_t(to.numel()) * to.element_size();
    TORCH_CHECK(c <= kU32Max);
    in[i] = ti.data_ptr();
    out[i] = to.data_ptr();
    cap[i] = uint32_t(c);
  }
  checkStatusTensors(status, sizes, int64_t(tsIn.size()), dev);
  auto* st = status ? status->data_ptr<uint8_t>() : nullptr;
  auto* sz = sizes ? reinterpret_cast<uint32_t*>(sizes->data_ptr<int32_t>()) : nullptr;
  const hipStream_t s = currentStream(dev);
  if (asFloat) {
    const FloatDecompressConfig cfg(floatTypeOf(tsOut.front().scalar_type()), ANSCodecConfig(kDefaultPrecision),
                                    false, checksum);
    const auto r = floatDecompress(res, cfg, uint32_t(tsIn.size()), in.data(), out.data(), cap.data(), st, sz, s);
    raiseOnChecksum(true, r.error != FloatDecompressError::None);
  } else {
    const ANSCodecConfig cfg(kDefaultPrecision, checksum);
    const auto r = ansDecodeBatchPointer(res, cfg, uint32_t(tsIn.size()), in.data(), out.data(), cap.data(), st,
                                         sz, s);
    raiseOnChecksum(false, r.error != ANSDecodeError::None);
  }
  return int64_t(res.getMaxMemoryUsage());
}

// DietGpu.cpp:652-683
int64_t decompress_data(bool asFloat, const std::vector<at::Tensor>& tsIn, const std::vector<at::Tensor>& tsOut,
                        bool checksum, const std::optional<at::Tensor>& tempMem,
                        const std::optional<at::Tensor>& status, const std::optional<at::Tensor>& sizes) {
  TORCH_CHECK(!tsIn.empty());
  const int dev = tsIn.front().get_device();
  TORCH_CHECK(dev >= 0, "inputs must be GPU tensors");
  c10::hip::HIPGuard guard(dev);
  auto res = makeStack(dev, tempMem);
  return decompressRes(asFloat, res, tsIn, tsOut, checksum, status, sizes);
}

// DietGpu.cpp:685-832
int64_t decompress_data_split_size(bool asFloat, const std::vector<at::Tensor>& tsIn, const at::Tensor& tOut,
                                   const at::Tensor& tSplit, bool checksum, const std::optional<at::Tensor>& tempMem,
                                   const std::optional<at::Tensor>& status, const std::optional<at::Tensor>& sizes) {
  TORCH_CHECK(!tsIn.empty());
  const int dev = tsIn.front().get_device();
  TORCH_CHECK(dev >= 0, "inputs must be GPU tensors");
  c10::hip::HIPGuard guard(dev);
  TORCH_CHECK(tSplit.is_contiguous() && tSplit.device().type() == at::kCPU && tSplit.scalar_type() == at::kInt);
  const int64_t n = tSplit.numel();
  TORCH_CHECK(n == int64_t(tsIn.size()), "one split size per compressed input");
  const int32_t* sp = tSplit.data_ptr<int32_t>();
  std::vector<uint32_t> split(static_cast<size_t>(n));
  std::vector<const void*> in(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    const auto& ti = tsIn[size_t(i)];
    TORCH_CHECK(ti.device().type() == at::kCUDA && ti.get_device() == dev && ti.is_contiguous());
    TORCH_CHECK(ti.scalar_type() == at::kByte);
    TORCH_CHECK(sp[i] > 0, "split sizes must be > 0");
    split[size_t(i)] = uint32_t(sp[i]);
    in[size_t(i)] = ti.data_ptr();
  }
  TORCH_CHECK(tOut.device().type() == at::kCUDA && tOut.get_device() == dev && tOut.is_contiguous());
  if (asFloat) checkOutDtype(tOut);
  checkStatusTensors(status, sizes, n, dev);
  auto res = makeStack(dev, tempMem);
  auto* st = status ? status->data_ptr<uint8_t>() : nullptr;
  auto* sz = sizes ? reinterpret_cast<uint32_t*>(sizes->data_ptr<int32_t>()) : nullptr;
  const hipStream_t s = currentStream(dev);
  if (asFloat) {
    const FloatDecompressConfig cfg(floatTypeOf(tOut.scalar_type()), ANSCodecConfig(kDefaultPrecision), false,
                                    checksum);
    const auto r = floatDecompressSplitSize(res, cfg, uint32_t(n), in.data(), tOut.data_ptr(), split.data(), st, sz, s);
    raiseOnChecksum(true, r.error != FloatDecompressError::None);
  } else {
    const ANSCodecConfig cfg(kDefaultPrecision, checksum);
    const auto r = ansDecodeBatchSplitSize(res, cfg, uint32_t(n), in.data(), tOut.data_ptr(), split.data(), st, sz, s);
    raiseOnChecksum(false, r.error != ANSDecodeError::None);
  }
  return int64_t(res.getMaxMemoryUsage());
}

// DietGpu.cpp:834-917
std::vector<at::Tensor> decompress_data_simple(bool asFloat, const std::vector<at::Tensor>& tsIn, bool checksum,
                                               std::optional<int64_t> tempMem) {
  TORCH_CHECK(!tsIn.empty());
  const int dev = tsIn.front().get_device();
  TORCH_CHECK(dev >= 0, "inputs must be GPU tensors");
  c10::hip::HIPGuard guard(dev);
  for (const auto& t : tsIn) {
    TORCH_CHECK(t.device().type() == at::kCUDA && t.get_device() == dev && t.is_contiguous());
  }
  std::optional<at::Tensor> scratch;
  if (tempMem && *tempMem >= int64_t(kSDMAlignment)) {
    scratch = at::empty({*tempMem}, tsIn.front().options().dtype(at::kByte));
  }
  const auto n = int64_t(tsIn.size());
  at::Tensor info = at::zeros({2, n}, tsIn.front().options().dtype(at::kInt));
  auto res = makeStack(dev, scratch);
  std::vector<const void*> in(tsIn.size());
  for (size_t i = 0; i < tsIn.size(); ++i) in[i] = tsIn[i].data_ptr();
  const hipStream_t s = currentStream(dev);
  auto* sizesDev = reinterpret_cast<uint32_t*>(info.data_ptr<int32_t>());
  if (asFloat) {
    floatGetCompressedInfo(res, in.data(), uint32_t(n), sizesDev, sizesDev + n, nullptr, s);
  } else {
    ansGetCompressedInfo(res, in.data(), uint32_t(n), sizesDev, nullptr, s);
  }
  const at::Tensor host = info.to(at::kCPU);
  const int32_t* h = host.data_ptr<int32_t>();
  std::vector<at::Tensor> outs;
  outs.reserve(tsIn.size());
  for (int64_t i = 0; i < n; ++i) {
    const int64_t size = h[i];
    if (asFloat) {
      const uint32_t ty = uint32_t(h[n + i]);
      TORCH_CHECK(ty == uint32_t(h[n]), "all archives must have the same float type");
      outs.push_back(at::empty({size}, tsIn.front().options().dtype(dtypeOf(ty))));
    } else {
      outs.push_back(at::empty({size}, tsIn.front().options().dtype(at::kByte)));
    }
  }
  decompressRes(asFloat, res, tsIn, outs, checksum, std::nullopt, std::nullopt);
  return outs;
}

}  // namespace
}  // namespace dietgpu

// DietGpu.cpp:921-978: schemas identical to the reference's
TORCH_LIBRARY(dietgpu, m) {
  m.def("max_float_compressed_output_size(Tensor[] ts) -> (int, int)");
  m.def("max_float_compressed_size(Tensor dtype, int size) -> int");
  m.def("max_any_compressed_output_size(Tensor[] ts) -> (int, int)");
  m.def("max_any_compressed_size(int bytes) -> int");
  m.def(
      "compress_data(bool compress_as_float, Tensor[] ts_in, bool checksum=False, Tensor? temp_mem=None, "
      "Tensor? out_compressed=None, Tensor? out_compressed_bytes=None) -> (Tensor, Tensor, int)");
  m.def(
      "compress_data_split_size(bool compress_as_float, Tensor t_in, Tensor t_in_split_sizes, bool checksum=False, "
      "Tensor? temp_mem=None, Tensor? out_compressed=None, Tensor? out_compressed_bytes=None) -> (Tensor[], Tensor, "
      "int)");
  m.def(
      "compress_data_simple(bool compress_as_float, Tensor[] ts_in, bool checksum=False, int? temp_mem=67108864) -> "
      "Tensor[]");
  m.def(
      "decompress_data(bool compress_as_float, Tensor[] ts_in, Tensor[] ts_out, bool checksum=False, Tensor? "
      "temp_mem=None, Tensor? out_status=None, Tensor? out_decompressed_words=None) -> (int)");
  m.def(
      "decompress_data_split_size(bool compress_as_float, Tensor[] ts_in, Tensor t_out, Tensor t_out_split_sizes, "
      "bool checksum=False, Tensor? temp_mem=None, Tensor? out_status=None, Tensor? out_decompressed_words=None) -> "
      "(int)");
  m.def(
      "decompress_data_simple(bool compress_as_float, Tensor[] ts_in, bool checksum=False, int? temp_mem=67108864) "
      "-> Tensor[]");
}

TORCH_LIBRARY_IMPL(dietgpu, CompositeExplicitAutograd, m) {
  m.impl("max_float_compressed_output_size", &dietgpu::max_float_compressed_output_size);
  m.impl("max_float_compressed_size", &dietgpu::max_float_compressed_size);
  m.impl("max_any_compressed_output_size", &dietgpu::max_any_compressed_output_size);
  m.impl("max_any_compressed_size", &dietgpu::max_any_compressed_size);
  m.impl("compress_data", &dietgpu::compress_data);
  m.impl("compress_data_split_size", &dietgpu::compress_data_split_size);
  m.impl("compress_data_simple", &dietgpu::compress_data_simple);
  m.impl("decompress_data", &dietgpu::decompress_data);
  m.impl("decompress_data_split_size", &dietgpu::decompress_data_split_size);
  m.impl("decompress_data_simple", &dietgpu::decompress_data_simple);
}
