// extern "C" boundary of libdietgpu_amd.so (declared in include/dietgpu_c.h).
// Each entry point forwards to the C++ API and converts exceptions into
// error codes + a thread-local message.
#include "dietgpu_c.h"

#include <exception>
#include <string>

#include "common.h"
#include "dietgpu/GpuANSCodec.h"
#include "dietgpu/GpuFloatCodec.h"
#include "dietgpu/StackDeviceMemory.h"
#include "profile.h"
#include "sync_arena.h"

using namespace dietgpu;

#include "capi_internal.h"

namespace {
thread_local std::string gLastError;

template <typename F>
int guarded(F&& f) {
  try {
    gLastError.clear();
    return f();
  } catch (const DietGpuError& e) {
    gLastError = e.what();
    return std::string(e.what()).find("HIP error") != std::string::npos ? DIETGPU_ERR_HIP
                                                                        : DIETGPU_ERR_INVALID;
  } catch (const std::exception& e) {
    gLastError = e.what();
    return DIETGPU_ERR_INVALID;
  } catch (...) {
    gLastError = "unknown error";
    return DIETGPU_ERR_INVALID;
  }
}

StackDeviceMemory& R(dietgpu_stack* r) {
  DG_CHECK(r && r->mem, "null dietgpu_stack");
  return *r->mem;
}

hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

FloatCodecConfig floatCfg(int ft, int pb, int ck) {
  DG_CHECK(ft >= 1 && ft <= 4, "float_type must be 1..4");
  return FloatCodecConfig(FloatType(ft), ANSCodecConfig(pb, false), false, ck != 0);
}

template <typename Status>
int statusCode(const Status& st) {
  if (st.errorInfo.empty()) return DIETGPU_OK;
  std::string msg;
  for (auto& e : st.errorInfo) msg += e.second;
  gLastError = msg;
  return DIETGPU_ERR_CHECKSUM;
}
}  // namespace

extern "C" {

const char* dietgpu_last_error(void) { return gLastError.c_str(); }
const char* dietgpu_version(void) { return "dietgpu_fork_amd 0.1 (gfx950)"; }

dietgpu_stack* dietgpu_stack_create(int device, void* ptr, size_t bytes) {
  dietgpu_stack* out = nullptr;
  int rc = guarded([&] {
    out = new dietgpu_stack{ptr ? new StackDeviceMemory(device, ptr, bytes)
                                : new StackDeviceMemory(device, bytes)};
    return DIETGPU_OK;
  });
  return rc == DIETGPU_OK ? out : nullptr;
}

void dietgpu_stack_destroy(dietgpu_stack* r) {
  if (r) {
    delete r->mem;
    delete r;
  }
}

size_t dietgpu_stack_max_usage(const dietgpu_stack* r) { return r ? r->mem->getMaxMemoryUsage() : 0; }
void dietgpu_stack_reset_max_usage(dietgpu_stack* r) {
  if (r) r->mem->resetMaxMemoryUsage();
}
size_t dietgpu_stack_size_total(const dietgpu_stack* r) { return r ? r->mem->getSizeTotal() : 0; }

uint32_t dietgpu_get_max_compressed_size(uint32_t bytes) {
  uint32_t v = 0;
  guarded([&] {
    v = getMaxCompressedSize(bytes);
    return DIETGPU_OK;
  });
  return v;
}

uint32_t dietgpu_get_max_float_compressed_size(int ft, uint32_t words) {
  uint32_t v = 0;
  guarded([&] {
    v = getMaxFloatCompressedSize(FloatType(ft), words);
    return DIETGPU_OK;
  });
  return v;
}

uint32_t dietgpu_get_max_sparse_float_compressed_size(int ft, uint32_t words) {
  uint32_t v = 0;
  guarded([&] {
    DG_CHECK(ft >= 1 && ft <= 4, "float_type must be 1..4");
    v = getMaxSparseFloatCompressedSize(FloatType(ft), words);
    return DIETGPU_OK;
  });
  return v;
}

int dietgpu_ans_encode_batch_stride(dietgpu_stack* res, int pb, int ck, uint32_t nb,
                                    const void* in_dev, uint32_t in_size, uint32_t in_stride,
                                    const uint32_t* hist_dev, void* out_dev, uint32_t out_stride,
                                    uint32_t* out_size_dev, void* stream) {
  return guarded([&] {
    ansEncodeBatchStride(R(res), ANSCodecConfig(pb, ck != 0), nb, in_dev, in_size, in_stride,
                         hist_dev, out_dev, out_stride, out_size_dev, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_ans_encode_batch_pointer(dietgpu_stack* res, int pb, int ck, uint32_t nb,
                                     const void** in, const uint32_t* in_size,
                                     const uint32_t* hist_dev, void** out, uint32_t* out_size_dev,
                                     void* stream) {
  return guarded([&] {
    ansEncodeBatchPointer(R(res), ANSCodecConfig(pb, ck != 0), nb, in, in_size, hist_dev, out,
                          out_size_dev, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_ans_encode_batch_split_size(dietgpu_stack* res, int pb, int ck, uint32_t nb,
                                        const void* in_dev, const uint32_t* split,
                                        const uint32_t* hist_dev, void* out_dev,
                                        uint32_t out_stride, uint32_t* out_size_dev,
                                        void* stream) {
  return guarded([&] {
    ansEncodeBatchSplitSize(R(res), ANSCodecConfig(pb, ck != 0), nb, in_dev, split, hist_dev,
                            out_dev, out_stride, out_size_dev, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_ans_decode_batch_stride(dietgpu_stack* res, int pb, int ck, uint32_t nb,
                                    const void* in_dev, uint32_t in_stride, void* out_dev,
                                    uint32_t out_stride, uint32_t out_cap, uint8_t* succ,
                                    uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(ansDecodeBatchStride(R(res), ANSCodecConfig(pb, ck != 0), nb, in_dev,
                                           in_stride, out_dev, out_stride, out_cap, succ, sizes,
                                           S(stream)));
  });
}

int dietgpu_ans_decode_batch_pointer(dietgpu_stack* res, int pb, int ck, uint32_t nb,
                                     const void** in, void** out, const uint32_t* cap,
                                     uint8_t* succ, uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(ansDecodeBatchPointer(R(res), ANSCodecConfig(pb, ck != 0), nb, in, out, cap,
                                            succ, sizes, S(stream)));
  });
}

int dietgpu_ans_decode_batch_split_size(dietgpu_stack* res, int pb, int ck, uint32_t nb,
                                        const void** in, void* out_dev, const uint32_t* split,
                                        uint8_t* succ, uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(ansDecodeBatchSplitSize(R(res), ANSCodecConfig(pb, ck != 0), nb, in,
                                              out_dev, split, succ, sizes, S(stream)));
  });
}

int dietgpu_ans_get_compressed_info(dietgpu_stack* res, const void** in, uint32_t nb,
                                    uint32_t* sizes, uint32_t* cks, void* stream) {
  return guarded([&] {
    ansGetCompressedInfo(R(res), in, nb, sizes, cks, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_ans_get_compressed_info_device(dietgpu_stack* res, const void** in_dev, uint32_t nb,
                                           uint32_t* sizes, uint32_t* cks, void* stream) {
  return guarded([&] {
    ansGetCompressedInfoDevice(R(res), in_dev, nb, sizes, cks, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_compress(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                           const void** in, const uint32_t* in_size, void** out,
                           uint32_t* out_size_dev, void* stream) {
  return guarded([&] {
    floatCompress(R(res), floatCfg(ft, pb, ck), nb, in, in_size, out, out_size_dev, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_compress_split_size(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                                      const void* in_dev, const uint32_t* split, void* out_dev,
                                      uint32_t out_stride, uint32_t* out_size_dev, void* stream) {
  return guarded([&] {
    floatCompressSplitSize(R(res), floatCfg(ft, pb, ck), nb, in_dev, split, out_dev, out_stride,
                           out_size_dev, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_compress_sparse(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                                  const void** in, const uint32_t* in_size, void** out,
                                  uint32_t* out_size_dev, void* stream) {
  return guarded([&] {
    floatCompressSparse(R(res), floatCfg(ft, pb, ck), nb, in, in_size, out, out_size_dev,
                        S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_decompress(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                             const void** in, void** out, const uint32_t* cap, uint8_t* succ,
                             uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(
        floatDecompress(R(res), floatCfg(ft, pb, ck), nb, in, out, cap, succ, sizes, S(stream)));
  });
}

int dietgpu_float_decompress_split_size(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                                        const void** in, void* out_dev, const uint32_t* split,
                                        uint8_t* succ, uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(floatDecompressSplitSize(R(res), floatCfg(ft, pb, ck), nb, in, out_dev,
                                               split, succ, sizes, S(stream)));
  });
}

int dietgpu_float_decompress_sparse(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                                    const void** in, void** out, const uint32_t* cap,
                                    uint8_t* succ, uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(floatDecompressSparse(R(res), floatCfg(ft, pb, ck), nb, in, out, cap, succ,
                                            sizes, S(stream)));
  });
}

int dietgpu_float_get_compressed_info(dietgpu_stack* res, const void** in, uint32_t nb,
                                      uint32_t* sizes, uint32_t* types, uint32_t* cks,
                                      void* stream) {
  return guarded([&] {
    floatGetCompressedInfo(R(res), in, nb, sizes, types, cks, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_get_compressed_info_device(dietgpu_stack* res, const void** in_dev,
                                             uint32_t nb, uint32_t* sizes, uint32_t* types,
                                             uint32_t* cks, void* stream) {
  return guarded([&] {
    floatGetCompressedInfoDevice(R(res), in_dev, nb, sizes, types, cks, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_compress_batch_stride(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                                        const void* in_dev, uint32_t words, uint64_t in_stride,
                                        void* out_dev, uint64_t out_stride,
                                        uint32_t* out_size_dev, void* stream) {
  return guarded([&] {
    floatCompressBatchStride(R(res), floatCfg(ft, pb, ck), nb, in_dev, words, in_stride, out_dev,
                             out_stride, out_size_dev, S(stream));
    return DIETGPU_OK;
  });
}

int dietgpu_float_decompress_batch_stride(dietgpu_stack* res, int ft, int pb, int ck, uint32_t nb,
                                          const void* in_dev, uint64_t in_stride, void* out_dev,
                                          uint64_t out_stride, uint32_t cap_words, uint8_t* succ,
                                          uint32_t* sizes, void* stream) {
  return guarded([&] {
    return statusCode(floatDecompressBatchStride(R(res), floatCfg(ft, pb, ck), nb, in_dev,
                                                 in_stride, out_dev, out_stride, cap_words, succ,
                                                 sizes, S(stream)));
  });
}

uint32_t dietgpu_device_error_count(int reset) {
  uint32_t v = 0;
  guarded([&] {
    v = deviceErrorCount(reset != 0);
    return DIETGPU_OK;
  });
  return v;
}

uint32_t dietgpu_barrier_fallback_count(int reset) {
  uint32_t v = 0;
  guarded([&] {
    v = barrierFallbackCount(reset != 0);
    return DIETGPU_OK;
  });
  return v;
}

void dietgpu_set_spin_cap(uint32_t polls) { setSpinCap(polls); }
void dietgpu_set_barrier_budget(uint32_t ticks) { setBarrierBudget(ticks); }
void dietgpu_set_dispatch_skew(uint32_t ticks) { setDispatchSkew(ticks); }
void dietgpu_set_compress_path(int mode) { setCompressPath(mode < 0 || mode > 2 ? 0 : mode); }

void dietgpu_profile_enable(int on) { prof::setEnabled(on != 0); }
void dietgpu_profile_filter(const char* kernel) { prof::setFilter(kernel); }
void dietgpu_profile_reset(void) { prof::reset(); }
int dietgpu_profile_query(const char* kernel, double* total_ms, uint64_t* launches) {
  return prof::query(kernel, total_ms, launches) ? DIETGPU_OK : DIETGPU_ERR_INVALID;
}

}  // extern "C"
