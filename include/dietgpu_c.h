/*
 * dietgpu_c.h -- C ABI of the MI355X-native dietgpu codec (libdietgpu_amd.so).
 *
 * The drop-in boundary.  Every entry point is a plain-pointer restatement of
 * one function of the reference's C++ API (NSagan271/dietgpu_fork, paths
 * relative to /root/reference/dietgpu), so an FFI (ctypes, cffi, JNI, cgo)
 * binds it without C++ types:
 *
 *   dietgpu_get_max_compressed_size          ans/GpuANSCodec.h:23   (GpuANSEncode.cu:13)
 *   dietgpu_ans_encode_batch_stride          ans/GpuANSCodec.h:64-98
 *   dietgpu_ans_encode_batch_pointer         ans/GpuANSCodec.h:100-131
 *   dietgpu_ans_encode_batch_split_size      ans/GpuANSCodec.h:133-167
 *   dietgpu_ans_decode_batch_stride          ans/GpuANSCodec.h:173-226
 *   dietgpu_ans_decode_batch_pointer         ans/GpuANSCodec.h:228-262
 *   dietgpu_ans_decode_batch_split_size      ans/GpuANSCodec.h:264-300
 *   dietgpu_ans_get_compressed_info          ans/GpuANSCodec.h:306-322
 *   dietgpu_ans_get_compressed_info_device   ans/GpuANSCodec.h:324-340
 *   dietgpu_get_max_float_compressed_size    float/GpuFloatCodec.h:32
 *   dietgpu_get_max_sparse_float_compressed_size float/GpuFloatCodec.h:33
 *   dietgpu_float_compress                   float/GpuFloatCodec.h:118-158
 *   dietgpu_float_compress_split_size        float/GpuFloatCodec.h:160-187
 *   dietgpu_float_compress_sparse            float/GpuFloatCodec.h:189-203
 *   dietgpu_float_decompress                 float/GpuFloatCodec.h:209-242
 *   dietgpu_float_decompress_split_size      float/GpuFloatCodec.h:244-280
 *   dietgpu_float_decompress_sparse          float/GpuFloatCodec.h:282-293
 *   dietgpu_float_get_compressed_info        float/GpuFloatCodec.h:299-309
 *   dietgpu_float_get_compressed_info_device float/GpuFloatCodec.h:311-321
 *   dietgpu_stack_*                          utils/StackDeviceMemory.h:127-272
 * MI355X extensions (no reference counterpart; zero host->device copies):
 *   dietgpu_float_compress_batch_stride, dietgpu_float_decompress_batch_stride
 *
 * Conventions: `stream` is a hipStream_t (NULL = default stream); the
 * `res` arena is the reference's StackDeviceMemory& first argument; float
 * sizes / capacities are in float words, ANS sizes in bytes, *_size_dev
 * outputs are device arrays of uint32.  ANSCodecConfig / FloatCodecConfig are
 * passed flattened as (prob_bits, use_checksum[, float_type]).  float_type:
 * 1 fp16, 2 bf16, 3 fp32, 4 fp64.  Every call returns DIETGPU_OK or an error
 * code; dietgpu_last_error() returns the message (thread-local).  Checksum
 * mismatches on decode return DIETGPU_ERR_CHECKSUM after all outputs are
 * written (the reference returns ANSDecodeStatus / FloatDecompressStatus).
 */
#ifndef DIETGPU_C_H
#define DIETGPU_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DIETGPU_OK 0
#define DIETGPU_ERR_INVALID 1
#define DIETGPU_ERR_HIP 2
#define DIETGPU_ERR_CHECKSUM 3

typedef struct dietgpu_stack dietgpu_stack;

const char* dietgpu_last_error(void);
const char* dietgpu_version(void);

/* StackDeviceMemory: ptr == NULL allocates `bytes` (may be 0); otherwise the
 * caller-owned region [ptr, ptr+bytes) is managed without ownership. */
dietgpu_stack* dietgpu_stack_create(int device, void* ptr, size_t bytes);
void dietgpu_stack_destroy(dietgpu_stack* res);
size_t dietgpu_stack_max_usage(const dietgpu_stack* res);
void dietgpu_stack_reset_max_usage(dietgpu_stack* res);
size_t dietgpu_stack_size_total(const dietgpu_stack* res);

uint32_t dietgpu_get_max_compressed_size(uint32_t uncompressed_bytes);
uint32_t dietgpu_get_max_float_compressed_size(int float_type, uint32_t words);
uint32_t dietgpu_get_max_sparse_float_compressed_size(int float_type, uint32_t words);

/* ---- ANS byte codec ---- */
int dietgpu_ans_encode_batch_stride(dietgpu_stack* res, int prob_bits, int use_checksum,
                                    uint32_t num_in_batch, const void* in_dev,
                                    uint32_t in_per_batch_size, uint32_t in_per_batch_stride,
                                    const uint32_t* histogram_dev, void* out_dev,
                                    uint32_t out_per_batch_stride, uint32_t* out_batch_size_dev,
                                    void* stream);
int dietgpu_ans_encode_batch_pointer(dietgpu_stack* res, int prob_bits, int use_checksum,
                                     uint32_t num_in_batch, const void** in,
                                     const uint32_t* in_size, const uint32_t* histogram_dev,
                                     void** out, uint32_t* out_size_dev, void* stream);
int dietgpu_ans_encode_batch_split_size(dietgpu_stack* res, int prob_bits, int use_checksum,
                                        uint32_t num_in_batch, const void* in_dev,
                                        const uint32_t* in_split_sizes,
                                        const uint32_t* histogram_dev, void* out_dev,
                                        uint32_t out_stride, uint32_t* out_size_dev,
                                        void* stream);
int dietgpu_ans_decode_batch_stride(dietgpu_stack* res, int prob_bits, int use_checksum,
                                    uint32_t num_in_batch, const void* in_dev,
                                    uint32_t in_per_batch_stride, void* out_dev,
                                    uint32_t out_per_batch_stride,
                                    uint32_t out_per_batch_capacity, uint8_t* out_success_dev,
                                    uint32_t* out_size_dev, void* stream);
int dietgpu_ans_decode_batch_pointer(dietgpu_stack* res, int prob_bits, int use_checksum,
                                     uint32_t num_in_batch, const void** in, void** out,
                                     const uint32_t* out_capacity, uint8_t* out_success_dev,
                                     uint32_t* out_size_dev, void* stream);
int dietgpu_ans_decode_batch_split_size(dietgpu_stack* res, int prob_bits, int use_checksum,
                                        uint32_t num_in_batch, const void** in, void* out_dev,
                                        const uint32_t* out_split_sizes,
                                        uint8_t* out_success_dev, uint32_t* out_size_dev,
                                        void* stream);
int dietgpu_ans_get_compressed_info(dietgpu_stack* res, const void** in, uint32_t num_in_batch,
                                    uint32_t* out_sizes_dev, uint32_t* out_checksum_dev,
                                    void* stream);
int dietgpu_ans_get_compressed_info_device(dietgpu_stack* res, const void** in_dev,
                                           uint32_t num_in_batch, uint32_t* out_sizes_dev,
                                           uint32_t* out_checksum_dev, void* stream);

/* ---- float codec ---- */
int dietgpu_float_compress(dietgpu_stack* res, int float_type, int prob_bits, int use_checksum,
                           uint32_t num_in_batch, const void** in, const uint32_t* in_size,
                           void** out, uint32_t* out_size_dev, void* stream);
int dietgpu_float_compress_split_size(dietgpu_stack* res, int float_type, int prob_bits,
                                      int use_checksum, uint32_t num_in_batch,
                                      const void* in_dev, const uint32_t* in_split_sizes,
                                      void* out_dev, uint32_t out_stride,
                                      uint32_t* out_size_dev, void* stream);
int dietgpu_float_compress_sparse(dietgpu_stack* res, int float_type, int prob_bits,
                                  int use_checksum, uint32_t num_in_batch, const void** in,
                                  const uint32_t* in_size, void** out, uint32_t* out_size_dev,
                                  void* stream);
int dietgpu_float_decompress(dietgpu_stack* res, int float_type, int prob_bits,
                             int use_checksum, uint32_t num_in_batch, const void** in,
                             void** out, const uint32_t* out_capacity,
                             uint8_t* out_success_dev, uint32_t* out_size_dev, void* stream);
int dietgpu_float_decompress_split_size(dietgpu_stack* res, int float_type, int prob_bits,
                                        int use_checksum, uint32_t num_in_batch,
                                        const void** in, void* out_dev,
                                        const uint32_t* out_split_sizes,
                                        uint8_t* out_success_dev, uint32_t* out_size_dev,
                                        void* stream);
int dietgpu_float_decompress_sparse(dietgpu_stack* res, int float_type, int prob_bits,
                                    int use_checksum, uint32_t num_in_batch, const void** in,
                                    void** out, const uint32_t* out_capacity,
                                    uint8_t* out_success_dev, uint32_t* out_size_dev,
                                    void* stream);
int dietgpu_float_get_compressed_info(dietgpu_stack* res, const void** in,
                                      uint32_t num_in_batch, uint32_t* out_sizes_dev,
                                      uint32_t* out_types_dev, uint32_t* out_checksum_dev,
                                      void* stream);
int dietgpu_float_get_compressed_info_device(dietgpu_stack* res, const void** in_dev,
                                             uint32_t num_in_batch, uint32_t* out_sizes_dev,
                                             uint32_t* out_types_dev,
                                             uint32_t* out_checksum_dev, void* stream);

/* ---- MI355X extensions ---- */
int dietgpu_float_compress_batch_stride(dietgpu_stack* res, int float_type, int prob_bits,
                                        int use_checksum, uint32_t num_in_batch,
                                        const void* in_dev, uint32_t in_per_batch_words,
                                        uint64_t in_per_batch_stride_bytes, void* out_dev,
                                        uint64_t out_per_batch_stride_bytes,
                                        uint32_t* out_size_dev, void* stream);
int dietgpu_float_decompress_batch_stride(dietgpu_stack* res, int float_type, int prob_bits,
                                          int use_checksum, uint32_t num_in_batch,
                                          const void* in_dev, uint64_t in_per_batch_stride_bytes,
                                          void* out_dev, uint64_t out_per_batch_stride_bytes,
                                          uint32_t out_per_batch_capacity_words,
                                          uint8_t* out_success_dev, uint32_t* out_size_dev,
                                          void* stream);

/* Kernel timing hook used by bench.py: when enabled, every launch of the
 * named kernel family ("encode", "decode", "hist", "coalesce") is bracketed
 * by hipEvents on its own stream; query returns the summed milliseconds and
 * the launch count since the last reset (synchronises the recorded events). */
void dietgpu_profile_enable(int on);
/* record only kernel family `kernel` (NULL or "" = every family) */
void dietgpu_profile_filter(const char* kernel);
int dietgpu_profile_query(const char* kernel, double* total_ms, uint64_t* launches);
void dietgpu_profile_reset(void);

/* ---- compressor error reporting (MI355X extension) ----
 * The single-pass compressor's cross-workgroup waits (team barrier, look-back)
 * are bounded.  A wait that runs out POISONS its element instead of producing
 * a wrong archive: that element's out_size is written as 0 (no valid archive
 * is shorter than 544 bytes) and the device error word counts it.
 * dietgpu_device_error_count synchronises the current device and returns the
 * count since the last reset (reset != 0 clears it). */
uint32_t dietgpu_device_error_count(int reset);
/* Number of single-pass compressor team-barrier fallbacks since the last
 * reset (reset != 0 clears it): a workgroup that waited out the barrier
 * budget (dietgpu_set_barrier_budget) for its team's partial histograms and
 * counted its element from the input instead.  Archives are unchanged; a
 * nonzero count without a competing kernel or a forced budget means a slow
 * hand-off.  Synchronises the current device. */
uint32_t dietgpu_barrier_fallback_count(int reset);
/* Test hook: polls each such wait may make before it gives up (default
 * 1 << 24).  0 makes every wait that would have to wait fail at once, which
 * forces the error path deterministically for elements of more than one
 * team member.  Passed to the kernels as an argument. */
void dietgpu_set_spin_cap(uint32_t polls);
/* Test hook: how long (100 MHz ticks) a single-pass compressor workgroup
 * waits for the other members of its element's team before it counts the
 * element's histogram from the input itself (default 20000 = 200 us).  The
 * fallback keeps the compressor live when other kernels hold CUs; 0 forces
 * it for every team wait (archives are unchanged). */
void dietgpu_set_barrier_budget(uint32_t ticks);
/* Test hook: every k_encode workgroup of the fused three-kernel path waits
 * (63 - g % 64) * ticks (100 MHz) at its start, so the workgroups start
 * publishing in about reverse index order within every 64 (late publication
 * by dispatched lower workgroups; the single-pass k_pcompress carries no
 * hook, see tools/variants.py pskew).  Archives are unchanged; 0 = off. */
void dietgpu_set_dispatch_skew(uint32_t ticks);
/* Test hook: which compressor takes a float / byte batch that both can
 * compress.  0 (default): the size rule (csrc/codec.hip persistentPreferred;
 * INTEGRATION.md, "Which compressor runs"): a batch goes to the three-kernel
 * path when it has at most 256 work items (elements x 8-block items per
 * element) or when it fits one round of teams that cannot be XCD-aligned,
 * and to the single-pass compressor otherwise; byte archives with a
 * checksum always go single-pass (the three-kernel path has no prologue
 * normalisation for them) unless mode 2 is set; 1: the single-pass compressor whenever
 * the batch is eligible (16 B-aligned inputs, elements of at most 1 MiB of
 * symbols, no caller histogram); 2: always the three-kernel path.  Archives
 * are byte-identical whatever the mode; other values mean 0. */
void dietgpu_set_compress_path(int mode);

#ifdef __cplusplus
}
#endif

#endif /* DIETGPU_C_H */
