/*
 * dietgpu_testhooks.h -- test-only entry points (libdietgpu_testhooks.so).
 *
 * Not part of the drop-in boundary (include/dietgpu_c.h) and not linked into
 * the product library libdietgpu_amd.so: the GPU tests load this library
 * beside it.  Return codes as in dietgpu_c.h; dietgpu_test_last_error()
 * holds the message of this thread's last failed call.
 */
#ifndef DIETGPU_TESTHOOKS_H
#define DIETGPU_TESTHOOKS_H

#include <stddef.h>
#include <stdint.h>

#include "dietgpu_c.h"

#ifdef __cplusplus
extern "C" {
#endif

const char* dietgpu_test_last_error(void);
/* Enqueue on `stream` a kernel of `workgroups` 256-thread workgroups that
 * each hold `lds_bytes` of LDS for `micros` microseconds (<= 1 s) and exit:
 * compute units held by another kernel while the compressor runs
 * (tests/test_gpu_progress.py). */
int dietgpu_test_occupy(void* stream, uint32_t micros, uint32_t workgroups, uint32_t lds_bytes);
/* hist_dev[b * 256 + s] = count of byte value s in element b of a stride
 * batch (nb <= 65535 elements of `size` bytes, `stride` bytes apart),
 * computed by the compressor's own histogram kernel (k_hist<0>, chunked as
 * the three-kernel path chunks it).  Replaces the reference's
 * ansHistogramBatch as its ANSStatisticsTest.cu:44-95 calls it
 * (ans/GpuANSStatistics.cuh:113-143). */
int dietgpu_test_histogram(dietgpu_stack* res, uint32_t nb, const void* in_dev, uint32_t size,
                           uint32_t stride, uint32_t* hist_dev, void* stream);

/* magic_dev[q] (q = 0 .. 2048) = the 32-bit division magic of pdf q as the
 * compressors compute it in registers (encMagicReg, csrc/encode.h: v_rcp_f64,
 * two Newton steps, an exact fix-up); q 0 -> 0, q 1 -> 0xffffffff.  Checked
 * against the closed form ceil(2^(32 + ceil(log2 q) - 1) / q) by the GPU tests;
 * the magic replaces the division x / pdf of the reference's encode step
 * (ans/GpuANSEncode.cuh:63-89). */
int dietgpu_test_enc_magic(uint32_t* magic_dev, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DIETGPU_TESTHOOKS_H */
