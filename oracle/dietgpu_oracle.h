/*
 * dietgpu_oracle.h -- CPU restatement of the NSagan271/dietgpu_fork codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in dietgpu_fork_amd/ may include, link
 * or call this.  It is used by tests/ (as the parity checker), by
 * __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline leg.
 *
 * All citations are relative to /root/reference/ (reference @ 2025-02-04).
 * Parity is pinned by the reference's own known-answer tests
 * (ans/ANSStatisticsTest.cu:127-207, ans/BatchPrefixSumTest.cu) and by an
 * independent pure-Python restatement (tests/pyref.py); see DESIGN.md.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* --- sizes (ans/GpuANSEncode.cu:13-25, float/GpuFloatCompress.cu:23-48,
 *     float/GpuSparseFloatCompress.cu:16-24) --- */
uint32_t or_max_compressed_size(uint32_t uncompressed_bytes);
uint32_t or_max_float_compressed_size(int float_type, uint32_t num_words);
uint32_t or_max_sparse_float_compressed_size(int float_type, uint32_t num_words);
uint32_t or_float_uncomp_data_size(int float_type, uint32_t num_words);

/* --- ANS statistics (ans/GpuANSStatistics.cuh:21-367) --- */
void or_ans_histogram(const uint8_t* in, size_t n, uint32_t hist[256]);
/* pdf/cdf of the quantized table; returns 0 on success.  total == 0 leaves
 * pdf/cdf zeroed (the reference leaves them untouched). */
int or_ans_normalize(const uint32_t hist[256], uint32_t total, int prob_bits,
                     uint32_t pdf[256], uint32_t cdf[256]);
uint32_t or_checksum(const uint8_t* in, size_t n);

/* --- ANS byte codec (ans/GpuANSEncode.cuh, ans/GpuANSDecode.cuh) ---
 * Encodes one batch element into `out` (capacity out_cap bytes).  If hist is
 * non-NULL it is used instead of computing the histogram.  Returns the archive
 * size in bytes, or 0 on error (capacity too small). */
uint32_t or_ans_encode(const uint8_t* in, uint32_t n, int prob_bits,
                       int use_checksum, const uint32_t* hist, uint8_t* out,
                       size_t out_cap);
/* Decodes one archive.  Returns 0 on success, 1 if the output capacity is too
 * small (size still reported), 2 on a header/format error, 3 on checksum
 * mismatch.  *out_size receives the decoded byte count. */
int or_ans_decode(const uint8_t* archive, int prob_bits, int use_checksum,
                  uint8_t* out, uint32_t out_cap, uint32_t* out_size);
/* header readout (ans/GpuANSInfo.cuh:16-37): returns uncompressed bytes */
uint32_t or_ans_info(const uint8_t* archive, uint32_t* checksum);
uint32_t or_ans_archive_size(const uint8_t* archive);

/* --- float codec (float/GpuFloatUtils.cuh, GpuFloatCompress.cuh,
 *     GpuFloatDecompress.cuh).  float_type: 1 fp16, 2 bf16, 3 fp32, 4 fp64.
 *     num_words counts floats. --- */
uint32_t or_float_compress(int float_type, const void* in, uint32_t num_words,
                           int prob_bits, int use_checksum, uint8_t* out,
                           size_t out_cap);
int or_float_decompress(const uint8_t* archive, int float_type, int prob_bits,
                        int use_checksum, void* out, uint32_t out_cap_words,
                        uint32_t* out_words);

/* --- sparse float codec (float/GpuSparseFloatCompress.cuh,
 *     GpuSparseFloatDecompress.cuh) --- */
uint32_t or_sparse_float_compress(int float_type, const void* in,
                                  uint32_t num_words, int prob_bits,
                                  int use_checksum, uint8_t* out,
                                  size_t out_cap);
int or_sparse_float_decompress(const uint8_t* archive, int float_type,
                               int prob_bits, int use_checksum, void* out,
                               uint32_t out_cap_words, uint32_t* out_words);

/* --- batch helpers used by the CPU baseline (serial unless threads > 1) --- */
double or_time_float_roundtrip(int float_type, const void* in,
                               uint32_t num_in_batch, uint32_t words_each,
                               size_t in_stride_bytes, int prob_bits,
                               int threads, uint64_t* comp_bytes_total,
                               double* enc_seconds, double* dec_seconds);
double or_time_ans_roundtrip(const uint8_t* in, uint32_t num_in_batch,
                             uint32_t bytes_each, size_t in_stride_bytes,
                             int prob_bits, int threads,
                             uint64_t* comp_bytes_total, double* enc_seconds,
                             double* dec_seconds);

#ifdef __cplusplus
}
#endif
