// Microbenchmark (dev tool): achievable HBM streaming rates on this device
// for 16 B-per-lane read / write / copy over 256 MiB buffers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
    u32x4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
    a[i] = u32x4{uint32_t(i), 1, 2, 3};
}
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) b[i] = a[i];
}

// each workgroup streams its own contiguous chunk (the histogram's pattern)
__global__ __launch_bounds__(256) void k_read_chunked(const u32x4* __restrict__ a, size_t n, size_t chunk,
                                                      uint32_t* out) {
  uint32_t acc = 0;
  const size_t b0 = size_t(blockIdx.x) * chunk, e = b0 + chunk < n ? b0 + chunk : n;
  for (size_t i = b0 + threadIdx.x; i < e; i += 256) {
    u32x4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t bytes = 256ull << 20, n = bytes / 16;
  u32x4 *a, *b, *c; uint32_t* o;
  hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&c, bytes); hipMalloc(&o, 4);
  hipMemset(a, 1, bytes); hipMemset(b, 2, bytes); hipMemset(c, 3, bytes);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (size_t chunkKB : {16, 64, 128, 512}) {
    const size_t chunk = chunkKB * 1024 / 16;
    const int grid = int(n / chunk);
    float ms; const int R = 10;
    hipEventRecord(e0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_read_chunked, dim3(grid), dim3(256), 0, 0, (r & 1) ? a : c, n, chunk, o);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("chunked %4zu KB/WG (grid %6d) read %.2f TB/s\n", chunkKB, grid, R * bytes / (ms * 1e-3) / 1e12);
  }
  for (int grid : {2048, 32768}) {
    float ms; const int R = 10;
    // alternate buffers so each pass misses the 256 MiB Infinity Cache
    hipEventRecord(e0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (r & 1) ? a : c, n, o);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("grid %5d read  %.2f TB/s\n", grid, R * bytes / (ms * 1e-3) / 1e12);
    hipEventRecord(e0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (r & 1) ? b : c, n);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("grid %5d write %.2f TB/s\n", grid, R * bytes / (ms * 1e-3) / 1e12);
    hipEventRecord(e0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (r & 1) ? a : c, b, n);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("grid %5d copy  %.2f TB/s (read+write bytes)\n", grid, R * 2 * bytes / (ms * 1e-3) / 1e12);
  }
  return 0;
}
