#include <hip/hip_runtime.h>
#include <cstdio>
template <int N> struct Chunk { uint32_t off, n; uint32_t w[N]; };
template <int N>
__global__ void k_table(uint32_t* dst, Chunk<N> c) {
  for (uint32_t i = threadIdx.x; i < c.n; i += blockDim.x) dst[c.off + i] = c.w[i];
}
int main() {
  uint32_t* d; hipMalloc(&d, 1 << 20);
  auto test = [&](auto tag) {
    constexpr int N = decltype(tag)::value;
    Chunk<N> c; c.off = 0; c.n = N; for (int i = 0; i < N; ++i) c.w[i] = i * 7 + 1;
    k_table<N><<<1, 256>>>(d, c);
    hipError_t e = hipGetLastError(); hipError_t e2 = hipDeviceSynchronize();
    static uint32_t h[1 << 16]; hipMemcpy(h, d, N * 4, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < N; ++i) bad += h[i] != uint32_t(i * 7 + 1);
    printf("N=%d bytes=%zu launch=%s sync=%s bad=%d\n", N, sizeof(c), hipGetErrorString(e), hipGetErrorString(e2), bad);
  };
  test(std::integral_constant<int, 1000>{});
  test(std::integral_constant<int, 2000>{});
  test(std::integral_constant<int, 4000>{});
  // timing: 200 back-to-back launches of the 4 KB variant
  Chunk<1000> c; c.off = 0; c.n = 1000;
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < 200; ++i) k_table<1000><<<1, 256>>>(d, c);
  hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
  printf("avg per 4KB table launch %.2f us\n", ms * 1000 / 200);
  return 0;
}
