// Issue cost of the VALU ops on the rANS encode step (gfx950): cycles per
// wave-instruction for v_mul_hi_u32, v_mul_lo_u32, v_mul_u32_u24 and
// v_add_u32, 8 independent chains, 1 and 4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1) + i * 977u;
  const uint32_t c = seed | 1u;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if constexpr (OP == 1) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if constexpr (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if constexpr (OP == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, int blocks) {
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 4 * 8);
  k<OP><<<blocks, 256>>>(out, cyc, 12345u);
  k<OP><<<blocks, 256>>>(out, cyc, 12345u);
  hipDeviceSynchronize();
  unsigned long long* h = new unsigned long long[blocks * 4];
  hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double sum = 0;
  for (int i = 0; i < blocks * 4; ++i) sum += double(h[i]);
  const double perInst = sum / (blocks * 4) / (double(kIters) * 8);
  std::printf("%-16s blocks %5d (waves/SIMD %d): %.2f cycles per wave-instruction\n", name, blocks,
              blocks / 256, perInst);
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int blocks : {256, 1024}) {
    run<0>("v_mul_hi_u32", blocks);
    run<3>("v_mul_lo_u32", blocks);
    run<1>("v_mul_u32_u24", blocks);
    run<2>("v_add_u32", blocks);
  }
  return 0;
}
