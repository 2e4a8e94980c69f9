// LDS histogram cost on gfx950 for the compressor's per-symbol counting:
// cycles per wave-instruction of ds_add_u32 under several counter layouts,
// 4 workgroups of 256 threads per CU (the compressor's occupancy), symbols
// from (a) bf16 N(0,1) exponents (the c2 data: few hot bins) and (b) uniform
// bytes.  Each lane counts 64 symbols held in 16 registers, 16 times over.
//   layout 0: 8 columns (lane & 7), row stride 9, u32 counters (the k_pcompress v4 layout)
//   layout 1: 32 columns (lane & 31), row stride 32, u16 pairs (bin >> 1 rows)
//   layout 2: 16 columns (lane & 15), row stride 16, u16 pairs
//   layout 3: 64 columns (lane), row stride 64, u16 pairs
//   layout 4: 32 columns, row stride 33, u32 counters
// Build: hipcc --offload-arch=gfx950 -O3 lds_hist.hip -o lds_hist
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

constexpr int kReps = 16;

template <int L>
__global__ __launch_bounds__(256) void k(const uint32_t* sym, uint32_t* out, unsigned long long* cyc) {
  __shared__ uint32_t h[256 * 33];
  for (int i = threadIdx.x; i < 256 * 33; i += 256) h[i] = 0;
  uint32_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = sym[(blockIdx.x * 16 + i) * 256 + threadIdx.x];
  const uint32_t lane = threadIdx.x & 63;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < kReps; ++r) {
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const uint32_t b = __builtin_amdgcn_ubfe(s[t / 4], 8 * (t & 3), 8);
      uint32_t addr, v = 1;
      if constexpr (L == 0) addr = b * 9 + (lane & 7);
      if constexpr (L == 1) addr = (b >> 1) * 32 + (lane & 31), v = 1u << (16 * (b & 1));
      if constexpr (L == 2) addr = (b >> 1) * 16 + (lane & 15), v = 1u << (16 * (b & 1));
      if constexpr (L == 3) addr = (b >> 1) * 64 + lane, v = 1u << (16 * (b & 1));
      if constexpr (L == 4) addr = b * 33 + (lane & 31);
      __hip_atomic_fetch_add(&h[addr], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  uint32_t acc = 0;
  for (int i = threadIdx.x; i < 256 * 33; i += 256) acc += h[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int L>
double run(const uint32_t* dsym, int blocks) {
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 4 * 8);
  k<L><<<blocks, 256>>>(dsym, out, cyc);
  k<L><<<blocks, 256>>>(dsym, out, cyc);
  hipDeviceSynchronize();
  std::vector<unsigned long long> hc(blocks * 4);
  hipMemcpy(hc.data(), cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double sum = 0;
  for (auto c : hc) sum += double(c);
  hipFree(out);
  hipFree(cyc);
  return sum / hc.size() / (double(kReps) * 64);
}

int main() {
  const int blocks = 1024;  // 4 per CU
  std::vector<uint32_t> sym(size_t(blocks) * 16 * 256);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd;
  uint32_t* d;
  hipMalloc(&d, sym.size() * 4);
  for (int dist = 0; dist < 2; ++dist) {
    for (auto& w : sym) {
      w = 0;
      for (int b = 0; b < 4; ++b) {
        uint32_t v;
        if (dist == 0) {
          float f = nd(rng);
          uint32_t u;
          std::memcpy(&u, &f, 4);
          v = (u >> 23) & 0xff;  // bf16 exponent byte = fp32 exponent
        } else {
          v = rng() & 0xff;
        }
        w |= v << (8 * b);
      }
    }
    hipMemcpy(d, sym.data(), sym.size() * 4, hipMemcpyHostToDevice);
    const char* dn = dist == 0 ? "bf16-exponent" : "uniform-byte";
    std::printf("%s: layout0 %.2f  layout1 %.2f  layout2 %.2f  layout3 %.2f  layout4 %.2f cycles/wave-instr\n", dn,
                run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks));
  }
  hipFree(d);
  return 0;
}
