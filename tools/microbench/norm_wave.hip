// Microbenchmark (dev tool): cycles of the one-wave normalisation that sits on
// k_pcompress's hand-off window (normalizeWave + encTableEntryReg, encode.h)
// for the histogram of one c2 element (524,288 bf16 N(0,1) words; symbol =
// exponent byte), and of the magic computed three ways: f64 division (the
// product), v_rcp_f64 + integer fix-up, and the kMagic table in global
// memory.  Also checks that the rcp form equals the exact magic for every
// pdf 2 .. 2048.  One workgroup, wave 0 timed with s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I dietgpu_fork_amd/csrc -I include \
//     tools/microbench/norm_wave.hip -o tools/microbench/norm_wave
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "encode.h"

using namespace dietgpu;

__device__ __forceinline__ uint32_t magicRcp(uint32_t q, uint32_t shift) {
  const uint64_t num = 1ull << (32 + shift);
  uint64_t m = uint64_t(double(num) * __builtin_amdgcn_rcp(double(q)));
  if (m * q > num) m -= 1;
  else if ((m + 1) * q <= num) m += 1;
  return uint32_t(m + (m * q != num));
}

__global__ __launch_bounds__(256) void k_norm(const uint32_t* hist, uint32_t total, int pb, int reps,
                                              uint64_t* cyc, uint32_t* outTbl, uint32_t* bad) {
  __shared__ __attribute__((aligned(16))) uint32_t tblS[kNumSymbols * 4];
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x == 0) *bad = 0;
  __syncthreads();
  // exhaustive check of the rcp magic (all waves)
  for (uint32_t q = 2 + threadIdx.x; q <= 2048; q += 256) {
    const uint32_t sh = 31 - __clz(q - 1);
    if (magicRcp(q, sh) != kMagic.m[q]) atomicAdd(bad, 1u);
  }
  if (threadIdx.x >= 64) return;
  uint64_t tN = 0, tT = 0, tR = 0, tG = 0;
  for (int r = 0; r < reps; ++r) {
    uint32_t c[4], cdf[4];
    for (int j = 0; j < 4; ++j) c[j] = hist[4 * lane + j];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    normalizeWave(c, cdf, total, pb);
    asm volatile("" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]));
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 4; ++j) {
      const uint4 e = encTableEntryReg(c[j], cdf[j], pb);
      *(lp<u32x4>)&tblS[4 * (4 * lane + j)] = u32x4{e.x, e.y, e.z, e.w};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t2 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 4; ++j) {
      const uint32_t q = c[j];
      const uint32_t sh = q > 1 ? 31 - __clz(q - 1) : 0;
      const uint32_t m = q > 1 ? magicRcp(q, sh) : (q ? 0xffffffffu : 0u);
      const uint4 e = encEntryPack(q, cdf[j], m, sh, pb);
      *(lp<u32x4>)&tblS[4 * (4 * lane + j)] = u32x4{e.x, e.y, e.z, e.w};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t3 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 4; ++j) {
      const uint4 e = encTableEntry(c[j], cdf[j], pb);
      *(lp<u32x4>)&tblS[4 * (4 * lane + j)] = u32x4{e.x, e.y, e.z, e.w};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t4 = __builtin_amdgcn_s_memtime();
    if (r > 0) {
      tN += t1 - t0;
      tT += t2 - t1;
      tR += t3 - t2;
      tG += t4 - t3;
    }
  }
  for (int k = 0; k < 16; ++k) outTbl[16 * lane + k] = tblS[16 * lane + k];
  if (lane == 0) {
    cyc[0] = tN / (reps - 1);
    cyc[1] = tT / (reps - 1);
    cyc[2] = tR / (reps - 1);
    cyc[3] = tG / (reps - 1);
  }
}

int main() {
  // histogram of one c2 element: bf16 exponent bytes of N(0,1) fp32 truncated
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  const uint32_t n = 524288;
  std::vector<uint32_t> h(256, 0);
  for (uint32_t i = 0; i < n; ++i) {
    float f = nd(rng);
    uint32_t u;
    std::memcpy(&u, &f, 4);
    const uint16_t w = uint16_t(u >> 16);
    h[(w >> 7) & 0xff]++;
  }
  uint32_t *dh, *dt, *bad;
  uint64_t* dc;
  hipMalloc(&dh, 1024);
  hipMalloc(&dt, 16384);
  hipMalloc(&dc, 64);
  hipMalloc(&bad, 4);
  hipMemcpy(dh, h.data(), 1024, hipMemcpyHostToDevice);
  for (int pb : {9, 10, 11}) {
    k_norm<<<1, 256>>>(dh, n, pb, 20, dc, dt, bad);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    uint64_t c[4];
    uint32_t b = 0;
    hipMemcpy(c, dc, 32, hipMemcpyDeviceToHost);
    hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    // s_memtime: the shader clock
    printf("pb %d: normalizeWave %llu cyc, table f64-div %llu, table rcp %llu, table kMagic %llu; rcp magic mismatches %u\n",
           pb, (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2],
           (unsigned long long)c[3], b);
  }
  return 0;
}
