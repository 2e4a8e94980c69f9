// Microbenchmark (dev tool): latency/throughput structure of the rANS decode
// step on gfx950.  Each wave runs NC independent chains of the decode step
// (64-bit table read -> mad24/ballot/mbcnt -> ring read -> v_perm) over
// synthetic LDS data; occupancy is set with dynamic LDS.  Prints cycles per
// wave-step and chain-steps per SIMD per 1000 cycles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#define LDS __attribute__((address_space(3)))

template <int NC, bool kPhased, int kSeg, int kRingW>
__global__ __launch_bounds__(256) void k_chain(uint32_t steps, uint32_t* out, uint64_t* cyc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  LDS u32x2* lut = (LDS u32x2*)smem;                      // 1024 entries
  LDS uint16_t* ring = (LDS uint16_t*)(smem + 8192);       // 256 words per chain-half
  LDS uint16_t* seg = (LDS uint16_t*)(smem + 8192 + 4 * NC * 4 * kRingW);  // 8 x 64 u16 per chain
  uint32_t acc8[NC][2];
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (uint32_t i = tid; i < 1024; i += 256) {
    uint32_t pdf = 1 + (i * 2654435761u >> 24) % 64;
    lut[i] = u32x2{pdf | ((i & 255) << 24), i & 63};
  }
  for (uint32_t i = tid; i < 4 * NC * 2 * kRingW; i += 256) ring[i] = uint16_t(i * 40503u);
  __syncthreads();
  uint32_t hv = lane >= 32 ? ~0u : 0u;
  asm volatile("" : "+v"(hv));
  uint32_t x[NC];
  int32_t ptr[NC][2];
  LDS const uint16_t* rl[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    x[c] = (1u << 20) + lane * 977u + c * 131u;
    ptr[c][0] = 100000; ptr[c][1] = 100000;
    acc8[c][0] = acc8[c][1] = 0;
    rl[c] = ring + (w * NC + c) * 2 * kRingW + (hv & kRingW);
  }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t t = 0; t < steps; ++t) {
    u32x2 e[NC];
    uint32_t xn[NC], v[NC];
    bool rd[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) e[c] = lut[x[c] & 1023];
    if (kPhased) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      xn[c] = __umul24(e[c].x, x[c] >> 10) + e[c].y;
      rd[c] = xn[c] < (1u << 15);
      const uint64_t vote = __builtin_amdgcn_ballot_w64(rd[c]);
      const int32_t cLo = __popc(uint32_t(vote)), cHi = __popc(uint32_t(vote >> 32));
      const int32_t baseLo = ptr[c][0] - cLo;
      const int32_t diff = ptr[c][1] - ptr[c][0] - cHi;
      ptr[c][0] = baseLo;
      ptr[c][1] -= cHi;
      const uint32_t vbase = uint32_t(baseLo) + (hv & uint32_t(diff));
      const uint32_t idx = __builtin_amdgcn_mbcnt_hi(uint32_t(vote >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(uint32_t(vote), vbase));
      v[c] = rl[c][idx & (kRingW - 1)];
      if (kSeg == 1) seg[((w * NC + c) * 8 + (t & 7)) * 64 + lane] = uint16_t(e[c].x >> 16);
      if (kSeg == 2) {  // accumulate 8 symbols per lane, one ds_write_b64 per 8 steps
        const uint32_t k = t & 7;
        acc8[c][k >> 2] = __builtin_amdgcn_perm(e[c].x, acc8[c][k >> 2], 0x03020100u + 0 * k);
      }
    }
    if (kSeg == 2 && (t & 7) == 7) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        *(LDS u32x2*)(seg + ((w * NC + c) * 64 + lane) * 4) = u32x2{acc8[c][0], acc8[c][1]};
    }
    if (kPhased) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = __builtin_amdgcn_perm(xn[c], v[c], rd[c] ? 0x05040100u : 0x07060504u);
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) acc ^= x[c] ^ acc8[c][0] ^ acc8[c][1];
  if (kSeg) acc ^= seg[tid];
  out[blockIdx.x * 256 + tid] = acc;
  if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int NC, bool kPhased, int kSeg = 0, int kRingW = 256>
void run(int wavesPerSimd, int cus) {
  // WGs of 4 waves (one per SIMD); wavesPerSimd WGs per CU via LDS
  const uint32_t need = 8192 + 4 * NC * 4 * kRingW + (kSeg ? 4 * NC * 1024 : 0);
  const uint32_t lds = std::max<uint32_t>(need, 160 * 1024 / wavesPerSimd - 512);
  if (need > 160 * 1024 / wavesPerSimd) { printf("skip NC=%d wps=%d ring=%d seg=%d (needs %u B)\n", NC, wavesPerSimd, kRingW, kSeg, need); return; }
  const uint32_t steps = 4096;
  const int wgs = cus * wavesPerSimd;
  uint32_t* out; uint64_t* cyc;
  hipMalloc(&out, wgs * 256 * 4); hipMalloc(&cyc, wgs * 4 * 8);
  hipLaunchKernelGGL((k_chain<NC, kPhased, kSeg, kRingW>), dim3(wgs), dim3(256), lds, 0, 64, out, cyc);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((k_chain<NC, kPhased, kSeg, kRingW>), dim3(wgs), dim3(256), lds, 0, steps, out, cyc);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  std::vector<uint64_t> h(wgs * 4);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  double avg = 0; for (auto v : h) avg += v; avg /= h.size();
  const double perStep = avg / steps;
  printf("ring=%d seg=%d NC=%d phased=%d waves/SIMD=%d lds=%u: %.0f cyc/wave-step, %.1f cyc/chain-step/SIMD, kernel %.3f ms\n",
         kRingW, kSeg, NC, int(kPhased), wavesPerSimd, lds, perStep, perStep / (NC * wavesPerSimd), ms);
  hipFree(out); hipFree(cyc);
}

int main() {
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int wps : {4, 5, 6, 8}) {
    run<4, true, 0, 256>(wps, cus);
    run<4, true, 0, 128>(wps, cus);
    run<2, true, 0, 128>(wps, cus);
    run<4, true, 1, 128>(wps, cus);
  }
  return 0;
}
