// Memory-pattern model of a compressor that reads each item twice: a
// histogram read of the NEXT round's item and a re-read of the CURRENT item
// for the encode (hoping the re-read, one round later, comes from the
// Infinity Cache).  Against the single-read pattern of k_pcompress.  c2 sizes:
// 1024 workgroups, 4 rounds of 64 KiB items (256 MiB input), 32 KiB of raw
// bytes (8 B stores) and 11.5 KiB of ANS payload (16 B stores) written per item.
// Build: hipcc --offload-arch=gfx950 -O3 hist_ahead.hip -o hist_ahead
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kItemVec = (64 << 10) / 16;   // 16 B vectors per item
constexpr int kRawVec = (32 << 10) / 8;     // 8 B raw stores per item
constexpr int kArchVec = 736;               // 16 B payload stores per item

template <int kPolicy>  // 0 plain, 1 nt
__device__ __forceinline__ uint32_t readItem(const u32x4* p) {
  uint32_t acc = 0;
  for (int i0 = threadIdx.x; i0 < kItemVec; i0 += 256 * 8) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = kPolicy ? __builtin_nontemporal_load(p + i0 + 256 * k) : p[i0 + 256 * k];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  return acc;
}

__device__ __forceinline__ void writeItem(u32x2* raw, u32x4* arch, uint32_t acc, int ntStores) {
  for (int i = threadIdx.x; i < kRawVec; i += 256) {
    if (ntStores) __builtin_nontemporal_store(u32x2{acc, uint32_t(i)}, raw + i);
    else raw[i] = u32x2{acc, uint32_t(i)};
  }
  for (int i = threadIdx.x; i < kArchVec; i += 256) arch[i] = u32x4{acc, 1, 2, uint32_t(i)};
}

// mode 0: single read per item (k_pcompress); mode 1: hist-ahead, re-read nt;
// mode 2: hist-ahead, re-read plain; mode 3: hist-ahead, both reads nt;
// mode 4: histogram read only (no re-read, no stores)
__global__ __launch_bounds__(256) void k_pattern(const u32x4* in, u32x2* raw, u32x4* arch, int rounds, int mode,
                                                 int ntStores, uint32_t* sink) {
  const int G = gridDim.x, w = blockIdx.x;
  uint32_t acc = 0;
  auto item = [&](int r) { return size_t(r) * G + w; };
  if (mode == 0) {
    for (int r = 0; r < rounds; ++r) {
      acc ^= readItem<1>(in + item(r) * kItemVec);
      writeItem(raw + item(r) * kRawVec, arch + item(r) * kArchVec, acc, ntStores);
    }
  } else if (mode == 4) {
    for (int r = 0; r < rounds; ++r) acc ^= readItem<0>(in + item(r) * kItemVec);
  } else {
    for (int r = 0; r <= rounds; ++r) {
      if (r < rounds)
        acc ^= mode == 3 ? readItem<1>(in + item(r) * kItemVec) : readItem<0>(in + item(r) * kItemVec);
      if (r > 0) {
        const size_t it = item(r - 1);
        acc ^= mode == 2 ? readItem<0>(in + it * kItemVec) : readItem<1>(in + it * kItemVec);
        writeItem(raw + it * kRawVec, arch + it * kArchVec, acc, ntStores);
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_scrub(const u32x4* a, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) acc ^= a[i].x;
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const int G = 1024, R = 4;
  u32x4 *in, *arch, *scrub;
  u32x2* raw;
  uint32_t* sink;
  (void)hipMalloc(&in, size_t(G) * R * kItemVec * 16);
  (void)hipMalloc(&raw, size_t(G) * R * kRawVec * 8);
  (void)hipMalloc(&arch, size_t(G) * R * kArchVec * 16);
  (void)hipMalloc(&scrub, 1ull << 30);
  (void)hipMalloc(&sink, 4);
  (void)hipMemset(in, 1, size_t(G) * R * kItemVec * 16);
  (void)hipMemset(scrub, 2, 1ull << 30);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"single-read (k_pcompress)", "hist-ahead, re-read nt", "hist-ahead, re-read plain",
                         "hist-ahead, both nt", "hist read only"};
  for (int ntS = 0; ntS < 2; ++ntS) {
    for (int mode = 0; mode < 5; ++mode) {
      for (int cold = 0; cold < 2; ++cold) {
        float best = 1e9, sum = 0;
        const int trials = 12;
        for (int t = 0; t < trials + 2; ++t) {
          if (cold) k_scrub<<<2048, 256>>>(scrub, (1ull << 30) / 16, sink);
          (void)hipEventRecord(e0);
          k_pattern<<<G, 256>>>(in, raw, arch, R, mode, ntS, sink);
          (void)hipEventRecord(e1);
          (void)hipEventSynchronize(e1);
          float ms = 0;
          (void)hipEventElapsedTime(&ms, e0, e1);
          if (t >= 2) {
            best = ms < best ? ms : best;
            sum += ms;
          }
        }
        printf("%-28s stores %-5s %-5s best %7.1f us  mean %7.1f us\n", names[mode], ntS ? "nt" : "plain",
               cold ? "cold" : "warm", best * 1e3, sum / trials * 1e3);
      }
    }
  }
  return 0;
}
