// Does a second pass over a buffer read just now come from the MALL
// (Infinity Cache) instead of HBM?  Read pass A over the whole buffer in
// ascending chunk order, then pass B ascending or descending (descending
// meets the most recently read chunks first), timed with events; buffer sizes
// around the MALL capacity.  A 512 MiB scrub buffer is read between trials.
// Build: hipcc --offload-arch=gfx950 -O3 mall_reread.hip -o mall_reread
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// workgroup b reads chunk (rev ? nChunks - 1 - b' : b') for b' = b, b + grid, ...
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, size_t nChunks, size_t chunk, int rev,
                                              uint32_t* out) {
  uint32_t acc = 0;
  for (size_t c = blockIdx.x; c < nChunks; c += gridDim.x) {
    const size_t cc = rev ? nChunks - 1 - c : c;
    const u32x4* p = a + cc * chunk;
    for (size_t i = threadIdx.x; i < chunk; i += 256) {
      const u32x4 v = __builtin_nontemporal_load(p + i) ;
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_read_plain(const u32x4* __restrict__ a, size_t nChunks, size_t chunk, int rev,
                                                    uint32_t* out) {
  uint32_t acc = 0;
  for (size_t c = blockIdx.x; c < nChunks; c += gridDim.x) {
    const size_t cc = rev ? nChunks - 1 - c : c;
    const u32x4* p = a + cc * chunk;
    for (size_t i = threadIdx.x; i < chunk; i += 256) {
      const u32x4 v = p[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t chunk = (64 << 10) / 16;  // 64 KiB per chunk
  u32x4 *buf, *scrub;
  uint32_t* o;
  (void)hipMalloc(&buf, 1ull << 30);
  (void)hipMalloc(&scrub, 1ull << 30);
  (void)hipMalloc(&o, 4);
  (void)hipMemset(buf, 1, 1ull << 30);
  (void)hipMemset(scrub, 2, 1ull << 30);
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreate(&e2);
  const int grid = 2048;
  for (int nt = 0; nt < 2; ++nt) {
    for (size_t mib : {64, 128, 192, 256, 384, 512}) {
      const size_t bytes = mib << 20, nChunks = bytes / 16 / chunk;
      for (int rev = 0; rev < 2; ++rev) {
        float best0 = 1e9, best1 = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
          k_read_plain<<<grid, 256>>>(scrub, (1ull << 30) / 16 / chunk, chunk, 0, o);
          (void)hipEventRecord(e0);
          if (nt) k_read<<<grid, 256>>>(buf, nChunks, chunk, 0, o);
          else k_read_plain<<<grid, 256>>>(buf, nChunks, chunk, 0, o);
          (void)hipEventRecord(e1);
          if (nt) k_read<<<grid, 256>>>(buf, nChunks, chunk, rev, o);
          else k_read_plain<<<grid, 256>>>(buf, nChunks, chunk, rev, o);
          (void)hipEventRecord(e2);
          (void)hipEventSynchronize(e2);
          float t0, t1;
          (void)hipEventElapsedTime(&t0, e0, e1);
          (void)hipEventElapsedTime(&t1, e1, e2);
          if (t0 < best0) best0 = t0;
          if (t1 < best1) best1 = t1;
        }
        std::printf("%s %4zu MiB: pass A %7.1f us (%6.2f TB/s)  pass B %s %7.1f us (%6.2f TB/s)\n",
                    nt ? "nt   " : "plain", mib, best0 * 1e3, bytes / (best0 * 1e-3) / 1e12, rev ? "desc" : "asc ",
                    best1 * 1e3, bytes / (best1 * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
