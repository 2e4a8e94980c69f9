// Device-side building blocks shared by all kernels (gfx950 / wave64).
#pragma once

#include "batch.h"
#include "common.h"

namespace dietgpu {

// Pointers into HBM carry address_space(1) so hipcc emits global_* (not
// flat_*) memory instructions: flat ops count on both vmcnt and lgkmcnt and
// force s_waitcnt vmcnt(0) lgkmcnt(0) at every LDS use.
#define DG_G __attribute__((address_space(1)))
template <typename T>
using gp = DG_G T*;

// LDS pointers (address_space(3)): ds_* instructions with 32-bit addresses
#define DG_L __attribute__((address_space(3)))
template <typename T>
using lp = DG_L T*;

template <typename T>
__device__ __forceinline__ gp<T> G(T* p) {
  return (gp<T>)p;
}

__device__ __forceinline__ gp<uint8_t> startOf(const BatchDesc& d, uint32_t b) {
  return G(d.start(b));
}

// 8 / 16-byte global accesses through native vector types (HIP's uint2 /
// uint4 classes cannot bind address_space(1) references)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld16(gp<const void> p) {
  const u32x4 v = *(gp<const u32x4>)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(gp<void> p, uint4 v) {
  *(gp<u32x4>)p = u32x4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint2 ld8(gp<const void> p) {
  const u32x2 v = *(gp<const u32x2>)p;
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void st8(gp<void> p, uint2 v) {
  *(gp<u32x2>)p = u32x2{v.x, v.y};
}
// Streaming variants (non-temporal): for data read or written exactly once in
// a call -- the compressor's input, the decompressor's output -- so that the
// caches (L2, MALL) keep the archives, which the other direction reads next.
__device__ __forceinline__ uint4 ld16nt(gp<const void> p) {
  const u32x4 v = __builtin_nontemporal_load((gp<const u32x4>)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16nt(gp<void> p, uint4 v) {
  __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (gp<u32x4>)p);
}
__device__ __forceinline__ void st8nt(gp<void> p, uint2 v) {
  __builtin_nontemporal_store(u32x2{v.x, v.y}, (gp<u32x2>)p);
}

template <int FT>
struct FloatTraits;
template <>
struct FloatTraits<0> {  // raw bytes (ANS codec)
  using WordT = uint8_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<1> {
  using WordT = uint16_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<2> {
  using WordT = uint16_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<3> {
  using WordT = uint32_t;
  static constexpr int kSegs = 1;
};
template <>
struct FloatTraits<4> {
  using WordT = uint64_t;
  static constexpr int kSegs = 2;
};

__device__ __forceinline__ uint32_t rotl32(uint32_t v, int s) {
  return (v << s) | (v >> (32 - s));
}
__device__ __forceinline__ uint32_t rotr32(uint32_t v, int s) {
  return (v >> s) | (v << (32 - s));
}
__device__ __forceinline__ uint64_t rotl64(uint64_t v, int s) {
  return (v << s) | (v >> (64 - s));
}

// ANS symbol(s) of one word, FloatTypeInfo<FT>::split
// (float/GpuFloatUtils.cuh:190-370)
template <int FT>
__device__ __forceinline__ uint32_t compOf(typename FloatTraits<FT>::WordT w, int seg) {
  if constexpr (FT == 0) {
    return w;
  } else if constexpr (FT == 1) {
    return uint32_t(w) >> 8;
  } else if constexpr (FT == 2) {
    return (uint32_t(w) >> 7) & 0xffu;
  } else if constexpr (FT == 3) {
    return rotl32(w, 1) >> 24;
  } else {
    const uint64_t v = rotl64(w, 1);
    return seg == 0 ? uint32_t(v >> 56) : uint32_t(v >> 48) & 0xffu;
  }
}

// ---------------------------------------------------------------------------
// reductions / scans for NT-thread workgroups (NT multiple of 64)
// ---------------------------------------------------------------------------
// Wave64 sum / inclusive scan on the VALU: DPP within rows of 16 lanes, then
// v_readlane across the four rows -- no LDS-pipe shuffles (ds_bpermute),
// whose round trips dominate these short latency-bound sequences.  Whole
// wave (every lane active).
__device__ __forceinline__ uint32_t waveSum(uint32_t v) {
  v += uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
  v += uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
  v += uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x141, 0xF, 0xF, true));  // row_half_mirror
  v += uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x140, 0xF, 0xF, true));  // row_mirror
  return uint32_t(__builtin_amdgcn_readlane(int(v), 0)) + uint32_t(__builtin_amdgcn_readlane(int(v), 16)) +
         uint32_t(__builtin_amdgcn_readlane(int(v), 32)) + uint32_t(__builtin_amdgcn_readlane(int(v), 48));
}
__device__ __forceinline__ uint32_t waveXor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t waveInclusiveScan(uint32_t v) {
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xF, 0xF, true));  // row_shr:1
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xF, 0xF, true));  // row_shr:2
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xF, 0xF, true));  // row_shr:4
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xF, 0xF, true));  // row_shr:8
  const uint32_t r0 = uint32_t(__builtin_amdgcn_readlane(int(v), 15));
  const uint32_t r1 = r0 + uint32_t(__builtin_amdgcn_readlane(int(v), 31));
  const uint32_t r2 = r1 + uint32_t(__builtin_amdgcn_readlane(int(v), 47));
  const uint32_t row = (threadIdx.x & 63) >> 4;
  return v + (row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}

template <int NT>
__device__ __forceinline__ uint32_t blockSum(uint32_t v, uint32_t* smem) {
  constexpr int W = NT / 64;
  v = waveSum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) smem[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) t += smem[i];
  return t;
}
template <int NT>
__device__ __forceinline__ uint32_t blockExclusiveScan(uint32_t v, uint32_t* smem,
                                                       uint32_t* total) {
  constexpr int W = NT / 64;
  const uint32_t inc = waveInclusiveScan(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 63) smem[threadIdx.x >> 6] = inc;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const uint32_t s = smem[i];
    before += (i < int(threadIdx.x >> 6)) ? s : 0u;
    all += s;
  }
  if (total) *total = all;
  return before + inc - v;
}

// sc1 (agent-scope relaxed) loads / stores: the cross-workgroup hand-offs'
// accesses (MI355X_MICROARCH.md, sc1 loads in place of an acquire)
__device__ __forceinline__ uint32_t ldSc1(gp<const uint32_t> p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// four consecutive words as two 8 B sc1 loads (each word carries its own tag,
// so the two halves need not be read at one instant)
__device__ __forceinline__ u32x4 ldSc1x4(gp<const u32x4> p) {
  gp<const uint64_t> q = (gp<const uint64_t>)p;
  const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return u32x4{uint32_t(a), uint32_t(a >> 32), uint32_t(b), uint32_t(b >> 32)};
}
// Sixteen bytes of a tagged-granule row in ONE sc1 load (a buffer load: the
// atomic-load path only has 8 B forms).  Every word carries its own epoch tag,
// so the load need not be single-copy atomic.  base: wave-uniform; byteOff:
// per lane, below 2^31.
#if defined(__HIP_DEVICE_COMPILE__)
using BufRsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ BufRsrc bufOf(gp<const void> base) {
  // dword 3: the raw-buffer format word of gfx9 (CK_BUFFER_RESOURCE_3RD_DWORD)
  return __builtin_amdgcn_make_buffer_rsrc((void*)(const void*)base, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ u32x4 ldSc1x4(BufRsrc r, uint32_t byteOff) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, byteOff, 0, /*sc1*/ 16);
}
#else  // host pass of the kernel templates: never called
struct BufRsrc {};
__device__ __forceinline__ BufRsrc bufOf(gp<const void>) { return {}; }
__device__ __forceinline__ u32x4 ldSc1x4(BufRsrc, uint32_t) { return u32x4{0, 0, 0, 0}; }
#endif
__device__ __forceinline__ void stSc1(gp<uint32_t> p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Test hook (dietgpu_set_dispatch_skew): workgroup g first waits
// (63 - g % 64) * skew ticks of the 100 MHz clock, so the workgroups start in
// about reverse index order within every 64.  One lane.
__device__ __forceinline__ void skewDelay(uint32_t skew) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t g = blockIdx.y * gridDim.x + blockIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t d = uint64_t(63 - (g & 63)) * skew;
  while (__builtin_amdgcn_s_memrealtime() - t0 < d) __builtin_amdgcn_s_sleep(8);
#else
  (void)skew;
#endif
}

}  // namespace dietgpu
