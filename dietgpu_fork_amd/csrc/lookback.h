// Cross-workgroup hand-off helpers of the persistent compressor
// (pcompress.h): sc1 (agent-scope relaxed) loads / stores, and a decoupled
// look-back over epoch-tagged, poison-carrying 8 B flags (MI355X_MICROARCH.md
// sc1 hand-off, row 1).  encode.h's lookBack (the three-kernel k_encode, whose
// flags are zeroed per call by k_normalize instead of epoch-tagged) uses the
// same bit layout -- status in bits 63:62, poison in bit 61 (kFlagPoisonE ==
// kFlagPoison), value in bits 31:0 -- so the two stay interchangeable.
#pragma once

#include "encode.h"
#include "sync_arena.h"

namespace dietgpu {

constexpr uint64_t kFlagPoison = 1ull << 61;
static_assert(kFlagPoison == kFlagPoisonE, "one poison bit for both look-backs");

// (ldSc1 / ldSc1x4 / stSc1: device.h)

// Decoupled look-back (encode.h lookBack) over earlier members [0, x) with
// epoch-tagged, poison-carrying flags: bits 63:62 status (1 aggregate, 2
// inclusive prefix), 61 poison, 47:32 epoch, 31:0 value.  A flag of another
// epoch reads as "not yet published".  Whole wave; returns the sum of the
// values of members [0, x); `poison` in: this member's own, out: whether any
// member [0, x] is poisoned (or the wait ran out of polls).
// (storeOwn = false: this member's aggregate flag is already published)
__device__ __forceinline__ uint32_t lookBackPoison(gp<uint64_t> f, uint32_t x, uint32_t agg,
                                                   uint32_t epoch, uint32_t cap, bool& poison,
                                                   bool storeOwn = true) {
  const uint32_t lane = laneId();
  const uint64_t tag = uint64_t(epoch) << 32;
  const uint64_t own = poison ? kFlagPoison : 0ull;
  if (storeOwn && lane == 0)
    __hip_atomic_store(f + x, (x == 0 ? kFlagPrefix : kFlagAgg) | own | tag | agg, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (x == 0) return 0;
  uint32_t excl = 0;
  uint64_t pz = 0;
  bool done = false;
  int32_t j = int32_t(x);
  for (uint32_t spins = 0; spins < cap;) {
    const int32_t k = j - 1 - int32_t(lane);
    const uint64_t v = k >= 0 ? __hip_atomic_load(f + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : (kFlagPrefix | tag);
    const uint32_t hi = uint32_t(v >> 32);
    const uint32_t status = (hi & kEpochMask) == epoch ? hi >> 30 : 0u;
    const uint64_t isPre = ballot(status == 2);
    const uint64_t isZero = ballot(status == 0);
    const uint32_t firstPre = isPre ? uint32_t(__builtin_ctzll(isPre)) : 64u;
    const uint64_t need = firstPre >= 63 ? ~0ull : (2ull << firstPre) - 1;
    if (isZero & need) {
      __builtin_amdgcn_s_sleep(2);
      ++spins;
      continue;
    }
    excl += waveSum(lane <= firstPre ? uint32_t(v) : 0u);
    pz |= ballot(lane <= firstPre && (v & kFlagPoison) != 0);
    if (firstPre < 64) {
      done = true;
      break;
    }
    j -= 64;
  }
  poison = poison || pz != 0 || !done;
  if (lane == 0)
    __hip_atomic_store(f + x, kFlagPrefix | (poison ? kFlagPoison : 0ull) | tag | uint64_t(excl + agg),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

}  // namespace dietgpu
