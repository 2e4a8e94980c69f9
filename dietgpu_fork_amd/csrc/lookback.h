// Cross-workgroup hand-off helpers of the persistent compressor
// (pcompress.h).  The epoch-tagged, poison-carrying decoupled look-back
// (lookBackPoison) lives in encode.h, shared with k_encode's fused coalesce;
// sc1 loads / stores are in device.h.
#pragma once

#include "encode.h"
#include "sync_arena.h"

namespace dietgpu {

constexpr uint64_t kFlagPoison = kFlagPoisonE;

}  // namespace dietgpu
