// Persistent per-(device, stream) device memory for the compressor's
// cross-workgroup state: look-back flags and tagged partial histograms of
// k_pcompress.
//
// Flags carry a per-call epoch instead of being zeroed before every call: a
// flag counts only if its epoch is the current call's, so stale values from
// earlier calls are ignored and no memset launch precedes k_pcompress.
//
// Calls on one stream are serial, so one arena per (device, stream) keeps
// concurrent calls on different streams apart (hipStreamPerThread is keyed per
// host thread, since that one handle names a different stream on each
// thread); the lease holds the arena's lock from epoch assignment to kernel
// launch, so host threads sharing a stream enqueue epochs in order.
//
// Under hipGraph stream capture every replay would reuse the captured epoch,
// so a capturing call takes its flags from the caller's StackDeviceMemory
// instead and zeroes them with a captured zeroing kernel (a graph node that re-runs
// on every replay); epoch 1.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>

#include "dietgpu/StackDeviceMemory.h"

namespace dietgpu {

// 16-bit epochs: look-back flags carry them in bits 47:32, tagged partial
// histograms in bits 31:16 (the arena is re-zeroed when they wrap)
constexpr uint32_t kEpochMask = 0xffffu;

// Regions of one arena.  Each kind of epoch-tagged word lives in a region of
// its own, so a stale word only ever overlaps a stale word of the same kind
// (a tag collision across kinds -- say a look-back flag's value bits read as
// a partial's epoch -- cannot happen whatever the shapes of earlier calls).
// kSyncArrive holds the three-kernel path's last-arrival counters (NormArgs,
// encode.h): untagged, they wrap back to zero at every element's last
// arrival, so they are zero between calls.  kSyncRows holds two buffers of
// histogram rows that k_hist (and the sparse compressor's k_sparseCount)
// accumulate with atomics for the dense encoder's normalisation: a call uses
// a buffer that must start zeroed -- the one the previous such call zeroed,
// whatever the epochs of the calls in between -- and its kernel zeroes the
// other one for the next call (SyncLease::rows).
enum SyncRegion : int { kSyncCounters = 0, kSyncFlags, kSyncPartials, kSyncLog, kSyncArrive, kSyncRows,
                        kSyncRegions };
// A lease that needs no region (only, say, histogram rows).
constexpr size_t kNoSyncRegions[kSyncRegions] = {};
// kSyncCounters layout: k_pcompress's two u64 dequeue counters.
constexpr size_t kSyncCounterBytes = 16;

class SyncLease {
 public:
  // Per region, >= `bytes[k]` zero-at-creation bytes for the current device
  // and `stream`, and this call's epoch (1 .. kEpochMask).
  // dequeue: the call runs k_pcompress, whose dequeue counter (epoch & 1)
  // must start at zero (see Arena::ctrDirty).
  // rowsBytes > 0: the call accumulates rowsBytes of histogram rows in
  // rows[0] (zero on entry) and zeroes the first rowsBytes of rows[1] for
  // the next call (bytes[kSyncRows] is ignored).
  SyncLease(StackDeviceMemory& res, hipStream_t stream, const size_t (&bytes)[kSyncRegions], bool dequeue = false,
            size_t rowsBytes = 0);

  SyncLease(const SyncLease&) = delete;
  SyncLease& operator=(const SyncLease&) = delete;

  void* base[kSyncRegions] = {};
  void* rows[2] = {};  // this call's row buffer, the next call's (rowsBytes > 0)
  uint32_t epoch = 0;
  bool capturing = false;

 private:
  GpuMemoryReservation<uint8_t> capMem_;
  std::unique_lock<std::mutex> lock_;
};

// Number of elements whose archive the compressor refused to finish since
// the last reset (a team barrier or look-back wait ran out of polls: the
// element's outSize is 0); synchronises the device.
uint32_t deviceErrorCount(bool reset);
// Number of k_pcompress team-barrier fallbacks since the last reset (a
// workgroup that waited out the barrier budget for its team's partial
// histograms and counted its element from the input; the archive is exact,
// the call slower); synchronises the device.
uint32_t barrierFallbackCount(bool reset);

// Polls allowed for each cross-workgroup wait of the compressor before it
// gives up and poisons the element (default 1 << 24, about 0.5 s).  0 makes
// every wait that has to wait fail: test hook for the error path.
void setSpinCap(uint32_t polls);
uint32_t spinCap();

// How long (100 MHz ticks of s_memrealtime) a compressor workgroup waits for
// its team's partial histograms before it counts the element from the input
// itself (default 20,000 = 200 us; normal team skew is a few us).  0 makes
// every team wait fall back at once: test hook for the slow path.
void setBarrierBudget(uint32_t ticks);
uint32_t barrierBudgetTicks();

// Test hook: workgroups of the fused three-kernel compressor (k_encode) wait
// (63 - g % 64) * ticks at their start (skewDelay, device.h), so they start in
// about reverse index order within every 64: the look-backs then wait on
// late-starting lower workgroups.  0 (default) is off.  (k_pcompress carries
// no hook; the test-only variant tools/variants.py pskew adds one.)
void setDispatchSkew(uint32_t ticks);
uint32_t dispatchSkew();

// Test hook: which compressor takes batches that both can: 0 (default) the
// size rule (persistentPreferred, codec.hip), 1 the single-pass k_pcompress
// whenever it can (16 B-aligned elements of at most 1 MiB of symbols, no
// caller histogram), 2 always the three-kernel path.  Archives are the same.
void setCompressPath(int mode);
int compressPath();

}  // namespace dietgpu
