// Check of BatchDesc's inline (kernel-argument) tables: the kernel resolves
// start(b) / size(b) of pointer- and split-mode descriptors whose tables
// ride in its first (InlineTable) argument and writes the VALUES out (never
// dereferences them), so a wrong offset shows up as a mismatch, not a fault.
//   hipcc --offload-arch=gfx950 -O3 -I../../dietgpu_fork_amd/csrc inline_table.hip -o inline_table
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "batch.h"

using namespace dietgpu;

__global__ void k_probe(const InlineTable, BatchDesc a, BatchDesc b, BatchDesc c, uint32_t nb,
                        unsigned long long* res) {
  const uint32_t e = blockIdx.x;
  if (threadIdx.x != 0 || e >= nb) return;
  res[6 * e + 0] = (unsigned long long)a.start(e);
  res[6 * e + 1] = a.size(e);
  res[6 * e + 2] = (unsigned long long)b.start(e);
  res[6 * e + 3] = b.size(e);
  res[6 * e + 4] = (unsigned long long)c.start(e);
  res[6 * e + 5] = c.size(e);
}

int main() {
  const uint32_t nb = 300;
  std::vector<uint64_t> A(nb), B(nb);
  std::vector<uint32_t> S(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    // low words with bit 31 set, like real device addresses (catches sign
    // extension of the 32-bit readfirstlane halves)
    A[i] = 0x7f1280000000ull + 4096ull * i;
    B[i] = 0x7ff0fff00000ull + 8192ull * i + 16;
    S[i] = 1000 + 3 * i;
  }
  // same packing as codec.hip uploadTables: [8 B bias] A | B | S
  InlineTable* t = new InlineTable();
  uint8_t* w = reinterpret_cast<uint8_t*>(t->w);
  std::memcpy(w + 8, A.data(), nb * 8);
  std::memcpy(w + 8 + nb * 8, B.data(), nb * 8);
  std::memcpy(w + 8 + nb * 16, S.data(), nb * 4);
  BatchDesc a = BatchDesc::pointers((const uint64_t*)8, (const uint32_t*)(8 + nb * 16));
  a.inl = BatchDesc::kInlPtrs | BatchDesc::kInlSizes;
  BatchDesc b = BatchDesc::pointers((const uint64_t*)(8 + nb * 8), nullptr, 77);
  b.inl = BatchDesc::kInlPtrs;
  BatchDesc c = BatchDesc::split((void*)0x5000000000ull, (const uint64_t*)(8 + nb * 8),
                                 (const uint32_t*)(8 + nb * 16));
  c.inl = BatchDesc::kInlOffsets | BatchDesc::kInlSizes;
  unsigned long long* d;
  hipMalloc(&d, nb * 6 * 8);
  hipMemset(d, 0, nb * 6 * 8);
  k_probe<<<nb, 64>>>(*t, a, b, c, nb, d);
  hipError_t e1 = hipGetLastError(), e2 = hipDeviceSynchronize();
  std::vector<unsigned long long> h(nb * 6);
  hipMemcpy(h.data(), d, nb * 6 * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (uint32_t i = 0; i < nb; ++i) {
    const unsigned long long want[6] = {A[i], S[i], B[i], 77, 0x5000000000ull + B[i], S[i]};
    for (int k = 0; k < 6; ++k) {
      if (h[6 * i + k] != want[k] && bad++ < 8)
        printf("elem %u field %d: got %llx want %llx\n", i, k, h[6 * i + k], want[k]);
    }
  }
  printf("inline table probe: launch=%s sync=%s mismatches=%d\n", hipGetErrorString(e1),
         hipGetErrorString(e2), bad);
  return bad != 0;
}
