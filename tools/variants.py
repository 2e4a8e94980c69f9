"""Dev tool: build kernel-variant libraries for same-box A/B timing.

Each variant is a scratch copy of dietgpu_fork_amd/csrc (under /tmp/var,
never the product tree) with a few source substitutions, built into
tools/ablibs/<name>.so (git-ignored); tools/ab.sh (c2 bench),
tools/debug/extras_ab.sh (secondary configs) and tools/debug/sp_ab.sh
(sparse) swap them in on the GPU box.  The variants below are the round-2
experiments recorded in DESIGN.md section 7; a substitution that no longer
matches the current sources fails loudly (earlier rounds' variants whose
anchors are gone stay here as the record of what was measured; --check
lists which still apply).
    usage: python tools/variants.py name...  |  python tools/variants.py --check"""
import os, shutil, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = "pcompress.h"
NOENC = (P, "const bool encOn = hasE && uwE0 != 0 && !poisonE;", "const bool encOn = false;")
NOHIST = [(P, "__hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u,", "if (sym == 0x1234u) __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u,"),
          (P, "__hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), add,", "if (sym == 0x1234u) __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), add,")]
NOSPLITST = (P, "splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, store);", "splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, false);")
NONORM = [(P, "bool ok = it.team == 1;", "bool ok = true;"),
          (P, "for (uint32_t k0 = 0; k0 < it.team; k0 += 16) {", "for (uint32_t k0 = 0; k0 < 0; k0 += 16) {"),
          (P, "const uint32_t q = it.n == 0 ? 0u : normalizeCount(count, it.n, A().pb, keys, red);", "const uint32_t q = tid == 0 ? 1024u : 0u;")]
STAMP = [
    (P, "namespace pc {", "__device__ unsigned long long g_stamp[4096 * 8 * 6];\n#define STAMP(ph) do { if (tid == 0 && itc < 8) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); asm volatile(\"\" : \"+v\"(t_)); ((volatile unsigned long long*)g_stamp)[(blockIdx.x * 8 + itc) * 6 + (ph)] = t_; } } while (0)\nnamespace pc {"),
    (P, "    if (!hasE && !hasL) break;\n", "    if (!hasE && !hasL) break;\n    STAMP(0);\n"),
    (P, "    if (hasL) publish(itemOf(iL, A(), IN()));", "    STAMP(1);\n    if (hasL) publish(itemOf(iL, A(), IN()));"),
    (P, "    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);", "    STAMP(2);\n    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);\n    STAMP(3);"),
    (P, "      iN = itemAt(++round);", "      STAMP(4);\n      iN = itemAt(++round);"),
    (P, "    iE = iL;\n    iL = iN;", "    STAMP(5);\n    ++itc;\n    iE = iL;\n    iL = iN;"),
    (P, "  uint32_t ckE = 0;\n", "  uint32_t ckE = 0;\n  uint32_t itc = 0;\n"),
    ("codec.hip", "uint32_t deviceErrorCount(bool reset) {", "extern \"C\" void* dietgpu_debug_stamps() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamp)); return p; }\n\nuint32_t deviceErrorCount(bool reset) {"),
]
STAMP2 = [
    (P, "namespace pc {", "__device__ unsigned long long g_stamp[4096 * 8 * 16];\n#define STAMP(ph) do { if (tid == 0 && itc < 8) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); asm volatile(\"\" : \"+v\"(t_)); ((volatile unsigned long long*)g_stamp)[(blockIdx.x * 8 + itc) * 16 + (ph)] = t_; } } while (0)\nnamespace pc {"),
    (P, "    if (!hasE && !hasL) break;\n", "    if (!hasE && !hasL) break;\n    STAMP(0);\n"),
    (P, "    if (hasL) publish(itemOf(iL, A(), IN()));", "    STAMP(1);\n    if (hasL) publish(itemOf(iL, A(), IN()));"),
    (P, "    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);", "    STAMP(2);\n    if (hasE) place(itemOf(iE, A(), IN()), poisonE, ckE);\n    STAMP(3);"),
    (P, "      iN = itemAt(++round);", "      STAMP(4);\n      iN = itemAt(++round);"),
    (P, "    iE = iL;\n    iL = iN;", "    STAMP(5);\n    ++itc;\n    iE = iL;\n    iL = iN;"),
    (P, "  uint32_t ck = 0;\n", "  uint32_t ck = 0;\n  uint32_t itc = 0;\n"),
    # inside place
    (P, "    if (p.flushed[0] | p.flushed[1]) asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    __syncthreads();\n", "    if (p.flushed[0] | p.flushed[1]) asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    __syncthreads();\n    STAMP(6);\n"),
    (P, "    if (it.x == 0) {\n      // header fields known before encoding", "    STAMP(7);\n    if (it.x == 0) {\n      // header fields known before encoding"),
    (P, "    if (nk == 0) return;\n    // payload", "    STAMP(8);\n    if (nk == 0) return;\n    // payload"),
    # inside barrierNormalize
    (P, "    const bool timedOut = readfirst(stateS) != 0;\n", "    const bool timedOut = readfirst(stateS) != 0;\n    STAMP(9);\n"),
    (P, "    const uint32_t q = it.n == 0 ? 0u : normalizeCount(count, it.n, A().pb, keys, red);", "    STAMP(10);\n    const uint32_t q = it.n == 0 ? 0u : normalizeCount(count, it.n, A().pb, keys, red);\n    STAMP(11);"),
    # inside publish: after the vmcnt(0)
    (P, "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    __syncthreads();\n    if (tid == 0) stSc1(G(A().arrive) + it.i, A().epoch);", "    STAMP(12);\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    __syncthreads();\n    STAMP(13);\n    if (tid == 0) stSc1(G(A().arrive) + it.i, A().epoch);"),
    ("codec.hip", "uint32_t deviceErrorCount(bool reset) {", "extern \"C\" void* dietgpu_debug_stamps() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamp)); return p; }\n\nuint32_t deviceErrorCount(bool reset) {"),
]
def STAG(ticks):
    return [(P, "  if (iL >= A().items) return;\n", "  if (iL >= A().items) return;\n  if (A().xcdTeams && (((blockIdx.x >> 3) / A().team) & 1)) {\n    const unsigned long long t0_ = __builtin_amdgcn_s_memrealtime();\n    while (__builtin_amdgcn_s_memrealtime() - t0_ < %dull) __builtin_amdgcn_s_sleep(8);\n  }\n" % ticks)]
NTLD = [(P, "      pv[g % D][k] = ld16(j0 < uw ? src + j0 : elem);", "      { const u32x4 v_ = __builtin_nontemporal_load((gp<const u32x4>)(j0 < uw ? src + j0 : elem)); pv[g % D][k] = make_uint4(v_.x, v_.y, v_.z, v_.w); }")]
NTST = [("encode.h", "    if (store) st8(raw + i0, make_uint2(r0, r1));", "    if (store) __builtin_nontemporal_store(u32x2{r0, r1}, (gp<u32x2>)(raw + i0));")]
PRIO = [(P, "    // E's word counts and L's histogram counts are in; E's aggregate goes out", "    __builtin_amdgcn_s_setprio(3);\n    // E's word counts and L's histogram counts are in; E's aggregate goes out"),
        (P, "    if (!hasE && !hasL) break;\n", "    if (!hasE && !hasL) break;\n    __builtin_amdgcn_s_setprio(0);\n")]
def STAG4(ticks):
    return [(P, "  if (iL >= A().items) return;\n", "  if (iL >= A().items) return;\n  {\n    const unsigned long long t0_ = __builtin_amdgcn_s_memrealtime();\n    const unsigned long long dl_ = (blockIdx.x >> 8) * %dull;\n    while (__builtin_amdgcn_s_memrealtime() - t0_ < dl_) __builtin_amdgcn_s_sleep(8);\n  }\n" % ticks)]
# per-wave phase stamps of the three-item pipeline (round 3): stamp[(wg, iteration, wave, phase)]
STAMP3 = [
    (P, "namespace pc {", "__device__ unsigned long long g_stamp[4096 * 8 * 4 * 16];\n#define STAMP(ph) do { if (lane == 0 && itc < 8) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); asm volatile(\"\" : \"+v\"(t_)); ((volatile unsigned long long*)g_stamp)[((blockIdx.x * 8 + itc) * 4 + w) * 16 + (ph)] = t_; } } while (0)\nnamespace pc {"),
    (P, "  uint32_t round = 0;\n", "  uint32_t round = 0;\n  uint32_t itc = 0;\n"),
    (P, "    // Segment-phase wave priority rotates", "    STAMP(0);\n    // Segment-phase wave priority rotates"),
    (P, "    __builtin_amdgcn_s_setprio(3);\n", "    STAMP(1);\n    __builtin_amdgcn_s_setprio(3);\n"),
    (P, "    // E's word counts and L's histogram counts are in\n    __syncthreads();\n", "    // E's word counts and L's histogram counts are in\n    __syncthreads();\n    STAMP(2);\n"),
    (P, "    if (hasL) publishHist(itemOf(iL, A(), IN()));", "    if (hasL) publishHist(itemOf(iL, A(), IN()));\n    STAMP(8);"),
    (P, "    if (hasE && w == 0) lookBackE(itemOf(iE, A(), IN()));", "    STAMP(3);\n    if (hasE && w == 0) lookBackE(itemOf(iE, A(), IN()));\n    STAMP(4);"),
    (P, "      const uint32_t ep = A().epoch;", "      STAMP(5);\n      const uint32_t ep = A().epoch;"),
    (P, "    if (hasE && w != 0) place(itemOf(iE, A(), IN()));", "    if (hasE && w != 0) place(itemOf(iE, A(), IN()));\n    STAMP(6);"),
    (P, "        if (L.x == 0) {\n          asm volatile", "        STAMP(7);\n        if (L.x == 0) {\n          asm volatile"),
    (P, "      lp<u32x4> red4 = (lp<u32x4>)&hist[0];", "      STAMP(10);\n      lp<u32x4> red4 = (lp<u32x4>)&hist[0];"),
    (P, "    iE = iL;\n", "    STAMP(9);\n    ++itc;\n    iE = iL;\n"),
    ("codec.hip", "uint32_t deviceErrorCount(bool reset) {", "extern \"C\" void* dietgpu_debug_stamps() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamp)); return p; }\n\nuint32_t deviceErrorCount(bool reset) {"),
]
# round-3 attribution variants of the three-item pipeline (outputs invalid)
V3NOENC = [(P, "const bool encOn = hasE && uwE0 != 0;", "const bool encOn = false;")]
V3NOHIST = [(P, "__hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u, __ATOMIC_RELAXED,\n                               __HIP_MEMORY_SCOPE_WORKGROUP);",
             "if (sym == 0x1234u) __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u, __ATOMIC_RELAXED,\n                               __HIP_MEMORY_SCOPE_WORKGROUP);"),
            (P, "__hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), add, __ATOMIC_RELAXED,",
             "if (sym == 0x1234u) __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), add, __ATOMIC_RELAXED,")]
V3NOSPLITST = [(P, "splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, store);", "splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, false);")]
# segment-phase priority schedules (round 3)
PRLINE = "      const uint32_t pr = (blockIdx.x / A().slotSpan + round) % 3u;"
def PRIO3(expr):
    return [(P, PRLINE, "      const uint32_t pr = " + expr + ";"),
            (P, "      else __builtin_amdgcn_s_setprio(2);\n    }", "      else if (pr == 2) __builtin_amdgcn_s_setprio(2);\n      else __builtin_amdgcn_s_setprio(3);\n    }")]
# round-3 window ablations (relative to the deferred-dequeue source)
POLL_PAR = """        // the first four members' missing rows in flight at once, into
        // their (now free) first-load registers; later members one by one
#pragma unroll
        for (uint32_t m = 0; m < kFirst; ++m)
          if (ballot((miss >> m) & 1u) != 0) pa[m] = ldSc1x4(hp + uint64_t(w + pc::kWaves * m) * (kNumSymbols / 4));
#pragma unroll
        for (uint32_t m = 0; m < kPer; ++m) {
          if ((miss >> m) & 1u) {
            const u32x4 v = m < kFirst ? pa[m] : ldSc1x4(hp + uint64_t(w + pc::kWaves * m) * (kNumSymbols / 4));"""
POLL_SER = """#pragma unroll
        for (uint32_t m = 0; m < kPer; ++m) {
          if ((miss >> m) & 1u) {
            const u32x4 v = ldSc1x4(hp + uint64_t(w + pc::kWaves * m) * (kNumSymbols / 4));"""
DEQ_A = """        deq = uint32_t(__hip_atomic_fetch_add(G(A().ctr) + (A().epoch & 1u) + z, 1ull, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT));"""
DEQ_EARLY = DEQ_A + """
      if (deq != ~0u)
        __hip_atomic_store(G(A().elog) + uint64_t(T) * A().maxR + round + 2,
                           (uint64_t(A().epoch) << 32) | min(2 * (A().grid / A().team) + deq, A().nb),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);"""
R_POLL = [(P, POLL_PAR, POLL_SER)]
R_DEQ = [(P, DEQ_A, DEQ_EARLY), (P, "      if (d != ~0u && lane == 0) {", "      if (d != ~0u && lane == 0 && d == 0x7fffffffu) {")]
R_Z = [(P, "(A().epoch & 1u) + z, 1ull", "(A().epoch & 1u), 1ull")]
# round-3 decode LDS attribution (outputs invalid; bench --no-verify only)
DH = "decode.h"
D_TBL = [(DH, "  for (int c = 0; c < NC; ++c) e[c] = lut[c][p[c]->x & mask];",
          "  for (int c = 0; c < NC; ++c) e[c] = lut[c][(p[c]->x & 0u) + (threadIdx.x & 63u)];")]
D_RING = [(DH, "    v[c] = q.ringLane[idx & (dec::kRing - 1)];", "    v[c] = q.ringLane[(idx & 0u) + (threadIdx.x & 31u)];")]
D_SEG = [(DH, "              for (int s = 0; s < S; ++s) segLane[c][s][tr * 32] = uint16_t(e0[c * S + s] >> 16);",
          "              for (int s = 0; s < S; ++s) if (e0[c * S + s] == 0x12345u) segLane[c][s][tr * 32] = uint16_t(e0[c * S + s] >> 16);")]
ENC512 = [("encode.h", "  constexpr uint32_t R = kFused ? enc::kRingFused : enc::kRing;",
           "  constexpr uint32_t R = kFused ? (FT == 0 ? enc::kRingFused : 512u) : enc::kRing;")]
SP = "sparse.hip"
# round 3: writers' ring store under an exec mask (2 SALU) instead of the
# trash-address select (1 VALU)
XW = [("encode.h", """  uint32_t dst;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(dst) : "v"(trashAddr), "v"(ringAddr), "s"(vote));
  *(lp<uint16_t>)size_t(dst) = uint16_t(p.x);""", r"""  uint64_t sav_;
  (void)trashAddr;
  asm volatile("s_and_saveexec_b64 %0, %1\n\tds_write_b16 %2, %3\n\ts_mov_b64 exec, %0"
               : "=&s"(sav_) : "s"(vote), "v"(ringAddr), "v"(p.x) : "memory", "scc");""")]
# round 4: member index from blockIdx (round 3) instead of the per-team start ticket
BIDX = [(P, "    memberS = takeTicket(ka.ticket + T, ka.team, ka.skew);",
         "    memberS = ka.xcdTeams ? (bid >> 3) % ka.team : bid % ka.team;")]
XREAD = "    X = readfirst(*(volatile uint32_t*)&memberS);"
BIDX0 = [(P, XREAD, "    X = ka.xcdTeams ? (bid >> 3) % ka.team : bid % ka.team;")]
SGPRX = [(P, XREAD, "    X = memberX;"),
         (P, "  auto teamX = [&](uint32_t& T, uint32_t& X) __attribute__((always_inline)) {",
             "  uint32_t memberX = 0;\n  auto teamX = [&](uint32_t& T, uint32_t& X) __attribute__((always_inline)) {"),
         (P, "  uint32_t round = 0;\n", "  memberX = readfirst(memberS);\n  uint32_t round = 0;\n")]
W2BIDX = [(P, "    X = memberX;", "    X = ka.xcdTeams ? (bid >> 3) % ka.team : bid % ka.team;")]
NOZERO = [("upload.hip", """__global__ __launch_bounds__(256) void k_zero(uint8_t* __restrict__ dst, size_t bytes) {
  const size_t stride = size_t(gridDim.x) * 256;
  const size_t i0 = size_t(blockIdx.x) * 256 + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(dst) | bytes) % 16 == 0) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (size_t i = i0; i < bytes / 16; i += stride) d[i] = make_uint4(0, 0, 0, 0);
  } else {
    for (size_t i = i0; i < bytes; i += stride) dst[i] = 0;
  }
}
""", ""), ("upload.hip", """  const size_t units = (reinterpret_cast<uintptr_t>(dst) | bytes) % 16 == 0 ? bytes / 16 : bytes;
  const uint32_t grid = uint32_t(std::min<size_t>(1024, (units + 255) / 256));
  k_zero<<<grid, 256, 0, s>>>(static_cast<uint8_t*>(dst), bytes);
  HIP_LAUNCH_CHECK();""", """  HIP_CHECK(hipMemsetAsync(dst, 0, bytes, s));""")]
# per-wave phase stamps of the round-4 window (two wave chains)
STAMP4 = [
    (P, "namespace pc {", "__device__ unsigned long long g_stamp[4096 * 8 * 4 * 16];\n#define STAMP(ph) do { if (laneNow() == 0 && itc < 8) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); asm volatile(\"\" : \"+v\"(t_)); ((volatile unsigned long long*)g_stamp)[((blockIdx.x * 8 + itc) * 4 + w) * 16 + (ph)] = t_; } } while (0)\nnamespace pc {"),
    (P, "  uint32_t round = 0;\n", "  uint32_t round = 0;\n  uint32_t itc = 0;\n"),
    (P, "    // Segment-phase wave priority rotates", "    STAMP(0);\n    // Segment-phase wave priority rotates"),
    (P, "    __builtin_amdgcn_s_setprio(3);\n", "    STAMP(1);\n    __builtin_amdgcn_s_setprio(3);\n"),
    (P, "      publishHist(itemOf(iL, A(), IN()));\n", "      publishHist(itemOf(iL, A(), IN()));\n      STAMP(2);\n"),
    (P, "      if (w != 1) markReady();", "      STAMP(3);\n      if (w != 1) markReady();"),
    (P, "        uint32_t ckL = kCk ? waveXor(ckAcc) : 0u;", "        STAMP(4);\n        uint32_t ckL = kCk ? waveXor(ckAcc) : 0u;"),
    (P, "        *(lp<u32x2>)&pdfS[4 * lane] =", "        STAMP(5);\n        *(lp<u32x2>)&pdfS[4 * lane] ="),
    (P, "      if (hasE) lookBackE(itemOf(iE, A(), IN()));\n", "      if (hasE) lookBackE(itemOf(iE, A(), IN()));\n      STAMP(6);\n"),
    (P, "      place(itemOf(iE, A(), IN()));\n", "      STAMP(7);\n      place(itemOf(iE, A(), IN()));\n      STAMP(8);\n"),
    (P, "    // the next round's element (nextS, wave 3)", "    STAMP(9);\n    // the next round's element (nextS, wave 3)"),
    (P, "      nextS = elemOfRound(round + 1);\n", "      nextS = elemOfRound(round + 1);\n      STAMP(10);\n"),
    (P, "    iE = iL;\n", "    ++itc;\n    iE = iL;\n"),
    ("codec.hip", "uint32_t deviceErrorCount(bool reset) {", "extern \"C\" void* dietgpu_debug_stamps() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamp)); return p; }\n\nuint32_t deviceErrorCount(bool reset) {"),
]
# round 4: partial histograms published with plain stores (the line stays in
# the XCD's L2; a same-XCD consumer's sc1 load is then an L2 hit), flags sc1
PLAINPART = [(P, "    stSc1(G(A().part) + uint64_t(it.i) * kNumSymbols + tid, tag | cnt);",
              "    __hip_atomic_store(G(A().part) + uint64_t(it.i) * kNumSymbols + tid, tag | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);")]
PLAINALL = PLAINPART + [
    (P, """      __hip_atomic_store(G(A().flags) + it.tb + it.x,
                         (it.x == 0 ? kFlagPrefix : kFlagAgg) | (uint64_t(A().epoch) << 32) | agg,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""", """      __hip_atomic_store(G(A().flags) + it.tb + it.x,
                         (it.x == 0 ? kFlagPrefix : kFlagAgg) | (uint64_t(A().epoch) << 32) | agg,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);"""),
    ("encode.h", """    __hip_atomic_store(f + x, kFlagPrefix | (poison ? kFlagPoisonE : 0ull) | tag | uint64_t(excl + agg),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""", """    __hip_atomic_store(f + x, kFlagPrefix | (poison ? kFlagPoisonE : 0ull) | tag | uint64_t(excl + agg),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);"""),
    (P, """    __hip_atomic_store(G(ka.elog) + uint64_t(T) * ka.maxR + r, tag | min(e, ka.nb), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);""", """    __hip_atomic_store(G(ka.elog) + uint64_t(T) * ka.maxR + r, tag | min(e, ka.nb), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);""")]
# test-only: k_pcompress workgroups start in about
# reverse index order within every 64 (skewDelay, 1 us steps), so its
# look-back and element-log waits meet late-starting lower workgroups; run
# by tools/skew_check.sh against tests/test_gpu_progress.py.  The product
# kernel carries no hook (a one-line hook tipped its register allocation,
# DESIGN.md section 7).
PSKEW = [(P, "  __syncthreads();  // histogram zeroed\n",
          "  if (tid == 0) skewDelay(100);\n  __syncthreads();  // histogram zeroed\n")]
# round 5: the decoder's raw float bytes loaded TWO 8-step segments ahead
# (three register buffers), for archives read cold from HBM
DEC2A = [(DH, """      int32_t g = min(nSeg, int32_t(nFull)) - 1;  // rvA holds segment g's bytes
      for (; g >= 1; g -= 2) {
        fullSeg(g, rvA, rvB);
        fullSeg(g - 1, rvB, rvA);
      }
      if (g == 0) fullSeg(0, rvA, rvB);""", """      uint32_t rvC[K][R];
      auto fullSeg2 = [&](int32_t g, const uint32_t (&cur)[K][R], uint32_t (&nxt2)[K][R]) {
        if constexpr (BAL)
          setPrioRemaining((chunksPerWG - 1 - pass) * uint32_t(nSeg) + uint32_t(g), chunksPerWG * uint32_t(nSeg));
        if (g > 1) loadRaw(g - 2, true, nxt2);
#pragma unroll
        for (int grp = int(dec::kSegSteps / dec::kUnroll) - 1; grp >= 0; --grp) {
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, kVec);
#pragma unroll
          for (int u = int(dec::kUnroll) - 1; u >= 0; --u) {
            const int tr = grp * int(dec::kUnroll) + u;
            uint32_t e0[K * S];
            decStepAll<false, K * S>(chains, allValid, lutC, mask, pb, hv, e0);
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
              for (int s = 0; s < S; ++s) segLane[c][s][tr * 32] = uint16_t(e0[c * S + s] >> 16);
          }
        }
        __builtin_amdgcn_wave_barrier();
        join(g, true, cur);
        __builtin_amdgcn_wave_barrier();
      };
      (void)fullSeg;
      int32_t g = min(nSeg, int32_t(nFull)) - 1;  // rvA holds segment g's bytes
      if (g >= 1) loadRaw(g - 1, true, rvB);
      for (; g >= 2; g -= 3) {
        fullSeg2(g, rvA, rvC);
        fullSeg2(g - 1, rvB, rvA);
        fullSeg2(g - 2, rvC, rvB);
      }
      if (g == 1) {
        fullSeg2(1, rvA, rvC);
        fullSeg2(0, rvB, rvC);
      } else if (g == 0) {
        fullSeg2(0, rvA, rvC);
      }""")]
# round 5: the decoder's partial (masked) segments unrolled like the full
# ones -- 8 steps with constant LDS offsets, the ring checked every 4 steps;
# steps past a block's end are no-ops of the masked step
DECMASK = [(DH, """      for (int32_t g = nSeg - 1; g >= int32_t(nFull); --g) {
        const int32_t tTop = min(int32_t(T) - 1, g * int32_t(dec::kSegSteps) + int32_t(dec::kSegSteps) - 1);
        const int32_t tBot = g * int32_t(dec::kSegSteps);
        for (int32_t t = tTop; t >= tBot; --t) {
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, kVec);
          bool vld[K * S];
#pragma unroll
          for (int c = 0; c < K; ++c) {
            const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
#pragma unroll
            for (int s = 0; s < S; ++s) vld[c * S + s] = uint32_t(t) * 32 + l < uw;
          }
          uint32_t e0[K * S];
          decStepAll<true, K * S>(chains, vld, lutC, mask, pb, hv, e0);
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s)
              if (vld[c * S + s]) segLane[c][s][(t - tBot) * 32] = uint16_t(e0[c * S + s] >> 16);
        }""", """      for (int32_t g = nSeg - 1; g >= int32_t(nFull); --g) {
        const int32_t tBot = g * int32_t(dec::kSegSteps);
#pragma unroll
        for (int grp = int(dec::kSegSteps / dec::kUnroll) - 1; grp >= 0; --grp) {
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) ringEnsure(st[c][s], lane, kVec);
#pragma unroll
          for (int u = int(dec::kUnroll) - 1; u >= 0; --u) {
            const int tr = grp * int(dec::kUnroll) + u;
            const uint32_t t = uint32_t(tBot + tr);
            bool vld[K * S];
#pragma unroll
            for (int c = 0; c < K; ++c) {
              const uint32_t uw = lane >= 32 ? uwH[c][1] : uwH[c][0];
#pragma unroll
              for (int s = 0; s < S; ++s) vld[c * S + s] = t * 32 + l < uw;
            }
            uint32_t e0[K * S];
            decStepAll<true, K * S>(chains, vld, lutC, mask, pb, hv, e0);
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
              for (int s = 0; s < S; ++s)
                if (vld[c * S + s]) segLane[c][s][tr * 32] = uint16_t(e0[c * S + s] >> 16);
          }
        }""")]
ENCMASK = [("encode.h", """      const uint32_t tEnd = min(T, (g + 1) * enc::kSegSteps);
      for (uint32_t t = g * enc::kSegSteps; t < tEnd; ++t) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) ringFlush<int(R - 32), R>(st[c][s], lane);
        const uint32_t tr = t - g * enc::kSegSteps;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          const bool valid = t * 32 + l < uw[c];
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const uint32_t sym = valid ? uint32_t(symLane[c][s][tr * 32]) : 0u;
            const u32x4 e = tbl[s][sym];
            encStep<true, R>(st[c][s], valid, e, hv);
          }
        }
      }""", """#pragma unroll
      for (int grp = 0; grp < int(enc::kSegSteps / enc::kUnroll); ++grp) {
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
          for (int s = 0; s < S; ++s) ringFlush<int(R - 128), R>(st[c][s], lane);
        u32x4 E[enc::kUnroll][K][S];
        bool vd[enc::kUnroll][K];
#pragma unroll
        for (int u = 0; u < int(enc::kUnroll); ++u) {
          const uint32_t tr = uint32_t(grp * int(enc::kUnroll) + u);
          const uint32_t t = g * enc::kSegSteps + tr;
#pragma unroll
          for (int c = 0; c < K; ++c) {
            vd[u][c] = t * 32 + l < uw[c];
#pragma unroll
            for (int s = 0; s < S; ++s)
              E[u][c][s] = tbl[s][vd[u][c] ? uint32_t(symLane[c][s][tr * 32]) : 0u];
          }
        }
#pragma unroll
        for (int u = 0; u < int(enc::kUnroll); ++u)
#pragma unroll
          for (int c = 0; c < K; ++c)
#pragma unroll
            for (int s = 0; s < S; ++s) encStep<true, R>(st[c][s], vd[u][c], E[u][c][s], hv);
        __builtin_amdgcn_sched_barrier(0);
      }""")]
NOPC = [("codec.hip", "  if (team > pc::kMaxTeam) return false;", "  if (team > 0) return false;")]
VARS = {
    "mask2": DECMASK + ENCMASK,
    "mask2nopc": DECMASK + ENCMASK + NOPC,
    "decmask": DECMASK,
    "dec2a": DEC2A,
    # the same with the SGPR count held at 80 (84 SGPRs admit 7 workgroups
    # per CU instead of 8, MI355X_MICROARCH.md "Residency")
    "dec2a80": DEC2A + [(DH, "__global__ __launch_bounds__(dec::kThreads) void k_decode(",
                         "__global__ __launch_bounds__(dec::kThreads) __attribute__((amdgpu_num_sgpr(80))) void k_decode(")],
    "pskew": PSKEW,
    # decoder output store cache policies (global_store_dwordx4 with the
    # policy bits in the instruction; "plain" = none)
    **{f"sp_{name}": [("device.h", """__device__ __forceinline__ void st16nt(gp<void> p, uint4 v) {
  __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (gp<u32x4>)p);
}""", """__device__ __forceinline__ void st16nt(gp<void> p, uint4 v) {
  asm volatile("global_store_dwordx4 %%0, %%1, off %s" :: "v"(p), "v"(u32x4{v.x, v.y, v.z, v.w}) : "memory");
}""" % pol)] for name, pol in (("plain", ""), ("sc0", "sc0"), ("sc1", "sc1"), ("sc01", "sc0 sc1"),
                                ("ntsc1", "nt sc1"), ("ntsc0", "nt sc0"), ("nt", "nt"))},
    # decoder output through plain stores instead of streaming ones
    "decnont": [("codec.hip", "if (streamOut) return launch(std::integral_constant<int, 0>{}, std::true_type{});",
                 "if (streamOut) return launch(std::integral_constant<int, 0>{}, std::false_type{});")],
    # a single-read c3 (4 MiB byte elements, teams of
    # 128 items) through k_pcompress, measured instead of extrapolated
    # (timing and archives only; checksummed byte archives would need the
    # per-member checksum gather widened past 64 lanes)
    # round 5: one segment of loads in flight (a shallower memory queue for
    # the hand-off window's loads, which queue behind the CU's streaming)
    "pcd1": [(P, "  constexpr int D = 2;", "  constexpr int D = 1;")],
    # round 5: the quotient's shift operand read from byte 3 of the table
    # entry by SDWA (one VALU per encode step fewer)
    "sdwa": [("encode.h", "  const uint32_t q = __umulhi(x, e.y) >> (e.w >> 24);",
              """  uint32_t q;
  asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
      : "=v"(q) : "v"(e.w), "v"(__umulhi(x, e.y)));""")],
    "pc128": [(P, "constexpr uint32_t kMaxTeam = 32;", "constexpr uint32_t kMaxTeam = 128;")],
    "bpw4": [("codec.hip", "      const uint32_t bpw = 8;", "      const uint32_t bpw = 4;")],
    # sparse count diagnostics (timing only: archives wrong)
    "sp_noga": [(SP, "      if (sum)\n        __hip_atomic_fetch_add(G(histRows)", "      if (sum == 0xFFFFFFFFu)\n        __hip_atomic_fetch_add(G(histRows)")],
    "sp_nolds": [(SP, "      if (i + 1 == n && gap) count(W(0));\n      if (v != W(0)) count(v);", "      if (v == W(0x12345u)) count(v);")],
    "sp_nostage": [(SP, "    if (i + 1 == n && gap) {\n      st[dst] = W(0);\n      if (v != W(0)) st[dst + 1] = v;\n    } else if (v != W(0)) {\n      st[dst] = v;\n    }", "    if (v == W(0x12345u)) st[dst] = v;")],
    "sp_r256": [(SP, "  const uint32_t R = std::min(tiles, kReduceRows);", "  const uint32_t R = std::min(tiles, 4 * kReduceRows);")],
    "slp0": [(P, "        if (spins) __builtin_amdgcn_s_sleep(2);", "")],
    "slp1": [(P, "        if (spins) __builtin_amdgcn_s_sleep(2);", "        if (spins) __builtin_amdgcn_s_sleep(1);")],
    "pcd3": [(P, "  constexpr int D = 2;", "  constexpr int D = 3;")],
    "kt2": [("sparse.hip", "constexpr uint32_t kExpandTiles = 1;", "constexpr uint32_t kExpandTiles = 2;")],
    "plainall": PLAINALL,
    "plainpart": PLAINPART,
    "stamp4": STAMP4,
    "nozero": NOZERO,
    "w2bidx": W2BIDX,
    "bidx0": BIDX0,
    "sgprx": SGPRX,
    "bidx": BIDX,
    "hcl": [(P, "lp<uint32_t> hcol = (lp<uint32_t>)&hist[l % pc::kHistCols];", "lp<uint32_t> hcol = (lp<uint32_t>)&hist[laneNow() % pc::kHistCols];")],
    "hcx": [(P, "lp<uint32_t> hcol = (lp<uint32_t>)&hist[l % pc::kHistCols];", "lp<uint32_t> hcol = (lp<uint32_t>)&hist[(l + (halfNow() ? 6u : 0u)) % pc::kHistCols];")],
    "dp1": [("codec.hip", "constexpr uint32_t kMaxDecodeChunks = 8;", "constexpr uint32_t kMaxDecodeChunks = 1;")],
    "dc4": [("codec.hip", "constexpr uint32_t kMaxDecodeChunks = 8;", "constexpr uint32_t kMaxDecodeChunks = 4;")],
    "dc16": [("codec.hip", "constexpr uint32_t kMaxDecodeChunks = 8;", "constexpr uint32_t kMaxDecodeChunks = 16;")],
    "kf8": [(P, "constexpr uint32_t kFirst = 4;                         // loaded before the barrier", "constexpr uint32_t kFirst = 8;                         // loaded before the barrier")],
    "sl0": [(P, "        if (spins) __builtin_amdgcn_s_sleep(2);", "        (void)spins;"),
            ("lookback.h", "      __builtin_amdgcn_s_sleep(2);", "      ;")],
    "xw": XW,
    "encprio": [("encode.h", "    // every wave's slot stores are complete before other waves copy them\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");", "    __builtin_amdgcn_s_setprio(2);\n    // every wave's slot stores are complete before other waves copy them\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");")],
    "d3": [(P, "  constexpr int D = 2;", "  constexpr int D = 3;")],
    "sp_nolb": [(SP, "    const uint32_t excl =\n        lookBackPoison(G(flags) + uint64_t(b) * tilesPerElem, tile, total, epoch, spinCap, pz);", "    const uint32_t excl = tile * 409u; (void)total;")],
    "sp_nowr": [(SP, "      list[dst] = W(0);\n      if (v != W(0)) list[dst + 1] = v;\n    } else if (v != W(0)) {\n      list[dst] = v;\n    }", "      (void)dst;\n    } else if (v == W(0x12345u)) {\n      list[dst] = v;\n    }")],
    "st4a": STAG4(300),
    "st4b": STAG4(600),
    "st4c": STAG4(900),
    "prio": PRIO,
    "prio2": [(PRIO[0][0], PRIO[0][1], PRIO[0][2].replace("setprio(3)", "setprio(2)")), PRIO[1]],
    "nopc": [("codec.hip", "  if (team > pc::kMaxTeam) return false;", "  if (team > 0) return false;")],
    "ntld": NTLD,
    "ntst": NTST,
    "ntldst": NTLD + NTST,
    "stag5": STAG(500),
    "stag10": STAG(1000),
    "stag16": STAG(1600),
    "stamp2": STAMP2,
    "stamp3": STAMP3,
    "v3noenc": V3NOENC,
    "v3nohist": V3NOHIST,
    "v3nosplitst": V3NOSPLITST,
    "v3noencnohist": V3NOENC + V3NOHIST,
    "pr4rot": PRIO3("(blockIdx.x / A().slotSpan + round) & 3u"),
    "prslot": PRIO3("(blockIdx.x / A().slotSpan) & 3u"),
    "prhalf": PRIO3("(blockIdx.x / A().slotSpan) >> 1"),
    "prhalfalt": PRIO3("((blockIdx.x / A().slotSpan) >> 1) ^ (round & 1u)"),
    "pr3rotrev": PRIO3("(3u - (blockIdx.x / A().slotSpan) + round) % 3u"),
    "stamp": STAMP,
    "enc512": ENC512,
    "d_tbl": D_TBL,
    "d_ring": D_RING,
    "d_seg": D_SEG,
    "r_poll": R_POLL,
    "r_deq": R_DEQ,
    "r_z": R_Z,
    "r_all3": R_POLL + R_DEQ + R_Z,
    "noenc_nohist": [NOENC] + NOHIST,
    "noenc_nohist_nosplitst": [NOENC, NOSPLITST] + NOHIST,
    "noenc_nonorm": [NOENC] + NONORM,
    "noenc_nohist_nonorm_nosplitst": [NOENC, NOSPLITST] + NOHIST + NONORM,
    "base": [],
    "hist2x": [(P, "__hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u, __ATOMIC_RELAXED,\n                               __HIP_MEMORY_SCOPE_WORKGROUP);",
                "__hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u, __ATOMIC_RELAXED,\n                               __HIP_MEMORY_SCOPE_WORKGROUP);\n        __hip_atomic_fetch_add(hcol + __umul24(sym, pc::kHistStride), 1u, __ATOMIC_RELAXED,\n                               __HIP_MEMORY_SCOPE_WORKGROUP);")],
    "nowait": [(P, "bool ok = it.team == 1;", "bool ok = true;"),
               (P, "G(A().part) + uint64_t(it.tb) * kNumSymbols + tid;", "G(A().part) + uint64_t(it.i) * kNumSymbols + tid;"),
               (P, "for (uint32_t k0 = 0; k0 < it.team; k0 += 16) {", "for (uint32_t k0 = 0; k0 < 1; k0 += 16) {"),
               (P, "acc[k] = k0 + k < it.team ?", "acc[k] = k0 + k < 1 ?"),
               (P, "const uint32_t q = it.n == 0 ? 0u : normalizeCount(count, it.n, A().pb, keys, red);",
                   "const uint32_t ownN = it.x * 32768u < it.n ? min(it.n - it.x * 32768u, 32768u) : 0u;\n    const uint32_t q = ownN == 0 ? 0u : normalizeCount(count, ownN, A().pb, keys, red);")],
    "noenc": [(P, "const bool encOn = hasE && uwE0 != 0 && !poisonE;", "const bool encOn = false;")],
    "noplace": [(P, "for (uint32_t v = tid; v < nv; v += pc::kThreads) {", "for (uint32_t v = tid; v < nv && nv == 0xFFFFFFFFu; v += pc::kThreads) {")],
    "nosplitst": [(P, "splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, store);", "splitVec<FT>(v, i0, it.n, raw, myT + off, myT + off, false);")],
}
# phase stamps of k_encode (0) / k_decode (1), the first 4096 workgroups
# (linear id blockIdx.y * gridDim.x + blockIdx.x), wave 0
# (tools/debug/stamp_small.py, tools/debug/stamp_dec.py)
EH = "encode.h"
SSTAMP = [
    ("device.h", "namespace dietgpu {", "namespace dietgpu {\nstatic __device__ unsigned long long g_sstamp[3 * 4096 * 16];\n#define SSTAMP(kid, ph) do { const unsigned wg_ = blockIdx.y * gridDim.x + blockIdx.x; if (threadIdx.x == 0 && wg_ < 4096) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); asm volatile(\"\" : \"+v\"(t_)); ((volatile unsigned long long*)g_sstamp)[((kid) * 4096 + wg_) * 16 + (ph)] = t_; } } while (0)"),
    (EH, "  const uint32_t wx = blockIdx.x, wy = blockIdx.y;\n  if (kFused && tail.skew", "  SSTAMP(0, 0);\n  const uint32_t wx = blockIdx.x, wy = blockIdx.y;\n  if (kFused && tail.skew"),
    (EH, "    proNormalize<S>(G(tail.rows), numInBatch, b, n, tail.pb, (lp<u32x4>)&ringS[0][0], tblS, pdfS);\n    __syncthreads();\n", "    proNormalize<S>(G(tail.rows), numInBatch, b, n, tail.pb, (lp<u32x4>)&ringS[0][0], tblS, pdfS);\n    __syncthreads();\n    SSTAMP(0, 1);\n"),
    (EH, "  if (vecIn)\n    run(std::true_type{});\n  else\n    run(std::false_type{});\n", "  if (vecIn)\n    run(std::true_type{});\n  else\n    run(std::false_type{});\n  SSTAMP(0, 2);\n"),
    (EH, "    const uint32_t nk = first < nBlocks ? min(uint32_t(Cfg::kBlocksPerWG), nBlocks - first) : 0u;\n", "    const uint32_t nk = first < nBlocks ? min(uint32_t(Cfg::kBlocksPerWG), nBlocks - first) : 0u;\n    SSTAMP(0, 3);\n"),
    (EH, "      if (lane < nk) preE[lane] = excl + inc - r;\n", "      if (lane < nk) preE[lane] = excl + inc - r;\n      SSTAMP(0, 4);\n"),
    (EH, "    copyPayload<R>(preE", "    SSTAMP(0, 5);\n    copyPayload<R>(preE"),
    (EH, "(gp<uint8_t>)(bwords + roundUp(nBlocks, 2)), &ringS[0][0], flE);\n", "(gp<uint8_t>)(bwords + roundUp(nBlocks, 2)), &ringS[0][0], flE);\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    SSTAMP(0, 6);\n"),
    (DH, "  gp<const uint8_t> base = startOf(in, b);\n  gp<const uint32_t> fh = (gp<const uint32_t>)base;\n", "  SSTAMP(1, 0);\n  gp<const uint8_t> base = startOf(in, b);\n  gp<const uint32_t> fh = (gp<const uint32_t>)base;\n"),
    (DH, "#pragma unroll\n  for (int s = 0; s < S; ++s) {\n    buildLut64(", "  SSTAMP(1, 1);\n#pragma unroll\n  for (int s = 0; s < S; ++s) {\n    buildLut64("),
    (DH, "  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, l = lane & 31;\n  uint32_t hv = lane >= 32", "  SSTAMP(1, 2);\n  const uint32_t w = readfirst(tid >> 6), lane = tid & 63, l = lane & 31;\n  uint32_t hv = lane >= 32"),
    (DH, "    for (int c = 0; c < K; ++c) T = max(T, max(divUp(uwH[c][0], 32), divUp(uwH[c][1], 32)));\n", "    for (int c = 0; c < K; ++c) T = max(T, max(divUp(uwH[c][0], 32), divUp(uwH[c][1], 32)));\n    SSTAMP(1, 3 + 3 * min(pass, 3u));\n"),
    (DH, "      // full segments: unrolled, unmasked\n", "      SSTAMP(1, 4 + 3 * min(pass, 3u));\n      // full segments: unrolled, unmasked\n"),
    (DH, "    if (vecIn && vecOut)\n      run(std::true_type{});\n    else\n      run(std::false_type{});\n", "    if (vecIn && vecOut)\n      run(std::true_type{});\n    else\n      run(std::false_type{});\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    SSTAMP(1, 5 + 3 * min(pass, 3u));\n"),
    ("codec.hip", "uint32_t deviceErrorCount(bool reset) {", "extern \"C\" void* dietgpu_debug_sstamps() { void* p = nullptr; (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_sstamp)); return p; }\n\nuint32_t deviceErrorCount(bool reset) {"),
]
VARS["stampsm"] = SSTAMP
# round 6: half of each CU's dispatch slots start `ticks` late, so their
# hand-off windows fall in the other slots' segment phases
def STHALF(ticks):
    return [(P, "  if (iL >= A().items) return;\n", "  if (iL >= A().items) return;\n  if (blockIdx.x / A().slotSpan >= 2) {\n    const unsigned long long t0_ = __builtin_amdgcn_s_memrealtime();\n    while (__builtin_amdgcn_s_memrealtime() - t0_ < %dull) __builtin_amdgcn_s_sleep(8);\n  }\n" % ticks)]
# round 6: the three-kernel path in launch groups whose input fits the MALL
def MALLSL(mib):
    return [("codec.hip", "  constexpr size_t kMallSliceBytes = 0;", "  constexpr size_t kMallSliceBytes = %dull << 20;" % mib)]
VARS["sl128"] = MALLSL(128)
VARS["sl192"] = MALLSL(192)
VARS["sl384"] = MALLSL(384)
VARS["sth5"] = STHALF(500)
VARS["sth10"] = STHALF(1000)
VARS["sth15"] = STHALF(1500)
# cost probes (wrong archives): the encode step without its ring write /
# without the step at all (full segments; table reads kept)
VARS["noemit"] = [(EH, 'asm volatile("s_and_saveexec_b64 %0, %1\\n\\tds_write_b16', 'if (0) asm volatile("s_and_saveexec_b64 %0, %1\\n\\tds_write_b16')]
# ring stores without the exec mask: non-writers store to a per-thread
# discard slot (v_cndmask on the vote), so a step's store no longer orders
# the next step's VALU behind an exec restore
TRASH = [
    (EH, "  gp<uint16_t> out[2];     // per half: slot data\n};",
     "  gp<uint16_t> out[2];     // per half: slot data\n  uint32_t trash;          // LDS byte address of this thread's discard slot\n};"),
    (EH, """  uint64_t sav;
  asm volatile("s_and_saveexec_b64 %0, %1\\n\\tds_write_b16 %2, %3\\n\\ts_mov_b64 exec, %0"
               : "=&s"(sav)
               : "s"(vote), "v"(ringAddr), "v"(p.x)
               : "memory", "scc");""",
     """  uint32_t wa;
  asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3\\n\\tds_write_b16 %0, %4"
               : "=&v"(wa)
               : "v"(p.trash), "v"(ringAddr), "s"(vote), "v"(p.x)
               : "memory");"""),
    (EH, "  __shared__ uint32_t cwE[Cfg::kBlocksPerWG];",
     "  __shared__ __attribute__((aligned(16))) uint16_t trashS[enc::kThreads];\n  __shared__ uint32_t cwE[Cfg::kBlocksPerWG];"),
    (EH, "      p.ringLane = p.ring + (hv & R);\n",
     "      p.ringLane = p.ring + (hv & R);\n      p.trash = uint32_t(size_t((lp<uint16_t>)&trashS[threadIdx.x]));\n"),
    (P, "  __shared__ __attribute__((aligned(16))) uint16_t rings[pc::kBlocksPerItem * pc::kRing];",
     "  __shared__ __attribute__((aligned(16))) uint16_t rings[pc::kBlocksPerItem * pc::kRing];\n  __shared__ __attribute__((aligned(16))) uint16_t trashS[pc::kThreads];"),
    (P, "    p.ringLane = p.ring + (hv & pc::kRing);\n",
     "    p.ringLane = p.ring + (hv & pc::kRing);\n    p.trash = uint32_t(size_t((lp<uint16_t>)&trashS[threadIdx.x]));\n"),
]
VARS["trash"] = TRASH
# k_sparseExpand writing each lane's word straight from the list gather
# (coalesced 4 B stores per step) instead of staging the tile in LDS
SPX = "sparse.hip"
EXPD_TAIL = (SPX, """  gp<W> y = (gp<W>)out.start(b);
#pragma unroll
  for (uint32_t t = 0; t < kT; ++t) {
    const uint32_t t0 = (tile0 + t) * kTileWords;
    if (t0 >= n) break;""", """  gp<W> y = (gp<W>)out.start(b);
#pragma unroll
  for (uint32_t t = 0; t < kT; ++t) {
    const uint32_t t0 = (tile0 + t) * kTileWords;
    if (t0 >= n || t0 < n) break;""")
# cost probes (wrong output): no tile prefix / no list gather in k_sparseExpand
VARS["expnopre"] = [(SPX, "  uint32_t pos = tilePrefix(G(tileCounts) + uint64_t(b) * tilesPerElem, tile0, red);",
                     "  uint32_t pos = 0; (void)red;")]
VARS["expnogather"] = [(SPX, "      buf[t][q] = f ? list[src] : W(0);", "      buf[t][q] = f ? W(src) : W(0);")]
# fp64 k_coalesce granularity (blocks per workgroup; 4 is the product's)
VARS["bpw8"] = [("codec.hip", "      const uint32_t bpw = 4;", "      const uint32_t bpw = 8;")]
VARS["bpw16"] = [("codec.hip", "      const uint32_t bpw = 4;", "      const uint32_t bpw = 16;")]
VARS["expdirect"] = [(SPX, "      buf[t][q] = f ? list[src] : W(0);",
                      "      if (i < n) ((gp<W>)out.start(b))[i] = f ? list[src] : W(0);"), EXPD_TAIL]
VARS["expdirectnt"] = [(SPX, "      buf[t][q] = f ? list[src] : W(0);",
                        "      if (i < n) __builtin_nontemporal_store(f ? list[src] : W(0), (gp<W>)out.start(b) + i);"), EXPD_TAIL]
VARS["noexec"] = [(EH, 'asm volatile("s_and_saveexec_b64 %0, %1\\n\\tds_write_b16 %2, %3\\n\\ts_mov_b64 exec, %0"',
                   'asm volatile("s_mov_b64 %0, %1\\n\\tds_write_b16 %2, %3"')]
VARS["noidx"] = [(EH, "const uint32_t ringAddr = uint32_t(size_t(p.ringLane + (idx & (kRing - 1))));",
                  "(void)idx; const uint32_t ringAddr = uint32_t(size_t(p.ringLane + (__builtin_amdgcn_mbcnt_lo(~0u, 0u) & 31)));")]
VARS["nostep"] = [(EH, "for (int s = 0; s < S; ++s) encStep<false, R>(st[c][s], true, E[u][c][s], hv);",
                   "for (int s = 0; s < S; ++s) st[c][s].x += E[u][c][s].z;"),
                  (P, "for (uint32_t u = 0; u < enc::kUnroll; ++u) encStep<false, pc::kRing>(p, true, Ev[u], hv);",
                   "for (uint32_t u = 0; u < enc::kUnroll; ++u) p.x += Ev[u].z;")]
# round 6: the decoder's archive reads streamed (read once per call): raw
# float bytes / compressed words as nontemporal loads
DEC = "decode.h"
DNT_RAW = [(DEC, "      const uint2 a = ld8(raw + i0);",
            "      const u32x2 a_ = __builtin_nontemporal_load((gp<const u32x2>)(raw + i0)); const uint2 a = make_uint2(a_.x, a_.y);"),
           (DEC, "      const uint4 a = ld16(raw + 2 * i0);", "      const uint4 a = ld16nt(raw + 2 * i0);")]
DNT_RING = [(DEC, "  if (vec) return *(gp<const u32x2>)p;", "  if (vec) return __builtin_nontemporal_load((gp<const u32x2>)p);")]
VARS["dnt_raw"] = DNT_RAW
VARS["dnt_ring"] = DNT_RING
VARS["dnt_both"] = DNT_RAW + DNT_RING
# the sparse compressor counting the list histogram for every batch (not only
# one element), the dense codec then skipping its k_hist pass over the lists
VARS["sphistall"] = [(SPX, "  bool countHist = nb == 1;", "  bool countHist = nb <= 64;")]
# round 6: 4-byte decode-table entries {sym:8 | pdf:12 | slot - cdf:12}
# (half the LDS bytes of the step's table gather, two more VALU per step)
VARS["lut32"] = [
    (DEC, "  __host__ __device__ static constexpr uint32_t lutBytes(int pb) { return S * (8u << pb); }",
     "  __host__ __device__ static constexpr uint32_t lutBytes(int pb) { return S * (4u << pb); }"),
    (DEC, """  const u32x2 e = lut[p.x & mask];
  uint32_t xn = __umul24(e.x, p.x >> pb) + e.y;""",
     """  const uint32_t e = ((lp<const uint32_t>)lut)[p.x & mask];
  uint32_t xn = __umul24(__builtin_amdgcn_ubfe(e, 12, 12), p.x >> pb) + (e & 0xfffu);"""),
    (DEC, "  return e.x;\n}", "  return e;\n}"),
    (DEC, """  u32x2 e[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) e[c] = lut[c][p[c]->x & mask];""",
     """  uint32_t e[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) e[c] = ((lp<const uint32_t>)lut[c])[p[c]->x & mask];"""),
    (DEC, "    xn[c] = __umul24(e[c].x, q.x >> pb) + e[c].y;",
     "    xn[c] = __umul24(__builtin_amdgcn_ubfe(e[c], 12, 12), q.x >> pb) + (e[c] & 0xfffu);"),
    (DEC, "    e0[c] = e[c].x;", "    e0[c] = e[c];"),
    (DEC, "      if (slot < total) lut[slot] = u32x2{pdfS[s[j]] | (s[j] << 24), slot - cs[j]};",
     "      if (slot < total) ((lp<uint32_t>)lut)[slot] = (s[j] << 24) | (pdfS[s[j]] << 12) | (slot - cs[j]);"),
]
# round 6: fewer, larger k_hist chunks for mid-size batch-1 elements
VARS["ht512"] = [("codec.hip", "  const uint32_t target = 2048;", "  const uint32_t target = 512;")]
VARS["ht1024"] = [("codec.hip", "  const uint32_t target = 2048;", "  const uint32_t target = 1024;")]
if sys.argv[1:] == ["--check"]:
    for name, subs in VARS.items():
        live = all(os.path.exists(f"{REPO}/dietgpu_fork_amd/csrc/{f}") and
                   open(f"{REPO}/dietgpu_fork_amd/csrc/{f}").read().count(a) >= 1 for f, a, _ in subs)
        print(f"{name:32s} {'applies' if live else 'stale (anchors gone)'}")
    sys.exit(0)
for name in sys.argv[1:]:
    root = f"/tmp/var/{name}"
    shutil.rmtree(root, ignore_errors=True)
    os.makedirs(f"{root}/dietgpu_fork_amd")
    shutil.copytree(f"{REPO}/dietgpu_fork_amd/csrc", f"{root}/dietgpu_fork_amd/csrc")
    os.symlink(f"{REPO}/include", f"{root}/include")
    for f, a, b in VARS[name]:
        p = f"{root}/dietgpu_fork_amd/csrc/{f}"
        s = open(p).read()
        n = s.count(a)
        assert n >= 1, (name, a[:60])
        open(p, "w").write(s.replace(a, b))
    subprocess.check_call(["make", "-s", "-j8", "-C", f"{root}/dietgpu_fork_amd/csrc", "../_lib/libdietgpu_amd.so"])
    shutil.copy(f"{root}/dietgpu_fork_amd/_lib/libdietgpu_amd.so", f"{REPO}/tools/ablibs/{name}.so")
    print("built", name)
