"""GPU dev tool: c4 fp64 (16 M words) compress / decompress times with
hipEvents and the per-family kernel breakdown; checks the roundtrip.
usage: python tools/debug/fp64_bench.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import codec as C  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
g = torch.Generator(device="cuda").manual_seed(4)
x = torch.randn(16777216, generator=g, device="cuda", dtype=torch.float64)
ws = C.Workspace(2 << 30)
arch, sizes = C.float_compress_pointer([x], prob_bits=10, ws=ws)
y = torch.empty_like(x)
row = [arch[0]]
ok, _ = C.float_decompress_pointer(row, [y], prob_bits=10, ws=ws)
torch.cuda.synchronize()
exact = int(ok[0]) == 1 and torch.equal(x.view(torch.int64), y.view(torch.int64))
tc = timed(lambda: C.float_compress_pointer([x], prob_bits=10, ws=ws), reps)
td = timed(lambda: C.float_decompress_pointer(row, [y], prob_bits=10, ws=ws), reps)
C.profile_reset()
C.profile(True)
for _ in range(4):
    C.float_compress_pointer([x], prob_bits=10, ws=ws)
torch.cuda.synchronize()
C.profile(False)
k = {}
for fam in ("hist", "normalize", "encode", "coalesce"):
    ms, n = C.profile_query(fam)
    if n:
        k[fam] = round(ms / n * 1e3, 1)
print(f"fp64 c4: compress {tc:.1f} us, decompress {td:.1f} us, exact {exact}, kernels(us) {k}", flush=True)
