"""GPU debug: how much of a short call's bench time is host work?  For the
sparse 1 x 15M fp32 and batch-1 bf16 extras: (a) the Python wrapper in a
back-to-back loop (what bench.py times), (b) the C ABI called directly with
prebuilt arguments, (c) a hipGraph of the call replayed back to back (GPU
time only).  usage: python tools/debug/host_overhead.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import _native as N  # noqa: E402
from dietgpu_fork_amd import codec as C  # noqa: E402


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def graph_time(fn, reps=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    return timed(g.replay, reps)


dev = torch.device("cuda")
ws = C.Workspace(2 << 30, dev)
L = N.lib()
st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731

# sparse 1 x 15M fp32, 90 % zeros
g = torch.Generator(device=dev).manual_seed(5)
f = torch.randn(15000000, generator=g, device=dev)
f[torch.rand(f.numel(), generator=g, device=dev) < 0.9] = 0.0
arch, sizes = C.sparse_compress([f], prob_bits=10, ws=ws)
y = torch.empty_like(f)
row = arch[0, : int(sizes[0])].clone()
ok = torch.empty([1], dtype=torch.uint8, device=dev)
sz = torch.empty([1], dtype=torch.int32, device=dev)
inP, inN = N.ptr_array([f.data_ptr()]), N.u32_array([f.numel()])
outP = N.ptr_array([arch.data_ptr()])
aP, oP, cap = N.ptr_array([row.data_ptr()]), N.ptr_array([y.data_ptr()]), N.u32_array([y.numel()])
cs = lambda: N.check(L.dietgpu_float_compress_sparse(ws.h, 3, 10, 0, 1, inP, inN, outP,  # noqa: E731
                                                     sizes.data_ptr(), st()))
cd = lambda: N.check(L.dietgpu_float_decompress_sparse(ws.h, 3, 10, 0, 1, aP, oP, cap,  # noqa: E731
                                                       ok.data_ptr(), sz.data_ptr(), st()))
print("sparse 1x15M compress   us: python", round(timed(lambda: C.sparse_compress([f], prob_bits=10, ws=ws)), 1),
      "c-abi", round(timed(cs), 1), "graph", round(graph_time(cs), 1), flush=True)
print("sparse 1x15M decompress us: python",
      round(timed(lambda: C.sparse_decompress([row], [y], prob_bits=10, ws=ws)), 1),
      "c-abi", round(timed(cd), 1), "graph", round(graph_time(cd), 1), flush=True)
torch.cuda.synchronize()
assert bool((ok == 1).all()) and torch.equal(f.view(torch.int32), y.view(torch.int32))

# batch-1 bf16 128*512*1024
x = torch.randn(1, 128 * 512 * 1024, generator=g, device=dev).to(torch.bfloat16)
a2, s2 = C.float_compress_stride(x, prob_bits=10, ws=ws)
y2 = torch.empty_like(x)
print("batch-1 bf16 compress   us: python",
      round(timed(lambda: C.float_compress_stride(x, prob_bits=10, ws=ws, out=a2, sizes=s2)), 1),
      "graph", round(graph_time(lambda: C.float_compress_stride(x, prob_bits=10, ws=ws, out=a2, sizes=s2)), 1),
      flush=True)
print("batch-1 bf16 decompress us: python",
      round(timed(lambda: C.float_decompress_stride(a2, x.shape[1], torch.bfloat16, prob_bits=10, ws=ws, out=y2)), 1),
      "graph",
      round(graph_time(lambda: C.float_decompress_stride(a2, x.shape[1], torch.bfloat16, prob_bits=10, ws=ws,
                                                           out=y2)), 1), flush=True)
