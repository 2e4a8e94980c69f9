"""GPU debug: back-to-back compress / decompress times of small bf16 batches
(the single-pass compressor's one-round shapes) with whatever library is
in-tree (tools/debug/lib_run.sh swaps variants in), and a roundtrip check.
usage: python tools/debug/small_time.py [NBxN ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import codec as C  # noqa: E402

dev = torch.device("cuda")
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def timed(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


SHAPES = ((1, 1000000), (1, 524288), (1, 262144), (3, 524288), (7, 300000), (16, 1000000), (33, 1000000),
          (64, 524288))
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
for nb, n in SHAPES:
    g = torch.Generator(device=dev).manual_seed(nb + n)
    x = (torch.randn(nb, n, generator=g, device=dev).view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
    ws = C.Workspace(512 << 20, dev)
    arch, sizes = C.float_compress_stride(x, ws=ws)
    y, ok, _ = C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws)
    torch.cuda.synchronize()
    assert bool((ok == 1).all()) and torch.equal(x.view(torch.int16), y.view(torch.int16))
    tc = timed(lambda: C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes))
    td = timed(lambda: C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y))
    print(f"{nb:3d} x {n:8d}: compress {tc:7.2f} us  decompress {td:7.2f} us", flush=True)
