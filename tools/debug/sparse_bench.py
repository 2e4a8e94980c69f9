"""GPU dev tool: time the sparse codec on BASELINE c4's sparse case (15 M fp32,
90 % zeros) with hipEvents, per kernel family; checks the roundtrip.
usage: python tools/debug/sparse_bench.py [reps]"""
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


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    g = torch.Generator(device="cuda").manual_seed(5)
    f = torch.randn(15000000, generator=g, device="cuda")
    f[torch.rand(f.numel(), generator=g, device="cuda") < 0.9] = 0.0
    ws = C.Workspace(1 << 30)
    arch, sizes = C.sparse_compress([f], ws=ws)
    y = torch.empty_like(f)
    row = [arch[0]]
    ok, _ = C.sparse_decompress(row, [y], ws=ws)
    exact = int(ok[0]) == 1 and torch.equal(f.view(torch.int32), y.view(torch.int32))
    tc = timed(lambda: C.sparse_compress([f], ws=ws), reps)
    td = timed(lambda: C.sparse_decompress(row, [y], ws=ws), reps)
    fam = {}
    for tag, fn in (("c", lambda: C.sparse_compress([f], ws=ws)), ("d", lambda: C.sparse_decompress(row, [y], ws=ws))):
        torch.cuda.synchronize()
        C.profile_reset()
        C.profile_filter(None)
        C.profile(True)
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        C.profile(False)
        for k in ("compress", "hist", "normalize", "encode", "coalesce", "decode", "sparse"):
            ms, n = C.profile_query(k)
            if n:
                fam[f"{tag}:{k}"] = round(ms / n * 1e3, 1)
    print(f"sparse c4: compress {tc:.1f} us, decompress {td:.1f} us, exact {exact}, ratio "
          f"{int(sizes[0]) / (f.numel() * 4):.4f}, kernels(us) {fam}")


if __name__ == "__main__":
    main()
