"""GPU box: the c4 sparse extras (1 x 15M and 5 x 15M fp32 at 90 % zeros,
1 x 15M bf16 at 50 %), a few compress / decompress calls each, for
rocprofv3 --kernel-trace --stats (per-kernel durations) and wall times."""
import sys
import time

import torch

sys.path.insert(0, ".")
from dietgpu_fork_amd import codec as C  # noqa: E402

dev = "cuda"
ws = C.Workspace(2 << 30, dev)
for nb, dt, zf in ((1, torch.float32, 0.9), (5, torch.float32, 0.9), (1, torch.bfloat16, 0.5)):
    g = torch.Generator(device=dev).manual_seed(5)
    fs = []
    for _ in range(nb):
        f = torch.randn(15000000, generator=g, device=dev).to(dt)
        f[torch.rand(f.numel(), generator=g, device=dev) < zf] = 0.0
        fs.append(f)
    arch, sizes = C.sparse_compress(fs, prob_bits=10, ws=ws)
    rows = [arch[i, : int(sizes[i])] for i in range(nb)]
    ys = [torch.empty_like(f) for f in fs]
    for _ in range(3):
        C.sparse_compress(fs, prob_bits=10, ws=ws)
        C.sparse_decompress(rows, ys, prob_bits=10, ws=ws)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        C.sparse_compress(fs, prob_bits=10, ws=ws)
    torch.cuda.synchronize()
    tc = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        C.sparse_decompress(rows, ys, prob_bits=10, ws=ws)
    torch.cuda.synchronize()
    td = (time.perf_counter() - t0) / reps
    ok = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8)) for a, b in zip(fs, ys))
    U = sum(f.numel() * f.element_size() for f in fs)
    Cb = int(sizes.to(torch.int64).sum())
    print(f"nb={nb} {dt} zeros={zf}: compress {tc*1e6:.1f} us decompress {td*1e6:.1f} us "
          f"ratio {Cb/U:.4f} alg {2*(U+Cb)/(tc+td)/1e9:.1f} GB/s exact={ok}", flush=True)
