"""GPU box: compress / decompress times of the one-large-element extras
(batch 1 x 128*512*1024 words, bf16 / fp16 / fp32) for A/B of libraries."""
import sys
import time

import torch

sys.path.insert(0, ".")
from dietgpu_fork_amd import codec as C  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
dev = "cuda"
for dt in (torch.bfloat16, torch.float16, torch.float32):
    words = 128 * 512 * 1024
    g = torch.Generator(device=dev).manual_seed(13)
    x = torch.randn(1, words, generator=g, device=dev).to(dt)
    ws = C.Workspace(1 << 30, dev)
    arch, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
    y, ok, _ = C.float_decompress_stride(arch, words, dt, prob_bits=10, ws=ws)
    assert bool((ok == 1).all()) and torch.equal(x.view(torch.uint8), y.view(torch.uint8))
    for _ in range(5):
        C.float_compress_stride(x, prob_bits=10, ws=ws, out=arch, sizes=sizes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(30):
        C.float_compress_stride(x, prob_bits=10, ws=ws, out=arch, sizes=sizes)
    torch.cuda.synchronize()
    tc = (time.perf_counter() - t0) / 30
    print(f"{tag} {str(dt)[6:]} compress {tc * 1e6:.1f} us", flush=True)
    del x, y, arch, ws
    torch.cuda.empty_cache()
