"""GPU debug: compress batches with the HIP library only (no decode) and
compare every archive byte with the CPU oracle; prints the first mismatch.
usage: python tools/debug/compress_vs_oracle.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import codec as C  # noqa: E402
from oracle import oracle as O  # noqa: E402


def check(sizes, dtype=torch.bfloat16, ft=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(n, generator=g).to(dtype) for n in sizes]
    ts = [x.cuda() for x in xs]
    arch, osz = C.float_compress_pointer(ts)
    torch.cuda.synchronize()
    osz = osz.cpu().tolist()
    bad = 0
    for i, x in enumerate(xs):
        w = x.view(torch.int16 if x.element_size() == 2 else torch.int32).numpy()
        w = w.view(np.uint16 if x.element_size() == 2 else np.uint32)
        ref = O.float_compress(w, ft)
        got = arch[i].cpu().numpy()
        if osz[i] != ref.size or not np.array_equal(got[: ref.size], ref):
            diff = np.nonzero(got[: min(ref.size, got.size)] != ref[: min(ref.size, got.size)])[0]
            print(f"  MISMATCH n={sizes[i]} size {osz[i]} vs {ref.size}; first diff at "
                  f"{diff[:8].tolist()} of {len(diff)}", flush=True)
            bad += 1
    print(f"sizes={sizes}: {'OK' if bad == 0 else f'{bad} bad'}", flush=True)


check([123457])
check([16, 31, 33, 4111], dtype=torch.float32, ft=3)
check([5, 4103, 70000], dtype=torch.float16, ft=1)
check([123457, 1000])
check([4095, 65536, 1, 300001])
check([32768 * 3 + 5])
check([32768 + 4096 * 6 + 100])
check([524288] * 4)
check([1, 7, 4096, 4097, 8191, 32767, 32768, 32769, 100000, 524287, 524288, 1048576])
check([3000] * 300 + [524288])
check([12345] * 1000)
