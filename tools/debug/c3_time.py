"""GPU debug: c3 compress / decompress times (1024 x 4 MiB bytes, uniform
over 16 symbols) with whatever library is in-tree (tools/ab scripts swap
variants in), a rocprof-free per-kernel breakdown, and oracle identity of
two elements.  usage: python tools/debug/c3_time.py [nb]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import codec as C  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = 4 << 20
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
x = torch.randint(0, 16, (nb, n), generator=g, device=dev, dtype=torch.uint8)
ws = C.Workspace(7 << 30, dev)
arch, sizes = C.ans_encode_stride(x, ws=ws)
y, ok, _ = C.ans_decode_stride(arch, n, ws=ws)
torch.cuda.synchronize()
CHECK = not os.environ.get("NOCHECK")  # cost-probe variants write wrong archives
assert not CHECK or (bool((ok == 1).all()) and torch.equal(x, y)), "roundtrip"
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn in (("compress", lambda: C.ans_encode_stride(x, ws=ws, out=arch, sizes=sizes)),
                 ("decompress", lambda: C.ans_decode_stride(arch, n, ws=ws, out=y))):
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(3):
        fn()
    b.record()
    b.synchronize()
    print(name, round(a.elapsed_time(b) / 3, 4), "ms")
C.profile_reset()
C.profile(True)
C.ans_encode_stride(x, ws=ws, out=arch, sizes=sizes)
torch.cuda.synchronize()
C.profile(False)
for k in ("compress", "hist", "normalize", "encode"):
    ms, launches = C.profile_query(k)
    if launches:
        print(" ", k, round(ms / launches, 4), "ms")
print("fallbacks", C.barrier_fallback_count(True), "errors", C.device_error_count(True))
from oracle import oracle as O  # noqa: E402  (checker only)

host = arch.cpu().numpy()
sz = sizes.cpu().tolist()
for i in ((0, nb - 1) if CHECK else ()):
    ref = O.ans_encode(x[i].cpu().numpy())
    assert sz[i] == ref.size and np.array_equal(host[i, :ref.size], ref), f"element {i} differs from oracle"
print("oracle identity ok")
