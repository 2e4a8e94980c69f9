"""GPU debug: phase timeline of the c2 decode (256 x 524288 bf16), warm and
cold (a 512 MiB read between compress and decode evicts the archives from
the Infinity Cache, as bench.py's decode_hbm does), from the stamp build
(python tools/variants.py stampsm, swapped in by tools/debug/lib_run.sh).
Per phase (passes 0 and 1 of the persistent loop): the median / 90th percentile over workgroups of its duration, and
the kernel span (first start to last end), in microseconds."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import _native as N  # noqa: E402
from dietgpu_fork_amd import codec as C  # noqa: E402

L = N.lib()
L.dietgpu_debug_sstamps.restype = ctypes.c_void_p
hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda")
PH = ["start", "hdr", "lut", "setup0", "partial0", "end0", "setup1", "partial1", "end1"]


def read():
    torch.cuda.synchronize()
    buf = torch.zeros(3 * 4096 * 16, dtype=torch.int64, device=dev)
    hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(L.dietgpu_debug_sstamps()),
                  ctypes.c_size_t(buf.numel() * 8), 3)
    torch.cuda.synchronize()
    return buf.cpu().numpy().reshape(3, 4096, 16)[1, :, :9].astype(np.float64)


def clear():
    z = torch.zeros(3 * 4096 * 16, dtype=torch.int64, device=dev)
    hip.hipMemcpy(ctypes.c_void_p(L.dietgpu_debug_sstamps()), ctypes.c_void_p(z.data_ptr()),
                  ctypes.c_size_t(z.numel() * 8), 3)
    torch.cuda.synchronize()


nb, n = 256, 524288
g = torch.Generator(device=dev).manual_seed(7)
x = torch.randn(nb, n, generator=g, device=dev).to(torch.bfloat16)
ws = C.Workspace(768 << 20, dev)
arch, sizes = C.float_compress_stride(x, ws=ws)
y, ok, _ = C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws)
evict = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
for mode in ("warm", "cold", "warm", "cold"):
    C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
    if mode == "cold":
        evict.add_(1)
    torch.cuda.synchronize()
    clear()
    C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
    a = read()
    a = a[a[:, 0] > 0]
    t0 = a[:, 0].min()
    last = np.where(a[:, 8] > 0, a[:, 8], a[:, 5])
    span = (last.max() - t0) * 0.01
    print(f"{mode}: {len(a)} workgroups, span {span:.1f} us; start spread {(a[:, 0].max() - t0) * 0.01:.1f} us")
    for i in range(1, 9):
        m = (a[:, i] > 0) & (a[:, i - 1] > 0)
        if not m.any():
            continue
        d = (a[m, i] - a[m, i - 1]) * 0.01
        print(f"   {PH[i - 1]:>7s} -> {PH[i]:<7s} median {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}")
