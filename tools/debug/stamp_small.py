"""GPU debug: phase timeline of k_encode / k_decode for small bf16 batches
from the stamp build (python tools/variants.py stampsm; swapped in with
tools/debug/lib_run.sh).  Per shape: the last compress / decompress call's
stamps of workgroups 0-63 of element 0 (wave 0), as microseconds after the
earliest workgroup start.
usage: python tools/debug/stamp_small.py [NBxN ...]"""
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
dev = torch.device("cuda")
NAMES = {0: ["start", "norm", "steps", "pre-lb", "lookback", "copy", "end"],
         1: ["start", "hdr", "lut", "setup", "partial", "end"]}


def read():
    torch.cuda.synchronize()
    p = L.dietgpu_debug_sstamps()
    buf = torch.empty(3 * 4096 * 16, dtype=torch.int64, device=dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(p), ctypes.c_size_t(buf.numel() * 8), 3)
    torch.cuda.synchronize()
    return buf.cpu().numpy().reshape(3, 4096, 16)


def show(st, kid, nwg):
    a = st[kid, :nwg, : len(NAMES[kid])].astype(np.float64)
    t0 = a[a > 0].min()
    rel = (a - t0) * 0.01  # 100 MHz ticks -> us
    print("   kernel", "encode" if kid == 0 else "decode", "phases:", " ".join(NAMES[kid]))
    for w in sorted(set([0, 1, nwg // 2, nwg - 1])):
        if w < nwg:
            print(f"   wg {w:3d}: " + " ".join(f"{v:7.2f}" for v in rel[w]))


FP64 = os.environ.get("FP64")  # c4's fp64 tensor instead (16 M words)
SHAPES = [(1, 4096), (1, 1000000), (8, 1000000)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
for nb, n in SHAPES:
    g = torch.Generator(device=dev).manual_seed(nb + n)
    dt = torch.float64 if FP64 else torch.bfloat16
    x = (torch.randn(nb, n, generator=g, device=dev, dtype=torch.float64) if FP64 else
         (torch.randn(nb, n, generator=g, device=dev).view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16))
    ws = C.Workspace(512 << 20, dev)
    arch, sizes = C.float_compress_stride(x, ws=ws)
    y, ok, _ = C.float_decompress_stride(arch, n, dt, ws=ws)
    for _ in range(20):
        C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
    st = read()
    print(f"{nb} x {n}:")
    nwgE = min(64, -(-n // (4096 * 8)))
    show(st, 0, max(1, nwgE))
    for _ in range(20):
        C.float_decompress_stride(arch, n, dt, ws=ws, out=y)
    st = read()
    nwgD = min(64, -(-n // (4096 * 8)))
    show(st, 1, max(1, nwgD))
