"""GPU debug: phase timeline of k_pcompress from a stamp-instrumented build
(tools/ablibs/stamp.so copied over the in-tree library; exports
dietgpu_debug_stamps).  One c2 compress; per iteration the spread of each
phase's start over workgroups and the median phase durations.
usage: python tools/debug/stamps.py"""
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
L.dietgpu_debug_stamps.restype = ctypes.c_void_p
hip = ctypes.CDLL("libamdhip64.so")
nb, n = 256, 524288
g = torch.Generator(device="cuda").manual_seed(1000)
x = (torch.randn(nb, n, generator=g, device="cuda").view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
ws = C.Workspace(768 << 20)
arch, sizes = C.float_compress_stride(x, ws=ws)
for _ in range(3):
    C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
torch.cuda.synchronize()
p = L.dietgpu_debug_stamps()
NS = 4096 * 8 * int(os.environ.get("STAMPS", "6"))
assert hip.hipMemset(ctypes.c_void_p(p), 0, NS * 8) == 0
torch.cuda.synchronize()
C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
torch.cuda.synchronize()
h = np.zeros(NS, dtype=np.uint64)
assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(p), NS * 8, 2) == 0
np.save(os.path.join(ROOT, "gpurun_out", "stamps.npy"), h)
st = h.reshape(4096, 8, -1)[:, :, :6].astype(np.float64)
used = st[:, :, 0] > 0
grid = int(used[:, 0].sum())
t0 = st[st > 0].min()
us = np.where(st > 0, (st - t0) / 100.0, np.nan)  # s_memrealtime: 100 MHz
print(f"workgroups with stamps: {grid}")
names = ["start", "segs done", "published", "placed", "barrier passed", "normalised"]
for it in range(8):
    m = used[:, it]
    if not m.any():
        break
    row = us[m, it, :]
    print(f"iter {it}: WGs {m.sum()}")
    for k in range(6):
        v = row[:, k]
        v = v[~np.isnan(v)]
        if v.size == 0:
            continue
        print(f"   {names[k]:15s} start min/med/max {v.min():8.2f} {np.median(v):8.2f} {v.max():8.2f}")
    d = np.diff(row, axis=1)
    print("   median phase us: " + "  ".join(f"{names[k+1]}={np.nanmedian(d[:, k]):.2f}" for k in range(5)))
