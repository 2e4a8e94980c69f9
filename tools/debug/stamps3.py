"""GPU debug: per-wave phase timeline of the three-item k_pcompress pipeline
from a stamp3-instrumented build (python tools/variants.py stamp3, then the
library copied over the in-tree one).  One c2 compress; per iteration the
median time of each phase boundary per wave, relative to the iteration start.
usage: python tools/debug/stamps3.py"""
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
nb, n = int(os.environ.get("NB", 256)), int(os.environ.get("NW", 524288))
g = torch.Generator(device="cuda").manual_seed(1000)
x = (torch.randn(nb, n, generator=g, device="cuda").view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
ws = C.Workspace(768 << 20)
arch, sizes = C.float_compress_stride(x, ws=ws)
for _ in range(200):
    C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
torch.cuda.synchronize()
p = L.dietgpu_debug_stamps()
NS = 4096 * 8 * 4 * 16
assert hip.hipMemset(ctypes.c_void_p(p), 0, NS * 8) == 0
torch.cuda.synchronize()
C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
torch.cuda.synchronize()
h = np.zeros(NS, dtype=np.uint64)
assert hip.hipMemcpy(h.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(p), NS * 8, 2) == 0
np.save(os.path.join(ROOT, "gpurun_out", "stamps3.npy"), h)
st = h.reshape(4096, 8, 4, 16).astype(np.float64)
used = st[:, :, 0, 0] > 0
t0 = st[st > 0].min()
us = np.where(st > 0, (st - t0) / 100.0, np.nan)  # s_memrealtime: 100 MHz
print(f"workgroups with stamps: {int(used[:, 0].sum())}; kernel span {np.nanmax(us):.1f} us")
import os as _os
if _os.environ.get("STAMP4"):
    names = {0: "top", 1: "segs", 2: "pubH", 10: "deq", 3: "gath", 4: "sig", 5: "norm", 6: "lb", 7: "plc0", 8: "plc1", 9: "syncC"}
    order = [0, 1, 2, 10, 3, 4, 5, 6, 7, 8, 9]
else:
    names = {0: "top", 1: "segs", 2: "syncA", 8: "pubH", 3: "split", 4: "wait", 5: "syncB", 10: "parts", 6: "place",
             7: "norm", 9: "syncC"}
    order = [0, 1, 2, 8, 3, 4, 5, 10, 6, 7, 9]
for it in range(8):
    m = used[:, it]
    if not m.any():
        break
    top = us[m, it, 0, 0]
    print(f"iter {it}: WGs {m.sum()}  start min/med/max {np.nanmin(top):.1f} {np.nanmedian(top):.1f} {np.nanmax(top):.1f}")
    for wv in range(4):
        rel = us[m, it, wv, :] - top[:, None]
        cells = []
        for k in order:
            v = rel[:, k]
            v = v[~np.isnan(v)]
            if v.size:
                cells.append(f"{names[k]}={np.median(v):.2f}")
        print(f"   w{wv}: " + " ".join(cells))
