import os, sys, ctypes
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import codec as C, _native as N
L = N.lib()
L.dietgpu_debug_set.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda")
nb, n = 256, 524288
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(nb, n, generator=g, device=dev).view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
ws = C.Workspace(768 << 20, dev)
arch, sizes = C.float_compress_stride(x, ws=ws)
y, ok, _ = C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws)
dbg = torch.zeros(2048 * 8 * 8, dtype=torch.int64, device=dev)
for rep in range(3):
    C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
    if rep == 2:
        L.dietgpu_debug_set(dbg.data_ptr())
    C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
    torch.cuda.synchronize()
L.dietgpu_debug_set(None)
d = dbg.view(2048, 8, 8).cpu().numpy()
used = d[:, :, 0] != 0
t0 = d[:, :, 0][used].min()
T = (d.astype(np.float64) - t0) / 100.0  # 100 MHz -> us
print("kernel span us", (d[:, :, 4][used].max() - t0) / 100.0)
wgs = np.nonzero(used[:, 0])[0]
print("WGs", len(wgs), "iters per WG", np.bincount(used.sum(1))[1:])
for it in range(6):
    m = used[:, it]
    if not m.any():
        continue
    seg = T[m, it, 1] - T[m, it, 0]
    pub = T[m, it, 2] - T[m, it, 1]
    plc = T[m, it, 3] - T[m, it, 2]
    lb = T[m, it, 7] - T[m, it, 2]
    bar = T[m, it, 6] - T[m, it, 3]
    nrm = T[m, it, 4] - T[m, it, 6]
    print(f"it{it}: n={m.sum()} start {np.median(T[m, it, 0]):.1f} segs {np.median(seg):.1f} pub {np.median(pub):.1f} "
          f"place {np.median(plc):.1f} (lookback {np.median(lb):.1f}) barwait {np.median(bar):.1f} norm {np.median(nrm):.1f} end {np.median(T[m, it, 4]):.1f} (p90 end {np.percentile(T[m, it, 4], 90):.1f})")
