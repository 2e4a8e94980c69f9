"""Per-wave phase trace of k_compress (GPU box; dev tool, not product).

  python tools/exp_trace_compress.py <lib built with EXPFLAGS=-DDG_TRACE>

Stamps (s_memrealtime, 100 MHz): 22 start, 1 phase 1 done, 2 arrived at the
team barrier, 3 table ready, 4 phase 2 done, 5 look-back done, 21 end."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DIETGPU_AMD_LIB"] = os.path.abspath(sys.argv[1])
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import _native as N  # noqa: E402
from dietgpu_fork_amd import codec as C  # noqa: E402

dev = torch.device("cuda", 0)
ft = int(os.environ.get("FT", "2"))
nb, n, pb = 256, 524288 if ft != 3 else 262144, 10
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(nb, n, generator=g, device=dev)
x = {1: x.half(), 2: x.bfloat16(), 3: x}[ft]
L = N.lib()
cols = L.dietgpu_get_max_float_compressed_size(ft, n)
comp = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
sizes = torch.empty([nb], dtype=torch.int32, device=dev)
ws = C.Workspace(768 << 20, dev)
es = x.element_size()
in_ptrs = N.ptr_array([x.data_ptr() + i * n * es for i in range(nb)])
comp_ptrs = N.ptr_array([comp.data_ptr() + i * cols for i in range(nb)])
u = N.u32_array([n] * nb)
stream = torch.cuda.current_stream(dev).cuda_stream
for _ in range(3):
    N.check(L.dietgpu_float_compress(ws.h, ft, pb, 0, nb, in_ptrs, u, comp_ptrs, sizes.data_ptr(), stream))
torch.cuda.synchronize()
if not hasattr(L, "dietgpu_debug_read"):  # not a trace build (PMC runs)
    sys.exit(0)
buf = np.zeros(16384 * 24, dtype=np.uint64)
L.dietgpu_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.dietgpu_debug_read(buf.ctypes.data, buf.nbytes) == 0
T = buf.reshape(16384, 24).astype(np.int64)
T = T[T[:, 22] > 0]
base = T[:, 22].min()
us = lambda a: (a - base) / 100.0  # noqa: E731
print("waves", len(T), "span (us) %.1f" % us(T[:, 21].max()))
for name, a, b in (("phase1", 22, 1), ("publish+arrive", 1, 2), ("wait table", 2, 3), ("phase2", 3, 4),
                   ("lookback", 4, 5), ("copyout", 5, 21), ("life", 22, 21)):
    d = (T[:, b] - T[:, a]) / 100.0
    print(f"{name:15s} us quantiles 0/10/50/90/100:", np.percentile(d, [0, 10, 50, 90, 100]).round(2).tolist())
seg = np.concatenate([T[:, 22:23], T[:, 6:14], T[:, 1:2]], axis=1)
print("phase 1 per segment (us, median): start->split0, split g->split g+1, split7->end:",
      np.median(np.diff(seg, axis=1), axis=0).round(2).tolist() if False else
      (np.median(np.diff(seg, axis=1), axis=0) / 100.0).round(2).tolist())
grid = np.arange(0, T[:, 21].max() - base + 1, 500)
for name, a, b in (("live", 22, 21), ("in phase1", 22, 1), ("waiting", 1, 3), ("in phase2", 3, 4), ("placing", 4, 21)):
    live = [int(((T[:, a] - base <= t) & (T[:, b] - base > t)).sum()) for t in grid]
    print(f"{name:10s} waves every 5 us:", live)
