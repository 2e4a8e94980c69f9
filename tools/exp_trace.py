"""Experiment 7 analysis (GPU box): per-wave stamps of k_decode (make exp
EXP=7): s_memrealtime at start (slot 22) / end (slot 21), s_memtime after the
steps of each full segment (slots 2 + g).  Dev tool, not part of the product."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# argv[1]: library built with the stamps (make exp EXP=7, or EXP=k EXPFLAGS=-DDG_TRACE)
LIB = sys.argv[1] if len(sys.argv) > 1 else "libdietgpu_amd_exp7.so"
os.environ["DIETGPU_AMD_LIB"] = os.path.join(ROOT, "dietgpu_fork_amd/_lib/exp", LIB)
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import _native as N  # noqa: E402
from dietgpu_fork_amd import codec as C  # noqa: E402

dev = torch.device("cuda", 0)
nb, n, pb = 256, 524288, 10
g = torch.Generator(device=dev).manual_seed(1000)
x = (torch.randn(nb, n, generator=g, device=dev).view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
L = N.lib()
cols = L.dietgpu_get_max_float_compressed_size(2, n)
comp = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
sizes = torch.empty([nb], dtype=torch.int32, device=dev)
out = torch.empty_like(x)
ok = torch.empty([nb], dtype=torch.uint8, device=dev)
osz = torch.empty([nb], dtype=torch.int32, device=dev)
ws = C.Workspace(768 << 20, dev)
in_ptrs = N.ptr_array([x.data_ptr() + i * n * 2 for i in range(nb)])
comp_ptrs = N.ptr_array([comp.data_ptr() + i * cols for i in range(nb)])
out_ptrs = N.ptr_array([out.data_ptr() + i * n * 2 for i in range(nb)])
u = N.u32_array([n] * nb)
stream = torch.cuda.current_stream(dev).cuda_stream
for _ in range(3):
    N.check(L.dietgpu_float_compress(ws.h, 2, pb, 0, nb, in_ptrs, u, comp_ptrs, sizes.data_ptr(), stream))
    N.check(L.dietgpu_float_decompress(ws.h, 2, pb, 0, nb, comp_ptrs, out_ptrs, u, ok.data_ptr(),
                                       osz.data_ptr(), stream))
torch.cuda.synchronize()
if LIB.endswith("exp7.so"):  # timing-only variants decode garbage
    assert torch.equal(out.view(torch.int16), x.view(torch.int16))
buf = np.zeros(16384 * 24, dtype=np.uint64)
L.dietgpu_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.dietgpu_debug_read(buf.ctypes.data, buf.nbytes) == 0
T = buf.reshape(16384, 24).astype(np.int64)
T = T[T[:, 22] > 0]
s_rt, e_rt = T[:, 22], T[:, 21]
base = s_rt.min()
life = (e_rt - s_rt) / 100.0
print("waves", len(T), "span (us) %.1f" % ((e_rt.max() - base) / 100.0))
print("wave life (us) quantiles 0/10/50/90/100:", np.percentile(life, [0, 10, 50, 90, 100]).round(1).tolist())
print("wave start (us) quantiles:", np.percentile((s_rt - base) / 100.0, [0, 50, 100]).round(1).tolist())
grid = np.arange(0, e_rt.max() - base + 1, 50)
live = np.array([((s_rt - base <= t) & (e_rt - base > t)).sum() for t in grid])
print("live waves every 5 us:", live[::10].tolist())
# per-segment cycles: stamps after steps of segment g (descending g)
seg = T[:, 2:18]
d = -np.diff(seg[:, ::-1], axis=1)  # g=15..0 order reversed: time between consecutive segments
steps_plus_join = np.diff(seg[:, ::-1][:, ::-1], axis=1)
print("cycles between consecutive segment stamps (median, g=15->0):",
      np.median(-np.diff(seg, axis=1)[:, ::-1], axis=0).astype(int).tolist())
print("loop start -> first stamp median:", int(np.median(seg[:, 15] - T[:, 1])))
