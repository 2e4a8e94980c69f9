"""Experiment 7 analysis (GPU box): per-wave s_memtime phase stamps of
k_decode (make exp EXP=7).  Runs the c2 bf16 workload once and prints
per-phase cycle statistics.  Dev tool, not part of the product."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DIETGPU_AMD_LIB"] = os.path.join(ROOT, "dietgpu_fork_amd/_lib/exp/libdietgpu_amd_exp7.so")
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
assert torch.equal(out.view(torch.int16), x.view(torch.int16))
buf = np.zeros(16384 * 24, dtype=np.uint64)
L.dietgpu_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.dietgpu_debug_read(buf.ctypes.data, buf.nbytes) == 0
T = buf.reshape(16384, 24)[:8192].astype(np.int64)
T = T[T[:, 0] > 0]
t0 = T[:, 0].min()
start, loop = T[:, 0] - t0, T[:, 1] - t0
print("waves", len(T), "kernel span (cyc)", (T[:, 3] - t0).max())
print("setup (start->loop): median %d p90 %d" % (np.median(loop - start), np.percentile(loop - start, 90)))
prev = T[:, 1]
steps, joins = [], []
for gseg in range(7, -1, -1):
    a, b_ = T[:, 2 + 2 * gseg], T[:, 3 + 2 * gseg]
    steps.append(a - prev)
    joins.append(b_ - a)
    prev = b_
steps, joins = np.array(steps), np.array(joins)
print("steps per segment: median", np.median(steps, axis=1).astype(int))
print("join per segment:  median", np.median(joins, axis=1).astype(int), "p90", np.percentile(joins, 90, axis=1).astype(int))
life = T[:, 3] - T[:, 0]
print("wave life median %d, p10 %d p90 %d" % (np.median(life), np.percentile(life, 10), np.percentile(life, 90)))
print("start times histogram (cycles):", np.histogram(start, bins=8)[0], np.histogram(start, bins=8)[1].astype(int))
hw = T[:, 23] & 0xffffffff
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
xcc = (T[:, 23] >> 32) & 0xf
print("distinct (xcc,se,cu,simd):", len(set(zip(xcc, se, cu, simd))))
rt = (T[:, 21] - T[:, 22]).astype(np.float64) / 100e6  # s_memrealtime: 100 MHz
cyc = (T[:, 3] - T[:, 0]).astype(np.float64)
print("shader clock estimate (GHz): median %.3f" % np.median(cyc / rt / 1e9))
for xc in sorted(set(xcc.tolist()))[:2]:
    m = xcc == xc
    st = np.sort(T[m, 0] - T[m, 0].min())
    print("xcc", xc, "waves", m.sum(), "start quantiles (cyc):", np.percentile(st, [0, 25, 50, 60, 75, 100]).astype(int),
          "end max", int((T[m, 3] - T[m, 0].min()).max()))
# concurrency from the chip-wide 100 MHz clock
s_rt, e_rt = T[:, 22], T[:, 21]
base = s_rt.min()
print("realtime span (us): %.1f" % ((e_rt.max() - base) / 100.0))
grid = np.arange(0, e_rt.max() - base + 1, 50)  # 0.5 us steps
live = np.array([((s_rt - base <= t) & (e_rt - base > t)).sum() for t in grid])
print("live waves over time (every 5 us):", live[::10].tolist())
print("wave start (us) quantiles:", np.percentile((s_rt - base) / 100.0, [0, 10, 25, 50, 75, 90, 100]).round(1).tolist())
print("wave life (us) quantiles:", np.percentile((e_rt - s_rt) / 100.0, [0, 10, 50, 90, 100]).round(1).tolist())
life_us = (e_rt - s_rt) / 100.0
for name, key in (("xcc", xcc), ("simd", simd), ("se", se)):
    print("life by", name, {int(k): round(float(life_us[key == k].mean()), 1) for k in sorted(set(key.tolist()))})
wv = np.arange(len(T))
print("life by wave-in-WG", {k: round(float(life_us[(wv % 4) == k].mean()), 1) for k in range(4)})
print("life by tensor parity (blockIdx.x)", {k: round(float(life_us[((wv // 4) % 4) == k].mean()), 1) for k in range(4)})
