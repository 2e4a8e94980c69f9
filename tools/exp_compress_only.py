"""Dev experiment: per-kernel times of the compress pipeline when run back to
back (compress only) versus alternating with decompress (the bench step)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import _native as N  # noqa: E402
from dietgpu_fork_amd import codec as C  # noqa: E402

dev = torch.device("cuda", 0)
nb, n, pb = 256, 524288, 10
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn(nb, n, generator=g, device=dev).view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
L = N.lib()
cols = L.dietgpu_get_max_float_compressed_size(2, n)
comp = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
sizes = torch.empty([nb], dtype=torch.int32, device=dev)
out = torch.empty_like(x)
ok = torch.empty([nb], dtype=torch.uint8, device=dev)
osz = torch.empty([nb], dtype=torch.int32, device=dev)
ws = C.Workspace(768 << 20, dev)
ip = N.ptr_array([x.data_ptr() + i * n * 2 for i in range(nb)])
cp = N.ptr_array([comp.data_ptr() + i * cols for i in range(nb)])
op = N.ptr_array([out.data_ptr() + i * n * 2 for i in range(nb)])
u = N.u32_array([n] * nb)
s = torch.cuda.current_stream(dev).cuda_stream


def comp_():
    N.check(L.dietgpu_float_compress(ws.h, 2, pb, 0, nb, ip, u, cp, sizes.data_ptr(), s))


def dec_():
    N.check(L.dietgpu_float_decompress(ws.h, 2, pb, 0, nb, cp, op, u, ok.data_ptr(), osz.data_ptr(), s))


for mode in ("compress-only", "alternating", "decompress-only"):
    for _ in range(3):
        comp_(); dec_()
    torch.cuda.synchronize()
    C.profile_reset(); C.profile(True)
    for _ in range(10):
        if mode != "decompress-only":
            comp_()
        if mode != "compress-only":
            dec_()
    torch.cuda.synchronize(); C.profile(False)
    r = {}
    for k in ("hist", "normalize", "encode", "coalesce", "decode"):
        ms, nl = C.profile_query(k)
        if nl:
            r[k] = round(ms / nl * 1000, 1)
    print(mode, r)
