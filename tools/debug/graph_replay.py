"""GPU debug: hipGraph capture/replay of the bf16 compress (and decompress),
per-element archive comparison with the CPU oracle on every replay.
usage: python tools/debug/graph_replay.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from dietgpu_fork_amd import codec as C  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.util import float_words  # noqa: E402

nb, n = 8, 524288
ws = C.Workspace(256 << 20)
x = torch.empty([nb, n], dtype=torch.bfloat16, device="cuda")
cols = C.max_float_compressed_size(2, n)
arch = torch.empty([nb, cols], dtype=torch.uint8, device="cuda")
sizes = torch.empty([nb], dtype=torch.int32, device="cuda")
y = torch.empty_like(x)


def load(seed, scale):
    w = float_words(2, nb * n, seed=seed, scale=scale)
    x.copy_(torch.from_numpy(w.view(np.int16)).view(nb, n).view(torch.bfloat16))
    torch.cuda.synchronize()
    return w


def check(tag, w):
    got = sizes.cpu().tolist()
    a = arch.cpu().numpy()
    bad = []
    for i in range(nb):
        ref = O.float_compress(w[i * n:(i + 1) * n], 2)
        if got[i] != ref.size or not np.array_equal(a[i, :ref.size], ref):
            d = np.nonzero(a[i, :min(ref.size, got[i])] != ref[:min(ref.size, got[i])])[0]
            bad.append((i, got[i], ref.size, int(d[0]) if d.size else None))
    ydiff = [(i, int((y[i].view(torch.int16) != x[i].view(torch.int16)).sum())) for i in range(nb)]
    print(tag, "err", C.device_error_count(reset=True), "bad archives", bad, "y mismatches", ydiff, flush=True)


stream = torch.cuda.Stream()
w = load(1, 1.0)
with torch.cuda.stream(stream):
    C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
    C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
stream.synchronize()
check("eager", w)
import ctypes
hip = ctypes.CDLL("libamdhip64.so")
for rep in range(2):
    w = load(100 + rep, 1 + rep)
    with torch.cuda.stream(stream):
        C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
        C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
    stream.synchronize()
    check(f"eager data {rep}", w)
for mode in ("compress-only", "compress+decompress"):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        st = ctypes.c_int(-1)
        rc = hip.hipStreamIsCapturing(ctypes.c_void_p(stream.cuda_stream), ctypes.byref(st))
        cur = torch.cuda.current_stream().cuda_stream
        rc2 = hip.hipStreamIsCapturing(ctypes.c_void_p(cur), ctypes.byref(ctypes.c_int(-1)))
        print("capturing status", rc, st.value, "stream", hex(stream.cuda_stream), "current", hex(cur), flush=True)
        C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
        if mode != "compress-only":
            C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
    for rep in range(4):
        w = load(100 + rep, 1 + rep)
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        if mode == "compress-only":
            with torch.cuda.stream(stream):
                C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
            stream.synchronize()
        check(f"{mode} replay {rep}", w)
    del g
