"""GPU debug: is a hipMemsetAsync captured into a torch CUDA graph re-run on
replay?  usage: python tools/debug/memset_probe.py"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
stream = torch.cuda.Stream()
for nbytes in (256, 4096, 1 << 20):
    t = torch.full([nbytes], 0xFF, dtype=torch.uint8, device="cuda")
    u = torch.zeros([nbytes], dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        rc = hip.hipMemsetAsync(ctypes.c_void_p(t.data_ptr()), 0, ctypes.c_size_t(nbytes),
                                ctypes.c_void_p(stream.cuda_stream))
        u.copy_(t)
    for rep in range(3):
        t.fill_(0xFF)
        u.fill_(7)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print(nbytes, "rc", rc, "rep", rep, "t zero:", bool((t == 0).all()), "u (copy after memset) zero:",
              bool((u == 0).all()), flush=True)
