"""GPU dev tool: one workload shape in isolation, for rocprofv3 --stats and
--pmc passes that see only that shape's kernels (the bench
extras mix shapes under one kernel name).  Builds the inputs, checks the
roundtrip bit for bit, then runs `reps` compress + decompress calls
back to back and prints whole-call times (events on the launch stream).
    usage: python tools/debug/shape_prof.py SHAPE [reps]
SHAPE: c3 | raw_bf16_b | raw_bf16_nb | raw_fp32_b | fp64_16m | fp64_1e8 |
       sp_fp64_5x15m | sp_fp32_5x15m | sp_fp32_1x15m90 | c2 | c5 | bf16_1e9 |
       bf16_16m | bf16_1m | fp32_16m"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import dietgpu_fork_amd  # noqa: E402,F401
from dietgpu_fork_amd import codec as C  # noqa: E402

DEV = "cuda"
IV = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def sparse(nb, n, dt, frac, seed=5):
    g = torch.Generator(device=DEV).manual_seed(seed)
    fs = []
    for _ in range(nb):
        f = torch.randn(n, generator=g, device=DEV, dtype=torch.float64 if dt == torch.float64 else torch.float32)
        f = f.to(dt)
        f[torch.rand(n, generator=g, device=DEV) < frac] = 0
        fs.append(f)
    return fs


def build(shape, ws):
    """-> (compress(), decompress(), check() -> bool)"""
    if shape == "c3":
        g = torch.Generator(device=DEV).manual_seed(3)
        x = torch.randint(0, 16, (1024, 4 << 20), generator=g, device=DEV, dtype=torch.uint8)
        arch, sizes = C.ans_encode_stride(x, ws=ws)
        y = torch.empty_like(x)
        return (lambda: C.ans_encode_stride(x, ws=ws, out=arch, sizes=sizes),
                lambda: C.ans_decode_stride(arch, x.shape[1], ws=ws, out=y),
                lambda: torch.equal(x, y))
    if shape.startswith("raw_"):
        dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}[shape.split("_")[1]]
        g = torch.Generator(device=DEV).manual_seed(23)
        if shape.endswith("_b"):
            ts = [torch.normal(0, 1.0, [512 * 1024], generator=g, device=DEV).to(dt) for _ in range(128)]
        else:
            ts = [torch.normal(0, 1.0, [128 * 512 * 1024], generator=g, device=DEV).to(dt)]
        bs = [t.view(torch.uint8) for t in ts]
        arch, sizes = C.ans_encode_pointer(bs, ws=ws)
        rows = [arch[i] for i in range(len(bs))]
        ys = [torch.empty_like(b) for b in bs]
        return (lambda: C.ans_encode_pointer(bs, ws=ws), lambda: C.ans_decode_pointer(rows, ys, ws=ws),
                lambda: all(torch.equal(a, b) for a, b in zip(bs, ys)))
    if shape.startswith("fp64_"):
        n = {"fp64_16m": 16777216, "fp64_1e8": 100000000}[shape]
        g = torch.Generator(device=DEV).manual_seed(4)
        x = torch.randn(n, generator=g, device=DEV, dtype=torch.float64)
        arch, _ = C.float_compress_pointer([x], prob_bits=9, ws=ws)
        y = torch.empty_like(x)
        row = [arch[0]]
        return (lambda: C.float_compress_pointer([x], prob_bits=9, ws=ws),
                lambda: C.float_decompress_pointer(row, [y], prob_bits=9, ws=ws),
                lambda: torch.equal(x.view(torch.int64), y.view(torch.int64)))
    if shape.startswith("sp_"):
        kind, nbn = shape.split("_")[1], shape.split("_")[2]
        dt = {"fp64": torch.float64, "fp32": torch.float32, "bf16": torch.bfloat16}[kind]
        frac = 0.9 if nbn.endswith("90") else 0.5
        nb = int(nbn.split("x")[0])
        fs = sparse(nb, 15000000, dt, frac)
        arch, sizes = C.sparse_compress(fs, prob_bits=9, ws=ws)
        ys = [torch.empty_like(f) for f in fs]
        rows = [arch[i, : int(sizes[i])] for i in range(nb)]
        iv = IV[fs[0].element_size()]
        return (lambda: C.sparse_compress(fs, prob_bits=9, ws=ws),
                lambda: C.sparse_decompress(rows, ys, prob_bits=9, ws=ws),
                lambda: all(torch.equal(a.view(iv), b.view(iv)) for a, b in zip(fs, ys)))
    if shape in ("c5", "bf16_1e9"):
        nb, n = (8192, 524288) if shape == "c5" else (1, 1070000000)
        x = torch.empty([nb, n], dtype=torch.bfloat16, device=DEV)
        g = torch.Generator(device=DEV).manual_seed(5)
        flat = x.view(-1)
        for i in range(0, flat.numel(), 1 << 28):
            m = min(1 << 28, flat.numel() - i)
            flat[i:i + m] = (torch.randn(m, generator=g, device=DEV).view(torch.int32) >> 16).to(
                torch.int16).view(torch.bfloat16)
        arch, sizes = C.float_compress_stride(x, ws=ws)
        y = torch.empty_like(x)
        return (lambda: C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes),
                lambda: C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y),
                lambda: torch.equal(x.view(torch.int16), y.view(torch.int16)))
    if shape in ("bf16_16m", "bf16_1m", "fp32_16m"):
        # batch-1 pointer-API calls (the bench's batch-1 sweep, FloatBenchmark.cu)
        n = 16_000_000 if shape.endswith("16m") else 1_000_000
        g = torch.Generator(device=DEV).manual_seed(6)
        x = torch.randn(n, generator=g, device=DEV)
        if shape.startswith("bf16"):
            x = (x.view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
        arch, _ = C.float_compress_pointer([x], prob_bits=10, ws=ws)
        y = torch.empty_like(x)
        row = [arch[0]]
        iv = torch.int16 if shape.startswith("bf16") else torch.int32
        return (lambda: C.float_compress_pointer([x], prob_bits=10, ws=ws),
                lambda: C.float_decompress_pointer(row, [y], prob_bits=10, ws=ws),
                lambda: torch.equal(x.view(iv), y.view(iv)))
    if shape == "c2":
        g = torch.Generator(device=DEV).manual_seed(0)
        x32 = torch.randn(256, 524288, generator=g, device=DEV)
        x = (x32.view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
        arch, sizes = C.float_compress_stride(x, ws=ws)
        y = torch.empty_like(x)
        return (lambda: C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes),
                lambda: C.float_decompress_stride(arch, 524288, torch.bfloat16, ws=ws, out=y),
                lambda: torch.equal(x.view(torch.int16), y.view(torch.int16)))
    raise SystemExit(f"unknown shape {shape}")


def timed(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    shape = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ws = C.Workspace(3 << 30)
    comp, decomp, check = build(shape, ws)
    decomp()
    torch.cuda.synchronize()
    assert check(), f"{shape}: roundtrip mismatch"
    comp()
    torch.cuda.synchronize()
    tc = timed(comp, reps)
    td = timed(decomp, reps)
    print(f"{shape}: compress {tc * 1e3:.1f} us, decompress {td * 1e3:.1f} us, exact True", flush=True)


if __name__ == "__main__":
    main()
