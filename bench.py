"""Benchmark: encode+decode GB/s of the bf16 float codec on MI355X.

N = 1 (headline, BASELINE.json configs[1], "c2"): a batch of 256 x 1 MiB bf16
tensors (524,288 words each), N(0,1) fp32 truncated to bf16, seeded.
N > 1 (BASELINE.json configs[4], "c5"): a FIXED batch of 8192 x 1 MiB bf16
tensors sharded by contiguous element ranges, 8192 / N per rank (strong
scaling; the tensors' contents do not depend on N).

One step = floatCompress (pointer API, the reference's drop-in path) ->
RCCL all-gather of the per-tensor compressed sizes (N > 1) -> floatDecompress.

value = (uncompressed bytes of the whole batch) / max over ranks of the step
time  (GB/s = 1e9 B/s, reference convention benchmark.py:158-159).

Run:  python bench.py [--gpus N --steps K --warmup W] [--workload c2|c5]
      torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
import glob
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "encode+decode GB/s (+ratio) on bf16 batch at 1/2/4/8 MI355X vs HBM roofline"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--settle-ms", type=float, default=100.0,
                   help="untimed back-to-back steps for this long after the warmup, before the timed "
                        "region (GPU clocks ramp over tens of ms; recorded in the line as settle_ms)")
    p.add_argument("--workload", choices=("auto", "c2", "c5"), default="auto",
                   help="auto: c2 at N=1, c5 (fixed 8192-tensor batch, sharded) at N>1")
    p.add_argument("--batch", type=int, default=256, help="c2 tensors per GPU")
    p.add_argument("--c5-batch", type=int, default=8192, help="c5 tensors in the whole job")
    p.add_argument("--words", type=int, default=524288)
    p.add_argument("--prob-bits", type=int, default=10)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=256,
                   help="tensors of the batch timed on the CPU oracle (rank 0, N=1)")
    p.add_argument("--no-kernel-events", action="store_true",
                   help="time without per-kernel hipEvents (diagnostic)")
    p.add_argument("--no-extras", dest="extras", action="store_false",
                   help="skip the secondary configs (c3 bytes, c4 fp64 / sparse, fp32 batch)")
    p.add_argument("--no-verify", dest="verify", action="store_false",
                   help="skip the round-trip check (kernel-variant timing experiments only)")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import _native as N
    from dietgpu_fork_amd import codec as C
    from dietgpu_fork_amd import dist as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world == 1 and args.gpus > 1:
        raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one rank/GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # launched by torch.distributed.run (WORLD_SIZE set), world 1 included:
    # the multi-GPU step runs as is -- RCCL process group, the size all-gather
    # inside every step, barriers and max-over-ranks timing
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    n, pb = args.words, args.prob_bits
    workload = args.workload if args.workload != "auto" else ("c2" if world == 1 else "c5")
    if workload == "c5":
        total = args.c5_batch
        if total % world:
            raise SystemExit(f"c5: {total} tensors do not shard evenly over {world} ranks")
        first, last = D.shard_range(total, rank, world)
        nb = last - first
        x = _bf16_rows(first, last, n, dev)
    else:
        nb = args.batch
        total = nb * world
        g = torch.Generator(device=dev).manual_seed(rank)  # seed 0
        x32 = torch.randn(nb, n, generator=g, device=dev, dtype=torch.float32)
        x = (x32.view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)  # truncation
        del x32
    U = nb * n * 2  # bytes per rank
    L = N.lib()
    ft = 2
    cols = L.dietgpu_get_max_float_compressed_size(ft, n)
    comp = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
    sizes = torch.empty([nb], dtype=torch.int32, device=dev)
    out = torch.empty_like(x)
    ok = torch.empty([nb], dtype=torch.uint8, device=dev)
    osz = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = C.Workspace(768 << 20, dev)

    in_ptrs = N.ptr_array([x.data_ptr() + i * n * 2 for i in range(nb)])
    in_size = N.u32_array([n] * nb)
    comp_ptrs = N.ptr_array([comp.data_ptr() + i * cols for i in range(nb)])
    out_ptrs = N.ptr_array([out.data_ptr() + i * n * 2 for i in range(nb)])
    caps = N.u32_array([n] * nb)
    stream = torch.cuda.current_stream(dev).cuda_stream
    if os.environ.get("DIETGPU_BENCH_ADDRS"):  # dev: buffer placement of this process
        print("addrs", {k: hex(t.data_ptr()) for k, t in (("x", x), ("comp", comp), ("out", out))},
              file=sys.stderr)

    def step():
        N.check(L.dietgpu_float_compress(ws.h, ft, pb, 0, nb, in_ptrs, in_size, comp_ptrs,
                                         sizes.data_ptr(), stream))
        if distributed:  # the only exchange: per-element compressed sizes (RCCL)
            D.gather_sizes(sizes, total)
        N.check(L.dietgpu_float_decompress(ws.h, ft, pb, 0, nb, comp_ptrs, out_ptrs, caps,
                                           ok.data_ptr(), osz.data_ptr(), stream))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.verify:
        assert bool((ok == 1).all()), "decode reported failure"
        assert torch.equal(out.view(torch.int16), x.view(torch.int16)), "roundtrip mismatch"
    comp_bytes = int(sizes.to(torch.int64).sum().item())

    FAMILIES = ("compress", "hist", "normalize", "encode", "coalesce", "decode")

    def query_families():
        fam = {}
        for k in FAMILIES:
            ms, launches = C.profile_query(k)
            if launches:
                fam[k] = {"avg_ms": ms / launches, "launches": launches}
        return fam

    # the dominant kernel family, from one profiled step (event pair around
    # every launch); the full per-kernel breakdown is taken after the timed
    # region so that the timed steps follow the settle phase directly
    C.profile_reset()
    C.profile_filter(None)
    C.profile(True)
    step()
    torch.cuda.synchronize()
    C.profile(False)
    probe = query_families()
    dominant = max(probe, key=lambda k: probe[k]["avg_ms"]) if probe else None

    # settle: untimed steps for a fixed wall time (clock ramp; no work of the
    # timed region is skipped or cached by it).  The step count is fixed up
    # front and agreed over ranks (every step of a rank > 1 has a collective)
    t_s = time.perf_counter()
    for _ in range(8):
        step()
    torch.cuda.synchronize()
    per_step = (time.perf_counter() - t_s) / 8
    settle_steps = max(0, int(args.settle_ms * 1e-3 / max(per_step, 1e-6)) - 8)
    if distributed:
        c = torch.tensor([settle_steps], dtype=torch.int64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        settle_steps = int(c.item())
    for _ in range(settle_steps):
        step()
    torch.cuda.synchronize()
    settle_steps += 8
    settle_ms = (time.perf_counter() - t_s) * 1e3

    # timed region: barrier + sync on both sides, K steps, max over ranks; the
    # dominant kernel is timed live with hipEvents on its launch stream (only
    # that family is recorded, so the other launches run back to back)
    C.profile_reset()
    C.profile_filter(dominant)
    C.profile(not args.no_kernel_events and dominant is not None)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    t1 = time.perf_counter()
    C.profile(False)
    C.profile_filter(None)
    live = query_families()
    # per-kernel breakdown of the other families: a profiled pass after the
    # timed region
    C.profile_reset()
    C.profile(True)
    for _ in range(max(args.warmup, 3)):
        step()
    torch.cuda.synchronize()
    C.profile(False)
    breakdown = query_families()
    # decode from HBM-sourced archives: the step above
    # decodes archives the compressor has just written, most of which are
    # still in the 256 MiB Infinity Cache (MALL).  Here, after each compress,
    # a 512 MiB fill evicts them before the decode is timed alone; the same
    # isolated timing without the fill is the warm figure.  Untimed for the
    # headline, which stays the reference's compress -> decompress loop.
    decode_cold = None if world > 1 else _decode_cold_warm(step_parts=(
        lambda: N.check(L.dietgpu_float_compress(ws.h, ft, pb, 0, nb, in_ptrs, in_size, comp_ptrs,
                                                 sizes.data_ptr(), stream)),
        lambda: N.check(L.dietgpu_float_decompress(ws.h, ft, pb, 0, nb, comp_ptrs, out_ptrs, caps,
                                                   ok.data_ptr(), osz.data_ptr(), stream))), dev=dev)
    if args.verify:
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int16), x.view(torch.int16)), "roundtrip mismatch (cold decode)"
    elapsed = t1 - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        cb = torch.tensor([comp_bytes], dtype=torch.int64, device=dev)
        dist.all_reduce(cb)
        comp_total = int(cb.item())
    else:
        comp_total = comp_bytes
    ms_per_step = elapsed / args.steps * 1e3
    value = total * n * 2 * args.steps / elapsed / 1e9
    fam = dict(breakdown)
    if dominant in live:
        fam[dominant] = live[dominant]  # the timed region's own measurement

    # algorithmic bytes per launch (Measurement): one launch covers
    # the whole batch; C = compressed bytes (raw section + ANS), U = input.
    algo = {"decode": U + comp_bytes, "encode": U + comp_bytes, "compress": U + comp_bytes, "hist": U,
            "coalesce": 2 * max(comp_bytes - U // 2, 0), "normalize": 0}
    roofline = None
    if dominant:
        ach = algo[dominant] / (fam[dominant]["avg_ms"] * 1e-3) / 1e9
        # PMC traffic is profiled on c2 (tools/profile_gpu.sh) for one build of
        # the library: taken only from a summary of THIS build (its sha256)
        traffic, tsrc = _pmc_traffic(dominant, ft) if workload == "c2" else (None, None)
        roofline = {"bound": "hbm", "kernel": KERNEL_OF[dominant], "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                    "traffic": traffic, "traffic_source": tsrc,
                    "algorithmic_bytes_per_launch": algo[dominant]}
    t_enc = sum(fam[k]["avg_ms"] for k in ("compress", "hist", "normalize", "encode", "coalesce") if k in fam)
    t_dec = fam.get("decode", {}).get("avg_ms", 0.0)
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "settle_ms": round(settle_ms, 1), "settle_steps": settle_steps,
        "higher_is_better": True,
        "scaling": "strong" if workload == "c5" else "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic",
        "distributed": distributed,
        "config": {"workload": (f"c5: batch={total} x {n * 2 // 1048576} MiB bf16 N(0,1) in total, "
                                f"{nb} per GPU" if workload == "c5" else
                                f"c2: batch={nb} x {n * 2 // 1048576} MiB bf16 N(0,1) per GPU"),
                   "batch_per_gpu": nb, "words_per_tensor": n, "prob_bits": pb,
                   "api": "floatCompress + floatDecompress (pointer API, C ABI)",
                   "parallelism": f"dp{world} (independent shards + RCCL size all-gather)"},
        "ratio": round(comp_total / (total * n * 2), 5),
        "encode_plus_decode_algorithmic_GBps": (round(2 * (U + comp_bytes) / ((t_enc + t_dec) * 1e-3) / 1e9, 1)
                                                if t_enc and t_dec else None),
        "compress_GBps_kernels": round(U / (t_enc * 1e-3) / 1e9, 1) if t_enc else None,
        "decompress_GBps_kernels": round(U / (t_dec * 1e-3) / 1e9, 1) if t_dec else None,
        "kernels": {k: round(v["avg_ms"], 5) for k, v in fam.items()},
        "kernels_note": "avg ms per launch: dominant kernel from hipEvents in the timed region, "
                        "others from a profiled pass outside it",
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if decode_cold:
        # the step with the decode reading its archives from HBM: the timed
        # step's own decode replaced by the isolated cold one
        t_hot, t_cold = decode_cold["decode_warm_ms"], decode_cold["decode_cold_ms"]
        dec_live = fam.get("decode", {}).get("avg_ms", t_hot)
        step_cold = ms_per_step - dec_live + t_cold
        decode_cold.update({
            "step_cold_ms": round(step_cold, 4),
            "encode_plus_decode_algorithmic_GBps_cold": round(2 * (U + comp_bytes) / (step_cold * 1e-3) / 1e9, 1),
            "decode_cold_algorithmic_GBps": round((U + comp_bytes) / (t_cold * 1e-3) / 1e9, 1),
            "decode_warm_algorithmic_GBps": round((U + comp_bytes) / (t_hot * 1e-3) / 1e9, 1)})
        line["decode_hbm"] = decode_cold
        line["encode_plus_decode_algorithmic_GBps_step"] = round(2 * (U + comp_bytes) / (ms_per_step * 1e-3) / 1e9, 1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = _cpu_baseline(x, min(args.cpu_sample, nb), pb)
    if world == 1 and workload == "c2" and args.extras:
        del comp, out, x, ws
        torch.cuda.empty_cache()
        line["extras"] = _extras(dev, pb)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


def _bf16_rows(first, last, n, dev, chunk=512):
    """Rows [first, last) of the c5 batch: N(0,1) fp32 truncated to bf16, the
    rows of chunk c drawn from seed c (seed 0 for the first
    chunk), so every row's contents are the same whatever the sharding."""
    import torch

    x = torch.empty([last - first, n], dtype=torch.bfloat16, device=dev)
    for c in range(first // chunk, -(-last // chunk)):
        g = torch.Generator(device=dev).manual_seed(c)
        x32 = torch.randn(chunk, n, generator=g, device=dev, dtype=torch.float32)
        a, b = max(first, c * chunk), min(last, (c + 1) * chunk)
        rows = (x32[a - c * chunk:b - c * chunk].view(torch.int32) >> 16).to(torch.int16)
        x[a - first:b - first] = rows.view(torch.bfloat16)
        del x32
    return x


def _decode_cold_warm(step_parts, dev, reps=8, flush_bytes=512 << 20):
    """Isolated decode times (torch events on the launch stream): `warm`
    right after a compress (archives partly in the MALL, as in the timed
    step), `cold` after a compress and a read of a flush_bytes buffer that
    evicts them (the decoder then reads its archives from HBM).  The flush
    only reads, so it leaves no dirty lines whose write-back would land in
    the timed decode."""
    import torch

    compress, decompress = step_parts
    scratch = torch.ones(flush_bytes // 4, dtype=torch.int32, device=dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for name, flush in (("warm", False), ("cold", True)):
        tot = 0.0
        for i in range(reps + 1):
            compress()
            if flush:
                scratch.sum()
            a.record()
            decompress()
            b.record()
            b.synchronize()
            if i:  # the first of each kind untimed
                tot += a.elapsed_time(b)
        res[f"decode_{name}_ms"] = round(tot / reps, 5)
    del scratch
    res["note"] = (f"decode timed alone after a compress; cold: a {flush_bytes >> 20} MiB read between them "
                   "evicts the archives from the 256 MiB Infinity Cache")
    return res


def _timed(fn, reps, min_ms=2.0, max_reps=50):
    """Average ms of fn() over back-to-back calls (torch events on the current
    stream, which is the stream the C ABI launches on): at least `reps`, and
    for short calls enough of them to cover ~min_ms, so the host's enqueue of
    one call overlaps the GPU work of the previous one (steady state)."""
    import torch

    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    b.synchronize()
    reps = max(reps, min(max_reps, int(min_ms / max(a.elapsed_time(b), 1e-3)) + 1))
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def _extras(dev, pb, reps=3):
    """Secondary BASELINE configs on this GPU (not the headline): whole-call
    compress and decompress times (every kernel of the call, inputs resident
    in HBM), ratio, and a bit-exact roundtrip check.  U/t is the reference's
    GB/s convention; `algorithmic_GBps` is 2(U + C) / (t_c + t_d)."""
    import torch

    from dietgpu_fork_amd import codec as C

    out = []

    fams = ("compress", "hist", "normalize", "encode", "coalesce", "decode", "sparse")

    def breakdown(fc, fd):
        """avg ms per launch of each kernel family over four back-to-back
        profiled calls of each direction (event pairs around every launch)"""
        r = {}
        for tag, fn in (("c", fc), ("d", fd)):
            torch.cuda.synchronize()
            C.profile_reset()
            C.profile_filter(None)
            # an unprofiled call first, so the GPU is busy while the host
            # enqueues the profiled ones: an event pair around a launch the
            # idle GPU waits for would time the host's launch latency too
            fn()
            C.profile(True)
            for _ in range(4):
                fn()
            torch.cuda.synchronize()
            C.profile(False)
            for k in fams:
                ms, launches = C.profile_query(k)
                if launches:
                    r[f"{tag}:{k}"] = round(ms / launches, 4)
        return r

    def roofline_of(U, C_bytes, tc, td, kern):
        """HBM roofline of the whole call (2(U + C) over compress + decompress
        time) and of its dominant data kernel: the family of the largest avg
        launch time among those with algorithmic bytes (U + C for the
        encoders and the decoder, U for the histogram pass), timed by the
        profiled pass's event pairs (which include each launch's overhead)."""
        call = 2 * (U + C_bytes) / ((tc + td) * 1e-3) / 1e9
        r = {"bound": "hbm", "peak": HBM_PEAK_GBPS, "unit": "GB/s",
             "call_achieved": round(call, 1), "call_frac": round(call / HBM_PEAK_GBPS, 4)}
        algo = {"compress": U + C_bytes, "encode": U + C_bytes, "decode": U + C_bytes, "hist": U}
        # (sparse calls: the dense kernels work on the compacted list, not on
        # U, so only the whole call is priced)
        cand = [(ms, k[2:]) for k, ms in (kern or {}).items()
                if k[2:] in algo and ms > 0 and "c:sparse" not in kern]
        if cand:
            ms, fam_ = max(cand)
            ach = algo[fam_] / (ms * 1e-3) / 1e9
            r.update({"kernel": KERNEL_OF[fam_], "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBPS, 4),
                      "algorithmic_bytes_per_launch": algo[fam_]})
        return r

    def record(name, U, C_bytes, tc, td, exact, **kw):
        out.append({"config": name, "uncompressed_bytes": U, "ratio": round(C_bytes / U, 5),
                    "compress_ms": round(tc, 4), "decompress_ms": round(td, 4),
                    "compress_GBps": round(U / tc / 1e6, 1), "decompress_GBps": round(U / td / 1e6, 1),
                    "encode_plus_decode_GBps": round(U / (tc + td) / 1e6, 1),
                    "algorithmic_GBps": round(2 * (U + C_bytes) / (tc + td) / 1e6, 1),
                    "roundtrip_bit_exact": bool(exact),
                    "roofline": roofline_of(U, C_bytes, tc, td, kw.get("kernels_ms")), **kw})

    # c3: 1024 x 4 MiB bytes, uniform over 16 symbols (4.0 bit/sym)
    nb, n = 1024, 4 << 20
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randint(0, 16, (nb, n), generator=g, device=dev, dtype=torch.uint8)
    ws = C.Workspace(7 << 30, dev)
    arch, sizes = C.ans_encode_stride(x, prob_bits=pb, ws=ws)
    y, ok, _ = C.ans_decode_stride(arch, n, prob_bits=pb, ws=ws)
    tc = _timed(lambda: C.ans_encode_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes), reps)
    td = _timed(lambda: C.ans_decode_stride(arch, n, prob_bits=pb, ws=ws, out=y), reps)
    exact = bool((ok == 1).all()) and torch.equal(x, y)
    kern = breakdown(lambda: C.ans_encode_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes),
                     lambda: C.ans_decode_stride(arch, n, prob_bits=pb, ws=ws, out=y))
    record("c3: 1024 x 4 MiB bytes, 4 bit/sym (ansEncodeBatchStride / ansDecodeBatchStride)",
           nb * n, int(sizes.to(torch.int64).sum()), tc, td, exact, kernels_ms=kern)
    del x, y, arch, ws
    torch.cuda.empty_cache()

    # float batches of the c2 shape in the other float types
    for dt, words in ((torch.float32, 262144), (torch.float16, 524288)):
        g = torch.Generator(device=dev).manual_seed(11)
        x = torch.randn(256, words, generator=g, device=dev).to(dt)
        ws = C.Workspace(1 << 30, dev)
        arch, sizes = C.float_compress_stride(x, prob_bits=pb, ws=ws)
        y, ok, _ = C.float_decompress_stride(arch, words, dt, prob_bits=pb, ws=ws)
        tc = _timed(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes), reps)
        td = _timed(lambda: C.float_decompress_stride(arch, words, dt, prob_bits=pb, ws=ws, out=y), reps)
        exact = bool((ok == 1).all()) and torch.equal(x.view(torch.uint8), y.view(torch.uint8))
        kern = breakdown(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes),
                         lambda: C.float_decompress_stride(arch, words, dt, prob_bits=pb, ws=ws, out=y))
        record(f"256 x 1 MiB {str(dt)[6:]} N(0,1) (floatCompress stride)", x.numel() * x.element_size(),
               int(sizes.to(torch.int64).sum()), tc, td, exact, kernels_ms=kern)
        del x, y, arch, ws

    # batch 1 x 128*512*1024 words (one large tensor):
    # the whole batch is a single element, so it takes the three-kernel path
    for dt in (torch.bfloat16, torch.float16, torch.float32):
        words = 128 * 512 * 1024
        g = torch.Generator(device=dev).manual_seed(13)
        x = torch.randn(1, words, generator=g, device=dev).to(dt)
        ws = C.Workspace(1 << 30, dev)
        arch, sizes = C.float_compress_stride(x, prob_bits=pb, ws=ws)
        y, ok, _ = C.float_decompress_stride(arch, words, dt, prob_bits=pb, ws=ws)
        tc = _timed(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes), reps)
        td = _timed(lambda: C.float_decompress_stride(arch, words, dt, prob_bits=pb, ws=ws, out=y), reps)
        exact = bool((ok == 1).all()) and torch.equal(x.view(torch.uint8), y.view(torch.uint8))
        kern = breakdown(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes),
                         lambda: C.float_decompress_stride(arch, words, dt, prob_bits=pb, ws=ws, out=y))
        record(f"batch 1 x 128*512*1024 {str(dt)[6:]} N(0,1) (one element)", x.numel() * x.element_size(),
               int(sizes.to(torch.int64).sum()), tc, td, exact, kernels_ms=kern)
        del x, y, arch, ws
        torch.cuda.empty_cache()

    # per-call latency of the torch ops (host validation + launch) on a small
    # batch: 8 x 4096 fp16, the kernels themselves take a few microseconds
    # (fp16, not bf16: these 220 small launches would otherwise share the
    # headline kernels' names in a rocprofv3 --stats summary of this command)
    xs = [torch.randn(4096, device=dev).to(torch.float16) for _ in range(8)]
    tmp = torch.empty([64 << 20], dtype=torch.uint8, device=dev)
    comp, csz, _ = torch.ops.dietgpu.compress_data(True, xs, False, tmp)
    rows = [comp[i, : int(csz[i])] for i in range(len(xs))]
    outs = [torch.empty_like(t) for t in xs]
    lat = {}
    for name, fn in (("compress_data", lambda: torch.ops.dietgpu.compress_data(True, xs, False, tmp)),
                     ("decompress_data", lambda: torch.ops.dietgpu.decompress_data(True, rows, outs, False, tmp))):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            fn()
        t_host = (time.perf_counter() - t0) / 200
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 200
        lat[name] = {"host_us_per_call": round(t_host * 1e6, 2), "us_per_call_synced": round(t_all * 1e6, 2)}
    out.append({"config": "torch.ops.dietgpu per-call latency, 8 x 4096 fp16, 64 MiB temp_mem", **lat})
    del xs, tmp, comp, rows, outs

    # c4: fp64 two-pass (16,777,216 words) and 90 %-sparse fp32 (15,000,000)
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn(16777216, generator=g, device=dev, dtype=torch.float64)
    ws = C.Workspace(2 << 30, dev)
    arch, sizes = C.float_compress_pointer([x], prob_bits=pb, ws=ws)
    y = torch.empty_like(x)
    row = [arch[0]]
    ok, _ = C.float_decompress_pointer(row, [y], prob_bits=pb, ws=ws)
    tc = _timed(lambda: C.float_compress_pointer([x], prob_bits=pb, ws=ws), reps)
    td = _timed(lambda: C.float_decompress_pointer(row, [y], prob_bits=pb, ws=ws), reps)
    exact = int(ok[0]) == 1 and torch.equal(x.view(torch.int64), y.view(torch.int64))
    kern = breakdown(lambda: C.float_compress_pointer([x], prob_bits=pb, ws=ws),
                     lambda: C.float_decompress_pointer(row, [y], prob_bits=pb, ws=ws))
    record("c4: 1 x 128 MiB fp64 N(0,1), two ANS passes", x.numel() * 8, int(sizes[0]), tc, td, exact,
           kernels_ms=kern)
    # sparse: the reference's SparseFloatBenchmark shape (15M words, 90 %
    # zeros) at batch 1 and 5
    for nbs in (1, 5):
        g = torch.Generator(device=dev).manual_seed(5)
        fs = []
        for _ in range(nbs):
            f = torch.randn(15000000, generator=g, device=dev)
            f[torch.rand(f.numel(), generator=g, device=dev) < 0.9] = 0.0
            fs.append(f)
        arch, sizes = C.sparse_compress(fs, prob_bits=pb, ws=ws)
        ys = [torch.empty_like(f) for f in fs]
        rows = [arch[i, : int(sizes[i])] for i in range(nbs)]
        ok, _ = C.sparse_decompress(rows, ys, prob_bits=pb, ws=ws)
        tc = _timed(lambda: C.sparse_compress(fs, prob_bits=pb, ws=ws), reps)
        td = _timed(lambda: C.sparse_decompress(rows, ys, prob_bits=pb, ws=ws), reps)
        exact = bool((ok == 1).all()) and all(torch.equal(a.view(torch.int32), b.view(torch.int32))
                                              for a, b in zip(fs, ys))
        kern = breakdown(lambda: C.sparse_compress(fs, prob_bits=pb, ws=ws),
                         lambda: C.sparse_decompress(rows, ys, prob_bits=pb, ws=ws))
        record(f"c4: {nbs} x 15M fp32, 90 % zeros (sparse bitmap + dense codec)", nbs * 15000000 * 4,
               int(sizes.to(torch.int64).sum()), tc, td, exact, kernels_ms=kern)
        del fs, ys, arch, rows
    del x, y, ws
    torch.cuda.empty_cache()
    out.extend(_extras_small_batches(dev, pb, record, breakdown))
    out.extend(_extras_batch1_sweep(dev, pb, record, breakdown))
    out.extend(_extras_reference_grid(dev))
    out.append(_extras_float_benchmark_grid(dev))
    out.append(_extras_sparse_benchmark_grid(dev))
    out.append(_extras_c5_g1(dev, pb))
    return out


def _bf16_trunc(nb, words, seed, dev):
    """[nb, words] N(0,1) fp32 truncated to bf16, generated in
    row chunks of at most 2^28 words (fp32 temporaries)."""
    import torch

    x = torch.empty([nb, words], dtype=torch.bfloat16, device=dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    flat = x.view(-1)
    step = 1 << 28
    for i in range(0, flat.numel(), step):
        m = min(step, flat.numel() - i)
        f = torch.randn(m, generator=g, device=dev, dtype=torch.float32)
        flat[i:i + m] = (f.view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16)
        del f
    return x


def _extras_small_batches(dev, pb, record, breakdown):
    """batches whose single-pass teams were not
    XCD-aligned before round 5 (1-7 multi-item elements; 33 x 1e6 words,
    whose teams cannot be aligned within the resident grid).  Timed as the
    library routes them (the size rule sends all four to the three-kernel
    path, csrc/codec.hip persistentPreferred), and once more forced through
    the single-pass compressor (dietgpu_set_compress_path) with its
    team-barrier fallback count over every timed call (must be 0: a
    fallback means a hand-off that waited out the 200 us budget)."""
    import torch

    from dietgpu_fork_amd import codec as C

    for nb, words in ((1, 1000000), (1, 524288), (3, 524288), (33, 1000000)):
        x = _bf16_trunc(nb, words, 17 + nb, dev)
        ws = C.Workspace(1 << 30, dev)
        arch, sizes = C.float_compress_stride(x, prob_bits=pb, ws=ws)
        y, ok, _ = C.float_decompress_stride(arch, words, torch.bfloat16, prob_bits=pb, ws=ws)
        tc = _timed(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes), 3,
                    max_reps=400)
        ref = arch.clone()
        C.barrier_fallback_count(reset=True)
        with C.compress_path("single-pass"):
            tc_sp = _timed(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes), 3,
                           max_reps=400)
        fb = C.barrier_fallback_count(reset=True)
        same = torch.equal(arch, ref)
        del ref
        td = _timed(lambda: C.float_decompress_stride(arch, words, torch.bfloat16, prob_bits=pb, ws=ws, out=y), 3,
                    max_reps=400)
        exact = bool((ok == 1).all()) and torch.equal(x.view(torch.int16), y.view(torch.int16))
        kern = breakdown(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes),
                         lambda: C.float_decompress_stride(arch, words, torch.bfloat16, prob_bits=pb, ws=ws,
                                                           out=y))
        record(f"small batch {nb} x {words} bf16 N(0,1) (floatCompress stride; size-rule path, "
               f"single-pass forced for the fallback count)",
               x.numel() * 2, int(sizes.to(torch.int64).sum()), tc, td, exact and same, kernels_ms=kern,
               single_pass_compress_ms=round(tc_sp, 4), barrier_fallbacks=fb)
        del x, y, arch, ws
    torch.cuda.empty_cache()
    return []


def _extras_batch1_sweep(dev, pb, record, breakdown):
    """The reference's published batch-1 bf16 curve (README.md:112-118, the
    A100 plot: 1e6 / 16e6 / 128e6 / 1.07e9 words)."""
    import torch

    from dietgpu_fork_amd import codec as C

    for words in (1000000, 16000000, 128000000, 1070000000):
        x = _bf16_trunc(1, words, 19, dev)
        ws = C.Workspace((1 << 30) + 2 * words * 2, dev)
        arch, sizes = C.float_compress_stride(x, prob_bits=pb, ws=ws)
        y, ok, _ = C.float_decompress_stride(arch, words, torch.bfloat16, prob_bits=pb, ws=ws)
        reps = 3 if words > 1e8 else 10
        tc = _timed(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes), reps,
                    max_reps=400)
        td = _timed(lambda: C.float_decompress_stride(arch, words, torch.bfloat16, prob_bits=pb, ws=ws, out=y),
                    reps, max_reps=400)
        exact = bool((ok == 1).all()) and torch.equal(x.view(torch.int16), y.view(torch.int16))
        kern = breakdown(lambda: C.float_compress_stride(x, prob_bits=pb, ws=ws, out=arch, sizes=sizes),
                         lambda: C.float_decompress_stride(arch, words, torch.bfloat16, prob_bits=pb, ws=ws,
                                                           out=y))
        record(f"batch-1 sweep: 1 x {words:.3g} bf16 N(0,1) (README.md:118 A100 curve)", x.numel() * 2,
               int(sizes.to(torch.int64).sum()), tc, td, exact, kernels_ms=kern)
        del x, y, arch, ws
        torch.cuda.empty_cache()
    return []


def _extras_reference_grid(dev):
    """benchmark.py:151-223, measured as the reference measures it: through
    torch.ops.dietgpu.compress_data / decompress_data with a 384 MiB temp
    buffer, float codec and raw-ANS byte codec on bf16 / fp16 / fp32
    N(0,1) data, non-batched (1 x 128*512*1024) and batched
    (128 x 512*1024); an event pair around each op call, the first of four
    runs untimed (benchmark.py:27-90), then the same calls back to back
    (device throughput without the host's per-call latency)."""
    import torch

    import dietgpu_fork_amd  # noqa: F401

    res = []
    tmp = torch.empty([384 << 20], dtype=torch.uint8, device=dev)
    for as_float in (True, False):
        for dt in (torch.bfloat16, torch.float16, torch.float32):
            for shape in ("non-batched [128 * 512 * 1024]", "batched [128, [512 * 1024]]"):
                g = torch.Generator(device=dev).manual_seed(23)
                if shape.startswith("non"):
                    ts = [torch.normal(0, 1.0, [128 * 512 * 1024], generator=g, device=dev).to(dt)]
                else:
                    ts = [torch.normal(0, 1.0, [512 * 1024], generator=g, device=dev).to(dt) for _ in range(128)]
                size_fn = (torch.ops.dietgpu.max_float_compressed_output_size if as_float
                           else torch.ops.dietgpu.max_any_compressed_output_size)
                rows, cols = size_fn(ts)
                comp = torch.empty([rows, cols], dtype=torch.uint8, device=dev)
                sizes = torch.zeros([len(ts)], dtype=torch.int, device=dev)
                outs = [torch.empty_like(t) for t in ts]
                st = torch.empty([len(ts)], dtype=torch.uint8, device=dev)
                osz = torch.empty([len(ts)], dtype=torch.int32, device=dev)
                comp_ts = [*comp]

                def fc():
                    torch.ops.dietgpu.compress_data(as_float, ts, False, tmp, comp, sizes)

                def fd():
                    torch.ops.dietgpu.decompress_data(as_float, comp_ts, outs, False, tmp, st, osz)

                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                tcs, tds = [], []
                for i in range(4):
                    a.record()
                    fc()
                    b.record()
                    torch.cuda.synchronize()
                    tcs.append(a.elapsed_time(b))
                    a.record()
                    fd()
                    b.record()
                    torch.cuda.synchronize()
                    tds.append(a.elapsed_time(b))
                exact = bool((st == 1).all()) and all(torch.equal(p.view(torch.uint8), q.view(torch.uint8))
                                                      for p, q in zip(ts, outs))
                U = sum(t.numel() * t.element_size() for t in ts)
                Cb = int(sizes.to(torch.int64).sum())
                tc_ref, td_ref = sum(tcs[1:]) / 3, sum(tds[1:]) / 3
                tc, td = _timed(fc, 3), _timed(fd, 3)
                call = 2 * (U + Cb) / ((tc + td) * 1e-3) / 1e9
                res.append({
                    "config": f"benchmark.py {'float codec' if as_float else 'raw ANS byte-wise'} "
                              f"{shape} {str(dt)[6:]} (torch.ops.dietgpu, 384 MiB temp)",
                    "uncompressed_bytes": U, "ratio": round(Cb / U, 5),
                    "ref_protocol_compress_ms": round(tc_ref, 4), "ref_protocol_decompress_ms": round(td_ref, 4),
                    "ref_protocol_compress_GBps": round(U / tc_ref / 1e6, 1),
                    "ref_protocol_decompress_GBps": round(U / td_ref / 1e6, 1),
                    "compress_ms": round(tc, 4), "decompress_ms": round(td, 4),
                    "compress_GBps": round(U / tc / 1e6, 1), "decompress_GBps": round(U / td / 1e6, 1),
                    "roundtrip_bit_exact": exact,
                    "roofline": {"bound": "hbm", "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                 "call_achieved": round(call, 1), "call_frac": round(call / HBM_PEAK_GBPS, 4)}})
                del ts, outs, comp, comp_ts
    del tmp
    torch.cuda.empty_cache()
    return res


FT_OF = {"float16": 1, "bfloat16": 2, "float32": 3, "float64": 4}
INT_OF = {2: "int16", 4: "int32", 8: "int64"}


def _grid_row(ft_name, nb, words, U, Cb, tc, td, exact, **kw):
    """One compact row of a benchmark grid: whole-call times (back-to-back
    calls, events on the launch stream), the reference's GB/s (U / t), and
    the call's HBM roofline 2(U + C) / (t_c + t_d) against 8 TB/s."""
    call = 2 * (U + Cb) / ((tc + td) * 1e-3) / 1e9
    return {"type": ft_name, "batch": nb, "words": words, "ratio": round(Cb / U, 5),
            "compress_ms": round(tc, 4), "decompress_ms": round(td, 4),
            "compress_GBps": round(U / tc / 1e6, 1), "decompress_GBps": round(U / td / 1e6, 1),
            "call_GBps": round(call, 1), "call_frac": round(call / HBM_PEAK_GBPS, 4),
            "roundtrip_bit_exact": bool(exact), **kw}


def _extras_float_benchmark_grid(dev):
    """The fork's own float_benchmark (FloatBenchmark.cu:401-427, README.md:20):
    fp16 / bf16 / fp32 / fp64, batch 1 x {1e5, 1.5e5, 1e6, 1.5e6, 1e7, 1.5e7,
    1e8} N(0,1) words, pb 9, floatCompress / floatDecompress pointer API
    (FloatBenchmark.cu:224-273).  Each point: bit-exact roundtrip check and
    whole-call roofline."""
    import torch

    from dietgpu_fork_amd import codec as C

    rows = []
    ws = C.Workspace(2 << 30, dev)
    for name, dt in (("float16", torch.float16), ("bfloat16", torch.bfloat16), ("float32", torch.float32),
                     ("float64", torch.float64)):
        for words in (100000, 150000, 1000000, 1500000, 10000000, 15000000, 100000000):
            g = torch.Generator(device=dev).manual_seed(10 + words)
            x = torch.randn(words, generator=g, device=dev, dtype=torch.float64 if dt == torch.float64
                            else torch.float32).to(dt)
            arch, sizes = C.float_compress_pointer([x], prob_bits=9, ws=ws)
            row = [arch[0]]
            y = torch.empty_like(x)
            ok, _ = C.float_decompress_pointer(row, [y], prob_bits=9, ws=ws)
            iv = getattr(torch, INT_OF[x.element_size()])
            exact = int(ok[0]) == 1 and torch.equal(x.view(iv), y.view(iv))
            reps = 3 if words >= 1e7 else 10
            tc = _timed(lambda: C.float_compress_pointer([x], prob_bits=9, ws=ws), reps, max_reps=400)
            td = _timed(lambda: C.float_decompress_pointer(row, [y], prob_bits=9, ws=ws), reps, max_reps=400)
            rows.append(_grid_row(name, 1, words, x.numel() * x.element_size(), int(sizes[0]), tc, td, exact))
            del x, y, arch, row
        torch.cuda.empty_cache()
    del ws
    torch.cuda.empty_cache()
    return {"config": "float_benchmark grid (FloatBenchmark.cu:421-427): 4 float types x batch 1 x "
                      "{1e5 .. 1e8} N(0,1) words, pb 9, floatCompress / floatDecompress pointer API",
            "rows": rows}


def _extras_sparse_benchmark_grid(dev):
    """The fork's sparse_float_benchmark (SparseFloatBenchmark.cu:395-447):
    fp16 / bf16 / fp32 / fp64 x batch {1, 3, 5} x {1e5, 1.5e5, 1e6, 1.5e6,
    1e7, 1.5e7} words per element, 50 % zeros (generateSparseFloats'
    default), N(0,1) nonzeros, pb 9, sparse compress / decompress.  Each
    point: bit-exact roundtrip check and whole-call roofline (U = the dense
    input bytes, as the reference's GB/s counts them)."""
    import torch

    from dietgpu_fork_amd import codec as C

    rows = []
    ws = C.Workspace(2 << 30, dev)
    for name, dt in (("float16", torch.float16), ("bfloat16", torch.bfloat16), ("float32", torch.float32),
                     ("float64", torch.float64)):
        for nbs in (1, 3, 5):
            for words in (100000, 150000, 1000000, 1500000, 10000000, 15000000):
                g = torch.Generator(device=dev).manual_seed(10 + nbs * words)
                fs = []
                for _ in range(nbs):
                    f = torch.randn(words, generator=g, device=dev,
                                    dtype=torch.float64 if dt == torch.float64 else torch.float32).to(dt)
                    f[torch.rand(words, generator=g, device=dev) < 0.5] = 0
                    fs.append(f)
                arch, sizes = C.sparse_compress(fs, prob_bits=9, ws=ws)
                ys = [torch.empty_like(f) for f in fs]
                rws = [arch[i, : int(sizes[i])] for i in range(nbs)]
                ok, _ = C.sparse_decompress(rws, ys, prob_bits=9, ws=ws)
                iv = getattr(torch, INT_OF[fs[0].element_size()])
                exact = bool((ok == 1).all()) and all(torch.equal(a.view(iv), b.view(iv)) for a, b in zip(fs, ys))
                reps = 3 if words >= 1e7 else 10
                tc = _timed(lambda: C.sparse_compress(fs, prob_bits=9, ws=ws), reps, max_reps=400)
                td = _timed(lambda: C.sparse_decompress(rws, ys, prob_bits=9, ws=ws), reps, max_reps=400)
                rows.append(_grid_row(name, nbs, words, nbs * words * fs[0].element_size(),
                                      int(sizes.to(torch.int64).sum()), tc, td, exact))
                del fs, ys, arch, rws
            torch.cuda.empty_cache()
    del ws
    torch.cuda.empty_cache()
    return {"config": "sparse_float_benchmark grid (SparseFloatBenchmark.cu:440-447): 4 float types x batch "
                      "{1, 3, 5} x {1e5 .. 1.5e7} words, 50 % zeros, pb 9, sparse compress / decompress",
            "rows": rows}


def _extras_c5_g1(dev, pb, steps=10):
    """c5 at G = 1 (BASELINE configs[4]: 8192 x 1 MiB bf16, the whole
    strong-scaling batch on one GPU): the N = 1 anchor of the scaling curve,
    same step as the headline (pointer API compress + decompress)."""
    import torch

    from dietgpu_fork_amd import _native as N
    from dietgpu_fork_amd import codec as C

    nb, n = 8192, 524288
    x = _bf16_rows(0, nb, n, dev)
    L = N.lib()
    cols = L.dietgpu_get_max_float_compressed_size(2, n)
    comp = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
    sizes = torch.empty([nb], dtype=torch.int32, device=dev)
    out = torch.empty_like(x)
    ok = torch.empty([nb], dtype=torch.uint8, device=dev)
    osz = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = C.Workspace(768 << 20, dev)
    in_ptrs = N.ptr_array([x.data_ptr() + i * n * 2 for i in range(nb)])
    in_size = N.u32_array([n] * nb)
    comp_ptrs = N.ptr_array([comp.data_ptr() + i * cols for i in range(nb)])
    out_ptrs = N.ptr_array([out.data_ptr() + i * n * 2 for i in range(nb)])
    caps = N.u32_array([n] * nb)
    stream = torch.cuda.current_stream(dev).cuda_stream
    C.barrier_fallback_count(reset=True)

    def step():
        N.check(L.dietgpu_float_compress(ws.h, 2, pb, 0, nb, in_ptrs, in_size, comp_ptrs, sizes.data_ptr(), stream))
        N.check(L.dietgpu_float_decompress(ws.h, 2, pb, 0, nb, comp_ptrs, out_ptrs, caps, ok.data_ptr(),
                                           osz.data_ptr(), stream))

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    exact = bool((ok == 1).all()) and torch.equal(out.view(torch.int16), x.view(torch.int16))
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    U = nb * n * 2
    Cb = int(sizes.to(torch.int64).sum())
    alg = 2 * (U + Cb) / (ms * 1e-3) / 1e9
    fb = C.barrier_fallback_count(reset=True)
    r = {"config": "c5 at G = 1: 8192 x 1 MiB bf16 N(0,1), pointer API compress + decompress "
                   "(BASELINE configs[4], the strong-scaling batch on one GPU)",
         "uncompressed_bytes": U, "ratio": round(Cb / U, 5), "ms_per_step": round(ms, 3),
         "GBps": round(U / ms / 1e6, 1), "steps": steps, "roundtrip_bit_exact": exact, "barrier_fallbacks": fb,
         "roofline": {"bound": "hbm", "peak": HBM_PEAK_GBPS, "unit": "GB/s", "call_achieved": round(alg, 1),
                      "call_frac": round(alg / HBM_PEAK_GBPS, 4)}}
    del x, comp, out, ws
    torch.cuda.empty_cache()
    return r


# profiling family (csrc/profile.h scopes) -> kernel symbol
KERNEL_OF = {"compress": "k_pcompress", "hist": "k_hist", "normalize": "k_normalize", "encode": "k_encode",
             "coalesce": "k_coalesce", "decode": "k_decode", "sparse": "k_sparse"}


def library_sha256():
    """sha256 of the HIP library this process runs (dietgpu_fork_amd/_lib)."""
    import hashlib

    p = os.path.join(ROOT, "dietgpu_fork_amd", "_lib", "libdietgpu_amd.so")
    try:
        return hashlib.sha256(open(p, "rb").read()).hexdigest()
    except OSError:
        return None


def _pmc_traffic(kernel, ft):
    """(HBM bytes per launch, source file) of `kernel`'s instance for float
    type `ft` from the newest committed rocprofv3 PMC summary
    (profiles/*pmc*.json, written by tools/pmc_summary.py, keyed per template
    instance) that was collected on THIS build of the library (its
    library_sha256): counters of another build would silently describe other
    code.  (None, reason) when there is none."""
    def natural(f):  # r01_v10 after r01_v9
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))]

    lib = library_sha256()
    # newest summary first; within a round the profile of the driver's own
    # command (profiles/rNN_driver_cmd_pmc.json) before the others
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")),
                   key=lambda f: (natural(f)[:2], "driver_cmd" in f, natural(f)))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if lib is None or d.get("library_sha256") != lib:
            continue
        for name, k in d.get("kernels", {}).items():
            if name.startswith(f"{KERNEL_OF[kernel]}<{ft},") and "hbm_bytes_per_launch" in k:
                return k["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, "no committed PMC summary of this library build (sha256 %s)" % (lib or "?")[:16]


def _cpu_baseline(x, sample, pb, min_seconds=12.0, max_passes=40):
    """Serial C oracle (oracle/dietgpu_oracle.c, the CPU restatement) on the
    same c2 tensors: whole compress+decompress passes over `sample` tensors,
    repeated until >= min_seconds of CPU work (a bounded sample, so the
    default bench still finishes in minutes).  value = bytes / seconds."""
    import numpy as np
    import torch

    from oracle import oracle as O

    words = x[:sample].view(torch.int16).cpu().numpy().view(np.uint16)
    U = words.nbytes
    tot = te_s = td_s = 0.0
    passes = 0
    comp = 0
    while passes < max_passes and (passes == 0 or tot < min_seconds):
        t, comp, te, td = O.time_float_roundtrip(words, 2, pb, threads=1)
        tot += t
        te_s += te
        td_s += td
        passes += 1
    # supplementary: the same oracle on 16 threads (the GPU box's CPU share;
    # elements split across threads), a few seconds of work
    T = min(16, os.cpu_count() or 1)
    mt_tot = 0.0
    mt_passes = 0
    while mt_passes < max_passes and (mt_passes == 0 or mt_tot < 4.0):
        mt_tot += O.time_float_roundtrip(words, 2, pb, threads=T)[0]
        mt_passes += 1
    multithread = {"value": round(mt_passes * U / mt_tot / 1e9, 4), "unit": "GB/s", "cores": T,
                   "passes": mt_passes, "seconds": round(mt_tot, 3)}
    return {"value": round(passes * U / tot / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "multithread": multithread,
            "sample": f"{sample} x {words.shape[1] * 2 // 1048576} MiB bf16 of the c2 batch, "
                      f"{passes} passes of compress+decompress, serial C oracle "
                      f"(oracle/dietgpu_oracle.c), 1 thread",
            "seconds": round(tot, 3), "compress_s": round(te_s, 3), "decompress_s": round(td_s, 3),
            "ratio": round(comp / U, 5), "host_cpus": os.cpu_count(), "host_cpu_model": _cpu_model()}


def _cpu_model():
    """The host CPU's model name (report the lscpu model)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


if __name__ == "__main__":
    main()
