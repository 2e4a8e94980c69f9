"""The compressor's persistent sync arena (csrc/sync_arena.{h,cpp}): the
single-pass k_pcompress and the fused three-kernel k_encode keep their
look-back flags, epoch-tagged, in the SAME per-stream region (kSyncFlags), and
neither zeroes it before a call.  A stale flag of one path must never be read
as current by the other, across alternating calls on one stream and across
the 16-bit epoch's wrap-around.  Outputs are sentinel-filled
before every call, so a byte the compressor failed to write shows; every
archive must equal the oracle's (the reference writes one archive per element
whatever the path, ans/GpuANSEncode.cuh:670-845)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import float_words

pytestmark = pytest.mark.gpu

DEV = "cuda"
SENTINEL = 0xAB


@pytest.fixture(scope="module")
def env():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import _native as N
    from dietgpu_fork_amd import codec as C

    return N, C


@pytest.fixture(autouse=True)
def _single_pass(env):
    """The aligned batches here are meant for the single-pass compressor
    (small batches take the three-kernel path by default: the size rule,
    codec.hip persistentPreferred)."""
    with env[1].compress_path("single-pass"):
        yield


class Batch:
    """bf16 elements in one device buffer; `aligned` False offsets every
    element by one word (not 16 B-aligned: the fused three-kernel path)."""

    def __init__(self, N, sizes, seed, aligned):
        self.N = N
        self.words = [float_words(2, n, seed=seed + i) for i, n in enumerate(sizes)]
        stride = max(sizes) + 64
        host = np.zeros(len(sizes) * stride, dtype=np.uint16)
        self.offs = [i * stride + (0 if aligned else 1) for i in range(len(sizes))]
        for o, w in zip(self.offs, self.words):
            host[o:o + w.size] = w
        self.x = torch.from_numpy(host.view(np.int16)).to(DEV)
        self.cols = N.lib().dietgpu_get_max_float_compressed_size(2, max(sizes))
        self.out = torch.empty([len(sizes), self.cols], dtype=torch.uint8, device=DEV)
        self.sizes = torch.empty([len(sizes)], dtype=torch.int32, device=DEV)
        self.in_ptrs = N.ptr_array([self.x.data_ptr() + 2 * o for o in self.offs])
        self.in_size = N.u32_array(sizes)
        self.out_ptrs = N.ptr_array([self.out.data_ptr() + i * self.cols for i in range(len(sizes))])

    def compress(self, ws, stream, fill=True):
        if fill:
            self.out.fill_(SENTINEL)
        self.N.check(self.N.lib().dietgpu_float_compress(ws.h, 2, 10, 0, len(self.words), self.in_ptrs,
                                                         self.in_size, self.out_ptrs, self.sizes.data_ptr(),
                                                         stream.cuda_stream))

    def check(self):
        sizes = self.sizes.cpu().tolist()
        host = self.out.cpu().numpy()
        for i, w in enumerate(self.words):
            ref = O.float_compress(w, 2)
            assert sizes[i] == ref.size, (i, sizes[i], ref.size)
            np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")


def test_alternating_paths_one_stream(env):
    """Single-pass and fused three-kernel calls back to back on one stream,
    the same shapes (so the flag words of one land on the other's)."""
    N, C = env
    ws = C.Workspace(256 << 20)
    s = torch.cuda.Stream()
    sizes = [300000, 524288, 70001, 4097, 200000]
    a = Batch(N, sizes, seed=11, aligned=True)
    u = Batch(N, sizes, seed=11, aligned=False)
    C.device_error_count(reset=True)
    with torch.cuda.stream(s):
        for k in range(8):
            b = a if k % 2 == 0 else u
            b.compress(ws, s)
            s.synchronize()
            b.check()
    assert C.device_error_count(reset=True) == 0


def test_epoch_wraparound(env):
    """More than 2^16 calls on a fresh stream (the arena's 16-bit epoch
    wraps and the arena is re-zeroed), alternating the two paths; archives
    checked before, around and after the wrap."""
    N, C = env
    ws = C.Workspace(64 << 20)
    s = torch.cuda.Stream()
    sizes = [70000, 40000]  # 3 and 2 single-pass items: look-back and partials
    a = Batch(N, sizes, seed=21, aligned=True)
    u = Batch(N, sizes, seed=21, aligned=False)
    C.device_error_count(reset=True)
    C.barrier_fallback_count(reset=True)
    total = (1 << 16) + 40
    checkpoints = {0, 1, 2, 3, 1000, (1 << 16) - 3, (1 << 16) - 2, (1 << 16) - 1, 1 << 16, (1 << 16) + 1,
                   (1 << 16) + 2, total - 2, total - 1}
    with torch.cuda.stream(s):
        for k in range(total):
            b = a if k % 2 == 0 else u
            if k in checkpoints:
                b.compress(ws, s)
                s.synchronize()
                b.check()
            else:
                b.compress(ws, s, fill=False)
    s.synchronize()
    assert C.device_error_count(reset=True) == 0
    assert C.barrier_fallback_count(reset=True) == 0


def test_prenormalised_sparse_after_single_pass(env):
    """The sparse compressor's dense list goes through the three-kernel
    encoder with a caller-normalised table (preNorm: no k_normalize, the
    encoder's fused look-back flags in the same kSyncFlags region): run it
    straight after single-pass calls (sentinel-filled outputs) on the same
    stream, alternating, and compare both with the oracle's archives."""
    N, C = env
    ws = C.Workspace(256 << 20)
    s = torch.cuda.Stream()
    a = Batch(N, [300000, 524288, 70001], seed=31, aligned=True)
    from tests.util import sparsify

    n = 3_000_000  # 30 % nonzeros: a list of > 2^20 words (three-kernel, preNorm)
    w = sparsify(float_words(3, n, seed=33), frac_zero=0.7, seed=34)
    ref = O.sparse_compress(w, 3)
    x = torch.from_numpy(w.view(np.int32)).to(DEV).view(torch.float32)
    C.device_error_count(reset=True)
    with torch.cuda.stream(s):
        for k in range(4):
            a.compress(ws, s)
            out, sizes = C.sparse_compress([x], ws=ws)
            s.synchronize()
            a.check()
            assert int(sizes[0]) == ref.size
            np.testing.assert_array_equal(out[0, : ref.size].cpu().numpy(), ref, err_msg=f"round {k}")
    assert C.device_error_count(reset=True) == 0


def test_three_kernel_rows_back_to_back(env):
    """Consecutive three-kernel calls on one stream whose prologue-
    normalisation rows change shape call to call: the rows of a
    call are [segments][nb][min(chunks, 64)] in one of the arena's two
    buffers, and each call's k_hist zeroes the other buffer for the next
    call, so every layout below reads rows the previous (different) layout
    zeroed.  Chunk counts 1, 2, 3, 5 and > 64, one and two segments (fp64),
    batch sizes 1 to 200; every archive (sentinel-filled output) must equal
    the oracle's."""
    N, C = env
    ws = C.Workspace(256 << 20)
    s = torch.cuda.Stream()
    cases = [(2, 1, 1_000_000), (3, 3, 12_000), (4, 200, 3_000), (2, 1, 8_192), (1, 16, 20_000),
             (4, 2, 300_000), (2, 1, 1_000_000), (3, 3, 12_000), (4, 200, 3_000), (1, 64, 4_096)]
    tdt = {1: torch.int16, 2: torch.int16, 3: torch.int32, 4: torch.int64}
    ndt = {1: np.int16, 2: np.int16, 3: np.int32, 4: np.int64}
    C.device_error_count(reset=True)
    with C.compress_path("three-kernel"), torch.cuda.stream(s):
        for k, (ft, nb, n) in enumerate(cases):
            words = [float_words(ft, n, seed=1000 * k + i) for i in range(nb)]
            x = torch.from_numpy(np.stack(words).view(ndt[ft])).to(DEV)
            cols = C.max_float_compressed_size(ft, n)
            out = torch.full([nb, cols], SENTINEL, dtype=torch.uint8, device=DEV)
            sizes = torch.empty([nb], dtype=torch.int32, device=DEV)
            C.float_compress_stride(x.view(tdt[ft]), ft=ft, ws=ws, out=out, sizes=sizes)
            s.synchronize()
            host, sz = out.cpu().numpy(), sizes.cpu().tolist()
            for i, w in enumerate(words):
                ref = O.float_compress(w, ft)
                assert sz[i] == ref.size, (k, i, sz[i], ref.size)
                np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"call {k} element {i}")
    assert C.device_error_count(reset=True) == 0


def test_sparse_rows_interleaved_with_three_kernel(env):
    """The single-element sparse compressor counts its list's histogram into
    the same arena row buffers (k_sparseCount, no zeroing launch) and zeroes
    the other buffer for the next call; it takes one epoch, the dense codec
    after it another, so the row buffers no longer follow epoch parity.
    Interleave sparse calls of different sizes (1 to 64 rows per element,
    fp32 and fp64: one and two segments) with three-kernel dense calls on
    one stream; every archive (sentinel-filled) must equal the oracle's."""
    N, C = env
    from tests.util import sparsify

    ws = C.Workspace(256 << 20)
    s = torch.cuda.Stream()
    tdt = {1: torch.int16, 2: torch.int16, 3: torch.int32, 4: torch.int64}
    ndt = {1: np.int16, 2: np.int16, 3: np.int32, 4: np.int64}
    fdt = {3: torch.float32, 4: torch.float64}
    steps = [("sparse", 3, 1, 3_000_000, 0.9), ("dense", 2, 3, 12_000, 0), ("sparse", 3, 1, 5_000, 0.5),
             ("sparse", 4, 1, 700_000, 0.8), ("dense", 4, 2, 300_000, 0), ("sparse", 3, 1, 300_000, 0.5),
             ("sparse", 3, 1, 3_000_000, 0.9), ("dense", 3, 5, 40_000, 0), ("sparse", 4, 1, 9_000, 0.3)]
    C.device_error_count(reset=True)
    with C.compress_path("three-kernel"), torch.cuda.stream(s):
        for k, (kind, ft, nb, n, frac) in enumerate(steps):
            if kind == "sparse":
                w = sparsify(float_words(ft, n, seed=500 + k), frac_zero=frac, seed=600 + k)
                ref = O.sparse_compress(w, ft)
                x = torch.from_numpy(w.view(ndt[ft])).to(DEV).view(fdt[ft])
                out, sizes = C.sparse_compress([x], ws=ws)
                s.synchronize()
                assert int(sizes[0]) == ref.size, (k, int(sizes[0]), ref.size)
                np.testing.assert_array_equal(out[0, : ref.size].cpu().numpy(), ref, err_msg=f"step {k}")
            else:
                words = [float_words(ft, n, seed=700 * k + i) for i in range(nb)]
                x = torch.from_numpy(np.stack(words).view(ndt[ft])).to(DEV)
                out = torch.full([nb, C.max_float_compressed_size(ft, n)], SENTINEL, dtype=torch.uint8, device=DEV)
                sizes = torch.empty([nb], dtype=torch.int32, device=DEV)
                C.float_compress_stride(x.view(tdt[ft]), ft=ft, ws=ws, out=out, sizes=sizes)
                s.synchronize()
                host, sz = out.cpu().numpy(), sizes.cpu().tolist()
                for i, ww in enumerate(words):
                    ref = O.float_compress(ww, ft)
                    assert sz[i] == ref.size, (k, i, sz[i], ref.size)
                    np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"step {k} element {i}")
    assert C.device_error_count(reset=True) == 0
