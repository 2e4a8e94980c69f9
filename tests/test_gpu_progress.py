"""Forward progress of the single-pass compressor (csrc/pcompress.h,
"Forward progress"): the team barrier is the only wait on workgroups that may
not be resident; when it runs past its time budget the workgroup counts the
element from the input itself.  Both paths must write the oracle's archive
byte for byte, and the compressor must finish correctly while another kernel
holds compute units (the reference's use case: compression beside
collectives, README.md:92-96)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import exp_bytes, float_words

pytestmark = pytest.mark.gpu

DEV = "cuda"
MIB = 1 << 20


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


@pytest.fixture(autouse=True)
def _single_pass(C):
    """Small batches take the three-kernel path by default (the size rule,
    codec.hip persistentPreferred): this module's batches are meant for the
    single-pass compressor whenever it can take them."""
    with C.compress_path("single-pass"):
        yield


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(512 << 20)


def _float_inputs(ft, sizes, seed0=0):
    ws_ = [float_words(ft, n, seed=seed0 + i) for i, n in enumerate(sizes)]
    dt = {1: torch.float16, 2: torch.bfloat16, 3: torch.float32}[ft]
    it = {1: torch.int16, 2: torch.int16, 3: torch.int32}[ft]
    ts = [torch.from_numpy(w.view(np.int16 if ft < 3 else np.int32).copy()).to(DEV).view(dt) for w in ws_]
    assert all(t.view(it).numel() == n for t, n in zip(ts, sizes))
    return ws_, ts


def _check_float(C, ws, ft, words, ts, checksum=False):
    out, sizes = C.float_compress_pointer(ts, ft=ft, checksum=checksum, ws=ws)
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i, w in enumerate(words):
        ref = O.float_compress(w, ft, checksum=checksum)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")


@pytest.mark.parametrize("ft", [1, 2, 3])
def test_barrier_fallback_writes_oracle_archives(C, ws, ft):
    """Budget 0: every member of a team of more than one counts its element
    from the input instead of summing the team's partials."""
    C.device_error_count(reset=True)
    try:
        C.set_barrier_budget(0)
        words, ts = _float_inputs(ft, [524288 // (ft // 3 + 1), 300001, 4097, 1, 70000], seed0=ft)
        _check_float(C, ws, ft, words, ts)
        _check_float(C, ws, ft, words, ts, checksum=True)
        datas = [exp_bytes(n, lam=20.0, seed=n) for n in (MIB, 123457, 65536)]
        bts = [torch.from_numpy(d).to(DEV) for d in datas]
        for ck in (False, True):
            out, sizes = C.ans_encode_pointer(bts, checksum=ck, ws=ws)
            sizes = sizes.cpu().tolist()
            host = out.cpu().numpy()
            for i, d in enumerate(datas):
                ref = O.ans_encode(d, 10, ck)
                assert sizes[i] == ref.size
                np.testing.assert_array_equal(host[i, : ref.size], ref)
    finally:
        C.set_barrier_budget(20000)
    assert C.device_error_count(reset=True) == 0


def test_compress_beside_occupying_kernel(C, ws):
    """A c2-shaped batch compressed while a 30 ms kernel on another stream
    holds half the LDS of every compute unit: fewer compressor workgroups fit
    than the grid has, so some teams cannot complete until it ends.  The
    archives must equal the oracle's and no element may be abandoned."""
    from dietgpu_fork_amd import _native as N

    nb = 96
    words = [float_words(2, 524288, seed=100 + i) for i in range(nb)]
    x = torch.from_numpy(np.stack(words).view(np.int16)).to(DEV).view(torch.bfloat16)
    C.device_error_count(reset=True)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    N.test_check(N.testlib().dietgpu_test_occupy(ctypes.c_void_p(side.cuda_stream), 30000, 256, 80 * 1024))
    out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
    torch.cuda.synchronize()
    assert C.device_error_count(reset=True) == 0
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i in range(nb):
        ref = O.float_compress(words[i], 2)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    y, ok, _ = C.float_decompress_stride(out, 524288, torch.bfloat16, ws=ws)
    assert bool((ok == 1).all())
    assert torch.equal(y.view(torch.int16), x.view(torch.int16))


@pytest.mark.parametrize("shape", ["c2", "c3"])
def test_out_of_order_dispatch(C, ws, shape):
    """Workgroups start in about REVERSE index order within every 64 (each
    waits (63 - g % 64) x 1 us first), so the look-backs wait on lower
    workgroups that start up to 63 us late: archives oracle-identical,
    nothing abandoned (no wait runs out of polls).

    What is covered: late PUBLICATION by lower workgroups, which have been
    dispatched (the delay runs after dispatch); a lower workgroup that is
    never dispatched cannot be emulated from software.  c3: k_encode's fused
    look-back, through the product's skew hook (dietgpu_set_dispatch_skew).
    c2: k_pcompress carries no hook, so with the
    product library this leg runs unskewed; tools/skew_check.sh runs it
    against the test-only variant library tools/ablibs/pskew.so
    (tools/variants.py pskew), whose k_pcompress starts skewed the same way
    (team look-back, element-log read, team barrier)."""
    C.device_error_count(reset=True)
    try:
        C.set_dispatch_skew(100)
        if shape == "c2":  # single pass, 2 rounds of dequeued elements
            nb = 320
            words = [float_words(2, 524288, seed=300 + i) for i in range(nb)]
            x = torch.from_numpy(np.stack(words).view(np.int16)).to(DEV).view(torch.bfloat16)
            out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
            refs = [O.float_compress(w, 2) for w in words]
        else:  # 4 MiB byte elements: three kernels, 64 encode workgroups each
            nb = 24
            rng = np.random.default_rng(31)
            data = rng.integers(0, 16, size=(nb, 4 * MIB), dtype=np.uint8)
            out, sizes = C.ans_encode_stride(torch.from_numpy(data).to(DEV), ws=ws)
            refs = [O.ans_encode(data[i]) for i in range(nb)]
        torch.cuda.synchronize()
    finally:
        C.set_dispatch_skew(0)
    assert C.device_error_count(reset=True) == 0
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i, ref in enumerate(refs):
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
