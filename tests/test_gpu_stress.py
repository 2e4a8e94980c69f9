"""GPU parity under the conditions the reference's own tests vary
(ans/test/ans_test.py, float/test/float_test.py): many small random sizes in
one batch, a non-default stream, many consecutive calls of changing shape
(the compressor's persistent sync arena and its epochs, csrc/sync_arena.cpp),
and batches too large for the inline kernel-argument tables (> 400
elements: device-resident tables).  Every archive is checked byte for byte
against the oracle and decoded back."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import exp_bytes

pytestmark = pytest.mark.gpu

DEV = "cuda"


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
    return C.Workspace(256 << 20)


def _bf16_words(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, generator=g) * (1 + seed % 5)).to(torch.bfloat16)


def _float_roundtrip(C, ws, xs, checksum=False):
    """xs: CPU bf16 tensors.  Compress on the GPU, compare with the oracle,
    decompress and compare with the input."""
    xd = [x.to(DEV) for x in xs]
    arch, sizes = C.float_compress_pointer(xd, prob_bits=10, checksum=checksum, ws=ws)
    sizes = sizes.cpu().tolist()
    host = arch.cpu().numpy()
    for i, x in enumerate(xs):
        ref = O.float_compress(x.view(torch.int16).numpy().view(np.uint16), 2, 10, checksum)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    rows = [arch[i, : sizes[i]] for i in range(len(xs))]
    outs = [torch.empty(x.numel(), dtype=torch.bfloat16, device=DEV) for x in xs]
    ok, _ = C.float_decompress_pointer(rows, outs, prob_bits=10, checksum=checksum, ws=ws)
    assert ok.cpu().tolist() == [1] * len(xs)
    for x, o in zip(xs, outs):
        assert torch.equal(o.cpu().view(torch.int16), x.view(torch.int16))
    return host, sizes


@pytest.mark.parametrize("checksum", [False, True])
def test_ans_100_random_sizes(C, ws, checksum):
    """ans_test.py's batch: 100 elements of random size in [100, 10000]."""
    rng = np.random.default_rng(100 + int(checksum))
    datas = [exp_bytes(int(n), lam=float(rng.uniform(1, 100)), seed=i)
             for i, n in enumerate(rng.integers(100, 10001, size=100))]
    ts = [torch.from_numpy(d).to(DEV) for d in datas]
    out, sizes = C.ans_encode_pointer(ts, prob_bits=10, checksum=checksum, ws=ws)
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i, d in enumerate(datas):
        ref = O.ans_encode(d, 10, checksum)
        assert sizes[i] == ref.size
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    outs = [torch.empty(d.size, dtype=torch.uint8, device=DEV) for d in datas]
    ok, _ = C.ans_decode_pointer([out[i, : sizes[i]] for i in range(100)], outs,
                                 prob_bits=10, checksum=checksum, ws=ws)
    assert ok.cpu().tolist() == [1] * 100
    for d, o in zip(datas, outs):
        np.testing.assert_array_equal(o.cpu().numpy(), d)


def test_float_non_default_stream(C, ws):
    xs = [_bf16_words(50000 + 777 * i, seed=i) for i in range(6)]
    ref_host, ref_sizes = _float_roundtrip(C, ws, xs)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        host, sizes = _float_roundtrip(C, ws, xs)
    torch.cuda.synchronize()
    assert sizes == ref_sizes
    for i, n in enumerate(sizes):
        np.testing.assert_array_equal(host[i, :n], ref_host[i, :n])


def test_float_many_calls_changing_shapes(C, ws):
    """40 consecutive calls: the batch and element sizes change every call, so
    the sync arena is reused across epochs and grows in between."""
    rng = np.random.default_rng(7)
    for it in range(40):
        nb = int(rng.integers(1, 24))
        xs = [_bf16_words(int(rng.integers(1, 200000)), seed=1000 * it + j) for j in range(nb)]
        _float_roundtrip(C, ws, xs, checksum=bool(it & 1))


@pytest.mark.parametrize("nb", [401, 700])
def test_float_batch_beyond_inline_tables(C, ws, nb):
    """More elements than the 8 KB inline kernel-argument table holds."""
    rng = np.random.default_rng(nb)
    xs = [_bf16_words(int(rng.integers(1, 6000)), seed=j) for j in range(nb)]
    _float_roundtrip(C, ws, xs)


@pytest.mark.parametrize("middle", ["fp64", "unaligned"])
def test_single_pass_after_three_kernel_call(C, ws, middle):
    """Single-pass call of >= 3 rounds (elements past the static rounds come
    from a dequeue counter), then a three-kernel call on the same stream (it
    takes an epoch but never runs k_pcompress), then the single-pass call
    again: the second single-pass call's counter must start at zero, or the
    elements it would dequeue first are silently never encoded."""
    nb, n = 3000, 4096  # one item per element: 1,024-member grid, 3 rounds
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(nb, n, generator=g) * 3).to(torch.bfloat16)
    xd = x.to(DEV).view(torch.int16)
    words = x.view(torch.int16).numpy().view(np.uint16)
    refs = [O.float_compress(words[i], 2) for i in range(nb)]

    cols = C.max_float_compressed_size(2, n)

    def single_pass():
        # fresh sentinels: a dropped element must not find the last call's archive
        out = torch.full([nb, cols], 0xAA, dtype=torch.uint8, device=DEV)
        sizes = torch.full([nb], -1, dtype=torch.int32, device=DEV)
        out, sizes = C.float_compress_stride(xd, ft=2, ws=ws, out=out, sizes=sizes)
        sizes = sizes.cpu().tolist()
        host = out.cpu().numpy()
        for i in range(nb):
            assert sizes[i] == refs[i].size, (i, sizes[i], refs[i].size)
            np.testing.assert_array_equal(host[i, : refs[i].size], refs[i], err_msg=f"element {i}")

    single_pass()
    if middle == "fp64":
        w64 = np.random.default_rng(3).standard_normal(70000).view(np.uint64)
        t64 = torch.from_numpy(w64.view(np.int64).copy()).to(DEV)
        out, sizes = C.float_compress_pointer([t64], ft=4, ws=ws)
        ref = O.float_compress(w64, 4)
        np.testing.assert_array_equal(out[0, : int(sizes[0])].cpu().numpy(), ref)
    else:
        big = xd.reshape(-1)
        out, sizes = C.float_compress_pointer([big[1:50001]], ft=2, ws=ws)
        ref = O.float_compress(words.reshape(-1)[1:50001], 2)
        np.testing.assert_array_equal(out[0, : int(sizes[0])].cpu().numpy(), ref)
    single_pass()
    assert C.device_error_count(reset=True) == 0
