"""GPU parity: HIP archives must be byte-identical to the oracle's and every
roundtrip bit-exact.  Calls the C ABI (through dietgpu_fork_amd.codec)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import NP_WORD, exp_bytes, float_words, sparsify

pytestmark = pytest.mark.gpu

DEV = "cuda"
TORCH_WORD = {1: torch.int16, 2: torch.int16, 3: torch.int32, 4: torch.int64}
NP_SIGNED = {1: np.int16, 2: np.int16, 3: np.int32, 4: np.int64}


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(512 << 20)


def to_dev_words(w, ft):
    return torch.from_numpy(w.view(NP_SIGNED[ft]).copy()).to(DEV)


def to_np_words(t, ft):
    return t.cpu().numpy().view(NP_WORD[ft])


ANS_SIZES = [0, 1, 31, 32, 33, 4095, 4096, 4097, 12345, 65536, 100003]


@pytest.mark.parametrize("pb", [9, 10, 11])
@pytest.mark.parametrize("checksum", [False, True])
def test_ans_pointer_parity(C, ws, pb, checksum):
    datas = [exp_bytes(n, lam=[1, 10, 100, 1000][i % 4], seed=i) for i, n in enumerate(ANS_SIZES)]
    ts = [torch.from_numpy(d).to(DEV) for d in datas]
    out, sizes = C.ans_encode_pointer(ts, prob_bits=pb, checksum=checksum, ws=ws)
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i, d in enumerate(datas):
        ref = O.ans_encode(d, pb, checksum)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        assert sizes[i] % 16 == 0
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    # decode from exactly-sized copies (size reported must be exact)
    arch = [out[i, : sizes[i]].clone() for i in range(len(ts))]
    outs = [torch.empty(max(d.size, 0), dtype=torch.uint8, device=DEV) for d in datas]
    ok, sz = C.ans_decode_pointer(arch, outs, prob_bits=pb, checksum=checksum, ws=ws)
    assert ok.cpu().tolist() == [1] * len(ts)
    assert sz.cpu().tolist() == [d.size for d in datas]
    for d, o in zip(datas, outs):
        np.testing.assert_array_equal(o.cpu().numpy(), d)


def test_ans_stride_roundtrip_and_capacity(C, ws):
    nb, n = 13, 8208  # ANSTest.cu:277-282
    data = np.stack([exp_bytes(n, lam=20.0, seed=100 + i) for i in range(nb)])
    t = torch.from_numpy(data).to(DEV)
    out, sizes = C.ans_encode_stride(t, ws=ws)
    sizes_h = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i in range(nb):
        ref = O.ans_encode(data[i])
        np.testing.assert_array_equal(host[i, : sizes_h[i]], ref)
    dec, ok, sz = C.ans_decode_stride(out, n, ws=ws)
    assert ok.cpu().tolist() == [1] * nb
    np.testing.assert_array_equal(dec.cpu().numpy(), data)
    # insufficient capacity -> success false, required size reported
    _, ok, sz = C.ans_decode_stride(out, n, ws=ws, capacity=n - 1)
    assert ok.cpu().tolist() == [0] * nb
    assert sz.cpu().tolist() == [n] * nb


def test_ans_user_histogram(C, ws):
    d = exp_bytes(50000, lam=10.0, seed=7)
    t = torch.from_numpy(d).to(DEV).view(1, -1)
    h = torch.from_numpy(O.histogram(d).astype(np.int32)).to(DEV)
    out, sizes = C.ans_encode_stride(t, ws=ws, histogram=h)
    ref = O.ans_encode(d)
    np.testing.assert_array_equal(out[0, : int(sizes[0])].cpu().numpy(), ref)


@pytest.mark.parametrize("user_hist", [False, True])
def test_ans_large_single_checksum(C, ws, user_hist):
    """One 6 MB element: ~1500 histogram chunks, so the partial histograms and
    byte-checksum partials go through the two-level reduction (k_histReduce)."""
    d = exp_bytes(6_000_000, lam=10.0, seed=9)
    t = torch.from_numpy(d).to(DEV).view(1, -1)
    h = torch.from_numpy(O.histogram(d).astype(np.int32)).to(DEV) if user_hist else None
    out, sizes = C.ans_encode_stride(t, ws=ws, histogram=h, checksum=True)
    ref = O.ans_encode(d, 10, True)
    np.testing.assert_array_equal(out[0, : int(sizes[0])].cpu().numpy(), ref)
    dec, ok, _ = C.ans_decode_stride(out, d.size, ws=ws, checksum=True)
    assert int(ok[0]) == 1 and np.array_equal(dec[0].cpu().numpy(), d)


def test_ans_uniform_16_symbols(C, ws):
    # c3 shape (4.0 bit / symbol), reduced batch
    rng = np.random.default_rng(3)
    data = rng.integers(0, 16, size=(4, 1 << 20), dtype=np.uint8)
    t = torch.from_numpy(data).to(DEV)
    out, sizes = C.ans_encode_stride(t, ws=ws)
    host = out.cpu().numpy()
    sizes_h = sizes.cpu().tolist()
    for i in range(4):
        ref = O.ans_encode(data[i])
        np.testing.assert_array_equal(host[i, : sizes_h[i]], ref)
    dec, ok, _ = C.ans_decode_stride(out, 1 << 20, ws=ws)
    np.testing.assert_array_equal(dec.cpu().numpy(), data)


FLOAT_SIZES = [0, 1, 2, 13, 4095, 4096, 4097, 12345, 65536, 100001]


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
@pytest.mark.parametrize("pb", [9, 10, 11])
def test_float_pointer_parity(C, ws, ft, pb):
    words = [float_words(ft, n, seed=10 + i) for i, n in enumerate(FLOAT_SIZES)]
    ts = [to_dev_words(w, ft) for w in words]
    out, sizes = C.float_compress_pointer(ts, ft=ft, prob_bits=pb, ws=ws)
    sizes_h = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i, w in enumerate(words):
        ref = O.float_compress(w, ft, pb)
        assert sizes_h[i] == ref.size, (i, sizes_h[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    arch = [out[i, : sizes_h[i]].clone() for i in range(len(ts))]
    outs = [torch.empty(w.size, dtype=TORCH_WORD[ft], device=DEV) for w in words]
    ok, sz = C.float_decompress_pointer(arch, outs, ft=ft, prob_bits=pb, ws=ws)
    assert ok.cpu().tolist() == [1] * len(ts)
    assert sz.cpu().tolist() == [w.size for w in words]
    for w, o in zip(words, outs):
        np.testing.assert_array_equal(to_np_words(o, ft), w)


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
def test_float_checksum(C, ws, ft):
    words = [float_words(ft, n, seed=20 + i) for i, n in enumerate([1, 5000, 70000])]
    ts = [to_dev_words(w, ft) for w in words]
    out, sizes = C.float_compress_pointer(ts, ft=ft, checksum=True, ws=ws)
    host = out.cpu().numpy()
    for i, w in enumerate(words):
        ref = O.float_compress(w, ft, 10, True)
        np.testing.assert_array_equal(host[i, : int(sizes[i])], ref)
    arch = [out[i, : int(sizes[i])].clone() for i in range(len(ts))]
    outs = [torch.empty(w.size, dtype=TORCH_WORD[ft], device=DEV) for w in words]
    C.float_decompress_pointer(arch, outs, ft=ft, checksum=True, ws=ws)
    # corrupt one raw byte -> checksum mismatch is reported
    bad = [a.clone() for a in arch]
    bad[2][40] ^= 0xFF
    from dietgpu_fork_amd import ChecksumMismatch

    with pytest.raises(ChecksumMismatch):
        C.float_decompress_pointer(bad, outs, ft=ft, checksum=True, ws=ws)


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
def test_float_unaligned_pointers(C, ws, ft):
    # inputs / outputs that are only word aligned (split-size style offsets)
    n = 9999
    w = float_words(ft, n + 3, seed=33)
    big = to_dev_words(w, ft)
    ts = [big[1:n + 1], big[3:]]
    out, sizes = C.float_compress_pointer(ts, ft=ft, ws=ws)
    host = out.cpu().numpy()
    np.testing.assert_array_equal(host[0, : int(sizes[0])], O.float_compress(w[1:n + 1], ft))
    np.testing.assert_array_equal(host[1, : int(sizes[1])], O.float_compress(w[3:], ft))
    dst = torch.empty(2 * n + 8, dtype=TORCH_WORD[ft], device=DEV)
    outs = [dst[1:n + 1], dst[n + 3: 2 * n + 3]]
    arch = [out[0, : int(sizes[0])], out[1, : int(sizes[1])]]
    C.float_decompress_pointer(arch, outs, ft=ft, ws=ws)
    np.testing.assert_array_equal(to_np_words(outs[0], ft), w[1:n + 1])
    np.testing.assert_array_equal(to_np_words(outs[1], ft), w[3:])


@pytest.mark.parametrize("ft", [2, 3])
def test_float_stride_batch(C, ws, ft):
    nb, n = 23, 30000
    w = np.stack([float_words(ft, n, seed=200 + i) for i in range(nb)])
    t = torch.from_numpy(w.view(NP_SIGNED[ft])).to(DEV)
    out, sizes = C.float_compress_stride(t, ft=ft, ws=ws)
    host = out.cpu().numpy()
    for i in range(nb):
        np.testing.assert_array_equal(host[i, : int(sizes[i])], O.float_compress(w[i], ft))
    dec, ok, _ = C.float_decompress_stride(out, n, TORCH_WORD[ft], ws=ws)
    np.testing.assert_array_equal(dec.cpu().numpy().view(NP_WORD[ft]), w)


SPARSE_SIZES = [0, 1, 2, 3, 17, 4096, 4097, 50001]


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
def test_sparse_parity(C, ws, ft):
    words = []
    for i, n in enumerate(SPARSE_SIZES):
        w = sparsify(float_words(ft, n, seed=40 + i), 0.9, seed=50 + i)
        words.append(w)
    # force both n-2 quirk branches
    words[4][-2] = 0
    words[5][-2] = 7
    words[6][-2] = 0
    words[6][-1] = 0
    ts = [to_dev_words(w, ft) for w in words]
    out, sizes = C.sparse_compress(ts, ft=ft, ws=ws)
    host = out.cpu().numpy()
    sizes_h = sizes.cpu().tolist()
    for i, w in enumerate(words):
        ref = O.sparse_compress(w, ft)
        assert sizes_h[i] == ref.size, (i, sizes_h[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    arch = [out[i, : sizes_h[i]].clone() for i in range(len(ts))]
    outs = [torch.empty(w.size, dtype=TORCH_WORD[ft], device=DEV) for w in words]
    ok, sz = C.sparse_decompress(arch, outs, ft=ft, ws=ws)
    assert ok.cpu().tolist() == [1] * len(ts)
    assert sz.cpu().tolist() == [w.size for w in words]
    for w, o in zip(words, outs):
        np.testing.assert_array_equal(to_np_words(o, ft), w)


def test_sparse_all_zero_and_dense(C, ws):
    ft = 3
    ws_ = [np.zeros(1000, np.uint32), float_words(3, 3000, seed=9), np.zeros(2, np.uint32)]
    ts = [to_dev_words(w, ft) for w in ws_]
    out, sizes = C.sparse_compress(ts, ft=ft, ws=ws)
    host = out.cpu().numpy()
    for i, w in enumerate(ws_):
        np.testing.assert_array_equal(host[i, : int(sizes[i])], O.sparse_compress(w, ft))
    arch = [out[i, : int(sizes[i])].clone() for i in range(3)]
    outs = [torch.empty(w.size, dtype=torch.int32, device=DEV) for w in ws_]
    C.sparse_decompress(arch, outs, ft=ft, ws=ws)
    for w, o in zip(ws_, outs):
        np.testing.assert_array_equal(to_np_words(o, ft), w)


@pytest.mark.parametrize("ft", [2, 3])
def test_sparse_large_lists(C, ws, ft):
    """Nonzero lists from empty to fully dense in one batch of 3 M-word
    elements (the dense codec's multi-chunk histogram path over lists whose
    lengths only the device knows)."""
    n = 3 << 20
    fracs = [0.9, 0.0, 0.5, 1.0, 0.999]
    words = [sparsify(float_words(ft, n, seed=70 + i), f, seed=80 + i) for i, f in enumerate(fracs)]
    ts = [to_dev_words(w, ft) for w in words]
    out, sizes = C.sparse_compress(ts, ft=ft, ws=ws)
    host = out.cpu().numpy()
    sizes_h = sizes.cpu().tolist()
    assert C.device_error_count(reset=True) == 0
    for i, w in enumerate(words):
        ref = O.sparse_compress(w, ft)
        assert sizes_h[i] == ref.size, (i, sizes_h[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    arch = [out[i, : sizes_h[i]].clone() for i in range(len(ts))]
    del out
    outs = [torch.empty(n, dtype=TORCH_WORD[ft], device=DEV) for _ in words]
    ok, sz = C.sparse_decompress(arch, outs, ft=ft, ws=ws)
    assert ok.cpu().tolist() == [1] * len(ts)
    for w, o in zip(words, outs):
        np.testing.assert_array_equal(to_np_words(o, ft), w)


def test_sparse_many_tiles(C, ws):
    """One element of more than 4,096 tiles of 4,096 words: the per-tile
    prefix of the earlier tiles' counts (k_sparseGather / k_sparseExpand,
    16 loads in flight per thread) then takes more than one round of loads;
    a ragged last tile and a second, one-tile element in the same batch."""
    ft = 2
    sizes = [4100 * 4096 + 123, 777]
    words = [sparsify(float_words(ft, n, seed=90 + i), 0.9, seed=95 + i) for i, n in enumerate(sizes)]
    ts = [to_dev_words(w, ft) for w in words]
    out, osz = C.sparse_compress(ts, ft=ft, ws=ws)
    host = out.cpu().numpy()
    osz_h = osz.cpu().tolist()
    for i, w in enumerate(words):
        ref = O.sparse_compress(w, ft)
        assert osz_h[i] == ref.size, (i, osz_h[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    arch = [out[i, : osz_h[i]].clone() for i in range(len(ts))]
    del out
    outs = [torch.empty(n, dtype=TORCH_WORD[ft], device=DEV) for n in sizes]
    ok, sz = C.sparse_decompress(arch, outs, ft=ft, ws=ws)
    assert ok.cpu().tolist() == [1, 1]
    assert sz.cpu().tolist() == sizes
    for w, o in zip(words, outs):
        np.testing.assert_array_equal(to_np_words(o, ft), w)
