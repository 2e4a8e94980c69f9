"""The reference's own statistics and size grids, run through the HIP path.

* ANSStatisticsTest.cu:127-149 (Normalization_NonZero: pdf[1] = 2^10 - 255,
  every other symbol 1) and :151-167 (Normalization_EqualWeight: every pdf
  2^10 / 256) encoded by BOTH compressors -- the single-pass k_pcompress
  (16 B-aligned input, forced by dietgpu_set_compress_path: one small element
  takes the three-kernel path by default) and the three-kernel k_hist ->
  k_encode path (16 B-aligned with its prologue normalisation, and a 1-byte-
  offset input, as test_gpu_api.py does) -- with the
  archive's pdf table equal to the golden kat_a_pdf / kat_b_pdf and the whole
  archive equal to the oracle's.
* ANSStatisticsTest.cu:44-95 (Histogram): exact byte histograms of a batch of
  3 elements of 1 .. 12,345,677 bytes with 11 bytes of stride padding, by the
  compressor's own histogram kernel (test hook dietgpu_test_histogram).
* ANSTest.cu:243-260 (ZeroSized, BatchPointer): the size lists {0}, {1},
  {1, 1}, {4096, 4095, 4096}, {1234, 2345, 3456}, {10000, 10013, 10000} x
  probBits 9 / 10 / 11 x lambda 1 / 10 / 100 / 1000, checksum on, on a
  non-blocking stream: archives byte-identical to the oracle, sizes
  multiples of 16, exact roundtrips.

The reference draws its symbols from std::mt19937(10) + exponential_distribution
<float>; the inputs here have the same shape (min(255, 256 * min(Exp(lambda),
1))) from numpy's generator, so parity is anchored on the oracle, not on the
reference's exact bytes."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import exp_bytes

pytestmark = pytest.mark.gpu

DEV = "cuda"
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "golden.npz")


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(256 << 20)


@pytest.fixture(scope="module")
def G():
    return np.load(GOLDEN)


def _kat_input(name):
    if name == "kat_a":  # ANSStatisticsTest.cu:129-137
        return np.concatenate([np.arange(256, dtype=np.uint8), np.ones(10000 - 256, dtype=np.uint8)])
    return np.tile(np.arange(256, dtype=np.uint8), 64)  # :153-159


def _on_device(d, offset):
    """d on the GPU starting `offset` bytes past a 256 B-aligned allocation."""
    big = torch.zeros(d.size + 32, dtype=torch.uint8, device=DEV)
    big[offset: offset + d.size] = torch.from_numpy(d).to(DEV)
    return big[offset: offset + d.size]


@pytest.mark.parametrize("path,offset", [("single-pass", 0), ("three-kernel", 0), ("three-kernel", 1)])
@pytest.mark.parametrize("name", ["kat_a", "kat_b"])
def test_normalization_kat(C, ws, G, name, path, offset):
    d = _kat_input(name)
    t = _on_device(d, offset)
    assert (t.data_ptr() % 16 == 0) == (offset == 0)
    with C.compress_path(path):
        out, sizes = C.ans_encode_pointer([t], prob_bits=10, checksum=False, ws=ws)
    arch = out[0, : int(sizes[0])].cpu().numpy()
    pdf = arch[32: 32 + 512].view(np.uint16).astype(np.uint32)  # after the 32 B ANS header
    np.testing.assert_array_equal(pdf, G[name + "_pdf"])
    if name == "kat_a":
        assert pdf[1] == (1 << 10) - 255 and all(pdf[i] == 1 for i in range(256) if i != 1)
    else:
        assert (pdf == (1 << 10) // 256).all()
    np.testing.assert_array_equal(arch, O.ans_encode(d, 10, False))
    assert C.device_error_count(reset=True) == 0


HIST_SIZES = [1, 2, 11, 32, 55, 1000, 1001, 1000000, 1024 * 1024, 1000001, 12345677]


def test_enc_magic_exhaustive(C):
    """The encode step's division x / pdf (ans/GpuANSEncode.cuh:63-89) is a
    multiply-high by a 32-bit magic computed in registers by every
    normalisation (v_rcp_f64, two Newton steps, exact fix-up): equal to the
    closed form ceil(2^(32 + ceil(log2 q) - 1) / q) for every pdf q <= 2^11."""
    got = C.test_enc_magic().numpy()
    want = [0, 0xFFFFFFFF] + [-(-(1 << (32 + (q - 1).bit_length() - 1)) // q) for q in range(2, (1 << 11) + 1)]
    assert got.tolist() == want


@pytest.mark.parametrize("size", HIST_SIZES)
def test_histogram_batch(C, ws, size):
    nb, pad = 3, 11  # ANSStatisticsTest.cu:61-78
    rows = np.zeros((nb, size + pad), dtype=np.uint8)
    for b in range(nb):
        rows[b, :size] = exp_bytes(size, lam=20.0 + 2 * b, seed=size + b)
    hist = C.test_histogram(torch.from_numpy(rows).to(DEV), size=size, ws=ws).cpu().numpy()
    for b in range(nb):
        np.testing.assert_array_equal(hist[b], np.bincount(rows[b, :size], minlength=256),
                                      err_msg=f"element {b}")


SIZE_LISTS = [[0], [1], [1, 1], [4096, 4095, 4096], [1234, 2345, 3456], [10000, 10013, 10000]]


@pytest.mark.parametrize("lam", [1.0, 10.0, 100.0, 1000.0])
@pytest.mark.parametrize("pb", [9, 10, 11])
def test_batch_pointer_size_grid(C, ws, pb, lam):
    s = torch.cuda.Stream()  # "run on a different stream" (ANSTest.cu:89-90)
    with torch.cuda.stream(s):
        for k, sizes in enumerate(SIZE_LISTS):
            datas = [exp_bytes(n, lam=lam, seed=100 * k + i) for i, n in enumerate(sizes)]
            ts = [torch.from_numpy(d).to(DEV) for d in datas]
            out, osz = C.ans_encode_pointer(ts, prob_bits=pb, checksum=True, ws=ws)
            osz = osz.cpu().tolist()
            host = out.cpu().numpy()
            for i, d in enumerate(datas):
                ref = O.ans_encode(d, pb, True)
                assert osz[i] % 16 == 0 and osz[i] == ref.size, (sizes, i, osz[i], ref.size)
                np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"{sizes} element {i}")
            outs = [torch.empty(d.size, dtype=torch.uint8, device=DEV) for d in datas]
            ok, dsz = C.ans_decode_pointer([out[i, : osz[i]] for i in range(len(ts))], outs,
                                           prob_bits=pb, checksum=True, ws=ws)
            assert ok.cpu().tolist() == [1] * len(ts)
            assert dsz.cpu().tolist() == sizes
            for d, o in zip(datas, outs):
                np.testing.assert_array_equal(o.cpu().numpy(), d)
    torch.cuda.synchronize()
