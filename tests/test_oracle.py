"""CPU tests of the oracle (oracle/dietgpu_oracle.c, test infrastructure
only) against the reference's known-answer tests, the committed golden
fixtures and the independent pure-Python restatement (tests/pyref.py).

Reference tests mirrored (paths relative to /root/reference/dietgpu):
  ans/test/ANSStatisticsTest.cu:127-207   normalisation KATs and bounds
  ans/test/ANSTest.cu:131-135,243-282     16 B archive sizes, roundtrip grid
  ans_test.py:21-26                       exact size reporting
  float/test/FloatTest.cu:287-340         float roundtrip grid
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import pyref
from tests.util import NP_WORD, exp_bytes, float_words, sparsify

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")


@pytest.fixture(scope="module")
def G():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# --- normalisation (ANSStatisticsTest.cu) -----------------------------------

def test_kat_one_dominant_symbol():
    # :127-149: 0..255 once + 9744 x 1 at pb 10 -> pdf[1] = 769, others 1
    d = np.concatenate([np.arange(256, dtype=np.uint8), np.ones(9744, dtype=np.uint8)])
    pdf, cdf = O.normalize(O.histogram(d), d.size, 10)
    assert pdf[1] == 769
    assert all(pdf[i] == 1 for i in range(256) if i != 1)
    assert cdf[0] == 0 and cdf[255] == 1024 - pdf[255]


def test_kat_uniform():
    # :151-167: 64 x (0..255) -> every pdf 4
    d = np.tile(np.arange(256, dtype=np.uint8), 64)
    pdf, _ = O.normalize(O.histogram(d), d.size, 10)
    assert (pdf == 4).all()


def test_kat_diff_positive_bumps_symbol_ids():
    # SURVEY Appendix B.2, GpuANSStatistics.cuh:266-267: counts 3 at symbols
    # 200..202 scale to 341 each (1023 < 1024); the diff>0 branch then adds
    # the missing 1 to symbol id 0, which is absent from the input
    h = np.zeros(256, dtype=np.uint32)
    h[200:203] = 3
    pdf, cdf = O.normalize(h, 9, 10)
    assert pdf[200] == pdf[201] == pdf[202] == 341
    assert pdf[0] == 1
    assert int(pdf.sum()) == 1024 and int(np.count_nonzero(pdf)) == 4
    assert cdf[200] == 1 and cdf[202] == 1 + 2 * 341
    assert pdf.tolist() == pyref.normalize(h.tolist(), 9, 10)
    d = np.repeat(np.arange(200, 203, dtype=np.uint8), 3)
    st, dec = O.ans_decode(O.ans_encode(d, 10), 10)
    assert st == 0 and np.array_equal(dec, d)


@pytest.mark.parametrize("pb", [9, 10, 11])
@pytest.mark.parametrize("seed", range(8))
def test_normalize_bounds(pb, seed):
    # :169-207: random histograms: sum == 2^pb, present symbols >= 1, absent 0
    rng = np.random.default_rng(seed)
    nsym = int(rng.integers(1, 257))
    h = np.zeros(256, dtype=np.uint32)
    syms = rng.choice(256, nsym, replace=False)
    # skewed counts; the total stays a u32 element size as in the reference
    h[syms] = rng.integers(1, 1000, nsym) ** rng.integers(1, 3, nsym)
    total = int(h.sum())
    assert total < 1 << 32
    pdf, cdf = O.normalize(h, total, pb)
    assert int(pdf.sum()) == 1 << pb
    assert ((pdf >= 1) == (h > 0)).all()
    assert np.array_equal(cdf, np.concatenate([[0], np.cumsum(pdf)[:-1]]))
    assert pdf.tolist() == pyref.normalize(h.tolist(), total, pb)


def test_golden_kat_tables(G):
    for name, d in (("kat_a", np.concatenate([np.arange(256, dtype=np.uint8), np.ones(9744, dtype=np.uint8)])),
                    ("kat_b", np.tile(np.arange(256, dtype=np.uint8), 64))):
        pdf, _ = O.normalize(O.histogram(d), d.size, 10)
        assert np.array_equal(pdf, G[f"{name}_pdf"])


# --- byte rANS ----------------------------------------------------------------

@pytest.mark.parametrize("pb", [9, 10, 11])
@pytest.mark.parametrize("ck", [0, 1])
def test_golden_c1(G, pb, ck):
    arch = O.ans_encode(G["c1_in"], pb, bool(ck))
    assert np.array_equal(arch, G[f"c1_pb{pb}_ck{ck}"])
    st, dec = O.ans_decode(G[f"c1_pb{pb}_ck{ck}"], pb, bool(ck))
    assert st == 0 and np.array_equal(dec, G["c1_in"])


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 4095, 4096, 4097, 12345])
@pytest.mark.parametrize("pb", [9, 11])
def test_ans_oracle_matches_pyref(n, pb):
    d = exp_bytes(n, lam=[1, 10, 100, 1000][n % 4], seed=n)
    a = O.ans_encode(d, pb)
    assert a.size % 16 == 0  # ANSTest.cu:131-135
    assert np.array_equal(a, np.frombuffer(bytes(pyref.ans_encode(d, pb)), dtype=np.uint8))
    st, dec = O.ans_decode(a, pb)
    assert st == 0 and np.array_equal(dec, d)
    assert np.array_equal(np.asarray(pyref.ans_decode(a, pb), dtype=np.uint8), d)


def test_ans_header_fields(G):
    a = G["c1_pb10_ck1"]
    hdr = a[:32].view(np.uint32)
    assert hdr[0] == 0xD00D0001            # magic | version
    assert hdr[1] == 16                    # blocks of 4 KiB
    assert hdr[2] == 65536                 # uncompressed bytes
    assert hdr[4] == 10 | 0x10             # prob bits | checksum flag
    assert hdr[5] == O.checksum(G["c1_in"])
    pdf = a[32:32 + 512].view(np.uint16)
    assert int(pdf.sum()) == 1024


def test_ans_checksum_and_corruption(G):
    a = G["c1_pb10_ck1"].copy()
    a[-40] ^= 0x5A  # flip a payload byte
    st, _ = O.ans_decode(a, 10, True)
    assert st != 0


def test_ans_capacity_failure(G):
    st, _ = O.ans_decode(G["c1_pb10_ck0"], 10, False, capacity=65535)
    assert st != 0


def test_ans_uniform_16_symbols():
    # c3 shape: 4.0 bit/sym -> ratio ~0.5 + overhead
    d = np.random.default_rng(3).integers(0, 16, 1 << 20).astype(np.uint8)
    a = O.ans_encode(d, 10)
    assert 0.50 < a.size / d.size < 0.55
    st, dec = O.ans_decode(a, 10)
    assert st == 0 and np.array_equal(dec, d)


def test_max_compressed_sizes():
    # getMaxCompressedSize (ans/GpuANSEncode.cu:13-25), SURVEY 8(a) a9 / a21
    assert O.max_compressed_size(65536) == 639520
    assert O.max_compressed_size(4194304) == 5800480
    assert O.max_float_compressed_size(2, 524288) == 1737280


# --- float codec --------------------------------------------------------------

@pytest.mark.parametrize("ft", [1, 2, 3, 4])
@pytest.mark.parametrize("n", [1, 13, 4095, 4096, 4097, 12345])
def test_golden_float(G, ft, n):
    w = G[f"f{ft}_n{n}_in"]
    assert w.dtype == NP_WORD[ft]
    arch = O.float_compress(w, ft, 10)
    assert np.array_equal(arch, G[f"f{ft}_n{n}_pb10"])
    st, dec = O.float_decompress(arch, ft, 10)
    assert st == 0 and np.array_equal(dec, w)


@pytest.mark.parametrize("pb", [9, 11])
def test_golden_float_pb_checksum(G, pb):
    w = G["f2_pbx_in"]
    arch = O.float_compress(w, 2, pb, True)
    assert np.array_equal(arch, G[f"f2_pb{pb}_ck1"])
    hdr = arch[:16].view(np.uint32)
    assert hdr[0] == 0xF00F0001 and hdr[1] == w.size and hdr[2] == 2 | 0x10
    # quirk: the checksum covers the first N *bytes*
    assert hdr[3] == O.checksum(w.view(np.uint8)[: w.size])
    st, dec = O.float_decompress(arch, 2, pb, True)
    assert st == 0 and np.array_equal(dec, w)


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
def test_float_ratio_normal(ft):
    # N(0,1): bf16 ANS byte = exponent (~2.5 bit) -> ratio ~0.67 (SURVEY 8(d)
    # c2); fp16's byte is sign|exponent|2 mantissa bits (~5 bit) -> ~0.81
    w = float_words(ft, 1 << 18, seed=11)
    arch = O.float_compress(w, ft, 10)
    ratio = arch.size / w.nbytes
    assert {1: 0.75 < ratio < 0.9, 2: 0.6 < ratio < 0.75, 3: 0.75 < ratio < 0.9,
            4: 0.8 < ratio < 0.95}[ft], ratio


def test_float_empty():
    for ft in (1, 2, 3, 4):
        w = np.zeros(0, dtype=NP_WORD[ft])
        arch = O.float_compress(w, ft, 10)
        st, dec = O.float_decompress(arch, ft, 10)
        assert st == 0 and dec.size == 0


# --- sparse -------------------------------------------------------------------

@pytest.mark.parametrize("ft", [2, 3])
@pytest.mark.parametrize("tag", ["z", "nz"])
def test_golden_sparse(G, ft, tag):
    w = G[f"s{ft}_{tag}_in"]
    arch = O.sparse_compress(w, ft, 10)
    assert np.array_equal(arch, G[f"s{ft}_{tag}_pb10"])
    st, dec = O.sparse_decompress(arch, ft, 10)
    assert st == 0 and np.array_equal(dec, w)
    # MSB-first bitmap after the 16 B header
    bits = np.unpackbits(arch[16:16 + (w.size + 7) // 8])[: w.size]
    assert np.array_equal(bits.astype(bool), w != 0)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 17])
def test_sparse_tiny(n):
    w = sparsify(float_words(3, n, seed=n), 0.5, seed=n)
    arch = O.sparse_compress(w, 3, 10)
    st, dec = O.sparse_decompress(arch, 3, 10)
    assert st == 0 and np.array_equal(dec, w)
