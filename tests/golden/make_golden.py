"""Generate the committed golden fixtures (tests/golden/golden.npz).

Inputs are seeded numpy draws shaped like the reference's own test
generators (SURVEY.md 8(c) golden-vector plan):
  * c1: 64 KiB of b = min(255, floor(256 * min(Exp(100), 1))) bytes
    (ANSTest.cu:18-31, default lambda :88), rng seed 1, archives for
    prob_bits 9/10/11 x checksum off/on;
  * float: fp16 / bf16 / fp32 / fp64 N(0,1) words (bf16 by fp32 truncation,
    FloatTest.cu:21-29) at sizes 1, 13, 4095, 4096, 4097, 12345, pb 10;
    bf16 4097 also at pb 9 and 11, with checksum;
  * sparse: fp32 / bf16 90 %-zero words with x[n-2] == 0 and != 0 (the
    compaction's n-2 quirk), pb 10;
  * normalisation KAT tables of ANSStatisticsTest.cu:127-167.

Every archive is produced by the C oracle (oracle/dietgpu_oracle.c) AND by
the independent pure-Python restatement (tests/pyref.py) where that covers
the case; the script refuses to write fixtures on any disagreement.  The
reference itself is CUDA-only and cannot be built or run here,
so these two restatements plus the reference's known-answer tests are the
pin.  Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
import pyref  # noqa: E402
from util import exp_bytes, float_words  # noqa: E402

FLOAT_SIZES = (1, 13, 4095, 4096, 4097, 12345)


def kat_inputs():
    # ANSStatisticsTest.cu:127-149: 0..255 once + 9744 x 1 (10000 total)
    a = np.concatenate([np.arange(256, dtype=np.uint8), np.ones(9744, dtype=np.uint8)])
    # :151-167: 64 copies of 0..255
    b = np.tile(np.arange(256, dtype=np.uint8), 64)
    return a, b


def main():
    fx = {}
    # c1
    c1 = exp_bytes(65536, lam=100.0, seed=1)
    fx["c1_in"] = c1
    for pb in (9, 10, 11):
        for ck in (0, 1):
            arch = O.ans_encode(c1, pb, bool(ck))
            ref = np.frombuffer(bytes(pyref.ans_encode(c1, pb, bool(ck))), dtype=np.uint8)
            assert np.array_equal(arch, ref), f"oracle/pyref disagree: c1 pb{pb} ck{ck}"
            st, dec = O.ans_decode(arch, pb, bool(ck))
            assert st == 0 and np.array_equal(dec, c1)
            fx[f"c1_pb{pb}_ck{ck}"] = arch
    # float
    for ft in (1, 2, 3, 4):
        for n in FLOAT_SIZES:
            w = float_words(ft, n, seed=100 * ft + n % 97)
            arch = O.float_compress(w, ft, 10, False)
            ref = np.frombuffer(bytes(pyref.float_compress(ft, w, 10)), dtype=np.uint8)
            assert np.array_equal(arch, ref), f"oracle/pyref disagree: ft{ft} n{n}"
            st, dec = O.float_decompress(arch, ft, 10)
            assert st == 0 and np.array_equal(dec, w)
            fx[f"f{ft}_n{n}_in"] = w
            fx[f"f{ft}_n{n}_pb10"] = arch
    w = float_words(2, 4097, seed=7)
    fx["f2_pbx_in"] = w
    for pb in (9, 11):
        arch = O.float_compress(w, 2, pb, True)
        ref = np.frombuffer(bytes(pyref.float_compress(2, w, pb, checksum=True, word_bytes=w.view(np.uint8))), dtype=np.uint8)
        assert np.array_equal(arch, ref), f"oracle/pyref disagree: bf16 pb{pb}"
        fx[f"f2_pb{pb}_ck1"] = arch
    # sparse (oracle only: pyref has no sparse path; decode round trip checked)
    for ft in (2, 3):
        for tag, zero_n2 in (("z", True), ("nz", False)):
            rng = np.random.default_rng(50 + ft)
            w = float_words(ft, 3000, seed=60 + ft)
            w[rng.random(w.size) < 0.9] = 0
            w[-2] = 0 if zero_n2 else (w[-2] | 1)
            arch = O.sparse_compress(w, ft, 10, False)
            st, dec = O.sparse_decompress(arch, ft, 10)
            assert st == 0 and np.array_equal(dec, w)
            fx[f"s{ft}_{tag}_in"] = w
            fx[f"s{ft}_{tag}_pb10"] = arch
    # normalisation KATs
    a, b = kat_inputs()
    for name, d in (("kat_a", a), ("kat_b", b)):
        h = O.histogram(d)
        pdf, cdf = O.normalize(h, d.size, 10)
        rp = np.asarray(pyref.normalize([int(v) for v in h], d.size, 10), dtype=np.uint32)
        assert np.array_equal(pdf, rp), f"oracle/pyref disagree: {name}"
        fx[f"{name}_pdf"] = pdf
    assert fx["kat_a_pdf"][1] == 769 and all(fx["kat_a_pdf"][i] == 1 for i in range(256) if i != 1)
    assert (fx["kat_b_pdf"] == 4).all()
    out = os.path.join(HERE, "golden.npz")
    np.savez_compressed(out, **fx)
    print("wrote", out, os.path.getsize(out), "bytes,", len(fx), "arrays")


if __name__ == "__main__":
    main()
