"""Shared input generators for the parity tests (seeded, numpy only)."""
import numpy as np

NP_WORD = {1: np.uint16, 2: np.uint16, 3: np.uint32, 4: np.uint64}
FT_NAME = {1: "fp16", 2: "bf16", 3: "fp32", 4: "fp64"}


def exp_bytes(n, lam=100.0, seed=1):
    """b = min(255, floor(256 * min(Exp(lam), 1))) -- ANSTest.cu:18-31 shape."""
    rng = np.random.default_rng(seed)
    x = rng.exponential(1.0 / lam, n)
    return np.minimum(255, np.floor(256.0 * np.minimum(x, 1.0))).astype(np.uint8)


def float_words(ft, n, seed=0, scale=1.0):
    """N(0,1) floats as raw words: bf16 by fp32 truncation (FloatTest.cu:21-29),
    fp16 by round-to-nearest, fp32 / fp64 native."""
    rng = np.random.default_rng(seed)
    if ft == 4:
        return (rng.standard_normal(n) * scale).astype(np.float64).view(np.uint64)
    f = (rng.standard_normal(n) * scale).astype(np.float32)
    if ft == 1:
        return f.astype(np.float16).view(np.uint16)
    if ft == 2:
        return (f.view(np.uint32) >> 16).astype(np.uint16)
    return f.view(np.uint32)


def sparsify(words, frac_zero=0.9, seed=5):
    rng = np.random.default_rng(seed)
    w = words.copy()
    w[rng.random(w.size) < frac_zero] = 0
    return w
