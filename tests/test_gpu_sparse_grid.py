"""The reference's sparse benchmark grid (float/SparseFloatBenchmark.cu:
402-447) as GPU parity tests: fp16 / bf16 / fp32 / fp64 x batch {1, 3, 5},
every element of the batch the same size (its "multipleOf": 100,000,
150,000, 1e6, 1.5e6, 1e7 and 1.5e7 words), 50 % of the words +0.0, float
checksum on, at probBits 9 as the reference runs it (the whole grid) and at
11 (the 1.5x column).  Every archive size is
16 B aligned and every roundtrip bit-exact; the first and last element of
each batch are byte-identical to the CPU oracle's archive.  The reference's
own check is only the roundtrip (with a nondeterministic sparsity pattern);
inputs here are seeded."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import NP_WORD

pytestmark = pytest.mark.gpu

DEV = "cuda"
TORCH_WORD = {1: torch.int16, 2: torch.int16, 3: torch.int32, 4: torch.int64}
DTYPE = {1: torch.float16, 2: torch.bfloat16, 3: torch.float32, 4: torch.float64}


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(2 << 30)


def _sparse_batch(ft, nb, n, frac_zero, seed):
    """nb tensors of n words: N(0,1) in the float type (bf16 by truncation as
    FloatTest.cu:21-29), then a Bernoulli(frac_zero) mask of +0.0."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    out = []
    for _ in range(nb):
        if ft == 4:
            x = torch.randn(n, generator=g, device=DEV, dtype=torch.float64)
        elif ft == 2:
            x = (torch.randn(n, generator=g, device=DEV).view(torch.int32) >> 16).to(torch.int16)
            x = x.view(torch.bfloat16)
        else:
            x = torch.randn(n, generator=g, device=DEV).to(DTYPE[ft])
        x = x.view(TORCH_WORD[ft])
        x[torch.rand(n, generator=g, device=DEV) < frac_zero] = 0
        out.append(x)
    return out


# the whole grid at pb 9 (SparseFloatBenchmark.cu:440-447: batch {1, 3, 5} x
# multipleOf {1e5, 1.5e5, 1e6, 1.5e6, 1e7, 1.5e7}); pb 11 on the 1.5x column
GRID = [(nb, n) for n in (100000, 150000, 1000000, 1500000, 10000000, 15000000) for nb in (1, 3, 5)]
CASES = ([(nb, n, 9) for nb, n in GRID] +
         [(nb, n, 11) for nb, n in GRID if n in (150000, 1500000, 15000000)])


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
@pytest.mark.parametrize("nb,n,pb", CASES)
def test_sparse_benchmark_grid(C, ws, ft, pb, nb, n):
    ts = _sparse_batch(ft, nb, n, 0.5, seed=1000 * ft + 10 * nb + pb)
    out, sizes = C.sparse_compress(ts, ft=ft, prob_bits=pb, checksum=True, ws=ws)
    sizes_h = sizes.cpu().tolist()
    assert all(s > 0 and s % 16 == 0 for s in sizes_h), sizes_h
    for i in sorted({0, nb - 1}):
        w = ts[i].cpu().numpy().view(NP_WORD[ft])
        ref = O.sparse_compress(w, ft, prob_bits=pb, checksum=True)
        assert sizes_h[i] == ref.size, (i, sizes_h[i], ref.size)
        np.testing.assert_array_equal(out[i, : ref.size].cpu().numpy(), ref, err_msg=f"element {i}")
    arch = [out[i, : sizes_h[i]] for i in range(nb)]
    outs = [torch.empty_like(t) for t in ts]
    ok, sz = C.sparse_decompress(arch, outs, ft=ft, prob_bits=pb, checksum=True, ws=ws)
    assert ok.cpu().tolist() == [1] * nb
    assert sz.cpu().tolist() == [n] * nb
    for a, b in zip(ts, outs):
        assert torch.equal(a, b)
    del ts, outs, out, arch
    torch.cuda.empty_cache()
