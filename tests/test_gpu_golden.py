"""GPU parity against the committed golden fixtures, at BASELINE.json's full
sizes, and through the torch.ops.dietgpu surface.  All calls go through the
HIP library (C ABI); the oracle only checks.

Full-size configs are checked by size-independent
properties -- bit-exact round trip, compression ratio, 16 B archive sizes --
plus byte-identity with the oracle on sampled elements."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import NP_WORD

pytestmark = pytest.mark.gpu

DEV = "cuda"
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")
NP_SIGNED = {1: np.int16, 2: np.int16, 3: np.int32, 4: np.int64}
FLOAT_DT = {1: torch.float16, 2: torch.bfloat16, 3: torch.float32, 4: torch.float64}


@pytest.fixture(scope="module")
def G():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(1 << 30)


def dev_words(w, ft):
    return torch.from_numpy(w.view(NP_SIGNED[ft]).copy()).to(DEV).view(FLOAT_DT[ft])


# --- golden fixtures ----------------------------------------------------------

@pytest.mark.parametrize("pb", [9, 10, 11])
@pytest.mark.parametrize("ck", [0, 1])
def test_golden_c1_gpu(C, ws, G, pb, ck):
    x = torch.from_numpy(G["c1_in"]).to(DEV)
    out, sizes = C.ans_encode_pointer([x], prob_bits=pb, checksum=bool(ck), ws=ws)
    ref = G[f"c1_pb{pb}_ck{ck}"]
    assert int(sizes[0]) == ref.size
    np.testing.assert_array_equal(out[0, : ref.size].cpu().numpy(), ref)
    y = torch.empty(65536, dtype=torch.uint8, device=DEV)
    ok, sz = C.ans_decode_pointer([torch.from_numpy(ref).to(DEV)], [y], prob_bits=pb,
                                  checksum=bool(ck), ws=ws)
    assert int(ok[0]) == 1 and int(sz[0]) == 65536
    assert torch.equal(y, x)


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
def test_golden_float_gpu(C, ws, G, ft):
    ns = (1, 13, 4095, 4096, 4097, 12345)
    xs = [dev_words(G[f"f{ft}_n{n}_in"], ft) for n in ns]
    out, sizes = C.float_compress_pointer(xs, ft=ft, prob_bits=10, ws=ws)
    for i, n in enumerate(ns):
        ref = G[f"f{ft}_n{n}_pb10"]
        assert int(sizes[i]) == ref.size, n
        np.testing.assert_array_equal(out[i, : ref.size].cpu().numpy(), ref, err_msg=str(n))
    arch = [torch.from_numpy(G[f"f{ft}_n{n}_pb10"]).to(DEV) for n in ns]
    ys = [torch.empty_like(x) for x in xs]
    ok, sz = C.float_decompress_pointer(arch, ys, ft=ft, prob_bits=10, ws=ws)
    assert ok.cpu().tolist() == [1] * len(ns) and sz.cpu().tolist() == list(ns)
    for x, y in zip(xs, ys):
        assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))


@pytest.mark.parametrize("pb", [9, 11])
def test_golden_float_pb_checksum_gpu(C, ws, G, pb):
    x = dev_words(G["f2_pbx_in"], 2)
    out, sizes = C.float_compress_pointer([x], ft=2, prob_bits=pb, checksum=True, ws=ws)
    ref = G[f"f2_pb{pb}_ck1"]
    np.testing.assert_array_equal(out[0, : int(sizes[0])].cpu().numpy(), ref)


@pytest.mark.parametrize("ft", [2, 3])
@pytest.mark.parametrize("tag", ["z", "nz"])
def test_golden_sparse_gpu(C, ws, G, ft, tag):
    x = dev_words(G[f"s{ft}_{tag}_in"], ft)
    out, sizes = C.sparse_compress([x], ft=ft, prob_bits=10, ws=ws)
    ref = G[f"s{ft}_{tag}_pb10"]
    np.testing.assert_array_equal(out[0, : int(sizes[0])].cpu().numpy(), ref)
    y = torch.empty_like(x)
    ok, sz = C.sparse_decompress([torch.from_numpy(ref).to(DEV)], [y], ft=ft, ws=ws)
    assert int(ok[0]) == 1 and torch.equal(x.view(torch.uint8), y.view(torch.uint8))


# --- full-size BASELINE configs -----------------------------------------------

def test_c2_full_bf16(C, ws):
    """c2: 256 x 524,288 bf16 N(0,1) (torch.randn seed 0, truncated)."""
    nb, n = 256, 524288
    g = torch.Generator(device=DEV).manual_seed(0)
    x = (torch.randn(nb, n, generator=g, device=DEV).view(torch.int32) >> 16).to(torch.int16)
    x = x.view(torch.bfloat16)
    out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
    s = sizes.cpu().numpy().astype(np.int64)
    assert (s % 16 == 0).all()
    ratio = s.sum() / (nb * n * 2)
    assert 0.66 < ratio < 0.69, ratio
    y, ok, sz = C.float_decompress_stride(out, n, torch.bfloat16, ws=ws)
    assert bool((ok == 1).all()) and bool((sz == n).all())
    assert torch.equal(y.view(torch.int16), x.view(torch.int16))
    for i in (0, 97, 255):  # sampled byte identity with the oracle
        w = x[i].view(torch.int16).cpu().numpy().view(np.uint16)
        ref = O.float_compress(w, 2, 10)
        np.testing.assert_array_equal(out[i, : s[i]].cpu().numpy(), ref)


def test_c3_uniform16_bytes(C, ws):
    """c3 shape (uniform over 16 symbols, 4 MiB elements) at 64 elements."""
    nb, n = 64, 4 << 20
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randint(0, 16, (nb, n), generator=g, device=DEV, dtype=torch.uint8)
    out, sizes = C.ans_encode_stride(x, prob_bits=10, ws=ws)
    s = sizes.cpu().numpy().astype(np.int64)
    assert 0.50 < s.sum() / (nb * n) < 0.54
    y, ok, sz = C.ans_decode_stride(out, n, ws=ws)
    assert bool((ok == 1).all()) and torch.equal(y, x)
    ref = O.ans_encode(x[5].cpu().numpy(), 10)
    np.testing.assert_array_equal(out[5, : s[5]].cpu().numpy(), ref)


def test_c4_fp64_and_sparse(C, ws):
    """c4: 16,777,216 fp64 N(0,1) (two ANS passes) + 90 %-sparse fp32."""
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(16777216, generator=g, device=DEV, dtype=torch.float64)
    out, sizes = C.float_compress_pointer([x], prob_bits=10, ws=ws)
    s = int(sizes[0])
    assert 0.85 < s / x.numel() / 8 < 0.93
    ref = O.float_compress(x.cpu().numpy().view(np.uint64), 4, 10)
    np.testing.assert_array_equal(out[0, :s].cpu().numpy(), ref)
    y = torch.empty_like(x)
    ok, _ = C.float_decompress_pointer([out[0, :s].clone()], [y], prob_bits=10, ws=ws)
    assert int(ok[0]) == 1 and torch.equal(x.view(torch.int64), y.view(torch.int64))

    g = torch.Generator(device=DEV).manual_seed(5)
    f = torch.randn(15000000, generator=g, device=DEV)
    f[torch.rand(f.numel(), generator=g, device=DEV) < 0.9] = 0.0
    out, sizes = C.sparse_compress([f], prob_bits=10, ws=ws)
    s = int(sizes[0])
    ref = O.sparse_compress(f.cpu().numpy().view(np.uint32), 3, 10)
    np.testing.assert_array_equal(out[0, :s].cpu().numpy(), ref)
    y = torch.empty_like(f)
    ok, _ = C.sparse_decompress([out[0, :s].clone()], [y], ws=ws)
    assert int(ok[0]) == 1 and torch.equal(f.view(torch.int32), y.view(torch.int32))


@pytest.mark.parametrize("ft,nb,n", [(1, 256, 262144), (3, 256, 262144), (4, 64, 524288)])
def test_throughput_shape_other_floats(C, ws, ft, nb, n):
    """Large fp16 / fp32 / fp64 batches (multi-generation grids, persistent
    decode workgroups with several chunks each): bit-exact round trip and
    byte identity with the oracle on a sampled element."""
    g = torch.Generator(device=DEV).manual_seed(20 + ft)
    x = torch.randn(nb, n, generator=g, device=DEV, dtype=torch.float64).to(FLOAT_DT[ft])
    out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
    s = sizes.cpu().numpy().astype(np.int64)
    y, ok, sz = C.float_decompress_stride(out, n, FLOAT_DT[ft], ws=ws)
    assert bool((ok == 1).all()) and bool((sz == n).all())
    assert torch.equal(y.view(torch.uint8), x.view(torch.uint8))
    i = nb // 3
    ref = O.float_compress(x[i].cpu().numpy().view(NP_WORD[ft]), ft, 10)
    np.testing.assert_array_equal(out[i, : s[i]].cpu().numpy(), ref)


# --- torch.ops.dietgpu (DietGpu.cpp) ------------------------------------------

def test_torch_ops_float_roundtrip(C):
    d = torch.ops.dietgpu
    xs = [torch.randn(n, device=DEV, dtype=torch.bfloat16) for n in (1, 4096, 70001)]
    comp, sizes, hw = d.compress_data(True, xs)
    assert comp.dtype == torch.uint8 and comp.shape[0] == 3 and hw >= 0
    for i, x in enumerate(xs):
        ref = O.float_compress(x.view(torch.int16).cpu().numpy().view(np.uint16), 2, 10)
        np.testing.assert_array_equal(comp[i, : int(sizes[i])].cpu().numpy(), ref)
    outs = [torch.empty_like(x) for x in xs]
    status = torch.empty(3, dtype=torch.uint8, device=DEV)
    words = torch.empty(3, dtype=torch.int32, device=DEV)
    d.decompress_data(True, [comp[i, : int(sizes[i])] for i in range(3)], outs, False, None,
                      status, words)
    assert status.cpu().tolist() == [1, 1, 1]
    assert words.cpu().tolist() == [x.numel() for x in xs]
    for x, y in zip(xs, outs):
        assert torch.equal(x.view(torch.int16), y.view(torch.int16))


def test_torch_ops_simple_and_split(C):
    d = torch.ops.dietgpu
    xs = [torch.randint(0, 7, (n,), device=DEV, dtype=torch.uint8) for n in (10, 5000)]
    comp = d.compress_data_simple(False, xs)
    dec = d.decompress_data_simple(False, comp)
    for x, y in zip(xs, dec):
        assert torch.equal(x, y)
    t = torch.randn(3000, device=DEV, dtype=torch.float16)
    split = torch.tensor([1000, 1, 1999], dtype=torch.int32)  # splits must be > 0
    comp, sizes, _ = d.compress_data_split_size(True, t, split)
    out = torch.empty_like(t)
    d.decompress_data_split_size(True, [c[: int(s)] for c, s in zip(comp, sizes)], out, split)
    assert torch.equal(out.view(torch.int16), t.view(torch.int16))
