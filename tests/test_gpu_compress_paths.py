"""GPU parity of the two compression paths (csrc/codec.hip encodeBatchDevice):
the single-pass k_pcompress (teams of at most pc::kMaxTeam = 32 workgroups,
i.e. elements of at most 1 MiB of ANS symbols) and the three-kernel
k_hist -> k_encode path (k_normalize / k_histReduce, or the encoder's
prologue normalisation) taken otherwise.  Both must write the
oracle's archive byte for byte, including dense blocks whose output spills
out of the 1024-word LDS rings and blocks that emit no words."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import exp_bytes

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


def _check_ans(C, ws, datas, pb=10, checksum=False):
    ts = [torch.from_numpy(d).to(DEV) for d in datas]
    out, sizes = C.ans_encode_pointer(ts, prob_bits=pb, checksum=checksum, ws=ws)
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i, d in enumerate(datas):
        ref = O.ans_encode(d, pb, checksum)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    arch = [out[i, : sizes[i]].clone() for i in range(len(ts))]
    outs = [torch.empty(d.size, dtype=torch.uint8, device=DEV) for d in datas]
    ok, _ = C.ans_decode_pointer(arch, outs, prob_bits=pb, checksum=checksum, ws=ws)
    assert ok.cpu().tolist() == [1] * len(ts)
    for d, o in zip(datas, outs):
        np.testing.assert_array_equal(o.cpu().numpy(), d)
    return host, sizes


@pytest.mark.parametrize("checksum", [False, True])
def test_team_limit_both_paths(C, ws, checksum):
    """1 MiB (team of 32: single pass) and 1 MiB + 1 (three kernels)."""
    for n in (MIB, MIB + 1):
        _check_ans(C, ws, [exp_bytes(n, lam=30.0, seed=n & 7), exp_bytes(n // 3, lam=3.0, seed=9)],
                   checksum=checksum)


def test_paths_write_identical_archives(C, ws):
    a = exp_bytes(200000, lam=50.0, seed=21)
    big = exp_bytes(MIB + 4096, lam=50.0, seed=22)
    h1, s1 = _check_ans(C, ws, [a])          # single pass
    h2, s2 = _check_ans(C, ws, [a, big])     # whole batch on the three-kernel path
    assert s1[0] == s2[0]
    np.testing.assert_array_equal(h1[0, : s1[0]], h2[0, : s2[0]])


@pytest.mark.parametrize("pb", [9, 11])
def test_dense_blocks_spill(C, ws, pb):
    """Uniform bytes: ~2048 words per block, beyond the 1024-word ring."""
    rng = np.random.default_rng(5)
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (4096 * 24 + 77, 65536, 5000)]
    _check_ans(C, ws, datas, pb=pb)


def test_constant_input_emits_no_words(C, ws):
    """A single symbol gets pdf = 2^pb: no block emits a word."""
    datas = [np.full(n, 7, dtype=np.uint8) for n in (4096 * 9, 4096 * 8 + 5, 1)]
    _check_ans(C, ws, datas)


@pytest.mark.parametrize("offset_words", [1, 3])
def test_float_unaligned_input(C, ws, offset_words):
    """Input not 16 B aligned: the three-kernel path (k_pcompress reads whole
    16 B vectors, so the host routes unaligned inputs to k_hist -> k_encode)."""
    g = torch.Generator().manual_seed(offset_words)
    base = torch.randn(70000 + offset_words, generator=g).to(torch.bfloat16)
    x = base[offset_words:]
    xd = base.to(DEV)[offset_words:]
    assert xd.data_ptr() % 16 != 0
    arch, sizes = C.float_compress_pointer([xd], prob_bits=10, ws=ws)
    ref = O.float_compress(x.view(torch.int16).numpy().view(np.uint16), 2)
    assert int(sizes[0]) == ref.size
    np.testing.assert_array_equal(arch[0, : ref.size].cpu().numpy(), ref)


@pytest.mark.parametrize("pb", [9, 11])
def test_dense_blocks_three_kernel_ring_overflow(C, ws, pb):
    """k_encode keeps each block's output in a 1024-word LDS ring and flushes
    only the overflow to its slot: uniform bytes (~2048 words per block) wrap
    the ring and spill several 256-word chunks; the > 1 MiB element sends the
    whole batch down the three-kernel path."""
    rng = np.random.default_rng(7)
    datas = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (4096 * 24 + 77, 65536, 5000)]
    datas.append(exp_bytes(MIB + 4096, lam=2.0, seed=23))
    _check_ans(C, ws, datas, pb=pb)
