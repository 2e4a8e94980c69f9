"""Team layouts of the single-pass compressor (csrc/pcompress.h, kXcd) and
the team barrier's hand-off: no shape may fall back to counting its element
from the input (dietgpu_barrier_fallback_count), and every archive must equal
the oracle's.

Shapes ("what's weak" #3): batches of fewer than 8 multi-item
elements (padded with idle teams to an XCD-aligned grid: batch 1 x 1e6 and
1 x 524,288 bf16 words, the reference's first published batch-1 point and
smoke's shape; 3 x 1 MiB), a batch whose teams cannot be XCD-aligned within
the resident grid (33 x 1e6 words: teams of 31 items, 33 teams in 1,024
slots; partials stored write-through), and c2 (256 x 1 MiB bf16).  The
reference's per-shape behaviour being one archive per element regardless of
grid (ans/GpuANSEncode.cuh:670-845), the oracle is the checker."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import exp_bytes, float_words

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


# Team-barrier budget while the no-fallback tests run: 5 ms instead of the
# default 200 us, so a co-tenant kernel or a slow dispatch on a shared box
# cannot trip the count; a hand-off that never lands (a stale
# partial read across XCDs) still waits it out and is counted.
BUDGET_TICKS = 500_000


@pytest.fixture(autouse=True)
def _single_pass(C):
    """Small batches take the three-kernel path by default (the size rule,
    codec.hip persistentPreferred): this module's batches are meant for the
    single-pass compressor whenever it can take them."""
    C.set_barrier_budget(BUDGET_TICKS)
    try:
        with C.compress_path("single-pass"):
            yield
    finally:
        C.set_barrier_budget(20000)


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(768 << 20)


def _bf16_batch(nb, n, seed0):
    words = [float_words(2, n, seed=seed0 + i) for i in range(nb)]
    x = torch.from_numpy(np.stack(words).view(np.int16)).to(DEV).view(torch.bfloat16)
    return words, x


@pytest.mark.parametrize("nb,n,check", [
    (1, 1000000, "all"), (1, 524288, "all"), (3, 524288, "all"), (7, 300000, "all"),
    (33, 1000000, "all"), (256, 524288, "sample")])
def test_bf16_team_layouts_no_fallback(C, ws, nb, n, check):
    words, x = _bf16_batch(nb, n, seed0=nb * 7 + n % 97)
    C.device_error_count(reset=True)
    C.barrier_fallback_count(reset=True)
    for _ in range(3):  # repeated calls: epochs advance, arena words are reused
        out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
    torch.cuda.synchronize()
    assert C.barrier_fallback_count(reset=True) == 0
    assert C.device_error_count(reset=True) == 0
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    idx = range(nb) if check == "all" else sorted({0, 1, 63, 64, 127, 128, 200, nb - 1})
    for i in idx:
        ref = O.float_compress(words[i], 2)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")
    y, ok, _ = C.float_decompress_stride(out, n, torch.bfloat16, ws=ws)
    assert bool((ok == 1).all())
    assert torch.equal(y.view(torch.int16), x.view(torch.int16))


@pytest.mark.parametrize("ck", [False, True])
def test_bytes_non_xcd_teams_no_fallback(C, ws, ck):
    """33 byte elements of 31 items (1,015,808 bytes): the write-through
    partials of k_pcompress<0, ck, false>, with and without the checksum
    partials."""
    nb, n = 33, 31 * 8 * 4096
    datas = [exp_bytes(n, lam=20.0, seed=900 + i) for i in range(nb)]
    x = torch.from_numpy(np.stack(datas)).to(DEV)
    C.device_error_count(reset=True)
    C.barrier_fallback_count(reset=True)
    out, sizes = C.ans_encode_stride(x, checksum=ck, ws=ws)
    torch.cuda.synchronize()
    assert C.barrier_fallback_count(reset=True) == 0
    assert C.device_error_count(reset=True) == 0
    sizes = sizes.cpu().tolist()
    host = out.cpu().numpy()
    for i in (0, 1, 15, 31, 32):
        ref = O.ans_encode(datas[i], 10, ck)
        assert sizes[i] == ref.size, (i, sizes[i], ref.size)
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")


def test_fallback_counter_counts(C, ws):
    """Budget 0 forces the fallback wherever a team member's partial was not
    in at the first look -- always for teams of more than 16 items (each wave
    loads only its first four members' partials before the window's barrier):
    the counter must see them, and the archives stay the oracle's."""
    words, x = _bf16_batch(3, 1000000, seed0=77)
    C.barrier_fallback_count(reset=True)
    try:
        C.set_barrier_budget(0)
        out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
        torch.cuda.synchronize()
    finally:
        C.set_barrier_budget(20000)
    assert C.barrier_fallback_count(reset=True) > 0
    assert C.device_error_count(reset=True) == 0
    host = out.cpu().numpy()
    for i, w in enumerate(words):
        ref = O.float_compress(w, 2)
        np.testing.assert_array_equal(host[i, : ref.size], ref)


def test_size_rule_routes_by_work_items(C, ws):
    """The size rule (codec.hip persistentPreferred): with
    the barrier budget at 0 every single-pass team of more than 16 items
    falls back, so the fallback counter shows which compressor ran.  3 x 1e6
    words (93 items) go to the three-kernel path by default (no fallback)
    and single-pass when forced; 16 x 1e6 (496 items, XCD-aligned) stay
    single-pass by default.  Archives are the oracle's either way."""
    cases = ((3, "auto", False), (3, "single-pass", True), (16, "auto", True))
    for nb, mode, single in cases:
        words, x = _bf16_batch(nb, 1000000, seed0=91 + nb)
        C.barrier_fallback_count(reset=True)
        try:
            C.set_barrier_budget(0)
            with C.compress_path(mode):
                out, sizes = C.float_compress_stride(x, prob_bits=10, ws=ws)
            torch.cuda.synchronize()
        finally:
            C.set_barrier_budget(BUDGET_TICKS)
        assert (C.barrier_fallback_count(reset=True) > 0) == single, (nb, mode)
        assert C.device_error_count(reset=True) == 0
        host = out.cpu().numpy()
        for i in (0, nb - 1):
            ref = O.float_compress(words[i], 2)
            np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"{nb} {mode} element {i}")
