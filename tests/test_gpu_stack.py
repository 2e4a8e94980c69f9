"""GPU tests of the temporary-memory and stream contract (SURVEY 8(a) a28,
8(b) "Ownership" / "Threading"): the StackDeviceMemory high-water mark the
torch ops return (DietGpu.cpp compress_data's third output), the hipMalloc
overflow path of a too-small temp_mem (correct archives, a warning), and
concurrent calls on two streams, whose single-pass compressor flags live in
separate per-stream arenas (csrc/sync_arena.cpp)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

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


def _bf16(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, generator=g) * (1 + seed % 3)).to(torch.bfloat16)


def _check(xs, comp, sizes):
    host = comp.cpu().numpy()
    sizes = sizes.cpu().tolist()
    for i, x in enumerate(xs):
        ref = O.float_compress(x.view(torch.int16).numpy().view(np.uint16), 2)
        assert sizes[i] == ref.size, i
        np.testing.assert_array_equal(host[i, : ref.size], ref, err_msg=f"element {i}")


def test_high_water_mark(C):
    xs = [_bf16(n, i) for i, n in enumerate((524288, 100000, 7))]
    tmp = torch.empty([64 << 20], dtype=torch.uint8, device=DEV)
    comp, sizes, used = torch.ops.dietgpu.compress_data(True, [x.to(DEV) for x in xs], False, tmp)
    assert 0 < used <= tmp.numel()
    _check(xs, comp, sizes)
    outs = [torch.empty(x.numel(), dtype=torch.bfloat16, device=DEV) for x in xs]
    rows = [comp[i, : int(sizes[i])] for i in range(len(xs))]
    used_d = torch.ops.dietgpu.decompress_data(True, rows, outs, False, tmp)
    assert 0 <= used_d <= tmp.numel()
    for x, o in zip(xs, outs):
        assert torch.equal(o.cpu().view(torch.int16), x.view(torch.int16))


def test_small_temp_mem_overflows_to_hipmalloc(C, capfd):
    """A temp_mem far too small for the call: the arena falls back to
    hipMalloc (with the reference's warning) and the archives are still exact."""
    xs = [_bf16(300000, i) for i in range(4)]
    tmp = torch.empty([4096], dtype=torch.uint8, device=DEV)
    comp, sizes, _ = torch.ops.dietgpu.compress_data(True, [x.to(DEV) for x in xs], False, tmp)
    torch.cuda.synchronize()
    _check(xs, comp, sizes)
    err = capfd.readouterr().err
    assert "StackDeviceMemory" in err


def test_concurrent_streams(C):
    """Two streams compress different batches at the same time, each with its
    own workspace; both sets of archives match the oracle (the single-pass
    compressor's epoch-tagged flags are per (device, stream))."""
    xa = [_bf16(524288, 10 + i) for i in range(64)]
    xb = [_bf16(262144 + 4096 * i, 100 + i) for i in range(48)]
    da, db = [x.to(DEV) for x in xa], [x.to(DEV) for x in xb]
    wa, wb = C.Workspace(128 << 20), C.Workspace(128 << 20)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    results = {}
    for rep in range(3):
        with torch.cuda.stream(sa):
            results["a"] = C.float_compress_pointer(da, ws=wa)
        with torch.cuda.stream(sb):
            results["b"] = C.float_compress_pointer(db, ws=wb)
        torch.cuda.synchronize()
        _check(xa, *results["a"])
        _check(xb, *results["b"])
