"""The reference's own float torch-op harness (dietgpu/float_test.py:13-108)
re-expressed against torch.ops.dietgpu: compress_data with checksum=True ->
archives truncated to the reported sizes -> decompress_data with checksum=True,
with and without temp_mem (out_status / out_sizes when it is given), for
bf16, fp16 and fp32 -- test_codec (1e4 / 1e5 / 1e6 words), test_large (one
123,456,789-word tensor: the multi-kernel path plus the float checksum and
its verification), test_simple and test_empty.  Beyond the reference's
roundtrip checks, the archives are compared with the CPU oracle (on every
element of test_codec, and whole for test_large's bf16 tensor)."""
import numpy as np
import pytest
import torch

import dietgpu_fork_amd  # noqa: F401  (registers torch.ops.dietgpu)
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
FT = {torch.float16: 1, torch.bfloat16: 2, torch.float32: 3}
NPW = {torch.float16: np.uint16, torch.bfloat16: np.uint16, torch.float32: np.uint32}
ITW = {torch.float16: torch.int16, torch.bfloat16: torch.int16, torch.float32: torch.int32}


def _words(t):
    return t.view(ITW[t.dtype]).cpu().numpy().view(NPW[t.dtype])


def run_test(ts, temp_mem=None, oracle_elems=()):
    """float_test.py:13-47 run_test, plus oracle identity of `oracle_elems`."""
    comp, sizes, _ = torch.ops.dietgpu.compress_data(True, ts, True, temp_mem)
    sizes_h = sizes.cpu().tolist()
    for i in oracle_elems:
        ref = O.float_compress(_words(ts[i]), FT[ts[i].dtype], checksum=True)
        assert sizes_h[i] == ref.size, (i, sizes_h[i], ref.size)
        np.testing.assert_array_equal(comp[i, : ref.size].cpu().numpy(), ref, err_msg=f"element {i}")
    # truncated to exactly the reported sizes: the sizes must be exact
    truncated = [t.narrow(0, 0, s).clone() for s, t in zip(sizes_h, [*comp])]
    out_ts = [torch.empty(t.size(), dtype=t.dtype, device=t.device) for t in ts]
    if temp_mem is not None:
        out_status = torch.empty([len(ts)], dtype=torch.uint8, device=DEV)
        out_sizes = torch.empty([len(ts)], dtype=torch.int32, device=DEV)
        torch.ops.dietgpu.decompress_data(True, truncated, out_ts, True, temp_mem, out_status, out_sizes)
        for t, status, size in zip(ts, out_status.cpu().tolist(), out_sizes.cpu().tolist()):
            assert status
            assert t.numel() == size
    else:
        torch.ops.dietgpu.decompress_data(True, truncated, out_ts, True)
    for a, b in zip(ts, out_ts):
        assert torch.equal(a.view(ITW[a.dtype]), b.view(ITW[b.dtype]))
    return sizes_h


@pytest.fixture(scope="module")
def temp_mem():
    return torch.empty([64 * 1024 * 1024], dtype=torch.uint8, device=DEV)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("tm", [False, True])
def test_codec(dt, tm, temp_mem):
    g = torch.Generator(device=DEV).manual_seed(7)
    ts = [torch.normal(0, 1.0, [i], dtype=torch.float32, device=DEV, generator=g).to(dt)
          for i in [10000, 100000, 1000000]]
    run_test(ts, temp_mem if tm else None, oracle_elems=range(len(ts)))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("tm", [False, True])
def test_large(dt, tm, temp_mem):
    g = torch.Generator(device=DEV).manual_seed(8)
    ts = [torch.normal(0, 1.0, [123456789], dtype=torch.float32, device=DEV, generator=g).to(dt)]
    sizes = run_test(ts, temp_mem if tm else None,
                     oracle_elems=(0,) if (dt == torch.bfloat16 and not tm) else ())
    # exponent-split ratios of N(0,1): bf16 ~0.67, fp16 ~0.86, fp32 ~0.84
    ratio = sizes[0] / (ts[0].numel() * ts[0].element_size())
    assert ratio < {torch.bfloat16: 0.70, torch.float16: 0.88, torch.float32: 0.86}[dt]
    del ts
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_simple(dt):
    g = torch.Generator(device=DEV).manual_seed(9)
    ts = [torch.normal(0, 1.0, [i], dtype=torch.float32, device=DEV, generator=g).to(dt)
          for i in [10000, 100000, 1000000]]
    cts = torch.ops.dietgpu.compress_data_simple(True, ts, True)
    for before, after in zip(ts, cts):
        # we should actually be compressing data
        assert before.numel() * before.element_size() > after.numel() * after.element_size()
    dts = torch.ops.dietgpu.decompress_data_simple(True, cts, True)
    for orig, after in zip(ts, dts):
        assert torch.equal(orig.view(ITW[dt]), after.view(ITW[dt]))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
def test_empty(dt):
    ts = [torch.empty([0], dtype=dt, device=DEV)]
    comp_ts = torch.ops.dietgpu.compress_data_simple(True, ts, True)
    assert comp_ts[0].numel() > 0  # should have a header
    ref = O.float_compress(np.zeros(0, dtype=NPW[dt]), FT[dt], checksum=True)
    np.testing.assert_array_equal(comp_ts[0].cpu().numpy(), ref)
    decomp_ts = torch.ops.dietgpu.decompress_data_simple(True, comp_ts, True)
    assert torch.equal(ts[0], decomp_ts[0])
