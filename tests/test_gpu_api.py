"""GPU coverage of the API paths beyond the pointer/stride entry points:
split-size ANS and float codecs (GpuANSCodec.h:130-167,265-300,
GpuFloatCodec.h:92-160), the reference's own split-size torch tests
(ans_test.py:79-139), the *GetCompressedInfo readouts (GpuANSInfo.cuh:16-57,
GpuFloatInfo.cuh:18-62), fp64 through torch.ops.dietgpu (an extension: the
reference rejects fp64 at DietGpu.cpp:569-573), the compressor's error path
(bounded waits poison an element: outSize 0 + device error count), hipGraph
capture / replay, and oversize requests.  Archives are compared byte for byte
with the CPU oracle (oracle/), roundtrips bit for bit."""
import ctypes
import random

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.util import NP_WORD, exp_bytes, float_words

pytestmark = pytest.mark.gpu

DEV = "cuda"
TORCH_WORD = {1: torch.int16, 2: torch.int16, 3: torch.int32, 4: torch.int64}
NP_SIGNED = {1: np.int16, 2: np.int16, 3: np.int32, 4: np.int64}
TORCH_FLOAT = {1: torch.float16, 2: torch.bfloat16, 3: torch.float32, 4: torch.float64}
WORD_BYTES = {1: 2, 2: 2, 3: 4, 4: 8}


@pytest.fixture(scope="module")
def C():
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec

    return codec


@pytest.fixture(scope="module")
def N(C):
    from dietgpu_fork_amd import _native

    return _native


@pytest.fixture(scope="module")
def ws(C):
    return C.Workspace(512 << 20)


def _s():
    return torch.cuda.current_stream().cuda_stream


def _ans_split_sizes(rng, nb):
    # interior splits must be multiples of 4 bytes (GpuANSCodec.h:16)
    sizes = [int(rng.integers(1, 20000)) for _ in range(nb)]
    return [s + (4 - s % 4) % 4 if i + 1 < nb else s for i, s in enumerate(sizes)]


@pytest.mark.parametrize("checksum", [False, True])
def test_ans_split_size_parity(C, N, ws, checksum):
    """ansEncodeBatchSplitSize / ansDecodeBatchSplitSize against the oracle."""
    rng = np.random.default_rng(7 + checksum)
    sizes = _ans_split_sizes(rng, 9)
    data = exp_bytes(sum(sizes), lam=10.0, seed=3)
    t = torch.from_numpy(data).to(DEV)
    cols = C.max_compressed_size(max(sizes))
    out = torch.empty([len(sizes), cols], dtype=torch.uint8, device=DEV)
    osz = torch.empty([len(sizes)], dtype=torch.int32, device=DEV)
    L = N.lib()
    N.check(L.dietgpu_ans_encode_batch_split_size(ws.h, 10, int(checksum), len(sizes), t.data_ptr(),
                                                  N.u32_array(sizes), None, out.data_ptr(), cols,
                                                  osz.data_ptr(), _s()))
    got = osz.cpu().tolist()
    host = out.cpu().numpy()
    off = 0
    for i, n in enumerate(sizes):
        ref = O.ans_encode(data[off:off + n], 10, checksum)
        assert got[i] == ref.size and got[i] % 16 == 0
        np.testing.assert_array_equal(host[i, :ref.size], ref, err_msg=f"element {i}")
        off += n
    rows = [out[i, :got[i]].clone() for i in range(len(sizes))]
    dec = torch.empty(sum(sizes), dtype=torch.uint8, device=DEV)
    ok = torch.empty([len(sizes)], dtype=torch.uint8, device=DEV)
    dsz = torch.empty([len(sizes)], dtype=torch.int32, device=DEV)
    N.check(L.dietgpu_ans_decode_batch_split_size(ws.h, 10, int(checksum), len(sizes),
                                                  N.ptr_array([r.data_ptr() for r in rows]),
                                                  dec.data_ptr(), N.u32_array(sizes), ok.data_ptr(),
                                                  dsz.data_ptr(), _s()))
    assert ok.cpu().tolist() == [1] * len(sizes)
    assert dsz.cpu().tolist() == sizes
    assert torch.equal(dec, t)


@pytest.mark.parametrize("ft", [1, 2, 3, 4])
@pytest.mark.parametrize("checksum", [False, True])
def test_float_split_size_parity(C, N, ws, ft, checksum):
    """floatCompressSplitSize / floatDecompressSplitSize against the oracle
    (16 B-multiple splits take the single-pass compressor, ragged ones the
    three-kernel path)."""
    rng = np.random.default_rng(ft * 10 + checksum)
    per16 = 16 // WORD_BYTES[ft]
    sizes = [int(rng.integers(1, 9000)) for _ in range(7)]
    sizes[1] = 300000
    sizes[2] = per16 * 4097  # 16 B multiple
    words = float_words(ft, sum(sizes), seed=ft)
    t = torch.from_numpy(words.view(NP_SIGNED[ft]).copy()).to(DEV)
    cols = C.max_float_compressed_size(ft, max(sizes))
    out = torch.empty([len(sizes), cols], dtype=torch.uint8, device=DEV)
    osz = torch.empty([len(sizes)], dtype=torch.int32, device=DEV)
    L = N.lib()
    N.check(L.dietgpu_float_compress_split_size(ws.h, ft, 10, int(checksum), len(sizes), t.data_ptr(),
                                                N.u32_array(sizes), out.data_ptr(), cols,
                                                osz.data_ptr(), _s()))
    got = osz.cpu().tolist()
    host = out.cpu().numpy()
    off = 0
    for i, n in enumerate(sizes):
        ref = O.float_compress(words[off:off + n], ft, 10, checksum)
        assert got[i] == ref.size and got[i] % 16 == 0
        np.testing.assert_array_equal(host[i, :ref.size], ref, err_msg=f"element {i}")
        off += n
    rows = [out[i, :got[i]].clone() for i in range(len(sizes))]
    dec = torch.empty_like(t)
    ok = torch.empty([len(sizes)], dtype=torch.uint8, device=DEV)
    dsz = torch.empty([len(sizes)], dtype=torch.int32, device=DEV)
    rc = L.dietgpu_float_decompress_split_size(ws.h, ft, 10, int(checksum), len(sizes),
                                               N.ptr_array([r.data_ptr() for r in rows]),
                                               dec.data_ptr(), N.u32_array(sizes), ok.data_ptr(),
                                               dsz.data_ptr(), _s())
    N.check(rc)
    assert ok.cpu().tolist() == [1] * len(sizes)
    assert dsz.cpu().tolist() == sizes
    assert torch.equal(dec, t)


@pytest.mark.parametrize("checksum", [False, True])
@pytest.mark.parametrize("n", [70001, 1_000_000])
def test_single_element_table_apis(C, N, ws, n, checksum):
    """One-element pointer and split-size calls: the three-kernel path gets
    stride descriptors of that element instead of an uploaded table
    (DeviceDescs, codec.hip), for the encoder, the float checksum view and
    the decoder's checksum verification alike.  The element sits at a 2-byte
    offset (not 16 B-aligned: always the three-kernel path) and, for the
    float codecs, in every float type; archives equal the oracle's, roundtrips
    are exact (ans/GpuANSCodec.h:93-167, float/GpuFloatCodec.h:92-160)."""
    L = N.lib()
    data = exp_bytes(n + 2, lam=10.0, seed=n % 97)
    buf = torch.from_numpy(data).to(DEV)
    ref = O.ans_encode(data[2:], 10, checksum)
    # pointer API
    arch, osz = C.ans_encode_pointer([buf[2:]], checksum=checksum, ws=ws)
    assert int(osz[0]) == ref.size
    np.testing.assert_array_equal(arch[0][: ref.size].cpu().numpy(), ref)
    y = torch.empty(n, dtype=torch.uint8, device=DEV)
    ok, dsz = C.ans_decode_pointer([arch[0][: ref.size].clone()], [y], checksum=checksum, ws=ws)
    assert ok.cpu().tolist() == [1] and dsz.cpu().tolist() == [n] and torch.equal(y, buf[2:])
    # split-size API (one split: the whole buffer from a 4 B-aligned base)
    cols = C.max_compressed_size(n + 2)
    out = torch.empty([1, cols], dtype=torch.uint8, device=DEV)
    N.check(L.dietgpu_ans_encode_batch_split_size(ws.h, 10, int(checksum), 1, buf.data_ptr(),
                                                  N.u32_array([n + 2]), None, out.data_ptr(), cols,
                                                  osz.data_ptr(), _s()))
    ref2 = O.ans_encode(data, 10, checksum)
    assert int(osz[0]) == ref2.size
    np.testing.assert_array_equal(out[0, : ref2.size].cpu().numpy(), ref2)
    dec = torch.empty(n + 2, dtype=torch.uint8, device=DEV)
    row = out[0, : ref2.size].clone()
    N.check(L.dietgpu_ans_decode_batch_split_size(ws.h, 10, int(checksum), 1, N.ptr_array([row.data_ptr()]),
                                                  dec.data_ptr(), N.u32_array([n + 2]), ok.data_ptr(),
                                                  dsz.data_ptr(), _s()))
    assert ok.cpu().tolist() == [1] and torch.equal(dec, buf)
    for ft in (1, 2, 3, 4):
        wb = WORD_BYTES[ft]
        words = float_words(ft, n + 1, seed=ft + n % 13)
        t = torch.from_numpy(words.view(NP_SIGNED[ft]).copy()).to(DEV)
        x = t[1:].view(TORCH_FLOAT[ft])  # one word in: not 16 B-aligned
        fref = O.float_compress(words[1:], ft, 10, checksum)
        farch, fsz = C.float_compress_pointer([x], ft=ft, checksum=checksum, ws=ws)
        assert int(fsz[0]) == fref.size, ft
        np.testing.assert_array_equal(farch[0][: fref.size].cpu().numpy(), fref, err_msg=f"ft {ft}")
        fy = torch.empty_like(x)
        ok, dsz = C.float_decompress_pointer([farch[0][: fref.size].clone()], [fy], ft=ft, checksum=checksum,
                                             ws=ws)
        assert ok.cpu().tolist() == [1] and dsz.cpu().tolist() == [n], ft
        assert torch.equal(fy.view(TORCH_WORD[ft]), t[1:]), ft
        # split-size API: one split from an unaligned base
        fcols = C.max_float_compressed_size(ft, n)
        fout = torch.empty([1, fcols], dtype=torch.uint8, device=DEV)
        N.check(L.dietgpu_float_compress_split_size(ws.h, ft, 10, int(checksum), 1, t.data_ptr() + wb,
                                                    N.u32_array([n]), fout.data_ptr(), fcols, fsz.data_ptr(),
                                                    _s()))
        assert int(fsz[0]) == fref.size, ft
        np.testing.assert_array_equal(fout[0, : fref.size].cpu().numpy(), fref, err_msg=f"split ft {ft}")
        fdec = torch.empty(n + 1, dtype=TORCH_WORD[ft], device=DEV)
        frow = fout[0, : fref.size].clone()
        N.check(L.dietgpu_float_decompress_split_size(ws.h, ft, 10, int(checksum), 1, N.ptr_array([frow.data_ptr()]),
                                                      fdec.data_ptr() + wb, N.u32_array([n]), ok.data_ptr(),
                                                      dsz.data_ptr(), _s()))
        assert ok.cpu().tolist() == [1] and torch.equal(fdec[1:], t[1:]), ft


def test_reference_ans_split_tests(C):
    """ans_test.py:79-139 (test_split_compress / test_split_decompress): byte
    mode, checksum on, 64 MiB temp memory, through torch.ops.dietgpu."""
    dev = torch.device("cuda:0")
    temp_mem = torch.empty([64 * 1024 * 1024], dtype=torch.uint8, device=dev)
    rnd = random.Random(1234)
    g = torch.Generator(device=dev).manual_seed(5)
    for _ in range(5):  # test_split_compress
        sizes = []
        for _ in range(rnd.randrange(1, 15)):
            size = rnd.randrange(1, 10000)
            size += 4 - (size % 4)
            sizes.append(size)
        t = torch.randint(0, 65, [sum(sizes)], dtype=torch.uint8, device=dev, generator=g)
        splits = torch.split(t, sizes)
        comp_ts, _, _ = torch.ops.dietgpu.compress_data_split_size(False, t, torch.IntTensor(sizes),
                                                                   True, temp_mem)
        decomp_ts = torch.ops.dietgpu.decompress_data_simple(False, comp_ts, True)
        for orig, decomp in zip(splits, decomp_ts):
            assert torch.equal(orig, decomp)
    for _ in range(5):  # test_split_decompress
        sizes = []
        for _ in range(rnd.randrange(1, 15)):
            size = rnd.randrange(1, 10000)
            size += 4 - (size % 4)
            sizes.append(size)
        t = torch.randint(0, 65, [sum(sizes)], dtype=torch.uint8, device=dev, generator=g)
        comp_ts = torch.ops.dietgpu.compress_data_simple(False, torch.split(t, sizes), True)
        decomp_t = torch.empty([sum(sizes)], dtype=torch.uint8, device=dev)
        torch.ops.dietgpu.decompress_data_split_size(False, comp_ts, decomp_t, torch.IntTensor(sizes),
                                                     True, temp_mem)
        assert torch.equal(t, decomp_t)


@pytest.mark.parametrize("device_ptrs", [False, True])
def test_compressed_info(C, N, ws, device_ptrs):
    """ansGetCompressedInfo{,Device} / floatGetCompressedInfo{,Device}:
    uncompressed size, float type and checksum read from the headers."""
    L = N.lib()
    datas = [exp_bytes(n, lam=10.0, seed=n) for n in (1, 3, 4097, 70000)]
    ts = [torch.from_numpy(d).to(DEV) for d in datas]
    out, osz = C.ans_encode_pointer(ts, checksum=True, ws=ws)
    rows = [out[i] for i in range(len(ts))]
    sizes = torch.zeros([len(ts)], dtype=torch.int32, device=DEV)
    cks = torch.zeros([len(ts)], dtype=torch.int32, device=DEV)
    if device_ptrs:
        ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=DEV)
        N.check(L.dietgpu_ans_get_compressed_info_device(ws.h, ptrs.data_ptr(), len(ts), sizes.data_ptr(),
                                                         cks.data_ptr(), _s()))
    else:
        N.check(L.dietgpu_ans_get_compressed_info(ws.h, N.ptr_array([r.data_ptr() for r in rows]), len(ts),
                                                  sizes.data_ptr(), cks.data_ptr(), _s()))
    assert sizes.cpu().tolist() == [d.size for d in datas]
    assert cks.cpu().tolist() == [int(O.checksum(d)) for d in datas]

    for ft in (1, 2, 3, 4):
        words = [float_words(ft, n, seed=n) for n in (1, 4096, 33333)]
        fts = [torch.from_numpy(w.view(NP_SIGNED[ft]).copy()).to(DEV).view(TORCH_FLOAT[ft])
               for w in words]
        fout, _ = C.float_compress_pointer(fts, checksum=True, ws=ws)
        frows = [fout[i] for i in range(len(fts))]
        sz = torch.zeros([len(fts)], dtype=torch.int32, device=DEV)
        ty = torch.zeros([len(fts)], dtype=torch.int32, device=DEV)
        ck = torch.zeros([len(fts)], dtype=torch.int32, device=DEV)
        if device_ptrs:
            ptrs = torch.tensor([r.data_ptr() for r in frows], dtype=torch.int64, device=DEV)
            N.check(L.dietgpu_float_get_compressed_info_device(ws.h, ptrs.data_ptr(), len(fts), sz.data_ptr(),
                                                               ty.data_ptr(), ck.data_ptr(), _s()))
        else:
            N.check(L.dietgpu_float_get_compressed_info(ws.h, N.ptr_array([r.data_ptr() for r in frows]),
                                                        len(fts), sz.data_ptr(), ty.data_ptr(), ck.data_ptr(),
                                                        _s()))
        assert sz.cpu().tolist() == [w.size for w in words]
        assert ty.cpu().tolist() == [ft] * len(words)
        refs = [O.float_compress(w, ft, 10, True) for w in words]
        assert ck.cpu().tolist() == [int(r[12:16].view(np.uint32)[0]) for r in refs]


def test_fp64_torch_ops(C):
    """fp64 through torch.ops.dietgpu: archives identical to the oracle's,
    decompression into fp64 outputs (an extension over DietGpu.cpp:569-573)."""
    words = [float_words(4, n, seed=n) for n in (1, 4097, 100000)]
    ts = [torch.from_numpy(w.view(np.int64).copy()).to(DEV).view(torch.float64) for w in words]
    comp, sizes, _ = torch.ops.dietgpu.compress_data(True, ts, False)
    sizes = sizes.cpu().tolist()
    host = comp.cpu().numpy()
    for i, w in enumerate(words):
        ref = O.float_compress(w, 4)
        assert sizes[i] == ref.size
        np.testing.assert_array_equal(host[i, :ref.size], ref)
    outs = [torch.empty_like(t) for t in ts]
    torch.ops.dietgpu.decompress_data(True, [comp[i, :sizes[i]] for i in range(len(ts))], outs, False)
    for a, b in zip(ts, outs):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    simple = torch.ops.dietgpu.compress_data_simple(True, ts, True)
    back = torch.ops.dietgpu.decompress_data_simple(True, simple, True)
    for a, b in zip(ts, back):
        assert b.dtype == torch.float64 and torch.equal(a.view(torch.int64), b.view(torch.int64))


def test_forced_wait_timeout_poisons(C, ws):
    """With the poll cap at 0 every cross-workgroup wait that has to wait
    fails: elements of more than one team member (single-pass path) or more
    than one encode workgroup (three-kernel path) must come back with outSize
    0 and be counted, never as a wrong archive; a batch whose elements need
    no wait (one team member each) is unaffected.  The cap is a kernel
    argument (dietgpu_set_spin_cap)."""
    C.device_error_count(reset=True)
    words = [float_words(2, n, seed=n) for n in (524288, 524288, 300000)]
    ts = [torch.from_numpy(w.view(np.int16).copy()).to(DEV).view(torch.bfloat16) for w in words]
    small = [float_words(2, n, seed=n) for n in (3000, 100)]
    sts = [torch.from_numpy(w.view(np.int16).copy()).to(DEV).view(torch.bfloat16) for w in small]
    try:
        C.set_spin_cap(0)
        out, osz = C.float_compress_pointer(ts, ws=ws)
        got = osz.cpu().tolist()
        nerr = C.device_error_count(reset=True)
        sout, sosz = C.float_compress_pointer(sts, ws=ws)
        sgot = sosz.cpu().tolist()
        snerr = C.device_error_count(reset=True)
        # a 1-byte offset input is not 16 B aligned: the three-kernel path
        big = torch.from_numpy(exp_bytes((4 << 20) + 1, lam=10.0, seed=9)).to(DEV)[1:]
        aout, aosz = C.ans_encode_pointer([big], ws=ws)
        agot = aosz.cpu().tolist()
        anerr = C.device_error_count(reset=True)
        # sparse: the dense archive's size writer adds the header + bitmap,
        # so an abandoned element keeps size 0 (not a header-sized stub)
        g = torch.Generator(device=DEV).manual_seed(21)
        sp = []
        for _ in range(2):
            f = torch.randn(600000, generator=g, device=DEV)
            f[torch.rand(f.numel(), generator=g, device=DEV) < 0.5] = 0.0
            sp.append(f)
        _, spsz = C.sparse_compress(sp, ws=ws)
        spgot = spsz.cpu().tolist()
        spnerr = C.device_error_count(reset=True)
        with pytest.raises(RuntimeError):
            torch.ops.dietgpu.compress_data_simple(True, ts[:1], False)
        C.device_error_count(reset=True)
    finally:
        C.set_spin_cap(1 << 24)
    assert got == [0, 0, 0] and nerr == 3
    assert agot == [0] and anerr == 1
    assert spgot == [0, 0] and spnerr == 2
    assert snerr == 0
    for i, w in enumerate(small):
        ref = O.float_compress(w, 2)
        assert sgot[i] == ref.size
        np.testing.assert_array_equal(sout[i, :ref.size].cpu().numpy(), ref)
    # with the default cap the same calls succeed (stale poisoned flags of
    # the failed call belong to an old epoch)
    out, osz = C.float_compress_pointer(ts, ws=ws)
    got = osz.cpu().tolist()
    for i, w in enumerate(words):
        ref = O.float_compress(w, 2)
        assert got[i] == ref.size
        np.testing.assert_array_equal(out[i, :ref.size].cpu().numpy(), ref)
    assert C.device_error_count(reset=True) == 0


def test_graph_capture_replay(C):
    """A compress + decompress captured in a hipGraph and replayed with new
    input data: every replay's archives match the oracle for that data (the
    compressor's flags come from the workspace, zeroed by a captured memset,
    instead of the per-stream epoch arena)."""
    nb, n = 8, 524288
    ws = C.Workspace(256 << 20)
    x = torch.empty([nb, n], dtype=torch.bfloat16, device=DEV)
    cols = C.max_float_compressed_size(2, n)
    arch = torch.empty([nb, cols], dtype=torch.uint8, device=DEV)
    sizes = torch.empty([nb], dtype=torch.int32, device=DEV)
    y = torch.empty_like(x)
    x.copy_(torch.from_numpy(float_words(2, nb * n, seed=1).view(np.int16)).view(nb, n).view(torch.bfloat16))
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):  # warm-up outside the capture
        C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
        C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
    stream.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        C.float_compress_stride(x, ws=ws, out=arch, sizes=sizes)
        C.float_decompress_stride(arch, n, torch.bfloat16, ws=ws, out=y)
    for rep in range(3):
        w = float_words(2, nb * n, seed=100 + rep, scale=1 + rep)
        x.copy_(torch.from_numpy(w.view(np.int16)).view(nb, n).view(torch.bfloat16))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.int16), x.view(torch.int16)), f"replay {rep}"
        got = sizes.cpu().tolist()
        for i in (0, nb - 1):
            ref = O.float_compress(w[i * n:(i + 1) * n], 2)
            assert got[i] == ref.size
            np.testing.assert_array_equal(arch[i, :ref.size].cpu().numpy(), ref)


@pytest.mark.parametrize("path", ["auto", "single-pass", "three-kernel"])
@pytest.mark.parametrize("sizes", [
    [123457], [123457, 1000], [4095, 65536, 1, 300001],
    [1, 7, 4096, 4097, 8191, 32767, 32768, 32769, 100000, 524287, 524288, 1048576],
    [3000] * 300 + [524288], [12345] * 600,
])
def test_single_pass_shapes(C, ws, sizes, path):
    """The persistent single-pass compressor over ragged batches: single
    elements with a partial last item, elements of one item, elements ending
    inside a block pair, batches of many rounds; and the same batches forced
    down the three-kernel path (prologue normalisation, masked partial
    segments) and routed by the size rule; bf16 archives identical to the
    oracle."""
    g = torch.Generator().manual_seed(len(sizes))
    xs = [torch.randn(n, generator=g).to(torch.bfloat16) for n in sizes]
    with C.compress_path(path):
        arch, osz = C.float_compress_pointer([x.to(DEV) for x in xs], ws=ws)
    got = osz.cpu().tolist()
    host = arch.cpu().numpy()
    for i, x in enumerate(xs):
        ref = O.float_compress(x.view(torch.int16).numpy().view(np.uint16), 2)
        assert got[i] == ref.size, (i, sizes[i])
        np.testing.assert_array_equal(host[i, :ref.size], ref, err_msg=f"element {i} n={sizes[i]}")


def test_diff_positive_kat_archive(C, ws):
    """SURVEY Appendix B.2 on the GPU: counts 3 at symbols 200..202 (pb 10);
    the device normalisation gives absent symbol 0 pdf 1 like the oracle, so
    the archives (pdf table included) are identical."""
    d = np.repeat(np.arange(200, 203, dtype=np.uint8), 3)
    out, osz = C.ans_encode_pointer([torch.from_numpy(d).to(DEV)], ws=ws)
    ref = O.ans_encode(d, 10)
    assert osz.cpu().tolist() == [ref.size]
    np.testing.assert_array_equal(out[0, :ref.size].cpu().numpy(), ref)


def test_cpp_api_program():
    """A C++ program written against include/dietgpu/*.h only (no torch),
    linked to libdietgpu_amd.so: pointer and split-size roundtrips of bytes
    and all four float types, sizes and compressed-info readouts."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "dietgpu_fork_amd", "_lib", "api_roundtrip")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
