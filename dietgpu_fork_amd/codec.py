"""Tensor-level wrappers of the C ABI (stride / pointer / split / sparse entry
points), used by tests and bench.py.  Every function runs the HIP kernels on
the torch current stream and returns device tensors; nothing here computes on
the CPU.
"""
import contextlib

import torch

from . import _native as N

FLOAT_TYPE = {torch.float16: 1, torch.bfloat16: 2, torch.float32: 3, torch.float64: 4}
WORD_DTYPE = {1: torch.int16, 2: torch.int16, 3: torch.int32, 4: torch.int64}


def _s():
    return torch.cuda.current_stream().cuda_stream


class Workspace:
    """A StackDeviceMemory over a torch uint8 buffer (reused across calls)."""

    def __init__(self, nbytes, device="cuda"):
        self.buf = torch.empty([max(int(nbytes), 256)], dtype=torch.uint8, device=device)
        self.stack = N.Stack(self.buf.get_device(), self.buf.data_ptr(), self.buf.numel())

    def max_usage(self):
        return self.stack.max_usage()

    @property
    def h(self):
        return self.stack.h


def _ws(ws, device):
    return ws if ws is not None else Workspace(256, device)


def test_histogram(x2d, size=None, ws=None):
    """Test hook (libdietgpu_testhooks.so): per-row byte histograms of a [nb, stride] uint8 CUDA tensor
    (the first `size` bytes of each row) by the compressor's histogram kernel."""
    nb, stride = x2d.shape
    size = stride if size is None else size
    hist = torch.empty([nb, 256], dtype=torch.int32, device=x2d.device)
    ws = _ws(ws, x2d.device)
    N.test_check(N.testlib().dietgpu_test_histogram(ws.h, nb, x2d.data_ptr(), size, stride, hist.data_ptr(), _s()))
    return hist


def test_enc_magic(device="cuda"):
    """Test hook (libdietgpu_testhooks.so): the compressors' in-register
    division magic of every pdf 0 .. 2048, as an int64 CPU tensor."""
    m = torch.empty([(1 << 11) + 1], dtype=torch.int32, device=device)
    N.test_check(N.testlib().dietgpu_test_enc_magic(m.data_ptr(), _s()))
    return m.cpu().to(torch.int64) & 0xffffffff


def max_compressed_size(nbytes):
    return N.size_or_raise(N.lib().dietgpu_get_max_compressed_size(int(nbytes)))


def max_float_compressed_size(ft, words):
    return N.size_or_raise(N.lib().dietgpu_get_max_float_compressed_size(int(ft), int(words)))


def max_sparse_float_compressed_size(ft, words):
    return N.size_or_raise(N.lib().dietgpu_get_max_sparse_float_compressed_size(int(ft),
                                                                                 int(words)))


def device_error_count(reset=True):
    """Elements the compressor abandoned (outSize 0) since the last reset;
    synchronises the device."""
    return int(N.lib().dietgpu_device_error_count(int(reset)))


def barrier_fallback_count(reset=True):
    """Single-pass compressor team-barrier fallbacks (a workgroup that counted
    its element from the input after waiting out the barrier budget; the
    archive is unchanged) since the last reset; synchronises the device."""
    return int(N.lib().dietgpu_barrier_fallback_count(int(reset)))


def set_dispatch_skew(ticks):
    """Test hook: emulate out-of-order workgroup dispatch (0 = off)."""
    N.lib().dietgpu_set_dispatch_skew(int(ticks))


def set_spin_cap(polls):
    """Test hook: polls per cross-workgroup wait of the compressor (default
    1 << 24; 0 makes every wait that has to wait fail)."""
    N.lib().dietgpu_set_spin_cap(int(polls))


def set_barrier_budget(ticks):
    """Test hook: 100 MHz ticks a single-pass compressor workgroup waits for
    its team before counting the element itself (default 20000; 0 forces the
    fallback on every team wait)."""
    N.lib().dietgpu_set_barrier_budget(int(ticks))


_PATHS = {"auto": 0, "single-pass": 1, "three-kernel": 2}


def set_compress_path(mode):
    """Test hook: "auto" (default: the size rule), "single-pass" (k_pcompress
    whenever the batch is eligible) or "three-kernel" (always k_hist ->
    k_encode).  Archives are identical whatever the mode."""
    N.lib().dietgpu_set_compress_path(_PATHS[mode])


@contextlib.contextmanager
def compress_path(mode):
    """set_compress_path(mode) for the body, "auto" after it."""
    set_compress_path(mode)
    try:
        yield
    finally:
        set_compress_path("auto")


# ------------------------------------------------------------------ ANS ----

def ans_encode_stride(data2d, prob_bits=10, checksum=False, ws=None, histogram=None,
                      out=None, sizes=None):
    """data2d: [nb, n] uint8 CUDA tensor -> (archives [nb, maxComp] uint8, sizes int32)"""
    nb, n = data2d.shape
    cols = max_compressed_size(n)
    out = out if out is not None else torch.empty([nb, cols], dtype=torch.uint8,
                                                  device=data2d.device)
    sizes = sizes if sizes is not None else torch.empty([nb], dtype=torch.int32,
                                                        device=data2d.device)
    ws = _ws(ws, data2d.device)
    rc = N.lib().dietgpu_ans_encode_batch_stride(
        ws.h, prob_bits, int(checksum), nb, data2d.data_ptr(), n, data2d.stride(0),
        histogram.data_ptr() if histogram is not None else None, out.data_ptr(), out.stride(0),
        sizes.data_ptr(), _s())
    N.check(rc)
    return out, sizes


def ans_decode_stride(archives2d, n, prob_bits=10, checksum=False, ws=None, out=None,
                      capacity=None):
    nb = archives2d.shape[0]
    cap = n if capacity is None else capacity
    out = out if out is not None else torch.empty([nb, max(cap, 1)], dtype=torch.uint8,
                                                  device=archives2d.device)
    ok = torch.empty([nb], dtype=torch.uint8, device=archives2d.device)
    sz = torch.empty([nb], dtype=torch.int32, device=archives2d.device)
    ws = _ws(ws, archives2d.device)
    rc = N.lib().dietgpu_ans_decode_batch_stride(
        ws.h, prob_bits, int(checksum), nb, archives2d.data_ptr(), archives2d.stride(0),
        out.data_ptr(), out.stride(0), cap, ok.data_ptr(), sz.data_ptr(), _s())
    N.check(rc)
    return out, ok, sz


def ans_encode_pointer(ts, prob_bits=10, checksum=False, ws=None):
    """ts: list of uint8 CUDA tensors -> (list of archive rows, sizes)"""
    nb = len(ts)
    dev = ts[0].device
    cols = max_compressed_size(max(t.numel() for t in ts))
    out = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
    sizes = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = _ws(ws, dev)
    rc = N.lib().dietgpu_ans_encode_batch_pointer(
        ws.h, prob_bits, int(checksum), nb, N.ptr_array([t.data_ptr() for t in ts]),
        N.u32_array([t.numel() for t in ts]), None,
        N.ptr_array([out.data_ptr() + i * cols for i in range(nb)]), sizes.data_ptr(), _s())
    N.check(rc)
    return out, sizes


def ans_decode_pointer(archives, outs, prob_bits=10, checksum=False, ws=None):
    nb = len(archives)
    dev = archives[0].device
    ok = torch.empty([nb], dtype=torch.uint8, device=dev)
    sz = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = _ws(ws, dev)
    rc = N.lib().dietgpu_ans_decode_batch_pointer(
        ws.h, prob_bits, int(checksum), nb, N.ptr_array([a.data_ptr() for a in archives]),
        N.ptr_array([o.data_ptr() for o in outs]), N.u32_array([o.numel() for o in outs]),
        ok.data_ptr(), sz.data_ptr(), _s())
    N.check(rc)
    return ok, sz


# ---------------------------------------------------------------- float ----

def float_compress_stride(x2d, ft=None, prob_bits=10, checksum=False, ws=None, out=None,
                          sizes=None):
    """x2d: [nb, n] float CUDA tensor (or int16/32/64 words with ft given)."""
    ft = ft or FLOAT_TYPE[x2d.dtype]
    nb, n = x2d.shape
    cols = max_float_compressed_size(ft, n)
    out = out if out is not None else torch.empty([nb, cols], dtype=torch.uint8,
                                                  device=x2d.device)
    sizes = sizes if sizes is not None else torch.empty([nb], dtype=torch.int32,
                                                        device=x2d.device)
    ws = _ws(ws, x2d.device)
    rc = N.lib().dietgpu_float_compress_batch_stride(
        ws.h, ft, prob_bits, int(checksum), nb, x2d.data_ptr(), n,
        x2d.stride(0) * x2d.element_size(), out.data_ptr(), out.stride(0), sizes.data_ptr(),
        _s())
    N.check(rc)
    return out, sizes


def float_decompress_stride(archives2d, n, dtype, prob_bits=10, checksum=False, ws=None,
                            out=None, capacity=None):
    ft = FLOAT_TYPE[dtype] if dtype in FLOAT_TYPE else None
    nb = archives2d.shape[0]
    cap = n if capacity is None else capacity
    out = out if out is not None else torch.empty([nb, max(cap, 1)], dtype=dtype,
                                                  device=archives2d.device)
    ft = ft or {2: 2, 4: 3, 8: 4}[out.element_size()]
    ok = torch.empty([nb], dtype=torch.uint8, device=archives2d.device)
    sz = torch.empty([nb], dtype=torch.int32, device=archives2d.device)
    ws = _ws(ws, archives2d.device)
    rc = N.lib().dietgpu_float_decompress_batch_stride(
        ws.h, ft, prob_bits, int(checksum), nb, archives2d.data_ptr(), archives2d.stride(0),
        out.data_ptr(), out.stride(0) * out.element_size(), cap, ok.data_ptr(), sz.data_ptr(),
        _s())
    N.check(rc)
    return out, ok, sz


def float_compress_pointer(ts, ft=None, prob_bits=10, checksum=False, ws=None):
    ft = ft or FLOAT_TYPE[ts[0].dtype]
    nb = len(ts)
    dev = ts[0].device
    cols = max_float_compressed_size(ft, max(t.numel() for t in ts))
    out = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
    sizes = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = _ws(ws, dev)
    rc = N.lib().dietgpu_float_compress(
        ws.h, ft, prob_bits, int(checksum), nb, N.ptr_array([t.data_ptr() for t in ts]),
        N.u32_array([t.numel() for t in ts]),
        N.ptr_array([out.data_ptr() + i * cols for i in range(nb)]), sizes.data_ptr(), _s())
    N.check(rc)
    return out, sizes


def float_decompress_pointer(archives, outs, ft=None, prob_bits=10, checksum=False, ws=None):
    ft = ft or FLOAT_TYPE[outs[0].dtype]
    nb = len(archives)
    dev = archives[0].device
    ok = torch.empty([nb], dtype=torch.uint8, device=dev)
    sz = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = _ws(ws, dev)
    rc = N.lib().dietgpu_float_decompress(
        ws.h, ft, prob_bits, int(checksum), nb, N.ptr_array([a.data_ptr() for a in archives]),
        N.ptr_array([o.data_ptr() for o in outs]), N.u32_array([o.numel() for o in outs]),
        ok.data_ptr(), sz.data_ptr(), _s())
    N.check(rc)
    return ok, sz


def sparse_compress(ts, ft=None, prob_bits=10, checksum=False, ws=None):
    ft = ft or FLOAT_TYPE[ts[0].dtype]
    nb = len(ts)
    dev = ts[0].device
    cols = max_sparse_float_compressed_size(ft, max(t.numel() for t in ts))
    out = torch.empty([nb, cols], dtype=torch.uint8, device=dev)
    sizes = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = _ws(ws, dev)
    rc = N.lib().dietgpu_float_compress_sparse(
        ws.h, ft, prob_bits, int(checksum), nb, N.ptr_array([t.data_ptr() for t in ts]),
        N.u32_array([t.numel() for t in ts]),
        N.ptr_array([out.data_ptr() + i * cols for i in range(nb)]), sizes.data_ptr(), _s())
    N.check(rc)
    return out, sizes


def sparse_decompress(archives, outs, ft=None, prob_bits=10, checksum=False, ws=None):
    ft = ft or FLOAT_TYPE[outs[0].dtype]
    nb = len(archives)
    dev = archives[0].device
    ok = torch.empty([nb], dtype=torch.uint8, device=dev)
    sz = torch.empty([nb], dtype=torch.int32, device=dev)
    ws = _ws(ws, dev)
    rc = N.lib().dietgpu_float_decompress_sparse(
        ws.h, ft, prob_bits, int(checksum), nb, N.ptr_array([a.data_ptr() for a in archives]),
        N.ptr_array([o.data_ptr() for o in outs]), N.u32_array([o.numel() for o in outs]),
        ok.data_ptr(), sz.data_ptr(), _s())
    N.check(rc)
    return ok, sz


def profile(on=True):
    N.lib().dietgpu_profile_enable(int(on))


def profile_filter(family=None):
    """Record only `family` (None = all families)."""
    N.lib().dietgpu_profile_filter(family.encode() if family else None)


def profile_reset():
    N.lib().dietgpu_profile_reset()


def profile_query(family):
    import ctypes

    ms = ctypes.c_double(0)
    n = ctypes.c_uint64(0)
    N.lib().dietgpu_profile_query(family.encode(), ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value
