"""PyTorch-ROCm operator surface: ``torch.ops.dietgpu.*``.

Mirror of the reference's ``TORCH_LIBRARY(dietgpu)`` (dietgpu/DietGpu.cpp:
921-978): the same ten operators with the same schemas, argument meaning,
validation (``TORCH_CHECK`` -> ``RuntimeError``) and return values, running on
the torch current HIP stream.  Each op validates tensors here and calls the
C ABI of libdietgpu_amd.so; all compute is in the HIP kernels.

Extension over the reference: fp64 tensors are accepted on decompression too
(the reference rejects them at DietGpu.cpp:569-573 / 742-746 although its
compressor produces them).
"""
import torch

from . import _native as N

kDefaultPrecision = 10  # DietGpu.cpp:119
kSDMAlignment = 256

_FLOAT_TYPES = {
    torch.float16: 1,
    torch.bfloat16: 2,
    torch.float32: 3,
    torch.float64: 4,
}
_DTYPE_OF = {v: k for k, v in _FLOAT_TYPES.items()}
_UINT32_MAX = 0xFFFFFFFF


def _check(cond, msg="Expected condition to hold"):
    if not cond:
        raise RuntimeError(msg)


def _float_type(t):
    ft = _FLOAT_TYPES.get(t.dtype)
    _check(ft is not None, f"unsupported dtype {t.dtype} for float compression")
    return ft


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _total_and_max(ts):
    """getTotalAndMaxSize, DietGpu.cpp:63-80"""
    total = 0
    mx = 0
    for t in ts:
        n = t.numel()
        _check(n * t.element_size() <= _UINT32_MAX, "tensor too large")
        total += n
        mx = max(mx, n)
    _check(mx <= _UINT32_MAX)
    return total, mx


def _stack_for(dev, temp_mem):
    if temp_mem is not None:
        _check(temp_mem.device.type == "cuda", "temp_mem must be a GPU tensor")
        _check(temp_mem.is_contiguous(), "temp_mem must be contiguous")
        _check(temp_mem.get_device() == dev, "temp_mem must be on the input device")
        nbytes = temp_mem.numel() * temp_mem.element_size()
        return N.Stack(dev, temp_mem.data_ptr() if nbytes else None, nbytes)
    return N.Stack(dev, None, 0)


# ---------------------------------------------------------------- sizes ----

def max_float_compressed_output_size(ts):
    """DietGpu.cpp:128-137 -> (rows, cols)"""
    _, mx = _total_and_max(ts)
    cols = N.size_or_raise(N.lib().dietgpu_get_max_float_compressed_size(_float_type(ts[0]), mx))
    return len(ts), cols


def max_float_compressed_size(dtype, size):
    """DietGpu.cpp:140-142"""
    return N.size_or_raise(N.lib().dietgpu_get_max_float_compressed_size(_float_type(dtype),
                                                                         int(size)))


def max_any_compressed_output_size(ts):
    """DietGpu.cpp:144-150"""
    _, mx = _total_and_max(ts)
    return len(ts), N.size_or_raise(
        N.lib().dietgpu_get_max_compressed_size(mx * ts[0].element_size()))


def max_any_compressed_size(nbytes):
    """DietGpu.cpp:152-154"""
    return N.size_or_raise(N.lib().dietgpu_get_max_compressed_size(int(nbytes)))


# ------------------------------------------------------------- compress ----

def _compress_res(compress_as_float, stack, ts, checksum, out_compressed, out_sizes):
    """compress_data_res, DietGpu.cpp:161-287"""
    _check(len(ts) > 0)
    dev = ts[0].get_device()
    rows, cols = (max_float_compressed_output_size(ts) if compress_as_float
                  else max_any_compressed_output_size(ts))
    for t in ts:
        _check(t.device.type == "cuda", "inputs must be GPU tensors")
        _check(t.is_contiguous(), "inputs must be contiguous")
        _check(t.get_device() == dev, "inputs must be on one device")
        if compress_as_float:
            _check(t.dtype == ts[0].dtype, "float inputs must share a dtype")
            _float_type(t)
    if out_compressed is not None:
        c = out_compressed
        _check(c.dtype == torch.uint8 and c.device.type == "cuda" and c.is_contiguous())
        _check(c.dim() == 2 and c.size(0) >= len(ts) and c.size(1) >= cols)
        _check(c.get_device() == dev)
        comp = c
    else:
        comp = torch.empty([len(ts), cols], dtype=torch.uint8, device=ts[0].device)
    if out_sizes is not None:
        s = out_sizes
        _check(s.dtype == torch.int32 and s.device.type == "cuda" and s.dim() == 1)
        _check(s.is_contiguous() and s.size(0) >= len(ts) and s.get_device() == dev)
        sizes = s
    else:
        sizes = torch.empty([len(ts)], dtype=torch.int32, device=ts[0].device)

    stride = comp.size(1)
    base = comp.data_ptr()
    in_ptrs = N.ptr_array([t.data_ptr() for t in ts])
    in_size = N.u32_array([t.numel() if compress_as_float else t.numel() * t.element_size()
                           for t in ts])
    out_ptrs = N.ptr_array([base + i * stride for i in range(len(ts))])
    L = N.lib()
    with torch.cuda.device(dev):
        if compress_as_float:
            rc = L.dietgpu_float_compress(stack.h, _float_type(ts[0]), kDefaultPrecision,
                                          int(checksum), len(ts), in_ptrs, in_size, out_ptrs,
                                          sizes.data_ptr(), _stream())
        else:
            rc = L.dietgpu_ans_encode_batch_pointer(stack.h, kDefaultPrecision, int(checksum),
                                                    len(ts), in_ptrs, in_size, None, out_ptrs,
                                                    sizes.data_ptr(), _stream())
    N.check(rc)
    return comp, sizes, int(stack.max_usage())


def compress_data(compress_as_float, ts_in, checksum=False, temp_mem=None,
                  out_compressed=None, out_compressed_bytes=None):
    """DietGpu.cpp:289-320"""
    _check(len(ts_in) > 0)
    dev = ts_in[0].get_device()
    stack = _stack_for(dev, temp_mem)
    try:
        return _compress_res(compress_as_float, stack, list(ts_in), checksum, out_compressed,
                             out_compressed_bytes)
    finally:
        stack.close()


def _matrix_to_tensors(n, matrix, sizes):
    """compressedMatrixToTensors, DietGpu.cpp:84-108"""
    host = sizes.to("cpu")
    N.check_archive_sizes(host[:n].tolist())
    flat = matrix.view(-1)
    cols = matrix.size(1)
    return [flat.narrow(0, i * cols, int(host[i])) for i in range(n)]


def compress_data_split_size(compress_as_float, t_in, t_in_split_sizes, checksum=False,
                             temp_mem=None, out_compressed=None, out_compressed_bytes=None):
    """DietGpu.cpp:322-470"""
    dev = t_in.get_device()
    _check(t_in.device.type == "cuda" and t_in.is_contiguous())
    ft = _float_type(t_in) if compress_as_float else 0
    if not compress_as_float:
        _check(t_in.data_ptr() % 4 == 0,
               "All splits should start on a 16 byte boundary; start pointer is not aligned")
    sp = t_in_split_sizes
    _check(sp.is_contiguous() and sp.device.type == "cpu" and sp.dtype == torch.int32)
    n = sp.numel()
    sizes_host = [int(v) for v in sp.tolist()]
    mx = 0
    for i, v in enumerate(sizes_host):
        _check(v > 0, "split sizes must be > 0")
        mx = max(mx, v)
        if not compress_as_float and i != n - 1:
            _check(v % 4 == 0, "All splits should start on a 16 byte boundary; the size of an "
                   "interior split is not a multiple of 16 bytes")
    L = N.lib()
    cols = N.size_or_raise(L.dietgpu_get_max_float_compressed_size(ft, mx) if compress_as_float
                           else L.dietgpu_get_max_compressed_size(mx))
    if out_compressed is not None:
        c = out_compressed
        _check(c.dtype == torch.uint8 and c.device.type == "cuda" and c.is_contiguous())
        _check(c.dim() == 2 and c.size(0) >= n and c.size(1) >= cols and c.get_device() == dev)
        comp = c
    else:
        comp = torch.empty([n, cols], dtype=torch.uint8, device=t_in.device)
    if out_compressed_bytes is not None:
        s = out_compressed_bytes
        _check(s.dtype == torch.int32 and s.device.type == "cuda" and s.dim() == 1)
        _check(s.is_contiguous() and s.size(0) >= n and s.get_device() == dev)
        sizes = s
    else:
        sizes = torch.empty([n], dtype=torch.int32, device=t_in.device)
    stack = _stack_for(dev, temp_mem)
    try:
        split = N.u32_array(sizes_host)
        with torch.cuda.device(dev):
            if compress_as_float:
                rc = L.dietgpu_float_compress_split_size(
                    stack.h, ft, kDefaultPrecision, int(checksum), n, t_in.data_ptr(), split,
                    comp.data_ptr(), comp.size(1), sizes.data_ptr(), _stream())
            else:
                rc = L.dietgpu_ans_encode_batch_split_size(
                    stack.h, kDefaultPrecision, int(checksum), n, t_in.data_ptr(), split, None,
                    comp.data_ptr(), comp.size(1), sizes.data_ptr(), _stream())
        N.check(rc)
        lst = _matrix_to_tensors(n, comp, sizes)
        return lst, sizes, int(stack.max_usage())
    finally:
        stack.close()


def compress_data_simple(compress_as_float, ts_in, checksum=False, temp_mem=67108864):
    """DietGpu.cpp:472-526"""
    _check(len(ts_in) > 0)
    scratch = None
    if temp_mem is not None and temp_mem > 0:
        scratch = torch.empty([int(temp_mem)], dtype=torch.uint8, device=ts_in[0].device)
    comp, sizes, _ = compress_data(compress_as_float, ts_in, checksum, scratch)
    host = sizes.to("cpu")
    _check(host.size(0) == len(ts_in))
    N.check_archive_sizes(host.tolist())
    cols = comp.size(1)
    flat = comp.view(-1)
    return [flat.narrow(0, i * cols, int(host[i])).clone() for i in range(len(ts_in))]


# ----------------------------------------------------------- decompress ----

def _check_out_dtype(t):
    _check(t.dtype in _FLOAT_TYPES, "float outputs must be float16, bfloat16, float32 or "
           "float64")


def _decompress_res(compress_as_float, stack, ts_in, ts_out, checksum, out_status, out_sizes):
    """decompress_data_res, DietGpu.cpp:536-650"""
    _check(len(ts_in) > 0 and len(ts_in) == len(ts_out))
    dev = ts_in[0].get_device()
    caps = []
    for ti, to in zip(ts_in, ts_out):
        _check(ti.device.type == "cuda" and ti.get_device() == dev and ti.is_contiguous())
        _check(to.device.type == "cuda" and to.get_device() == dev and to.is_contiguous())
        _check(ti.dtype == torch.uint8, "compressed inputs must be uint8")
        if compress_as_float:
            _check_out_dtype(to)
        cap = to.numel() if compress_as_float else to.numel() * to.element_size()
        _check(cap <= _UINT32_MAX)
        caps.append(cap)
    for t, dt in ((out_status, torch.uint8), (out_sizes, torch.int32)):
        if t is not None:
            _check(t.is_contiguous() and t.device.type == "cuda" and t.dtype == dt)
            _check(t.numel() == len(ts_in) and t.get_device() == dev)
    L = N.lib()
    in_ptrs = N.ptr_array([t.data_ptr() for t in ts_in])
    out_ptrs = N.ptr_array([t.data_ptr() for t in ts_out])
    cap = N.u32_array(caps)
    st = out_status.data_ptr() if out_status is not None else None
    sz = out_sizes.data_ptr() if out_sizes is not None else None
    with torch.cuda.device(dev):
        if compress_as_float:
            rc = L.dietgpu_float_decompress(stack.h, _float_type(ts_out[0]), kDefaultPrecision,
                                            int(checksum), len(ts_in), in_ptrs, out_ptrs, cap, st,
                                            sz, _stream())
            if rc == N.DIETGPU_ERR_CHECKSUM:
                raise RuntimeError("floatDecompress: checksum mismatch seen on decoded data; "
                                   "archive cannot be unpacked")
        else:
            rc = L.dietgpu_ans_decode_batch_pointer(stack.h, kDefaultPrecision, int(checksum),
                                                    len(ts_in), in_ptrs, out_ptrs, cap, st, sz,
                                                    _stream())
            if rc == N.DIETGPU_ERR_CHECKSUM:
                raise RuntimeError("ANSDecode: checksum mismatch seen on decoded data; "
                                   "archive cannot be unpacked")
    N.check(rc)
    return int(stack.max_usage())


def decompress_data(compress_as_float, ts_in, ts_out, checksum=False, temp_mem=None,
                    out_status=None, out_decompressed_words=None):
    """DietGpu.cpp:652-683"""
    _check(len(ts_in) > 0)
    dev = ts_in[0].get_device()
    stack = _stack_for(dev, temp_mem)
    try:
        return _decompress_res(compress_as_float, stack, list(ts_in), list(ts_out), checksum,
                               out_status, out_decompressed_words)
    finally:
        stack.close()


def decompress_data_split_size(compress_as_float, ts_in, t_out, t_out_split_sizes,
                               checksum=False, temp_mem=None, out_status=None,
                               out_decompressed_words=None):
    """DietGpu.cpp:685-832"""
    _check(len(ts_in) > 0)
    dev = ts_in[0].get_device()
    sp = t_out_split_sizes
    _check(sp.is_contiguous() and sp.device.type == "cpu" and sp.dtype == torch.int32)
    n = sp.numel()
    _check(n == len(ts_in), "one split size per compressed input")
    split = [int(v) for v in sp.tolist()]
    for ti, v in zip(ts_in, split):
        _check(ti.device.type == "cuda" and ti.get_device() == dev and ti.is_contiguous())
        _check(ti.dtype == torch.uint8)
        _check(v > 0, "split sizes must be > 0")
    _check(t_out.device.type == "cuda" and t_out.get_device() == dev and t_out.is_contiguous())
    if compress_as_float:
        _check_out_dtype(t_out)
    for t, dt in ((out_status, torch.uint8), (out_decompressed_words, torch.int32)):
        if t is not None:
            _check(t.is_contiguous() and t.device.type == "cuda" and t.dtype == dt)
            _check(t.numel() == n and t.get_device() == dev)
    L = N.lib()
    stack = _stack_for(dev, temp_mem)
    try:
        in_ptrs = N.ptr_array([t.data_ptr() for t in ts_in])
        sps = N.u32_array(split)
        st = out_status.data_ptr() if out_status is not None else None
        sz = out_decompressed_words.data_ptr() if out_decompressed_words is not None else None
        with torch.cuda.device(dev):
            if compress_as_float:
                rc = L.dietgpu_float_decompress_split_size(
                    stack.h, _float_type(t_out), kDefaultPrecision, int(checksum), n, in_ptrs,
                    t_out.data_ptr(), sps, st, sz, _stream())
                if rc == N.DIETGPU_ERR_CHECKSUM:
                    raise RuntimeError("floatDecompress: checksum mismatch seen on decoded "
                                       "data; archive cannot be unpacked")
            else:
                rc = L.dietgpu_ans_decode_batch_split_size(
                    stack.h, kDefaultPrecision, int(checksum), n, in_ptrs, t_out.data_ptr(), sps,
                    st, sz, _stream())
                if rc == N.DIETGPU_ERR_CHECKSUM:
                    raise RuntimeError("ANSDecode: checksum mismatch seen on decoded data; "
                                       "archive cannot be unpacked")
        N.check(rc)
        return int(stack.max_usage())
    finally:
        stack.close()


def decompress_data_simple(compress_as_float, ts_in, checksum=False, temp_mem=67108864):
    """DietGpu.cpp:834-917"""
    _check(len(ts_in) > 0)
    dev = ts_in[0].get_device()
    for t in ts_in:
        _check(t.device.type == "cuda" and t.get_device() == dev and t.is_contiguous())
    scratch = None
    if temp_mem is not None and temp_mem >= kSDMAlignment:
        scratch = torch.empty([int(temp_mem)], dtype=torch.uint8, device=ts_in[0].device)
    n = len(ts_in)
    info = torch.zeros([2, n], dtype=torch.int32, device=ts_in[0].device)
    stack = _stack_for(dev, scratch)
    try:
        L = N.lib()
        in_ptrs = N.ptr_array([t.data_ptr() for t in ts_in])
        with torch.cuda.device(dev):
            if compress_as_float:
                rc = L.dietgpu_float_get_compressed_info(stack.h, in_ptrs, n, info[0].data_ptr(),
                                                         info[1].data_ptr(), None, _stream())
            else:
                rc = L.dietgpu_ans_get_compressed_info(stack.h, in_ptrs, n, info[0].data_ptr(),
                                                       None, _stream())
        N.check(rc)
        host = info.to("cpu").tolist()
        outs = []
        for i in range(n):
            size, ty = host[0][i], host[1][i]
            if compress_as_float:
                _check(ty == host[1][0], "all archives must have the same float type")
                _check(ty in _DTYPE_OF, "not a float archive")
                outs.append(torch.empty([size], dtype=_DTYPE_OF[ty], device=ts_in[0].device))
            else:
                outs.append(torch.empty([size], dtype=torch.uint8, device=ts_in[0].device))
        _decompress_res(compress_as_float, stack, list(ts_in), outs, checksum, None, None)
        return outs
    finally:
        stack.close()


# ------------------------------------------------------ torch.ops.dietgpu ----

SCHEMAS = {
    "max_float_compressed_output_size": "(Tensor[] ts) -> (int, int)",
    "max_float_compressed_size": "(Tensor dtype, int size) -> int",
    "max_any_compressed_output_size": "(Tensor[] ts) -> (int, int)",
    "max_any_compressed_size": "(int bytes) -> int",
    "compress_data": "(bool compress_as_float, Tensor[] ts_in, bool checksum=False, "
                     "Tensor? temp_mem=None, Tensor? out_compressed=None, "
                     "Tensor? out_compressed_bytes=None) -> (Tensor, Tensor, int)",
    "compress_data_split_size": "(bool compress_as_float, Tensor t_in, Tensor t_in_split_sizes, "
                                "bool checksum=False, Tensor? temp_mem=None, "
                                "Tensor? out_compressed=None, Tensor? out_compressed_bytes=None)"
                                " -> (Tensor[], Tensor, int)",
    "compress_data_simple": "(bool compress_as_float, Tensor[] ts_in, bool checksum=False, "
                            "int? temp_mem=67108864) -> Tensor[]",
    "decompress_data": "(bool compress_as_float, Tensor[] ts_in, Tensor[] ts_out, "
                       "bool checksum=False, Tensor? temp_mem=None, Tensor? out_status=None, "
                       "Tensor? out_decompressed_words=None) -> (int)",
    "decompress_data_split_size": "(bool compress_as_float, Tensor[] ts_in, Tensor t_out, "
                                  "Tensor t_out_split_sizes, bool checksum=False, "
                                  "Tensor? temp_mem=None, Tensor? out_status=None, "
                                  "Tensor? out_decompressed_words=None) -> (int)",
    "decompress_data_simple": "(bool compress_as_float, Tensor[] ts_in, bool checksum=False, "
                              "int? temp_mem=67108864) -> Tensor[]",
}

_IMPLS = {
    "max_float_compressed_output_size": max_float_compressed_output_size,
    "max_float_compressed_size": max_float_compressed_size,
    "max_any_compressed_output_size": max_any_compressed_output_size,
    "max_any_compressed_size": max_any_compressed_size,
    "compress_data": compress_data,
    "compress_data_split_size": compress_data_split_size,
    "compress_data_simple": compress_data_simple,
    "decompress_data": decompress_data,
    "decompress_data_split_size": decompress_data_split_size,
    "decompress_data_simple": decompress_data_simple,
}

_LIB = None


def register():
    """Define TORCH_LIBRARY(dietgpu) (idempotent).  After this, the reference's
    harness code (``torch.ops.dietgpu.compress_data(...)``) runs unchanged."""
    global _LIB
    if _LIB is not None:
        return
    N.lib()  # fail loudly if the HIP library is missing
    lib = torch.library.Library("dietgpu", "DEF")
    for name, schema in SCHEMAS.items():
        lib.define(name + schema)
        lib.impl(name, _IMPLS[name], "CompositeExplicitAutograd")
    _LIB = lib
