"""ctypes binding of the CPU restatement (oracle/dietgpu_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the dietgpu_fork_amd package.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdietgpu_oracle.so")
_lib = None

FLOAT_TYPES = {"float16": 1, "bfloat16": 2, "float32": 3, "float64": 4}
WORD_SIZE = {1: 2, 2: 2, 3: 4, 4: 8}


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32, u64, i32, sz, vp = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.c_size_t, ctypes.c_void_p)
        P32 = ctypes.POINTER(ctypes.c_uint32)
        L.or_max_compressed_size.restype = u32
        L.or_max_compressed_size.argtypes = [u32]
        L.or_max_float_compressed_size.restype = u32
        L.or_max_float_compressed_size.argtypes = [i32, u32]
        L.or_max_sparse_float_compressed_size.restype = u32
        L.or_max_sparse_float_compressed_size.argtypes = [i32, u32]
        L.or_float_uncomp_data_size.restype = u32
        L.or_float_uncomp_data_size.argtypes = [i32, u32]
        L.or_ans_histogram.argtypes = [vp, sz, vp]
        L.or_ans_normalize.restype = i32
        L.or_ans_normalize.argtypes = [vp, u32, i32, vp, vp]
        L.or_checksum.restype = u32
        L.or_checksum.argtypes = [vp, sz]
        L.or_ans_encode.restype = u32
        L.or_ans_encode.argtypes = [vp, u32, i32, i32, vp, vp, sz]
        L.or_ans_decode.restype = i32
        L.or_ans_decode.argtypes = [vp, i32, i32, vp, u32, P32]
        L.or_ans_info.restype = u32
        L.or_ans_info.argtypes = [vp, P32]
        L.or_ans_archive_size.restype = u32
        L.or_ans_archive_size.argtypes = [vp]
        L.or_float_compress.restype = u32
        L.or_float_compress.argtypes = [i32, vp, u32, i32, i32, vp, sz]
        L.or_float_decompress.restype = i32
        L.or_float_decompress.argtypes = [vp, i32, i32, i32, vp, u32, P32]
        L.or_sparse_float_compress.restype = u32
        L.or_sparse_float_compress.argtypes = [i32, vp, u32, i32, i32, vp, sz]
        L.or_sparse_float_decompress.restype = i32
        L.or_sparse_float_decompress.argtypes = [vp, i32, i32, i32, vp, u32, P32]
        dp = ctypes.POINTER(ctypes.c_double)
        L.or_time_float_roundtrip.restype = ctypes.c_double
        L.or_time_float_roundtrip.argtypes = [i32, vp, u32, u32, sz, i32, i32,
                                              ctypes.POINTER(u64), dp, dp]
        L.or_time_ans_roundtrip.restype = ctypes.c_double
        L.or_time_ans_roundtrip.argtypes = [vp, u32, u32, sz, i32, i32,
                                            ctypes.POINTER(u64), dp, dp]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def max_compressed_size(nbytes):
    return lib().or_max_compressed_size(nbytes)


def max_float_compressed_size(ft, n):
    return lib().or_max_float_compressed_size(ft, n)


def max_sparse_float_compressed_size(ft, n):
    return lib().or_max_sparse_float_compressed_size(ft, n)


def histogram(data):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    h = np.zeros(256, dtype=np.uint32)
    lib().or_ans_histogram(_ptr(data), data.size, _ptr(h))
    return h


def normalize(hist, total, prob_bits):
    hist = np.ascontiguousarray(hist, dtype=np.uint32)
    pdf = np.zeros(256, dtype=np.uint32)
    cdf = np.zeros(256, dtype=np.uint32)
    rc = lib().or_ans_normalize(_ptr(hist), total, prob_bits, _ptr(pdf), _ptr(cdf))
    assert rc == 0
    return pdf, cdf


def checksum(data):
    data = np.ascontiguousarray(data).view(np.uint8).ravel()
    return lib().or_checksum(_ptr(data), data.size)


def ans_encode(data, prob_bits=10, checksum=False, hist=None):
    data = np.ascontiguousarray(data).view(np.uint8).ravel()
    cap = max(max_compressed_size(data.size), 1 << 16) + 64 * 1024
    out = np.zeros(cap, dtype=np.uint8)
    h = None if hist is None else _ptr(np.ascontiguousarray(hist, dtype=np.uint32))
    n = lib().or_ans_encode(_ptr(data), data.size, prob_bits, int(checksum), h,
                            _ptr(out), cap)
    assert n > 0, "oracle encode failed"
    return out[:n].copy()


def ans_decode(archive, prob_bits=10, checksum=False, capacity=None):
    archive = np.ascontiguousarray(archive, dtype=np.uint8)
    size = lib().or_ans_info(_ptr(archive), None)
    cap = size if capacity is None else capacity
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    got = ctypes.c_uint32(0)
    st = lib().or_ans_decode(_ptr(archive), prob_bits, int(checksum), _ptr(out), cap,
                             ctypes.byref(got))
    return st, out[: got.value] if st == 0 else out


def float_compress(words, ft, prob_bits=10, checksum=False):
    words = np.ascontiguousarray(words)
    n = words.size
    cap = max_float_compressed_size(ft, n) + 64
    out = np.zeros(cap, dtype=np.uint8)
    sz = lib().or_float_compress(ft, _ptr(words), n, prob_bits, int(checksum),
                                 _ptr(out), cap)
    assert sz > 0, "oracle float compress failed"
    return out[:sz].copy()


_NP_WORD = {1: np.uint16, 2: np.uint16, 3: np.uint32, 4: np.uint64}


def float_decompress(archive, ft, prob_bits=10, checksum=False, capacity=None):
    archive = np.ascontiguousarray(archive, dtype=np.uint8)
    n = int(archive[4:8].view(np.uint32)[0])
    cap = n if capacity is None else capacity
    out = np.zeros(max(cap, 1), dtype=_NP_WORD[ft])
    got = ctypes.c_uint32(0)
    st = lib().or_float_decompress(_ptr(archive), ft, prob_bits, int(checksum),
                                   _ptr(out), cap, ctypes.byref(got))
    return st, out[: got.value]


def sparse_compress(words, ft, prob_bits=10, checksum=False):
    words = np.ascontiguousarray(words)
    n = words.size
    cap = max_sparse_float_compressed_size(ft, n) + 64
    out = np.zeros(cap, dtype=np.uint8)
    sz = lib().or_sparse_float_compress(ft, _ptr(words), n, prob_bits, int(checksum),
                                        _ptr(out), cap)
    assert sz > 0, "oracle sparse compress failed"
    return out[:sz].copy()


def sparse_decompress(archive, ft, prob_bits=10, checksum=False, capacity=None):
    archive = np.ascontiguousarray(archive, dtype=np.uint8)
    n = int(archive[0:4].view(np.uint32)[0])
    cap = n if capacity is None else capacity
    out = np.zeros(max(cap, 1), dtype=_NP_WORD[ft])
    got = ctypes.c_uint32(0)
    st = lib().or_sparse_float_decompress(_ptr(archive), ft, prob_bits, int(checksum),
                                          _ptr(out), cap, ctypes.byref(got))
    return st, out[: got.value]


def time_float_roundtrip(words2d, ft, prob_bits=10, threads=1):
    """Serial (threads=1) CPU compress+decompress of a [nb, n] word matrix."""
    words2d = np.ascontiguousarray(words2d)
    nb, n = words2d.shape
    comp = ctypes.c_uint64(0)
    e = ctypes.c_double(0)
    d = ctypes.c_double(0)
    t = lib().or_time_float_roundtrip(ft, _ptr(words2d), nb, n, words2d.strides[0],
                                      prob_bits, threads, ctypes.byref(comp),
                                      ctypes.byref(e), ctypes.byref(d))
    return t, comp.value, e.value, d.value


def time_ans_roundtrip(bytes2d, prob_bits=10, threads=1):
    bytes2d = np.ascontiguousarray(bytes2d, dtype=np.uint8)
    nb, n = bytes2d.shape
    comp = ctypes.c_uint64(0)
    e = ctypes.c_double(0)
    d = ctypes.c_double(0)
    t = lib().or_time_ans_roundtrip(_ptr(bytes2d), nb, n, bytes2d.strides[0], prob_bits,
                                    threads, ctypes.byref(comp), ctypes.byref(e),
                                    ctypes.byref(d))
    return t, comp.value, e.value, d.value
