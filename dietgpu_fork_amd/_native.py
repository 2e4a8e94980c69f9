"""ctypes binding of libdietgpu_amd.so (the C ABI in include/dietgpu_c.h).

The HIP library is the only compute path: if it is missing this module raises
at import time -- there is no CPU fallback.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libdietgpu_amd.so")
CSRC = os.path.join(_HERE, "csrc")

DIETGPU_OK = 0
DIETGPU_ERR_INVALID = 1
DIETGPU_ERR_HIP = 2
DIETGPU_ERR_CHECKSUM = 3


class DietGpuError(RuntimeError):
    pass


class ChecksumMismatch(DietGpuError):
    pass


def build(jobs=8):
    """Compile the HIP library for gfx950 in-tree (hipcc; no GPU needed)."""
    subprocess.check_call(["make", "-s", f"-j{jobs}", "-C", CSRC])


def _declare(L):
    c_u32, c_u64, c_int, c_size, vp = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int,
                                       ctypes.c_size_t, ctypes.c_void_p)
    P = ctypes.c_void_p  # all device / host pointers passed as void*
    sig = {
        "dietgpu_last_error": (ctypes.c_char_p, []),
        "dietgpu_device_error_count": (c_u32, [c_int]),
        "dietgpu_barrier_fallback_count": (c_u32, [c_int]),
        "dietgpu_set_spin_cap": (None, [c_u32]),
        "dietgpu_set_barrier_budget": (None, [c_u32]),
        "dietgpu_set_dispatch_skew": (None, [c_u32]),
        "dietgpu_set_compress_path": (None, [c_int]),
        "dietgpu_version": (ctypes.c_char_p, []),
        "dietgpu_stack_create": (vp, [c_int, P, c_size]),
        "dietgpu_stack_destroy": (None, [vp]),
        "dietgpu_stack_max_usage": (c_size, [vp]),
        "dietgpu_stack_reset_max_usage": (None, [vp]),
        "dietgpu_stack_size_total": (c_size, [vp]),
        "dietgpu_get_max_compressed_size": (c_u32, [c_u32]),
        "dietgpu_get_max_float_compressed_size": (c_u32, [c_int, c_u32]),
        "dietgpu_get_max_sparse_float_compressed_size": (c_u32, [c_int, c_u32]),
        "dietgpu_ans_encode_batch_stride": (c_int, [vp, c_int, c_int, c_u32, P, c_u32, c_u32, P,
                                                    P, c_u32, P, P]),
        "dietgpu_ans_encode_batch_pointer": (c_int, [vp, c_int, c_int, c_u32, P, P, P, P, P, P]),
        "dietgpu_ans_encode_batch_split_size": (c_int, [vp, c_int, c_int, c_u32, P, P, P, P,
                                                        c_u32, P, P]),
        "dietgpu_ans_decode_batch_stride": (c_int, [vp, c_int, c_int, c_u32, P, c_u32, P, c_u32,
                                                    c_u32, P, P, P]),
        "dietgpu_ans_decode_batch_pointer": (c_int, [vp, c_int, c_int, c_u32, P, P, P, P, P, P]),
        "dietgpu_ans_decode_batch_split_size": (c_int, [vp, c_int, c_int, c_u32, P, P, P, P, P,
                                                        P]),
        "dietgpu_ans_get_compressed_info": (c_int, [vp, P, c_u32, P, P, P]),
        "dietgpu_ans_get_compressed_info_device": (c_int, [vp, P, c_u32, P, P, P]),
        "dietgpu_float_compress": (c_int, [vp, c_int, c_int, c_int, c_u32, P, P, P, P, P]),
        "dietgpu_float_compress_split_size": (c_int, [vp, c_int, c_int, c_int, c_u32, P, P, P,
                                                      c_u32, P, P]),
        "dietgpu_float_compress_sparse": (c_int, [vp, c_int, c_int, c_int, c_u32, P, P, P, P, P]),
        "dietgpu_float_decompress": (c_int, [vp, c_int, c_int, c_int, c_u32, P, P, P, P, P, P]),
        "dietgpu_float_decompress_split_size": (c_int, [vp, c_int, c_int, c_int, c_u32, P, P, P,
                                                        P, P, P]),
        "dietgpu_float_decompress_sparse": (c_int, [vp, c_int, c_int, c_int, c_u32, P, P, P, P,
                                                    P, P]),
        "dietgpu_float_get_compressed_info": (c_int, [vp, P, c_u32, P, P, P, P]),
        "dietgpu_float_get_compressed_info_device": (c_int, [vp, P, c_u32, P, P, P, P]),
        "dietgpu_float_compress_batch_stride": (c_int, [vp, c_int, c_int, c_int, c_u32, P, c_u32,
                                                        c_u64, P, c_u64, P, P]),
        "dietgpu_float_decompress_batch_stride": (c_int, [vp, c_int, c_int, c_int, c_u32, P,
                                                          c_u64, P, c_u64, c_u32, P, P, P]),
        "dietgpu_profile_enable": (None, [c_int]),
        "dietgpu_profile_filter": (None, [ctypes.c_char_p]),
        "dietgpu_profile_reset": (None, []),
        "dietgpu_profile_query": (c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_uint64)]),
    }
    # test hooks absent from older builds (same-box A/B of earlier libraries)
    optional = {"dietgpu_set_barrier_budget", "dietgpu_set_dispatch_skew",
                "dietgpu_barrier_fallback_count", "dietgpu_set_compress_path"}
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return sig


EXPORTED = None
_lib = None
TESTLIB_PATH = os.path.join(_HERE, "_lib", "libdietgpu_testhooks.so")
TEST_EXPORTED = None
_testlib = None


def testlib():
    """The test-hook library (include/dietgpu_testhooks.h): GPU tests only,
    never loaded by the package itself."""
    global _testlib, TEST_EXPORTED
    if _testlib is None:
        lib()
        if not os.path.exists(TESTLIB_PATH):
            raise ImportError(f"dietgpu_fork_amd: test-hook library not built ({TESTLIB_PATH})")
        T = ctypes.CDLL(TESTLIB_PATH, mode=ctypes.RTLD_GLOBAL)
        c_u32, c_int, P = ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
        sig = {"dietgpu_test_last_error": (ctypes.c_char_p, []),
               "dietgpu_test_occupy": (c_int, [P, c_u32, c_u32, c_u32]),
               "dietgpu_test_histogram": (c_int, [P, c_u32, P, c_u32, c_u32, P, P]),
               "dietgpu_test_enc_magic": (c_int, [P, P])}
        for name, (res, args) in sig.items():
            f = getattr(T, name)
            f.restype = res
            f.argtypes = args
        TEST_EXPORTED = sorted(sig)
        _testlib = T
    return _testlib


def test_check(rc):
    """check() for the test-hook library's return codes."""
    if rc != DIETGPU_OK:
        raise DietGpuError(testlib().dietgpu_test_last_error().decode(errors="replace"))


def lib():
    global _lib, EXPORTED
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"dietgpu_fork_amd: HIP library not built ({LIB_PATH}); run "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
        # torch first, so the process shares torch's HIP runtime (same soname)
        import torch  # noqa: F401
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        EXPORTED = sorted(_declare(L))
        _lib = L
    return _lib


def check(rc):
    if rc == DIETGPU_OK:
        return
    msg = lib().dietgpu_last_error().decode(errors="replace")
    if rc == DIETGPU_ERR_CHECKSUM:
        raise ChecksumMismatch(msg)
    raise DietGpuError(msg)


def size_or_raise(v):
    """A dietgpu_get_max_*compressed_size result: 0 means the C ABI caught an
    error (e.g. an input too large for 32-bit archive sizes)."""
    if v == 0:
        raise DietGpuError(lib().dietgpu_last_error().decode(errors="replace") or
                           "maximum compressed size query failed")
    return v


def check_archive_sizes(sizes):
    """Compressed sizes read back to the host: 0 marks an element whose
    compression was poisoned (a bounded cross-workgroup wait ran out; see
    dietgpu_device_error_count in include/dietgpu_c.h)."""
    bad = [i for i, v in enumerate(sizes) if int(v) == 0]
    if bad:
        raise DietGpuError(f"compression of batch element(s) {bad[:8]} was abandoned "
                           f"(device error count {lib().dietgpu_device_error_count(1)})")


def ptr_array(values):
    """Host array of pointers / uint32 for the C ABI (kept alive by caller)."""
    return (ctypes.c_void_p * len(values))(*values)


def u32_array(values):
    return (ctypes.c_uint32 * len(values))(*values)


class Stack:
    """RAII wrapper of dietgpu_stack (StackDeviceMemory)."""

    def __init__(self, device, ptr=None, nbytes=0):
        self.h = lib().dietgpu_stack_create(int(device), ptr, int(nbytes))
        if not self.h:
            raise DietGpuError(lib().dietgpu_last_error().decode())

    def max_usage(self):
        return lib().dietgpu_stack_max_usage(self.h)

    def close(self):
        if self.h:
            lib().dietgpu_stack_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
