"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
function include/dietgpu_c.h declares, answers the host-only queries like
the reference, and the torch.ops.dietgpu surface carries the reference's
exact schemas (dietgpu/DietGpu.cpp:923-942).  No GPU compute is issued."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dietgpu_c.h")

# TORCH_LIBRARY_FRAGMENT(dietgpu) schemas, DietGpu.cpp:923-942 (verbatim)
REF_SCHEMAS = {
    "max_float_compressed_output_size": "(Tensor[] ts) -> (int, int)",
    "max_float_compressed_size": "(Tensor dtype, int size) -> int",
    "max_any_compressed_output_size": "(Tensor[] ts) -> (int, int)",
    "max_any_compressed_size": "(int bytes) -> int",
    "compress_data": "(bool compress_as_float, Tensor[] ts_in, bool checksum=False, Tensor? temp_mem=None, "
                     "Tensor? out_compressed=None, Tensor? out_compressed_bytes=None) -> (Tensor, Tensor, int)",
    "compress_data_split_size": "(bool compress_as_float, Tensor t_in, Tensor t_in_split_sizes, bool checksum=False, "
                                "Tensor? temp_mem=None, Tensor? out_compressed=None, "
                                "Tensor? out_compressed_bytes=None) -> (Tensor[], Tensor, int)",
    "compress_data_simple": "(bool compress_as_float, Tensor[] ts_in, bool checksum=False, "
                            "int? temp_mem=67108864) -> Tensor[]",
    "decompress_data": "(bool compress_as_float, Tensor[] ts_in, Tensor[] ts_out, bool checksum=False, "
                       "Tensor? temp_mem=None, Tensor? out_status=None, "
                       "Tensor? out_decompressed_words=None) -> (int)",
    "decompress_data_split_size": "(bool compress_as_float, Tensor[] ts_in, Tensor t_out, Tensor t_out_split_sizes, "
                                  "bool checksum=False, Tensor? temp_mem=None, Tensor? out_status=None, "
                                  "Tensor? out_decompressed_words=None) -> (int)",
    "decompress_data_simple": "(bool compress_as_float, Tensor[] ts_in, bool checksum=False, "
                              "int? temp_mem=67108864) -> Tensor[]",
}


@pytest.fixture(scope="module")
def N():
    from dietgpu_fork_amd import _native

    if not os.path.exists(_native.LIB_PATH):
        _native.build()
    _native.lib()
    return _native


def declared_functions(header=HEADER):
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dietgpu_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("dietgpu_ans_encode_batch_pointer", "dietgpu_ans_decode_batch_pointer",
                 "dietgpu_float_compress", "dietgpu_float_decompress",
                 "dietgpu_float_compress_sparse", "dietgpu_float_decompress_sparse",
                 "dietgpu_stack_create", "dietgpu_get_max_compressed_size"):
        assert must in names


def test_library_exports_every_declared_symbol(N):
    L = N.lib()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing
    # and the Python binding declares a signature for each of them
    assert sorted(N.EXPORTED) == declared_functions()


def test_test_hooks_live_in_their_own_library(N):
    """The test-only kernels are not in the product library: they are built
    into libdietgpu_testhooks.so (include/dietgpu_testhooks.h), which the GPU
    tests load beside it."""
    L = N.lib()
    hdr = os.path.join(ROOT, "include", "dietgpu_testhooks.h")
    hooks = [f for f in declared_functions(hdr) if f.startswith("dietgpu_test_")]
    assert hooks and all(not hasattr(L, f) for f in hooks)
    assert not any(f.startswith("dietgpu_test_") for f in declared_functions())
    T = N.testlib()
    assert all(hasattr(T, f) for f in hooks)
    assert N.TEST_EXPORTED == hooks


def test_host_queries_match_reference(N):
    L = N.lib()
    assert L.dietgpu_version().decode().startswith("dietgpu")
    # getMaxCompressedSize (ans/GpuANSEncode.cu:13-25)
    assert L.dietgpu_get_max_compressed_size(65536) == 639520
    assert L.dietgpu_get_max_compressed_size(4194304) == 5800480
    # getMaxFloatCompressedSize (float/GpuFloatCompress.cu:23-48): c2 row
    assert L.dietgpu_get_max_float_compressed_size(2, 524288) == 1737280
    from oracle import oracle as O

    for ft in (1, 2, 3, 4):
        for n in (0, 1, 4096, 100003):
            assert L.dietgpu_get_max_float_compressed_size(ft, n) == O.max_float_compressed_size(ft, n)
            assert (L.dietgpu_get_max_sparse_float_compressed_size(ft, n)
                    == O.max_sparse_float_compressed_size(ft, n))


def test_invalid_arguments_report_errors(N):
    L = N.lib()
    # prob bits out of range is rejected before any device work
    rc = L.dietgpu_float_compress(None, 2, 12, 0, 0, None, None, None, None, None)
    assert rc != N.DIETGPU_OK
    assert L.dietgpu_last_error()


def test_torch_op_schemas(N):
    import dietgpu_fork_amd  # noqa: F401  (registers torch.ops.dietgpu)

    for name, schema in REF_SCHEMAS.items():
        op = getattr(torch.ops.dietgpu, name)
        got = str(op.default._schema)
        ref = str(torch._C.parse_schema(f"dietgpu::{name}{schema}"))  # canonical form
        assert got == ref, (name, got, ref)


def test_torch_size_ops_on_cpu(N):
    import dietgpu_fork_amd  # noqa: F401

    d = torch.ops.dietgpu
    assert d.max_any_compressed_size(65536) == 639520
    assert d.max_float_compressed_size(torch.empty(0, dtype=torch.bfloat16), 524288) == 1737280
    ts = [torch.empty(524288, dtype=torch.bfloat16), torch.empty(1000, dtype=torch.bfloat16)]
    assert tuple(d.max_float_compressed_output_size(ts)) == (2, 1737280)


def test_torch_ops_reject_cpu_tensors(N):
    import dietgpu_fork_amd  # noqa: F401

    with pytest.raises(RuntimeError):
        torch.ops.dietgpu.compress_data(True, [torch.zeros(16, dtype=torch.float16)])


def test_oversize_requests_raise():
    """Sizes whose archives cannot be described with 32-bit sizes raise
    (the reference aborts: GpuANSEncode.cu:22 CHECK_LE) instead of returning
    a bound the caller would allocate and overrun."""
    import torch

    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec as C
    from dietgpu_fork_amd._native import DietGpuError

    with pytest.raises(DietGpuError):
        C.max_compressed_size(0xFFFFFFFF)
    with pytest.raises(DietGpuError):
        C.max_float_compressed_size(3, 1_100_000_000)  # 4.67e9 bytes
    with pytest.raises(DietGpuError):
        C.max_float_compressed_size(4, 1_000_000_000)
    # the reference's largest published batch-1 point (README.md:118): the
    # bound exceeds INT32_MAX but is a valid u32, as in
    # float/GpuFloatCompress.cu:23-47
    n = 1_070_000_000
    assert C.max_float_compressed_size(2, n) == 32 + C.max_compressed_size(n) + (n + 15) // 16 * 16
    with pytest.raises(RuntimeError):
        torch.ops.dietgpu.max_any_compressed_size(4_000_000_000)
    assert C.max_float_compressed_size(2, 524288) == 1737280


def test_native_op_library_is_loaded(N):
    """torch.ops.dietgpu comes from the native TORCH_LIBRARY library
    (csrc/torch_ops.cpp), loaded like the reference's extension."""
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import ops

    assert os.path.exists(ops.LIB_PATH)
    ops.register()
    maps = open("/proc/self/maps").read()
    assert "libdietgpu_torch.so" in maps and "libdietgpu_amd.so" in maps
    assert ops.max_any_compressed_size(4096) == torch.ops.dietgpu.max_any_compressed_size(4096)


def test_cpp_api_program_links():
    """tests/cpp/api_roundtrip.cpp (built by build()) links libdietgpu_amd.so
    through include/dietgpu/*.h; without a GPU it reports so (exit 2)."""
    import subprocess

    exe = os.path.join(ROOT, "dietgpu_fork_amd", "_lib", "api_roundtrip")
    assert os.path.exists(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode in (0, 2), r.stderr


def test_import_raises_without_the_library(tmp_path):
    """No silent fallback: a package copy whose HIP libraries are not built
    fails at `import dietgpu_fork_amd` (Boundary)."""
    import shutil
    import subprocess
    import sys

    shutil.copytree(os.path.join(ROOT, "dietgpu_fork_amd"), tmp_path / "dietgpu_fork_amd",
                    ignore=shutil.ignore_patterns("_lib", "csrc", "__pycache__"))
    r = subprocess.run([sys.executable, "-c", "import dietgpu_fork_amd"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "ImportError" in r.stderr and "not built" in r.stderr, r.stderr[-2000:]
