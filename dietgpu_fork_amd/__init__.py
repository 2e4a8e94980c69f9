"""dietgpu_fork_amd -- MI355X-native (gfx950) rANS entropy codec.

Drop-in for NSagan271/dietgpu_fork's hot path: batched byte rANS
encode/decode, the exponent-split fp16/bf16/fp32/fp64 float codec and the
sparse float codec, behind the reference's C++ API (include/dietgpu/*.h), a
C ABI (include/dietgpu_c.h, libdietgpu_amd.so) and the ``torch.ops.dietgpu``
operator surface (dietgpu/DietGpu.cpp).

``import dietgpu_fork_amd`` registers ``torch.ops.dietgpu.*``.
"""
from . import _native  # noqa: F401
from ._native import ChecksumMismatch, DietGpuError, build  # noqa: F401

__all__ = ["ops", "codec", "build", "DietGpuError", "ChecksumMismatch", "load_library"]


def load_library():
    """Equivalent of ``torch.ops.load_library("libdietgpu.so")`` in the
    reference harnesses: registers the ``dietgpu`` operator namespace."""
    from . import ops

    ops.register()


try:  # register on import when the HIP library is present
    load_library()
except ImportError:
    pass
