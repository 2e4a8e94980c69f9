"""dietgpu_fork_amd -- MI355X-native (gfx950) rANS entropy codec.

Drop-in for NSagan271/dietgpu_fork's hot path: batched byte rANS
encode/decode, the exponent-split fp16/bf16/fp32/fp64 float codec and the
sparse float codec, behind the reference's C++ API (include/dietgpu/*.h), a
C ABI (include/dietgpu_c.h, libdietgpu_amd.so) and the ``torch.ops.dietgpu``
operator surface (dietgpu/DietGpu.cpp).

``import dietgpu_fork_amd`` registers ``torch.ops.dietgpu.*`` and raises
ImportError when libdietgpu_amd.so or libdietgpu_torch.so is not built.
"""
from . import _native  # noqa: F401
from ._native import ChecksumMismatch, DietGpuError, build  # noqa: F401

__all__ = ["ops", "codec", "build", "DietGpuError", "ChecksumMismatch", "load_library"]


def load_library():
    """Equivalent of ``torch.ops.load_library("libdietgpu.so")`` in the
    reference harnesses: registers the ``dietgpu`` operator namespace."""
    from . import ops

    ops.register()


# register on import: a missing HIP or operator library raises ImportError
# here (there is no CPU fallback; build with __graft_entry__.build())
load_library()
