"""PyTorch-ROCm operator surface: ``torch.ops.dietgpu.*``.

The operators are native: ``TORCH_LIBRARY(dietgpu)`` in
``csrc/torch_ops.cpp``, built into ``_lib/libdietgpu_torch.so`` and loaded
with ``torch.ops.load_library`` exactly as the reference's harnesses load its
``DietGpu.cpp`` extension (dietgpu/DietGpu.cpp:921-978: same ten operators,
schemas, validation and return values).  This module only loads that library
and forwards ``ops.<name>(...)`` to ``torch.ops.dietgpu.<name>``.
"""
import os

import torch

from . import _native as N

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libdietgpu_torch.so")

OPS = (
    "max_float_compressed_output_size",
    "max_float_compressed_size",
    "max_any_compressed_output_size",
    "max_any_compressed_size",
    "compress_data",
    "compress_data_split_size",
    "compress_data_simple",
    "decompress_data",
    "decompress_data_split_size",
    "decompress_data_simple",
)

_LOADED = False


def register():
    """Load the native operator library (idempotent); fails loudly when it or
    the HIP codec library it links is missing."""
    global _LOADED
    if _LOADED:
        return
    N.lib()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"dietgpu_fork_amd: operator library not built ({LIB_PATH}); run "
                          "`python -c 'import __graft_entry__ as g; g.build()'`")
    torch.ops.load_library(LIB_PATH)
    _LOADED = True


def __getattr__(name):
    if name in OPS:
        register()
        return getattr(torch.ops.dietgpu, name)
    raise AttributeError(name)
