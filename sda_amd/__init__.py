"""sda_amd -- MI355X (gfx950) engine for SDA's secret-sharing hot path.

The product is the C-ABI library `libsda_engine.so` (include/sda_engine.h) built from the
hand-written HIP kernels in `csrc/`.  This package holds its Python binding (`engine`), the
scheme descriptors (`schemes`), the synthetic-input generator (`synth`) and the multi-GPU
driver (`distributed`).  There is no CPU fallback anywhere in the package.
"""
from . import schemes  # noqa: F401
from .engine import Engine, SdaError, load_library  # noqa: F401

__all__ = ["Engine", "SdaError", "load_library", "schemes"]
