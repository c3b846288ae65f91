"""Native ops: the HIP/C++ core compiled into ``parallel_kd_tree_amd._C``.

There is deliberately no PyTorch fallback for device work: if the extension is missing the
import fails loudly (build it with ``python -m parallel_kd_tree_amd._build``).
"""
from __future__ import annotations

import importlib

_C = None


def native():
    """Return the loaded extension module (raises ImportError with a build hint)."""
    global _C
    if _C is None:
        try:
            _C = importlib.import_module("parallel_kd_tree_amd._C")
        except ImportError as e:  # pragma: no cover - exercised only without a build
            raise ImportError(
                "parallel_kd_tree_amd native extension is not built; run "
                "`python -m parallel_kd_tree_amd._build` (hipcc --offload-arch=gfx950)") from e
    return _C


def native_path() -> str:
    return native().__file__


from .build import (GpuTreeBuilder, ReferenceTreeBuilder, build_cpu, build_gpu, build_gpu_checked, check_unique_ids,
                    build_reference_gpu_checked,  # noqa: E402
                    gpu_builder, reference_builder)
from .query import nn_gpu, unpack, finalize, nn_cpu  # noqa: E402

__all__ = ["native", "native_path", "GpuTreeBuilder", "build_gpu", "build_gpu_checked", "build_cpu", "check_unique_ids", "gpu_builder", "nn_gpu", "unpack", "finalize", "nn_cpu"]
