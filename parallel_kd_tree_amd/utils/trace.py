"""roctx ranges from Python (native ``trace_push`` / ``trace_pop``, csrc/include/pkdtree/trace.hpp).

``rocprofv3 --marker-trace`` records them next to the kernel trace; without a tool attached a
range costs one library call. Native phases (pkd.build, pkd.levelN, pkd.subtree,
pkd.generate, pkd.nn_*) are marked in C++; the distributed phases are marked here.
"""
from __future__ import annotations

import contextlib

from ..ops import native


@contextlib.contextmanager
def trace_range(name: str):
    n = native()
    n.trace_push(name)
    try:
        yield
    finally:
        n.trace_pop()
