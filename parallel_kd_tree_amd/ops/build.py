"""Tree-build ops.

GPU: the level-synchronous HIP builder (csrc/gpu/build_global.hip + build_subtree.hip);
CPU: the native exact / reference-mode builders (csrc/cpu/cpu_tree.cpp).
Both return the implicit in-order tree ``(tree_pts [n, d] float32, tree_ids [n] int32)``:
slot k holds the node whose segment median is k (root at n // 2).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import native


class GpuTreeBuilder:
    """Reusable builder for a fixed (n, dim) on one device.

    Holds the plan and a workspace from the torch caching allocator, so repeated builds
    (benchmarks, rebuilds of a streaming index) allocate nothing.
    """

    TOP_BAND_MISS = 0x20  # error bit: a sampled band (top levels or a triple) missed its median: rebuild unsampled

    def __init__(self, n: int, dim: int, depth0: int = 0, subtree_max: int = 0, allow_top: bool = True):
        self._b = native().GpuBuilder(int(n), int(dim), int(depth0), int(subtree_max), bool(allow_top))
        self.n, self.dim, self.depth0 = int(n), int(dim), int(depth0)
        self.subtree_max_arg = int(subtree_max)

    @property
    def workspace_bytes(self) -> int:
        return self._b.workspace_bytes

    @property
    def global_levels(self) -> int:
        return self._b.global_levels

    @property
    def subtree_max(self) -> int:
        return self._b.subtree_max

    @property
    def split_parts(self) -> int:
        """Parts of a split build (0: one stream; see PKD_SPLIT* in README)."""
        return self._b.split_parts

    def describe(self) -> str:
        return self._b.describe()

    @property
    def column_stride(self) -> int:
        return int(self._b.column_stride)

    def build_columns(self, cols: torch.Tensor):
        """Build from SoA columns [dim + 1, column_stride] (the last row holds the ids' bits), the
        distributed leaves' input layout; returns (tree_pts, tree_ids)."""
        return tuple(self._b.build_columns(cols))

    @property
    def sampled_top(self) -> bool:
        """Levels 0..3 come from the sampled top pass (csrc/gpu/top4.hpp)."""
        return bool(self._b.sampled_top)

    @property
    def sampled(self) -> bool:
        """Some levels come from a sample (the top pass or a sampled triple): the error word may
        carry TOP_BAND_MISS, and such a build is redone unsampled (build_gpu_checked)."""
        return bool(self._b.sampled)

    def top_band_report(self):
        """Per top node (heap 0..14) of the last build: (band rows, rank inside the median's
        fine bin, rows the scatter staged at the node). Synchronises."""
        v = list(self._b.top_band_report())
        return [tuple(v[3 * i:3 * i + 3]) for i in range(len(v) // 3)]

    def g3_report(self):
        """The last sampled triple of the last build (synchronises): (level, per-segment rows
        [n, staged per tag 0..6, certain per great-grandchild 0..7, inserted per great-grandchild
        0..7, bad]); None without a sampled triple."""
        v = list(self._b.g3_report())
        if not v:
            return None
        return v[0], [v[1 + 25 * i:26 + 25 * i] for i in range((len(v) - 1) // 25)]

    def read_error(self) -> int:
        """Sticky device error word of the last build (0 = ok). Synchronises."""
        return int(self._b.read_error()[0])

    def error_words(self) -> torch.Tensor:
        """A device copy (int32 [4]: error word, first failure code, level, value) of the last
        build's error words, ordered after it on the current stream: no host sync."""
        return self._b.error_words().clone()

    def accumulate_error(self, acc: torch.Tensor) -> None:
        """Fold the last build's error word into ``acc`` (int32 [>= 3] on the device): OR of the
        words, builds with an error, builds with TOP_BAND_MISS. Stream-ordered, no host sync."""
        self._b.accumulate_error(acc)

    def read_error_detail(self):
        """(error word, first failure code, level, value). Synchronises."""
        return tuple(int(v) for v in self._b.read_error())

    def build(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0,
              out_pts: Optional[torch.Tensor] = None, out_ids: Optional[torch.Tensor] = None):
        return tuple(self._b.build(points, ids, int(id_base), out_pts, out_ids))

    def build_rows(self, rows: torch.Tensor):
        """Build from rows [n, dim+1]: coordinates followed by the id bits (int32 viewed as f32)."""
        return tuple(self._b.build_rows(rows.contiguous()))

    def soa_input(self, device) -> torch.Tensor:
        """[(dim + 1), n] float32 view of the builder's input columns (row ``dim`` = id bits)."""
        return self._b.soa_input(torch.device(device))

    def build_from_soa(self, device):
        return tuple(self._b.build_from_soa(torch.device(device)))


class ReferenceTreeBuilder:
    """Reference-mode builder on the GPU (csrc/gpu/build_reference.hip): the reference's own
    tree (first n - 1 points sorted per segment), by per-level rank selection."""

    def __init__(self, n: int, dim: int, depth0: int = 0):
        self._b = native().ReferenceBuilder(int(n), int(dim), int(depth0))
        self.n, self.dim, self.depth0 = int(n), int(dim), int(depth0)

    def build(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0):
        return tuple(self._b.build(points.contiguous(), ids, int(id_base)))

    def read_ties(self) -> int:
        """Segments of the last build whose tree equal keys decided (there the reference's
        unstable std::sort decides: the tree may differ from the binary's). Synchronises."""
        return int(self._b.read_ties())

    def read_tie_slots(self):
        """Median slots of the last build's tied segments (at most ``tie_slots_cap`` of them)."""
        return list(self._b.read_tie_slots())

    @property
    def tie_slots_cap(self) -> int:
        return int(self._b.tie_slots_cap)

    @property
    def global_levels(self) -> int:
        return int(self._b.global_levels)


_builders: dict = {}


def reference_builder(n: int, dim: int, depth0: int = 0, device=None) -> ReferenceTreeBuilder:
    key = ("reference", int(n), int(dim), int(depth0), device)
    b = _builders.get(key)
    if b is None:
        if len(_builders) > 8:
            _builders.clear()
        b = _builders[key] = ReferenceTreeBuilder(n, dim, depth0)
    return b


def gpu_builder(n: int, dim: int, depth0: int = 0, subtree_max: int = 0, device=None) -> GpuTreeBuilder:
    """A cached builder for (n, dim, depth0, subtree_max) on `device`."""
    key = (int(n), int(dim), int(depth0), int(subtree_max), device)
    b = _builders.get(key)
    if b is None:
        if len(_builders) > 8:
            _builders.clear()
        b = _builders[key] = GpuTreeBuilder(n, dim, depth0, subtree_max)
    return b


def build_gpu(points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0, depth0: int = 0,
              subtree_max: int = 0):
    """Build the exact tree of ``points`` ([n, d] float32 on a GPU). Explicit ``ids`` must be
    distinct: the exact order (coordinate, id) is only total for unique ids. A build whose
    sampled levels missed a median is redone unsampled (build_gpu_checked), so the result is
    always the exact tree; GpuTreeBuilder.build is the asynchronous form that leaves that check
    (read_error()) to the caller."""
    if not points.is_cuda:
        raise ValueError("build_gpu needs a GPU tensor")
    tp, ti, _ = build_gpu_checked(points, ids, id_base, depth0, subtree_max)
    return tp, ti


def build_gpu_checked(points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0,
                      depth0: int = 0, subtree_max: int = 0):
    """build_gpu, then -- for builds with sampled levels -- a host check of the error word: a
    band that missed its median (error bit TOP_BAND_MISS) is rebuilt without sampling. Misses
    are rare but not negligible: z = 6 for the top levels (~2e-9 per node), z = 5 for the
    sampled triples (about one miss per 2000 builds of 100 M points), and duplicate-heavy data
    whose median arenas are too large to stream always miss. A missed build stops at its first
    failed check (every later kernel returns), so the builder stays reusable. Returns
    (tree_pts, tree_ids, builder). Synchronises only for sampled builds."""
    points = points.contiguous()
    b = gpu_builder(points.shape[0], points.shape[1], depth0, subtree_max, points.device)
    tp, ti = b.build(points, ids, id_base)
    if b.sampled and (b.read_error() & GpuTreeBuilder.TOP_BAND_MISS):
        key = ("unsampled", points.shape[0], points.shape[1], depth0, subtree_max, points.device)
        fb = _builders.get(key)
        if fb is None:
            fb = _builders[key] = GpuTreeBuilder(points.shape[0], points.shape[1], depth0, subtree_max,
                                                 allow_top=False)
        tp, ti = fb.build(points, ids, id_base, tp, ti)
        b = fb
    return tp, ti, b


def check_unique_ids(ids: Optional[torch.Tensor]) -> None:
    """Explicit ids must be distinct (ValueError otherwise): with two equal (key, id) pairs
    the median rank is ambiguous and the exact builders' output is undefined."""
    if ids is None or ids.numel() < 2:
        return
    if torch.unique(ids.reshape(-1)).numel() != ids.numel():
        raise ValueError("point ids must be distinct")


def build_reference_gpu_checked(points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0,
                                depth0: int = 0):
    """The reference tree on the GPU. Where equal keys decided a segment (std::sort is unstable,
    so there the reference binary's tree is its library's introsort's choice, which depends on
    the segment's exact input order), the tree is REPAIRED on the host: the sorts of the tied
    segments' ancestors and the tied subtrees are replayed with a bit-exact replica of std::sort
    (native reference_repair) and only those slots are patched; every other subtree keeps the
    GPU's slots. A warning names the tie count. Returns (tree_pts, tree_ids, ties). Synchronises."""
    import warnings
    points = points.contiguous()
    b = reference_builder(points.shape[0], points.shape[1], depth0, points.device)
    tp, ti = b.build(points, ids, id_base)
    ties = b.read_ties()
    if ties:
        n, dim = points.shape
        cids = ids.to(torch.int64) if ids is not None else None
        # the host sorts read one key per row and level: only the levels' columns travel when the
        # rows are wider (500 k x 128D: 19 of 128 columns); their axis at depth d is then column d
        levels = max(1, int(n).bit_length())
        if levels < dim:
            host = points[:, [(depth0 + d) % dim for d in range(levels)]].cpu()
            hdepth0 = 0
        else:
            host, hdepth0 = points.cpu(), depth0
        if ties <= b.tie_slots_cap:
            # the GPU tree's slot -> input row (ids are distinct: invert them through a scatter)
            if cids is None:
                rows = (ti.to(torch.int64) - id_base).to(torch.int32).cpu()
            else:
                inv = torch.empty(int(cids.max()) - int(cids.min()) + 1, dtype=torch.int64, device=cids.device)
                inv[cids - int(cids.min())] = torch.arange(n, device=cids.device)
                rows = inv[ti.to(torch.int64) - int(cids.min())].to(torch.int32).cpu()
            perm, slots = native().reference_repair(host, rows, b.read_tie_slots(), int(hdepth0), cpu_threads())
            sl = slots.to(points.device)
            rw = perm.to(points.device).to(torch.int64)[sl]
            tp[sl] = points[rw]
            ti[sl] = (rw + id_base).to(torch.int32) if ids is None else ids.to(points.device)[rw].to(torch.int32)
            how = f"replayed their sorts on the host and patched {slots.numel()} of {n} slots"
        else:
            hids = (torch.arange(n, dtype=torch.int64) + id_base).to(torch.int32) if ids is None else ids.cpu()
            _, perm = build_cpu(host, torch.arange(n, dtype=torch.int32), "reference", hdepth0, cpu_threads())
            rw = perm.to(points.device).to(torch.int64)
            tp = points[rw].contiguous()
            ti = hids.to(points.device)[rw].contiguous()
            how = "rebuilt the tree with the threaded host std::sort builder"
        warnings.warn(f"reference mode: {ties} segment(s) of this input are decided by equal keys, where the "
                      f"reference's unstable std::sort picks the order; {how}", RuntimeWarning, stacklevel=2)
    return tp, ti, ties


def cpu_threads() -> int:
    """Threads of the host builders' fallbacks (the reference mode's std::sort builder gives the
    same tree for any count)."""
    import os
    return max(1, min(64, os.cpu_count() or 1))


def build_cpu(points: torch.Tensor, ids: Optional[torch.Tensor] = None, mode: str = "exact", depth0: int = 0,
              threads: int = 1):
    """Native CPU build. ``mode='reference'`` reproduces the reference tree exactly
    (first n-1 points sorted per node, kdtree_sequential.cpp:46-48)."""
    points = points.detach().to("cpu", torch.float32).contiguous()
    if ids is not None:
        ids = ids.to("cpu", torch.int32).contiguous()
    return tuple(native().build_cpu(points, ids, mode, int(depth0), int(threads)))
