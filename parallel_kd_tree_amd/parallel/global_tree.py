"""Global decomposition: ONE exact kd-tree over P ranks (any P <= 64).

North-star design (BASELINE.json): the reference's forest of independent per-rank trees
(kdtree_mpi.cpp:204-253) becomes a single distributed tree:

1. bounding box: allreduce MIN / MAX of the per-rank boxes;
2. top LL levels, level by level: every rank histograms its points (routed below the pivots
   decided so far) into linear buckets of its node's cell, the histograms are allreduced (SUM),
   the bucket holding each node's median is found, the few points of that bucket are
   all-gathered and ranked under the (key, id) order -> the exact pivot point of every node at
   that level, identical on every rank;
3. the T = 2^LL top-level leaves are dealt to the ranks in contiguous runs and every point
   travels to the rank owning its leaf, one all-to-all round per leaf of a rank;
4. each rank builds its leaves' subtrees (depth LL).

The result is slot-for-slot the tree a single GPU builds on the concatenated points.

The GPU implementation is the native C++ builder (csrc/cpu/global_builder.cpp, Python handle
:class:`~parallel_kd_tree_amd.parallel.native_global.NativeGlobalBuilder`) on RCCL. This module
holds what both paths share -- :class:`DistTree` (a rank's share of the tree and the replicated
top tree, with the query / gather / check helpers) -- and :class:`GlobalTreeBuilder`, the same
schedule on host tensors over gloo (CPU tests and the CPU rehearsal of ``bench.py``): torch code
with the kernels' arithmetic for the per-rank steps, and the native geometry and exchange
planner (``global_layout`` / ``global_plan``) so both paths agree on who owns what.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from . import comm
from .geometry import composite_u64, make_params, segment

TOP_BINS = 8192  # nodes * bins per top level (LDS histogram in the kernel)
DONE = 0xFFFFFFFF


def layout(n_total: int, P: int, k: int = -1) -> dict:
    """Who owns what (csrc/cpu/global_builder.cpp, global_plan::make_layout): LL top levels,
    T leaves, leaf runs per rank, every rank's share (slot range, complete-subtree blocks and
    the top rows between them), the top nodes' slots and owners (-1: boundary)."""
    return ops.native().global_layout(int(n_total), int(P), int(k))


def _to_rows(points: torch.Tensor, ids: Optional[torch.Tensor], id_base: int) -> torch.Tensor:
    n, dim = points.shape
    if ids is None:
        ids = (torch.arange(n, dtype=torch.int64, device=points.device) + int(id_base)).to(torch.int32)
    rows = torch.empty((n, dim + 1), dtype=torch.float32, device=points.device)
    rows[:, :dim] = points
    rows[:, dim] = ids.to(torch.int32).view(torch.float32)
    return rows


def signed_keys(pts: torch.Tensor, ids: torch.Tensor, axis: int) -> torch.Tensor:
    """Composite (orderable(key) << 32 | id) keys as int64 with the top bit flipped, so that
    signed order == the builder's unsigned order."""
    kb = pts[:, axis].contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ok = torch.where((kb & 0x80000000) != 0, (~kb) & 0xFFFFFFFF, kb | 0x80000000)
    ib = ids.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return ((ok ^ 0x80000000) << 32) | ib


def _signed_keys(rows: torch.Tensor, dim: int, axis: int) -> torch.Tensor:
    return signed_keys(rows[:, :dim], rows[:, dim], axis)


def _u64_to_signed(v: int) -> int:
    v ^= 1 << 63
    return v - (1 << 64) if v >= (1 << 63) else v


# --------------------------------------------------------------------------- CPU reference ops
# Same arithmetic as csrc/gpu/dist_ops.hip; used when the points live on the CPU (gloo tests).
def _bucket_cpu(x: torch.Tensor, lo: torch.Tensor, scale: torch.Tensor, nb: int) -> torch.Tensor:
    t = (x - lo) * scale
    t = torch.nan_to_num(t, nan=0.0, posinf=float(nb - 1), neginf=0.0)
    return t.clamp(0, nb - 1).to(torch.int64)


def _route_cpu(rows, dim, node, pivots_signed, axis):
    live = node != DONE
    h = node[live]
    k = _signed_keys(rows[live], dim, axis)
    pv = pivots_signed[h]
    nh = torch.where(k < pv, 2 * h + 1, torch.where(k > pv, 2 * h + 2, torch.full_like(h, DONE)))
    node[live] = nh
    return node


class _HostOps:
    """Per-rank top-level ops on host tensors (gloo tests): the torch reference of the HIP
    kernels in csrc/gpu/dist_ops.hip (same bucketing arithmetic, same routing)."""

    @staticmethod
    def route_hist(rows, dim, node, level, pivots_u64, prev_axis, axis, params, bins):
        nodes = 1 << level
        if level > 0:
            piv = torch.tensor([_u64_to_signed(int(v)) for v in pivots_u64], dtype=torch.int64)
            _route_cpu(rows, dim, node, piv, prev_axis)
        live = node != DONE
        j = node[live] - (nodes - 1)
        prm = torch.from_numpy(params)
        b = _bucket_cpu(rows[live, axis], prm[j, 0], prm[j, 1], bins)
        return torch.bincount(j * bins + b, minlength=nodes * bins).to(torch.int32)

    @staticmethod
    def collect_middle(rows, dim, node, level, axis, params, bins, bstar):
        nodes = 1 << level
        live = (node != DONE).nonzero().flatten()
        j = node[live] - (nodes - 1)
        prm = torch.from_numpy(params)
        b = _bucket_cpu(rows[live, axis], prm[j, 0], prm[j, 1], bins)
        sel = live[b == torch.from_numpy(bstar.astype(np.int64))[j]]
        out = torch.empty((sel.numel(), dim + 2), dtype=torch.float32)
        out[:, :dim + 1] = rows[sel]
        out[:, dim + 1] = node[sel].to(torch.int32).view(torch.float32)
        return out

    @staticmethod
    def pack(rows, dim, node, levels, pivots_u64, last_axis):
        """Rows grouped by top-level leaf (stable) and the rows per leaf (k_pack_* kernels)."""
        T = 1 << levels
        if levels > 0:
            piv = torch.tensor([_u64_to_signed(int(v)) for v in pivots_u64], dtype=torch.int64)
            _route_cpu(rows, dim, node, piv, last_axis)
        live = (node != DONE).nonzero().flatten()
        leaf = node[live] - (T - 1)
        order = torch.sort(leaf, stable=True).indices
        return rows[live[order]].contiguous(), torch.bincount(leaf, minlength=T).to(torch.int64)


@dataclass
class DistTree:
    """A rank's share of the global tree plus the replicated top tree.

    The share is the slot range [slot_lo, slot_lo + n) of the global in-order tree: complete
    subtrees ("blocks", each a valid implicit tree with its own root depth) and the top rows
    between them -- one block rooted at depth log2 P for a power-of-two P. ``top_rows`` holds
    all T - 1 top-tree rows in heap order; ``top_slots[h]`` is the global slot of the boundary
    rows (between two ranks' shares, outside every share) and -1 otherwise."""
    n_total: int
    dim: int
    depth0: int
    P: int
    rank: int
    tree_pts: torch.Tensor           # this rank's share (in-order), slots [slot_lo, slot_lo + n)
    tree_ids: torch.Tensor
    slot_lo: int
    top_slots: List[int] = field(default_factory=list)
    top_rows: Optional[torch.Tensor] = None   # [T - 1, dim + 1] top-tree rows, heap order
    timings: Dict[str, float] = field(default_factory=dict)
    layout: Optional[dict] = None

    @property
    def blocks(self) -> List[Tuple[int, int, int, int]]:
        """(offset in the share, points, root depth, heap node) of every complete subtree."""
        return list(self.layout["blocks"][self.rank])

    @property
    def between(self) -> List[int]:
        """Heap nodes of the top rows between this rank's blocks (inside its share)."""
        return list(self.layout["between"][self.rank])

    def gather_full(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Assemble the whole in-order tree on every rank (for checks and small N)."""
        dev = self.tree_pts.device
        rows = torch.empty((self.tree_pts.shape[0], self.dim + 1), dtype=torch.float32, device=dev)
        rows[:, :self.dim] = self.tree_pts
        rows[:, self.dim] = self.tree_ids.view(torch.float32)
        parts = _all_gather_var(rows)
        full = torch.empty((self.n_total, self.dim + 1), dtype=torch.float32, device=dev)
        for r, part in enumerate(parts):
            lo = int(self.layout["share_lo"][r])
            full[lo:lo + part.shape[0]] = part
        if self.top_rows is not None:
            for i, s in enumerate(self.top_slots):
                if s >= 0:
                    full[s] = self.top_rows[i].to(dev)
        return full[:, :self.dim].contiguous(), full[:, self.dim].contiguous().view(torch.int32)

    def query_packed(self, queries: torch.Tensor, method: str = "auto", routed: bool = True,
                     count_work: bool = False) -> torch.Tensor:
        """Exact NN over the whole distributed tree, packed (d2 << 32 | id), on every rank.

        routed (default): queries are replicated on every rank (as in kdtree_mpi.cpp:234-243),
        but each is searched where it can matter:
          1. every query descends the replicated top tree to its home leaf; only the rank
             owning that leaf searches it (in the block holding the leaf) -> ~Q / P searches
             per rank; one MIN all-reduce gives every query a candidate radius;
          2. a rank searches a query in one of its other blocks (or, for the home block, never
             again) only if the query's best ball reaches that block's cell (the box cut out by
             the top pivots above it), starting from the candidate radius; a second MIN
             all-reduce gives the answer.
        The top rows between blocks and the boundary rows are brute-forced (<= 63 rows).
        routed=False: every rank searches every query in all its blocks (one MIN all-reduce).
        ``self.last_query_work`` holds this rank's (query, block) searches of the last call (the
        native routed search counts them only with ``count_work=True``: two extra device-to-host
        reads and communicator waits; -1 otherwise)."""
        dev = self.tree_pts.device
        q = queries.to(dev, torch.float32).contiguous()
        Q = q.shape[0]
        native = getattr(self, "native", None)
        if native is not None and routed and method == "auto":
            # the native routed search (GlobalBuilder::query): home block, MIN all-reduce, reach
            # blocks, MIN all-reduce -- device lists, no per-block Python loop
            packed, work = native.query(q, bool(count_work))
            self.last_query_work = int(work) if count_work else -1
            return packed
        packed = torch.full((Q,), ops.query.INF_PACKED, dtype=torch.int64, device=dev)
        blocks = [b for b in self.blocks if b[1] > 0]
        work = 0
        if not routed:
            for b in blocks:
                packed = torch.minimum(packed, self._search_block(b, q, method, None))
                work += Q
        else:
            home_blk = self._home_blocks(q)  # [Q]: index into `blocks` of this rank, -1 elsewhere
            for i, b in enumerate(blocks):
                sel = (home_blk == i).nonzero().flatten()
                if sel.numel():
                    packed[sel] = self._search_block(b, q[sel], method, None)
                    work += int(sel.numel())
        packed = self._brute_top(packed, q)
        packed = comm.min_packed_(packed)
        if routed:
            d2 = ops.unpack(packed)[0].to(torch.float64)
            for i, b in enumerate(blocks):
                lo, hi = self._block_box(b)
                gap = torch.clamp(lo[None, :] - q.double(), min=0) + torch.clamp(q.double() - hi[None, :], min=0)
                bd2 = (gap * gap).sum(1)
                # conservative: the box bound is exact math, point distances are fp32 sums
                reach = (bd2 <= d2 * (1 + 1e-5) + 1e-30) & (home_blk != i)
                sel = reach.nonzero().flatten()
                if sel.numel():
                    packed[sel] = self._search_block(b, q[sel], method, packed[sel].clone())
                    work += int(sel.numel())
            packed = comm.min_packed_(packed)
        self.last_query_work = work
        return packed

    # ---- routed-query helpers ----------------------------------------------------------
    def _search_block(self, b, q, method, into):
        """Packed NN of queries q in block b (MIN-combined with / pruned by `into`)."""
        from ..models.kdtree import KDTree
        off, n, depth, _ = b
        t = KDTree(self.tree_pts[off:off + n], self.tree_ids[off:off + n], self.depth0 + depth)
        if t.tree_pts.is_cuda:
            return t.query_packed(q, method, into=into)
        r = _local_packed(t, q, method).to(q.device)
        return r if into is None else torch.minimum(r, into)

    def _brute_top(self, packed, q):
        """MIN with the top rows between this rank's blocks and (rank 0) the boundary rows."""
        dev = packed.device
        rows = [int(self.layout["top_slot"][h]) - self.slot_lo for h in self.between]
        if rows:
            sel = torch.tensor(rows, dtype=torch.int64, device=dev)
            packed = torch.minimum(packed, _brute_packed(self.tree_pts[sel], self.tree_ids[sel], q).to(dev))
        if self.top_rows is not None and self.rank == 0:
            valid = [i for i, s in enumerate(self.top_slots) if s >= 0]
            if valid:
                tr = self.top_rows[valid].to(dev)
                pk = _brute_packed(tr[:, :self.dim].contiguous(), tr[:, self.dim].contiguous().view(torch.int32), q)
                packed = torch.minimum(packed, pk.to(dev))
        return packed

    def _pivot_keys(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """(axis, split coordinate) of every top node (heap order), on the tree's device."""
        T1 = 0 if self.top_rows is None else int(self.top_rows.shape[0])
        axes = torch.tensor([(self.depth0 + (h + 1).bit_length() - 1) % self.dim for h in range(T1)],
                            dtype=torch.int64)
        keys = self.top_rows[torch.arange(T1), axes].float() if T1 else torch.empty(0)
        return axes.to(self.tree_pts.device), keys.to(self.tree_pts.device)

    def _home_blocks(self, q: torch.Tensor) -> torch.Tensor:
        """Index of the block (of this rank's blocks with points) holding each query's home leaf:
        the leaf reached by descending the top tree (coordinate < pivot -> left, else right,
        the search's own near side); -1 when the home leaf belongs to another rank."""
        LL, T = int(self.layout["LL"]), int(self.layout["T"])
        axes, keys = self._pivot_keys()
        h = torch.zeros(q.shape[0], dtype=torch.int64, device=q.device)
        for _ in range(LL):
            go_right = q.gather(1, axes[h][:, None])[:, 0] >= keys[h]
            h = 2 * h + 1 + go_right.to(torch.int64)
        leaf = h - (T - 1)
        out = torch.full_like(leaf, -1)
        blocks = [b for b in self.blocks if b[1] > 0]
        for i, (_, _, depth, heap) in enumerate(blocks):
            s = LL - depth  # levels between the block root and the top-level leaves
            first = ((heap + 1) << s) - T  # first leaf of the block
            out = torch.where((leaf >= first) & (leaf < first + (1 << s)), torch.full_like(out, i), out)
        return out

    def _block_box(self, b) -> Tuple[torch.Tensor, torch.Tensor]:
        """The cell of a block: [lo, hi] per axis cut out by the top pivots above its root
        (closed: points equal to a pivot's coordinate may sit on either side)."""
        if not hasattr(self, "_boxes"):
            self._boxes = {}
        heap = b[3]
        if heap not in self._boxes:
            lo = torch.full((self.dim,), float("-inf"), dtype=torch.float64)
            hi = torch.full((self.dim,), float("inf"), dtype=torch.float64)
            top = self.top_rows.detach().cpu() if self.top_rows is not None else None
            child = heap
            while child > 0:
                h = (child - 1) // 2
                a = (self.depth0 + (h + 1).bit_length() - 1) % self.dim
                v = float(top[h, a])
                if child == 2 * h + 1:
                    hi[a] = min(hi[a], v)
                else:
                    lo[a] = max(lo[a], v)
                child = h
            dev = self.tree_pts.device
            self._boxes[heap] = (lo.to(dev), hi.to(dev))
        return self._boxes[heap]

    def check_top_routing(self) -> str:
        """'' when every block of this rank lies on the correct side of every top-tree pivot
        above it (the cross-rank part of the tree invariant, which a per-rank invariant check
        cannot see): for each block and each ancestor h of its root, the block's smallest /
        largest composite key on h's axis is above / below h's pivot."""
        if self.top_rows is None or self.top_rows.shape[0] == 0:
            return ""
        top = self.top_rows.to(self.tree_pts.device)
        tkeys = {}
        for off, n, depth, heap in self.blocks:
            if n <= 0:
                continue
            pts, ids = self.tree_pts[off:off + n], self.tree_ids[off:off + n]
            child = heap
            while child > 0:
                h = (child - 1) // 2
                lvl = (h + 1).bit_length() - 1
                axis = (self.depth0 + lvl) % self.dim
                if h not in tkeys:
                    tkeys[h] = int(signed_keys(top[h:h + 1, :self.dim], top[h:h + 1, self.dim], axis)[0])
                k = signed_keys(pts, ids, axis)
                if child == 2 * h + 1 and int(k.max()) >= tkeys[h]:
                    return f"block at heap node {heap} reaches above the pivot of top node {h}"
                if child == 2 * h + 2 and int(k.min()) <= tkeys[h]:
                    return f"block at heap node {heap} reaches below the pivot of top node {h}"
                child = h
        return ""


def _local_packed(tree, queries, method):
    """Packed (d2, id) per query on one rank's tree: GPU kernels for exact GPU trees, the
    reference search procedure (csrc/cpu/cpu_tree.cpp) for CPU or reference-mode trees."""
    if tree.tree_pts.is_cuda and tree.mode == "exact":
        if tree.n == 0:
            return torch.full((queries.shape[0],), ops.query.INF_PACKED, dtype=torch.int64, device=tree.device)
        return tree.query_packed(queries, method)
    if tree.n == 0:
        return torch.full((queries.shape[0],), ops.query.INF_PACKED, dtype=torch.int64)
    slots, d2 = ops.nn_cpu(tree.tree_pts.cpu(), queries.cpu().to(torch.float32), tree.depth0)
    ids = tree.tree_ids.cpu().to(torch.int64)[slots] & 0xFFFFFFFF
    return ((d2.view(torch.int32).to(torch.int64) << 32) | ids).to(tree.tree_pts.device)


def _brute_packed(pts, ids, queries):
    """Packed (d2, id) minimum over a small point set (the replicated top rows)."""
    if pts.is_cuda:
        return ops.nn_gpu(pts.contiguous(), ids.contiguous(), queries.to(pts.device, torch.float32), "brute")
    q = queries.cpu().to(torch.float32)
    best = torch.full((q.shape[0],), ops.query.INF_PACKED, dtype=torch.int64)
    for i in range(pts.shape[0]):
        acc = torch.zeros(q.shape[0], dtype=torch.float32)
        for c in range(pts.shape[1]):  # reference summation order, separately rounded
            t = pts[i, c].cpu() - q[:, c]
            acc = acc + t * t
        v = (acc.view(torch.int32).to(torch.int64) << 32) | (int(ids[i]) & 0xFFFFFFFF)
        best = torch.minimum(best, v)
    return best


def _run_rounds(R: int, issue, consume) -> None:
    """The exchange schedule of the native builder: round j + 1's all-to-all is started
    before round j's payload is consumed (its leaf subtree built), so every exchange but the
    first overlaps a build. ``issue(j)`` returns ``(payload, handles)``."""
    pending = issue(0)
    for j in range(R):
        payload, handles = pending
        for hd in handles:
            if hd is not None:
                hd.wait()
        if j + 1 < R:
            pending = issue(j + 1)
        consume(j, payload)


def _all_gather_var(t: torch.Tensor) -> List[torch.Tensor]:
    """all_gather of tensors whose first dimension differs per rank."""
    P = comm.world()
    if P == 1:
        return [t]
    cnt = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    cnts = torch.empty(P, dtype=torch.int64, device=t.device)
    comm.all_gather_into_(cnts, cnt)
    sizes = cnts.tolist()
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = torch.empty((P,) + tuple(pad.shape), dtype=t.dtype, device=t.device)
    comm.all_gather_into_(outs, pad)
    return [outs[r, :s] for r, s in enumerate(sizes)]


class GlobalTreeBuilder:
    """The global decomposition on host tensors over gloo (any P <= 64): the schedule of the
    native builder with torch code for the per-rank steps. GPU builds use
    :class:`~parallel_kd_tree_amd.parallel.native_global.NativeGlobalBuilder`."""

    def __init__(self, n_total: int, dim: int, device: Optional[torch.device] = None, depth0: int = 0,
                 pipeline_k: Optional[int] = None):
        self.P = comm.world()
        self.rank = comm.rank()
        self.device = device if device is not None else torch.device("cpu")
        if self.device.type != "cpu":
            raise ValueError("GlobalTreeBuilder runs on host tensors; GPU builds use NativeGlobalBuilder")
        if self.P > 64:
            raise ValueError("global decomposition supports at most 64 ranks")
        self.n_total, self.dim, self.depth0 = int(n_total), int(dim), int(depth0)
        if self.n_total >= 1 << 32:
            raise ValueError("point ids are 32-bit: at most 2^32 - 1 points")
        if pipeline_k is None:
            pipeline_k = int(os.environ.get("PKD_PIPELINE_K", "-1"))
        self.k = int(pipeline_k)
        self.layout = layout(self.n_total, self.P, self.k)
        self.LL = int(self.layout["LL"])
        self.slot_lo = int(self.layout["share_lo"][self.rank])
        self.n_leaf = int(self.layout["share_n"][self.rank])
        self.top_slots = [int(s) if o < 0 else -1 for s, o in zip(self.layout["top_slot"], self.layout["top_owner"])]

    def read_error(self) -> int:
        return 0

    def _exchange_plan(self, counts: torch.Tensor) -> dict:
        """Split sizes of the exchange from every rank's per-leaf counts [T, 4] (rows, err, id
        base, local points). The matrix is all-gathered, so every rank checks every leaf's
        total against the tree geometry (global_plan::make_plan): a failure raises on all ranks
        together instead of leaving peers blocked inside the exchange."""
        P, T = self.P, int(self.layout["T"])
        full = torch.empty(P * T * 4, dtype=torch.int64)
        comm.all_gather_into_(full, counts.reshape(-1))
        rc, send_rows, send_off, recv_rows, leaf_start = ops.native().global_plan(
            full.tolist(), self.n_total, P, self.k, self.rank)
        if rc != 0:
            raise RuntimeError("global exchange plan: middle-bucket overflow reported by the host path")
        fv = full.view(P, T, 4)
        return {"send_rows": send_rows, "send_off": send_off, "recv_rows": recv_rows,
                "src_base": fv[:, 0, 2].tolist(), "src_n": fv[:, 0, 3].tolist()}

    def build(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0) -> DistTree:
        """Top levels down to depth LL, one count exchange, one all-to-all round per leaf of a
        rank (gloo async work), each leaf subtree built while the next round is in flight."""
        dim, P = self.dim, self.P
        lay = self.layout
        LL, T, R = self.LL, int(lay["T"]), int(lay["R"])
        ops_h = _HostOps
        rows = _to_rows(points.to(torch.float32), ids, id_base)
        n_local = rows.shape[0]
        # 1. bounding box
        if n_local > 0:
            lo = points.amin(0).to(torch.float32)
            hi = points.amax(0).to(torch.float32)
        else:
            lo = torch.full((dim,), float("inf"))
            hi = torch.full((dim,), float("-inf"))
        comm.all_reduce_(lo, dist.ReduceOp.MIN)
        comm.all_reduce_(hi, dist.ReduceOp.MAX)
        root_cell = np.stack([lo.numpy(), hi.numpy()], 1).astype(np.float32)  # [dim][2]
        cells = {0: root_cell}
        node = torch.zeros(n_local, dtype=torch.int64)
        pivots = np.zeros(max(T - 1, 1), dtype=np.uint64)
        top_rows = torch.zeros((max(T - 1, 1), dim + 1), dtype=torch.float32)
        # 2. top levels
        for level in range(LL):
            nodes = 1 << level
            first = nodes - 1
            axis = (self.depth0 + level) % dim
            prev_axis = (self.depth0 + level - 1) % dim
            bins = TOP_BINS // nodes
            params = np.zeros((nodes, 2), dtype=np.float32)
            for j in range(nodes):
                c = cells.get(first + j, root_cell)
                params[j] = make_params(c[axis, 0], c[axis, 1], bins)
            hist = ops_h.route_hist(rows, dim, node, level, pivots, prev_axis, axis, params, bins)
            comm.all_reduce_(hist, dist.ReduceOp.SUM)
            hh = hist.numpy().astype(np.int64).reshape(nodes, bins)
            bstar = np.zeros(nodes, dtype=np.int64)
            cless = np.zeros(nodes, dtype=np.int64)
            sizes = [segment(self.n_total, first + j)[1] for j in range(nodes)]
            for j in range(nodes):
                if sizes[j] <= 0:
                    bstar[j] = -1
                    continue
                r = sizes[j] // 2
                cum = np.cumsum(hh[j])
                if cum[-1] != sizes[j]:
                    raise RuntimeError(f"top level {level} node {first + j}: {cum[-1]} points, expected {sizes[j]}")
                b = int(np.searchsorted(cum, r, side="right"))
                bstar[j] = b
                cless[j] = int(cum[b - 1]) if b > 0 else 0
            mid_local = ops_h.collect_middle(rows, dim, node, level, axis, params, bins,
                                             np.where(bstar < 0, bins + 1, bstar))
            mids = torch.cat(_all_gather_var(mid_local), 0)
            mnode = mids[:, dim + 1].contiguous().view(torch.int32).numpy().astype(np.int64) & 0xFFFFFFFF
            mid_np = mids.numpy()
            for j in range(nodes):
                h = first + j
                if bstar[j] < 0:
                    pivots[h] = np.uint64(0xFFFFFFFFFFFFFFFF)
                    continue
                sel = mid_np[mnode == h]
                keys = composite_u64(sel[:, axis], sel[:, dim].view(np.uint32))
                order = np.argsort(keys, kind="stable")
                t = sizes[j] // 2 - int(cless[j])
                if not (0 <= t < len(order)):
                    raise RuntimeError(f"top level {level} node {h}: middle bucket has {len(order)} points, "
                                       f"rank {t} requested")
                pr = sel[order[t]]
                pivots[h] = keys[order[t]]
                top_rows[h] = torch.from_numpy(pr[:dim + 1].copy())
                cl = cells.get(h, root_cell).copy()
                cr = cl.copy()
                cl[axis, 1] = pr[axis]
                cr[axis, 0] = pr[axis]
                cells[2 * h + 1] = cl
                cells[2 * h + 2] = cr
        # 3. pack by leaf, exchange plan
        last_axis = (self.depth0 + LL - 1) % dim
        send, leaf_rows = ops_h.pack(rows, dim, node, LL, pivots, last_axis)
        counts = torch.zeros((T, 4), dtype=torch.int64)
        counts[:, 0] = leaf_rows
        counts[:, 2] = int(id_base)
        counts[:, 3] = n_local
        plan = self._exchange_plan(counts)
        # 4. my share: the top rows between my leaves, then one round per leaf
        me = self.rank
        a = int(lay["leaf_lo"][me])
        mine = int(lay["leaf_lo"][me + 1]) - a
        tp = torch.empty((self.n_leaf, dim), dtype=torch.float32)
        ti = torch.empty((self.n_leaf,), dtype=torch.int32)
        for h, (s, o) in enumerate(zip(lay["top_slot"], lay["top_owner"])):
            if o == me and s >= 0:
                tp[s - self.slot_lo] = top_rows[h, :dim]
                ti[s - self.slot_lo] = top_rows[h, dim:].contiguous().view(torch.int32)

        def issue(j):
            parts = [send[o:o + r] for o, r in zip(plan["send_off"][j], plan["send_rows"][j])]
            inp = torch.cat(parts, 0) if parts else send[:0]
            recv = torch.empty((sum(plan["recv_rows"][j]), dim + 1), dtype=torch.float32)
            hd = comm.all_to_all_single_async(recv, inp.contiguous(), plan["recv_rows"][j], plan["send_rows"][j])
            return recv, [hd]

        def consume(j, recv):
            if j >= mine:
                return
            t = a + j
            n_j = int(lay["leaf_n"][t])
            if n_j > 0:
                o = int(lay["leaf_slot"][t]) - self.slot_lo
                tp[o:o + n_j], ti[o:o + n_j] = ops.build_cpu(recv[:, :dim].contiguous(),
                                                             recv[:, dim].contiguous().view(torch.int32), "exact",
                                                             self.depth0 + LL, 1)

        _run_rounds(R, issue, consume)
        return DistTree(self.n_total, dim, self.depth0, P, me, tp, ti, self.slot_lo, list(self.top_slots),
                        top_rows[: max(T - 1, 0)], {}, lay)
