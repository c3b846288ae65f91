"""Global decomposition: ONE exact kd-tree over P ranks (P a power of two).

North-star design (BASELINE.json): the reference's forest of independent per-rank trees
(kdtree_mpi.cpp:204-253) becomes a single distributed tree:

1. bounding box: allreduce MIN / MAX of the per-rank boxes;
2. top log2(P) levels, level by level: every rank histograms its points (routed below the
   pivots decided so far) into linear buckets of its node's cell, the histograms are
   allreduced (SUM), the bucket holding each node's median is found, the few points of that
   bucket are all-gathered and ranked under the (key, id) order -> the exact pivot point of
   every node at that level, identical on every rank;
3. one all-to-all: every point goes to the rank owning its top-level leaf (rank r owns heap
   node P-1+r), pivots stay replicated;
4. each rank builds its subtree (depth log2 P) with the single-GPU builder.

The result is slot-for-slot the tree a single GPU builds on the concatenated points.
Communication uses torch.distributed: backend "nccl" (= RCCL over xGMI) on MI355X, "gloo" in
CPU tests, where the per-rank device ops run as torch code with identical arithmetic.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..utils.trace import trace_range
from . import comm
from .geometry import composite_u64, make_params, median_slot, segment

TOP_BINS = 8192  # nodes * bins per top level (LDS histogram in the kernel)
DONE = 0xFFFFFFFF


def _to_rows(points: torch.Tensor, ids: Optional[torch.Tensor], id_base: int) -> torch.Tensor:
    n, dim = points.shape
    if ids is None:
        ids = (torch.arange(n, dtype=torch.int64, device=points.device) + int(id_base)).to(torch.int32)
    rows = torch.empty((n, dim + 1), dtype=torch.float32, device=points.device)
    rows[:, :dim] = points
    rows[:, dim] = ids.to(torch.int32).view(torch.float32)
    return rows


def _signed_keys(rows: torch.Tensor, dim: int, axis: int) -> torch.Tensor:
    """Composite keys as int64 with the top bit flipped, so signed order == unsigned order."""
    kb = rows[:, axis].contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ok = torch.where((kb & 0x80000000) != 0, (~kb) & 0xFFFFFFFF, kb | 0x80000000)
    ib = rows[:, dim].contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return ((ok ^ 0x80000000) << 32) | ib


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
    def pack(rows, dim, node, levels, pivots_u64, last_axis, P, k):
        """Rows sorted by destination slot (round j, rank r) -> j * P + r, where rank r owns the
        2^k leaves r * 2^k + j at depth log2(P) + k (dest_slot in csrc/gpu/dist_ops.hip)."""
        piv = torch.tensor([_u64_to_signed(int(v)) for v in pivots_u64], dtype=torch.int64)
        _route_cpu(rows, dim, node, piv, last_axis)
        live = (node != DONE).nonzero().flatten()
        leaves = P << k
        leaf = node[live] - (leaves - 1)
        dest = (leaf & ((1 << k) - 1)) * P + (leaf >> k)
        order = torch.sort(dest, stable=True).indices
        return rows[live[order]].contiguous(), torch.bincount(dest, minlength=leaves).to(torch.int64)


@dataclass
class DistTree:
    """A rank's share of the global tree plus the replicated top tree."""
    n_total: int
    dim: int
    depth0: int
    P: int
    rank: int
    tree_pts: torch.Tensor           # this rank's subtree (in-order), slots [slot_lo, slot_lo + n)
    tree_ids: torch.Tensor
    slot_lo: int
    top_slots: List[int] = field(default_factory=list)
    top_rows: Optional[torch.Tensor] = None   # [P-1, dim+1] pivot rows, heap order
    timings: Dict[str, float] = field(default_factory=dict)

    def gather_full(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Assemble the whole in-order tree on every rank (for checks and small N)."""
        dev = self.tree_pts.device
        rows = torch.empty((self.tree_pts.shape[0], self.dim + 1), dtype=torch.float32, device=dev)
        rows[:, :self.dim] = self.tree_pts
        rows[:, self.dim] = self.tree_ids.view(torch.float32)
        parts = _all_gather_var(rows)
        full = torch.empty((self.n_total, self.dim + 1), dtype=torch.float32, device=dev)
        for r, part in enumerate(parts):
            lo, _ = segment(self.n_total, self.P - 1 + r)
            full[lo:lo + part.shape[0]] = part
        if self.top_rows is not None:
            for i, s in enumerate(self.top_slots):
                if s >= 0:
                    full[s] = self.top_rows[i].to(dev)
        return full[:, :self.dim].contiguous(), full[:, self.dim].contiguous().view(torch.int32)

    def query_packed(self, queries: torch.Tensor, method: str = "auto") -> torch.Tensor:
        """Exact NN over the whole distributed tree: local subtree + top pivots, MIN-reduced."""
        from ..models.kdtree import KDTree
        local = KDTree(self.tree_pts, self.tree_ids, self.depth0 + int(math.log2(self.P)))
        packed = _local_packed(local, queries, method)
        if self.top_rows is not None and self.rank == 0:
            valid = [i for i, s in enumerate(self.top_slots) if s >= 0]
            if valid:
                tr = self.top_rows[valid].to(packed.device)
                pk = _brute_packed(tr[:, :self.dim].contiguous(), tr[:, self.dim].contiguous().view(torch.int32),
                                   queries.to(packed.device))
                packed = torch.minimum(packed, pk)
        return comm.min_packed_(packed)


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
    """Packed (d2, id) minimum over a small point set (the replicated top pivots)."""
    if pts.is_cuda:
        return ops.nn_gpu(pts, ids, queries.to(pts.device, torch.float32), "brute")
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
    """The exchange schedule shared by the device and host paths: round j's all-to-all is
    waited for, round j + 1's is started, and only then is round j's payload consumed (its
    leaf subtree built), so every exchange but the first overlaps a build. ``issue(j)`` returns
    ``(payload, handles)``; a handle is an async work object or None (already complete)."""
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
    """Builds the global tree; reusable across builds of the same (n_total, dim).

    On GPU every top-level decision is made on the device (csrc/gpu/dist_ops.hip): per level
    one route+histogram pass, an allreduce(SUM) of the histogram, the median bucket per node,
    one compaction pass of that bucket, a fixed-size all-gather of the compacted rows and a
    radix select of the exact pivot. Nothing is read back until the all-to-all needs its split
    sizes. Host tensors (gloo tests) take the torch reference path with the same arithmetic.
    """

    def __init__(self, n_total: int, dim: int, device: Optional[torch.device] = None, depth0: int = 0,
                 timings: bool = False):
        self.P = comm.world()
        self.rank = comm.rank()
        if self.P & (self.P - 1):
            raise ValueError(f"global decomposition needs a power-of-two world size, got {self.P}")
        if self.P > 64:
            raise ValueError("global decomposition supports at most 64 ranks")
        self.L = int(math.log2(self.P))
        self.n_total, self.dim, self.depth0 = int(n_total), int(dim), int(depth0)
        if self.n_total >= 1 << 32:
            raise ValueError("point ids are 32-bit: at most 2^32 - 1 points")
        self.device = device if device is not None else comm.device()
        leaf = self.P - 1 + self.rank
        self.slot_lo, self.n_leaf = segment(self.n_total, leaf)
        self.top_slots = [median_slot(self.n_total, h) if segment(self.n_total, h)[1] > 0 else -1
                          for h in range(self.P - 1)]
        self.record_timings = timings
        self._builder = None
        self._ws: Dict[str, torch.Tensor] = {}
        self._scale = 1
        self._leaf_builders: Dict[tuple, object] = {}  # pipelined exchange: leaf builders, pivot slots
        self._main_used = False  # the one-round exchange's builder has built at least once
        if self.device.type == "cuda" and self.n_leaf > 0:
            self._builder = ops.GpuTreeBuilder(self.n_leaf, dim, depth0 + self.L)

    def read_error(self) -> int:
        """Device error word of the last build (0 = ok): the local subtree build's, plus 8 if the
        compact exchange's id bitmaps disagreed with the received row counts. Synchronises."""
        e = self._builder.read_error() if (self._builder is not None and self._main_used) else 0
        for b in self._leaf_builders.values():
            if isinstance(b, ops.GpuTreeBuilder):
                e |= b.read_error()
        if "err" in self._ws:
            e |= int(self._ws["err"][0].item()) & 8
        return e

    # ------------------------------------------------------------------------------------
    def build(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None, id_base: int = 0) -> DistTree:
        if self.device.type == "cuda":
            return self._build_device(points, ids, id_base)
        return self._build_host(points, ids, id_base)

    # ---------------------------------------------------------------- device (HIP + RCCL) path
    def _cap(self, level: int, scale: int) -> int:
        """Middle-bucket rows a rank may contribute at `level` (uniform data: about
        n_total * 2^level / (8192 * P)); overflow is detected and the build retried. Must be
        the same on every rank: it sizes the all-gather."""
        expect = self.n_total * (1 << level) // (TOP_BINS * self.P) + 1
        return int(min(max(2048, 3 * expect) * scale, max(self.n_total, 1)))

    def _buf(self, name: str, shape, dtype) -> torch.Tensor:
        t = self._ws.get(name)
        n = int(np.prod(shape))
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:n].view(shape)

    def _tick(self, timings: Dict[str, float], name: str, t0: List[float]) -> None:
        if self.record_timings:
            torch.cuda.synchronize(self.device)
            now = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + (now - t0[0]) * 1e3
            t0[0] = now

    def pipeline_k(self) -> int:
        """Exchange rounds 2^k per build: each rank's subtree is split k more levels down by
        the distributed top levels, and the leaf subtrees are built one by one while the next
        leaf's rows are in flight. The exchange only dominates at P = 2 (300 MB per direction
        over the one xGMI link between the two GPUs, ~4-5 ms, next to a 7.2 ms local build), so
        P = 2 takes two rounds (half the exchange hidden behind the first leaf's build, for
        ~0.2 ms of extra top level and the slightly lower efficiency of two 25 M builds); at
        P >= 4 the exchange is short and one round is kept. PKD_PIPELINE_K overrides."""
        env = os.environ.get("PKD_PIPELINE_K")
        k = int(env) if env is not None else {2: 1}.get(self.P, 0)
        k = max(0, min(k, 6 - self.L))  # at most 64 leaves (32 nodes per top level)
        if self.P == 1:
            k = 0
        return k

    def _top_device(self, pts, idt, id_base, scale, timings, t0, k):
        nat = ops.native()
        dim, P, L = self.dim, self.P, self.L
        LL, R = L + k, 1 << k
        leaves = P << k
        n_local = pts.shape[0]
        dev = self.device
        box = self._buf("box", (2 * dim,), torch.int64)
        box.fill_(0xFFFFFFFF)
        nat.top_bbox(pts, box)
        comm.all_reduce_(box, dist.ReduceOp.MIN)
        cells = self._buf("cells", ((2 * leaves - 1) * dim * 2,), torch.float32)
        nat.top_root_cell(box, dim, cells)
        node = self._buf("node", (max(n_local, 1),), torch.int32)
        pivots = torch.full((max(leaves - 1, 1),), -1, dtype=torch.int64, device=dev)
        top_rows = torch.zeros((max(leaves - 1, 1), dim + 1), dtype=torch.float32, device=dev)
        err = self._buf("err", (4,), torch.int32)
        err.zero_()
        sel = self._buf("sel", (32 * 4,), torch.int32)
        hist = self._buf("hist", (TOP_BINS,), torch.int32)
        self._tick(timings, "bbox", t0)
        for level in range(LL):
            nodes = 1 << level
            bins = TOP_BINS // nodes
            axis = (self.depth0 + level) % dim
            prev_axis = (self.depth0 + level - 1) % dim
            sizes = [segment(self.n_total, nodes - 1 + j)[1] for j in range(nodes)]
            h = hist[: nodes * bins]
            h.zero_()
            nat.top_route_hist(pts, idt, id_base, node, level, pivots, prev_axis, axis, cells, bins, h)
            comm.all_reduce_(h, dist.ReduceOp.SUM)
            nat.top_select(h, level, bins, sizes, sel, err)
            cap = self._cap(level, scale)
            words = nat.top_middle_words(dim, cap)
            buf = self._buf("mid", (words,), torch.float32)
            nat.top_collect(pts, idt, id_base, node, level, axis, cells, bins, sel, buf, cap)
            gathered = self._buf("gathered", (P * words,), torch.float32)
            comm.all_gather_into_(gathered, buf)
            nat.top_pivot(gathered, P, cap, level, axis, dim, sizes, sel, pivots, top_rows, cells, err)
            self._tick(timings, f"top_level{level}", t0)
        last_axis = (self.depth0 + LL - 1) % dim
        # Compact exchange (implicit ids): 12-B rows plus one bit per (source row, destination);
        # the receiver rebuilds the ids from the bitmaps (csrc/gpu/dist_ops.hip, ids_from_bitmaps).
        compact = idt is None and os.environ.get("PKD_COMPACT_EXCHANGE", "1") != "0"
        rs = dim if compact else dim + 1
        send = self._buf("send_c" if compact else "send", (max(n_local, 1), rs), torch.float32)
        # per destination slot (round j, rank r): rows, err, id base, n_local
        counts = torch.empty(4 * leaves, dtype=torch.int64, device=dev)
        cv = counts.view(leaves, 4)
        cv[:, 2] = int(id_base)
        cv[:, 3] = int(n_local)
        words = max(1, (n_local + 31) // 32)
        bm = self._buf("bm", (leaves, words), torch.int32) if compact else None
        scratch = self._buf("scratch", (nat.top_pack_scratch_bytes(n_local, leaves),), torch.uint8)
        nat.top_pack(pts, idt, id_base, node, LL, pivots, last_axis, leaves, send, bm, counts, err, scratch, k)
        plan = self._exchange_plan(counts, k)  # the only host read-back of the build
        self._tick(timings, "pack", t0)
        if plan is None:
            return None
        ex = {"compact": compact, "rs": rs, "bm": bm, "words": words, "err": err, "R": R, "LL": LL,
              "src_base": plan["src_base"], "src_n": plan["src_n"], "starts": plan["starts"]}
        return send, plan["in_splits"], plan["out_splits"], top_rows, ex

    def _exchange_plan(self, counts: torch.Tensor, k: int) -> Optional[dict]:
        """Split sizes of the exchange from every rank's per-slot counts.

        ``counts`` is int64 [P << k, 4] in destination-slot order (round j, rank r) -> j * P + r:
        rows, error word, id base, local point count. The matrix is all-gathered (P * 2^k * 32 B
        per rank), so every rank sees every rank's error bits and checks every subtree's row
        total against the tree geometry: a failure raises on all ranks together instead of
        leaving peers blocked inside the exchange. Returns None when a top level's middle bucket
        overflowed its all-gather slot (the caller retries with larger slots)."""
        P, R = self.P, 1 << k
        full = torch.empty(P * P * R * 4, dtype=torch.int64, device=counts.device)
        comm.all_gather_into_(full, counts.reshape(-1))
        full = full.cpu().view(P, R, P, 4)  # [source rank][round][destination rank][field]
        errs = 0
        for v in full[..., 1].unique().tolist():
            errs |= int(v)
        if errs & 1:
            # a middle bucket overflowed its all-gather slot: that level's pivot (and every level
            # routed through it, hence a possible err 2 below it) is void; retry larger
            return None
        if errs & 2:
            raise RuntimeError("global top levels: histogram totals disagree with the tree geometry")
        got = full[..., 0].sum(0)  # [round][destination rank]
        for q in range(P):
            for j in range(R):
                want = segment(self.n_total, (P + q) * R - 1 + j)[1]
                if int(got[j, q]) != want:
                    raise RuntimeError(f"global exchange: rank {q} would receive {int(got[j, q])} points in round "
                                       f"{j} for a subtree of {want}")
        me = self.rank
        in_splits = [full[me, j, :, 0].tolist() for j in range(R)]    # rows to each rank in round j
        out_splits = [full[:, j, me, 0].tolist() for j in range(R)]   # rows from each rank in round j
        starts = np.concatenate([[0], np.cumsum([sum(v) for v in in_splits])]).astype(np.int64).tolist()
        return {"in_splits": in_splits, "out_splits": out_splits, "starts": starts,
                "src_base": full[:, 0, 0, 2].tolist(), "src_n": full[:, 0, 0, 3].tolist()}

    def _inner_pivots(self, k: int):
        """(output slots, heap nodes) of the pivots inside this rank's subtree above its 2^k
        pipelined leaves, as device index tensors (geometry only, cached)."""
        key = ("inner", k)
        if key not in self._leaf_builders:
            m = self.P - 1 + self.rank
            inner = [h for lvl in range(k) for h in range((m + 1) * (1 << lvl) - 1, (m + 2) * (1 << lvl) - 1)]
            keep = [(median_slot(self.n_total, h) - self.slot_lo, h) for h in inner if segment(self.n_total, h)[1] > 0]
            if keep:
                si = torch.tensor([a for a, _ in keep], dtype=torch.int64, device=self.device)
                hi = torch.tensor([h for _, h in keep], dtype=torch.int64, device=self.device)
                self._leaf_builders[key] = (si, hi)
            else:
                self._leaf_builders[key] = (None, None)
        return self._leaf_builders[key]

    def _leaf_builder(self, n: int, depth: int):
        b = self._leaf_builders.get((n, depth))
        if b is None:
            b = self._leaf_builders[(n, depth)] = ops.GpuTreeBuilder(n, self.dim, depth)
        return b

    def _build_device(self, points, ids, id_base) -> DistTree:
        dim, P, L = self.dim, self.P, self.L
        timings: Dict[str, float] = {}
        t0 = [time.perf_counter()]
        pts = points.to(self.device, torch.float32).contiguous()
        idt = None if ids is None else ids.to(self.device, torch.int32).contiguous()
        k = self.pipeline_k()
        scale = self._scale  # sticky: a skewed input pays its all-gather retry once, not per build
        while True:
            with trace_range("pkd.dist.top_levels"):
                res = self._top_device(pts, idt, int(id_base), scale, timings, t0, k)
            if res is not None:
                break
            if all(self._cap(l, scale) >= self.n_total for l in range(L + k)):
                raise RuntimeError("global top levels: middle buckets inconsistent at full capacity")
            scale *= 8
        self._scale = scale
        send, in_splits, out_splits, top_rows, ex = res
        R, LL, rs = ex["R"], ex["LL"], ex["rs"]
        src_words = [max(1, (int(v) + 31) // 32) for v in ex["src_n"]]
        bm_off = np.concatenate([[0], np.cumsum(src_words)[:-1]]).astype(np.int64).tolist()
        nat = ops.native()

        def issue(j):
            """Start round j: the rows of leaf j of every rank (+ their id bitmaps)."""
            recv = self._buf(f"recv{j}", (sum(out_splits[j]), rs), torch.float32)
            a, b = ex["starts"][j], ex["starts"][j + 1]
            handles = [comm.all_to_all_single_async(recv, send[a:b], out_splits[j], in_splits[j])]
            recv_bm = None
            if ex["compact"]:
                recv_bm = self._buf(f"recv_bm{j}", (sum(src_words),), torch.int32)
                handles.append(comm.all_to_all_single_async(recv_bm, ex["bm"][j * P:(j + 1) * P].reshape(-1),
                                                            src_words, [ex["words"]] * P))
            return (recv, recv_bm), handles

        def local_tree(recv, recv_bm, j, n_j, builder, out_pts=None, out_ids=None):
            if ex["compact"]:
                off = np.concatenate([[0], np.cumsum(out_splits[j])[:-1]]).astype(np.int64).tolist()
                lids = self._buf("ids", (max(n_j, 1),), torch.int32)[:n_j]
                scr = self._buf("bm_scratch", (nat.ids_from_bitmaps_scratch_bytes(max(src_words), P),), torch.uint8)
                nat.ids_from_bitmaps(recv_bm, off, out_splits[j], bm_off, src_words, ex["src_base"], lids, scr,
                                     ex["err"])
                return builder.build(recv, lids, 0, out_pts, out_ids)
            if out_pts is None:
                return builder.build_rows(recv)
            tp_, ti_ = builder.build_rows(recv)
            out_pts.copy_(tp_)
            out_ids.copy_(ti_)
            return out_pts, out_ids

        with trace_range("pkd.dist.exchange_and_build"):
            if R == 1:
                out = {}

                def consume(j, payload):
                    self._tick(timings, "all_to_all", t0)
                    if self.n_leaf == 0:
                        out["t"] = (torch.empty((0, dim), dtype=torch.float32, device=self.device),
                                    torch.empty((0,), dtype=torch.int32, device=self.device))
                    else:
                        out["t"] = local_tree(payload[0], payload[1], 0, self.n_leaf, self._builder)
                        self._main_used = True

                _run_rounds(1, issue, consume)
                tp, ti = out["t"]
            else:
                # my subtree: node m = P - 1 + rank at depth L; its 2^k leaves at depth LL are the
                # heap nodes first_leaf + j; the R - 1 pivots between them come from top_rows
                m = P - 1 + self.rank
                first_leaf = (m + 1) * R - 1
                tp = torch.empty((self.n_leaf, dim), dtype=torch.float32, device=self.device)
                ti = torch.empty((self.n_leaf,), dtype=torch.int32, device=self.device)
                si, hi = self._inner_pivots(k)
                if si is not None:
                    rows = top_rows[hi]
                    tp[si] = rows[:, :dim]
                    ti[si] = rows[:, dim].contiguous().view(torch.int32)

                def consume(j, payload):
                    recv, recv_bm = payload
                    lo_j, n_j = segment(self.n_total, first_leaf + j)
                    if n_j > 0:
                        a = lo_j - self.slot_lo
                        local_tree(recv, recv_bm, j, n_j, self._leaf_builder(n_j, self.depth0 + LL),
                                   tp[a:a + n_j], ti[a:a + n_j])

                _run_rounds(R, issue, consume)
                self._tick(timings, "all_to_all", t0)
        self._tick(timings, "local_build", t0)
        return DistTree(self.n_total, dim, self.depth0, P, self.rank, tp, ti, self.slot_lo,
                        list(self.top_slots), top_rows[: P - 1], timings)

    # ---------------------------------------------------------------- host (gloo) reference path
    def _build_host(self, points: torch.Tensor, ids: Optional[torch.Tensor], id_base: int) -> DistTree:
        """The torch reference of the device path, same schedule: top levels down to depth
        log2(P) + k, one count exchange, 2^k all-to-all rounds (gloo async work on host
        tensors), each leaf subtree built while the next round is in flight."""
        dim, P, L = self.dim, self.P, self.L
        k = self.pipeline_k()
        LL, R = L + k, 1 << k
        leaves = P << k
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
        pivots = np.zeros(max(leaves - 1, 1), dtype=np.uint64)
        top_rows = torch.zeros((max(leaves - 1, 1), dim + 1), dtype=torch.float32)
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
        # 3. exchange plan: per destination slot (round j, rank r) rows, err, id base, n_local
        last_axis = (self.depth0 + LL - 1) % dim
        send, slot_rows = ops_h.pack(rows, dim, node, LL, pivots, last_axis, P, k)
        counts = torch.zeros((leaves, 4), dtype=torch.int64)
        counts[:, 0] = slot_rows
        counts[:, 2] = int(id_base)
        counts[:, 3] = n_local
        plan = self._exchange_plan(counts, k)
        in_splits, out_splits, starts = plan["in_splits"], plan["out_splits"], plan["starts"]
        # 4. rounds: exchange leaf j + 1 while leaf j's subtree builds
        m = P - 1 + self.rank
        first_leaf = (m + 1) * R - 1
        tp = torch.empty((self.n_leaf, dim), dtype=torch.float32)
        ti = torch.empty((self.n_leaf,), dtype=torch.int32)
        for lvl in range(k):  # pivots inside my subtree above its 2^k leaves
            for h in range((m + 1) * (1 << lvl) - 1, (m + 2) * (1 << lvl) - 1):
                if segment(self.n_total, h)[1] > 0:
                    s_ = median_slot(self.n_total, h) - self.slot_lo
                    tp[s_] = top_rows[h, :dim]
                    ti[s_] = top_rows[h, dim:].contiguous().view(torch.int32)

        def issue(j):
            recv = torch.empty((sum(out_splits[j]), dim + 1), dtype=torch.float32)
            hd = comm.all_to_all_single_async(recv, send[starts[j]:starts[j + 1]], out_splits[j], in_splits[j])
            return recv, [hd]

        def consume(j, recv):
            lo_j, n_j = segment(self.n_total, first_leaf + j)
            if n_j > 0:
                a = lo_j - self.slot_lo
                tp[a:a + n_j], ti[a:a + n_j] = ops.build_cpu(recv[:, :dim].contiguous(),
                                                             recv[:, dim].contiguous().view(torch.int32), "exact",
                                                             self.depth0 + LL, 1)

        _run_rounds(R, issue, consume)
        return DistTree(self.n_total, dim, self.depth0, P, self.rank, tp, ti, self.slot_lo,
                        list(self.top_slots), top_rows[: P - 1], {})
