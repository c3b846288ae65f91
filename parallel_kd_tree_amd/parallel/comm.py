"""Communication layer over torch.distributed.

On MI355X the backend is "nccl", which is RCCL over xGMI; CPU tests use "gloo" with the same
code. Rendezvous comes from the torchrun environment (RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT), replacing the reference's MPI_Init / Comm_rank / Comm_size
(kdtree_mpi.cpp:177-183). Every collective here is tiny (config broadcast, MIN reductions,
histograms) except the all-to-all redistribution of the global decomposition.
"""
from __future__ import annotations

import contextlib
import ctypes
import datetime
import os
import sys
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

_device: Optional[torch.device] = None


@contextlib.contextmanager
def stdout_to_stderr():
    """Point fd 1 at stderr (C and C++ stdio included) for the duration of the block: gloo
    ("[Gloo] Rank r is connected ...") and RCCL (its version banner) print on stdout during
    initialisation, and stdout carries only the protocol / the bench JSON line."""
    libc = ctypes.CDLL(None)
    sys.stdout.flush()
    libc.fflush(None)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def init(backend: Optional[str] = None, device: Optional[torch.device] = None, timeout_s: int = 600) -> None:
    """Initialise the default process group from the environment (idempotent). With the
    nccl backend the communicator is created eagerly (device_id), inside the stdout guard."""
    global _device
    if dist.is_initialized():
        return
    if backend is None:
        backend = "nccl" if (device is not None and device.type == "cuda") else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29512")
    kw = {}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    with stdout_to_stderr():
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
        if backend == "nccl":
            # first collective on the communicator: any lazy RCCL setup prints here, not later
            dist.barrier(device_ids=[device.index] if device is not None else None)
    _device = device if device is not None else torch.device("cpu")


def is_initialized() -> bool:
    return dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def device() -> torch.device:
    return _device if _device is not None else torch.device("cpu")


def barrier() -> None:
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device().index])
        else:
            dist.barrier()


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def forest_slice(n: int, p: int, r: int) -> Tuple[int, int]:
    """Rank r's generation-order slice: local = n // p, remainder to the last rank
    (kdtree_mpi.cpp:208-216). Returns (first_row, rows)."""
    local = n // p
    first = local * r
    if r == p - 1:
        local += n % p
    return first, local


def broadcast_ints(vals: List[int], src: int = 0) -> List[int]:
    """MPI_Bcast of the {seed, dim, N} config (kdtree_mpi.cpp:199)."""
    t = torch.tensor(vals, dtype=torch.int64)
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            t = t.to(device())
        dist.broadcast(t, src)
    return [int(v) for v in t.tolist()]


def allreduce_(t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    return all_reduce_(t, op)


def max_float(v: float) -> float:
    t = torch.tensor([v], dtype=torch.float64, device=device())
    allreduce_(t, dist.ReduceOp.MAX)
    return float(t.item())


def min_packed_(packed: torch.Tensor) -> torch.Tensor:
    """MIN-reduce packed (d2 << 32 | id) results. The packing never sets bit 63, so the
    signed int64 MIN equals the unsigned one (reference: MPI_Reduce MIN, kdtree_mpi.cpp:253,
    which drops the id; here the id rides along)."""
    return allreduce_(packed, dist.ReduceOp.MIN)


# ---- collectives used by the global decomposition ---------------------------------------
# RCCL ("nccl") takes device tensors directly. gloo (CPU tests, and the multi-rank GPU tests
# that run every rank on one card) only gets host tensors: device tensors are staged.
def _staged(t: torch.Tensor) -> bool:
    return t.is_cuda and dist.get_backend() == "gloo"


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if not dist.is_initialized() or world() == 1:
        return t
    if _staged(t):
        c = t.cpu()
        dist.all_reduce(c, op=op)
        t.copy_(c)
    else:
        dist.all_reduce(t, op=op)
    return t


def all_gather_into_(out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """out[r * t.numel():(r + 1) * t.numel()] = t of rank r (fixed-size all-gather)."""
    P = world()
    if not dist.is_initialized() or P == 1:
        out.view(-1)[: t.numel()].copy_(t.view(-1))
        return out
    if _staged(t) or dist.get_backend() == "gloo":
        c = t.cpu().contiguous()
        parts = [torch.empty_like(c) for _ in range(P)]
        dist.all_gather(parts, c)
        out.view(-1).copy_(torch.cat([p.view(-1) for p in parts]))
    else:
        dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1))
    return out


class _StagedWork:
    """Handle of an all-to-all on host copies of device tensors (gloo): the exchange runs
    asynchronously on gloo's thread; wait() joins it and copies the result to the device."""

    def __init__(self, work, host_out: torch.Tensor, out: torch.Tensor):
        self._work, self._host_out, self._out = work, host_out, out

    def wait(self) -> bool:
        self._work.wait()
        self._out.copy_(self._host_out)
        return True

    def is_completed(self) -> bool:
        return self._work.is_completed()


def all_to_all_single_async(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None):
    """Starts an all-to-all and returns a handle whose wait() orders the caller's current
    stream after it (RCCL runs it on its own stream, overlapping later compute; gloo runs it
    on its own thread, device tensors staged through host copies). With one rank there is
    nothing to overlap: the copy is done and the handle is None."""
    if not dist.is_initialized() or world() == 1:
        all_to_all_single_(out, inp, out_splits, in_splits)
        return None
    if _staged(inp):
        host_out = torch.empty(out.shape, dtype=out.dtype)
        w = dist.all_to_all_single(host_out, inp.cpu(), out_splits, in_splits, async_op=True)
        return _StagedWork(w, host_out, out)
    return dist.all_to_all_single(out, inp, out_splits, in_splits, async_op=True)


def all_to_all_single_(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> torch.Tensor:
    if not dist.is_initialized() or world() == 1:
        out.copy_(inp)
        return out
    if _staged(inp):
        co = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(co, inp.cpu(), out_splits, in_splits)
        out.copy_(co)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits)
    return out
