"""On-disk tree layout.

The reference never serialises its tree; the natural layout is the implicit
in-order permutation (F3), i.e. exactly the reference's post-build ``point_list`` order.
File = little-endian header + ids (uint32[n]) + coords (float32[n * dim]), slot order:

    magic  b"PKDTREE\\x01"  (8 bytes)
    u32    version (1)
    u32    dim
    u64    n
    u32    depth0      depth of slot range [0, n) (0 for whole trees)
    u32    mode        0 = exact (key, id) order, 1 = reference (sort-first-n-1) tree
    u64    reserved
"""
from __future__ import annotations

import struct
from pathlib import Path

import numpy as np
import torch

MAGIC = b"PKDTREE\x01"
_HDR = struct.Struct("<8sIIQIIQ")
MODES = {"exact": 0, "reference": 1}


def save_tree(path, tree_pts: torch.Tensor, tree_ids: torch.Tensor, depth0: int = 0, mode: str = "exact"):
    pts = tree_pts.detach().to("cpu", torch.float32).contiguous().numpy()
    ids = tree_ids.detach().to("cpu", torch.int32).contiguous().numpy().view(np.uint32)
    n, dim = pts.shape
    with open(path, "wb") as f:
        f.write(_HDR.pack(MAGIC, 1, dim, n, int(depth0), MODES[mode], 0))
        f.write(ids.astype("<u4", copy=False).tobytes())
        f.write(pts.astype("<f4", copy=False).tobytes())


def load_tree(path):
    """Returns (tree_pts float32 [n, dim], tree_ids int32 [n], depth0, mode). Memory-maps."""
    path = Path(path)
    with open(path, "rb") as f:
        magic, ver, dim, n, depth0, mode, _ = _HDR.unpack(f.read(_HDR.size))
    if magic != MAGIC or ver != 1:
        raise ValueError(f"{path}: not a pkdtree file")
    ids = np.memmap(path, dtype="<u4", mode="r", offset=_HDR.size, shape=(n,))
    pts = np.memmap(path, dtype="<f4", mode="r", offset=_HDR.size + 4 * n, shape=(n, dim))
    inv = {v: k for k, v in MODES.items()}
    return (torch.from_numpy(np.array(pts)), torch.from_numpy(np.array(ids).view(np.int32)), int(depth0),
            inv[int(mode)])
