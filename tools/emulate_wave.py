"""CPU emulation of wave_build (csrc/gpu/build_subtree.hip) — lanes as numpy vectors.
Used to debug the wave-level subtree builder without a GPU."""
import numpy as np
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DONE = 0xFFFF
MID = 0x8000
KSMALL = 16


def orderable(f):
    b = np.asarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return np.where(b & 0x80000000, (~b) & 0xFFFFFFFF, b | 0x80000000).astype(np.uint64)


def pow2_floor(v):
    return 1 if v <= 1 else 1 << (int(v).bit_length() - 1)


def make_params(lo, hi, nb):
    span = np.float32(hi) - np.float32(lo)
    return np.float32(lo), (np.float32(nb) / span if span > 0 else np.float32(0))


def bucket_of(x, lo, sc, nb):
    t = (np.float32(x) - lo) * sc
    t = np.minimum(np.maximum(np.nan_to_num(t, nan=0.0), 0), nb - 1)
    return t.astype(np.uint32)


def wave_build(rows, n0, dim, depth0, cell0):
    """rows: [dim+1, n0] float32 (row dim = id bits). Returns slot order (in-order idx)."""
    ln = np.arange(64)
    slot = np.zeros(n0, dtype=np.uint64)
    slot[:] = np.arange(n0)
    wsub = np.zeros(max(n0, 1), dtype=np.uint64)
    wsub[0] = n0
    ids = rows[dim].view(np.uint32).astype(np.uint64)
    wcA = np.zeros((16, dim, 2), np.float32); wcB = np.zeros((16, dim, 2), np.float32)
    wcA[0] = cell0
    WI = 4
    t = 0
    while True:
        m = n0 >> t
        if m == 0:
            break
        S = 1 << t
        axis = (depth0 + t) % dim
        kcol = rows[axis]
        more = (n0 >> (t + 1)) > 0
        q = ln[None, :] + 64 * np.arange(WI)[:, None]      # [WI, 64]
        sl = np.where(q < n0, slot[np.minimum(q, n0 - 1)], DONE << 16).astype(np.uint64)
        sid = (sl >> 16).astype(np.int64)
        act = sid != DONE
        idx = (sl & 0xFFFF).astype(np.int64)
        kf = np.where(act, kcol[np.minimum(idx, n0 - 1)], 0).astype(np.float32)
        ev = [wsub[j] if (more and j < S) else 0 for j in range(S)]
        np_ = np.full((WI, 64), -1, np.int64); ns = np.zeros((WI, 64), np.uint64)
        if m > KSMALL:
            B = min(64, max(2, pow2_floor(m // 2)))
            plo = np.zeros(16, np.float32); psc = np.zeros(16, np.float32)
            for j in range(S):
                plo[j], psc[j] = make_params(wcA[j, axis, 0], wcA[j, axis, 1], B)
            hist = np.zeros(S * B, np.int64)
            bk = np.zeros((WI, 64), np.int64)
            for k in range(WI):
                for l in range(64):
                    if act[k, l]:
                        s_ = sid[k, l]
                        bk[k, l] = int(bucket_of(kf[k, l], plo[s_], psc[s_], B))
                        hist[s_ * B + bk[k, l]] += 1
            bst = np.zeros(16, np.int64); cle = np.zeros(16, np.int64); cmi = np.zeros(16, np.int64)
            for j in range(S):
                r = int(wsub[j] & 0xFFFF) // 2
                c = 0
                for b in range(B):
                    v = hist[j * B + b]
                    if r < c + v:
                        bst[j], cle[j], cmi[j] = b, c, v
                        break
                    c += v
            z = np.full((WI, 64), 3)
            for k in range(WI):
                for l in range(64):
                    if act[k, l]:
                        bs = bst[sid[k, l]]
                        z[k, l] = 0 if bk[k, l] < bs else (1 if bk[k, l] == bs else 2)
            run = [0, 0, 0]
            pz = np.zeros((WI, 64), np.int64)
            bas = np.zeros((3, 16), np.int64)
            for k in range(WI):
                masks = [z[k] == zz for zz in range(3)]
                pre = [run[zz] + np.concatenate([[0], np.cumsum(masks[zz])[:-1]]) for zz in range(3)]
                for l in range(64):
                    if z[k, l] < 3:
                        pz[k, l] = pre[z[k, l]][l]
                        s_ = sid[k, l]
                        if l + 64 * k == int(wsub[s_] >> 16):
                            for zz in range(3):
                                bas[zz, s_] = pre[zz][l]
                for zz in range(3):
                    run[zz] += int(masks[zz].sum())
            for k in range(WI):
                for l in range(64):
                    zz = z[k, l]
                    if zz < 3:
                        s_ = sid[k, l]
                        start = 0 if zz == 0 else (cle[s_] if zz == 1 else cle[s_] + cmi[s_])
                        np_[k, l] = int(wsub[s_] >> 16) + start + pz[k, l] - bas[zz, s_]
                        nsid = 2 * s_ if zz == 0 else (2 * s_ + 1 if zz == 2 else (MID | s_))
                        ns[k, l] = idx[k, l] | (nsid << 16)
            for k in range(WI):
                for l in range(64):
                    if np_[k, l] >= 0:
                        slot[np_[k, l]] = ns[k, l]
            np_[:] = -1
            for k in range(WI):
                for l in range(64):
                    qq = l + 64 * k
                    if qq >= n0:
                        continue
                    s = int(slot[qq]); tag = s >> 16
                    if tag != DONE and (tag & MID):
                        s_ = tag & 0x7FFF; ix = s & 0xFFFF
                        e = int(wsub[s_]); jn = e & 0xFFFF
                        zlo = (e >> 16) + cle[s_]; zc = cmi[s_]
                        mk = int(orderable(kcol[ix])); mid = int(ids[ix])
                        rank = 0
                        for r in range(zc):
                            o = int(slot[zlo + r]) & 0xFFFF
                            qk = int(orderable(kcol[o])); qi = int(ids[o])
                            rank += (qk < mk or (qk == mk and qi < mid))
                        tt = jn // 2 - cle[s_]
                        nsid = 2 * s_ if rank < tt else (2 * s_ + 1 if rank > tt else DONE)
                        np_[k, l] = zlo + rank; ns[k, l] = ix | (nsid << 16)
                        if rank == tt and more:
                            wcB[2 * s_] = wcA[s_]; wcB[2 * s_ + 1] = wcA[s_]
                            wcB[2 * s_, axis, 1] = kcol[ix]; wcB[2 * s_ + 1, axis, 0] = kcol[ix]
            wcA, wcB = wcB, wcA
        else:
            keyv = np.zeros(n0, np.uint64)
            for k in range(WI):
                for l in range(64):
                    if act[k, l]:
                        keyv[l + 64 * k] = orderable(kf[k, l])
            for k in range(WI):
                for l in range(64):
                    if not act[k, l]:
                        continue
                    s_ = sid[k, l]; ix = idx[k, l]
                    e = int(wsub[s_]); jlo = e >> 16; jn = e & 0xFFFF
                    mk = int(orderable(kf[k, l])); mid = int(ids[ix])
                    rank = 0
                    for r in range(jn):
                        qk = int(keyv[jlo + r])
                        if qk < mk or (qk == mk and jlo + r != l + 64 * k and ids[int(slot[jlo + r]) & 0xFFFF] < mid):
                            rank += 1
                    half = jn // 2
                    nsid = 2 * s_ if rank < half else (2 * s_ + 1 if rank > half else DONE)
                    np_[k, l] = jlo + rank; ns[k, l] = ix | (nsid << 16)
        for k in range(WI):
            for l in range(64):
                if np_[k, l] >= 0:
                    slot[np_[k, l]] = ns[k, l]
        if more:
            for j in range(S):
                lo, mm = int(ev[j]) >> 16, int(ev[j]) & 0xFFFF
                mr = mm - mm // 2 - 1 if mm >= 1 else 0
                wsub[2 * j] = (lo << 16) | (mm // 2)
                wsub[2 * j + 1] = ((lo + mm // 2 + 1) << 16) | mr
        t += 1
    return (slot & 0xFFFF).astype(np.int64)


if __name__ == "__main__":
    import torch
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    for n in [17, 33, 60, 100, 200, 256]:
        x = pk.generate_problem(n, 3, n)
        rows = np.zeros((4, n), np.float32)
        rows[:3] = x.numpy().T
        rows[3] = np.arange(n, dtype=np.uint32).view(np.float32)
        cell = np.stack([x.numpy().min(0), x.numpy().max(0)], 1)
        order = wave_build(rows, n, 3, 0, cell)
        _, ci = ops.build_cpu(x, None, "exact", 0, 1)
        print(n, "emu == cpu:", np.array_equal(order, ci.numpy()))
