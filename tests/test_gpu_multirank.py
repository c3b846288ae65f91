"""The native global decomposition over REAL RCCL with several ranks sharing one card.

The box these run on has one MI355X, and RCCL refuses two ranks on one device ("Duplicate GPU
detected") -- unless every rank looks like its own host: a per-rank NCCL_HOSTID makes RCCL
treat the ranks as separate nodes, which then talk over its socket transport on the loopback
interface. Everything else is the multi-GPU code path as it runs on an 8-GPU node: the same
RCCL communicators (torch's process group plus the builder's own), the same grouped
send/recv all-to-all rounds, allreduces and all-gathers, the same kernels. Only the transport
differs from xGMI. The assembled tree must be slot-for-slot the single-process exact tree and
queries must equal brute force."""
import json
import os
import subprocess
import sys
import time
import traceback
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

from test_distributed_cpu import _free_port

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _worker(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      NCCL_HOSTID=f"pkd-test-rank{rank}", NCCL_SOCKET_IFNAME="lo")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    try:
        torch.set_num_threads(1)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        from parallel_kd_tree_amd.parallel import comm
        comm.init(backend="nccl", device=dev, timeout_s=150)
        fn(rank, world, *args)
        comm.barrier()
        comm.destroy()
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))


def run_rccl(world, fn, *args):
    """`world` ranks on cuda:0, each its own RCCL 'host'; fails if any rank fails."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    errs = []
    try:
        for _ in range(world):
            errs.append(q.get(timeout=100))
    except Exception:  # a rank died or hangs in a collective: end the group instead of hanging
        for p in procs:
            if p.is_alive():
                p.kill()
        raise AssertionError(f"only {len(errs)} of {world} ranks finished: {[e for _, e in errs if e]}")
    for p in procs:
        p.join(60)
    bad = [e for _, e in errs if e]
    assert not bad, bad[0]


def _case(rank, world, n, dim, seed, dupes, k=-1):
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.native_global import NativeGlobalBuilder
    dev = torch.device("cuda", 0)
    first, cnt = comm.forest_slice(n, world, rank)
    if dupes:
        g = torch.Generator().manual_seed(seed)
        full = torch.randint(0, 3, (n + 10, dim), generator=g).float()
    else:
        full = pk.generate_problem(seed, dim, n + 10)
    x = full[first:first + cnt].to(dev)
    b = NativeGlobalBuilder(n, dim, dev, pipeline_k=k, timeout_s=60)
    b.set_profile(True)
    t = b.build(x, id_base=first + 1)
    t = b.build(x, id_base=first + 1)  # reuse of the builder's buffers
    b.sync()
    assert b.read_error() == 0
    ph = b.phases()
    assert {"top_ms", "pack_ms", "plan_wait_ms", "exchange_ms", "leaf_ms", "total_ms", "sent_bytes"} <= set(ph)
    assert ph["rounds"] == b.layout["R"] and ph["total_ms"] > 0
    assert t.check_top_routing() == ""
    tp, ti = t.gather_full()
    cp, ci = ops.build_cpu(full[:n], None, "exact", 0, 1)
    assert torch.equal(ti.cpu(), ci + 1), f"rank {rank}: global tree differs from the single-process tree"
    assert torch.equal(tp.cpu(), cp)
    q = full[n:].to(dev)
    d2, ids = ops.unpack(t.query_packed(q))
    ref = ((full[:n][None].double() - full[n:][:, None].double()) ** 2).sum(-1).min(1).values
    got = ((full[:n][ids.cpu() - 1].double() - full[n:].double()) ** 2).sum(-1)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("world,n,dim,dupes", [(2, 300_000, 3, False), (4, 400_000, 3, False), (3, 300_001, 3, False),
                                               (4, 50_001, 5, False), (2, 40_000, 2, True), (4, 7, 3, False),
                                               (6, 200_000, 3, False), (8, 800_003, 3, False)])
def test_global_tree_rccl(world, n, dim, dupes):
    run_rccl(world, _case, n, dim, 21, dupes)


@pytest.mark.parametrize("world,k", [(2, 0), (2, 3), (4, 2), (8, 1), (3, 0)])
def test_global_tree_rccl_pipeline_depth(world, k):
    """Extra top levels: every rank's share split into more leaves, each built while the next
    leaf's rows are in flight (k = 0 at a power of two: one all-to-all). Same tree for every k."""
    run_rccl(world, _case, 200_001, 3, 23, False, k)


def _stuck_peer(rank, world):
    """Rank 1 never joins the build: rank 0's bounded wait must give up with a rank-tagged error
    (and abort its communicator) instead of hanging."""
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.native_global import NativeGlobalBuilder
    dev = torch.device("cuda", 0)
    n = 100_000
    first, cnt = comm.forest_slice(n, world, rank)
    x = pk.generate_slice(3, 3, first, cnt, device=dev)
    b = NativeGlobalBuilder(n, 3, dev, timeout_s=4)
    if rank == 1:
        time.sleep(12)
        return
    t0 = time.time()
    with pytest.raises(RuntimeError, match=r"rank 0: .*(watchdog|asynchronous)"):
        b.build(x, id_base=first + 1)
    assert time.time() - t0 < 30


def test_stuck_peer_raises():
    run_rccl(2, _stuck_peer)


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_rccl_share_gpu(gpus):
    """bench.py --gpus N on one card (the rehearsal mode of the driver's multi-GPU run): one JSON
    line from rank 0, the tree checked across ranks, the per-phase breakdown on stderr."""
    env = dict(os.environ, PKD_BENCH_SHARE_GPU="1")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--points", "2000000",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == gpus and line["config"]["parallelism"] == f"global{gpus}"
    assert line["config"]["tree_checked"] and not line["config"]["headline"]
    phases = [json.loads(s) for s in r.stderr.splitlines() if s.startswith('{"phases_max_over_ranks_ms"')]
    assert len(phases) == 1 and phases[0]["phases_max_over_ranks_ms"]["leaf_ms"] > 0


def _routed(rank, world, n, dim, nq):
    """10 000 queries on the distributed tree: each is searched on its home rank, then only where
    its best ball reaches -- brute-force answers with ~1/P of the per-rank query work."""
    import parallel_kd_tree_amd as pk
    from parallel_kd_tree_amd import ops
    from parallel_kd_tree_amd.parallel import comm
    from parallel_kd_tree_amd.parallel.native_global import NativeGlobalBuilder
    dev = torch.device("cuda", 0)
    first, cnt = comm.forest_slice(n, world, rank)
    full = pk.generate_problem(31, dim, n + nq)
    b = NativeGlobalBuilder(n, dim, dev, timeout_s=60)
    t = b.build(full[first:first + cnt].to(dev), id_base=first + 1)
    q = full[n:].to(dev)
    d2, ids = ops.unpack(t.query_packed(q, count_work=True))
    work = t.last_query_work
    d2a, _ = ops.unpack(t.query_packed(q, routed=False))
    assert torch.equal(d2, d2a)
    pts = full[:n].to(dev).double()
    ref = torch.cat([torch.cdist(q[i:i + 500].double(), pts).pow(2).min(1).values for i in range(0, nq, 500)])
    got = ((pts[ids.to(dev) - 1] - q.double()) ** 2).sum(-1)
    assert torch.allclose(got, ref, rtol=0, atol=1e-9)
    tot = torch.tensor([work], dtype=torch.int64, device=dev)
    comm.all_reduce_(tot)
    assert int(tot) < 1.3 * nq, f"{int(tot)} (query, block) searches over {world} ranks for {nq} queries"


@pytest.mark.parametrize("world,dim", [(4, 3), (3, 4)])
def test_routed_queries_rccl(world, dim):
    run_rccl(world, _routed, 400_000, dim, 10_000)


@pytest.mark.parametrize("gpus,dim", [(3, 3), (4, 2)])
def test_kdtree_dist_global_routed_queries_cli(gpus, dim):
    """kdtree_dist --decomp global answers 10 000 queries by the native routed search
    (GlobalBuilder::query: home block, MIN all-reduce, reach blocks, MIN all-reduce) and prints
    exactly what the CPU executable prints."""
    args = ["--queries", "10000", "7", str(dim), "200000"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    g = subprocess.run([str(ROOT / "bin" / "kdtree_dist"), "--gpus", str(gpus), "--share-gpu", "--decomp", "global",
                        *args], capture_output=True, text=True, timeout=300, env=env)
    assert g.returncode == 0, g.stderr[-2000:]
    c = subprocess.run([str(ROOT / "bin" / "kdtree_sequential"), *args], capture_output=True, text=True, timeout=300)
    assert c.returncode == 0, c.stderr[-2000:]
    strip = lambda out: [l for l in out.splitlines() if l.startswith("ID:")]  # noqa: E731
    assert len(strip(g.stdout)) == 10000 and strip(g.stdout) == strip(c.stdout)
