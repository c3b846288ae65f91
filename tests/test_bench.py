"""bench.py driver contract on the CPU: one JSON line from rank 0, self-launch of N ranks
without torchrun (the reference's `mpirun -np P`, Makefile:36), failure propagation."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench(*args, env=None, timeout=300):
    e = dict(os.environ, PKD_SKIP_BUILD="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _one_json(stdout):
    lines = [l for l in stdout.splitlines() if l.strip()]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_single_cpu():
    r = _bench("--device", "cpu", "--points", "100000", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stderr
    j = _one_json(r.stdout)
    assert j["n_gpus"] == 1 and j["steps"] == 2 and j["warmup"] == 1 and j["config"]["n_points"] == 100000
    assert j["config"]["tree_checked"] and j["higher_is_better"] and j["unit"] == "Mpoints/s"


def test_bench_self_launch_two_ranks():
    """No WORLD_SIZE in the env: bench.py spawns its ranks itself; rank 0 alone prints."""
    r = _bench("--gpus", "2", "--device", "cpu", "--points", "60000", "--steps", "1", "--warmup", "1")
    assert r.returncode == 0, r.stderr
    j = _one_json(r.stdout)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "global2" and j["config"]["tree_checked"]


def test_bench_self_launch_four_ranks_pipelined():
    r = _bench("--gpus", "4", "--device", "cpu", "--points", "40001", "--steps", "1", "--warmup", "0",
               "--pipeline-k", "1")
    assert r.returncode == 0, r.stderr
    assert _one_json(r.stdout)["n_gpus"] == 4


def test_bench_three_ranks():
    """A world size that is not a power of two: uneven leaf runs, same checked tree."""
    r = _bench("--gpus", "3", "--device", "cpu", "--points", "30001", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr
    j = _one_json(r.stdout)
    assert j["n_gpus"] == 3 and j["config"]["parallelism"] == "global3" and j["config"]["tree_checked"]
    assert "(not the headline config)" in j["metric"] and j["config"]["headline"] is False
    # a host rehearsal is labelled as one, never as a GPU measurement
    assert "rehearsal" in j["metric"] and j["config"]["shared_gpu"] is False


def test_bench_headline_rehearsal_is_labelled():
    """The headline config run as a host (gloo) rehearsal: same metric stem, but labelled and
    headline false, so it can never pass for the 100 M x 3D measurement."""
    r = _bench("--gpus", "2", "--device", "cpu", "--points", "20000", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr
    j = _one_json(r.stdout)
    assert j["config"]["headline"] is False and "rehearsal" in j["metric"]


def test_bench_launcher_propagates_rank_failure():
    """A dead rank ends the job with a non-zero status and no JSON line (the other rank,
    blocked in a collective, is stopped by the launcher)."""
    r = _bench("--gpus", "2", "--device", "cpu", "--points", "20000", "--steps", "1", "--warmup", "0",
               env={"PKD_BENCH_FAIL_RANK": "1"}, timeout=200)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "rank 1 exited with 7" in r.stderr


def test_bench_world_mismatch_rejected():
    r = _bench("--gpus", "2", "--device", "cpu", env={"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_builds_in_launcher_before_ranks():
    """The self-launcher brings the build up to date before any rank exists; the ranks then only
    verify signatures (no compile, O(1) work) before they join the communicator."""
    r = _bench("--gpus", "2", "--device", "cpu", "--points", "20000", "--steps", "1", "--warmup", "0",
               env={"PKD_SKIP_BUILD": "0", "PKD_BENCH_TRACE_BUILD": "1"}, timeout=1200)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stderr.splitlines() if l.startswith("bench.py:") and ": build " in l]
    assert lines and lines[0].startswith("bench.py: launcher: build"), r.stderr
    ranks = [l for l in lines if l.startswith("bench.py: rank ")]
    assert len(ranks) == 2, r.stderr
    for l in ranks:
        assert "build up to date" in l, l
        ms = float(l.rsplit("(", 1)[1].split(" ms")[0])
        assert ms < 20_000, l
