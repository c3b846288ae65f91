"""kdtree_gpu (single MI355X) prints byte-identical results to the exact CPU executable."""
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def out(exe, args, stdin=None):
    r = subprocess.run([str(exe), *map(str, args)], input=stdin, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return [l for l in r.stdout.splitlines() if not l.startswith("elapsed time")]


@pytest.mark.parametrize("cfg", [(42, 3, 1024), (7, 2, 50000), (3, 8, 200000), (5, 128, 20000), (1, 3, 1)])
def test_gpu_cli_matches_cpu(bin_dir, cfg):
    assert out(bin_dir / "kdtree_gpu", cfg) == out(bin_dir / "kdtree_sequential", cfg)


def test_gpu_cli_eval_mode(bin_dir):
    a = out(bin_dir / "kdtree_gpu", [], stdin="3\n")
    b = out(bin_dir / "kdtree_sequential", ["--threads", "16"], stdin="3\n")
    assert a == b and a[0] == "READY" and a[-1] == "DONE"


@pytest.mark.parametrize("cfg", [(42, 3, 1024), (3, 8, 200000), (1, 3, 1)])
def test_dist_cli_one_rank(bin_dir, cfg):
    """kdtree_dist (native RCCL forest driver, kdtree_mpi.cpp's protocol) with one rank: same
    lines as the CPU executable; the RCCL init / broadcast / reduce path runs for real."""
    assert out(bin_dir / "kdtree_dist", ["--gpus", 1, *cfg]) == out(bin_dir / "kdtree_sequential", cfg)


def test_dist_cli_eval_mode_and_metrics(bin_dir):
    r = subprocess.run([str(bin_dir / "kdtree_dist"), "--gpus", "1", "--metrics-json"], input="3\n",
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    b = out(bin_dir / "kdtree_sequential", ["--threads", "16"], stdin="3\n")
    assert lines == b and lines[0] == "READY" and lines[-1] == "DONE"
    assert '"decomp": "forest"' in r.stderr and '"ranks": 1' in r.stderr


@pytest.mark.parametrize("seed", [3, 42])
@pytest.mark.parametrize("exe", ["kdtree_gpu", "kdtree_dist"])
def test_eval_mode_matches_reference_fixture(bin_dir, exe, seed):
    """The graded evaluation path (seed on stdin, 500k x 128) prints exactly what the real
    reference binary printed (tests/fixtures, pinned against the compiled reference by
    test_reference_parity.py)."""
    from pathlib import Path
    fix = (Path(__file__).parent / "fixtures" / f"ref_eval_seed{seed}.txt").read_text().splitlines()
    args = ["--gpus", 1] if exe == "kdtree_dist" else []
    assert out(bin_dir / exe, args, stdin=f"{seed}\n") == fix


@pytest.mark.parametrize("k", [0, 2])
@pytest.mark.parametrize("cfg", [(42, 3, 1024), (3, 8, 200000), (9, 3, 1_000_003), (5, 128, 20000)])
def test_dist_cli_global_one_rank(bin_dir, cfg, k):
    """kdtree_dist --decomp global (native GlobalBuilder over RCCL: allreduce, allgather and
    grouped send/recv run for real with one rank; --pipeline-k 2 exchanges in 4 rounds and
    builds 4 leaves) prints the same lines as the CPU executable."""
    args = ["--gpus", 1, "--decomp", "global", "--pipeline-k", k, *cfg]
    assert out(bin_dir / "kdtree_dist", args) == out(bin_dir / "kdtree_sequential", cfg)


def test_dist_cli_global_metrics_and_queries(bin_dir):
    r = subprocess.run([str(bin_dir / "kdtree_dist"), "--gpus", "1", "--decomp=global", "--metrics-json",
                        "--queries", "300", "11", "4", "100000"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if not l.startswith("elapsed time")]
    assert lines == out(bin_dir / "kdtree_sequential", ["--queries", 300, 11, 4, 100000])
    assert len(lines) == 302 and '"decomp": "global"' in r.stderr


def test_dist_cli_forest_slices_reuse_workspace_after_misses(bin_dir):
    """kdtree_dist --ranks 4 on one process: four forest slices built one after another on ONE
    shared workspace, every slice's sampled top forced to miss (z = 0.01 bands): each missed slice is redone unsampled and the next slice's sampled builder
    starts on the workspace the miss and its rebuild left. Output equals the CPU executable.
    (The reference stream's 3-D values are near-unique, so the z = 0.01 bands do the missing.)"""
    import os
    cfg = [17, 3, 1_600_000]
    env = dict(os.environ, PKD_AB="1", PKD_TOP_MIN_N="0", PKD_TOP_Z="0.01")
    r = subprocess.run([str(bin_dir / "kdtree_dist"), "--gpus", "1", "--ranks", "4", *map(str, cfg)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if not l.startswith("elapsed time")]
    # the forest's MIN over the ranks' exact trees is the exact NN over all points
    assert lines == out(bin_dir / "kdtree_sequential", cfg)
