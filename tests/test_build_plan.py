"""The GPU builder's level plan, checked on the host (no GPU needed: the plan is made when a
GpuTreeBuilder is constructed, csrc/gpu/build_global.hip make_plan). Guards the round-6 choices:
the 4-level tail at dims 4..8 where it saves a row-moving pass (100 M x 8D: three triples and a
4-level tail, no pair pass), sampled triples at dims 2..8, and the knobs that switch them off."""
import importlib

import pytest

from parallel_kd_tree_amd import ops


def _plan(n, dim, depth0=0):
    lines = ops.GpuTreeBuilder(n, dim, depth0, 0).describe().split("\n")[1:]
    return {
        "tail": sum(" tail" in ln for ln in lines),
        "pair_passes": sum(" pair" in ln for ln in lines),
        "triples": sum(" triple" in ln for ln in lines),
        "g3": sum(" g3" in ln for ln in lines),
        "sampled_top": sum(" sampled" in ln for ln in lines),
        "levels": len(lines),
    }


@pytest.fixture
def ab(monkeypatch):
    monkeypatch.setenv("PKD_AB", "1")
    yield monkeypatch
    importlib.import_module("parallel_kd_tree_amd.ops.build")._builders.clear()


def test_headline_plan_3d():
    p = _plan(100_000_000, 3)
    assert p["levels"] == 16 and p["sampled_top"] == 4
    assert p["tail"] == 3 and p["triples"] == 3 and p["g3"] == 2 and p["pair_passes"] == 0


def test_8d_plan_has_no_pair_pass():
    p = _plan(100_000_000, 8)
    assert p["levels"] == 17 and p["sampled_top"] == 4
    assert p["tail"] == 4 and p["triples"] == 3 and p["pair_passes"] == 0
    assert p["g3"] == 2  # sampled triples at levels 4-6 and 7-9 (rows of <= 8 dims)


def test_tail4_off_brings_the_pair_back(ab):
    ab.setenv("PKD_TAIL4", "0")
    p = _plan(100_000_000, 8)
    assert p["tail"] == 3 and p["pair_passes"] > 0


@pytest.mark.parametrize("n,dim", [(100_000_000, 4), (100_000_000, 5), (100_000_000, 6), (10_000_000, 8),
                                   (1_500_001, 8), (2_000_000, 5)])
def test_tail4_saves_a_pass(ab, n, dim):
    """Wherever the 4-level tail is planned, the plan has fewer row-moving passes than without it."""
    def passes(p):  # top (one pass), each triple, each pair, the tail
        return (1 if p["sampled_top"] else 0) + p["triples"] + p["pair_passes"] + (1 if p["tail"] else 0)

    p4 = _plan(n, dim)
    if p4["tail"] != 4:
        pytest.skip("no 4-level tail planned at this size")
    ab.setenv("PKD_TAIL4", "0")
    p3 = _plan(n, dim)
    assert p3["tail"] == 3
    # a pair pass counts as a pass of its own; a triple covers three levels, so compare levels per pass
    assert passes(p4) <= passes(p3)
    assert p4["pair_passes"] <= p3["pair_passes"]


def test_3d_keeps_the_3_level_tail():
    for n in (100_000_000, 12_500_000, 1_000_000_000):
        assert _plan(n, 3)["tail"] in (0, 3)


def test_g3_max_dim_knob(ab):
    assert _plan(100_000_000, 5)["g3"] == 2
    ab.setenv("PKD_G3_MAX_DIM", "3")
    assert _plan(100_000_000, 5)["g3"] == 0
    assert _plan(100_000_000, 3)["g3"] == 2
