"""bench.py's host logic (no GPU): the weak-scaling shapes, the closed forms
every step is checked against (against the oracle on small sums), the
roofline byte model and the kernel names the roofline line reports."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_weak_scaling_shapes_hold_2_30_positions_per_gpu():
    for n in (1, 2, 4, 8):
        heaps = bench.heaps_for(n)
        P, E, _ = bench.expected(heaps)
        assert P == n << 30
    assert bench.heaps_for(1) == [31] * 6
    with pytest.raises(SystemExit):
        bench.heaps_for(3)


@pytest.mark.parametrize("heaps", [[3, 3, 3], [2, 5, 7], [4, 4, 4], [6, 6, 6, 6], [1, 1], [0, 5]])
def test_closed_forms_match_the_oracle(heaps):
    from oracle.oracle import Game  # checker only
    P, E, root = bench.expected(heaps)
    sol = Game("sum_four_to_one", "heaps=" + ":".join(map(str, heaps))).solve(1 << 20)
    assert (sol.count, sol.edges, sol.root_line.split()[0]) == (P, E, root)


def test_scaling_workloads_have_goldens():
    """Every bench shape N = 1, 2, 4, 8 has a whole-solve golden (the N > 1
    steps check their root line against it) whose counts and root value are
    the closed forms'."""
    for n in (1, 2, 4, 8):
        heaps = bench.heaps_for(n)
        e = bench.golden_for_params("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)))
        assert e is not None, n
        P, E, root = bench.expected(heaps)
        assert (e["positions"], e["edges"], e["root_line"].split()[0]) == (P, E, root)
        assert e["win"] + e["loss"] == P


def test_level_counts_and_compulsory_bytes():
    """Per-level position counts (digit-sum distribution) and the dense
    layout's compulsory byte model."""
    import itertools
    heaps = [3, 2, 4]
    n = bench.level_counts(heaps)
    root = sum(heaps)
    want = [0] * (root + 1)
    for hs in itertools.product(*[range(h + 1) for h in heaps]):
        want[root - sum(hs)] += 1
    assert n == want
    m = bench.dense_bytes(heaps, 2)
    P, E, _ = bench.expected(heaps)
    assert abs(m["resolve_compulsory"] - sum(2 * (n[L] + (n[L + 1] if L + 1 <= root else 0)
                                                  + (n[L + 2] if L + 2 <= root else 0)) + n[L] / 8
                                             for L in range(root + 1))) < 1e-6
    assert m["resolve_per_edge"] == 2.125 * P + 2 * E
    assert m["pull_per_edge"] == (E + P) / 8
    # the bench shape: about 6.1 B per position must move per resolve
    big = bench.dense_bytes([31] * 6, 2)
    assert 6.0 * 2 ** 30 < big["resolve_compulsory"] < 6.2 * 2 ** 30


def test_keyed_model():
    assert bench.keyed_bytes(10, 100) == (24 * 10 + 8 * 100, 12 * 10 + 12 * 100)


def test_kernel_names_come_from_the_library():
    from gamesmanmpi_amd import _lib
    assert _lib.RESOLVE_KERNELS[1] == "k_dense_resolve8p"
    assert _lib.PULL_KERNELS[1] == "k_dense_pull_words"


def test_planes_traffic_is_a_launch_weighted_mean(monkeypatch):
    """The PMC pass may hold several solves: the bench's PLANES traffic is
    bytes per launch over the pass's own launches, not scaled by them."""
    import bench
    rows = {"k_plane_resolve_x2": (36.0e6, 234.0), "k_plane_run": (0.13e6, 4.0)}
    monkeypatch.setattr(bench, "pmc_traffic_total", lambda k, w: rows.get(k, (None, 0)))
    t = bench.planes_traffic("k_plane_resolve_x2", "w")
    assert abs(t - (36.0e6 * 234 + 0.13e6 * 4) / 238) < 1.0
    assert 0.13e6 < t < 36.0e6
    monkeypatch.setattr(bench, "pmc_traffic_total", lambda k, w: (None, 0))
    assert bench.planes_traffic("k_plane_resolve_x2", "w") is None
