"""RANKED layout (gamesmanmpi_amd/csrc/gm_ranked.h): toot-and-otto positions
at computed indices -- column stacks + the first player's T count -- with no
keys stored and no dedup.  Checked against the reference-generated tables
(tests/test_gpu_parity.py::test_gpu_solve_matches_golden[toot_*-ranked]),
the oracle on degenerate boards (tests/test_gpu_edge_shapes.py), the 5x4 /
6x4 goldens (tests/test_gpu_full_size.py), and here word for word against
the BUCKETED layout, on keys that are not positions, and across a stopped
and resumed solve."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solver(params, layout):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("toot_and_otto_bitstring", params), layout=layout)
    return s, s.solve()


@pytest.mark.parametrize("params", ["length=4,height=4", "length=4,height=3", "length=3,height=4"])
def test_ranked_equals_bucketed_word_for_word(params):
    """The same positions (as keys) and every word equal to the BUCKETED
    layout's, on the fixed-board kernels (4x4) and the generic ones."""
    sr, rr = _solver(params, "ranked")
    sb, rb = _solver(params, "bucketed")
    assert rr.extra["layout"] == "ranked" and rb.extra["layout"] == "bucketed"
    assert (rr.positions, rr.edges, rr.primitives, rr.root_line) == (rb.positions, rb.edges, rb.primitives,
                                                                      rb.root_line)
    kr, kb = np.sort(sr.positions()), np.sort(sb.positions())
    np.testing.assert_array_equal(kr, kb)
    np.testing.assert_array_equal(sr.query(kb), sb.query(kb))
    assert sr.checksum() == sb.checksum()


def test_ranked_query_of_non_positions():
    """Keys that are no reachable position read GM_NO_WORD: a piece over a
    gap, inconsistent hands, the wrong turn bit, stray high bits."""
    s, r = _solver("length=4,height=4", "ranked")
    keys = s.positions()
    k = int(keys[len(keys) // 2])
    A = 16
    bad = [
        k ^ (1 << (2 * A + 12)),           # turn bit flipped
        k ^ (1 << (2 * A + 6)),            # the first mover's T count changed
        k | (1 << 63),                     # stray high bit
        (1 << 12) | (6 << 32) | (6 << 35) | (5 << 38) | (6 << 41) | (1 << 44),  # a T floating on row 3
    ]
    w = s.query(np.array(bad, np.uint64))
    assert (w == 0xFFFFFFFF).all(), w
    ok = s.query(keys[:1000])
    assert (ok != 0xFFFFFFFF).all()


@pytest.mark.parametrize("cut", [3, 17, 17 + 5, 33])
def test_ranked_stop_resume(cut):
    """Stop after step `cut` (forward levels 0..16, backward 17..33 on 4x4)
    and resume in the same solver: the same counts, root and words."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s0, r0 = _solver("length=4,height=4", "ranked")
    s = Solver(GameSpec("toot_and_otto_bitstring", "length=4,height=4"), layout="ranked")
    assert s.solve_steps(0, cut) is None
    r = s.solve_steps(cut, 0)
    assert (r.positions, r.edges, r.primitives, r.root_line) == (r0.positions, r0.edges, r0.primitives, r0.root_line)
    assert s.checksum() == s0.checksum()
