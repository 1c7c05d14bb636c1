"""Host enumeration of descriptor-less game files (gamesmanmpi_amd/generic.py,
SURVEY §8f row 3): the module's own functions, breadth first, into a CSR
graph.  Checked against the golden tables' position sets and edge counts
(fixtures from the reference's modules) and against the product
descriptor's host expansion."""
import os

import numpy as np
import pytest

from conftest import ROOT, load_table

GAMES = os.path.join(ROOT, "tests", "games")


def _load(path):
    from gamesmanmpi_amd.solver_launcher import ensure_src_utils, load_game
    ensure_src_utils()
    return load_game(path)


def test_enumerate_grid_tictactoe_matches_golden(golden_summary):
    from gamesmanmpi_amd.generic import enumerate_game
    mod = _load(os.path.join(GAMES, "grid_tictactoe.py"))
    g = enumerate_game(mod, keep_positions=True)
    info = golden_summary["tic_tac_toe_np"]
    assert g.n == info["positions"] == 5478
    assert g.edges == info["edges"]
    assert int((g.prim != 4).sum()) == info["primitives"]
    t = load_table("tic_tac_toe_np")
    canon = sorted(np.asarray(p, np.int8).tobytes() for p in g.positions)
    want = sorted(bytes(r[:n]) for r, n in zip(t["canon"], t["clen"]))
    assert canon == want


def test_enumerate_sum_game_matches_descriptor():
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.generic import enumerate_game
    import gamesmanmpi_amd.games.sum_four_to_one as mod
    _load(os.path.join(ROOT, "gamesmanmpi_amd", "games", "sum_four_to_one.py"))
    saved = mod.HEAPS
    try:
        mod.HEAPS = (2, 5, 7)
        g = enumerate_game(mod)
        spec = GameSpec("sum_four_to_one", "heaps=2:5:7")
        keys = np.array([int(n) for n in g.names], np.uint64)
        pr, nc, ch = spec.host_expand(keys)
        np.testing.assert_array_equal(pr, g.prim)
        for i in range(g.n):
            want = [int(x) for x in ch[i, :nc[i]]]
            got = [int(g.names[j]) for j in g.children[g.offsets[i]:g.offsets[i + 1]]]
            assert got == want
        assert g.n == 3 * 6 * 8
    finally:
        mod.HEAPS = saved


def test_enumerate_limit():
    from gamesmanmpi_amd.generic import enumerate_game
    mod = _load(os.path.join(GAMES, "grid_tictactoe.py"))
    with pytest.raises(ValueError):
        enumerate_game(mod, limit=100)
