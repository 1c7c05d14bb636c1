"""GPU: the explicit-graph retrograde (gm_graph_solve) for game files without
a device descriptor, bit-exact against the reference's golden tables and
against the descriptor pipeline."""
import os

import numpy as np
import pytest

from conftest import ROOT, load_table

pytestmark = pytest.mark.gpu
GAMES = os.path.join(ROOT, "tests", "games")


def _load(path):
    from gamesmanmpi_amd.solver_launcher import ensure_src_utils, load_game
    ensure_src_utils()
    return load_game(path)


def test_gpu_graph_grid_tictactoe_matches_golden(golden_summary):
    from gamesmanmpi_amd.generic import GenericSolver, enumerate_game
    g = enumerate_game(_load(os.path.join(GAMES, "grid_tictactoe.py")), keep_positions=True)
    s = GenericSolver(g)
    r = s.solve()
    info = golden_summary["tic_tac_toe_np"]
    assert (r.positions, r.edges, r.primitives) == (info["positions"], info["edges"], info["primitives"])
    assert r.root_line == info["root_line"]
    _, val, rem = s.dump()
    t = load_table("tic_tac_toe_np")
    canon = [np.asarray(p, np.int8).tobytes() for p in g.positions]
    order = sorted(range(g.n), key=lambda i: canon[i])
    np.testing.assert_array_equal(val[order], t["value"])
    np.testing.assert_array_equal(rem[order], t["remoteness"])


def test_gpu_graph_sum_game_matches_dense():
    from gamesmanmpi_amd.generic import GenericSolver, enumerate_game
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    import gamesmanmpi_amd.games.sum_four_to_one as mod
    _load(os.path.join(ROOT, "gamesmanmpi_amd", "games", "sum_four_to_one.py"))
    saved = mod.HEAPS
    try:
        mod.HEAPS = (7, 7, 7, 7)
        g = enumerate_game(mod)
        gs = GenericSolver(g)
        r = gs.solve()
    finally:
        mod.HEAPS = saved
    d = Solver(GameSpec("sum_four_to_one", "heaps=7:7:7:7"), layout="dense")
    rd = d.solve()
    assert (r.positions, r.edges, r.primitives, r.root_line) == (rd.positions, rd.edges, rd.primitives, rd.root_line)
    keys = np.array([int(n) for n in g.names], np.uint64)
    w = d.query(keys)
    _, val, rem = gs.dump()
    np.testing.assert_array_equal(val, (w & 3).astype(np.uint8))
    np.testing.assert_array_equal(rem, (w >> 2).astype(np.uint32))


def test_gpu_graph_cycle_is_reported():
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.generic import GenericSolver, enumerate_game
    g = enumerate_game(_load(os.path.join(GAMES, "two_cycle.py")))
    assert g.n == 3
    with pytest.raises(_lib.GmError, match="never resolve"):
        GenericSolver(g).solve()
