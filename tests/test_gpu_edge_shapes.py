"""Edge shapes of the rank-indexable games on the GPU, against the oracle
(oracle/, CPU restatement of four_to_one.py:7-22 and the reference-canonical
retrograde): trivial and one-move games, zero-height heaps, tables narrower
than one 256-prefix group (the octet kernels' group size), and both layouts.
Parity is bit-exact on every reachable position."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = [
    ("four_to_one", "start=0", "LOSS in 0 moves"),
    ("four_to_one", "start=1", "WIN in 1 moves"),
    ("four_to_one", "start=2", "WIN in 1 moves"),
    ("four_to_one", "start=3", None),
    ("sum_four_to_one", "heaps=0", None),
    ("sum_four_to_one", "heaps=0:0", None),
    ("sum_four_to_one", "heaps=5:0", None),
    ("sum_four_to_one", "heaps=0:7", None),
    ("sum_four_to_one", "heaps=1:1:1", None),
    ("sum_four_to_one", "heaps=7:7", None),        # 8 prefixes: one partial group
    ("sum_four_to_one", "heaps=15:15", None),
    ("sum_four_to_one", "heaps=7:7:7", None),      # 64 prefixes
    ("sum_four_to_one", "heaps=31:31", None),
    ("sum_four_to_one", "heaps=3:7:7:7", None),    # base[1] = 8, W = 512
    ("sum_four_to_one", "heaps=2:5:0:6", None),    # non-power-of-two
]


@pytest.mark.parametrize("layout", ["dense", "hashed"])
@pytest.mark.parametrize("name,params,root", SHAPES)
def test_edge_shape_matches_oracle(name, params, root, layout):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    from oracle.oracle import Game  # checker only
    spec = GameSpec(name, params)
    s = Solver(spec, layout=layout)
    r = s.solve()
    sol = Game(name, params).solve(1 << 20)
    assert (r.positions, r.edges, r.root_line) == (sol.count, sol.edges, sol.root_line)
    if root is not None:
        assert r.root_line == root
    keys, val, rem = s.dump()
    assert len(keys) == sol.count
    for k, v, m in zip(keys.tolist(), val.tolist(), rem.tolist()):
        assert (v, m) == tuple(sol.lookup(spec.decode(k))), (k, v, m)


KEYED_SHAPES = [
    ("toot_and_otto_bitstring", "length=1,height=1"),
    ("toot_and_otto_bitstring", "length=2,height=1"),
    ("toot_and_otto_bitstring", "length=1,height=3"),
    ("toot_and_otto_bitstring", "length=2,height=2"),
    ("toot_and_otto_bitstring", "length=3,height=2"),
    ("toot_and_otto_bitstring", "length=2,height=4"),
    ("othello_bit_new", "length=2,height=2"),   # the root is primitive: one level
    ("othello_bit_new", "length=4,height=4"),
    ("mttt", ""),
]


@pytest.mark.parametrize("layout,flags", [("bucketed", 0), ("bucketed", 128), ("hashed", 0)])
@pytest.mark.parametrize("name,params", KEYED_SHAPES)
def test_keyed_edge_shape_matches_oracle(name, params, layout, flags):
    """Small and degenerate boards through both keyed layouts (bucketed:
    provisioned partitions, and GM_F_BK_EXACT = 128, the counted form): a
    primitive root, levels of one position, single-bucket levels (partitions
    mostly empty) -- every position against the oracle."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    from oracle.oracle import Game  # checker only
    spec = GameSpec(name, params)
    sol = Game(name, params).solve(1 << 22)
    s = Solver(spec, layout=layout, positions=max(64, sol.count), flags=flags)
    r = s.solve()
    assert r.extra["layout"] == layout
    assert (r.positions, r.edges, r.root_line) == (sol.count, sol.edges, sol.root_line)
    keys, val, rem = s.dump()
    assert len(keys) == sol.count
    for k, v, m in zip(keys.tolist(), val.tolist(), rem.tolist()):
        assert (v, m) == tuple(sol.lookup(spec.decode(k))), (k, v, m)


@pytest.mark.parametrize("name,params", [x for x in KEYED_SHAPES if x[0] == "toot_and_otto_bitstring"])
def test_ranked_edge_shape_matches_oracle(name, params):
    """toot-and-otto's RANKED layout (gm_ranked.h) on degenerate boards: one
    column, one row, boards that fill before a word forms -- every position
    against the oracle."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    from oracle.oracle import Game  # checker only
    spec = GameSpec(name, params)
    sol = Game(name, params).solve(1 << 22)
    s = Solver(spec, layout="ranked")
    r = s.solve()
    assert r.extra["layout"] == "ranked"
    assert (r.positions, r.edges, r.root_line) == (sol.count, sol.edges, sol.root_line)
    keys, val, rem = s.dump()
    assert len(keys) == sol.count
    for k, v, m in zip(keys.tolist(), val.tolist(), rem.tolist()):
        assert (v, m) == tuple(sol.lookup(spec.decode(k))), (k, v, m)
