"""Symmetric solves (params "symmetry=1": orbit representatives under the
module's symmetry_functions(), othello_bit_new.py:224-235): the solve
stores fewer positions, prints the same root line, and every one of the
54,089 reachable othello 4x4 positions reads back its golden value and
remoteness -- single table and md5-sharded keyed tables."""
import numpy as np
import pytest

from conftest import CASES, load_table

pytestmark = pytest.mark.gpu

SYM = ("othello_bit_new", "length=4,height=4,symmetry=1")


def _golden_keys():
    from gamesmanmpi_amd.games import GameSpec
    t = load_table("othello_4x4")
    return GameSpec(*CASES["othello_4x4"]).encode_batch(t["canon"], t["clen"]), t


def test_symmetric_single_table_matches_golden(golden_summary):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec(*SYM))
    r = s.solve()
    info = golden_summary["othello_4x4"]
    assert r.root_line == info["root_line"] == "LOSS in 12 moves"
    keys, t = _golden_keys()
    spec = GameSpec(*SYM)
    canon = spec.symmetry(keys)
    # player_flip changes the side to move but not the piece count, so from
    # the standard start (no passes) p and flip(p) are never both reachable:
    # every orbit holds one reachable position, and about half of them are
    # stored as the flipped image
    assert r.positions == len(np.unique(canon)) <= info["positions"]
    assert 0 < (canon != keys).sum() < len(keys)
    w = s.query(keys)  # non-canonical keys: the query maps them to their representative
    np.testing.assert_array_equal(w & 3, t["value"])
    np.testing.assert_array_equal(w >> 2, t["remoteness"])
    stored, _, _ = s.dump()
    np.testing.assert_array_equal(np.sort(stored), np.unique(canon))


@pytest.mark.parametrize("world", [3, 8])
def test_symmetric_keyed_shards_match_golden(world, golden_summary):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    spec = GameSpec(*SYM)
    r, shards = group_keyed_solve(spec, world)
    assert r.root_line == golden_summary["othello_4x4"]["root_line"]
    table = {}
    for rank, sh in enumerate(shards):
        k, v, m = sh.dump()
        if len(k):
            assert (spec.owners_host(k, world) == rank).all()  # md5 owner of the representative
        table.update(zip(k.tolist(), zip(v.tolist(), m.tolist())))
    keys, t = _golden_keys()
    got = np.array([table[int(c)] for c in spec.symmetry(keys)])
    np.testing.assert_array_equal(got[:, 0], t["value"])
    np.testing.assert_array_equal(got[:, 1], t["remoteness"])
