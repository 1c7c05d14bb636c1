"""BASELINE config 3 (toot_and_otto_bitstring as shipped: 6x4,
toot_and_otto_bitstring.py:8) pinned at its OWN size by the reference module
itself, on samples (tests/golden/make_golden.py toot_6x4_fixtures; the full
game, 1.19e9 positions, is pinned by the oracle_mt fingerprint only):

  * movegen/toot_6x4.json -- 400 random-playout positions: primitive() and
    the ORDERED children of gen_moves/do_move (src/game_state.py:32-40), and
    str(pos) (the md5 partition input, src/game_state.py:28);
  * md5_owner.json rows "toot_6x4" -- GameState.get_hash(P), P = 1..8;
  * deep/toot_6x4.json -- 220 positions with >= 16 of 24 pieces placed, each
    solved exhaustively through the module (every position reachable from it)
    with the reference-canonical retrograde.

CPU here: the product's 6x4 descriptor run on the host (gm_host_expand,
gm_str_utf8, gm_owner_host) and the C restatement (oracle/oracle.c) against
the vectors.  GPU (-m gpu): the full 6x4 solve on the RANKED (default) and
BUCKETED layouts, queried at the deep positions: value and remoteness exact."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

GAME = ("toot_and_otto_bitstring", "length=6,height=4")


def _rows(kind):
    with open(os.path.join(GOLDEN, kind, "toot_6x4.json")) as f:
        return json.load(f)


def test_movegen_vectors_cover_every_depth():
    rows = _rows("movegen")
    assert len(rows) >= 400
    depths = {r["pieces"] for r in rows}
    assert min(depths) == 0 and max(depths) >= 20
    assert sum(1 for r in rows if r["primitive"] != 4) >= 20  # terminal positions too
    deep = _rows("deep")["rows"]
    assert len(deep) >= 200 and min(r["pieces"] for r in deep) >= 16
    assert {r["value"] for r in deep} >= {0, 1, 2}  # WIN, LOSS and TIE all present


def test_product_descriptor_6x4_vs_reference_movegen():
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec(*GAME)
    rows = _rows("movegen")
    keys = np.array([spec.encode(bytes.fromhex(r["pos"])) for r in rows], np.uint64)
    pr, nc, ch = spec.host_expand(keys)
    for i, row in enumerate(rows):
        assert pr[i] == row["primitive"], row["pos"]
        assert [spec.decode(k).hex() for k in ch[i, :nc[i]]] == row["children"], row["pos"]
        assert spec.str_utf8(keys[i]).hex() == row["str_utf8"], row["pos"]
        assert spec.decode(keys[i]).hex() == row["pos"]


def test_product_md5_owners_6x4():
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec(*GAME)
    with open(os.path.join(GOLDEN, "md5_owner.json")) as f:
        rows = [r for r in json.load(f) if r["game"] == "toot_6x4"]
    assert len(rows) >= 50
    for row in rows:
        key = np.array([spec.encode(bytes.fromhex(row["canon"]))], np.uint64)
        assert spec.str_utf8(int(key[0])).hex() == row["str_utf8"]
        for P, owner in row["owners"].items():
            assert spec.owners_host(key, int(P))[0] == owner, (row["canon"], P)


def test_oracle_6x4_vs_reference_movegen():
    from oracle.oracle import Game
    g = Game(*GAME)
    for row in _rows("movegen"):
        prim, kids = g.expand(bytes.fromhex(row["pos"]))
        assert prim == row["primitive"], row["pos"]
        assert [k.hex() for k in kids] == row["children"], row["pos"]


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["auto", "bucketed"])
def test_gpu_toot_6x4_deep_positions_match_reference(layout):
    """The full 6x4 solve, queried at the 220 reference-solved deep positions."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    spec = GameSpec(*GAME)
    deep = _rows("deep")["rows"]
    keys = np.array([spec.encode(bytes.fromhex(r["pos"])) for r in deep], np.uint64)
    s = Solver(spec, layout=layout)
    r = s.solve()
    assert r.extra["layout"] == ("ranked" if layout == "auto" else "bucketed")
    assert r.root_line == "LOSS in 24 moves"
    w = s.query(keys)
    assert (w != 0xFFFFFFFF).all(), "a reference-reachable position is missing"
    for i, row in enumerate(deep):
        assert (int(w[i]) & 3, int(w[i]) >> 2) == (row["value"], row["remoteness"]), row
    del s
