"""The -sd solution database (gamesmanmpi_amd/db.py): rank files written in
the launcher's format are read back as one table and queried by game
position, keyed (descriptor games) and by str(position) (graph games)."""
import io
import json
import os
from contextlib import redirect_stdout

import numpy as np
import pytest

from conftest import ROOT

OWN_SUM = os.path.join(ROOT, "gamesmanmpi_amd", "games", "sum_four_to_one.py")


def _write_rank(root, rank, **arrays):
    d = os.path.join(root, "stats", str(rank))
    os.makedirs(d, exist_ok=True)
    np.savez_compressed(os.path.join(d, "solution.npz"), **arrays)
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump({"owned_by_rank": rank}, f)


def test_keyed_db_matches_oracle(tmp_path):
    from oracle.oracle import Game
    from gamesmanmpi_amd.db import main
    game = tmp_path / "sum_four_to_one.py"
    game.write_text(open(OWN_SUM).read().replace(
        "HEAPS = (31, 31, 31, 31, 31, 31)", "HEAPS = (4, 6, 3)"))
    sol = Game("sum_four_to_one", "heaps=4:6:3").solve()
    keys = np.arange(5 * 7 * 4, dtype=np.uint64)
    vr = np.array([sol.lookup(str(k).encode()) for k in keys.tolist()])
    # two "ranks", interleaved ownership
    for r in range(2):
        m = keys % 2 == r
        _write_rank(tmp_path / "sd", r, keys=keys[m], value=vr[m, 0].astype(np.uint8),
                    remoteness=vr[m, 1].astype(np.uint32))
    out = io.StringIO()
    with redirect_stdout(out):
        rc = main([str(tmp_path / "sd"), "--game", str(game), "0", "139", "57"])
    assert rc == 0
    lines = out.getvalue().splitlines()
    names = ("WIN", "LOSS", "TIE", "DRAW")
    for line, k in zip(lines, (0, 139, 57)):
        v, m = sol.lookup(str(k).encode())
        assert line == "%d: %s in %d moves" % (k, names[v], m)
    out = io.StringIO()
    with redirect_stdout(out):
        main([str(tmp_path / "sd"), "--game", str(game)])  # initial position
    assert out.getvalue().strip() == "139: " + sol.root_line


def test_graph_db_by_name(tmp_path):
    from gamesmanmpi_amd.db import SolutionDB
    _write_rank(tmp_path / "sd", 0, names=np.array(["a", "b"]),
                value=np.array([0, 1], np.uint8), remoteness=np.array([3, 0], np.uint32))
    db = SolutionDB(str(tmp_path / "sd"))
    assert db.lookup("b") == (1, 0)
    assert db.lookup("zz") is None


def test_duplicate_keys_refused(tmp_path):
    from gamesmanmpi_amd.db import SolutionDB
    for r in range(2):
        _write_rank(tmp_path / "sd", r, keys=np.array([5], np.uint64),
                    value=np.array([0], np.uint8), remoteness=np.array([1], np.uint32))
    with pytest.raises(ValueError):
        SolutionDB(str(tmp_path / "sd"))


def test_checkpoint_meta_format_is_checked(tmp_path):
    """checkpoint.read_meta refuses unknown formats (restore would otherwise
    load buffers laid out by another build)."""
    import json
    from gamesmanmpi_amd import checkpoint
    d = tmp_path / "ck"
    d.mkdir()
    (d / "meta.json").write_text(json.dumps({"format": checkpoint.FORMAT + 1}))
    with pytest.raises(ValueError):
        checkpoint.read_meta(str(d))
    (d / "meta.json").write_text(json.dumps({"format": checkpoint.FORMAT, "game": "mttt",
                                             "params": "", "step": 3}))
    assert checkpoint.read_meta(str(d))["step"] == 3
