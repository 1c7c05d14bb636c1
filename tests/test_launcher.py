"""The drop-in boundary: reference-API game files load, validate, map to
their device descriptors and pass the descriptor-vs-module replay check
(gamesmanmpi_amd/solver_launcher.py, games.spec_for_module/verify).

CPU tests load the reference's OWN game files (only where /root/reference
exists; third-party imports they need come from tests/golden/refstubs).  The
GPU test runs the launcher end to end on a game file shipped here."""
import importlib.util
import io
import os
import shutil
import sys
from contextlib import redirect_stdout

import numpy as np
import pytest

from conftest import REFERENCE, ROOT, has_reference

STUBS = os.path.join(ROOT, "tests", "golden", "refstubs")
OWN_SUM = os.path.join(ROOT, "gamesmanmpi_amd", "games", "sum_four_to_one.py")


def _load(path, name, **overrides):
    from gamesmanmpi_amd import solver_launcher as sl
    if STUBS not in sys.path:
        sys.path.insert(0, STUBS)
    sl.ensure_src_utils()
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for k, v in overrides.items():
        setattr(mod, k, v)
    if "length" in overrides:
        mod.area = mod.length * mod.height
    sl.validate(mod)
    return mod


def test_compat_utils_semantics():
    from gamesmanmpi_amd import solver_launcher as sl
    sys.path.insert(0, os.path.join(ROOT, "gamesmanmpi_amd", "compat"))
    spec = importlib.util.spec_from_file_location(
        "compat_utils", os.path.join(ROOT, "gamesmanmpi_amd", "compat", "src",
                                     "utils.py"))
    u = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(u)
    assert (u.WIN, u.LOSS, u.TIE, u.DRAW, u.UNDECIDED) == (0, 1, 2, 3, 4)
    assert u.PRIMITIVES == (0, 1, 2, 3)
    assert [u.negate(x) for x in range(5)] == [1, 0, 2, 3, 4]
    assert [u.to_str(x) for x in range(5)] == ["WIN", "LOSS", "TIE", "DRAW",
                                                "UNDECIDED"]
    assert u.reduce_singleton(lambda a, b: (a, b), [7]) == (7, None)
    assert u.reduce_singleton(lambda a, b: a + b, [1, 2, 3]) == 6
    assert sl.COMPAT.endswith("compat")


@pytest.mark.skipif(not has_reference(), reason="reference not mounted")
def test_compat_utils_match_reference_module():
    spec = importlib.util.spec_from_file_location(
        "ref_utils", os.path.join(REFERENCE, "src", "utils.py"))
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    spec = importlib.util.spec_from_file_location(
        "compat_utils2", os.path.join(ROOT, "gamesmanmpi_amd", "compat", "src",
                                      "utils.py"))
    ours = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ours)
    for name in ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED", "PRIMITIVES",
                 "PRIMITIVE_REMOTENESS", "UNKNOWN_REMOTENESS", "STATE_MAP"):
        assert getattr(ours, name) == getattr(ref, name), name
    for x in range(5):
        assert ours.negate(x) == ref.negate(x)
        assert ours.to_str(x) == ref.to_str(x)


REF_GAMES = [
    ("four_to_one.py", {}),
    ("mttt.py", {}),
    ("tic_tac_toe_np.py", {}),
    ("toot_and_otto_bitstring.py", {}),                       # 6x4 as shipped
    ("toot_and_otto_bitstring.py", {"length": 4, "height": 3}),
    ("othello_bit_new.py", {"length": 4, "height": 4}),       # config 5 size
]


@pytest.mark.skipif(not has_reference(), reason="reference not mounted")
@pytest.mark.parametrize("fname,overrides", REF_GAMES)
def test_reference_game_files_map_and_verify(fname, overrides):
    from gamesmanmpi_amd.games import spec_for_module
    mod = _load(os.path.join(REFERENCE, "test_games", fname), "gm_launch_test",
                **overrides)
    spec = spec_for_module(mod, os.path.splitext(fname)[0])
    assert spec.verify(mod, samples=150) == 150


@pytest.mark.skipif(not has_reference(), reason="reference not mounted")
def test_modified_game_file_is_refused():
    """A game file whose rules differ from its descriptor must not be
    silently solved with stale rules."""
    from gamesmanmpi_amd.games import spec_for_module
    mod = _load(os.path.join(REFERENCE, "test_games", "four_to_one.py"),
                "gm_launch_mod")
    mod.gen_moves = lambda x: [-1]  # a different game
    spec = spec_for_module(mod, "four_to_one")
    with pytest.raises(ValueError):
        spec.verify(mod, samples=50)


def test_unknown_game_file_is_refused():
    from gamesmanmpi_amd.games import spec_for_module

    class M:
        __file__ = "/tmp/chess.py"
    with pytest.raises(ValueError):
        spec_for_module(M())


def test_own_sum_game_file_verifies():
    from gamesmanmpi_amd.games import spec_for_module
    mod = _load(OWN_SUM, "gm_sum_launch", HEAPS=(5, 7, 3))
    spec = spec_for_module(mod, "sum_four_to_one")
    assert spec.params == "heaps=5:7:3"
    assert spec.verify(mod, samples=200) == 200


def test_missing_api_function_raises():
    from gamesmanmpi_amd import solver_launcher as sl

    class M:
        initial_position = do_move = gen_moves = None
    with pytest.raises(AttributeError):
        sl.validate(M())


@pytest.mark.gpu
def test_launcher_end_to_end(tmp_path):
    """Launcher on a game file (the shipped sum game with edited HEAPS):
    prints the reference's root line and writes -sd output."""
    from gamesmanmpi_amd import solver_launcher as sl
    from oracle.oracle import Game
    game = tmp_path / "sum_four_to_one.py"
    src = open(OWN_SUM).read().replace(
        "HEAPS = (31, 31, 31, 31, 31, 31)", "HEAPS = (4, 6, 3)")
    game.write_text(src)
    out = io.StringIO()
    with redirect_stdout(out):
        rc = sl.main([str(game), "-sd", str(tmp_path / "sd")])
    assert rc == 0
    want = Game("sum_four_to_one", "heaps=4:6:3").solve().root_line
    assert out.getvalue().strip().splitlines()[0] == want
    z = np.load(tmp_path / "sd" / "stats" / "0" / "solution.npz")
    assert len(z["keys"]) == 5 * 7 * 4
    # the solution database answers for the initial position (db.py)
    from gamesmanmpi_amd.db import main as db_main
    out = io.StringIO()
    with redirect_stdout(out):
        assert db_main([str(tmp_path / "sd"), "--game", str(game)]) == 0
    assert out.getvalue().strip().endswith(want)
    shutil.rmtree(tmp_path / "sd")


@pytest.mark.gpu
def test_launcher_graph_path_for_file_without_descriptor(tmp_path):
    """A game file with no device descriptor (tests/games/grid_tictactoe.py)
    is enumerated on the host with its own functions and solved on the GPU:
    same root line as the reference's tic_tac_toe_np (TIE in 9 moves)."""
    from gamesmanmpi_amd import solver_launcher as sl
    game = os.path.join(ROOT, "tests", "games", "grid_tictactoe.py")
    out = io.StringIO()
    with redirect_stdout(out):
        rc = sl.main([game, "-sd", str(tmp_path / "sd")])
    assert rc == 0
    assert out.getvalue().strip().splitlines()[0] == "TIE in 9 moves"
    z = np.load(tmp_path / "sd" / "stats" / "0" / "solution.npz")
    assert len(z["names"]) == 5478


def test_checkpoint_flag_refuses_foreign_directory(tmp_path):
    """-ck on a directory holding files that are not a checkpoint exits
    non-zero before touching anything (no GPU needed: the check comes
    first); the directory and its files stay as they were."""
    from gamesmanmpi_amd import solver_launcher as sl
    game = tmp_path / "sum_four_to_one.py"
    game.write_text(open(OWN_SUM).read().replace(
        "HEAPS = (31, 31, 31, 31, 31, 31)", "HEAPS = (4, 6, 3)"))
    results = tmp_path / "results"
    results.mkdir()
    (results / "notes.txt").write_text("precious")
    (results / "sub").mkdir()
    with pytest.raises(SystemExit) as ei:
        sl.main([str(game), "-ck", str(results)])
    assert ei.value.code not in (0, None)
    assert sorted(os.listdir(results)) == ["notes.txt", "sub"]
    assert (results / "notes.txt").read_text() == "precious"


def test_checkpoint_helpers_only_touch_their_own_files(tmp_path):
    """checkpoint.check_target / latest / _remove_ours on the host: a
    foreign directory is refused, an interrupted save's DIR.old is found,
    and removal deletes exactly the checkpoint's files."""
    import json
    from gamesmanmpi_amd import checkpoint as ck
    d = tmp_path / "ck"
    ck.check_target(str(d))  # absent: fine
    d.mkdir()
    ck.check_target(str(d))  # empty: fine
    (d / "x.txt").write_text("x")
    with pytest.raises(ck.NotACheckpoint):
        ck.check_target(str(d))
    (d / "x.txt").unlink()
    meta = {"format": ck.FORMAT, "game": "g", "params": "", "step": 3}
    (d / "meta.json").write_text(json.dumps(meta))
    for n in ("table", "levels", "scratch"):
        (d / (n + ".bin")).write_bytes(b"\0" * 8)
    ck.check_target(str(d))
    assert ck.latest(str(d)) == str(d)
    # an interrupted save: only DIR.old holds the checkpoint
    os.replace(d, str(d) + ".old")
    assert ck.latest(str(d)) == str(d) + ".old"
    extra = tmp_path / "ck.old" / "keep.txt"
    extra.write_text("k")
    ck._remove_ours(str(d) + ".old")
    assert os.listdir(tmp_path / "ck.old") == ["keep.txt"]


def test_checkpoint_save_reuses_a_crashed_tmp(tmp_path, monkeypatch):
    """a save() that crashed while its .bin files streamed out
    leaves DIR.tmp holding our .bin files and no meta.json; the next save()
    must reuse it (not raise NotACheckpoint), while a .tmp holding foreign
    files is still refused.  Host-only: the device streaming is stubbed."""
    import types
    from gamesmanmpi_amd import checkpoint as ck
    d = str(tmp_path / "ck")
    tmp = tmp_path / "ck.tmp"
    tmp.mkdir()
    (tmp / "table.bin").write_bytes(b"\1" * 16)  # the crash left this
    monkeypatch.setattr(ck, "_stream_out", lambda t, path, torch: open(path, "wb").write(b"\0" * 8))
    monkeypatch.setattr(ck, "_plan_dict", lambda s: {"mode": 0})
    fake_torch = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda dev=None: None))
    solver = types.SimpleNamespace(world=1, torch=fake_torch, device="cpu", buffers=(0, 0, 0),
                                   spec=types.SimpleNamespace(name="g", params=""), layout="auto",
                                   positions_hint=1, max_table_bytes=0, flags=0, steps=4)
    ck.save(solver, d, 2)
    assert ck.read_meta(d)["step"] == 2
    assert not os.path.exists(str(tmp))
    # a foreign file in the scratch directory is still refused
    tmp.mkdir()
    (tmp / "notes.txt").write_text("mine")
    with pytest.raises(ck.NotACheckpoint):
        ck.save(solver, d, 3)
    assert (tmp / "notes.txt").read_text() == "mine"


def test_replicated_table_writes_each_ranks_md5_share(tmp_path):
    """Under torchrun a game whose RANKED table fits one GPU is solved whole
    on every rank; -sd then writes, per rank, the positions the reference's
    md5 partition gives that rank (src/game_state.py:22-30): the shares are
    disjoint and cover every position."""
    import types
    import numpy as np
    from gamesmanmpi_amd import solver_launcher as sl
    from gamesmanmpi_amd.games import GameSpec
    from oracle.oracle import Game  # checker only
    params = "length=3,height=3"
    spec = GameSpec("toot_and_otto_bitstring", params)
    sol = Game("toot_and_otto_bitstring", params).solve(1 << 20)
    canon, clen, val, rem = sol.dump(stride=24)
    keys = spec.encode_batch(canon, clen)
    fake = types.SimpleNamespace(replicated=True, dump=lambda: (keys, val, rem))
    res = types.SimpleNamespace(root_line=sol.root_line)
    world = 3
    seen = []
    for r in range(world):
        sl.write_stats(str(tmp_path), r, spec, fake, res, world)
        z = np.load(tmp_path / "stats" / str(r) / "solution.npz")
        assert (spec.owners_host(z["keys"], world) == r).all()
        seen.append(z["keys"])
    allk = np.concatenate(seen)
    assert len(allk) == len(keys) and len(np.unique(allk)) == len(keys)
