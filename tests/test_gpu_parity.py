"""GPU parity: the HIP pipeline (through the C-ABI) against the reference's
golden tables, the oracle, and size-independent properties at full sizes.
Bit-exact: every reachable position's value AND remoteness must match."""
import hashlib

import numpy as np
import pytest

from conftest import ALL_CASES, CASES, load_table

pytestmark = pytest.mark.gpu


def _solve(stem, params, positions=0, layout="auto"):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    spec = GameSpec(stem, params)
    s = Solver(spec, positions=positions, layout=layout)
    return spec, s, s.solve()


DENSE_GAMES = ("four_to_one", "sum_four_to_one")
GOLDEN_RUNS = [(n, "hashed") for n in sorted(CASES)] + [
    (n, "dense") for n in sorted(CASES) if CASES[n][0] in DENSE_GAMES] + [
    (n, "bucketed") for n in sorted(CASES) if CASES[n][0] not in DENSE_GAMES] + [
    (n, "ranked") for n in sorted(CASES) if CASES[n][0] == "toot_and_otto_bitstring"]


@pytest.mark.parametrize("name,layout", GOLDEN_RUNS)
def test_gpu_solve_matches_golden(name, layout, golden_summary):
    info = golden_summary[name]
    stem, params = CASES[name]
    spec, s, r = _solve(stem, params, positions=info["positions"],
                        layout=layout)
    assert r.extra["layout"] == layout
    assert r.positions == info["positions"]
    assert r.edges == info["edges"]
    assert r.primitives == info["primitives"]
    assert r.root_line == info["root_line"]
    keys, val, rem = s.dump()
    t = load_table(name)
    stride = t["canon"].shape[1] if t is not None else 7
    canon, clen = spec.decode_batch(keys, stride=stride)
    order = sorted(range(len(keys)), key=lambda i: bytes(canon[i, :clen[i]]))
    order = np.array(order, np.int64)
    canon, clen, val, rem = canon[order], clen[order], val[order], rem[order]
    if t is None:  # sha-only fixture (toot 4x4: 3,468,773 positions)
        h = hashlib.sha256()
        h.update(canon.tobytes())
        h.update(val.tobytes())
        h.update(rem.tobytes())
        assert h.hexdigest() == info["table_sha256"]
        return
    np.testing.assert_array_equal(canon, t["canon"])
    np.testing.assert_array_equal(val, t["value"])
    np.testing.assert_array_equal(rem, t["remoteness"])


@pytest.mark.parametrize("layout", ["hashed", "dense"])
def test_gpu_matches_oracle_sum_game(layout):
    """Mid-size synthetic (65,536 positions, 61 levels) vs the oracle."""
    from oracle.oracle import Game
    spec, s, r = _solve("sum_four_to_one", "heaps=15:15:15:15", layout=layout)
    sol = Game("sum_four_to_one", "heaps=15:15:15:15").solve(1 << 17)
    assert (r.positions, r.edges) == (sol.count, sol.edges)
    assert r.root_line == sol.root_line
    keys, val, rem = s.dump()
    for k, v, m in zip(keys.tolist(), val.tolist(), rem.tolist()):
        assert sol.lookup(str(k).encode()) == (v, m), k


@pytest.mark.parametrize("layout", ["hashed", "dense"])
def test_gpu_fto_chain_closed_form(layout):
    """Four-To-One chain at N=3000: 3001 levels deep."""
    spec, s, r = _solve("four_to_one", "start=3000", layout=layout)
    keys, val, rem = s.dump()
    x = keys.astype(np.int64)
    np.testing.assert_array_equal(val, np.where(x % 3 == 0, 1, 0))
    want = np.where(x % 3 == 0, 2 * (x // 3), 2 * (x // 3) + 1)
    np.testing.assert_array_equal(rem.astype(np.int64), want)
    assert r.root_line == "LOSS in 2000 moves"


def _sprague_grundy_check(keys, val, heaps):
    """Sum of Four-To-One heaps: a position is LOSS iff XOR of (h_i mod 3)
    is 0 (each heap is a subtraction game {1,2} with Grundy value h mod 3)."""
    x = keys.astype(np.int64)
    g = np.zeros_like(x)
    for h in heaps:
        g ^= (x % (h + 1)) % 3
        x //= (h + 1)
    np.testing.assert_array_equal(val, np.where(g == 0, 1, 0).astype(np.uint8))


@pytest.mark.parametrize("layout", ["hashed", "dense"])
def test_gpu_sum_game_sprague_grundy_1m(layout):
    heaps = (15, 15, 15, 15, 15)  # 1,048,576 positions
    spec, s, r = _solve("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)),
                        layout=layout)
    assert r.positions == 16 ** 5
    keys, val, rem = s.dump()
    _sprague_grundy_check(keys, val, heaps)


def test_gpu_md5_owner_kernel():
    import torch
    import json
    import os
    from conftest import GOLDEN
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    with open(os.path.join(GOLDEN, "md5_owner.json")) as f:
        rows = json.load(f)
    by_game = {}
    for row in rows:
        by_game.setdefault(row["game"], []).append(row)
    for game, rs in by_game.items():
        spec = GameSpec(*ALL_CASES[game])
        keys = np.array([spec.encode(bytes.fromhex(r["canon"])) for r in rs],
                        np.uint64)
        kd = torch.from_numpy(keys.view(np.int64)).cuda()
        ps = sorted(int(p) for p in rs[0]["owners"])
        assert ps == list(range(1, 9)), ps  # the fixture's P = 1..8, every one checked
        for P in ps:
            od = torch.empty(len(keys), dtype=torch.int32, device="cuda")
            _lib.check(_lib.load().gm_owner(spec.id, kd.data_ptr(), len(keys),
                                            P, od.data_ptr(), None))
            got = od.cpu().numpy().tolist()
            assert got == [r["owners"][str(P)] for r in rs], (game, P)


def test_gpu_dense_and_hashed_agree_nonpow2():
    """Non-power-of-two heaps exercise the division paths of both layouts:
    every word identical."""
    _, a, ra = _solve("sum_four_to_one", "heaps=6:9:4:11", layout="dense")
    _, b, rb = _solve("sum_four_to_one", "heaps=6:9:4:11", layout="hashed")
    assert (ra.positions, ra.edges, ra.root_line) == (rb.positions, rb.edges, rb.root_line)
    ka, va, ma = a.dump()
    kb, vb, mb = b.dump()
    oa, ob = np.argsort(ka), np.argsort(kb)
    np.testing.assert_array_equal(ka[oa], kb[ob])
    np.testing.assert_array_equal(va[oa], vb[ob])
    np.testing.assert_array_equal(ma[oa], mb[ob])


def test_gpu_full_size_synthetic_properties():
    """BASELINE config 4 at full size (2^30 positions, dense): root line,
    counts, and the Sprague-Grundy value rule on a 2^20 random sample."""
    heaps = (31,) * 6
    spec, s, r = _solve("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)),
                        layout="dense")
    assert r.positions == 1 << 30
    assert r.edges == 12280922112
    assert r.root_line == "LOSS in 126 moves"  # XOR of 31%3=1 six times = 0
    rng = np.random.default_rng(0)
    keys = rng.integers(0, 1 << 30, size=1 << 20, dtype=np.uint64)
    w = s.query(keys)
    _sprague_grundy_check(keys, (w & 3).astype(np.uint8), heaps)


@pytest.mark.parametrize("name", ["tic_tac_toe_np", "othello_4x4", "sum_fto_6_6_6_6", "toot_4x3"])
def test_gpu_one_shot_solve_and_query(name, golden_summary):
    """SURVEY §8b's one-shot pair: gm_solve(game, root, 1, buffers) then
    gm_query(game, keys, n, words) on the table it keeps, every golden
    position's word bit-exact (toot 4x3 and tic-tac-toe on BUCKETED levels:
    the home-slot search of k_bk_query); gm_release drops it and a query then
    fails."""
    import ctypes
    import torch
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    if name not in CASES:
        pytest.skip("no golden table %s" % name)
    stem, params = CASES[name]
    info = golden_summary[name]
    spec = GameSpec(stem, params)
    L = _lib.load()
    plan = _lib.gm_plan_t()
    _lib.check(L.gm_plan(spec.id, info["positions"], 0, 0, ctypes.byref(plan)))
    dev = torch.device("cuda")
    table = torch.empty(plan.table_bytes, dtype=torch.uint8, device=dev)
    levels = torch.empty(max(1, plan.level_capacity), dtype=torch.int64, device=dev)
    scratch = torch.empty(plan.scratch_bytes, dtype=torch.uint8, device=dev)
    b = _lib.gm_buffers()
    b.table, b.table_slots = table.data_ptr(), plan.table_slots
    b.levels, b.level_capacity = levels.data_ptr(), plan.level_capacity
    b.scratch, b.scratch_bytes = scratch.data_ptr(), plan.scratch_bytes
    b.stream, b.mode, b.table_bytes = torch.cuda.current_stream().cuda_stream, plan.mode, plan.table_bytes
    r = _lib.gm_result()
    _lib.check(L.gm_solve(spec.id, spec.root_key, 1, ctypes.byref(b), ctypes.byref(r)))
    assert (r.positions, r.edges) == (info["positions"], info["edges"])
    t = load_table(name)
    keys = spec.encode_batch(t["canon"], t["clen"])
    kd = torch.from_numpy(np.ascontiguousarray(keys.astype(np.int64))).to(dev)
    wd = torch.empty(len(keys), dtype=torch.int32, device=dev)
    _lib.check(L.gm_query(spec.id, kd.data_ptr(), len(keys), wd.data_ptr()))
    w = wd.cpu().numpy().astype(np.uint32)
    np.testing.assert_array_equal(w & 3, t["value"])
    np.testing.assert_array_equal(w >> 2, t["remoteness"])
    _lib.check(L.gm_release(spec.id))
    assert L.gm_query(spec.id, kd.data_ptr(), len(keys), wd.data_ptr()) == _lib.GM_EINVAL


@pytest.mark.gpu
def test_gpu_one_process_multi_gpu_solve():
    """gm_solve(game, root, ngpus, buf[ngpus]) from one process: with every
    visible GPU (the driver's 8-GPU node) the sum bench shape of that many
    GPUs solves to the closed-form counts and root value; with more GPUs than
    visible it fails with GM_EINVAL before any allocation (a one-GPU box
    runs only this half)."""
    import ctypes
    import torch
    from gamesmanmpi_amd import _lib, dist as gdist
    from gamesmanmpi_amd.games import GameSpec
    n = torch.cuda.device_count()
    L = _lib.load()
    spec = GameSpec("sum_four_to_one", "heaps=31:31:31:%d" % (32 * (n + 1) - 1))
    bufs = (_lib.gm_buffers * (n + 1))()
    r = _lib.gm_result()
    assert L.gm_solve(spec.id, spec.root_key, n + 1, bufs, ctypes.byref(r)) == _lib.GM_EINVAL
    assert b"visible" in L.gm_last_error()
    if n < 2:
        return
    heaps = [31, 31, 31, 32 * n - 1]
    spec = GameSpec("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)))
    res = gdist.solve_one_process(spec, n)
    P = 1
    for h in heaps:
        P *= h + 1
    assert res.positions == P
    g = 0
    for h in heaps:
        g ^= h % 3
    assert res.root_value == (1 if g == 0 else 0)  # Sprague-Grundy: LOSS iff the XOR of h mod 3 is 0
    _lib.check(L.gm_release(spec.id))
