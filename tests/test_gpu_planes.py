"""PLANES layout (gamesmanmpi_amd/csrc/gm_plane.h): sum_four_to_one with heaps
0 and 1 of 32 values, every position's order-form word in natural rank
order, resolved plane level by plane level.

Checked against the CPU oracle (oracle/oracle.c, pinned to the reference's
own game modules by tests/test_oracle.py) position by position on small
shapes, against the level-major DENSE layout word for word, and at full size
(2^30; the 2-, 4- and 8-GPU bench shapes 2^31..2^33 as in-process shard
groups are in tests/test_gpu_full_size.py) by whole-solve fingerprints against tests/golden/checksums.json
(oracle/oracle_mt.c)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _planes(params, **kw):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("sum_four_to_one", params), layout="planes", **kw)
    return s, s.solve()


def _oracle(params):
    """The CPU restatement's row solver (oracle/oracle_mt.c, pinned to the
    DFS oracle and the reference-generated tables by tests/test_oracle.py):
    stats + the word (value | remoteness << 2) of every rank."""
    from oracle.oracle import Game
    sol = Game("sum_four_to_one", params).solve_rows()
    sol.refresh(True)
    return sol


def _oracle_words(sol, n):
    return np.array([sol.word(k) for k in range(n)], np.uint32)


LEVELS = 65536  # GM_F_PLANE_LEVELS: one launch per plane level instead of the one-launch backward


@pytest.mark.parametrize("flags", [0, LEVELS])
@pytest.mark.parametrize("params", ["heaps=31:31", "heaps=31:31:1", "heaps=31:31:3", "heaps=31:31:2:5",
                                    "heaps=31:31:4:0:2", "heaps=31:31:7:7",
                                    "heaps=31:31:1:2:1:2:1",      # five outer digits, mixed bases
                                    "heaps=31:31:1:1:1:1:1:1"])   # six (kPlaneMaxOuter)
def test_planes_match_oracle(params, flags):
    """Every position's value and remoteness (and the counts / root line)
    equal the oracle's, including non-power-of-two and zero-height outer
    heaps and the plane-less K = 2 shape -- on the one-launch backward
    (k_plane_flow, the default with outer heaps) and on one launch per plane
    level (GM_F_PLANE_LEVELS)."""
    s, r = _planes(params, flags=flags)
    sol = _oracle(params)
    flow = params != "heaps=31:31" and not flags
    assert r.extra["layout"] == "planes" and r.extra["resolve_kernel"] == (
        "k_plane_flow" if flow else "k_plane_resolve_x2")  # 8-bit words
    assert (r.positions, r.edges, r.primitives, r.root_line) == (sol.count, sol.edges, sol.stats["primitives"],
                                                                  sol.root_line)
    keys, val, rem = s.dump()
    assert len(keys) == sol.count
    np.testing.assert_array_equal(np.sort(keys), np.arange(sol.count, dtype=np.uint64))
    want = _oracle_words(sol, sol.count)[keys.astype(np.int64)]
    np.testing.assert_array_equal(val, want & 3)
    np.testing.assert_array_equal(rem, want >> 2)
    ck = s.checksum()
    assert (ck["checksum"], ck["win"], ck["loss"]) == ("%016x" % sol.stats["checksum"], sol.stats["win"],
                                                       sol.stats["loss"])


@pytest.mark.parametrize("flags", [LEVELS, 0])
@pytest.mark.parametrize("params", ["heaps=31:31:7:7:7:7", "heaps=31:31:15:15:15"])
def test_planes_level_pairs_match_oracle(params, flags):
    """Shapes whose narrow plane levels go through k_plane_pair in the
    per-level schedule (GM_F_PLANE_LEVELS: two levels per launch, the level-s
    planes resolved redundantly by their level-(s+1) parents and stored by
    one): four and three outer digits of power-of-two bases, levels of
    33..1200 planes paired; and the same shapes on the one-launch backward --
    counts, root, whole-table fingerprint and 20,000 sampled words equal the
    oracle's."""
    s, r = _planes(params, flags=flags)
    assert r.extra["resolve_kernel"] == ("k_plane_resolve_x2" if flags else "k_plane_flow")
    sol = _oracle(params)
    assert r.extra["layout"] == "planes"
    assert (r.positions, r.edges, r.primitives, r.root_line) == (sol.count, sol.edges, sol.stats["primitives"],
                                                                  sol.root_line)
    ck = s.checksum()
    assert (ck["checksum"], ck["win"], ck["loss"]) == ("%016x" % sol.stats["checksum"], sol.stats["win"],
                                                       sol.stats["loss"])
    rng = np.random.default_rng(6)
    keys = rng.integers(0, sol.count, 20000, dtype=np.uint64)
    w = s.query(keys)
    want = np.array([sol.word(int(k)) for k in keys], np.uint32)
    np.testing.assert_array_equal(w, want)


def test_planes_kernel_families_agree():
    """16-bit order forms (GM_F_WORDS16, k_plane_resolve) and the one-plane
    kernel on 8-bit words (GM_F_PLANE_X1) give the same words as the
    default packed 8-bit kernel."""
    from gamesmanmpi_amd import _lib
    params = "heaps=31:31:15:15"
    s8, r8 = _planes(params)
    s16, r16 = _planes(params, flags=_lib.GM_F_WORDS16)
    s1, r1 = _planes(params, flags=_lib.GM_F_PLANE_X1)
    assert (r8.extra["word_bits"], r16.extra["word_bits"], r1.extra["word_bits"]) == (8, 16, 8)
    assert (r8.extra["resolve_kernel"], r16.extra["resolve_kernel"], r1.extra["resolve_kernel"]) == (
        "k_plane_flow", "k_plane_resolve", "k_plane_resolve")
    assert r8.root_line == r16.root_line == r1.root_line
    keys = np.arange(32 * 32 * 16 * 16, dtype=np.uint64)
    w = s8.query(keys)
    np.testing.assert_array_equal(w, s16.query(keys))
    np.testing.assert_array_equal(w, s1.query(keys))


def test_planes_equal_level_major():
    """PLANES and the level-major DENSE table agree word for word (and on
    keys outside the state space: GM_NO_WORD)."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    params = "heaps=31:31:31:7"
    s, r = _planes(params)
    d = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    rd = d.solve()
    assert (r.positions, r.edges, r.primitives, r.root_line) == (rd.positions, rd.edges, rd.primitives, rd.root_line)
    keys = np.arange(32 * 32 * 32 * 8 + 5, dtype=np.uint64)
    w = s.query(keys)
    np.testing.assert_array_equal(w, d.query(keys))
    assert (w[-5:] == 0xFFFFFFFF).all()


def test_planes_positions_and_checksum_match_level_major():
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    params = "heaps=31:31:6:9"
    s, _ = _planes(params)
    d = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    d.solve()
    np.testing.assert_array_equal(np.sort(s.positions()), np.sort(d.positions()))
    assert s.checksum() == d.checksum()


def _gold(name):
    with open(os.path.join(GOLDEN, "checksums.json")) as f:
        return json.load(f)[name]


def _check_gold(e, r, cks):
    assert (r.positions, r.edges, r.primitives, r.root_line) == (e["positions"], e["edges"], e["primitives"],
                                                                  e["root_line"])
    tot = sum(int(c["checksum"], 16) for c in cks) % (1 << 64)
    assert "%016x" % tot == e["checksum"]
    assert sum(c["positions"] for c in cks) == e["positions"]
    assert (sum(c["win"] for c in cks), sum(c["loss"] for c in cks)) == (e["win"], e["loss"])


@pytest.mark.parametrize("flags", [0, LEVELS])
def test_planes_sum_31x6_checksum(flags):
    """BASELINE config 4, the bench shape (2^30 positions): every position's
    value and remoteness by fingerprint against the CPU restatement -- the
    one-launch backward (the bench's) and the per-level launches."""
    e = _gold("sum_31x6")
    s, r = _planes(e["params"], flags=flags)
    assert r.extra["word_bits"] == 8
    assert r.extra["resolve_kernel"] == ("k_plane_resolve_x2" if flags else "k_plane_flow")
    _check_gold(e, r, [s.checksum()])
    r2 = s.solve()  # again on the same table: the flags' epochs and the ticket counters start over
    _check_gold(e, r2, [s.checksum()])


LS, RR = 4096, 2048  # GM_F_PLANE_LEVEL_SYNC, GM_F_PLANE_ROUND_ROBIN
GROUP_CASES = [  # world, params, flags: the deal each exercises
    (2, "heaps=31:31:3:15", 0),         # staged, blocks of 8
    (3, "heaps=31:31:3:23", 0),         # staged, blocks of 8
    (4, "heaps=31:31:3:15", 0),         # staged, blocks of 4
    (8, "heaps=31:31:3:15", 0),         # staged, blocks of 2 (the halo is a whole block)
    (3, "heaps=31:31:3:63", 0),         # 64 values / 3 ranks: level-synchronous, round robin
    (2, "heaps=31:31:3:15", LS),        # level-synchronous
    (4, "heaps=31:31:3:63", LS),        # level-synchronous, link-spreading deal (two rounds)
    (8, "heaps=31:31:1:127", LS),       # level-synchronous, link-spreading deal
    (4, "heaps=31:31:3:63", LS | RR),   # level-synchronous, round robin
]


@pytest.mark.parametrize("world,params,flags", GROUP_CASES)
def test_planes_group_matches_single(world, params, flags):
    """Shards of the PLANES layout solved as an in-process group, for every
    deal (the staged pipeline: one block per rank, halo rows copied as they
    complete; the level-synchronous deals: boundary slices exchanged per
    plane level): every position answered by exactly one shard, word-equal
    to the one-table solve."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    s1, r1 = _planes(params)
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world, flags=flags)
    assert rg.extra["layout"] == "planes"
    assert (rg.positions, rg.edges, rg.primitives, rg.root_line) == (r1.positions, r1.edges, r1.primitives,
                                                                      r1.root_line)
    keys = s1.positions()
    want = s1.query(keys)
    out = np.full(len(keys), 0xFFFFFFFF, np.uint32)
    hits = np.zeros(len(keys), np.int64)
    for sh in shards:
        w = sh.query(keys)
        own = w != 0xFFFFFFFF
        out[own] = w[own]
        hits += own
    assert (hits == 1).all()
    np.testing.assert_array_equal(out, want)
    assert sum(len(sh.positions()) for sh in shards) == len(keys)


@pytest.mark.parametrize("world", [2, 4])
def test_planes_group_matches_oracle(world):
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    params = "heaps=31:31:2:7"
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world)
    sol = _oracle(params)
    assert (rg.positions, rg.edges, rg.root_line) == (sol.count, sol.edges, sol.root_line)
    keys = np.arange(sol.count, dtype=np.uint64)
    want = _oracle_words(sol, sol.count)
    got = np.full(sol.count, 0xFFFFFFFF, np.uint32)
    for sh in shards:
        w = sh.query(keys)
        own = w != 0xFFFFFFFF
        assert (got[own] == 0xFFFFFFFF).all()
        got[own] = w[own]
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("cut", [1, 187, 187 + 40, 187 + 124])
def test_planes_stop_resume(cut):
    """Stop after step `cut` (forward; mid-backward; the last plane level)
    and resume in the same solver: identical words and counts."""
    params = "heaps=31:31:31:31:31:31"
    e = _gold("sum_31x6")
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("sum_four_to_one", e["params"]), layout="planes")
    assert s.solve_steps(0, cut) is None
    r = s.solve_steps(cut, 0)
    _check_gold(e, r, [s.checksum()])
    del params


@pytest.mark.parametrize("world", [2, 4])
def test_planes_group_pipelined_equals_in_order(world):
    """Level-synchronous shards exchange each level's boundary planes on a
    comm stream while the next launches run (own part / boundary part split, the RCCL path's
    schedule); GM_F_SHARD_INORDER exchanges after each whole level.  Same
    words either way."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec("sum_four_to_one", "heaps=31:31:7:7:15")
    ls = _lib.GM_F_PLANE_LEVEL_SYNC
    rp, sp = group_solve(spec, world, flags=ls)
    ri, si = group_solve(spec, world, flags=ls | _lib.GM_F_SHARD_INORDER)
    assert (rp.positions, rp.edges, rp.root_line) == (ri.positions, ri.edges, ri.root_line)
    keys = np.arange(32 * 32 * 8 * 8 * 16, dtype=np.uint64)
    for a, b in zip(sp, si):
        np.testing.assert_array_equal(a.query(keys), b.query(keys))


@pytest.mark.parametrize("flags", [LEVELS, 64, 1024])  # 8-bit packed, 16-bit, one plane per half-wave
def test_planes_runs_equal_single_launches(flags):
    """Narrow plane levels run as one-workgroup runs (k_plane_run, a
    barrier between levels) give the words of one grid launch per level
    (GM_F_PLANE_NO_RUNS), for every kernel family."""
    from gamesmanmpi_amd import _lib
    params = "heaps=31:31:7:7:15"
    sa, ra = _planes(params, flags=flags)
    sb, rb = _planes(params, flags=flags | _lib.GM_F_PLANE_NO_RUNS)
    assert (ra.positions, ra.edges, ra.root_line) == (rb.positions, rb.edges, rb.root_line)
    keys = np.arange(32 * 32 * 8 * 8 * 16, dtype=np.uint64)
    np.testing.assert_array_equal(sa.query(keys), sb.query(keys))
    assert sa.checksum() == sb.checksum()


# Relative 8-bit order forms (gm_plane.h, word form 3): root digit sums
# 254 .. 505 -- remoteness beyond the absolute 8-bit forms' 254 -- in one byte
# per position, each word taken relative to its digit sum's window.
REL_CASES = ["heaps=31:31:200",      # root sum 262: the smallest kind, one outer heap
             "heaps=31:31:3:230",    # 295, every d % 4 class on both phases
             "heaps=31:31:443"]      # 505 = kPlaneRelMaxSum: the window's edge


@pytest.mark.parametrize("params", REL_CASES)
def test_planes_relative_match_oracle(params):
    """Every position's value and remoteness equals the oracle's at root
    digit sums above 253 (relative forms: 8-bit words, the packed kernel)."""
    s, r = _planes(params)
    sol = _oracle(params)
    assert r.extra["word_bits"] == 8 and r.extra["resolve_kernel"] == "k_plane_resolve_x2"
    assert (r.positions, r.edges, r.primitives, r.root_line) == (sol.count, sol.edges, sol.stats["primitives"],
                                                                  sol.root_line)
    keys = np.arange(sol.count, dtype=np.uint64)
    np.testing.assert_array_equal(s.query(keys), _oracle_words(sol, sol.count))
    ck = s.checksum()
    assert (ck["checksum"], ck["win"], ck["loss"]) == ("%016x" % sol.stats["checksum"], sol.stats["win"],
                                                       sol.stats["loss"])


def test_planes_relative_root_beyond_absolute_bytes():
    """A root whose remoteness itself exceeds 254 (the absolute 8-bit forms'
    limit), and one digit sum past the relative window: 16-bit words."""
    from gamesmanmpi_amd import _lib
    s, r = _planes("heaps=31:31:3:400")  # root sum 465
    assert r.extra["word_bits"] == 8 and r.root_remoteness > 254
    s16, r16 = _planes("heaps=31:31:3:400", flags=_lib.GM_F_WORDS16)
    assert r16.extra["word_bits"] == 16 and r16.root_line == r.root_line
    keys = np.arange(32 * 32 * 4 * 401, dtype=np.uint64)
    np.testing.assert_array_equal(s.query(keys), s16.query(keys))
    assert s.checksum() == s16.checksum()
    _, rw = _planes("heaps=31:31:444")  # root sum 506
    assert rw.extra["word_bits"] == 16


def test_planes_relative_runs_and_resume():
    """Relative forms: one-workgroup runs (per-group specialisation by the
    outer digit sum mod 4) equal one launch per level, and a solve stopped
    mid-backward resumes to the same words."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    params = "heaps=31:31:7:7:200"  # root sum 276
    sa, ra = _planes(params)
    sb, rb = _planes(params, flags=_lib.GM_F_PLANE_NO_RUNS)
    assert ra.extra["word_bits"] == 8 and ra.root_line == rb.root_line
    keys = np.arange(32 * 32 * 8 * 8 * 201, dtype=np.uint64)
    w = sa.query(keys)
    np.testing.assert_array_equal(w, sb.query(keys))
    sc = Solver(GameSpec("sum_four_to_one", params), layout="planes")
    T = sc.steps // 2
    assert sc.solve_steps(0, T + 101) is None
    rc = sc.solve_steps(T + 101, 0)
    assert rc.root_line == ra.root_line
    np.testing.assert_array_equal(sc.query(keys), w)


REL_GROUP_CASES = [
    (4, "heaps=31:31:3:255", 0, "one"),    # staged, k = 5, blocks of 64
    (8, "heaps=31:31:3:255", 0, "own"),    # staged, blocks of 32, the RCCL schedule's rehearsal
    (2, "heaps=31:31:3:255", 0, "one"),    # staged, k = 5 (1 mod 4) also for two ranks
    (8, "heaps=31:31:1:255", LS, "one"),   # level-synchronous, link-spreading deal
]


@pytest.mark.parametrize("world,params,flags,streams", REL_GROUP_CASES)
def test_planes_relative_group_matches_oracle(world, params, flags, streams):
    """Relative forms on shards (the 4- and 8-GPU bench shapes' word form):
    every position's word from its one owner equals the oracle's."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world, flags=flags, streams=streams)
    sol = _oracle(params)
    assert rg.extra["word_bits"] == 8
    assert (rg.positions, rg.edges, rg.root_line) == (sol.count, sol.edges, sol.root_line)
    keys = np.arange(sol.count, dtype=np.uint64)
    want = _oracle_words(sol, sol.count)
    got = np.full(sol.count, 0xFFFFFFFF, np.uint32)
    for sh in shards:
        w = sh.query(keys)
        own = w != 0xFFFFFFFF
        assert (got[own] == 0xFFFFFFFF).all()
        got[own] = w[own]
    np.testing.assert_array_equal(got, want)


ROW_GROUP_CASES = [  # the row deal: heap 1 holds 32 values per rank
    (2, "heaps=31:63:3:15", "one"),
    (2, "heaps=31:63:3:15", "own"),
    (2, "heaps=31:63:7", "own"),          # one outer heap
    (3, "heaps=31:95:2:7", "own"),
    (4, "heaps=31:127:31:31", "one"),     # 4.2e6 positions, two outer heaps of 32
    (8, "heaps=31:255:3:3", "own"),       # root digit sum 292: relative words
    (8, "heaps=31:255:1:1:1", "one"),     # relative words, three outer heaps
]


@pytest.mark.parametrize("world,params,streams", ROW_GROUP_CASES)
def test_planes_row_deal_group_matches_oracle(world, params, streams):
    """The row deal (gm_plane_run.h plane_shape): rank r owns heap-1 values
    [32r, 32r + 32) of every plane and streams each level's rows 30, 31 to
    rank r + 1.  One stream (halo copies in order) and own streams (mode 4,
    the RCCL schedule's rehearsal): every position's word, answered by its
    one owner, equals the oracle's."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world, streams=streams)
    sol = _oracle(params)
    assert rg.extra["layout"] == "planes"
    assert (rg.positions, rg.edges, rg.primitives, rg.root_line) == (sol.count, sol.edges, sol.stats["primitives"],
                                                                     sol.root_line)
    keys = np.arange(sol.count, dtype=np.uint64)
    want = _oracle_words(sol, sol.count)
    got = np.full(sol.count, 0xFFFFFFFF, np.uint32)
    for sh in shards:
        w = sh.query(keys)
        own = w != 0xFFFFFFFF
        assert (got[own] == 0xFFFFFFFF).all()
        got[own] = w[own]
    np.testing.assert_array_equal(got, want)


def test_planes_queued_solves_equal_blocking_ones():
    """gm_solver_solve_async / gm_solver_collect (the bench's timed loop):
    queued one-table solves run back to back and each one's counts, root
    and fingerprint equal a blocking solve's; tickets are collected in
    order, at most 8 outstanding, and a misuse is an error, not a hang."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("sum_four_to_one", "heaps=31:31:9:6:3"))
    r0 = s.solve()
    assert r0.extra["layout"] == "planes"
    ck0 = s.checksum()["checksum"]
    want = (r0.positions, r0.edges, r0.primitives, r0.root_line)
    tickets = [s.solve_async() for _ in range(8)]
    assert tickets == list(range(tickets[0], tickets[0] + 8))
    with pytest.raises(_lib.GmError):  # the ring is full
        s.solve_async()
    with pytest.raises(_lib.GmError):  # out of order
        s.collect(tickets[1])
    for t in tickets:
        r = s.collect(t)
        assert (r.positions, r.edges, r.primitives, r.root_line) == want
        assert r.ms_total > 0 and r.ms_backward > 0
    assert s.checksum()["checksum"] == ck0
    t = s.solve_async()  # interleaved with a blocking solve
    r1 = s.solve()
    r2 = s.collect(t)
    assert (r1.positions, r1.root_line) == (r2.positions, r2.root_line) == (want[0], want[3])
    assert s.checksum()["checksum"] == ck0
