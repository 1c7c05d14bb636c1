"""Sharded dense solves on ONE GPU: every shard of a
job runs in this process (gm_solve_group) with the same kernels and halo
geometry the RCCL path uses, and must agree word-for-word with the
unsharded solve and the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _single(params):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    return s.solve(), s


def _group(params, world):
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    return group_solve(GameSpec("sum_four_to_one", params), world)


def _words_by_owner(shards, keys):
    """Each key answered by the shard that owns it (others: NO_WORD)."""
    out = np.full(len(keys), 0xFFFFFFFF, np.uint32)
    hits = np.zeros(len(keys), np.int64)
    for s in shards:
        w = s.query(keys)
        own = w != 0xFFFFFFFF
        out[own] = w[own]
        hits += own
    return out, hits


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_group_matches_single(world):
    params = "heaps=7:7:7:15"  # top heap 16 values; slices of 64 prefixes
    r1, s1 = _single(params)
    rg, shards = _group(params, world)
    assert (rg.positions, rg.edges, rg.primitives, rg.root_line) == (
        r1.positions, r1.edges, r1.primitives, r1.root_line)
    keys, val, rem = s1.dump()
    w, hits = _words_by_owner(shards, keys)
    assert (hits == 1).all()  # every position owned by exactly one shard
    np.testing.assert_array_equal(w & 3, val)
    np.testing.assert_array_equal(w >> 2, rem)


def test_group_matches_oracle():
    from oracle.oracle import Game
    params = "heaps=3:3:15:7"  # Z = 4*16 = 64, top heap 8 values
    rg, shards = _group(params, 4)
    sol = Game("sum_four_to_one", params).solve(1 << 14)
    assert (rg.positions, rg.edges, rg.root_line) == (sol.count, sol.edges,
                                                      sol.root_line)
    keys = np.arange(4 * 4 * 16 * 8, dtype=np.uint64)
    w, hits = _words_by_owner(shards, keys)
    assert (hits == 1).all()
    for k in keys.tolist():
        assert sol.lookup(str(k).encode()) == (w[k] & 3, w[k] >> 2), k


def test_bench_geometry_two_shards():
    """The N=2 bench workload's shape (31^k x 63: blocks of 8 top values,
    four per rank, round robin, packed word halos) at one GPU's scale:
    31:31:31:31:63 = 2^26 positions."""
    params = "heaps=31:31:31:31:63"
    r1, s1 = _single(params)
    rg, shards = _group(params, 2)
    assert (rg.positions, rg.edges, rg.root_line) == (r1.positions, r1.edges,
                                                      r1.root_line)
    rng = np.random.default_rng(1)
    keys = rng.integers(0, 32 ** 4 * 64, size=1 << 16, dtype=np.uint64)
    w, hits = _words_by_owner(shards, keys)
    assert (hits == 1).all()
    np.testing.assert_array_equal(w, s1.query(keys))


@pytest.mark.parametrize("world", [2, 3])
def test_non_pow2_round_robin_blocks(world):
    """A top heap of 48 values (not a power of two: per-lane kernels,
    division-based block mapping, unpacked band-clipped word halos), blocks
    of 8 dealt round robin; every position's word equal to the unsharded
    solve's."""
    params = "heaps=3:7:15:47"
    r1, s1 = _single(params)
    rg, shards = _group(params, world)
    assert (rg.positions, rg.edges, rg.primitives, rg.root_line) == (
        r1.positions, r1.edges, r1.primitives, r1.root_line)
    keys, val, rem = s1.dump()
    w, hits = _words_by_owner(shards, keys)
    assert (hits == 1).all()
    np.testing.assert_array_equal(w & 3, val)
    np.testing.assert_array_equal(w >> 2, rem)


def test_bad_geometry_is_refused():
    from gamesmanmpi_amd import _lib
    with pytest.raises(_lib.GmError):
        _group("heaps=7:7:7:15", 16)  # blocks of 1 top value: halo spans ranks


@pytest.mark.parametrize("world,params,npos", [
    (3, "heaps=31:31:31:31:127", 32 ** 4 * 128),   # 16 blocks: 6 / 5 / 5 per rank
    (4, "heaps=31:31:31:31:127", 32 ** 4 * 128),   # the N=4 bench shape, smaller
    (8, "heaps=31:31:31:255", 32 ** 3 * 256),      # the N=8 bench shape, smaller
    (2, "heaps=31:31:31:3:15", 32 ** 3 * 4 * 16),  # one block per rank
])
def test_pipelined_halo_exchange_wide_blocks(world, params, npos):
    """Blocks of >= 4 top values take the overlapped schedule (own part,
    exchange on the comm stream, boundary slices after the previous level's
    halo arrived) with packed word halos; every sampled word equal to the
    unsharded solve's."""
    r1, s1 = _single(params)
    rg, shards = _group(params, world)
    assert (rg.positions, rg.edges, rg.root_line) == (r1.positions, r1.edges, r1.root_line)
    rng = np.random.default_rng(world)
    keys = rng.integers(0, npos, size=1 << 18, dtype=np.uint64)
    w, hits = _words_by_owner(shards, keys)
    assert (hits == 1).all()
    np.testing.assert_array_equal(w, s1.query(keys))
