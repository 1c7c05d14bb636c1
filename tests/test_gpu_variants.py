"""GPU parity of every dense resolve variant: the A/B knobs
select other kernels / sweep orders for the same solve, and each must give
the same words as the default path, the closed-form counts and the
Sprague-Grundy values.  Shapes exercise the quad kernels' paths: live-group
lists with top-major XCD shares (C >= 8 columns), column jobs, column walks,
the unpipelined and the one-prefix kernels, and shard halos in 16 and 32
bits."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD1 = [
    {},
    {"GM_WORDS32": "1"},
    {"GM_DENSE_PIPE": "0"},
    {"GM_DENSE_SWEEP": "cols"},
    {"GM_DENSE_SWEEP": "walk"},
    {"GM_DENSE_RESOLVE": "scalar"},
    {"GM_PULL_BAND": "1"},
    {"GM_GROUP_TILE": "-1"},
    {"GM_GROUP_TILE": "4"},
]


def _expected(heaps):
    P = 1
    for h in heaps:
        P *= h + 1
    E = sum(P * (2 * h - 1) // (h + 1) for h in heaps if h >= 1)
    g = 0
    for h in heaps:
        g ^= h % 3
    return P, E, "LOSS" if g == 0 else "WIN"


def _solve(params, monkeypatch, env):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    for k in ("GM_DENSE_PIPE", "GM_DENSE_SWEEP", "GM_DENSE_RESOLVE", "GM_PULL_BAND", "GM_GROUP_TILE",
              "GM_WORDS32"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    r = s.solve()
    keys, val, rem = s.dump()
    order = np.argsort(keys)
    return r, keys[order], val[order], rem[order]


@pytest.mark.parametrize("params", ["heaps=15:15:15:15:7", "heaps=31:7:31:15"])
def test_world1_variants_agree(params, monkeypatch):
    heaps = [int(h) for h in params.split("=")[1].split(":")]
    P, E, root = _expected(heaps)
    base = None
    for env in WORLD1:
        r, keys, val, rem = _solve(params, monkeypatch, env)
        assert (r.positions, r.edges, r.root_line.split()[0]) == (P, E, root), env
        if base is None:
            base = (keys, val, rem)
            # Sprague-Grundy: LOSS iff the XOR of (heap mod 3) is 0
            k = keys.astype(np.int64)
            g = np.zeros(len(k), np.int64)
            for h in heaps:
                g ^= (k % (h + 1)) % 3
                k //= h + 1
            np.testing.assert_array_equal(val == 1, g == 0)
            continue
        np.testing.assert_array_equal(keys, base[0], err_msg=str(env))
        np.testing.assert_array_equal(val, base[1], err_msg=str(env))
        np.testing.assert_array_equal(rem, base[2], err_msg=str(env))


@pytest.mark.parametrize("env", [{}, {"GM_HALO_COLS4": "1"}, {"GM_WORDS32": "1"}, {"GM_HALO32": "1"},
                                 {"GM_PULL_COLS": "1"}])
@pytest.mark.parametrize("world", [2, 3])
def test_shard_halo_word_widths(env, world, monkeypatch):
    """Column-order halos (Z % 256 == 0): 16-bit shard tables with 16-bit
    halos (default, k_dense_resolve8c), 32-bit tables with 16-bit halos,
    32-bit tables and halos -- each against the single-table solve."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    params = "heaps=15:15:15:15:31"  # Z = 16^3 = 4096 prefixes (16 columns) per slice
    for k in ("GM_HALO32", "GM_WORDS32", "GM_HALO_COLS4", "GM_PULL_COLS"):
        monkeypatch.delenv(k, raising=False)
    s1 = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    r1 = s1.solve()
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world)
    assert (rg.positions, rg.edges, rg.root_line) == (r1.positions, r1.edges, r1.root_line)
    wide = "GM_WORDS32" in env or "GM_HALO32" in env
    assert rg.extra["word_bits"] == (32 if wide else 16), rg.extra
    keys, val, rem = s1.dump()
    out = np.full(len(keys), 0xFFFFFFFF, np.uint32)
    for s in shards:
        w = s.query(keys)
        own = w != 0xFFFFFFFF
        out[own] = w[own]
    np.testing.assert_array_equal(out & 3, val)
    np.testing.assert_array_equal(out >> 2, rem)


@pytest.mark.parametrize("world,params", [(8, "heaps=15:15:15:15:127"), (4, "heaps=15:15:15:15:63"),
                                          (8, "heaps=15:15:15:15:31")])
def test_shard_geometries_like_the_bench(world, params):
    """The bench's N-rank structure at a smaller slice size: round-robin
    blocks of 8 top values (two per rank at N = 8), 16-bit tables, packed
    16-bit halos in column order.  The in-process group checks every level's
    halo word count against what the receiving rank would post (the RCCL
    path's receive size) and the words against the single-table solve."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s1 = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    r1 = s1.solve()
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world)
    assert (rg.positions, rg.edges, rg.root_line) == (r1.positions, r1.edges, r1.root_line)
    assert rg.extra["word_bits"] == 16
    keys, val, rem = s1.dump()
    out = np.full(len(keys), 0xFFFFFFFF, np.uint32)
    hits = np.zeros(len(keys), np.int64)
    for s in shards:
        w = s.query(keys)
        own = w != 0xFFFFFFFF
        out[own] = w[own]
        hits += own
    assert (hits == 1).all()
    np.testing.assert_array_equal(out & 3, val)
    np.testing.assert_array_equal(out >> 2, rem)
