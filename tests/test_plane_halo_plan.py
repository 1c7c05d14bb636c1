"""Halo plans of PLANES shards (gm_plane_halo_plan, host only): what every
shard sends to each peer at each step is exactly what that peer posts to
receive from it -- the pairing the RCCL exchange relies on -- for the staged
pipeline (steps = halo rows, one block per rank, sends to rank + 1 only) and
the level-synchronous deals (steps = plane levels; round robin, and the
link-spreading deal that must put a shard's halo on world / 2 links at N = 4
and 8 while moving the same planes in total).  DESIGN.md §6a."""
import numpy as np
import pytest

from gamesmanmpi_amd._lib import GM_F_PLANE_LEVEL_SYNC, GM_F_PLANE_ROUND_ROBIN
from gamesmanmpi_amd.dist import plane_halo_plan
from gamesmanmpi_amd.games import GameSpec


def _plans(params, world, flags=0):
    spec = GameSpec("sum_four_to_one", params)
    plans = [plane_halo_plan(spec, r, world, flags) for r in range(world)]
    for r in range(world):
        for p in range(world):
            np.testing.assert_array_equal(plans[r][:, p, 0], plans[p][:, r, 1],
                                          err_msg="shard %d -> %d" % (r, p))
        assert not plans[r][:, r, :].any()  # never itself
    return plans


def _peers(plan):
    return sorted(int(p) for p in np.nonzero(plan[:, :, 0].sum(axis=0))[0])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_shape_spreads_links(world):
    params = "heaps=31:31:31:31:31:%d" % (32 * world - 1)
    spread = _plans(params, world, GM_F_PLANE_LEVEL_SYNC)
    rr = _plans(params, world, GM_F_PLANE_LEVEL_SYNC | GM_F_PLANE_ROUND_ROBIN)
    total = lambda ps: sum(int(p[:, :, 0].sum()) for p in ps)
    assert total(spread) == total(rr) > 0
    for r in range(world):
        assert _peers(rr[r]) in ([(r + 1) % world], [])
        # world 2: one peer either way; 4: two links; 8: four
        want = 1 if world == 2 else world // 2
        assert len(_peers(spread[r])) in (want, want - 1 if r else want)
    if world >= 4:
        # the busiest link carries at most ~1 / (world / 2) of what the one
        # round-robin link does (plus one block's share for the round seams)
        busiest = max(int(p[:, :, 0].sum(axis=0).max()) for p in spread)
        rr_link = max(int(p[:, :, 0].sum()) for p in rr)
        assert busiest <= rr_link * (2.0 / world + 0.3)


@pytest.mark.parametrize("params,world", [("heaps=31:31:3:15", 2), ("heaps=31:31:3:23", 3),
                                          ("heaps=31:31:3:63", 4), ("heaps=31:31:1:127", 8),
                                          ("heaps=31:31:3:3:47", 3), ("heaps=31:31:7:7", 4)])
def test_test_shape_plans_pair(params, world):
    _plans(params, world)
    _plans(params, world, GM_F_PLANE_LEVEL_SYNC)
    _plans(params, world, GM_F_PLANE_LEVEL_SYNC | GM_F_PLANE_ROUND_ROBIN)


def test_spreading_deal_only_where_it_applies():
    """Non-power-of-two worlds and partial rounds keep the round-robin deal:
    every shard's halo goes to rank + 1."""
    for params, world in (("heaps=31:31:3:47", 3), ("heaps=31:31:3:15", 4)):
        for r, plan in enumerate(_plans(params, world, GM_F_PLANE_LEVEL_SYNC)):
            assert _peers(plan) in ([(r + 1) % world], [])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_staged_bench_shape_rows(world):
    """The staged pipeline on the bench shapes: one block of 32 top values
    per rank, the halo = the last two slices, sent to rank + 1 row by row
    (one row per lower-digit sum 0..93), 2 x 32^3 planes per step in all."""
    params = "heaps=31:31:31:31:31:%d" % (32 * world - 1)
    plans = _plans(params, world)
    Z = 32 ** 3
    cls = np.convolve(np.convolve(np.ones(32), np.ones(32)), np.ones(32)).astype(np.int64)
    for r, plan in enumerate(plans):
        sent = plan[:, :, 0].sum(axis=1).astype(np.int64)
        assert _peers(plan) == ([r + 1] if r + 1 < world else [])
        if r + 1 < world:
            assert sent.sum() == 2 * Z
            np.testing.assert_array_equal(sent[:94], 2 * cls)
            assert not sent[94:].any()
        got = plan[:, :, 1].sum(axis=1).astype(np.int64)
        assert got.sum() == (2 * Z if r else 0)


def test_staged_only_where_blocks_divide():
    """A last heap whose values do not split evenly over the ranks keeps the
    level-synchronous deal (steps = plane levels, more of them than rows)."""
    spec_params, world = "heaps=31:31:3:23", 3  # 24 values / 3 ranks: staged, rows 0..3
    plans = _plans(spec_params, world)
    assert all(not p[4:].any() for p in plans)
    plans = _plans("heaps=31:31:3:63", 3)  # 64 values: not divisible by 3
    assert any(p[4:].any() for p in plans)


@pytest.mark.parametrize("params,world", [("heaps=31:63:3:15", 2), ("heaps=31:95:2:7", 3),
                                          ("heaps=31:127:31:31:31:31", 4), ("heaps=31:255:31:31:31:31", 8)])
def test_row_deal_plans(params, world):
    """The row deal (heap 1 in 32-row slabs): step = plane level, every
    level's planes travel from rank r to rank r + 1 only (two rows each: the
    unit is a list entry), rank 0 receives and the last rank sends nothing,
    and a level carries exactly its plane count."""
    plans = _plans(params, world)
    outer = [int(h) + 1 for h in params.split("=")[1].split(":")[2:]]
    n = np.ones(1, np.int64)
    for b in outer:
        n = np.convolve(n, np.ones(b, np.int64))
    for r in range(world):
        assert _peers(plans[r]) == ([r + 1] if r + 1 < world else [])
        if r + 1 < world:
            np.testing.assert_array_equal(plans[r][:len(n), r + 1, 0], n)
            assert not plans[r][len(n):, :, :].any()
    assert not plans[0][:, :, 1].any()
