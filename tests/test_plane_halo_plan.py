"""Halo plans of PLANES shards (gm_plane_halo_plan, host only): what every
shard sends to each peer after each plane level is exactly what that peer
posts to receive from it, for the round-robin deal and for the link-
spreading deal -- the pairing the RCCL exchange relies on.
The spreading deal must put a shard's halo on world / 2 links at N = 4 and 8
(bench shapes) while moving the same planes in total."""
import numpy as np
import pytest

from gamesmanmpi_amd._lib import GM_F_PLANE_ROUND_ROBIN
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
    spread = _plans(params, world)
    rr = _plans(params, world, GM_F_PLANE_ROUND_ROBIN)
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
    _plans(params, world, GM_F_PLANE_ROUND_ROBIN)


def test_spreading_deal_only_where_it_applies():
    """Non-power-of-two worlds and partial rounds keep the round-robin deal:
    every shard's halo goes to rank + 1."""
    for params, world in (("heaps=31:31:3:47", 3), ("heaps=31:31:3:15", 4)):
        for r, plan in enumerate(_plans(params, world)):
            assert _peers(plan) in ([(r + 1) % world], [])
