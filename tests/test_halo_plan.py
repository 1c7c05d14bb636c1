"""Fail-fast exchange plan of sharded dense solves (gm_shard_halo_sigs, host
only): for every level, what a rank sends must be exactly what its
neighbour posts to receive -- bits go down, words go up (DESIGN.md
§Multi-GPU; the check gm_solver_solve runs over RCCL / the host transport
before level 0 and turns into GM_ECORRUPT instead of a hung receive).
Covers the bench's 2^30 shape at N = 2, 4, 8 and the test shapes."""
import numpy as np
import pytest

from gamesmanmpi_amd.dist import halo_sigs
from gamesmanmpi_amd.games import GameSpec


def _pairs_match(spec, world):
    sig = [halo_sigs(spec, r, world) for r in range(world)]
    for r in range(world):
        down, up = (r - 1) % world, (r + 1) % world
        np.testing.assert_array_equal(sig[r][:, 0], sig[down][:, 1], err_msg="bits r=%d" % r)
        np.testing.assert_array_equal(sig[r][:, 2], sig[up][:, 3], err_msg="words r=%d" % r)
    return sig


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_shape_plans_pair(world):
    spec = GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31")
    sig = _pairs_match(spec, world)
    # messages exist: some level sends words and bits on some rank
    empty = np.uint64(1469598103934665603)  # fingerprint of "no message"
    assert any((s[:, 2] != empty).any() for s in sig)
    assert any((s[:, 0] != empty).any() for s in sig)


@pytest.mark.parametrize("params,world", [("heaps=15:15:15:15:31", 2), ("heaps=15:15:15:15:31", 3),
                                          ("heaps=15:15:15:15:127", 8), ("heaps=7:7:7:7:7", 2)])
def test_test_shape_plans_pair(params, world):
    _pairs_match(GameSpec("sum_four_to_one", params), world)


def test_a_wrong_geometry_is_detected():
    """Fingerprints of a different world do not pair: the check that turns
    a mis-launched rank into GM_ECORRUPT would fire."""
    spec = GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31")
    a = halo_sigs(spec, 0, 4)
    b = halo_sigs(spec, 1, 8)  # rank 1 of a different world
    assert (a[:, 2] != b[:, 3]).any()
