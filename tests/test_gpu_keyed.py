"""GPU: md5-sharded keyed solves through the gm_ks_* ABI, every shard of a
job in one process on one MI355X (GroupExchange; the RCCL variant differs
only in the exchange object).  Bit-exact against the reference's golden
tables; every position must sit on its md5 owner (src/game_state.py:22-30).
BASELINE config 5 is othello 4x4 over 8 ranks."""
import numpy as np
import pytest

from conftest import CASES, load_table

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,world", [
    ("othello_4x4", 8), ("othello_4x4", 3), ("tic_tac_toe_np", 2),
    ("mttt", 5), ("toot_3x3", 4), ("toot_4x3", 8), ("four_to_one_64", 3),
    ("sum_fto_6_6_6_6", 7),
])
def test_gpu_group_keyed_matches_golden(name, world, golden_summary):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    spec = GameSpec(*CASES[name])
    r, shards = group_keyed_solve(spec, world)
    info = golden_summary[name]
    assert (r.positions, r.edges, r.primitives) == (
        info["positions"], info["edges"], info["primitives"])
    assert r.root_line == info["root_line"]
    dumps = [s.dump() for s in shards]
    keys = np.concatenate([d[0] for d in dumps])
    val = np.concatenate([d[1] for d in dumps])
    rem = np.concatenate([d[2] for d in dumps])
    assert len(np.unique(keys)) == len(keys)
    for rank, d in enumerate(dumps):
        if len(d[0]):
            assert (spec.owners_host(d[0], world) == rank).all()
    t = load_table(name)
    canon, clen = spec.decode_batch(keys, stride=t["canon"].shape[1])
    order = np.array(sorted(range(len(keys)),
                            key=lambda i: bytes(canon[i, :clen[i]])), np.int64)
    np.testing.assert_array_equal(canon[order], t["canon"])
    np.testing.assert_array_equal(val[order], t["value"])
    np.testing.assert_array_equal(rem[order], t["remoteness"])


def test_gpu_keyed_shard_refuses_whole_solve():
    """A keyed shard of a world > 1 job cannot be solved alone."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import GpuShard
    sh = GpuShard(GameSpec("tic_tac_toe_np", ""), 0, 2)
    with pytest.raises(_lib.GmError):
        sh.solver.solve()
