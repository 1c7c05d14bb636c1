"""The md5-sharded keyed level loop (gamesmanmpi_amd.keyed.keyed_solve) on
CPU: in-process groups (GroupExchange) and gloo worlds 2 and 3
(TorchExchange), each rank's shard the test-only HostShard.  Checks the
whole job against the reference's golden tables bit-exactly, and that every
position lives on its md5 owner (src/game_state.py:22-30)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import CASES, load_table


def _spec(name):
    from gamesmanmpi_amd.games import GameSpec
    return GameSpec(*CASES[name])


def _check_tables(name, spec, dumps, world):
    keys = np.concatenate([d[0] for d in dumps])
    val = np.concatenate([d[1] for d in dumps])
    rem = np.concatenate([d[2] for d in dumps])
    assert len(np.unique(keys)) == len(keys), "a position on two shards"
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


@pytest.mark.parametrize("name,world", [
    ("tic_tac_toe_np", 1), ("tic_tac_toe_np", 4), ("mttt", 3),
    ("four_to_one_20", 2), ("sum_fto_2_5_7", 5), ("toot_3x3", 8), ("four_to_one", 5),
])
def test_group_keyed_matches_golden(name, world, golden_summary):
    from gamesmanmpi_amd.keyed import GroupExchange, keyed_solve
    from keyed_host import HostShard
    spec = _spec(name)
    shards = [HostShard(spec, g, world) for g in range(world)]
    r = keyed_solve(shards, GroupExchange())
    info = golden_summary[name]
    assert r.positions == info["positions"]
    assert r.edges == info["edges"]
    assert r.primitives == info["primitives"]
    assert r.root_line == info["root_line"]
    _check_tables(name, spec, [s.dump() for s in shards], world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from gamesmanmpi_amd.keyed import TorchExchange, keyed_solve
        from keyed_host import HostShard
        spec = _spec(name)
        shard = HostShard(spec, rank, world)
        r = keyed_solve([shard], TorchExchange(torch.device("cpu")))
        q.put((rank, (r.positions, r.edges, r.primitives, r.root_line,
                      r.levels), shard.dump()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("tic_tac_toe_np", 2), ("mttt", 3)])
def test_gloo_keyed_matches_golden(name, world, golden_summary):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    info = golden_summary[name]
    for _, totals, _ in out:
        assert totals == out[0][1]  # every rank reports the whole job
    assert out[0][1][:4] == (info["positions"], info["edges"],
                             info["primitives"], info["root_line"])
    _check_tables(name, _spec(name), [d for _, _, d in out], world)
