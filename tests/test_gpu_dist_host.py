"""Sharded dense solves, one process per rank, over the host-staged
transport (gamesmanmpi_amd.dist.HostTransport over torch.distributed gloo):
the RCCL path's geometry, halo plan check and reductions with the transfers
carried through host memory, so two ranks can share one GPU.  Every
position's word equals the single-table solve's; totals equal on every
rank."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PARAMS = "heaps=15:15:15:15:31"


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gamesmanmpi_amd.dist import ShardedSolver
        from gamesmanmpi_amd.games import GameSpec
        spec = GameSpec("sum_four_to_one", PARAMS)
        s = ShardedSolver(spec, rank, world, device="cuda:0", transport="host")
        r = s.solve()
        from gamesmanmpi_amd.solver import Solver
        s1 = Solver(spec, device="cuda:0", layout="dense")
        keys, val, rem = s1.dump()
        w = s.query(keys)
        q.put((rank, (r.positions, r.edges, r.primitives, r.root_line), keys, val, rem, w))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_transport_matches_single_table(world):
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=200) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    r1 = Solver(GameSpec("sum_four_to_one", PARAMS), layout="dense").solve()
    for o in out:
        assert o[1] == (r1.positions, r1.edges, r1.primitives, r1.root_line)
    keys, val, rem = out[0][2], out[0][3], out[0][4]
    words = np.full(len(keys), 0xFFFFFFFF, np.uint64)
    hits = np.zeros(len(keys), np.int64)
    for o in out:
        own = o[5] != 0xFFFFFFFF
        words[own] = o[5][own]
        hits += own
    assert (hits == 1).all()
    np.testing.assert_array_equal(words & 3, val)
    np.testing.assert_array_equal(words >> 2, rem)
