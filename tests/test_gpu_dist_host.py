"""Sharded sum-game solves, one process per rank, over the host-staged
transport (gamesmanmpi_amd.dist.HostTransport over torch.distributed gloo):
the RCCL path's geometry, halo plan check and reductions with the transfers
carried through host memory, so two or three ranks can share one GPU.

Checked against the CPU oracle (oracle/oracle_mt.c's row solver, pinned to
the DFS oracle and the reference-generated tables by tests/test_oracle.py):
every position answered by exactly one rank, with the oracle's value and
remoteness; counts and root line equal on every rank.  Both sharded
layouts: PLANES (heaps 0 and 1 of 32 values -- the bench's layout; the
staged pipeline with its row-by-row transfers, and the level-synchronous
deal) and the level-major DENSE table."""
import os
import socket

import numpy as np
import pytest

from conftest import collect_workers

pytestmark = pytest.mark.gpu

LEVEL_SYNC = 4096  # _lib.GM_F_PLANE_LEVEL_SYNC (kept literal: the parent never loads the library)
CASES = {  # (layout, world, deal) -> (params, flags)
    ("planes", 2, "staged"): ("heaps=31:31:3:15", 0),
    ("planes", 3, "staged"): ("heaps=31:31:3:23", 0),
    ("planes", 4, "staged"): ("heaps=31:31:2:7:15", 0),
    ("planes", 2, "rows"): ("heaps=31:63:3:15", 0),     # the row deal (heap 1 split in 32-row slabs)
    ("planes", 3, "rows"): ("heaps=31:95:3:7", 0),
    ("planes", 2, "level-sync"): ("heaps=31:31:3:15", LEVEL_SYNC),
    ("planes", 3, "level-sync"): ("heaps=31:31:3:23", LEVEL_SYNC),
    ("dense", 2, ""): ("heaps=15:15:15:15:31", 0),
    ("dense", 3, ""): ("heaps=15:15:15:15:31", 0),
}


def _worker(rank, world, port, q, params, layout, flags):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gamesmanmpi_amd.dist import ShardedSolver
        from gamesmanmpi_amd.games import GameSpec
        spec = GameSpec("sum_four_to_one", params)
        s = ShardedSolver(spec, rank, world, device="cuda:0", transport="host", layout=layout, flags=flags)
        r = s.solve()
        n = 1
        for h in params.split("=")[1].split(":"):
            n *= int(h) + 1
        w = s.query(np.arange(n, dtype=np.uint64))
        q.put((rank, r.extra["layout"], (r.positions, r.edges, r.primitives, r.root_line), w))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("layout,world,deal", sorted(CASES))
def test_host_transport_matches_oracle(layout, world, deal):
    import torch.multiprocessing as mp
    from oracle.oracle import Game  # checker only
    params, flags = CASES[(layout, world, deal)]
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, params, layout, flags)) for r in range(world)]
    for p in procs:
        p.start()
    out = collect_workers(q, procs, world)
    sol = Game("sum_four_to_one", params).solve_rows()
    sol.refresh(True)
    for o in out:
        assert o[1] == layout
        assert o[2] == (sol.count, sol.edges, sol.stats["primitives"], sol.root_line)
    want = np.array([sol.word(k) for k in range(sol.count)], np.uint32)
    got = np.full(sol.count, 0xFFFFFFFF, np.uint32)
    hits = np.zeros(sol.count, np.int64)
    for o in out:
        own = o[3] != 0xFFFFFFFF
        got[own] = o[3][own]
        hits += own
    assert (hits == 1).all()
    np.testing.assert_array_equal(got, want)
