"""Multi-process side of the sharded solve, on CPU with gloo (world size 2
and 4): the RCCL-id bootstrap broadcast, and every rank's shard geometry
(host-only ABI) fitting its neighbours' -- blocks tile the top heap, each
rank's halo slices are exactly the slices its neighbour sends."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, params, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gamesmanmpi_amd.games import GameSpec
        spec = GameSpec("sum_four_to_one", params)
        # bootstrap exactly as dist.ShardedSolver._comm_init does it
        fake_id = bytes(range(128)) if rank == 0 else None
        obj = [fake_id]
        dist.broadcast_object_list(obj, src=0)
        info = spec.shard_info(rank, world)
        gathered = [None] * world
        dist.all_gather_object(gathered, info)
        q.put((rank, obj[0], gathered))
    finally:
        dist.destroy_process_group()


def _run(world, params):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, params, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out)


@pytest.mark.parametrize("world,params", [
    (2, "heaps=31:31:31:31:31:63"),   # bench N=2 workload
    (4, "heaps=31:31:31:31:31:127"),  # bench N=4 workload
    (8, "heaps=31:31:31:31:31:255"),  # bench N=8 workload
    (2, "heaps=7:7:7:15"),
    (3, "heaps=7:7:7:15"),
])
def test_gloo_bootstrap_and_geometry(world, params):
    out = _run(world, params)
    for rank, uid, infos in out:
        assert uid == bytes(range(128))
        assert infos == out[0][2]  # every rank sees the same geometry
    infos = out[0][2]
    B, nblocks, Z, E = (infos[0][k] for k in ("B", "nblocks", "Z", "E"))
    assert Z % 64 == 0 and B >= 2
    assert nblocks == -(-E // B) and nblocks >= world
    for r, i in enumerate(infos):
        assert (i["B"], i["nblocks"], i["Z"], i["E"], i["rank"], i["world"]) == (B, nblocks, Z, E, r, world)
        # round robin: rank r owns blocks r, r + world, ...
        assert i["nb"] == len(range(r, nblocks, world))
        assert i["Wl"] == i["nb"] * (B + 4) * Z  # two halo slices each side
    assert sum(i["nb"] for i in infos) == nblocks
    if "31:31:31:31:31:" in params:
        # bench shape: 2^30 positions per GPU, blocks of 8, four per rank
        assert (B, nblocks, Z) == (8, 4 * world, 32 ** 4)
        assert all(i["nb"] == 4 for i in infos)
