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


@pytest.mark.parametrize("case,params", [("toot_4x3", "length=4,height=3"),
                                         ("othello_4x4", "length=4,height=4")])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_md5_shard_bound_holds_every_shard(case, params, world):
    """keyed._shard_bound (the positions one md5 shard is planned for) covers
    the largest shard of the golden table's positions, per level too, and
    gm_plan_keyed_shard scales the shard's edge bound with its share (round
    3 planned every shard for the whole board's edges)."""
    import ctypes
    import numpy as np
    from conftest import load_table
    from gamesmanmpi_amd import _lib, keyed
    from gamesmanmpi_amd.games import GameSpec
    name = "toot_and_otto_bitstring" if case.startswith("toot") else "othello_bit_new"
    spec = GameSpec(name, params)
    t = load_table(case)
    keys = spec.encode_batch(t["canon"], t["clen"])
    own = spec.owners_host(keys, world)
    sizes = np.bincount(own, minlength=world)
    bound = keyed._shard_bound(spec, world, len(keys))
    assert sizes.max() <= bound and sizes.sum() == len(keys)
    # the uniform-hash spread the 3 % slack is for: a few sqrt of the share
    share = len(keys) / world
    assert sizes.max() - share < 6 * share ** 0.5 + 16
    for lv in np.unique(t["level"]):
        m = t["level"] == lv
        per = np.bincount(own[m], minlength=world)
        assert per.max() - m.sum() / world < 6 * (m.sum() / world) ** 0.5 + 16
    # edges: a shard of half the positions is planned for about half the edges
    full, half = _lib.gm_plan_t(), _lib.gm_plan_t()
    P = len(keys)
    _lib.check(_lib.load().gm_plan_keyed_shard(spec.id, 0, world, P, 0, 0, ctypes.byref(full)))
    _lib.check(_lib.load().gm_plan_keyed_shard(spec.id, 0, world, P // 2, 0, 0, ctypes.byref(half)))
    assert half.table_slots < 0.6 * full.table_slots + 2048


@pytest.mark.parametrize("n", [2, 4, 8])
def test_plan_multi_sum_bench_shapes(n):
    """gm_plan_multi for the bench's N-GPU workloads (31^5 x (32N - 1)):
    N PLANES shards of the staged deal, about equal in size, each about the 2^30
    one-table plan (the sizes gm_solve(.., ngpus = N, ..) allocates)."""
    from gamesmanmpi_amd import _lib, dist as gdist
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec("sum_four_to_one", "heaps=" + ":".join(["31"] * 5 + [str(32 * n - 1)]))
    plans = gdist.plan_multi(spec, n)
    assert len(plans) == n
    assert {int(p.mode) for p in plans} == {_lib.GM_MODE_PLANES}
    sizes = [int(p.table_bytes) for p in plans]  # the end ranks carry one halo fewer
    assert max(sizes) <= 1.1 * min(sizes)
    one = gdist.plan_multi(GameSpec("sum_four_to_one", "heaps=" + ":".join(["31"] * 6)), 1)[0]
    assert int(one.mode) == _lib.GM_MODE_PLANES
    # a shard holds 2^30 positions (1 GiB of 8- or 16-bit words + bits + halo rows)
    assert one.table_bytes <= plans[0].table_bytes <= 2.5 * one.table_bytes


@pytest.mark.parametrize("n", [2, 4, 8])
def test_plan_multi_keyed_shards_fit_together(n):
    """toot 6x4 (BASELINE config 3's board) on n md5 shards: every shard's
    plan is about 1/n of the job, so the n shards together stay near the
    one-table plan (round 3: each shard planned for the whole board's
    edges, 4 shards > 288 GB)."""
    from gamesmanmpi_amd import _lib, dist as gdist
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec("toot_and_otto_bitstring", "length=6,height=4")
    plans = gdist.plan_multi(spec, n)
    one = gdist.plan_multi(spec, 1, flags=_lib.GM_F_FORCE_HASHED)[0]  # the one-table keyed plan
    assert int(one.mode) == _lib.GM_MODE_BUCKETED
    assert int(gdist.plan_multi(spec, 1)[0].mode) == _lib.GM_MODE_RANKED  # one GPU: computed indices
    assert {int(p.mode) for p in plans} == {_lib.GM_MODE_BUCKETED}
    total = sum(int(p.table_bytes) + 8 * int(p.level_capacity) for p in plans)
    single = int(one.table_bytes) + 8 * int(one.level_capacity)
    assert total < 2.3 * single, (total / 2 ** 30, single / 2 ** 30)
    assert total < 250 * 2 ** 30  # n shards fit one MI355X as an in-process group


def test_gm_solve_more_gpus_than_visible_is_an_error():
    """gm_solve(.., ngpus, ..) with more GPUs than the process sees fails
    with GM_EINVAL before touching any buffer (this box sees none)."""
    import ctypes
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec("sum_four_to_one", "heaps=31:31:31:63")
    bufs = (_lib.gm_buffers * 2)()
    r = _lib.gm_result()
    L = _lib.load()
    rc = L.gm_solve(spec.id, spec.root_key, 2, bufs, ctypes.byref(r))
    assert rc == _lib.GM_EINVAL
    assert b"visible" in L.gm_last_error()
    assert L.gm_solve(spec.id, spec.root_key, 0, bufs, ctypes.byref(r)) == _lib.GM_EINVAL
