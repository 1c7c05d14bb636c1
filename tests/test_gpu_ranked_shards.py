"""md5 shards of the RANKED layout (gamesmanmpi_amd/csrc/gm_ranked_shard.h):
toot-and-otto on several GPUs with every position resolved by its md5 owner
(src/game_state.py:22-30), each level's words exchanged after it.  Rehearsed
on one GPU as in-process groups -- every shard on a stream of its own with
device copies for the transfers (the RCCL schedule's order), or all on one
stream -- and over the host transport in two processes (gloo).

Checked: counts, root and every word of every shard's table against the
one-GPU RANKED solve (itself pinned to the reference-generated tables up to
4x4, tests/test_gpu_parity.py), the oracle_mt fingerprint (5x4);
and ownership -- each shard resolved exactly the positions whose md5 owner
(gm_owner, bit-exact with get_hash: test_gpu_md5_owner_kernel) it is."""
import os
import socket

import numpy as np
import pytest

from conftest import collect_workers

pytestmark = pytest.mark.gpu


def _one_gpu(params):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("toot_and_otto_bitstring", params), layout="ranked")
    return s, s.solve()


def _owners(spec, keys, world):
    import torch
    from gamesmanmpi_amd import _lib
    kd = torch.from_numpy(keys.astype(np.uint64).view(np.int64)).cuda()
    od = torch.empty(len(keys), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().gm_owner(spec.id, kd.data_ptr(), len(keys), world, od.data_ptr(), None))
    return od.cpu().numpy()


@pytest.mark.parametrize("params,world,streams", [
    ("length=4,height=3", 2, "own"), ("length=4,height=3", 3, "own"), ("length=4,height=3", 4, "one"),
    ("length=3,height=4", 8, "own"), ("length=4,height=4", 5, "own"), ("length=4,height=4", 2, "one"),
])
def test_ranked_shards_match_one_gpu_and_owners(params, world, streams):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    spec = GameSpec("toot_and_otto_bitstring", params)
    s1, r1 = _one_gpu(params)
    r, shards = group_keyed_solve(spec, world, layout="ranked", streams=streams)
    assert r.extra["layout"] == "ranked" and r.extra["partition"] == "md5"
    assert (r.positions, r.edges, r.primitives, r.root_line) == (r1.positions, r1.edges, r1.primitives, r1.root_line)
    keys = s1.positions()
    want = s1.query(keys)
    for sh in shards:  # every shard ends with the whole table
        np.testing.assert_array_equal(sh.query(keys), want)
    own = _owners(spec, keys, world)
    tot = 0
    for g, sh in enumerate(shards):
        resolved, owned = sh.shard_stats()
        assert owned == int((own == g).sum()), (g, owned)
        assert resolved == owned, (g, resolved, owned)
        tot += owned
    assert tot == r1.positions


def test_ranked_shards_5x4_fingerprint():
    """toot 5x4 (BASELINE's board family, 3.8e7 positions) on four md5
    shards: the whole-table fingerprint on every shard equals the oracle_mt
    golden (parity unpinned by reference fixtures beyond 4x4, as on one GPU)."""
    import json
    from conftest import GOLDEN
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    with open(os.path.join(GOLDEN, "checksums.json")) as fh:
        e = json.load(fh)["toot_5x4"]
    r, shards = group_keyed_solve(GameSpec(e["game"], e["params"]), 4, layout="ranked", streams="own")
    assert (r.positions, r.edges, r.primitives, r.root_line) == (e["positions"], e["edges"], e["primitives"],
                                                                  e["root_line"])
    for sh in (shards[0], shards[3]):
        assert sh.checksum()["checksum"] == e["checksum"]
    assert sum(sh.shard_stats()[1] for sh in shards) == e["positions"]
    assert all(sh.shard_stats()[0] == sh.shard_stats()[1] for sh in shards)


def _worker(rank, world, port, q, params):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gamesmanmpi_amd.games import GameSpec
        from gamesmanmpi_amd.keyed import dist_keyed_solve
        r, sh = dist_keyed_solve(GameSpec("toot_and_otto_bitstring", params), device="cuda:0", stage="cpu",
                                 layout="ranked")
        q.put((rank, (r.positions, r.edges, r.primitives, r.root_line), sh.shard_stats(), sh.checksum()["checksum"]))
    finally:
        dist.destroy_process_group()


def test_ranked_shards_host_transport_two_processes():
    """Two processes on one GPU (gloo, the host-staged transport: mode 3 of
    run_ranked_shards, pairwise rounds): both ranks end with the one-GPU
    counts, root and fingerprint, each resolving its own md5 share."""
    import torch.multiprocessing as mp
    params, world = "length=4,height=3", 2
    s1, r1 = _one_gpu(params)
    ck = s1.checksum()["checksum"]
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(g, world, port, q, params)) for g in range(world)]
    for p in procs:
        p.start()
    out = collect_workers(q, procs, world)
    tot = 0
    for rank, counts, (resolved, owned), c in out:
        assert counts == (r1.positions, r1.edges, r1.primitives, r1.root_line)
        assert resolved == owned
        assert c == ck
        tot += owned
    assert tot == r1.positions


def test_ranked_shards_toot_6x4_eight_shards():
    """BASELINE config 3 at its own size on the reference's production
    partition (run_savio.sh: md5 ranks; src/game_state.py:22-30): toot 6x4 on
    eight md5 shards as an in-process group (all on one stream).  Every
    shard's fingerprint equals the oracle_mt golden, the shards own and
    resolve exactly their md5 shares, and the 220 reference-solved deep
    positions (tests/golden/deep/toot_6x4.json) read their exact value and
    remoteness on the shards."""
    import json
    from conftest import GOLDEN
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    with open(os.path.join(GOLDEN, "checksums.json")) as fh:
        e = json.load(fh)["toot_6x4"]
    spec = GameSpec(e["game"], e["params"])
    r, shards = group_keyed_solve(spec, 8, layout="ranked", streams="one")
    assert r.extra["layout"] == "ranked" and r.extra["partition"] == "md5"
    assert (r.positions, r.edges, r.primitives, r.root_line) == (e["positions"], e["edges"], e["primitives"],
                                                                  e["root_line"])
    for sh in (shards[0], shards[5]):
        assert sh.checksum()["checksum"] == e["checksum"]
    stats = [sh.shard_stats() for sh in shards]
    assert all(res == own for res, own in stats)
    assert sum(own for _, own in stats) == e["positions"]
    with open(os.path.join(GOLDEN, "deep", "toot_6x4.json")) as fh:
        deep = json.load(fh)["rows"]
    keys = np.array([spec.encode(bytes.fromhex(row["pos"])) for row in deep], np.uint64)
    own = _owners(spec, keys, 8)
    for g in (0, 3, 7):
        w = shards[g].query(keys)
        for i, row in enumerate(deep):
            assert (int(w[i]) & 3, int(w[i]) >> 2) == (row["value"], row["remoteness"]), (g, row)
    # the deep positions spread over the shards' md5 shares
    assert len(set(own.tolist())) == 8
    del shards
