"""GPU: md5-sharded keyed solves, every shard of a job in one process on one
MI355X -- BUCKETED shards (gm_bucketed_shard.h, gm_solve_group: the
all-to-alls as device copies) for games whose every move advances one
level, HASHED shards through the gm_ks_* ABI (GroupExchange) otherwise --
and two processes over torch.distributed.  Bit-exact against the
reference's golden tables; every position must sit on its md5 owner
(src/game_state.py:22-30).  BASELINE config 5 is othello 4x4 over 8
ranks."""
import numpy as np
import pytest

from conftest import CASES, collect_workers, load_table

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,world", [
    ("othello_4x4", 8), ("othello_4x4", 3), ("tic_tac_toe_np", 2),
    ("mttt", 5), ("toot_3x3", 4), ("toot_4x3", 8), ("four_to_one_64", 3),
    ("sum_fto_6_6_6_6", 7), ("four_to_one", 5),  # README.md:13: four_to_one over 5 ranks
])
def test_gpu_group_keyed_matches_golden(name, world, golden_summary):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    spec = GameSpec(*CASES[name])
    r, shards = group_keyed_solve(spec, world)
    # games whose every move advances one level run as md5-sharded BUCKETED
    # levels (gm_bucketed_shard.h), the others on HASHED shards
    assert r.extra["layout"] == ("hashed" if name.startswith(("four_to_one", "sum_")) else "bucketed")
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


def _check_golden_shards(name, r, shards, world, golden_summary):
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec(*CASES[name])
    info = golden_summary[name]
    assert (r.positions, r.edges, r.primitives, r.root_line) == (
        info["positions"], info["edges"], info["primitives"], info["root_line"])
    dumps = [s.dump() for s in shards]
    for rank, d in enumerate(dumps):
        if len(d[0]):
            assert (spec.owners_host(d[0], world) == rank).all()
    keys = np.concatenate([d[0] for d in dumps])
    val = np.concatenate([d[1] for d in dumps])
    rem = np.concatenate([d[2] for d in dumps])
    t = load_table(name)
    canon, clen = spec.decode_batch(keys, stride=t["canon"].shape[1])
    order = np.array(sorted(range(len(keys)), key=lambda i: bytes(canon[i, :clen[i]])), np.int64)
    np.testing.assert_array_equal(canon[order], t["canon"])
    np.testing.assert_array_equal(val[order], t["value"])
    np.testing.assert_array_equal(rem[order], t["remoteness"])


@pytest.mark.parametrize("name,world", [("othello_4x4", 8), ("toot_4x3", 3), ("tic_tac_toe_np", 2)])
def test_gpu_group_keyed_hashed_shards_still_golden(name, world, golden_summary):
    """The HASHED md5 shards (the path of games the bucketed levels do not
    serve) on games both layouts serve."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    r, shards = group_keyed_solve(GameSpec(*CASES[name]), world, layout="hashed")
    assert r.extra["layout"] == "hashed"
    _check_golden_shards(name, r, shards, world, golden_summary)


LOCAL = 16384  # _lib.GM_F_BKS_LOCAL


@pytest.mark.parametrize("name,world", [("othello_4x4", 8), ("toot_4x3", 3), ("tic_tac_toe_np", 2), ("mttt", 5),
                                        ("toot_3x3", 4)])
def test_gpu_group_keyed_local_dedup_matches_golden(name, world, golden_summary):
    """md5-sharded BUCKETED levels in the local-dedup form (GM_F_BKS_LOCAL:
    each rank dedups its own children first and hashes / sends each unique
    child once): every position on its md5 owner, words equal to the
    reference-generated tables."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    r, shards = group_keyed_solve(GameSpec(*CASES[name]), world, flags=LOCAL)
    assert r.extra["layout"] == "bucketed"
    _check_golden_shards(name, r, shards, world, golden_summary)


@pytest.mark.parametrize("flags", [0, LOCAL])
@pytest.mark.parametrize("world", [2, 4, 7])
def test_gpu_bucketed_shards_toot_5x4_checksum(world, flags):
    """toot 5x4 (70,184,763 positions) on 2 / 4 / 7 md5 BUCKETED shards: the
    shards' fingerprints (each over the positions it owns) add up to the CPU
    restatement's golden (oracle/oracle_mt.c; beyond 4x4 no reference
    fixture exists -- parity against the restatement, as on one GPU)."""
    import json
    import os
    import torch
    from conftest import GOLDEN
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    e = json.load(open(os.path.join(GOLDEN, "checksums.json")))["toot_5x4"]
    r, shards = group_keyed_solve(GameSpec(e["game"], e["params"]), world, flags=flags)
    assert r.extra["layout"] == "bucketed"
    assert (r.positions, r.edges, r.primitives, r.root_line) == (e["positions"], e["edges"], e["primitives"],
                                                                  e["root_line"])
    cks = [s.checksum() for s in shards]
    assert "%016x" % (sum(int(c["checksum"], 16) for c in cks) % (1 << 64)) == e["checksum"]
    assert sum(c["positions"] for c in cks) == e["positions"]
    assert (sum(c["win"] for c in cks), sum(c["loss"] for c in cks), sum(c["tie"] for c in cks)) == (
        e["win"], e["loss"], e["tie"])
    del shards
    torch.cuda.empty_cache()


def test_gpu_keyed_shard_refuses_whole_solve():
    """A keyed shard of a world > 1 job cannot be solved alone."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import GpuShard
    sh = GpuShard(GameSpec("tic_tac_toe_np", ""), 0, 2)
    with pytest.raises(_lib.GmError):
        sh.solver.solve()


def _dist_worker(rank, world, port, q, name, flags=0):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gamesmanmpi_amd.games import GameSpec
        from gamesmanmpi_amd.keyed import dist_keyed_solve
        spec = GameSpec(*CASES[name])
        r, shard = dist_keyed_solve(spec, device="cuda:0", stage="cpu", flags=flags)
        keys, val, rem = shard.dump()
        q.put((rank, (r.positions, r.edges, r.primitives, r.root_line),
               keys, val, rem))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,flags", [("othello_4x4", 0), ("toot_4x3", 0), ("toot_4x3", LOCAL)])
def test_gpu_keyed_two_processes_torch_exchange(name, flags, golden_summary):
    """The one-process-per-rank path (the code the launcher runs under
    torchrun): md5-sharded BUCKETED shards (ShardedSolver; the library's
    level loop with the host-staged transport over gloo here, RCCL send /
    recv on an 8-GPU node) with two ranks sharing one GPU.  othello 4x4 and toot 4x3 bit-exact against the reference-
    generated tables, positions on their md5 owners."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q, name, flags)) for r in range(2)]
    for p in procs:
        p.start()
    out = collect_workers(q, procs, 2, limit=150)
    info = golden_summary[name]
    for _, tot, _, _, _ in out:
        assert tot == (info["positions"], info["edges"], info["primitives"], info["root_line"])
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec(*CASES[name])
    keys = np.concatenate([o[2] for o in out])
    val = np.concatenate([o[3] for o in out])
    rem = np.concatenate([o[4] for o in out])
    for rank, o in enumerate(out):
        assert (spec.owners_host(o[2], 2) == rank).all()
    t = load_table(name)
    canon, clen = spec.decode_batch(keys, stride=t["canon"].shape[1])
    order = np.array(sorted(range(len(keys)), key=lambda i: bytes(canon[i, :clen[i]])), np.int64)
    np.testing.assert_array_equal(canon[order], t["canon"])
    np.testing.assert_array_equal(val[order], t["value"])
    np.testing.assert_array_equal(rem[order], t["remoteness"])


@pytest.mark.parametrize("layout", ["bucketed", "hashed", "auto"])
def test_gpu_kernel_timing_toggles_on_explicit_layouts(layout):
    """set_kernel_timing re-sends the flags the solver was CREATED with
    (layout bits included): per-kernel timing on a bucketed or hashed
    solver, same root and counts as without."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s = Solver(GameSpec("toot_and_otto_bitstring", "length=4,height=3"), layout=layout)
    r0 = s.solve()
    s.set_kernel_timing(True)
    r1 = s.solve()
    s.set_kernel_timing(False)
    assert (r0.positions, r0.edges, r0.root_line) == (r1.positions, r1.edges, r1.root_line)
    assert r1.n_resolve_launches > 0


@pytest.mark.parametrize("name,world,flags", [("othello_4x4", 8, 0), ("othello_4x4", 8, LOCAL), ("toot_4x3", 3, 0),
                                              ("toot_4x3", 5, LOCAL)])
def test_gpu_group_keyed_rccl_stream_rehearsal(name, world, flags, golden_summary):
    """The md5 all-to-alls' RCCL stream order rehearsed on one GPU
    (gm_bucketed_shard.h mode 4): every shard on a stream of its own, its
    kernels and copies there as one rank's would be, each all-to-all as
    device copies on the receivers' streams behind every sender's ready
    event, then every stream behind every receiver's -- BASELINE config 5
    (othello 4x4 on 8 md5 shards) against the reference-generated table."""
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    r, shards = group_keyed_solve(GameSpec(*CASES[name]), world, flags=flags, streams="own")
    assert r.extra["layout"] == "bucketed"
    _check_golden_shards(name, r, shards, world, golden_summary)
