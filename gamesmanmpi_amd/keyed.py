"""md5-sharded solves of keyed games (keyed).

Games whose every move advances one level (tic-tac-toe, toot-and-otto,
othello) run as md5-sharded BUCKETED levels inside the library
(gm_bucketed_shard.h: the level loop, both all-to-alls and the size reads
are native; group_keyed_solve / dist_keyed_solve pick it).  Every other
keyed game runs on HASHED shards driven by the loop below.

The reference partitions positions over MPI ranks by
owner(pos) = md5(str(pos)) % world (GameState.get_hash,
src/game_state.py:22-30) and sends one pickled LOOK_UP / RESOLVE message per
tree edge (src/process.py:146-185).  Here the partition rule is the same,
but each level moves its traffic in two bulk all-to-all(v) exchanges:

  forward  (L = 0 .. T-2)  own level-L positions -> children + owners
                           (gm_ks_expand), deduplicated, bucketed by owner,
                           all-to-all, inserted by their owners (gm_ks_insert)
  backward (L = T-1 .. 0)  own level-L positions -> children in gen_moves
                           order (gm_ks_counts / gm_ks_children), distinct
                           children queried at their owners
                           (gm_solver_query), words sent back, expanded to
                           one per edge, reduced (gm_ks_reduce)

`keyed_solve` is written once over the shards LOCAL to this process and an
exchange object:
  TorchExchange  one shard per process (torch.distributed.run); all_to_all
                 _single over RCCL on GPUs (gloo in the CPU tests)
  GroupExchange  every shard of a job in one process: the exchange is a
                 transpose of the send lists (runs the md5 job on one GPU)
A shard is `GpuShard` (libgamesman_hip.so, this module); the CPU tests drive
the same loop with a host shard built on the descriptor's host functions.
"""
import contextlib
import ctypes
import time

from . import _lib
from .games import GameSpec
from .solver import SolveResult, Solver


# ---------------------------------------------------------------------------
# exchanges
# ---------------------------------------------------------------------------
# An exchange moves, for every local shard, one flat tensor whose first
# counts[0] entries go to rank 0, the next counts[1] to rank 1, ... .  The
# per-destination counts stay on the device until the exchange reads them:
# ONE host read per exchange (send and receive sizes together); a reply that
# retraces a previous exchange reuses its sizes and reads nothing.
class GroupExchange:
    """All shards in this process: recv[dst][src] = send[src][dst]."""

    def all_to_all(self, flats, counts_dev):
        """-> (per shard: list of received tensors by source, sizes) where
        sizes[g] = (sent per destination, received per source)"""
        import torch
        n = len(flats)
        c = torch.stack(counts_dev).cpu().tolist()  # the one host read
        parts = [list(torch.split(f, c[g])) for g, f in enumerate(flats)]
        recv = [[parts[src][dst] for src in range(n)] for dst in range(n)]
        sizes = [(c[g], [c[src][g] for src in range(n)]) for g in range(n)]
        return recv, sizes

    def reply(self, flats, sizes):
        """Send back along a previous exchange: flats[g] holds, by source,
        the answers to what shard g received (sizes[g][1]); returns per
        shard the answers by destination of its original send."""
        import torch
        n = len(flats)
        parts = [list(torch.split(f, sizes[g][1])) for g, f in enumerate(flats)]
        return [[parts[dst][src] for dst in range(n)] for src in range(n)]

    def allreduce_sum(self, values):
        return [sum(col) for col in zip(*values)]


class TorchExchange:
    """One shard per process over the initialised torch.distributed default
    group.  Tensors live on `device` (cuda for RCCL, cpu for gloo);
    `stage` = a device to run the collectives on instead (e.g. cpu with gloo
    when several ranks share one GPU in tests -- RCCL needs one GPU per
    rank)."""

    def __init__(self, device, stage=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.device = torch, dist, device
        self.stage = torch.device(stage) if stage is not None else device

    def all_to_all(self, flats, counts_dev):
        torch, dist = self.torch, self.dist
        (flat,), (cnt,) = flats, counts_dev
        cnt = cnt.to(torch.int64).to(self.stage)
        got = torch.empty_like(cnt)
        dist.all_to_all_single(got, cnt)
        both = torch.cat([cnt, got]).tolist()  # the one host read
        w = len(both) // 2
        in_sizes, out_sizes = both[:w], both[w:]
        out = self._move(flat, in_sizes, out_sizes)
        return [list(torch.split(out, out_sizes))], [(in_sizes, out_sizes)]

    def reply(self, flats, sizes):
        torch = self.torch
        (flat,), ((sent, received),) = flats, sizes
        out = self._move(flat, received, sent)  # back along the same pairs
        return [list(torch.split(out, sent))]

    def _move(self, flat, in_sizes, out_sizes):
        torch, dist = self.torch, self.dist
        inp = flat.to(self.stage)
        out = torch.empty(sum(out_sizes), dtype=inp.dtype, device=self.stage)
        dist.all_to_all_single(out, inp, out_sizes, in_sizes)
        return out.to(self.device)

    def allreduce_sum(self, values):
        (v,) = values
        t = self.torch.tensor(v, dtype=self.torch.int64, device=self.stage)
        self.dist.all_reduce(t)
        return [int(x) for x in t.tolist()]


# ---------------------------------------------------------------------------
# the GPU shard
# ---------------------------------------------------------------------------
class GpuShard:
    """Rank `rank`'s keyed table on a GPU: a HASHED Solver driven step by
    step through gm_ks_*.  `positions`: bound on this shard's positions
    (default: 2x its md5 share of the game's bound)."""

    def __init__(self, spec, rank, world, device=None, positions=0,
                 stream=None):
        import torch
        self.torch = torch
        self.spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
        self.rank, self.world = int(rank), int(world)
        if not positions:
            positions = 2 * self.spec.positions_bound // self.world + 4096
        dev = torch.device(device if device is not None else "cuda")
        self.stream = stream or torch.cuda.Stream(device=dev)
        self.solver = Solver(self.spec, positions=positions, device=dev,
                             layout="hashed", rank=self.rank,
                             world=self.world, stream=self.stream)
        self.device = self.solver.device
        self.h = self.solver.handle
        self.L = _lib.load()
        self.fanout = float(_lib.GM_MAXCHILD)  # children per position seen

    def context(self):
        torch = self.torch
        stack = contextlib.ExitStack()
        stack.enter_context(torch.cuda.device(self.device))
        stack.enter_context(torch.cuda.stream(self.stream))
        return stack

    def begin(self, root_owned):
        _lib.check(self.L.gm_ks_begin(self.h, 1 if root_owned else 0))

    def level_size(self, level):
        n = ctypes.c_uint64()
        _lib.check(self.L.gm_ks_level_size(self.h, level, ctypes.byref(n)))
        return n.value

    def expand(self, level):
        """(child keys int64, owners int32) of the own level-L positions, in
        no particular order (duplicates included)."""
        torch = self.torch
        width = self.level_size(level)
        cap = int(width * min(self.fanout * 1.25 + 1, _lib.GM_MAXCHILD)) + 64
        n = ctypes.c_uint64()
        while True:
            keys = torch.empty(cap, dtype=torch.int64, device=self.device)
            owners = torch.empty(cap, dtype=torch.int32, device=self.device)
            rc = self.L.gm_ks_expand(self.h, level, keys.data_ptr(),
                                     owners.data_ptr(), cap, self.world,
                                     ctypes.byref(n))
            if rc == _lib.GM_EFULL and n.value > cap:
                cap = n.value  # exact size now known: expand again
                continue
            _lib.check(rc)
            break
        if width:
            self.fanout = max(1.0, n.value / width)
        return keys[:n.value], owners[:n.value]

    def insert(self, level, keys):
        keys = keys.contiguous()
        if keys.numel():
            _lib.check(self.L.gm_ks_insert(self.h, level, keys.data_ptr(),
                                           keys.numel()))

    def finalize(self, level):
        _lib.check(self.L.gm_ks_finalize(self.h, level))

    def children(self, level):
        """(offsets int64[n+1], child keys, owners) of the own level-L
        positions, children of position i at [offsets[i], offsets[i+1])."""
        torch = self.torch
        n = self.level_size(level)
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=self.device)
        if n == 0:
            empty = torch.empty(0, dtype=torch.int64, device=self.device)
            return offsets, empty, empty.to(torch.int32)
        counts = torch.empty(n, dtype=torch.int64, device=self.device)
        _lib.check(self.L.gm_ks_counts(self.h, level, counts.data_ptr()))
        offsets[1:] = torch.cumsum(counts, 0)
        total = int(offsets[-1].item())
        keys = torch.empty(max(1, total), dtype=torch.int64,
                           device=self.device)
        owners = torch.empty(max(1, total), dtype=torch.int32,
                             device=self.device)
        if total:
            _lib.check(self.L.gm_ks_children(
                self.h, level, offsets.data_ptr(), keys.data_ptr(),
                owners.data_ptr(), self.world))
        return offsets, keys[:total], owners[:total]

    def lookup(self, keys):
        """Words of keys this shard owns (GM_NO_WORD if absent)."""
        torch = self.torch
        keys = keys.contiguous()
        words = torch.empty(keys.numel(), dtype=torch.int32,
                            device=self.device)
        if keys.numel():
            _lib.check(self.L.gm_solver_query(self.h, keys.data_ptr(),
                                              keys.numel(),
                                              words.data_ptr()))
        return words

    def reduce(self, level, offsets, words):
        if offsets.numel() <= 1:
            return
        words = words.contiguous()
        if words.numel() == 0:  # every position primitive: any valid address
            words = self.torch.zeros(1, dtype=self.torch.int32,
                                     device=self.device)
        _lib.check(self.L.gm_ks_reduce(self.h, level, offsets.data_ptr(),
                                       words.data_ptr()))

    def end(self):
        r = _lib.gm_result()
        _lib.check(self.L.gm_ks_end(self.h, ctypes.byref(r)))
        return r

    def dump(self):
        """(keys, value, remoteness) of the positions this shard owns."""
        return self.solver.dump()


# ---------------------------------------------------------------------------
# the level loop
# ---------------------------------------------------------------------------
def _bucket(torch, keys, owners, world):
    """keys grouped by owner, on the device: (keys[perm], perm, counts per
    owner as a device tensor)."""
    perm = torch.argsort(owners, stable=True)
    counts = torch.bincount(owners.long(), minlength=world)
    return keys[perm], perm, counts


def _distinct(torch, keys, owners):
    """distinct keys with their owners, and each original key's index among
    them (None when there are no keys)"""
    if not keys.numel():
        return keys, owners, None
    ukeys, inv = torch.unique(keys, return_inverse=True)
    own = torch.empty(ukeys.numel(), dtype=owners.dtype, device=owners.device)
    own[inv] = owners
    return ukeys, own, inv


def keyed_solve(shards, exchange):
    """Solve the job whose LOCAL shards are `shards` (every rank for a
    group, this rank's one shard under torch.distributed).  Returns the
    whole job's SolveResult (the same on every rank).  Per level and shard
    the host reads sizes three times: the expanded child count
    (gm_ks_expand), the distinct count (torch.unique) and the exchange
    sizes; the backward's replies retrace the query exchange and read none."""
    s0 = shards[0]
    torch, spec, world = s0.torch, s0.spec, s0.world
    T = spec.max_levels
    root_owner = int(spec.owners_host([spec.root_key], world)[0])
    widths = [[0] * T for _ in shards]
    ctx = [sh.context() for sh in shards]
    with contextlib.ExitStack() as stack:
        for c in ctx:
            stack.enter_context(c)
        t0 = time.perf_counter()
        for sh in shards:
            sh.begin(sh.rank == root_owner)
        for L in range(T - 1):
            flats, counts = [], []
            for sh in shards:
                keys, owners = sh.expand(L)
                keys, owners, _ = _distinct(torch, keys, owners)  # duplicates need not travel
                flat, _, cnt = _bucket(torch, keys, owners, world)
                flats.append(flat)
                counts.append(cnt)
            recv, _ = exchange.all_to_all(flats, counts)
            for sh, lists in zip(shards, recv):
                sh.insert(L, torch.cat(lists))
                sh.finalize(L)
        t1 = time.perf_counter()
        for L in range(T - 1, -1, -1):
            flats, counts, state = [], [], []
            for g, sh in enumerate(shards):
                offsets, keys, owners = sh.children(L)
                widths[g][L] = offsets.numel() - 1
                # one query per distinct child (a position reached from
                # several parents of this shard is asked for once)
                keys, owners, inv = _distinct(torch, keys, owners)
                flat, perm, cnt = _bucket(torch, keys, owners, world)
                flats.append(flat)
                counts.append(cnt)
                state.append((offsets, perm, keys.numel(), inv))
            recv, sizes = exchange.all_to_all(flats, counts)
            replies = [sh.lookup(torch.cat(lists)) for sh, lists in zip(shards, recv)]
            answers = exchange.reply(replies, sizes)
            for sh, lists, (offsets, perm, n, inv) in zip(shards, answers,
                                                          state):
                words = torch.empty(n, dtype=torch.int32, device=sh.device)
                words[perm] = torch.cat(lists)
                if inv is not None:
                    words = words[inv]  # back to one word per edge
                sh.reduce(L, offsets, words)
        t2 = time.perf_counter()
        res = [sh.end() for sh in shards]
    local = []
    for r, w in zip(res, widths):
        owned_root = (r.root_word + 1) if r.root_word != _lib.GM_NO_WORD else 0
        local.append([r.positions, r.edges, r.primitives, owned_root] + w)
    tot = exchange.allreduce_sum(local)
    t3 = time.perf_counter()
    if tot[3] == 0:
        raise _lib.GmError(_lib.GM_ECORRUPT, "root unresolved")
    word = tot[3] - 1
    per_level = tot[4:]
    return SolveResult(
        root_value=word & 3, root_remoteness=word >> 2, positions=tot[0],
        edges=tot[1], primitives=tot[2],
        levels=sum(1 for x in per_level if x),
        max_level_width=max(per_level), ms_total=(t3 - t0) * 1e3,
        ms_forward=(t1 - t0) * 1e3, ms_backward=(t2 - t1) * 1e3,
        extra={"layout": "hashed", "partition": "md5", "world": world,
               "root_owner": root_owner})


def bucketed_shards_apply(spec, world):
    """True when the md5-sharded BUCKETED levels serve this game (every move
    advances one level: tic-tac-toe, toot-and-otto, othello), i.e. the
    library plans a bucketed shard for it."""
    plan = _lib.gm_plan_t()
    return _lib.load().gm_plan_keyed_shard(
        spec.id, 0, int(world), _shard_bound(spec, world, 0), 0, 0,
        ctypes.byref(plan)) == 0


def _shard_bound(spec, world, positions):
    """positions bound of one md5 shard: its share of the job's bound plus
    3 % and 64 K.  md5 (src/game_state.py:22-30) is a uniform hash, so the
    largest of W shards of P positions exceeds P / W by a few sqrt(P / W)
    (tests/test_dist_cpu.py checks the bound against the owners of the
    golden tables' positions); the 64 K floor covers small games.  Round 3
    planned 2x the share, which put toot 6x4 on 4 shards of one GPU out of
    memory."""
    return int(int(positions or spec.positions_bound) * 1.03) // int(world) + 65536


def ranked_shards_apply(spec, world):
    """True when md5 shards of the RANKED index space serve this game
    (toot-and-otto boards: gm_ranked_shard.h)."""
    plan = _lib.gm_plan_t()
    return _lib.load().gm_plan_keyed_shard(
        spec.id, 0, int(world), 0, _lib.GM_F_RANKED_SHARD, 0, ctypes.byref(plan)) == 0


def _pick(spec, world, layout):
    if layout not in ("auto", "bucketed", "hashed", "ranked"):
        raise ValueError("layout: auto, ranked, bucketed or hashed")
    if layout == "hashed":
        return "hashed"
    if layout == "ranked":
        if not ranked_shards_apply(spec, world):
            raise ValueError("%r: md5-sharded RANKED tables are toot-and-otto boards only" % (spec,))
        return "ranked"
    if bucketed_shards_apply(spec, world):
        return "bucketed"
    if layout == "bucketed":
        raise ValueError("%r: md5-sharded bucketed levels need every move to "
                         "advance one level" % (spec,))
    return "hashed"


def group_keyed_solve(spec, world, device=None, layout="auto", flags=0, streams="one"):
    """Every md5 shard of a `world`-rank job in this process, on one GPU.
    layout "auto": md5-sharded BUCKETED levels where they apply (the
    library's all-to-all level loop, gm_bucketed_shard.h), else HASHED
    shards driven by keyed_solve.  streams "one": every shard on one stream;
    "own" (bucketed): each shard on a stream of its own, the all-to-alls as
    device copies between them -- the one-GPU rehearsal of the RCCL
    stream order.  Returns (SolveResult, shards): Solvers (bucketed) or
    GpuShards (hashed), both with dump()."""
    import torch
    from .dist import _group_streams
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    dev = torch.device(device if device is not None else "cuda")
    ss = _group_streams(dev, world, streams)
    stream = ss[0]
    pick = _pick(spec, world, layout)
    if pick in ("bucketed", "ranked"):
        per = _shard_bound(spec, world, 0)
        shards = [Solver(spec, positions=per, device=dev, layout=pick,
                         rank=g, world=world, stream=ss[g], flags=flags)
                  for g in range(world)]
        arr = (ctypes.c_void_p * world)(*[s.handle.value for s in shards])
        r = _lib.gm_result()
        torch.cuda.synchronize(dev)
        with torch.cuda.device(dev):
            _lib.check(_lib.load().gm_solve_group(arr, world, ctypes.byref(r)))
        res = shards[0]._result(r)
        res.extra.update({"partition": "md5", "world": world})
        return res, shards
    shards = [GpuShard(spec, g, world, device=dev, stream=stream)
              for g in range(world)]
    return keyed_solve(shards, GroupExchange()), shards


def dist_keyed_solve(spec, device=None, positions=0, stage=None,
                     layout="auto", flags=0):
    """This process's shard of an md5-sharded job over the initialised
    torch.distributed default group; `positions`: bound for the whole job
    (0: the game's own); stage="cpu": collectives through host memory
    (several ranks sharing one GPU in tests); flags: kernel-family flags of
    the BUCKETED shards (e.g. _lib.GM_F_BKS_LOCAL: every level in the
    local-dedup form).  Returns (SolveResult, shard)."""
    import torch.distributed as dist
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    world = dist.get_world_size()
    pick = _pick(spec, world, layout)
    if pick in ("bucketed", "ranked"):
        from .dist import ShardedSolver
        shard = ShardedSolver(spec, dist.get_rank(), world, device=device,
                              transport="host" if stage == "cpu" else "rccl",
                              layout=pick, flags=flags,
                              positions=_shard_bound(spec, world, positions))
        res = shard.solve()
        res.extra.update({"partition": "md5", "world": world})
        return res, shard
    per_shard = 2 * int(positions) // world + 4096 if positions else 0
    shard = GpuShard(spec, dist.get_rank(), world, device=device,
                     positions=per_shard)
    return keyed_solve([shard], TorchExchange(shard.device, stage)), shard
