"""Multi-GPU drivers for PLANES and DENSE solves.

The reference spreads a solve over MPI ranks by md5 ownership and one
pickled message per tree edge (src/game_state.py:22-30,
src/process.py:146-185).  Here a rank owns a block of the top heap's values
and the library exchanges two boundary slices per level over RCCL, inside
one enqueued solve (no host round trip per level).

  ShardedSolver   one process per GPU (torch.distributed.run); RCCL id
                  bootstrapped with torch.distributed, or -- transport="host"
                  -- halos staged through host memory and carried by the
                  default torch.distributed group (gloo on a CPU box or when
                  ranks share a GPU), the same geometry and reductions
  group_solve     every shard of a job in ONE process on one GPU, halos by
                  device-to-device copies -- the same kernels and halo
                  geometry, for parity tests on a single device
"""
import ctypes
import types

from . import _lib
from .games import GameSpec
from .solver import Solver


class ShardedSolver(Solver):
    """Shard `rank` of `world` of a dense solve; needs an initialised
    torch.distributed default group (any backend) for the bootstrap."""

    def __init__(self, spec, rank, world, device=None, transport="rccl", layout="auto", **kw):
        super().__init__(spec, device=device, rank=rank, world=world,
                         layout=layout, **kw)
        self._xfer = None
        if world > 1:
            if transport == "host":
                self._xfer = HostTransport()
                _lib.check(_lib.load().gm_solver_set_transport(self._h, self._xfer.fn, None))
            elif transport == "rccl":
                self._comm_init()
            else:
                raise ValueError("transport: 'rccl' or 'host'")

    def _comm_init(self):
        import torch.distributed as dist
        L = _lib.load()
        uid = ctypes.create_string_buffer(_lib.GM_COMM_ID_BYTES)
        if self.rank == 0:
            _lib.check(L.gm_comm_unique_id(uid))
        obj = [uid.raw if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        raw = obj[0]
        buf = ctypes.create_string_buffer(raw, len(raw))
        with self.torch.cuda.device(self.device):
            _lib.check(L.gm_solver_comm_init(self._h, buf))


class HostTransport:
    """gm_xfer_fn over the default torch.distributed group: the library hands
    halo bytes in host memory; paired send / receive with isend + irecv,
    all-gathers with all_gather.  Errors become a non-zero return (the solve
    fails with GM_EHIP instead of hanging)."""

    def __init__(self):
        self.fn = _lib.XFER_FN(self._call)

    @staticmethod
    def _view(ptr, n):
        import numpy as np
        import torch
        if not n:
            return torch.empty(0, dtype=torch.uint8)
        arr = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))
        return torch.from_numpy(arr)

    def _call(self, ctx, op, sbuf, sbytes, speer, rbuf, rbytes, rpeer):
        import torch.distributed as dist
        try:
            send, recv = self._view(sbuf, sbytes), self._view(rbuf, rbytes)
            if op == _lib.GM_XFER_SENDRECV:
                reqs = []
                if sbytes:
                    reqs.append(dist.isend(send, speer))
                if rbytes:
                    reqs.append(dist.irecv(recv, rpeer))
                for r in reqs:
                    r.wait()
            elif op == _lib.GM_XFER_ALLGATHER:
                world = dist.get_world_size()
                parts = list(recv.view(world, sbytes).unbind(0))
                dist.all_gather(parts, send.clone())
            else:
                return 1
            return 0
        except Exception:  # noqa: BLE001 -- reported to the library as a failed transfer
            import traceback
            traceback.print_exc()
            return 1


def halo_sigs(spec, rank, world, flags=0):
    """The per-level halo fingerprints shard `rank` of `world` checks against
    its neighbours before level 0 (host only): uint64 [levels, 4] = bits
    sent down, bits received from above, words sent up, words received."""
    import numpy as np
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    T = int(spec.max_levels)
    out = np.zeros((T, 4), np.uint64)
    _lib.check(_lib.load().gm_shard_halo_sigs(spec.id, rank, world, flags, out.ctypes.data, T))
    return out


def plane_halo_plan(spec, rank, world, flags=0):
    """PLANES shards: shard `rank`'s halo plan (host only): uint64
    [levels, world, 2] = boundary planes sent to / received from each peer
    after each plane level (rows past the last plane level are 0)."""
    import numpy as np
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    T = int(spec.max_levels)
    out = np.zeros((T, world, 2), np.uint64)
    _lib.check(_lib.load().gm_plane_halo_plan(spec.id, rank, world, flags, out.ctypes.data, T))
    return out


def group_solve(spec, world, device=None, kernel_timing=False, flags=0, layout="auto", streams="one"):
    """Solve all `world` shards in this process (one GPU).  streams="one":
    every shard on one stream, halos copied in order (the parity path);
    "own": every shard on a stream of its own -- the one-GPU rehearsal of
    the RCCL staged schedule (send / receive streams, receive window,
    events and joins of gm_plane_run.h's mode 1, device copies for the
    transfers).  Returns (SolveResult of the whole job, [shard Solvers])."""
    import torch
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    dev = torch.device(device if device is not None else "cuda")
    # explicit streams (torch's default stream has handle 0, which the ABI
    # reads as "library-owned stream per solver")
    ss = _group_streams(dev, world, streams)
    shards = [Solver(spec, device=dev, rank=g, world=world, layout=layout,
                     kernel_timing=kernel_timing, stream=ss[g], flags=flags)
              for g in range(world)]
    arr = (ctypes.c_void_p * world)(*[s.handle.value for s in shards])
    r = _lib.gm_result()
    torch.cuda.synchronize(dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().gm_solve_group(arr, world, ctypes.byref(r)))
    return shards[0]._result(r), shards


def _group_streams(dev, world, streams):
    import torch
    if streams == "one":
        return [torch.cuda.Stream(device=dev)] * int(world)
    if streams == "own":
        return [torch.cuda.Stream(device=dev) for _ in range(int(world))]
    raise ValueError("streams: 'one' or 'own'")


def plan_multi(spec, ngpus, positions=0, flags=0, max_table_bytes=0):
    """The ngpus shard plans gm_solve(.., ngpus, ..) runs (host only): a
    list of gm_plan_t, shard i for device i."""
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    plans = (_lib.gm_plan_t * int(ngpus))()
    _lib.check(_lib.load().gm_plan_multi(spec.id, int(ngpus), int(positions), int(flags),
                                         int(max_table_bytes), plans))
    return list(plans)


def solve_one_process(spec, ngpus, positions=0, flags=0):
    """SURVEY §8b's gm_solve(game, root, ngpus, ..) from ONE process: shard
    i on cuda:i (buffers from torch), one RCCL communicator per device and
    one host thread per device inside the library.  The reference runs the
    same job as `mpiexec -n P` (solver_launcher.py:30,76-84).  Returns the
    whole job's SolveResult; the shards' buffers are kept alive until the
    next solve of the game (gm_release)."""
    import torch
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    plans = plan_multi(spec, ngpus, positions, flags)
    L = _lib.load()
    bufs = (_lib.gm_buffers * int(ngpus))()
    keep = []
    for i, plan in enumerate(plans):
        dev = torch.device("cuda", i)
        with torch.cuda.device(dev):
            table = torch.empty(plan.table_bytes, dtype=torch.uint8, device=dev)
            levels = torch.empty(max(1, plan.level_capacity), dtype=torch.int64, device=dev)
            scratch = torch.empty(plan.scratch_bytes, dtype=torch.uint8, device=dev)
        keep.append((table, levels, scratch))
        b = bufs[i]
        b.table, b.table_slots, b.table_bytes = table.data_ptr(), plan.table_slots, plan.table_bytes
        b.levels, b.level_capacity = levels.data_ptr(), plan.level_capacity
        b.scratch, b.scratch_bytes = scratch.data_ptr(), plan.scratch_bytes
        b.stream, b.flags, b.mode = 0, int(flags), plan.mode
    for i in range(int(ngpus)):
        torch.cuda.synchronize(i)
    r = _lib.gm_result()
    _lib.check(L.gm_solve(spec.id, spec.root_key, int(ngpus), bufs, ctypes.byref(r)))
    _KEEP[spec.id] = keep
    res = Solver._result(types.SimpleNamespace(spec=spec, plan=plans[0]), r)
    res.extra.update({"gpus": int(ngpus), "process": "one"})
    return res


_KEEP = {}  # game id -> the torch buffers of its last one-process multi-GPU solve
