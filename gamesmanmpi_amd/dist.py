"""Multi-GPU drivers for DENSE solves.

The reference spreads a solve over MPI ranks by md5 ownership and one
pickled message per tree edge (src/game_state.py:22-30,
src/process.py:146-185).  Here a rank owns a block of the top heap's values
and the library exchanges two boundary slices per level over RCCL, inside
one enqueued solve (no host round trip per level).

  ShardedSolver   one process per GPU (torch.distributed.run); RCCL id
                  bootstrapped with torch.distributed
  group_solve     every shard of a job in ONE process on one GPU, halos by
                  device-to-device copies -- the same kernels and halo
                  geometry, for parity tests on a single device
"""
import ctypes

from . import _lib
from .games import GameSpec
from .solver import Solver


class ShardedSolver(Solver):
    """Shard `rank` of `world` of a dense solve; needs an initialised
    torch.distributed default group (any backend) for the bootstrap."""

    def __init__(self, spec, rank, world, device=None, **kw):
        super().__init__(spec, device=device, rank=rank, world=world,
                         layout="dense", **kw)
        if world > 1:
            self._comm_init()

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


def group_solve(spec, world, device=None, kernel_timing=False, flags=0):
    """Solve all `world` shards in this process (one GPU, one stream).
    Returns (SolveResult of the whole job, [shard Solvers])."""
    import torch
    spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
    dev = torch.device(device if device is not None else "cuda")
    # one explicit stream for every shard (torch's default stream has handle
    # 0, which the ABI reads as "library-owned stream per solver")
    stream = torch.cuda.Stream(device=dev)
    shards = [Solver(spec, device=dev, rank=g, world=world, layout="dense",
                     kernel_timing=kernel_timing, stream=stream, flags=flags)
              for g in range(world)]
    arr = (ctypes.c_void_p * world)(*[s.handle.value for s in shards])
    r = _lib.gm_result()
    torch.cuda.synchronize(dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().gm_solve_group(arr, world, ctypes.byref(r)))
    return shards[0]._result(r), shards
