"""Single-GPU solve driver: allocates HBM buffers with PyTorch-ROCm, hands
their addresses to libgamesman_hip.so and reads results back.

Stands in for one rank of the reference's Process (src/process.py:10-267):
``Solver.solve()`` is Process.run until the root is resolved, and
``Solver.query()`` reads the table that replaces the resolved/remote
CacheDicts (src/cache_dict.py).  No CPU fallback exists: without a gfx950
device the library returns GM_ENOGPU and this raises.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .games import GameSpec

NAMES = ("WIN", "LOSS", "TIE", "DRAW")


@dataclass
class SolveResult:
    root_value: int
    root_remoteness: int
    positions: int
    edges: int
    primitives: int
    levels: int
    max_level_width: int
    ms_total: float
    ms_forward: float
    ms_backward: float
    ms_expand_kernels: float = 0.0
    ms_resolve_kernels: float = 0.0
    n_expand_launches: int = 0
    n_resolve_launches: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def root_line(self):
        """Exactly what src/process.py:47-52 prints."""
        return "%s in %d moves" % (NAMES[self.root_value],
                                   self.root_remoteness)


class Solver:
    """Owns the device buffers of one game's solve on one GPU."""

    def __init__(self, spec, positions=0, device=None, kernel_timing=False,
                 layout="auto", max_table_bytes=0, rank=0, world=1,
                 stream=None, flags=0):
        """layout: "auto" (planes, else the level-major dense table, when
        the descriptor supports it and the table fits max_table_bytes; the
        ranked table for toot-and-otto; else bucketed levels when every move
        advances one level; else the keyed hash table), "planes" (sum games
        whose first two heaps hold 32 values: natural rank order,
        gm_plane.h), "dense" (the level-major dense table), "ranked"
        (toot-and-otto positions at computed indices, gm_ranked.h),
        "bucketed" or "hashed" (the open-addressing hash table).
        flags: kernel-family flags (_lib.GM_F_WORDS32 / GM_F_RESOLVE_SCALAR /
        GM_F_SHARD_INORDER, A/B runs), fixed for this solver's lifetime.
        rank/world > 1: this object is one shard of a dense / planes multi-
        GPU solve (gamesmanmpi_amd.dist), or with layout="bucketed" /
        "hashed" one md5 shard of a keyed solve (gamesmanmpi_amd.keyed;
        `positions` is then this shard's bound); stream: a torch stream to
        run on."""
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("gamesmanmpi_amd needs a ROCm GPU (gfx950); "
                               "no device is visible")
        self.torch = torch
        self.spec = spec if isinstance(spec, GameSpec) else GameSpec(*spec)
        self.device = torch.device(device if device is not None else "cuda")
        self.kernel_timing = kernel_timing
        if layout not in ("auto", "planes", "dense", "hashed", "bucketed", "ranked"):
            raise ValueError("layout must be auto, planes, dense, ranked, bucketed or hashed")
        self.layout = layout
        self.max_table_bytes = int(max_table_bytes)
        self.rank, self.world = int(rank), int(world)
        self.stream = stream
        if flags & ~_lib.KERNEL_FLAGS:
            raise ValueError("flags: kernel-family flags only (%#x)" % _lib.KERNEL_FLAGS)
        self.flags = int(flags)
        self.positions_hint = int(positions or self.spec.positions_bound)
        # the layout planned: `layout`, except that "auto" falls back to the
        # hashed table when a bucketed plan hits a layout limit (solve())
        self._planned_layout = layout
        self._h = None
        self._bufs = None
        self._alloc(self.positions_hint)

    def _alloc(self, positions):
        torch = self.torch
        L = _lib.load()
        self._free()
        plan = _lib.gm_plan_t()
        flags = self.flags | {"hashed": _lib.GM_F_FORCE_HASHED | _lib.GM_F_HASH_TABLE,
                              "bucketed": _lib.GM_F_FORCE_HASHED,
                              "dense": _lib.GM_F_LEVEL_MAJOR}.get(self._planned_layout, 0)
        if self.world > 1 and self.layout in ("bucketed", "ranked"):
            # an md5 shard of bucketed levels (`positions` bounds this
            # shard), or of the RANKED index space (toot-and-otto)
            if self.layout == "ranked":
                flags |= _lib.GM_F_RANKED_SHARD
            _lib.check(L.gm_plan_keyed_shard(self.spec.id, self.rank,
                                             self.world, int(positions), flags,
                                             self.max_table_bytes,
                                             ctypes.byref(plan)))
        elif self.world > 1 and self.layout != "hashed":
            _lib.check(L.gm_plan_shard(self.spec.id, self.rank, self.world,
                                       flags, self.max_table_bytes,
                                       ctypes.byref(plan)))
        else:
            _lib.check(L.gm_plan(self.spec.id, int(positions), flags,
                                 self.max_table_bytes, ctypes.byref(plan)))
        if self.layout == "dense" and plan.mode != _lib.GM_MODE_DENSE:
            raise ValueError("%r has no dense layout (or it does not fit)"
                             % (self.spec,))
        if self.layout == "planes" and plan.mode != _lib.GM_MODE_PLANES:
            raise ValueError("%r has no planes layout (heaps 0 and 1 of 32 "
                             "values), or it does not fit" % (self.spec,))
        if self.layout == "ranked" and plan.mode != _lib.GM_MODE_RANKED:
            raise ValueError("%r has no ranked layout (toot-and-otto boards), or it "
                             "does not fit" % (self.spec,))
        if self.layout == "bucketed" and plan.mode != _lib.GM_MODE_BUCKETED:
            raise ValueError("%r: bucketed levels need every move to advance "
                             "one level" % (self.spec,))
        with torch.cuda.device(self.device):
            table = torch.empty(plan.table_bytes, dtype=torch.uint8,
                                device=self.device)
            levels = torch.empty(max(1, plan.level_capacity),
                                 dtype=torch.int64, device=self.device)
            scratch = torch.empty(plan.scratch_bytes, dtype=torch.uint8,
                                  device=self.device)
            stream = self.stream or torch.cuda.current_stream(self.device)
        self._tensors = (table, levels, scratch)
        b = _lib.gm_buffers()
        b.table = table.data_ptr()
        b.table_slots = plan.table_slots
        b.levels = levels.data_ptr()
        b.level_capacity = plan.level_capacity
        b.scratch = scratch.data_ptr()
        b.scratch_bytes = plan.scratch_bytes
        b.stream = stream.cuda_stream
        b.flags = flags | (_lib.GM_F_KERNEL_TIMING if self.kernel_timing else 0)
        b.mode = plan.mode
        b.table_bytes = plan.table_bytes
        self._bufs = b
        self._cflags = flags  # the flags the solver was created with (layout bits included)
        self.plan = plan
        h = ctypes.c_void_p()
        _lib.check(L.gm_solver_create_shard(self.spec.id, self.rank,
                                            self.world, ctypes.byref(b),
                                            ctypes.byref(h)))
        self._h = h

    def _free(self):
        if self._h is not None:
            _lib.load().gm_solver_destroy(self._h)
            self._h = None
        self._tensors = None

    def __del__(self):
        try:
            self._free()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass

    @property
    def handle(self):
        return self._h

    def shard_stats(self):
        """md5 shards of the RANKED layout: (slots this shard resolved in its
        last solve, reached positions its md5 owner rule gives it)."""
        out = (ctypes.c_uint64 * 2)()
        _lib.check(_lib.load().gm_rk_shard_stats(self._h, out))
        return int(out[0]), int(out[1])

    def set_kernel_timing(self, on):
        """Time every kernel launch with HIP events (on the solve stream)."""
        self.kernel_timing = bool(on)
        _lib.check(_lib.load().gm_solver_set_flags(
            self._h, self._cflags | (_lib.GM_F_KERNEL_TIMING if on else 0)))

    def solve(self, max_retries=4):
        """Full solve from the root; grows the buffers on GM_EFULL."""
        L = _lib.load()
        r = _lib.gm_result()
        if self.world > 1:
            max_retries = 0  # shard tables are sized exactly
        attempt = 0
        while True:
            try:
                with self.torch.cuda.device(self.device):
                    _lib.check(L.gm_solver_solve(self._h, ctypes.byref(r)))
                break
            except _lib.TableFull:
                if attempt == max_retries:
                    raise
                attempt += 1
                self.positions_hint *= 2
                self._alloc(self.positions_hint)
            except _lib.LayoutLimit:
                # a bucketed level past 2^29 positions or a fine bucket past
                # its LDS capacity: "auto" may use the hashed table instead
                # (once); an explicit layout keeps the error
                if (self.layout != "auto" or self._planned_layout != "auto" or self.world > 1
                        or int(self.plan.mode) != _lib.GM_MODE_BUCKETED):
                    raise
                self._planned_layout = "hashed"
                self._alloc(self.positions_hint)
        return self._result(r)

    # -- queued solves (one-table PLANES) ------------------------------------
    def solve_async(self):
        """Enqueue a full solve on the solver's stream and return its ticket
        without waiting (gm_solver_solve_async; one-table PLANES solvers).
        Solves queued back to back run back to back on the GPU; collect()
        each one, in ticket order (at most 8 outstanding)."""
        L = _lib.load()
        t = ctypes.c_uint64()
        with self.torch.cuda.device(self.device):
            _lib.check(L.gm_solver_solve_async(self._h, ctypes.byref(t)))
        return int(t.value)

    def collect(self, ticket):
        """Wait for queued solve `ticket`; its SolveResult (ms_total is the
        solve's device span)."""
        L = _lib.load()
        r = _lib.gm_result()
        with self.torch.cuda.device(self.device):
            _lib.check(L.gm_solver_collect(self._h, int(ticket), ctypes.byref(r)))
        return self._result(r)

    # -- stop / resume (checkpoints: gamesmanmpi_amd.checkpoint) ------------
    @property
    def steps(self):
        """Steps of a full solve (gm_solver_set_steps): forward levels
        0..T-1, then backward levels T-1..0."""
        return 2 * int(self.plan.max_levels)

    def solve_steps(self, first=0, stop=0):
        """Run steps [first, stop) of the solve (stop 0 = to the end).
        Returns the SolveResult when the solve completed, None when it
        stopped early -- the state then stays in this solver's buffers
        (save it with checkpoint.save, or continue with first=stop).  No
        buffer regrowth: a table that fills raises TableFull."""
        L = _lib.load()
        _lib.check(L.gm_solver_set_steps(self._h, int(first), int(stop)))
        r = _lib.gm_result()
        with self.torch.cuda.device(self.device):
            rc = L.gm_solver_solve(self._h, ctypes.byref(r))
        if rc == _lib.GM_PARTIAL:
            return None
        _lib.check(rc)
        return self._result(r)

    @property
    def buffers(self):
        """(table, level store, scratch) device tensors (uint8 / int64 /
        uint8): everything a stopped solve leaves behind."""
        return self._tensors

    def _result(self, r):
        return SolveResult(
            root_value=r.root_value, root_remoteness=r.root_remoteness,
            positions=r.positions, edges=r.edges, primitives=r.primitives,
            levels=r.levels, max_level_width=r.max_level_width,
            ms_total=r.ms_total, ms_forward=r.ms_forward,
            ms_backward=r.ms_backward,
            ms_expand_kernels=r.ms_expand_kernels,
            ms_resolve_kernels=r.ms_resolve_kernels,
            n_expand_launches=r.n_expand_launches,
            n_resolve_launches=r.n_resolve_launches,
            extra={"layout": _lib.MODE_NAMES[self.plan.mode],
                   "word_bits": r.word_bits,
                   "resolve_kernel": _lib.RESOLVE_KERNELS.get(r.kernels & 0xFFFF),
                   "pull_kernel": _lib.PULL_KERNELS.get(r.kernels >> 16),
                   "table_bytes": self.plan.table_bytes})

    # -- reading the table -------------------------------------------------
    def query(self, keys):
        """Words (value | remoteness << 2; GM_NO_WORD if unreachable) of
        `keys` (numpy uint64 array)."""
        torch = self.torch
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        if len(keys) == 0:
            return np.zeros(0, np.uint32)
        kd = torch.from_numpy(keys.view(np.int64)).to(self.device)
        wd = torch.empty(len(keys), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(_lib.load().gm_solver_query(
                self._h, kd.data_ptr(), len(keys), wd.data_ptr()))
        return wd.cpu().numpy().view(np.uint32)

    def positions(self):
        """Every reachable key (numpy uint64, level order)."""
        torch = self.torch
        n = ctypes.c_uint64()
        L = _lib.load()
        rc = L.gm_solver_positions(self._h, None, 0, ctypes.byref(n))
        if rc not in (0, _lib.GM_EFULL):
            _lib.check(rc)
        out = torch.empty(max(1, n.value), dtype=torch.int64,
                          device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(L.gm_solver_positions(self._h, out.data_ptr(),
                                             n.value, ctypes.byref(n)))
        return out[:n.value].cpu().numpy().view(np.uint64)

    def checksum(self):
        """Whole-solve fingerprint (gm_solver_checksum): dict with the
        order-independent checksum of every reachable position's
        (canonical bytes, value, remoteness), the position count and the
        W/L/T/D histogram."""
        out = np.zeros(6, np.uint64)
        with self.torch.cuda.device(self.device):
            _lib.check(_lib.load().gm_solver_checksum(self._h,
                                                      out.ctypes.data))
        v = [int(x) for x in out]
        return {"checksum": "%016x" % v[0], "positions": v[1], "win": v[2],
                "loss": v[3], "tie": v[4], "draw": v[5]}

    def dump(self):
        """(keys u64, value u8, remoteness u32) for every reachable
        position."""
        keys = self.positions()
        w = self.query(keys)
        if (w == _lib.GM_NO_WORD).any():
            raise RuntimeError("unresolved positions in the table")
        return keys, (w & 3).astype(np.uint8), (w >> 2).astype(np.uint32)


def solve(name, params="", positions=0, device=None):
    """Convenience: solve game `name` (reference file stem) on one GPU."""
    s = Solver(GameSpec(name, params), positions=positions, device=device)
    return s.solve(), s
