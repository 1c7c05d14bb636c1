"""Game files without a device descriptor.

The reference drives any module that implements the game-module API
(initial_position / gen_moves / do_move / primitive, README.md:28-88)
through GameState.expand and .primitive (src/game_state.py:32-40,58-84).
Here the host does exactly that enumeration -- the module's own functions,
breadth first from initial_position() -- and builds a CSR graph of the
reachable positions; the retrograde pass runs on the GPU
(gm_graph_solve: rounds of "resolve every position whose children are all
resolved", the same reduction as the descriptor pipeline).

Positions are identified by str(pos), the identity the reference itself
hashes (GameState.get_hash, src/game_state.py:22-30); two positions with the
same str() are one position, as they are one shelve key there.  Host
enumeration runs at Python speed (about 10^4-10^5 positions/s), so this path
is for game files without a descriptor, not for the headline configs.
"""
import ctypes
import time
from collections import deque

import numpy as np

from . import _lib
from .solver import SolveResult

UNDECIDED = 4


class GameGraph:
    """Reachable positions of a module: ids in breadth-first order (root =
    0), names (str(pos)), primitive codes, CSR children in gen_moves order."""

    def __init__(self, names, prim, offsets, children, positions=None):
        self.names = names
        self.prim = prim
        self.offsets = offsets
        self.children = children
        self.positions = positions

    @property
    def n(self):
        return len(self.names)

    @property
    def edges(self):
        return int(self.offsets[-1])


def enumerate_game(module, limit=50_000_000, keep_positions=False):
    """Breadth-first enumeration with the module's own functions.  A
    position's children are do_move(pos, m) for m in gen_moves(pos), only
    for positions whose primitive() is UNDECIDED (Process.lookup,
    src/process.py:109-132)."""
    root = module.initial_position()
    ids = {str(root): 0}
    names = [str(root)]
    objs = [root]
    prim = []
    offsets = [0]
    children = []
    queue = deque([0])
    while queue:
        i = queue.popleft()
        pos = objs[i]
        p = int(module.primitive(pos))
        prim.append(p)
        if p == UNDECIDED:
            for m in module.gen_moves(pos):
                c = module.do_move(pos, m)
                k = str(c)
                j = ids.get(k)
                if j is None:
                    j = len(names)
                    if j >= limit:
                        raise ValueError("more than %d positions" % limit)
                    ids[k] = j
                    names.append(k)
                    objs.append(c)
                    queue.append(j)
                children.append(j)
        offsets.append(len(children))
        if not keep_positions:
            objs[i] = None
    return GameGraph(names, np.asarray(prim, np.uint8),
                     np.asarray(offsets, np.int64),
                     np.asarray(children, np.uint32),
                     objs if keep_positions else None)


class GenericSolver:
    """Solve an enumerated GameGraph on one GPU (no descriptor needed)."""

    def __init__(self, graph, device=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("gamesmanmpi_amd needs a ROCm GPU (gfx950); "
                               "no device is visible")
        self.torch = torch
        self.graph = graph
        self.device = torch.device(device if device is not None else "cuda")
        self.words = None

    def solve(self):
        torch, g = self.torch, self.graph
        t0 = time.perf_counter()
        with torch.cuda.device(self.device):
            dev = self.device
            prim = torch.from_numpy(g.prim).to(dev)
            offsets = torch.from_numpy(g.offsets).to(dev)
            ch = g.children if len(g.children) else np.zeros(1, np.uint32)
            children = torch.from_numpy(ch.view(np.int32)).to(dev)
            words = torch.empty(g.n, dtype=torch.int32, device=dev)
            scratch = torch.zeros(4096, dtype=torch.uint8, device=dev)
            stream = torch.cuda.current_stream(dev)
            r = _lib.gm_result()
            _lib.check(_lib.load().gm_graph_solve(
                prim.data_ptr(), offsets.data_ptr(), children.data_ptr(),
                g.n, 0, words.data_ptr(), scratch.data_ptr(),
                stream.cuda_stream, ctypes.byref(r)))
        self.words = words.cpu().numpy().view(np.uint32)
        return SolveResult(
            root_value=r.root_value, root_remoteness=r.root_remoteness,
            positions=r.positions, edges=r.edges, primitives=r.primitives,
            levels=r.levels, max_level_width=0, ms_total=r.ms_total,
            ms_forward=0.0, ms_backward=r.ms_total,
            n_resolve_launches=r.n_resolve_launches,
            extra={"layout": "graph", "rounds": r.levels,
                   "host_enumeration_s": getattr(g, "enum_s", None),
                   "wall_s": time.perf_counter() - t0})

    def dump(self):
        """(names, value u8, remoteness u32) for every reachable position."""
        w = self.words
        return self.graph.names, (w & 3).astype(np.uint8), (w >> 2).astype(np.uint32)


def solve_module(module, device=None, limit=50_000_000):
    """Enumerate `module` on the host and solve it on the GPU."""
    t0 = time.perf_counter()
    g = enumerate_game(module, limit=limit)
    g.enum_s = time.perf_counter() - t0
    s = GenericSolver(g, device=device)
    return s.solve(), s
