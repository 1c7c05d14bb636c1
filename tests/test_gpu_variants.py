"""GPU parity of every dense kernel family: the kernel-family
flags (include/gamesman.h GM_F_WORDS32 / GM_F_RESOLVE_SCALAR /
GM_F_SHARD_INORDER, fixed when a solver is created) select other kernels
for the same solve, and each must give the same words as the default path,
the closed-form counts and the Sprague-Grundy values.  Shapes exercise the
live-group lists with top-major XCD shares (C >= 8 columns), column jobs,
the one-prefix kernel, shard halos in 16 and 32 bits, and in-order
exchanges.  A table planned for 16-bit words refuses a 32-bit kernel with
GM_EINVAL instead of running it."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORDS32, SCALAR, INORDER, WORDS16 = 4, 8, 16, 64  # _lib.GM_F_*
WORLD1 = [0, WORDS16, WORDS32, SCALAR]
KERNELS1 = {WORDS16: "k_dense_resolve8p", WORDS32: "k_dense_resolve4p", SCALAR: "k_dense_resolve"}


def _default_kernel(heaps):
    """8-bit words (k_dense_resolve16p) when the second heap's base is >= 16
    and every remoteness fits (root_sum <= 253), else 16-bit octets."""
    return "k_dense_resolve16p" if heaps[1] + 1 >= 16 and sum(heaps) <= 253 else "k_dense_resolve8p"


def _expected(heaps):
    P = 1
    for h in heaps:
        P *= h + 1
    E = sum(P * (2 * h - 1) // (h + 1) for h in heaps if h >= 1)
    g = 0
    for h in heaps:
        g ^= h % 3
    return P, E, "LOSS" if g == 0 else "WIN"


def _solve(params, flags):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    heaps = [int(h) for h in params.split("=")[1].split(":")]
    s = Solver(GameSpec("sum_four_to_one", params), layout="dense", flags=flags)
    r = s.solve()
    assert r.extra["resolve_kernel"] == (KERNELS1[flags] if flags else _default_kernel(heaps)), r.extra
    keys, val, rem = s.dump()
    order = np.argsort(keys)
    return r, keys[order], val[order], rem[order]


@pytest.mark.parametrize("params", ["heaps=15:15:15:15:7", "heaps=31:7:31:15", "heaps=63:31:31:31:63",
                                    "heaps=127:15:127"])
def test_world1_variants_agree(params):
    heaps = [int(h) for h in params.split("=")[1].split(":")]
    P, E, root = _expected(heaps)
    base = None
    for env in WORLD1:
        r, keys, val, rem = _solve(params, env)
        assert (r.positions, r.edges, r.root_line.split()[0]) == (P, E, root), env
        if base is None:
            base = (keys, val, rem)
            # Sprague-Grundy: LOSS iff the XOR of (heap mod 3) is 0
            k = keys.astype(np.int64)
            g = np.zeros(len(k), np.int64)
            for h in heaps:
                g ^= (k % (h + 1)) % 3
                k //= h + 1
            np.testing.assert_array_equal(val == 1, g == 0)
            continue
        np.testing.assert_array_equal(keys, base[0], err_msg=str(env))
        np.testing.assert_array_equal(val, base[1], err_msg=str(env))
        np.testing.assert_array_equal(rem, base[2], err_msg=str(env))


@pytest.mark.parametrize("flags", [0, WORDS32, INORDER, WORDS32 | INORDER, SCALAR])
@pytest.mark.parametrize("world", [2, 3])
def test_shard_halo_word_widths(flags, world):
    """Column-order halos (Z % 256 == 0): 16-bit shard tables with 16-bit
    halos (default, k_dense_resolve8c), 32-bit tables with 16-bit halos
    (k_dense_resolve4c), the one-prefix kernel, overlapped and in-order
    exchanges -- each against the single-table solve."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    params = "heaps=15:15:15:15:31"  # Z = 16^3 = 4096 prefixes (16 columns) per slice
    s1 = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    r1 = s1.solve()
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world, flags=flags)
    assert (rg.positions, rg.edges, rg.root_line) == (r1.positions, r1.edges, r1.root_line)
    wide = bool(flags & (WORDS32 | SCALAR))
    assert rg.extra["word_bits"] == (32 if wide else 16), rg.extra
    want = "k_dense_resolve" if flags & SCALAR else "k_dense_resolve4c" if wide else "k_dense_resolve8c"
    assert rg.extra["resolve_kernel"] == want, rg.extra
    keys, val, rem = s1.dump()
    out = np.full(len(keys), 0xFFFFFFFF, np.uint32)
    for s in shards:
        w = s.query(keys)
        own = w != 0xFFFFFFFF
        out[own] = w[own]
    np.testing.assert_array_equal(out & 3, val)
    np.testing.assert_array_equal(out >> 2, rem)


@pytest.mark.parametrize("world,params", [(8, "heaps=15:15:15:15:127"), (4, "heaps=15:15:15:15:63"),
                                          (8, "heaps=15:15:15:15:31")])
def test_shard_geometries_like_the_bench(world, params):
    """The bench's N-rank structure at a smaller slice size: round-robin
    blocks of 8 top values (two per rank at N = 8), 16-bit tables, packed
    16-bit halos in column order.  The in-process group checks every level's
    halo word count against what the receiving rank would post (the RCCL
    path's receive size) and the words against the single-table solve."""
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    s1 = Solver(GameSpec("sum_four_to_one", params), layout="dense")
    r1 = s1.solve()
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world)
    assert (rg.positions, rg.edges, rg.root_line) == (r1.positions, r1.edges, r1.root_line)
    assert rg.extra["word_bits"] == 16
    keys, val, rem = s1.dump()
    out = np.full(len(keys), 0xFFFFFFFF, np.uint32)
    hits = np.zeros(len(keys), np.int64)
    for s in shards:
        w = s.query(keys)
        own = w != 0xFFFFFFFF
        out[own] = w[own]
        hits += own
    assert (hits == 1).all()
    np.testing.assert_array_equal(out & 3, val)
    np.testing.assert_array_equal(out >> 2, rem)


def test_16bit_table_refuses_32bit_kernels():
    """The round-1 fault class (a 32-bit kernel writing past a 16-bit word
    area): kernel families are fixed at creation from the flags the table
    was planned with.  A 16-bit plan (GM_F_WORDS16) handed GM_F_WORDS32 at
    creation, an 8-bit plan handed GM_F_WORDS16, or a solver asked to switch
    afterwards, returns GM_EINVAL; the solver keeps solving correctly."""
    import torch
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    L = _lib.load()
    spec = GameSpec("sum_four_to_one", "heaps=15:15:15:15:7")
    for planned, given in ((_lib.GM_F_WORDS16, _lib.GM_F_WORDS32), (0, _lib.GM_F_WORDS16)):
        plan = _lib.gm_plan_t()
        _lib.check(L.gm_plan(spec.id, 0, planned, 0, ctypes.byref(plan)))
        assert plan.mode == _lib.GM_MODE_DENSE
        table = torch.empty(plan.table_bytes, dtype=torch.uint8, device="cuda")
        scratch = torch.empty(plan.scratch_bytes, dtype=torch.uint8, device="cuda")
        b = _lib.gm_buffers()
        b.table, b.table_slots, b.table_bytes = table.data_ptr(), plan.table_slots, plan.table_bytes
        b.scratch, b.scratch_bytes = scratch.data_ptr(), plan.scratch_bytes
        b.mode, b.flags = plan.mode, given
        h = ctypes.c_void_p()
        assert L.gm_solver_create(spec.id, ctypes.byref(b), ctypes.byref(h)) == _lib.GM_EINVAL
        assert b"flags need" in L.gm_last_error()
    s16 = Solver(spec, layout="dense", flags=_lib.GM_F_WORDS16)
    assert s16.solve().extra["word_bits"] == 16
    s = Solver(spec, layout="dense")
    r = s.solve()
    assert r.extra["word_bits"] == 8
    assert L.gm_solver_set_flags(s.handle, _lib.GM_F_WORDS32) == _lib.GM_EINVAL
    assert L.gm_solver_set_flags(s.handle, _lib.GM_F_RESOLVE_SCALAR) == _lib.GM_EINVAL
    assert L.gm_solver_set_flags(s.handle, _lib.GM_F_WORDS16) == _lib.GM_EINVAL
    assert s.solve().root_line == r.root_line
