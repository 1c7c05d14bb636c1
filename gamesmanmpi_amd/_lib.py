"""ctypes binding of the C-ABI in include/gamesman.h (libgamesman_hip.so).

torch is imported before the library is loaded so both share one HIP runtime
(torch/lib/libamdhip64.so.7 has the same soname the library links against);
device buffers allocated by torch are then valid addresses for the kernels.
There is no CPU fallback: if the library is missing this module raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# GM_LIBPATH: an alternative in-tree build of the same ABI (A/B runs of
# kernel variants, tools/diag_streams.sh)
LIBPATH = os.environ.get("GM_LIBPATH") or os.path.join(HERE, "libgamesman_hip.so")

GM_EINVAL, GM_EHIP, GM_EFULL, GM_ECORRUPT, GM_ENOGPU, GM_ELIMIT = -1, -2, -3, -4, -5, -6
GM_PARTIAL = 1  # gm_solver_solve stopped at the gm_solver_set_steps bound
GM_F_KERNEL_TIMING = 1
GM_F_FORCE_HASHED = 2
# kernel-family flags: given to gm_plan AND gm_buffers.flags (fixed for the
# solver's lifetime; include/gamesman.h)
GM_F_WORDS32 = 4
GM_F_RESOLVE_SCALAR = 8
GM_F_SHARD_INORDER = 16
GM_F_HASH_TABLE = 32  # gm_plan, keyed games: open-addressing table, not BUCKETED
GM_F_WORDS16 = 64  # dense: 16-bit words where 8-bit ones would be chosen
GM_F_BK_EXACT = 128  # bucketed: count pass + exact partition offsets
GM_F_GRAPH = 256  # dense one-table solves replay captured HIP graphs
GM_F_LEVEL_MAJOR = 512  # the level-major DENSE layout where PLANES would apply
GM_F_PLANE_X1 = 1024  # PLANES A/B: one plane per half-wave (k_plane_resolve)
GM_F_PLANE_ROUND_ROBIN = 2048  # PLANES shards A/B: round-robin blocks (one halo link)
GM_F_PLANE_LEVEL_SYNC = 4096  # PLANES shards A/B: level-synchronous deal instead of the staged pipeline
GM_F_PLANE_NO_RUNS = 8192  # PLANES A/B: no one-workgroup runs of narrow levels / keys
GM_F_BKS_LOCAL = 16384  # md5-sharded bucketed: local dedup before hashing / sending
GM_F_RANKED_SHARD = 32768  # gm_plan_keyed_shard: md5 shards of the RANKED layout (toot-and-otto)
GM_F_PLANE_LEVELS = 65536  # PLANES A/B: per-level launches instead of the one-launch backward (k_plane_flow)
KERNEL_FLAGS = (GM_F_WORDS32 | GM_F_RESOLVE_SCALAR | GM_F_SHARD_INORDER | GM_F_WORDS16 | GM_F_BK_EXACT
                | GM_F_GRAPH | GM_F_LEVEL_MAJOR | GM_F_PLANE_X1 | GM_F_PLANE_ROUND_ROBIN
                | GM_F_PLANE_LEVEL_SYNC | GM_F_PLANE_NO_RUNS | GM_F_PLANE_LEVELS
                | GM_F_BKS_LOCAL)
# gm_result.kernels codes (gm_solver.hip DenseResolveKind / DensePullKind)
RESOLVE_KERNELS = {1: "k_dense_resolve8p", 2: "k_dense_resolve8c", 3: "k_dense_resolve4p",
                   4: "k_dense_resolve4c", 5: "k_dense_resolve4", 6: "k_dense_resolve",
                   7: "k_dense_resolve16p", 8: "k_plane_resolve", 9: "k_plane_resolve_x2",
                   10: "k_rk_backward", 11: "k_plane_flow"}
PULL_KERNELS = {1: "k_dense_pull_words", 2: "k_dense_pull", 3: "k_plane_reach"}
GM_MODE_HASHED, GM_MODE_DENSE, GM_MODE_BUCKETED, GM_MODE_PLANES, GM_MODE_RANKED = 0, 1, 2, 3, 4
# host-staged transport (include/gamesman.h gm_xfer_fn)
GM_XFER_SENDRECV, GM_XFER_ALLGATHER = 0, 1
XFER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int)
MODE_NAMES = {0: "hashed", 1: "dense", 2: "bucketed", 3: "planes", 4: "ranked"}
GM_MAXCHILD = 32
GM_COMM_ID_BYTES = 128
GM_NO_WORD = 0xFFFFFFFF


class GmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


class TableFull(GmError):
    """GM_EFULL: the buffers are too small; re-planning larger fixes it."""


class LayoutLimit(GmError):
    """GM_ELIMIT: a limit of the layout that more memory cannot lift (a
    bucketed hash bucket over capacity, a level too wide); never retried."""


class gm_plan_t(ctypes.Structure):
    _fields_ = [("table_bytes", ctypes.c_uint64),
                ("table_slots", ctypes.c_uint64),
                ("level_capacity", ctypes.c_uint64),
                ("scratch_bytes", ctypes.c_uint64),
                ("max_levels", ctypes.c_uint32),
                ("mode", ctypes.c_uint32)]


class gm_buffers(ctypes.Structure):
    _fields_ = [("table", ctypes.c_void_p),
                ("table_slots", ctypes.c_uint64),
                ("levels", ctypes.c_void_p),
                ("level_capacity", ctypes.c_uint64),
                ("scratch", ctypes.c_void_p),
                ("scratch_bytes", ctypes.c_uint64),
                ("stream", ctypes.c_void_p),
                ("flags", ctypes.c_uint32),
                ("mode", ctypes.c_uint32),
                ("table_bytes", ctypes.c_uint64)]


class gm_result(ctypes.Structure):
    _fields_ = [("root_word", ctypes.c_uint32),
                ("root_value", ctypes.c_int32),
                ("root_remoteness", ctypes.c_uint64),
                ("positions", ctypes.c_uint64),
                ("edges", ctypes.c_uint64),
                ("primitives", ctypes.c_uint64),
                ("levels", ctypes.c_uint32),
                ("max_level_width", ctypes.c_uint32),
                ("ms_total", ctypes.c_double),
                ("ms_forward", ctypes.c_double),
                ("ms_backward", ctypes.c_double),
                ("ms_expand_kernels", ctypes.c_double),
                ("ms_resolve_kernels", ctypes.c_double),
                ("n_expand_launches", ctypes.c_uint64),
                ("n_resolve_launches", ctypes.c_uint64),
                ("word_bits", ctypes.c_uint32),
                ("kernels", ctypes.c_uint32)]


# every symbol include/gamesman.h declares (tests check the exports)
EXPORTS = (
    "gm_game_lookup", "gm_game_info", "gm_root", "gm_encode", "gm_decode",
    "gm_encode_batch", "gm_decode_batch", "gm_str_utf8", "gm_host_expand", "gm_host_level", "gm_symmetry", "gm_abi_sizes", "gm_plan", "gm_solver_create",
    "gm_solver_solve", "gm_solver_solve_async", "gm_solver_collect", "gm_solver_query", "gm_solver_positions",
    "gm_solver_checksum",
    "gm_solver_destroy", "gm_solve", "gm_plan_multi", "gm_query", "gm_release", "gm_owner", "gm_owner_host",
    "gm_plan_shard", "gm_plan_keyed_shard", "gm_solver_create_shard", "gm_comm_unique_id",
    "gm_solver_comm_init", "gm_solve_group", "gm_solver_set_flags", "gm_solver_set_steps",
    "gm_shard_info", "gm_solver_set_transport", "gm_shard_halo_sigs", "gm_plane_halo_plan", "gm_rk_shard_stats",
    "gm_ks_begin", "gm_ks_level_size", "gm_ks_expand", "gm_ks_insert",
    "gm_ks_finalize", "gm_ks_counts", "gm_ks_children", "gm_ks_reduce",
    "gm_ks_end", "gm_graph_solve",
    "gm_last_error", "gm_version",
)

_lib = None


def load():
    """Load libgamesman_hip.so (after torch) and declare signatures."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  -- share torch's HIP runtime (see docstring)
    if not os.path.exists(LIBPATH):
        raise ImportError(
            "libgamesman_hip.so not built: run `python -c 'import "
            "__graft_entry__ as g; g.build()'` (or `make -C gamesmanmpi_amd`)")
    L = ctypes.CDLL(LIBPATH)
    c = ctypes
    P = c.POINTER
    sig = {
        "gm_game_lookup": [c.c_char_p, c.c_char_p, P(c.c_int)],
        "gm_game_info": [c.c_int, P(c.c_uint64), P(c.c_uint32), P(c.c_uint32)],
        "gm_root": [c.c_int, P(c.c_uint64)],
        "gm_encode": [c.c_int, c.c_char_p, c.c_size_t, P(c.c_uint64)],
        "gm_decode": [c.c_int, c.c_uint64, c.c_void_p, c.c_size_t,
                      P(c.c_size_t)],
        "gm_encode_batch": [c.c_int, c.c_void_p, c.c_size_t, c.c_void_p,
                            c.c_size_t, c.c_void_p],
        "gm_decode_batch": [c.c_int, c.c_void_p, c.c_size_t, c.c_void_p,
                            c.c_size_t, c.c_void_p],
        "gm_str_utf8": [c.c_int, c.c_uint64, c.c_void_p, c.c_size_t,
                        P(c.c_size_t)],
        "gm_host_expand": [c.c_int, c.c_void_p, c.c_size_t, c.c_void_p,
                           c.c_void_p, c.c_void_p],
        "gm_host_level": [c.c_int, c.c_void_p, c.c_size_t, c.c_void_p],
        "gm_symmetry": [c.c_int, c.c_int, c.c_void_p, c.c_size_t, c.c_void_p],
        "gm_abi_sizes": [c.c_void_p],
        "gm_plan": [c.c_int, c.c_uint64, c.c_uint32, c.c_uint64,
                    P(gm_plan_t)],
        "gm_solver_create": [c.c_int, P(gm_buffers), P(c.c_void_p)],
        "gm_solver_solve": [c.c_void_p, P(gm_result)],
        "gm_solver_solve_async": [c.c_void_p, P(c.c_uint64)],
        "gm_solver_collect": [c.c_void_p, c.c_uint64, P(gm_result)],
        "gm_solver_query": [c.c_void_p, c.c_void_p, c.c_uint64, c.c_void_p],
        "gm_solver_positions": [c.c_void_p, c.c_void_p, c.c_uint64,
                                P(c.c_uint64)],
        "gm_solver_checksum": [c.c_void_p, c.c_void_p],
        "gm_solve": [c.c_int, c.c_uint64, c.c_int, P(gm_buffers),
                     P(gm_result)],
        "gm_plan_multi": [c.c_int, c.c_int, c.c_uint64, c.c_uint32, c.c_uint64, P(gm_plan_t)],
        "gm_query": [c.c_int, c.c_void_p, c.c_size_t, c.c_void_p],
        "gm_release": [c.c_int],
        "gm_owner": [c.c_int, c.c_void_p, c.c_uint64, c.c_int, c.c_void_p,
                     c.c_void_p],
        "gm_owner_host": [c.c_int, c.c_void_p, c.c_size_t, c.c_int,
                          c.c_void_p],
        "gm_plan_shard": [c.c_int, c.c_int, c.c_int, c.c_uint32, c.c_uint64,
                          P(gm_plan_t)],
        "gm_plan_keyed_shard": [c.c_int, c.c_int, c.c_int, c.c_uint64, c.c_uint32,
                                c.c_uint64, P(gm_plan_t)],
        "gm_solver_create_shard": [c.c_int, c.c_int, c.c_int, P(gm_buffers),
                                   P(c.c_void_p)],
        "gm_comm_unique_id": [c.c_void_p],
        "gm_solver_comm_init": [c.c_void_p, c.c_void_p],
        "gm_solve_group": [c.POINTER(c.c_void_p), c.c_int, P(gm_result)],
        "gm_solver_set_flags": [c.c_void_p, c.c_uint32],
        "gm_solver_set_steps": [c.c_void_p, c.c_uint32, c.c_uint32],
        "gm_shard_info": [c.c_int, c.c_int, c.c_int, P(c.c_uint64)],
        "gm_solver_set_transport": [c.c_void_p, XFER_FN, c.c_void_p],
        "gm_shard_halo_sigs": [c.c_int, c.c_int, c.c_int, c.c_uint32, c.c_void_p, c.c_uint32],
        "gm_plane_halo_plan": [c.c_int, c.c_int, c.c_int, c.c_uint32, c.c_void_p, c.c_uint32],
        "gm_rk_shard_stats": [c.c_void_p, c.c_void_p],
        "gm_ks_begin": [c.c_void_p, c.c_int],
        "gm_ks_level_size": [c.c_void_p, c.c_int, P(c.c_uint64)],
        "gm_ks_expand": [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p,
                         c.c_uint64, c.c_int, P(c.c_uint64)],
        "gm_ks_insert": [c.c_void_p, c.c_int, c.c_void_p, c.c_uint64],
        "gm_ks_finalize": [c.c_void_p, c.c_int],
        "gm_ks_counts": [c.c_void_p, c.c_int, c.c_void_p],
        "gm_ks_children": [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p,
                           c.c_void_p, c.c_int],
        "gm_ks_reduce": [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p],
        "gm_ks_end": [c.c_void_p, P(gm_result)],
        "gm_graph_solve": [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint64,
                           c.c_uint64, c.c_void_p, c.c_void_p, c.c_void_p,
                           P(gm_result)],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = c.c_int
    L.gm_solver_destroy.argtypes = [c.c_void_p]
    L.gm_solver_destroy.restype = None
    L.gm_last_error.restype = c.c_char_p
    L.gm_version.restype = c.c_char_p
    _lib = L
    return L


def check(rc):
    if rc == 0:
        return
    msg = load().gm_last_error().decode(errors="replace")
    if rc == GM_EFULL:
        raise TableFull(rc, msg)
    if rc == GM_ELIMIT:
        raise LayoutLimit(rc, msg)
    raise GmError(rc, msg)
