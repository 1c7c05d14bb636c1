"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker (or the timed CPU baseline).  The
product package gamesmanmpi_amd never imports it.  See oracle.c's header for
what is restated from the reference and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

WIN, LOSS, TIE, DRAW, UNDECIDED = 0, 1, 2, 3, 4
NAMES = ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED")


def build():
    """Compile liboracle.so in place (gcc; no reference sources involved)."""
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.or_game.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.or_root.argtypes = [ctypes.c_int, ctypes.c_void_p,
                              ctypes.POINTER(ctypes.c_int)]
        L.or_expand.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_int), ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.or_solve.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.or_solve.restype = ctypes.c_void_p
        for f in ("or_count", "or_edges"):
            getattr(L, f).argtypes = [ctypes.c_void_p]
            getattr(L, f).restype = ctypes.c_uint64
        L.or_root_word.argtypes = [ctypes.c_void_p]
        L.or_root_word.restype = ctypes.c_uint32
        L.or_dump.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p]
        L.or_lookup.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                ctypes.c_int]
        L.or_lookup.restype = ctypes.c_uint32
        L.or_free.argtypes = [ctypes.c_void_p]
        L.or_last_error.restype = ctypes.c_char_p
        # multi-threaded restatements (oracle_mt.c)
        L.or_threads.restype = ctypes.c_int
        L.or_solve_levels.argtypes = [ctypes.c_int, ctypes.c_int]
        L.or_solve_levels.restype = ctypes.c_void_p
        L.or_lsolve_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.or_lsolve_lookup.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.c_int]
        L.or_lsolve_lookup.restype = ctypes.c_uint32
        L.or_lsolve_free.argtypes = [ctypes.c_void_p]
        L.or_solve_rows.argtypes = [ctypes.c_int]
        L.or_solve_rows.restype = ctypes.c_void_p
        L.or_rsolve_stats.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p]
        L.or_rsolve_word.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.or_rsolve_word.restype = ctypes.c_uint32
        L.or_rsolve_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def _err():
    return lib().or_last_error().decode()


class Game:
    """One oracle game instance: name as in the reference's test_games file
    stem, params like "length=4,height=4" / "start=20" / "heaps=31:31"."""

    def __init__(self, name, params=""):
        self.name, self.params = name, params
        self.h = lib().or_game(name.encode(), params.encode())
        if self.h < 0:
            raise ValueError(_err())

    def root(self):
        buf = ctypes.create_string_buffer(32)
        n = ctypes.c_int()
        lib().or_root(self.h, buf, ctypes.byref(n))
        return buf.raw[:n.value]

    def expand(self, canon):
        prim = ctypes.c_int()
        nch = ctypes.c_int()
        ch = ctypes.create_string_buffer(32 * 64)
        lens = (ctypes.c_int * 64)()
        rc = lib().or_expand(self.h, canon, len(canon), ctypes.byref(prim),
                             ch, lens, ctypes.byref(nch))
        if rc:
            raise ValueError(_err())
        raw = ch.raw
        return prim.value, [raw[32 * i:32 * i + lens[i]]
                            for i in range(nch.value)]

    def solve(self, max_positions=1 << 20):
        return Solution(self, max_positions)

    def solve_levels(self, keep=True):
        """Multi-threaded tier-synchronous solve (oracle_mt.c, all
        OpenMP threads); keep=False frees levels as the backward pass goes
        (large games: only stats and the checksum remain)."""
        return LevelSolution(self, keep)

    def solve_rows(self):
        """Multi-threaded row solve of an int game (sum_four_to_one /
        four_to_one; oracle_mt.c)."""
        return RowSolution(self)


def threads():
    """OpenMP threads the multi-threaded solvers use."""
    return lib().or_threads()


STAT_KEYS = ("positions", "edges", "primitives", "root_word", "checksum",
             "win", "loss", "tie", "draw")


class _Stats:
    def _fill(self, raw):
        self.stats = dict(zip(STAT_KEYS, [int(x) for x in raw]))
        self.count = self.stats["positions"]
        self.edges = self.stats["edges"]
        w = self.stats["root_word"]
        self.root_value, self.root_remoteness = w & 3, w >> 2

    @property
    def root_line(self):
        return "%s in %d moves" % (NAMES[self.root_value],
                                   self.root_remoteness)


class LevelSolution(_Stats):
    def __init__(self, game, keep):
        self.game = game
        self.h = lib().or_solve_levels(game.h, 1 if keep else 0)
        if not self.h:
            raise RuntimeError(_err())
        raw = np.zeros(9, np.uint64)
        lib().or_lsolve_stats(self.h, raw.ctypes.data)
        self._fill(raw)

    def lookup(self, canon):
        w = lib().or_lsolve_lookup(self.h, canon, len(canon))
        if w == 0xFFFFFFFF:
            raise KeyError(canon)
        return w & 3, w >> 2

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_lsolve_free(self.h)
            self.h = None


class RowSolution(_Stats):
    def __init__(self, game):
        self.game = game
        self.h = lib().or_solve_rows(game.h)
        if not self.h:
            raise RuntimeError(_err())
        self.refresh(False)

    def refresh(self, with_checksum=True):
        raw = np.zeros(9, np.uint64)
        lib().or_rsolve_stats(self.h, 1 if with_checksum else 0,
                              raw.ctypes.data)
        self._fill(raw)
        return self.stats

    def word(self, rank):
        return lib().or_rsolve_word(self.h, int(rank))

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_rsolve_free(self.h)
            self.h = None


class Solution:
    def __init__(self, game, max_positions):
        self.game = game
        self.h = lib().or_solve(game.h, max_positions)
        if not self.h:
            raise RuntimeError(_err())
        self.count = lib().or_count(self.h)
        self.edges = lib().or_edges(self.h)
        w = lib().or_root_word(self.h)
        self.root_value, self.root_remoteness = w & 3, w >> 2

    @property
    def root_line(self):
        # src/process.py:47-52 format
        return "%s in %d moves" % (NAMES[self.root_value],
                                   self.root_remoteness)

    def dump(self, stride=24):
        """Every solved position, sorted by canonical bytes:
        (canon[n, stride] u8, clen u8, value u8, remoteness u32)."""
        n = self.count
        canon = np.zeros((n, stride), np.uint8)
        clen = np.zeros(n, np.uint8)
        val = np.zeros(n, np.uint8)
        rem = np.zeros(n, np.uint32)
        rc = lib().or_dump(self.h, canon.ctypes.data, stride,
                           clen.ctypes.data, val.ctypes.data, rem.ctypes.data)
        if rc:
            raise RuntimeError("dump failed")
        order = sorted(range(n), key=lambda i: bytes(canon[i, :clen[i]]))
        order = np.array(order, dtype=np.int64)
        return canon[order], clen[order], val[order], rem[order]

    def lookup(self, canon):
        w = lib().or_lookup(self.h, canon, len(canon))
        if w == 0xFFFFFFFF:
            raise KeyError(canon)
        return w & 3, w >> 2

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_free(self.h)
            self.h = None
