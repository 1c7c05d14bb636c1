#!/usr/bin/env python3
"""Generate tests/golden/checksums.json: whole-solve fingerprints of the
configs too large for per-position fixtures, from the multi-threaded CPU
restatement (oracle/oracle_mt.c).

Each entry: positions, edges, primitives, root line, value histogram and the
order-independent checksum of every reachable position's (canonical bytes,
value, remoteness) -- gm_solver_checksum computes the same function on the
GPU (gamesmanmpi_amd/csrc/gm_codec.h pos_checksum).

How the oracle behind these numbers is pinned: tests/test_oracle.py checks
oracle_mt against the golden per-position tables generated from the
reference's own game modules (TTT, othello 4x4, toot up to 4x4, Four-To-One,
sums) and against oracle.c's scalar DFS; toot 5x4 and 6x4 also reproduce
SURVEY.md Appendix B (counts, W/L/T histogram, root line) from the survey's
independent C++ probe.  Beyond 4x4 no reference fixture exists: parity there
is against this restatement, pinned on the smaller boards.

Usage: python tests/golden/make_checksums.py [case ...]   (all by default;
toot_6x4 needs ~25 GB of RAM and ~20 min on 8 cores)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.oracle import Game, threads  # noqa: E402

OUT = os.path.join(HERE, "checksums.json")

CASES = {
    "toot_4x4": ("toot_and_otto_bitstring", "length=4,height=4", "levels"),
    "toot_5x4": ("toot_and_otto_bitstring", "length=5,height=4", "levels"),
    "toot_6x4": ("toot_and_otto_bitstring", "length=6,height=4", "levels"),
    "othello_4x4": ("othello_bit_new", "length=4,height=4", "levels"),
    "sum_31x6": ("sum_four_to_one", "heaps=31:31:31:31:31:31", "rows"),
    "sum_15x5": ("sum_four_to_one", "heaps=15:15:15:15:15", "rows"),
    # the bench's N-rank shapes (31^5 x (32N - 1)): their root lines let the
    # multi-GPU bench check the root remoteness as well as the closed forms
    "sum_31x5_63": ("sum_four_to_one", "heaps=31:31:31:31:31:63", "rows"),
    "sum_31x5_127": ("sum_four_to_one", "heaps=31:31:31:31:31:127", "rows"),
    "sum_31x5_255": ("sum_four_to_one", "heaps=31:31:31:31:31:255", "rows"),
    # the same shapes with the long heap second (heap 1): the row deal's
    # bench shapes -- the game is symmetric in its heaps, so
    # counts and root lines equal the ones above, the key-order checksum not
    "sum_31_63_31x4": ("sum_four_to_one", "heaps=31:63:31:31:31:31", "rows"),
    "sum_31_127_31x4": ("sum_four_to_one", "heaps=31:127:31:31:31:31", "rows"),
    "sum_31_255_31x4": ("sum_four_to_one", "heaps=31:255:31:31:31:31", "rows"),
}


def run(name):
    stem, params, how = CASES[name]
    g = Game(stem, params)
    t0 = time.time()
    if how == "levels":
        sol = g.solve_levels(keep=False)
        st = dict(sol.stats)
    else:
        sol = g.solve_rows()
        st = dict(sol.refresh(True))
    st.update({"game": stem, "params": params, "root_line": sol.root_line,
               "solver": "oracle_mt " + how, "threads": threads(),
               "seconds": round(time.time() - t0, 1)})
    st["checksum"] = "%016x" % st["checksum"]
    del sol
    return st


def main():
    todo = sys.argv[1:] or list(CASES)
    try:
        with open(OUT) as fh:
            data = json.load(fh)
    except (OSError, ValueError):
        data = {}
    for name in todo:
        data[name] = run(name)
        print(name, json.dumps(data[name]), flush=True)
        with open(OUT, "w") as fh:
            json.dump(data, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
