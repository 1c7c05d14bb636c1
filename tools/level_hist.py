"""Positions per level of a solved keyed game (toot: pieces on the board):
    python tools/level_hist.py [L H]"""
import sys

import numpy as np

sys.path.insert(0, ".")


def main():
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    L, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (6, 4)
    s = Solver(GameSpec("toot_and_otto_bitstring", "length=%d,height=%d" % (L, H)), layout="bucketed")
    r = s.solve()
    keys = np.asarray(s.positions(), dtype=np.uint64)
    A = L * H
    occ = (keys | (keys >> np.uint64(A))) & np.uint64((1 << A) - 1)
    lev = np.bitwise_count(occ)
    h = np.bincount(lev, minlength=A + 1)
    print("positions", r.positions, "edges", r.edges)
    print("per level:", h.tolist())


if __name__ == "__main__":
    main()
