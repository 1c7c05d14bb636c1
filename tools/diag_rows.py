#!/usr/bin/env python3
"""Row-deal diagnostic: solve a small row-deal group, compare every position
with the oracle, histogram the mismatches by (rank, local row, h0, outer
digits sum) -- which rows / columns go wrong first."""
import sys

import numpy as np

sys.path.insert(0, ".")


def main():
    from collections import Counter
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    from oracle.oracle import Game
    params = sys.argv[1] if len(sys.argv) > 1 else "heaps=31:63:3:15"
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    heaps = [int(h) for h in params.split("=")[1].split(":")]
    rg, shards = group_solve(GameSpec("sum_four_to_one", params), world)
    sol = Game("sum_four_to_one", params).solve_rows()
    sol.refresh(True)
    print("gpu", rg.root_line, "oracle", sol.root_line)
    keys = np.arange(sol.count, dtype=np.uint64)
    want = np.array([sol.word(k) for k in range(sol.count)], np.uint32)
    for r, sh in enumerate(shards):
        w = sh.query(keys)
        own = w != 0xFFFFFFFF
        bad = own & (w != want)
        print("rank", r, "owns", int(own.sum()), "bad", int(bad.sum()))
        idx = np.nonzero(bad)[0][:20000]
        c = Counter()
        first = []
        for k in idx:
            x = int(k)
            dig = []
            for h in heaps:
                dig.append(x % (h + 1))
                x //= h + 1
            c[(dig[1] - 32 * r)] += 1
            if len(first) < 12:
                first.append((dig, "got", int(w[k]) & 3, int(w[k]) >> 2, "want", int(want[k]) & 3, int(want[k]) >> 2))
        print(" by local row:", sorted(c.items())[:40])
        for f in first:
            print("  ", f)


if __name__ == "__main__":
    main()
