"""Diagnostic: first positions where a sharded group solve and the
single-table solve disagree (prints key, heaps, level, words)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from gamesmanmpi_amd.games import GameSpec
from gamesmanmpi_amd.solver import Solver
from gamesmanmpi_amd.dist import group_solve

params = sys.argv[1] if len(sys.argv) > 1 else "heaps=7:7:7:15"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 3
heaps = [int(h) for h in params.split("=")[1].split(":")]
spec = GameSpec("sum_four_to_one", params)
s = Solver(spec, layout="dense")
r = s.solve()
rg, shards = group_solve(spec, world)
print("single", r.root_line, r.positions, r.edges, "group", rg.root_line, rg.positions, rg.edges)
keys, val, rem = s.dump()
w = np.full(len(keys), 0xFFFFFFFF, np.uint32)
owner = np.full(len(keys), -1)
for g, sh in enumerate(shards):
    x = sh.query(keys)
    own = x != 0xFFFFFFFF
    w[own] = x[own]
    owner[own] = g
bad = np.nonzero(((w & 3) != val) | ((w >> 2) != rem))[0]
print("mismatches", len(bad))
def digits(k):
    out = []
    for h in heaps:
        out.append(int(k % (h + 1)))
        k //= h + 1
    return out
for i in bad[:12]:
    k = int(keys[i])
    d = digits(k)
    print(k, d, "level", sum(heaps) - sum(d), "owner", owner[i], "single", int(val[i]), int(rem[i]),
          "group", int(w[i] & 3), int(w[i] >> 2))
