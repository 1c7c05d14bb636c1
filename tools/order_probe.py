"""Allocation-order probe: toot 6x4 solve times after a dense
solve or cold.  A script, not a test: run as
    python tools/order_probe.py dense_first|cold
"""
import sys, time, json
sys.path.insert(0, ".")
import torch
from gamesmanmpi_amd.games import GameSpec
from gamesmanmpi_amd.solver import Solver
def toot(tag):
    s = Solver(GameSpec("toot_and_otto_bitstring", "length=6,height=4"))
    out = []
    for i in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter(); r = s.solve(); torch.cuda.synchronize()
        out.append(round((time.perf_counter() - t0) * 1e3, 1))
    print(tag, out, r.extra["layout"], flush=True)
    del s; torch.cuda.empty_cache()
def main():
    if sys.argv[1] == "dense_first":
        d = Solver(GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31"))
        for i in range(5): d.solve()
        del d; torch.cuda.empty_cache()
    toot(sys.argv[1])
    toot(sys.argv[1] + "_again")


if __name__ == "__main__":
    main()
