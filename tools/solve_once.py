#!/usr/bin/env python3
"""Solves of one game (for profiler passes and A/B timing):
    python tools/solve_once.py GAME [PARAMS] [LAYOUT] [REPEATS] [timing]
e.g. toot_and_otto_bitstring "length=6,height=4" bucketed 3 (env SOLVE_FLAGS:
GM_F_* kernel flags of the solver, e.g. 256 = GM_F_GRAPH).  The first
solve warms up; each later one prints a JSON line (the last with per-kernel
timing and the whole-solve checksum).  REPEATS 0: one solve, printed; with
`timing` it runs with per-kernel timing (one launch per dense level, as the
bench's roofline solve does -- the PMC passes use this form).""" 
import json
import os
import sys
import time

sys.path.insert(0, ".")


def main():
    import torch
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    name = sys.argv[1]
    params = sys.argv[2] if len(sys.argv) > 2 else ""
    layout = sys.argv[3] if len(sys.argv) > 3 else "auto"
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    s = Solver(GameSpec(name, params), layout=layout, flags=int(os.environ.get("SOLVE_FLAGS", "0")))
    if reps == 0 and len(sys.argv) > 5 and sys.argv[5] == "timing":
        s.set_kernel_timing(True)
    for i in range(reps + 1):
        last = i == reps
        if last and reps > 0:
            s.set_kernel_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = s.solve()
        wall = time.perf_counter() - t0
        if i == 0 and reps > 0:
            continue
        out = {"game": name, "params": params, "layout": r.extra["layout"], "positions": r.positions,
               "edges": r.edges, "root": r.root_line, "wall_ms": wall * 1e3, "ms_total": r.ms_total,
               "ms_forward": r.ms_forward, "ms_backward": r.ms_backward}
        if last and reps > 0:
            out.update({"ms_expand_kernels": r.ms_expand_kernels, "ms_resolve_kernels": r.ms_resolve_kernels,
                        "n_expand_launches": r.n_expand_launches, "n_resolve_launches": r.n_resolve_launches,
                        "checksum": s.checksum()})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
