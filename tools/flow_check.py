#!/usr/bin/env python3
"""The one-launch PLANES backward (k_plane_flow) against the per-level
launches (GM_F_PLANE_LEVELS) word for word on a few shapes, several solves
each: which planes (outer digits) differ.  Diagnostic tool."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")


def main():
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    shapes = sys.argv[1:] or ["heaps=31:31:1:127", "heaps=31:31:3:63", "heaps=31:31:127", "heaps=31:31:7:7"]
    for params in shapes:
        spec = GameSpec("sum_four_to_one", params)
        ref = Solver(spec, layout="planes", flags=_lib.GM_F_PLANE_LEVELS)
        ref.solve()
        keys = ref.positions()
        want = ref.query(keys)
        s = Solver(spec, layout="planes")
        heaps = [int(h) for h in params.split("=")[1].split(":")]
        for rep in range(int(os.environ.get("REPS", "4"))):
            if os.environ.get("POISON"):  # a stale or early read of a neighbour row shows
                import torch
                s._tensors[0][:s.plan.table_slots].fill_(0xAA)
                torch.cuda.synchronize()
            r = s.solve()
            got = s.query(keys)
            bad = np.nonzero(got != want)[0]
            planes = sorted({int(k) // 1024 for k in keys[bad]})
            print(params, "rep", rep, r.extra["resolve_kernel"], "bad words", len(bad), "planes", len(planes),
                  planes[:12], flush=True)
        del s, ref


if __name__ == "__main__":
    main()
