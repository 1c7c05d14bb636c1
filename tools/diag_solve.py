#!/usr/bin/env python3
"""Time solves of the bench shape WITHOUT result checks (kernel-variant
diagnostics built with -DGM_DIAG_SKIP skip loads or stores, so their results
are wrong by construction):  GM_LIBPATH=... python tools/diag_solve.py"""
import json
import os
import sys

sys.path.insert(0, ".")


def main():
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    spec = GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31")
    s = Solver(spec, device="cuda:0")
    ms = []
    for _ in range(3):
        try:
            r = s.solve()
            ms.append(r.ms_total)
        except Exception as e:  # wrong-by-construction variants may fail the root check
            ms.append(str(e)[:60])
    print(json.dumps({"lib": os.environ.get("GM_LIBPATH", "default"), "ms": ms}))


if __name__ == "__main__":
    main()
