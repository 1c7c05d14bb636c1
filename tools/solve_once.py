#!/usr/bin/env python3
"""One solve of a game (for profiler passes): python tools/solve_once.py GAME [PARAMS] [LAYOUT]
e.g. toot_and_otto_bitstring "length=6,height=4" hashed.  Prints one JSON line."""
import json
import sys

sys.path.insert(0, ".")


def main():
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    name = sys.argv[1]
    params = sys.argv[2] if len(sys.argv) > 2 else ""
    layout = sys.argv[3] if len(sys.argv) > 3 else "auto"
    s = Solver(GameSpec(name, params), layout=layout)
    r = s.solve()
    print(json.dumps({"game": name, "params": params, "positions": r.positions,
                      "edges": r.edges, "root": r.root_line, "ms_total": r.ms_total,
                      "ms_forward": r.ms_forward, "ms_backward": r.ms_backward}), flush=True)


if __name__ == "__main__":
    main()
