#!/usr/bin/env python3
"""Wall / device time of an md5-sharded keyed group solve (every shard of a
W-rank job in this process on one GPU; BUCKETED shards where they apply),
the same shards re-solved REPS times, next to the one-GPU solve:
    python tools/group_keyed_time.py GAME PARAMS WORLD [REPS] [FLAGS]
(FLAGS 16384 = GM_F_BKS_LOCAL: local dedup before the owners)"""
import ctypes
import json
import sys
import time

sys.path.insert(0, ".")


def main():
    import torch
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    from gamesmanmpi_amd.solver import Solver
    game, params, world = sys.argv[1], sys.argv[2], int(sys.argv[3])
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    flags = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    spec = GameSpec(game, params)
    if world == 1:
        s = Solver(spec)
        for i in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = s.solve()
            wall = (time.perf_counter() - t0) * 1e3
            if i:
                print(json.dumps({"world": 1, "layout": r.extra["layout"], "positions": r.positions,
                                  "root": r.root_line, "wall_ms": wall, "ms_forward": r.ms_forward,
                                  "ms_backward": r.ms_backward}), flush=True)
        return
    r, shards = group_keyed_solve(spec, world, flags=flags)
    arr = (ctypes.c_void_p * world)(*[s.handle.value for s in shards])
    L = _lib.load()
    for i in range(reps):
        res = _lib.gm_result()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.device(shards[0].device):
            _lib.check(L.gm_solve_group(arr, world, ctypes.byref(res)))
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        rr = shards[0]._result(res)
        print(json.dumps({"world": world, "flags": flags, "layout": rr.extra["layout"], "positions": rr.positions,
                          "root": rr.root_line, "wall_ms": wall, "ms_forward": rr.ms_forward,
                          "ms_backward": rr.ms_backward}), flush=True)


if __name__ == "__main__":
    main()
