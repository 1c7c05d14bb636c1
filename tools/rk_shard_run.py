#!/usr/bin/env python3
"""toot md5 shards of the RANKED layout as an in-process group on one GPU
(every shard's kernels alone on the GPU when streams="one"): solve REPS
times, print one JSON line per solve.  Under rocprofv3 --kernel-trace this is
the input of tools/rk_shard_model.py.
    python tools/rk_shard_run.py WORLD [PARAMS] [REPS] [STREAMS]"""
import json
import sys
import time

sys.path.insert(0, ".")


def main():
    import torch
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.keyed import group_keyed_solve
    world = int(sys.argv[1])
    params = sys.argv[2] if len(sys.argv) > 2 else "length=6,height=4"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    streams = sys.argv[4] if len(sys.argv) > 4 else "one"
    spec = GameSpec("toot_and_otto_bitstring", params)
    for i in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r, shards = group_keyed_solve(spec, world, layout="ranked", streams=streams)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"world": world, "params": params, "streams": streams, "positions": r.positions,
                          "edges": r.edges, "root": r.root_line, "wall_ms_incl_setup": wall,
                          "ms_forward": r.ms_forward, "ms_backward": r.ms_backward,
                          "stats": [sh.shard_stats() for sh in shards]}), flush=True)
        del shards
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
