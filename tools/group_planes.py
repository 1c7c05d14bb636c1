#!/usr/bin/env python3
"""Device time per shard of the N-GPU bench shape: every shard of
31^5 x (32N-1) solved as ONE in-process group on this GPU (the PLANES shard
kernels, boundary planes copied device-to-device between levels), the same
shards re-solved REPS times; prints one JSON line per solve.  On one GPU the
shards' launches run back to back on one stream, so ms_backward / N is a
shard's device time per level sweep -- what each GPU of an N-GPU run spends
in kernels, before the exchange.
In the staged deal (the default where the last heap splits evenly) the
shards run one after another, so ms_backward / N is one rank's key sweep
with its launch floor; FLAGS 4096 (GM_F_PLANE_LEVEL_SYNC) times the
level-synchronous deal instead.
    python tools/group_planes.py WORLD [REPS] [FLAGS]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, ".")


def main():
    import torch
    import bench
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    world = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    heaps = bench.heaps_for(world)
    spec = GameSpec("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)))
    stream = torch.cuda.Stream()
    shards = [Solver(spec, rank=g, world=world, stream=stream, flags=flags) for g in range(world)]
    arr = (ctypes.c_void_p * world)(*[s.handle.value for s in shards])
    L = _lib.load()
    for i in range(reps + 1):
        r = _lib.gm_result()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(L.gm_solve_group(arr, world, ctypes.byref(r)))
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        res = shards[0]._result(r)
        if i == 0:
            continue  # warm-up
        print(json.dumps({"world": world, "heaps": heaps, "flags": flags, "positions": res.positions, "root": res.root_line,
                          "layout": res.extra.get("layout"), "wall_ms": wall, "ms_forward": res.ms_forward,
                          "ms_backward": res.ms_backward, "ms_backward_per_shard": res.ms_backward / world,
                          "word_bits": res.extra.get("word_bits"),
                          "stage_k": os.environ.get("GM_PLANE_STAGE_K", "default")}), flush=True)


if __name__ == "__main__":
    main()
