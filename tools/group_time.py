#!/usr/bin/env python3
"""Wall time of an in-process group solve (dist.group_solve: every shard of
the N-GPU bench shape on this one GPU, one stream), to compare the per-shard
kernels with the one-table solve:  python tools/group_time.py WORLD [REPS]"""
import json
import sys
import time

sys.path.insert(0, ".")


def main():
    import torch
    import bench
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    world = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    heaps = bench.heaps_for(world)
    spec = GameSpec("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)))
    for i in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r, shards = group_solve(spec, world)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"world": world, "positions": r.positions, "root": r.root_line, "wall_ms": wall,
                          "ms_total": r.ms_total, "ms_forward": r.ms_forward, "ms_backward": r.ms_backward,
                          "word_bits": r.extra.get("word_bits"), "kernels": r.extra.get("kernels")}), flush=True)
        del shards


if __name__ == "__main__":
    main()
