#!/usr/bin/env python3
"""The bench's N-rank sharded workload solved as an in-process group on ONE
GPU (gm_solve_group: all shards' kernels on one stream, halos by device
copies): checks the full-size geometry, memory and closed-form results of
what `bench.py --gpus N` runs one process per GPU, and times it (the time
is the N shards' work serialised on one device, not an N-GPU time).

    python tools/group_bench.py N [steps]
"""
import json
import sys
import time

sys.path.insert(0, ".")


def main():
    world = int(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    import torch
    from bench import expected, heaps_for
    from gamesmanmpi_amd.dist import group_solve
    from gamesmanmpi_amd.games import GameSpec
    heaps = heaps_for(world)
    spec = GameSpec("sum_four_to_one", "heaps=" + ":".join(map(str, heaps)))
    t0 = time.perf_counter()
    r, shards = group_solve(spec, world)
    first = time.perf_counter() - t0
    P, E, root = expected(heaps)
    ok = (r.positions, r.edges, r.root_line.split()[0]) == (P, E, root)
    import ctypes
    from gamesmanmpi_amd import _lib
    arr = (ctypes.c_void_p * world)(*[s.handle.value for s in shards])
    times = []
    for _ in range(steps):
        res = _lib.gm_result()
        torch.cuda.synchronize()
        t = time.perf_counter()
        _lib.check(_lib.load().gm_solve_group(arr, world, ctypes.byref(res)))
        times.append(time.perf_counter() - t)
    print(json.dumps({"world": world, "heaps": heaps, "positions": r.positions,
                      "edges": r.edges, "root": r.root_line, "closed_form_ok": ok,
                      "first_solve_s": round(first, 3),
                      "group_solve_ms": [round(x * 1e3, 2) for x in times],
                      "table_bytes_per_shard": shards[0].plan.table_bytes}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
