#!/usr/bin/env python3
"""Benchmark: positions solved per second on the synthetic sum-of-Four-To-One
state space (BASELINE.json config 4).

A "step" is one complete strong solve from the root: table reset, forward
expansion of every level, retrograde pass of every level, root word back on
the host.  N=1 workload: heaps 31^6 = 2^30 = 1,073,741,824 positions,
187 levels, 12,280,922,112 edges.  For N>1 (one process per GPU, launched by
torch.distributed.run) the heaps are 31^5 x (32N-1): 2^30 positions per
GPU; the ranks split the last heap's values into blocks of 8 dealt round
robin and exchange two boundary slices per block and level over RCCL
(DESIGN.md §Multi-GPU).  Every step's counts and root value
are checked against closed forms; a wrong solve aborts the run.

Prints ONE JSON line (rank 0).  Fields beyond the driver contract:
  roofline      dominant kernel's algorithmic bytes per launch / its
                HIP-event-timed average duration, vs 8 TB/s; traffic from
                the committed PMC passes
  cpu_baseline  the oracle (oracle/, one core) on a bounded sample of the
                same game family, timed on this host
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)


def heaps_for(world):
    """Weak scaling, 2^30 positions per GPU: heaps 31^5 x (32N - 1).  N=1 is
    SURVEY §8d's 31^6 (2^30 positions, 187 levels, b = 11.4375).  The ranks
    split the last heap into blocks of 8 values dealt round robin, four per
    rank (round robin keeps the ranks' per-level work
    within 1.11 / 1.19 / 1.41x of the mean at N = 2 / 4 / 8; one contiguous
    block of 32 per rank would give 1.51 / 2.53 / 4.58x)."""
    if world not in (1, 2, 4, 8):
        raise SystemExit("--gpus must be 1, 2, 4 or 8")
    return [31] * 5 + [32 * world - 1]


def expected(heaps):
    """Closed forms the solve must reproduce: positions = prod(h+1);
    edges = sum_i P*(2h_i - 1)/(h_i + 1) (a heap h >= 2 has moves -1,-2, a
    heap of 1 only -1); root value by Sprague-Grundy: each heap is the
    subtraction game {1,2} with Grundy value h mod 3, so the root is a LOSS
    iff the XOR of (h_i mod 3) is 0."""
    P = 1
    for h in heaps:
        P *= h + 1
    E = sum(P * (2 * h - 1) // (h + 1) for h in heaps if h >= 1)
    g = 0
    for h in heaps:
        g ^= h % 3
    return P, E, ("LOSS" if g == 0 else "WIN")


def algorithmic_bytes(positions, edges, layout, word_bytes=4):
    """Bytes each kernel family must move, per DESIGN.md §Roofline.
    hashed (SURVEY §8d keyed model): expand 24 B/position + 8 B/edge,
      resolve 12 B/position + 12 B/edge (8-B keys, 4-B value words).
    dense (level-major perfect hash, key implicit in the slot):
      pull: one reach bit per parent link + one written bit per position
            = (edges + positions) / 8 B (parent links = edges);
      resolve: own reach bit + one word written per position, one child
            word per edge = 4.125 B/position + 4 B/edge with 32-bit words,
            2.125 B/position + 2 B/edge with the 16-bit table (word_bytes 2,
            DESIGN.md §3: K_SUM remoteness < 2^15)."""
    if layout == "dense":
        return ((edges + positions) / 8.0,
                (word_bytes + 0.125) * positions + word_bytes * edges)
    return 24 * positions + 8 * edges, 12 * positions + 12 * edges


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py --traffic
    from separate rocprofv3 --pmc passes of this bench), or None when no
    pass of this workload is recorded."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            row = json.load(fh).get(kernel)
    except (OSError, ValueError):
        return None, None
    if not row or row.get("workload") != workload:
        return None, None
    return row["bytes_per_launch"], "profiles/pmc_traffic.json (%s)" % row.get("source", "?")


def dense_resolve_kernel(word_bits, world=1):
    """Name of the dense resolve kernel the library launches for the bench
    shape (power-of-two heaps, base >= 8): over the live-group lists, the
    software-pipelined eight-prefixes-per-lane form on the 16-bit table (the
    solve reports word_bits 16), else the four-prefixes-per-lane form, unless
    the A/B knobs (GM_DENSE_RESOLVE / GM_DENSE_SWEEP / GM_DENSE_PIPE) select
    another."""
    if word_bits == 16:
        return "k_dense_resolve8p" if world == 1 else "k_dense_resolve8c"
    if os.environ.get("GM_DENSE_RESOLVE") == "scalar":
        return "k_dense_resolve"
    sweep = os.environ.get("GM_DENSE_SWEEP", "list")
    if sweep == "cols":
        return "k_dense_resolve4c"
    if sweep == "walk":
        return "k_dense_resolve4w"
    if os.environ.get("GM_DENSE_PIPE") == "0":
        return "k_dense_resolve4"
    return "k_dense_resolve4p"


def model_8d_bytes(positions, edges):
    """SURVEY §8d per-position figure 36 + 20*b (whole solve)."""
    return 36 * positions + 20 * edges


def cpu_baseline(sample_heaps="31:31:31:31:31"):
    """Oracle (one core, scalar C port) on a bounded sample: the same game
    family at 2^25 positions (about 10-20 s)."""
    from oracle.oracle import Game
    g = Game("sum_four_to_one", "heaps=" + sample_heaps)
    t0 = time.perf_counter()
    sol = g.solve(1 << 25)
    dt = time.perf_counter() - t0
    return {"value": sol.count / dt, "unit": "positions/s", "cores": 1,
            "kind": "port",
            "sample": "oracle/ scalar C retrograde, sum_four_to_one heaps=%s "
                      "(%d positions, %d edges, root %s), %.2f s"
                      % (sample_heaps, sol.count, sol.edges, sol.root_line, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--heaps", default=None,
                    help="override the synthetic heaps, e.g. 31:31:31:31")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--layout", default="auto", choices=["auto", "dense", "hashed"])
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver

    heaps = [int(h) for h in args.heaps.split(":")] if args.heaps else heaps_for(world)
    params = "heaps=" + ":".join(str(h) for h in heaps)
    spec = GameSpec("sum_four_to_one", params)
    if world > 1:
        from gamesmanmpi_amd.dist import ShardedSolver
        solver = ShardedSolver(spec, rank, world, device="cuda:%d" % local)
    else:
        solver = Solver(spec, device="cuda:%d" % local, layout=args.layout)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        solver.solve()
    barrier()
    t0 = time.perf_counter()
    results = []
    for _ in range(args.steps):
        results.append(solver.solve())
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    r = results[-1]
    layout = r.extra["layout"]
    # whole-job position count: sharded results are already summed over ranks
    positions_total = r.positions if world > 1 else r.positions
    P, E, root_value = expected(heaps)
    for x in results:
        if (x.positions, x.edges) != (P, E) or x.root_line.split()[0] != root_value:
            raise SystemExit("WRONG RESULT: %d positions, %d edges, %s; expected %d, %d, %s"
                             % (x.positions, x.edges, x.root_line, P, E, root_value))

    # roofline of the dominant kernel: one extra solve with HIP events
    # around every launch, on the stream the kernels run on
    solver.set_kernel_timing(True)
    tr = solver.solve()
    solver.set_kernel_timing(False)
    if world > 1:
        tr_pos, tr_edges = tr.positions // world, tr.edges // world  # per GPU
    else:
        tr_pos, tr_edges = tr.positions, tr.edges
    word_bits = tr.extra.get("word_bits", 32) or 32
    fwd_b, bwd_b = algorithmic_bytes(tr_pos, tr_edges, layout, word_bits // 8)
    if tr.ms_resolve_kernels >= tr.ms_expand_kernels:
        kname, kb, kms, kn = (dense_resolve_kernel(word_bits, world) if layout == "dense"
                              else "k_resolve", bwd_b, tr.ms_resolve_kernels,
                              tr.n_resolve_launches)
    else:
        kname, kb, kms, kn = ("k_dense_pull" if layout == "dense"
                              else "k_expand", fwd_b, tr.ms_expand_kernels,
                              tr.n_expand_launches)
    achieved = (kb / kn) / (kms / kn / 1e3) / 1e9  # GB/s
    workload = "sum_four_to_one heaps=%s" % ":".join(map(str, heaps))
    traffic, traffic_src = pmc_traffic(kname, workload)
    line = {
        "metric": "positions solved/sec (node)",
        "value": positions_total * args.steps / elapsed,
        "unit": "positions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64 keys / u%d words (integer)" % word_bits,
        "data": "synthetic: sum of Four-To-One heaps, fully determined state space",
        "config": {"workload": workload,
                   "positions_per_gpu": r.positions // world, "edges_per_gpu": r.edges // world,
                   "levels": r.levels, "root": r.root_line,
                   "layout": layout,
                   "parallelism": ("round-robin top-heap blocks x%d, RCCL halo exchange" % world
                                   if world > 1 else "1 GPU")},
        "roofline": {"bound": "hbm", "kernel": kname,
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": kb / kn,
                     "model": ("dense: resolve %.3f B/position + %d B/edge (%d-bit words), pull (edges + positions)/8 B"
                               % (word_bits / 8 + 0.125, word_bits // 8, word_bits)
                               if layout == "dense" else
                               "SURVEY 8d keyed: expand 24 B/position + 8 B/edge, resolve 12 B/position + 12 B/edge"),
                     "launches": kn, "ms_kernel_total": kms,
                     "ms_per_launch": kms / kn,
                     "algorithmic_bytes_total": kb},
        "phase_ms": {"forward": r.ms_forward, "backward": r.ms_backward,
                     "solve_wall": r.ms_total,
                     "expand_kernels": tr.ms_expand_kernels,
                     "resolve_kernels": tr.ms_resolve_kernels},
        "model_8d": {"bytes_per_position": model_8d_bytes(r.positions, r.edges) / r.positions,
                     "equiv_GBps_per_gpu": model_8d_bytes(r.positions, r.edges) / world
                     * args.steps / elapsed / 1e9,
                     "frac_of_peak": model_8d_bytes(r.positions, r.edges) / world
                     * args.steps / elapsed / 1e9 / HBM_PEAK_GBS},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
