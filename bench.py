#!/usr/bin/env python3
"""Benchmark: positions solved per second on the synthetic sum-of-Four-To-One
state space (BASELINE.json config 4).

A "step" is one complete strong solve from the root: state reset, forward
expansion of every level, retrograde pass of every level, root word back on
the host.  N=1 workload: heaps 31^6 = 2^30 = 1,073,741,824 positions,
187 levels, 12,280,922,112 edges.  For N>1 (one process per GPU, launched by
torch.distributed.run) the heaps are 31 x (32N-1) x 31^4: 2^30 positions per
GPU (the game is symmetric in its heaps: the same state space as
31^5 x (32N-1) with the long heap second); rank r holds heap-1 values
[32r, 32r + 32) of every plane -- the one-GPU table's planes and levels -- and
streams each level's last two rows to rank r + 1 over RCCL, which needs them
for that level only (the row deal).  Every step's counts, root value AND root remoteness are
checked: counts and value by closed forms, the remoteness against the
CPU restatement's solve of the same workload (tests/golden/checksums.json,
or this run's cpu_baseline).

Prints ONE JSON line (rank 0).  Fields beyond the driver contract:
  roofline      dominant kernel, HIP-event-timed average launch duration;
                achieved/frac on the bytes the layout must move (compulsory:
                own words written, live words of the two child rows read once,
                reach bits), plus frac_pmc (HBM bytes the counters saw,
                profiles/pmc_traffic.json) and frac_per_edge_model (one child
                word read per edge, the round-1 figure) -- DESIGN.md §5
  keyed         BASELINE config 3 as shipped (toot 6x4, 1.19e9 positions) on
                the layout the planner picks (RANKED: positions at computed
                indices) and, as "bucketed", on the keyed BUCKETED levels:
                solve time, positions/s, per-pass bytes and rates (the
                layout's compulsory bytes; §8d's keyed-table model),
                fingerprint parity vs the CPU restatement
  cpu_baseline  the multi-threaded CPU restatement (oracle/oracle_mt.c row
                solver, all host threads) on the SAME workload
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
QDEPTH = 4  # queued one-table solves outstanding in the timed loop (the library allows 8)


def heaps_for(world):
    """Weak scaling, 2^30 positions per GPU: heaps 31 x (32N - 1) x 31^4.  N=1
    is SURVEY §8d's 31^6 (2^30 positions, 187 levels, b = 11.4375).  The long
    heap is heap 1, the planes' row axis: rank r owns its values
    [32r, 32r + 32), i.e. a 32 x 32 slab of every plane -- each rank's table
    is the one-GPU table -- and the only cross-rank edge is rows 0, 1 reading
    rank r - 1's rows 30, 31 of the same plane (round 4 split
    the LAST heap in blocks of 32 and trailed by a block of keys per rank)."""
    if world not in (1, 2, 4, 8):
        raise SystemExit("--gpus must be 1, 2, 4 or 8")
    return [31] * 6 if world == 1 else [31, 32 * world - 1] + [31] * 4


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


def level_counts(heaps):
    """Positions per level (level L = root_sum - digit sum): coefficients of
    prod_i (1 + x + ... + x^h_i), reversed."""
    c = [1]
    for h in heaps:
        n = [0] * (len(c) + h)
        for i, v in enumerate(c):
            for j in range(h + 1):
                n[i + j] += v
        c = n
    return c[::-1]


def dense_bytes(heaps, word_bytes):
    """Per-solve byte models of the dense layout.
    compulsory -- what any schedule of this layout must move from HBM:
      resolve(L): own words written + the live words of rows L+1 and L+2
                  read once + own reach bits = (3w + 1/8) B per position;
      pull(L):    own reach bits written + rows L-1, L-2 read = 3/8 B.
    per_edge -- the round-1 model: one child word per edge (2.125 B/position
      + 2 B/edge at w = 2), which counts L2/MALL hits as HBM bytes."""
    n = level_counts(heaps)
    T = len(n)
    res = pull = 0.0
    for L in range(T):
        nx = lambda k: n[k] if 0 <= k < T else 0  # noqa: E731
        res += word_bytes * (n[L] + nx(L + 1) + nx(L + 2)) + n[L] / 8.0
        pull += (n[L] + nx(L - 1) + nx(L - 2)) / 8.0
    P, E, _ = expected(heaps)
    return {"resolve_compulsory": res, "pull_compulsory": pull,
            "resolve_per_edge": (word_bytes + 0.125) * P + word_bytes * E,
            "pull_per_edge": (E + P) / 8.0}


def plane_bytes(heaps, word_bytes):
    """Per-solve byte models of the PLANES layout (planes of
    32 x 32 positions, plane level l = sum of the outer heaps 2..K-1).
    compulsory -- what any schedule of this layout must move from HBM:
      resolve(l): the level's own planes written + the planes of levels l-1
                  and l-2 (its children's planes) read once
                  = w KiB x (n(l) + n(l-1) + n(l-2));
      reach:      one bit per 32-position row written (a reached row holds
                  every h0 up to the start: gm_plane.h plane_reach_body).
    requested -- what the kernel asks of the memory system: own plane
      written + every neighbour plane row read (one per outer heap and move
      that exists), L2 / Infinity-Cache hits included."""
    outer = heaps[2:]
    n = [1]
    for h in outer:
        m = [0] * (len(n) + h)
        for i, v in enumerate(n):
            for j in range(h + 1):
                m[i + j] += v
        n = m
    pb = 1024 * word_bytes
    nx = lambda k: n[k] if 0 <= k < len(n) else 0  # noqa: E731
    comp = sum(pb * (n[l] + nx(l - 1) + nx(l - 2)) for l in range(len(n)))
    planes = 1
    for h in outer:
        planes *= h + 1
    nbr = sum(planes * sum(min(v, 2) for v in range(h + 1)) // (h + 1) for h in outer)
    P = planes * 1024
    return {"resolve_compulsory": comp, "resolve_requested": pb * (planes + nbr),
            "pull_compulsory": P / 256.0, "pull_requested": P / 256.0, "launches": len(n)}


def keyed_bytes(positions, edges):
    """SURVEY §8d algorithmic bytes of the keyed table: expand 24 B/position
    + 8 B/edge, resolve 12 B/position + 12 B/edge (8-B keys, 4-B words)."""
    return 24 * positions + 8 * edges, 12 * positions + 12 * edges


def _kernel_sources_sha16():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from pmc_summary import kernel_sources_sha16
        return kernel_sources_sha16(ROOT)
    except (ImportError, OSError):
        return None
    finally:
        sys.path.pop(0)


def _kernel_code_sha16(kernel):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        from codeobj import kernel_code_sha16
        return kernel_code_sha16(os.path.join(ROOT, "gamesmanmpi_amd", "libgamesman_hip.so"), kernel)
    except ImportError:
        return None
    finally:
        sys.path.pop(0)


def _pmc_row(kernel, workload, path=None):
    """The committed PMC summary's row for `kernel` (profiles/pmc_traffic.json,
    tools/pmc_summary.py --traffic over separate rocprofv3 --pmc passes of
    this bench) and a note: None when no pass of this workload and kernel is
    recorded, or when the kernel's machine code changed since the passes ran
    (the counters describe other code: rerun tools/gpu_session.sh TAG pmc).
    The key is the measured kernel's own gfx950 code (tools/codeobj.py), so
    host-side edits and other kernels leave the figure valid; rows written
    before that key existed fall back to the kernel-source hash."""
    path = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            row = json.load(fh).get(kernel)
    except (OSError, ValueError):
        return None, None
    if not row or row.get("workload") != workload:
        return None, None
    rel = os.path.relpath(path, ROOT)
    if "kernel_code_sha16" in row:
        now = _kernel_code_sha16(kernel)
        if not now or row["kernel_code_sha16"] != now:
            return None, "stale: %s (%s) measured %s code %s, this library's is %s" % (
                rel, row.get("source", "?"), kernel, row["kernel_code_sha16"], now)
        return row, "%s (%s, %s code %s)" % (rel, row.get("source", "?"), kernel, now)
    now = _kernel_sources_sha16()
    if row.get("kernel_sources_sha16") != now:
        return None, "stale: profiles/pmc_traffic.json (%s) measured kernel sources %s, these are %s" % (
            row.get("source", "?"), row.get("kernel_sources_sha16"), now)
    return row, "profiles/pmc_traffic.json (%s, kernel sources %s)" % (row.get("source", "?"), now)


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed PMC summary, or
    None (see _pmc_row), and where the figure comes from."""
    row, note = _pmc_row(kernel, workload)
    return (row["bytes_per_launch"] if row else None), note


def pmc_traffic_total(kernel, workload):
    """(HBM bytes per launch, launches per solve) of `kernel` from the
    committed PMC summary, or (None, 0)."""
    row, _ = _pmc_row(kernel, workload)
    if not row:
        return None, 0
    return row["bytes_per_launch"], row.get("launches", 0)


def planes_traffic(kernel, workload):
    """PLANES backward HBM bytes per launch: the PMC bytes of `kernel` and of
    the one-workgroup runs (k_plane_run) over all their launches in the PMC
    pass -- a launch-weighted mean, whatever number of solves the pass held --
    or None."""
    rows = [r for r in (pmc_traffic_total(k, workload) for k in (kernel, "k_plane_run")) if r[0] and r[1]]
    if not rows:
        return None
    return sum(b * n for b, n in rows) / sum(n for _, n in rows)


def ranked_pmc(words):
    """The RANKED kernels' counter bytes per solve from the committed PMC
    passes of one toot 6x4 solve (profiles/pmc_ranked.json, tools/pmc_ranked.sh
    + tools/pmc_summary.py --traffic), each only while the kernel's gfx950
    code is the one measured; the backward's write bytes against the words it
    produces (one byte per reached position)."""
    path = os.path.join(ROOT, "profiles", "pmc_ranked.json")
    res = {}
    for k in ("k_rk_backward", "k_rk_reach4", "k_rk_boards_sl"):
        row, note = _pmc_row(k, "toot_and_otto_bitstring length=6,height=4", path)
        if not row:
            res[k] = {"source": note}
            continue
        n = row.get("launches", 0)
        res[k] = {"fetch_bytes_per_solve": row["fetch_bytes_per_launch"] * n,
                  "write_bytes_per_solve": row["write_bytes_per_launch"] * n,
                  "l2_hit_rate": row.get("l2_hit_rate"), "launches": n, "source": note}
    b = res["k_rk_backward"]
    if "write_bytes_per_solve" in b:
        b["write_bytes_over_words_produced"] = b["write_bytes_per_solve"] / words
    return res


def golden(name):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "checksums.json")) as fh:
            return json.load(fh).get(name)
    except (OSError, ValueError):
        return None


def golden_for_params(game, params):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "checksums.json")) as fh:
            data = json.load(fh)
    except (OSError, ValueError):
        return None
    for e in data.values():
        if e.get("game") == game and e.get("params") == params:
            return e
    return None


def cpu_baseline(params):
    """The multi-threaded CPU restatement (oracle_mt.c row solver, every
    OpenMP thread of this host) on the same workload: solve time only
    (reachability + retrograde of every position)."""
    from oracle.oracle import Game, threads
    g = Game("sum_four_to_one", params)
    t0 = time.perf_counter()
    sol = g.solve_rows()
    dt = time.perf_counter() - t0
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 0
    omp = os.environ.get("OMP_NUM_THREADS")
    why = ("OMP_NUM_THREADS=%s, set by the GPU box's environment as this job's CPU share "
           "(the harness asks that it be left as is)" % omp) if omp else "every CPU the process may run on"
    out = {"value": sol.count / dt, "unit": "positions/s", "cores": threads(),
           "kind": "port",
           "sample": "full workload: oracle/oracle_mt.c row solver (OpenMP, %d threads = %s; host nproc %d, "
                     "CPUs in this process's affinity mask %d), sum_four_to_one %s: %d positions, %d edges, "
                     "root %s, %.2f s.  For scale: the reference's own Python job loop solves mttt (5,478 "
                     "positions) at ~84 positions/s on one core (SURVEY.md section 6)"
                     % (threads(), why, os.cpu_count() or 0, allowed, params, sol.count, sol.edges,
                        sol.root_line, dt)}
    return out, sol.root_line


def keyed_atomics():
    """Atomic operations of the keyed solve (north_star: "rocprof must show
    ... atomic throughput"), from the committed counter passes
    (tools/pmc_atomics.sh -> profiles/keyed_atomics.json): L2 atomic requests
    and LDS atomic wave-instructions per solve and per second of kernel
    time, with a reference rate; None when absent or measured on other
    kernel sources."""
    path = os.path.join(ROOT, "profiles", "keyed_atomics.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        try:
            from pmc_atomics_summary import sources_sha16
            now = sources_sha16(ROOT)
        finally:
            sys.path.pop(0)
    except (OSError, ValueError, ImportError):
        return None
    if d.get("sources_sha16") != now:
        return {"stale": "profiles/keyed_atomics.json measured sources %s, these are %s" % (d.get("sources_sha16"), now)}
    t = d["total"]
    top = sorted(d["kernels"].items(), key=lambda kv: -(kv[1].get("l2_atomic_requests", 0) + kv[1].get("lds_atomic_insts", 0)))
    return {"source": "profiles/keyed_atomics.json (%s)" % d.get("source"),
            "l2_atomic_requests": t["l2_atomic_requests"], "l2_atomic_per_s": t.get("l2_atomic_per_s"),
            "lds_atomic_insts": t["lds_atomic_insts"], "lds_atomic_insts_per_s": t.get("lds_atomic_insts_per_s"),
            "reference": "memory-side atomics ~5e9 wave-instructions/s chip-wide (1.3 TB/s, MI355X_MICROARCH.md); "
                         "one L2 atomic request = one 64-B piece",
            "by_kernel": {k: {"l2": v.get("l2_atomic_requests"), "lds": v.get("lds_atomic_insts"),
                              "ms": v.get("kernel_ms")} for k, v in top[:6]}}


def ranked_bytes(nslots, positions, edges):
    """Compulsory bytes of the RANKED layout (gm_ranked.h): forward -- the
    per-board primitive byte and the reach + expandable bits of every slot
    written; backward -- the reach bits read, per reached position its board
    byte read and its word written, per edge the child's word read."""
    return nslots // 8 * 3, nslots // 8 + 2 * positions + edges


def _keyed_solve(device, layout):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    import torch
    params = "length=6,height=4"
    s = Solver(GameSpec("toot_and_otto_bitstring", params), device=device, layout=layout)
    s.solve()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = s.solve()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    s.set_kernel_timing(True)
    tr = s.solve()
    s.set_kernel_timing(False)
    lay = r.extra["layout"]
    fwd_b, bwd_b = keyed_bytes(r.positions, r.edges)
    out = {"workload": "toot_and_otto_bitstring " + params,
           "layout": lay,
           "positions": r.positions, "edges": r.edges, "root": r.root_line,
           "solve_ms": wall * 1e3, "positions_per_s": r.positions / wall,
           "ms_forward": r.ms_forward, "ms_backward": r.ms_backward,
           "kernels": {}}
    # the bytes each pass must move: SURVEY §8d's keyed-table model, or for
    # RANKED the layout's own compulsory bytes (no keys, no dedup)
    if lay == "ranked":
        fb, bb = ranked_bytes(int(s.plan.table_slots), r.positions, r.edges)
        model = "ranked_bytes"
    else:
        fb, bb, model = fwd_b, bwd_b, "model_8d_bytes"
    names = ("expand", "resolve") if lay == "hashed" else ("forward", "backward")
    for name, b, ms, n in ((names[0], fb, tr.ms_expand_kernels, tr.n_expand_launches),
                           (names[1], bb, tr.ms_resolve_kernels, tr.n_resolve_launches)):
        if n and ms > 0:
            out["kernels"][name] = {"launches": n, "ms_total": ms, model: b,
                                    "achieved_GBps": b / (ms / 1e3) / 1e9,
                                    "frac": b / (ms / 1e3) / 1e9 / HBM_PEAK_GBS}
    if lay == "ranked":
        out["pmc"] = ranked_pmc(r.positions)
    # the whole solve against its own layout's bytes; for RANKED, SURVEY
    # §8d's keyed-table bytes (work it does NOT do: no keys are moved) only as
    # an equivalent rate comparable with the keyed layouts, never as a
    # roofline fraction (it exceeded 1)
    if lay == "ranked":
        out["ranked_frac_whole_solve"] = (fb + bb) / wall / 1e9 / HBM_PEAK_GBS
        out["keyed_equiv_GBps"] = (fwd_b + bwd_b) / wall / 1e9
    else:
        out["model_8d_frac_whole_solve"] = (fwd_b + bwd_b) / wall / 1e9 / HBM_PEAK_GBS
    e = golden("toot_6x4")
    if e is not None:
        ck = s.checksum()
        out["parity"] = {"vs": "tests/golden/checksums.json toot_6x4 (oracle_mt)",
                         "checksum": ck["checksum"],
                         "ok": (ck["checksum"] == e["checksum"] and r.positions == e["positions"]
                                and r.edges == e["edges"] and r.root_line == e["root_line"])}
    del s
    torch.cuda.empty_cache()
    return out


def keyed_record(device):
    """BASELINE config 3 as shipped: toot_and_otto_bitstring 6x4 on the
    layout the planner picks (RANKED: positions at computed indices), and on
    the keyed BUCKETED levels (what every keyed game without a rank function
    runs, othello included) as a sub-record; each: one warm-up solve, one
    timed, one with kernel timing, fingerprint vs tests/golden/checksums.json."""
    out = _keyed_solve(device, "auto")
    if out["layout"] != "bucketed":
        b = _keyed_solve(device, "bucketed")
        b["atomics"] = keyed_atomics()
        out["bucketed"] = b
    else:
        out["atomics"] = keyed_atomics()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--heaps", default=None,
                    help="override the synthetic heaps, e.g. 31:31:31:31")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-keyed", action="store_true",
                    help="skip the toot 6x4 keyed-table sub-record")
    ap.add_argument("--layout", default="auto", choices=["auto", "planes", "dense", "hashed"])
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="N>1 halo exchange: RCCL (one GPU per rank), or host-staged over "
                         "gloo -- every rank on cuda:0, for rehearsing the N-rank bench on "
                         "one GPU (not a performance path)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    host = args.transport == "host"
    if host:
        local = 0  # every rank on the one GPU
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if host:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver

    heaps = [int(h) for h in args.heaps.split(":")] if args.heaps else heaps_for(world)
    params = "heaps=" + ":".join(str(h) for h in heaps)
    spec = GameSpec("sum_four_to_one", params)
    if world > 1:
        from gamesmanmpi_amd.dist import ShardedSolver
        solver = ShardedSolver(spec, rank, world, device="cuda:%d" % local,
                               transport="host" if host else "rccl")
    else:
        solver = Solver(spec, device="cuda:%d" % local, layout=args.layout)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    warm = None
    for _ in range(args.warmup):
        warm = solver.solve()
    # one-table PLANES: the K solves are QUEUED (gm_solver_solve_async, at
    # most QDEPTH outstanding) so they run back to back on the GPU with no
    # host round trip between them; each one is still a whole solve of its
    # own, collected and checked below (other layouts: plain solve() calls)
    queued = (world == 1 and warm is not None and warm.extra.get("layout") == "planes"
              and hasattr(solver, "solve_async"))
    barrier()
    t0 = time.perf_counter()
    results = []
    if queued:
        tickets = []
        for _ in range(args.steps):
            if len(tickets) == QDEPTH:
                results.append(solver.collect(tickets.pop(0)))
            tickets.append(solver.solve_async())
        for t in tickets:
            results.append(solver.collect(t))
    else:
        for _ in range(args.steps):
            results.append(solver.solve())
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if host else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    r = results[-1]
    layout = r.extra["layout"]
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
    word_bits = tr.extra.get("word_bits", 32) or 32
    workload = "sum_four_to_one heaps=%s" % ":".join(map(str, heaps))
    if layout == "planes":
        m = plane_bytes(heaps, word_bits // 8)
        # plane_bytes counts 32 x 32 planes over the outer heaps: per rank
        # already when heap 1 is the dealt one (the row deal), the whole job
        # when the last heap is
        div = world if heaps[1] == 31 else 1
        model = {"resolve_compulsory": m["resolve_compulsory"] / div,
                 "pull_compulsory": m["pull_compulsory"] / div,
                 "resolve_per_edge": m["resolve_requested"] / div,
                 "pull_per_edge": m["pull_requested"] / div}
        resolve_k, pull_k = tr.extra.get("resolve_kernel", "?"), tr.extra.get("pull_kernel", "?")
    elif layout == "dense":
        model = dense_bytes(heaps if world == 1 else heaps[:-1] + [(heaps[-1] + 1) // world - 1],
                            word_bits // 8)
        resolve_k, pull_k = tr.extra.get("resolve_kernel", "?"), tr.extra.get("pull_kernel", "?")
    else:
        fwd, bwd = keyed_bytes(tr.positions // world, tr.edges // world)
        model = {"resolve_compulsory": bwd, "pull_compulsory": fwd,
                 "resolve_per_edge": bwd, "pull_per_edge": fwd}
        resolve_k, pull_k = "k_resolve", "k_expand"
    if tr.ms_resolve_kernels >= tr.ms_expand_kernels:
        kname, kb, ke, kms, kn = (resolve_k, model["resolve_compulsory"], model["resolve_per_edge"],
                                  tr.ms_resolve_kernels, tr.n_resolve_launches)
    else:
        kname, kb, ke, kms, kn = (pull_k, model["pull_compulsory"], model["pull_per_edge"],
                                  tr.ms_expand_kernels, tr.n_expand_launches)
    t_launch = kms / kn / 1e3  # seconds per launch
    achieved = (kb / kn) / t_launch / 1e9  # GB/s
    traffic, traffic_src = pmc_traffic(kname, workload)
    if layout == "planes" and traffic is not None:
        # the backward's launches are this kernel plus the one-workgroup runs
        # of narrow levels (k_plane_run): their PMC bytes over all of them,
        # per launch (the PMC pass may hold several solves: weight by its own
        # launch counts, not by this solve's)
        traffic = planes_traffic(kname, workload) or traffic
    roof = {"bound": "hbm", "kernel": kname,
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_unit": "HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE; PLANES: over the backward's "
                            "grid launches and one-workgroup runs together)",
            "traffic_source": traffic_src,
            "frac_pmc": (traffic / t_launch / 1e9 / HBM_PEAK_GBS) if traffic else None,
            "frac_per_edge_model": (ke / kn) / t_launch / 1e9 / HBM_PEAK_GBS,
            "algorithmic_bytes_per_launch": kb / kn,
            "per_edge_model_bytes_per_launch": ke / kn,
            "model": ({"planes": "compulsory bytes of the PLANES layout: per plane level, the level's own "
                                 "%d-bit words written + the planes of the two child levels read once "
                                 "(w KiB x (n(l) + n(l-1) + n(l-2)) per launch); frac_per_edge_model = every "
                                 "neighbour-plane row the kernel requests (L2/MALL hits included)" % word_bits,
                       "dense": "compulsory bytes of the dense layout: resolve (3w + 1/8) B per position "
                                "(own %d-bit word written, live words of rows L+1 and L+2 read once, reach "
                                "bit); pull 3/8 B per position" % word_bits}.get(
                          layout, "SURVEY 8d keyed: expand 24 B/position + 8 B/edge, resolve 12 B/position + "
                                  "12 B/edge")),
            "timing": ("HIP events on the solve stream in an extra solve of the same launch schedule: "
                       + ("one event pair around the whole backward, ONE launch of k_plane_flow (every plane "
                          "level; planes wait for their neighbours by ready flags, gm_plane.h)"
                          if layout == "planes" and world == 1 and kname == "k_plane_flow" else
                          "one event pair around the whole backward (nothing but its %d resolve launches: "
                          "grid-wide k_plane_resolve* for wide plane levels, one-workgroup k_plane_run for runs "
                          "of narrow ones), average = span / launches" % kn if layout == "planes" and world == 1
                          else "one event pair around this rank's whole staged backward (%d launches over its "
                          "keys, halo waits included), average = span / launches" % kn if layout == "planes"
                          else "an event pair around each launch, summed")),
            "launches": kn, "ms_kernel_total": kms, "ms_per_launch": kms / kn,
            "algorithmic_bytes_total": kb}

    # root remoteness: the CPU restatement's solve of the same workload
    root_ref, root_src = None, None
    g = golden_for_params("sum_four_to_one", params)
    if g is not None:
        root_ref, root_src = g["root_line"], "tests/golden/checksums.json (oracle_mt)"
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, cpu_root = cpu_baseline(params)
        if root_ref is None:
            root_ref, root_src = cpu_root, "cpu_baseline (oracle_mt) of this run"
        elif cpu_root != root_ref:
            raise SystemExit("CPU restatement disagrees with its golden: %s vs %s" % (cpu_root, root_ref))
    if root_ref is not None:
        for x in results + [tr]:
            if x.root_line != root_ref:
                raise SystemExit("WRONG ROOT: %s, the CPU restatement gives %s" % (x.root_line, root_ref))

    line = {
        "metric": "positions solved/sec (node)",
        "value": P * args.steps / elapsed,
        "unit": "positions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("u%d order-form words, integer (%s table: keys implicit in the slot)" % (word_bits, layout)
                  if layout in ("dense", "planes") else "u64 keys / u32 words, integer"),
        "data": "synthetic: sum of Four-To-One heaps, fully determined state space",
        "config": {"workload": workload,
                   "positions_per_gpu": P // world, "edges_per_gpu": E // world,
                   "levels": r.levels, "root": r.root_line, "root_checked_against": root_src,
                   "layout": layout,
                   "parallelism": ((("row deal: heap 1 in 32-row slabs x%d, each level's last two rows per plane "
                                     "streamed to the next rank" if layout == "planes" and heaps[1] != 31 else
                                     "staged pipeline: one block of the top heap per rank x%d, halo rows "
                                     "streamed to the next rank" if layout == "planes" else
                                     "round-robin top-heap blocks x%d, one halo exchange per level") % world
                                    + ", %s" % ("host-staged (gloo, all ranks on one GPU: rehearsal, not a "
                                                "performance figure)" if host else "RCCL"))
                                   if world > 1 else "1 GPU")},
        "roofline": roof,
        "step_issue": ("queued solves (gm_solver_solve_async, <= %d outstanding): back to back on the GPU, "
                       "each collected and checked; solve_wall = one solve's device span" % QDEPTH
                       if queued else "one blocking solve() per step"),
        "phase_ms": {"forward": r.ms_forward, "backward": r.ms_backward,
                     "solve_wall": r.ms_total,
                     "expand_kernels": tr.ms_expand_kernels,
                     "resolve_kernels": tr.ms_resolve_kernels},
    }
    if rank == 0 and world == 1 and not args.no_keyed:
        del solver
        torch.cuda.empty_cache()
        line["keyed"] = keyed_record("cuda:%d" % local)
    if cpu is not None:
        line["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
