#!/usr/bin/env python3
"""Drop-in for the reference's launcher (solver_launcher.py:1-98).

    reference:  mpiexec -n P python solver_launcher.py GAME_FILE [--debug] [-sd DIR]
    here:       python -m gamesmanmpi_amd.solver_launcher GAME_FILE [--debug] [-sd DIR]
                torchrun --nproc-per-node N -m gamesmanmpi_amd.solver_launcher GAME_FILE

Same positional argument and flags (solver_launcher.py:9-28), same game
loading (imp.load_source + src.utils.game_module, :41-42), same validation
of the four API functions (:55-66), and the same single output line on the
root's rank: "<WIN|LOSS|TIE|DRAW> in <r> moves" (src/process.py:47-52).

What differs, by design:
  * the game file is paired with its device descriptor (by file stem) and
    the pairing is verified by replaying the module's own functions on
    sampled positions before solving (--no-verify skips it);
  * one process per GPU via torch.distributed.run instead of mpiexec ranks;
  * -sd writes the solution per rank as <DIR>/stats/<rank>/solution.npz
    (keys, value, remoteness) plus meta.json -- the binary counterpart of the
    reference's <DIR>/stats/<rank>/{resolved,remote} shelve files
    (src/cache_dict.py:19-42);
  * values are the order-independent reading of the reference's reduction
    (DESIGN.md §Parity); results are deterministic.
"""
import argparse
import importlib.util
import json
import logging
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
COMPAT = os.path.join(HERE, "compat")


def ensure_src_utils():
    """Game files `import src.utils` (e.g. four_to_one.py:5).  Use an
    importable reference `src` package when there is one, otherwise our
    compat copy of the constants (gamesmanmpi_amd/compat/src/utils.py)."""
    try:
        import src.utils  # noqa: F401
    except ImportError:
        for m in [m for m in sys.modules if m == "src" or m.startswith("src.")]:
            del sys.modules[m]
        sys.path.insert(0, COMPAT)
        import src.utils  # noqa: F401
    return sys.modules["src.utils"]


def load_game(path):
    """imp.load_source('game_module', path) (solver_launcher.py:41)."""
    spec = importlib.util.spec_from_file_location("game_module", path)
    if spec is None:
        raise FileNotFoundError(path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def validate(mod):
    """solver_launcher.py:55-66: the four API functions must exist."""
    for name in ("initial_position", "do_move", "gen_moves", "primitive"):
        try:
            getattr(mod, name)
        except AttributeError as e:
            print("Could not find method", e.args[0])
            raise


def build_parser():
    p = argparse.ArgumentParser(prog="gamesmanmpi_amd.solver_launcher")
    p.add_argument("game_file", help="game to solve for")
    p.add_argument("--debug", help="Enables or disables logging",
                   action="store_true")
    p.add_argument("-sd", "--statsdir",
                   help="location to store statistics about game",
                   action="store")
    # additions
    p.add_argument("--layout", choices=["auto", "dense", "ranked", "bucketed", "hashed", "graph"],
                   default="auto",
                   help="table layout (DESIGN.md §Layout); graph = host-"
                        "enumerated positions, for files without a descriptor")
    p.add_argument("--positions", type=int, default=0,
                   help="capacity estimate for boards without a known bound")
    p.add_argument("--no-verify", action="store_true",
                   help="skip replaying the module against its descriptor")
    p.add_argument("--verify-samples", type=int, default=200)
    p.add_argument("--ranked-shards", action="store_true",
                   help="under torchrun, toot-and-otto: md5-owned RANKED shards (every position "
                        "resolved by its md5 owner, level words exchanged over RCCL) instead of "
                        "the default, every rank solving the whole RANKED table; the shards' "
                        "trace model predicts 22.4 ms at 8 GPUs against 8.5 ms on one "
                        "(DESIGN.md section 6c), and their RCCL path has not run on hardware")
    p.add_argument("--ranked-replicated", action="store_true",
                   help="(the default under torchrun; kept for old command lines)")
    p.add_argument("--json", action="store_true",
                   help="also print a JSON line with counts and timings")
    p.add_argument("--symmetries", action="store_true",
                   help="solve orbit representatives under the game module's "
                        "symmetry_functions() (othello_bit_new: player_flip); "
                        "every position keeps its own value and remoteness")
    p.add_argument("-ck", "--checkpoint", metavar="DIR",
                   help="one-GPU solves: checkpoint the solver state into DIR "
                        "every --checkpoint-every levels and resume from DIR "
                        "when it holds a checkpoint of the same game "
                        "(gamesmanmpi_amd.checkpoint); removed on completion")
    p.add_argument("--checkpoint-every", type=int, default=32, metavar="N",
                   help="levels (steps) between checkpoints")
    return p


DENSE_STEMS = ("four_to_one", "sum_four_to_one")  # rank-indexable descriptors


def ranked_fits(spec, local, world=1, replicated=False):
    """The game has a RANKED plan (toot-and-otto) that fits this GPU's free
    memory with a margin: the one-table plan, or (world > 1, not replicated)
    an md5 shard's (the table + owner bit planes + level exchange buffers)."""
    import ctypes
    from gamesmanmpi_amd import _lib
    p = _lib.gm_plan_t()
    if world > 1 and not replicated:
        rc = _lib.load().gm_plan_keyed_shard(spec.id, 0, world, 0, _lib.GM_F_RANKED_SHARD, 0, ctypes.byref(p))
    else:
        rc = _lib.load().gm_plan(spec.id, 0, 0, 0, ctypes.byref(p))
    if rc != 0 or p.mode != _lib.GM_MODE_RANKED:
        return False
    import torch
    free, _ = torch.cuda.mem_get_info(local)
    return p.table_bytes + p.scratch_bytes < 0.8 * free


def agreed_ranked(spec, layout, local, world=1, replicated=False):
    """Under torchrun: do ALL ranks take the replicated RANKED path?  Each
    rank's own answer (ranked_fits: its GPU's free memory) is combined with a
    MIN all-reduce, so every rank branches the same way and the collectives
    of the path they take match (a rank alone on the md5 keyed path would
    wait in its all-to-all for peers that never enter it).  An explicit
    --layout ranked that does not fit on every rank is an error, not a silent
    switch to the keyed path."""
    import torch
    import torch.distributed as dist
    if layout not in ("auto", "ranked"):
        return False
    mine = bool(ranked_fits(spec, local, world, replicated))
    dev = torch.device("cuda", local) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if mine else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    every = bool(int(t.item()))
    if layout == "ranked" and not every:
        raise SystemExit("--layout ranked: the RANKED table of %s does not fit on every rank's GPU "
                         "(this rank: %s)" % (spec.name, "fits" if mine else "does not fit"))
    return every


def write_stats(statsdir, rank, spec, solver, result, world=1):
    """<statsdir>/stats/<rank>/solution.npz (+ meta.json).  world > 1 with a
    replicated table (every rank solved the whole game): this rank writes the
    positions the reference's md5 partition gives it (src/game_state.py:22-30)."""
    import numpy as np
    d = os.path.join(statsdir, "stats", str(rank))
    os.makedirs(d, exist_ok=True)
    keys, val, rem = solver.dump()
    if world > 1 and getattr(solver, "replicated", False):
        own = spec.owners_host(keys, world) == rank
        keys, val, rem = keys[own], val[own], rem[own]
    canon, lens = spec.decode_batch(keys, stride=32)
    np.savez_compressed(os.path.join(d, "solution.npz"), keys=keys,
                        canon=canon, clen=lens, value=val, remoteness=rem)
    with open(os.path.join(d, "meta.json"), "w") as f:
        json.dump({"game": spec.name, "params": spec.params,
                   "root": result.root_line, "positions": len(keys),
                   "owned_by_rank": rank,
                   "value_codes": {"WIN": 0, "LOSS": 1, "TIE": 2, "DRAW": 3}},
                  f, indent=1)


def solve_generic(args, game, rank, world, local):
    """Game files without a device descriptor: the
    module's own functions enumerate the positions on the host
    (gamesmanmpi_amd/generic.py), the GPU runs the retrograde.  One GPU:
    under torchrun only rank 0 solves."""
    import torch
    from gamesmanmpi_amd.generic import solve_module
    if rank == 0:
        torch.cuda.set_device(local)
        result, solver = solve_module(game, device="cuda:%d" % local)
        print(result.root_line, flush=True)  # src/process.py:47-52
        if args.json:
            print(json.dumps({"game": os.path.basename(args.game_file),
                              "root": result.root_line,
                              "positions": result.positions,
                              "edges": result.edges,
                              "ms_total": result.ms_total,
                              "host_enumeration_s": result.extra["host_enumeration_s"],
                              "layout": "graph", "ranks": 1}), flush=True)
        if args.statsdir:
            import numpy as np
            d = os.path.join(args.statsdir, "stats", "0")
            os.makedirs(d, exist_ok=True)
            names, val, rem = solver.dump()
            np.savez_compressed(os.path.join(d, "solution.npz"),
                                names=np.array(names), value=val, remoteness=rem)
            with open(os.path.join(d, "meta.json"), "w") as f:
                json.dump({"game": os.path.basename(args.game_file),
                           "root": result.root_line, "positions": len(names),
                           "layout": "graph", "key": "str(position)",
                           "value_codes": {"WIN": 0, "LOSS": 1, "TIE": 2, "DRAW": 3}},
                          f, indent=1)
    return 0


def main(argv=None):
    args = build_parser().parse_args(argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.debug:  # src/debug.py:10-18: logging to logs/proc<rank>
        os.makedirs("logs", exist_ok=True)
        logging.basicConfig(filename="logs/proc%d" % rank, level=logging.DEBUG)

    utils = ensure_src_utils()
    game = load_game(args.game_file)
    utils.game_module = game
    validate(game)

    root = os.path.dirname(HERE)
    if root not in sys.path:
        sys.path.insert(0, root)
    from gamesmanmpi_amd.games import spec_for_module
    try:
        spec = spec_for_module(game, os.path.splitext(
            os.path.basename(args.game_file))[0])
    except ValueError as e:  # no device descriptor for this file
        if args.layout not in ("auto", "graph"):
            raise
        logging.debug("%s: solving through the host-enumerated graph", e)
        return solve_generic(args, game, rank, world, local)
    if args.layout == "graph":
        return solve_generic(args, game, rank, world, local)
    if args.symmetries:
        if not hasattr(game, "symmetry_functions"):
            raise SystemExit("%s defines no symmetry_functions()" % args.game_file)
        from gamesmanmpi_amd.games import GameSpec
        spec = GameSpec(spec.name, (spec.params + ",symmetry=1").lstrip(","))
        if not args.no_verify:
            spec.verify_symmetries(game, samples=args.verify_samples)
    if not args.no_verify:
        n = spec.verify(game, samples=args.verify_samples)
        logging.debug("descriptor %r verified on %d positions", spec, n)

    if args.checkpoint and world > 1:
        raise SystemExit("-ck/--checkpoint covers one-GPU solves (a sharded solve's state spans ranks)")
    if args.checkpoint:
        # never write into (or later delete) a directory that holds anything
        # but a checkpoint of ours
        from gamesmanmpi_amd import checkpoint
        try:
            checkpoint.check_target(args.checkpoint)
        except checkpoint.NotACheckpoint as e:
            raise SystemExit("-ck: %s" % e)
    import torch
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if spec.name in DENSE_STEMS and args.layout != "hashed":
            # top-heap blocks, RCCL halo exchange (gamesmanmpi_amd.dist)
            from gamesmanmpi_amd.dist import ShardedSolver
            solver = ShardedSolver(spec, rank, world, device="cuda:%d" % local)
            result = solver.solve()
        elif not args.ranked_shards and agreed_ranked(spec, args.layout, local, world, True):
            # (the default) every rank solves the whole RANKED table
            # and writes the md5 share the reference's partition gives it
            from gamesmanmpi_amd.solver import Solver
            solver = Solver(spec, positions=args.positions, device="cuda:%d" % local, layout="ranked")
            solver.replicated = True
            result = solver.solve()
            result.extra.update({"partition": "replicated", "world": world})
        elif args.ranked_shards and agreed_ranked(spec, args.layout, local, world):
            # (--ranked-shards) md5 shards of the RANKED index space -- every
            # position resolved by its md5 owner (src/game_state.py:22-30),
            # each level's words exchanged over RCCL (gm_ranked_shard.h);
            # every rank ends with the whole table and writes its md5 share
            from gamesmanmpi_amd.keyed import dist_keyed_solve
            result, solver = dist_keyed_solve(spec, device="cuda:%d" % local, layout="ranked")
            solver.replicated = True
        else:
            # the reference's md5 partition, all-to-all per level (keyed.py)
            from gamesmanmpi_amd.keyed import dist_keyed_solve
            result, shard = dist_keyed_solve(spec, device="cuda:%d" % local,
                                             positions=args.positions)
            solver = getattr(shard, "solver", shard)  # (GpuShard wraps its Solver; a bucketed shard is one)
    elif args.checkpoint:
        from gamesmanmpi_amd import checkpoint
        from gamesmanmpi_amd.solver import Solver
        first = 0
        src = checkpoint.latest(args.checkpoint)  # DIR, or DIR.old after an interrupted save
        if src is not None:
            meta = checkpoint.read_meta(src)
            if (meta["game"], meta["params"]) != (spec.name, spec.params):
                raise SystemExit("%s holds a checkpoint of %s %s, not %s %s"
                                 % (src, meta["game"], meta["params"],
                                    spec.name, spec.params))
            solver, first = checkpoint.restore(args.checkpoint, device="cuda:%d" % local)
            logging.debug("resuming %r at step %d of %d", spec, first, solver.steps)
        else:
            solver = Solver(spec, positions=args.positions,
                            device="cuda:%d" % local, layout=args.layout)
        result = checkpoint.solve_checkpointed(solver, args.checkpoint,
                                               args.checkpoint_every, first=first)
    else:
        from gamesmanmpi_amd.solver import Solver
        solver = Solver(spec, positions=args.positions,
                        device="cuda:%d" % local, layout=args.layout)
        result = solver.solve()
    if rank == 0:
        print(result.root_line, flush=True)  # src/process.py:47-52
        if args.json:
            print(json.dumps({"game": spec.name, "params": spec.params,
                              "root": result.root_line,
                              "positions": result.positions,
                              "edges": result.edges,
                              "ms_total": result.ms_total,
                              "layout": result.extra.get("layout"),
                              "ranks": world}), flush=True)
    if args.statsdir:
        write_stats(args.statsdir, rank, spec, solver, result, world)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
