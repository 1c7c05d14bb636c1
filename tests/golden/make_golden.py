#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE'S OWN
GAME MODULES (/root/reference/test_games/*.py) and, for the root lines, from
the reference's own job loop (src/process.py) driven through an in-process
fake of mpi4py.

Runs ONLY in the build container (the reference never travels to the GPU box);
the fixtures it writes are data (inputs and expected outputs) and are
committed.  Third-party modules the reference needs but this image lacks
(bitstring, mpi4py, cachetools, objgraph) are replaced by the small shims in
tests/golden/refstubs/ (our code, written from those packages' published
semantics).

What it writes (see tests/golden/README.md):
  tables/<game>.npz      every reachable position: canonical bytes (sorted),
                         value code (src/utils.py:3), remoteness, level
  movegen/<game>.json    sampled positions: primitive + ORDERED children bytes
                         (src/game_state.py:32-40 expand order)
  md5_owner.json         GameState.get_hash(P) (src/game_state.py:22-30)
  movegen/toot_6x4.json, deep/toot_6x4.json
                         BASELINE config 3 at its own size, by samples
                         (--only toot_6x4; toot_6x4_fixtures)
  reference_runs.json    root lines printed by Process.run
                         (src/process.py:47-52) under the fake MPI
  summary.json           positions/edges/levels/histograms/root line per game

Per-position values use the REFERENCE-CANONICAL retrograde (SURVEY.md §8a
rows A8/A9): value = WIN if any child LOSS, else TIE if any TIE, else DRAW if
any DRAW, else LOSS; remoteness = 1 + min rem over LOSS children for WIN,
otherwise 1 + max rem over all children; primitives have remoteness 0
(src/process.py:122,243).

Usage:  python tests/golden/make_golden.py [--skip-mpi] [--only NAME ...]
"""
import argparse
import hashlib
import importlib.util
import io
import json
import os
import random
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
STUBS = os.path.join(HERE, "refstubs")
REPO = os.path.dirname(os.path.dirname(HERE))

WIN, LOSS, TIE, DRAW, UNDECIDED = 0, 1, 2, 3, 4
NAMES = ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED")


def _setup_path():
    for p in (REF, STUBS):
        if p in sys.path:
            sys.path.remove(p)
    sys.path.insert(0, REF)
    sys.path.insert(0, STUBS)


def load_ref_game(fname, modname, **overrides):
    """Load a reference game file the way solver_launcher.py:41-42 does
    (imp.load_source) and apply board-size overrides to module globals (the
    files read length/height/area at call time: SURVEY Appendix C.4)."""
    _setup_path()
    path = os.path.join(REF, "test_games", fname)
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for k, v in overrides.items():
        setattr(mod, k, v)
    if "length" in overrides or "height" in overrides:
        mod.area = mod.length * mod.height
    return mod


def load_own_game(path, modname):
    _setup_path()
    spec = importlib.util.spec_from_file_location(modname, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def canon_bytes(pos):
    """Canonical byte form of a position (what the C-ABI's gm_encode takes)."""
    if isinstance(pos, np.ndarray):
        return pos.astype(np.int8).tobytes()
    if isinstance(pos, (int, np.integer)):
        return str(int(pos)).encode("ascii")
    if isinstance(pos, str):
        return pos.encode("ISO-8859-1")
    raise TypeError(type(pos))


def hkey(pos):
    return pos.tobytes() if isinstance(pos, np.ndarray) else pos


def explore(mod):
    """Full reachable graph through the module's own API
    (initial_position/gen_moves/do_move/primitive)."""
    root = mod.initial_position()
    seen = {hkey(root): root}
    prim = {}
    children = {}
    level = {hkey(root): 0}
    order = [hkey(root)]
    i = 0
    while i < len(order):
        k = order[i]
        i += 1
        pos = seen[k]
        p = mod.primitive(pos)
        prim[k] = p
        if p != UNDECIDED:
            children[k] = []
            continue
        ch = []
        for m in mod.gen_moves(pos):
            c = mod.do_move(pos, m)
            ck = hkey(c)
            ch.append(ck)
            if ck not in seen:
                seen[ck] = c
                level[ck] = level[k] + 1
                order.append(ck)
        if not ch:
            raise RuntimeError("non-primitive position without moves")
        children[k] = ch
    return root, seen, prim, children, level, order


def retrograde(prim, children, order):
    """Reference-canonical value/remoteness, iterative
    post-order so it is valid for any DAG (edges may skip levels)."""
    val, rem = {}, {}
    for start in reversed(order):
        if start in val:
            continue
        stack = [(start, 0)]
        while stack:
            k, it = stack.pop()
            if k in val:
                continue
            if prim[k] != UNDECIDED:
                val[k], rem[k] = prim[k], 0
                continue
            ch = children[k]
            while it < len(ch) and ch[it] in val:
                it += 1
            if it < len(ch):
                stack.append((k, it))
                stack.append((ch[it], 0))
                continue
            cv = [val[c] for c in ch]
            cr = [rem[c] for c in ch]
            if LOSS in cv:
                v = WIN
                r = 1 + min(r for x, r in zip(cv, cr) if x == LOSS)
            else:
                v = TIE if TIE in cv else DRAW if DRAW in cv else LOSS
                r = 1 + max(cr)
            val[k], rem[k] = v, r
    return val, rem


def write_table(name, seen, prim, children, level, val, rem, root, outdir,
                store=True):
    keys = sorted(seen.keys(), key=lambda k: canon_bytes(seen[k]))
    width = max(len(canon_bytes(seen[k])) for k in keys)
    canon = np.zeros((len(keys), width), dtype=np.uint8)
    clen = np.zeros(len(keys), dtype=np.uint8)
    for i, k in enumerate(keys):
        b = canon_bytes(seen[k])
        canon[i, :len(b)] = np.frombuffer(b, dtype=np.uint8)
        clen[i] = len(b)
    value = np.array([val[k] for k in keys], dtype=np.uint8)
    remo = np.array([rem[k] for k in keys], dtype=np.uint32)
    lev = np.array([level[k] for k in keys], dtype=np.uint32)
    nchild = np.array([len(children[k]) for k in keys], dtype=np.uint8)
    if store:
        buf = io.BytesIO()
        np.savez_compressed(buf, canon=canon, clen=clen, value=value,
                            remoteness=remo, level=lev, nchild=nchild)
        os.makedirs(os.path.join(outdir, "tables"), exist_ok=True)
        with open(os.path.join(outdir, "tables", name + ".npz"), "wb") as f:
            f.write(buf.getvalue())
    h = hashlib.sha256()
    h.update(canon.tobytes())
    h.update(value.tobytes())
    h.update(remo.tobytes())
    rk = hkey(root)
    hist = [int((value == v).sum()) for v in range(4)]
    lev_hist = np.bincount(lev).tolist()
    return {
        "positions": len(keys),
        "edges": int(sum(len(children[k]) for k in keys)),
        "primitives": int(sum(1 for k in keys if prim[k] != UNDECIDED)),
        "levels": len(lev_hist),
        "max_level_width": int(max(lev_hist)),
        "level_hist": lev_hist,
        "value_hist_WLTD": hist,
        "root_canon_hex": canon_bytes(root).hex(),
        "root_value": NAMES[val[rk]],
        "root_remoteness": int(rem[rk]),
        "root_line": "%s in %d moves" % (NAMES[val[rk]], rem[rk]),
        "table_sha256": h.hexdigest(),
    }


def write_movegen(name, mod, seen, prim, children, outdir, nsample=400,
                  seed=0):
    rng = random.Random(seed)
    keys = list(seen.keys())
    keys.sort(key=lambda k: canon_bytes(seen[k]))
    sample = keys if len(keys) <= nsample else rng.sample(keys, nsample)
    rk = hkey(mod.initial_position())
    if rk not in sample:
        sample = [rk] + sample
    rows = []
    for k in sample:
        pos = seen[k]
        p = mod.primitive(pos)
        ch = []
        if p == UNDECIDED:
            ch = [canon_bytes(mod.do_move(pos, m)).hex()
                  for m in mod.gen_moves(pos)]
        rows.append({"pos": canon_bytes(pos).hex(), "primitive": int(p),
                     "children": ch, "str_utf8": str(pos).encode("utf-8").hex()})
    os.makedirs(os.path.join(outdir, "movegen"), exist_ok=True)
    with open(os.path.join(outdir, "movegen", name + ".json"), "w") as f:
        json.dump(rows, f, indent=0)


def md5_owner_vectors(samples):
    """Owner ranks from the reference's own GameState.get_hash
    (src/game_state.py:22-30)."""
    _setup_path()
    import src.utils  # reference module
    if src.utils.game_module is None:
        src.utils.game_module = load_ref_game("four_to_one.py", "gm_fto_md5")
    from src.game_state import GameState
    out = []
    for game, pos in samples:
        gs = GameState(pos)
        out.append({
            "game": game,
            "str_utf8": str(pos).encode("utf-8").hex(),
            "canon": canon_bytes(pos).hex(),
            "md5": hashlib.md5(str(pos).encode("utf-8")).hexdigest(),
            "owners": {str(P): gs.get_hash(P) for P in (1, 2, 3, 4, 5, 6, 7, 8)},
        })
    return out


# ---------------------------------------------------------------------------
# Reference job loop under the fake MPI
# ---------------------------------------------------------------------------
def run_reference_mpi(game_mod, nranks, timeout=600.0, int_keys=False):
    """Drive src/process.py's Process.run on `nranks` threads and capture the
    root line it prints (src/process.py:47-52)."""
    import contextlib
    import shutil
    import tempfile
    _setup_path()
    for m in list(sys.modules):
        if m == "src" or m.startswith("src."):
            del sys.modules[m]
    import src.utils
    src.utils.game_module = game_mod
    from mpi4py import MPI
    from src.game_state import GameState
    from src.job import Job
    from src.process import Process
    from src import cache_dict
    if int_keys:
        # reference defect src/cache_dict.py:78-79: shelve __contains__ needs
        # str keys; stringify ints the way __getitem__/__setitem__ already do.
        orig = cache_dict.CacheDict.__contains__

        def _contains(self, item):
            return orig(self, str(item) if isinstance(item, int) else item)
        cache_dict.CacheDict.__contains__ = _contains
    Process.IS_FINISHED = False
    world = MPI.World(nranks)
    scratch = tempfile.mkdtemp(prefix="gm_ref_")
    lines = []
    errors = []
    lock = threading.Lock()

    def rank_main(r):
        comm = MPI.Comm(world, r)
        out = io.StringIO()
        try:
            with contextlib.redirect_stdout(out):
                pass
            proc = Process(r, nranks, comm, comm.send, comm.recv, comm.Abort,
                           stats_dir=scratch)
            if proc.rank == proc.root:
                proc.add_job(Job(Job.LOOK_UP, GameState(GameState.INITIAL_POS),
                                 proc.rank, Job.INITIAL_JOB_ID))
            # capture the root print: Process.run prints then aborts
            import builtins
            real_print = builtins.print

            def cap_print(*a, **k):
                with lock:
                    lines.append(" ".join(str(x) for x in a))
            proc_globals = sys.modules["src.process"].__dict__
            proc_globals["print"] = cap_print
            try:
                proc.run()
            finally:
                proc_globals.pop("print", None)
                del real_print
        except MPI._Aborted:
            pass
        except BaseException as e:  # noqa: BLE001
            world.aborted.set()
            errors.append(repr(e))

    t0 = time.time()
    threads = [threading.Thread(target=rank_main, args=(r,), daemon=True)
               for r in range(nranks)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
    wall = time.time() - t0
    shutil.rmtree(scratch, ignore_errors=True)
    return {"ranks": nranks, "lines": lines, "errors": errors,
            "messages": world.messages, "wall_s": round(wall, 3)}


GAMES = {
    # name: (loader, kwargs)
    "four_to_one": ("four_to_one.py", {}),
    "mttt": ("mttt.py", {}),
    "tic_tac_toe_np": ("tic_tac_toe_np.py", {}),
    "othello_4x4": ("othello_bit_new.py", {"length": 4, "height": 4}),
    "toot_3x3": ("toot_and_otto_bitstring.py", {"length": 3, "height": 3}),
    "toot_4x3": ("toot_and_otto_bitstring.py", {"length": 4, "height": 3}),
    "toot_3x4": ("toot_and_otto_bitstring.py", {"length": 3, "height": 4}),
    # too large to commit as a table: summary + sha256 of the sorted table
    "toot_4x4": ("toot_and_otto_bitstring.py", {"length": 4, "height": 4}),
}
SHA_ONLY = {"toot_4x4"}


def toot_6x4_fixtures(outdir, n_movegen=400, n_deep=220, seed=6):
    """BASELINE config 3 at its own size (toot_and_otto_bitstring.py:8 as
    shipped, 6x4: 1,187,212,827 positions -- too many to enumerate here), pinned
    by the reference module itself on SAMPLES:
      movegen/toot_6x4.json  positions from random playouts of the module's
                             own gen_moves/do_move, each with primitive() and
                             the ordered children (src/game_state.py:32-40)
      md5 rows               GameState.get_hash for P = 1..8 (game_state.py:22-30)
      deep/toot_6x4.json     positions with >= 16 pieces placed, each solved
                             EXHAUSTIVELY through the module (every position
                             reachable from it) with the reference-canonical
                             retrograde: value and remoteness of the position
    Returns the md5 samples."""
    mod = load_ref_game("toot_and_otto_bitstring.py", "gm_toot_6x4", length=6, height=4)
    rng = random.Random(seed)
    root = mod.initial_position()
    pool, depth = {root: 0}, {}
    while len(pool) < 6 * n_movegen:  # playout positions, every depth
        pos, d = root, 0
        while mod.primitive(pos) == UNDECIDED:
            pos = mod.do_move(pos, rng.choice(mod.gen_moves(pos)))
            d += 1
            pool.setdefault(pos, d)
    keys = sorted(pool, key=canon_bytes)
    sample = [root] + rng.sample([k for k in keys if k != root], n_movegen - 1)
    rows = []
    for pos in sample:
        p = mod.primitive(pos)
        ch = [canon_bytes(mod.do_move(pos, m)).hex() for m in mod.gen_moves(pos)] if p == UNDECIDED else []
        rows.append({"pos": canon_bytes(pos).hex(), "primitive": int(p), "children": ch,
                     "str_utf8": str(pos).encode("utf-8").hex(), "pieces": pool[pos]})
    os.makedirs(os.path.join(outdir, "movegen"), exist_ok=True)
    with open(os.path.join(outdir, "movegen", "toot_6x4.json"), "w") as f:
        json.dump(rows, f, indent=0)

    def subdag(pos, cap=20000):
        seen, order, prim, children = {pos: True}, [pos], {}, {}
        i = 0
        while i < len(order):
            k = order[i]
            i += 1
            p = mod.primitive(k)
            prim[k] = p
            if p != UNDECIDED:
                children[k] = []
                continue
            ch = []
            for m in mod.gen_moves(k):
                c = mod.do_move(k, m)
                ch.append(c)
                if c not in seen:
                    seen[c] = True
                    order.append(c)
                    if len(order) > cap:
                        return None
            children[k] = ch
        return order, prim, children

    deep, tried = [], set()
    while len(deep) < n_deep:
        pos, d = root, 0
        target = rng.randint(16, 23)
        while d < target and mod.primitive(pos) == UNDECIDED:
            pos = mod.do_move(pos, rng.choice(mod.gen_moves(pos)))
            d += 1
        if d < 16 or pos in tried:
            continue
        tried.add(pos)
        sub = subdag(pos)
        if sub is None:
            continue
        order, prim, children = sub
        val, rem = retrograde(prim, children, order)
        deep.append({"pos": canon_bytes(pos).hex(), "pieces": d, "value": int(val[pos]),
                     "remoteness": int(rem[pos]), "primitive": int(prim[pos]),
                     "subgraph_positions": len(order)})
    os.makedirs(os.path.join(outdir, "deep"), exist_ok=True)
    with open(os.path.join(outdir, "deep", "toot_6x4.json"), "w") as f:
        json.dump({"game": "toot_and_otto_bitstring", "params": "length=6,height=4",
                   "source": "reference test_games/toot_and_otto_bitstring.py (length=6, height=4) through "
                             "tests/golden/make_golden.py toot_6x4_fixtures, seed %d" % seed,
                   "semantics": "value / remoteness by the reference-canonical retrograde (SURVEY.md 8a A8/A9) "
                                "over every position reachable from the listed one",
                   "rows": deep}, f, indent=0)
    hist = [sum(1 for r in deep if r["value"] == v) for v in range(4)]
    print("toot_6x4 fixtures: %d movegen rows, %d deep positions (W/L/T/D %s)" % (len(rows), len(deep), hist),
          flush=True)
    return [("toot_6x4", p) for p in [root] + rng.sample(sample, 59)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-mpi", action="store_true")
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    outdir = args.out
    summary_path = os.path.join(outdir, "summary.json")
    summary = {}
    if os.path.exists(summary_path):
        with open(summary_path) as f:
            summary = json.load(f)
    md5_samples = []

    todo = dict(GAMES)
    # Four-To-One chains of other heights (module's initial_position patched)
    for n in (20, 64):
        todo["four_to_one_%d" % n] = ("four_to_one.py", {"initial_position":
                                                        (lambda n=n: n)})
    # our own synthetic game file (sum of Four-To-One heaps), same API
    own = os.path.join(REPO, "gamesmanmpi_amd", "games", "sum_four_to_one.py")
    for heaps in ((3, 3, 3), (4, 4, 4), (2, 5, 7), (6, 6, 6, 6)):
        todo["sum_fto_" + "_".join(map(str, heaps))] = ("OWN", heaps)

    if args.only and "toot_6x4" in args.only:
        md5_samples += toot_6x4_fixtures(outdir)
    for name, (fname, kw) in todo.items():
        if args.only and name not in args.only:
            continue
        t0 = time.time()
        if fname == "OWN":
            mod = load_own_game(own, "gm_" + name)
            mod.HEAPS = tuple(kw)
        else:
            mod = load_ref_game(fname, "gm_" + name, **kw)
        root, seen, prim, children, level, order = explore(mod)
        val, rem = retrograde(prim, children, order)
        info = write_table(name, seen, prim, children, level, val, rem, root,
                           outdir, store=name not in SHA_ONLY)
        info["table_committed"] = name not in SHA_ONLY
        write_movegen(name, mod, seen, prim, children, outdir)
        info["source"] = ("reference test_games/" + fname if fname != "OWN"
                          else "gamesmanmpi_amd/games/sum_four_to_one.py")
        info["overrides"] = ({k: v for k, v in kw.items()
                              if not callable(v)} if fname != "OWN"
                             else {"HEAPS": list(kw)})
        if "initial_position" in (kw if fname != "OWN" else {}):
            info["overrides"]["initial_position"] = int(root)
        info["gen_s"] = round(time.time() - t0, 2)
        summary[name] = info
        print(name, info["positions"], info["edges"], info["root_line"],
              info["gen_s"], "s", flush=True)
        rng = random.Random(1)
        ks = list(seen.keys())
        for k in [hkey(root)] + rng.sample(ks, min(40, len(ks))):
            md5_samples.append((name, seen[k]))

    if md5_samples:
        md5_path = os.path.join(outdir, "md5_owner.json")
        rows = []
        if os.path.exists(md5_path):  # keep other games' rows (merge)
            with open(md5_path) as f:
                done = {g for g, _ in md5_samples}
                rows = [r for r in json.load(f) if r["game"] not in done]
        rows += md5_owner_vectors(md5_samples)
        with open(md5_path, "w") as f:
            json.dump(rows, f, indent=0)
    with open(summary_path, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)

    if not args.skip_mpi:
        runs = {}
        fto = load_ref_game("four_to_one.py", "gm_fto_mpi")
        for P in (1, 2, 5):
            runs["four_to_one_n%d" % P] = run_reference_mpi(fto, P,
                                                            int_keys=True)
            print("four_to_one", P, runs["four_to_one_n%d" % P], flush=True)
        mt = load_ref_game("mttt.py", "gm_mttt_mpi")
        runs["mttt_n1"] = run_reference_mpi(mt, 1, timeout=900)
        print("mttt", runs["mttt_n1"], flush=True)
        with open(os.path.join(outdir, "reference_runs.json"), "w") as f:
            json.dump(runs, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
