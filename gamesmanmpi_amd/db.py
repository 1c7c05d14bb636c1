"""Solution database written by the launcher's -sd option, and queries on it.

The reference keeps a rank's results in shelve files
`<DIR>/stats/<rank>/{resolved,remote}` (src/cache_dict.py:19-42): value and
remoteness per position key.  The launcher writes the binary counterpart,
`<DIR>/stats/<rank>/solution.npz` + `meta.json` per rank (solver_launcher.py
write_stats), and this module reads any number of rank directories back as
one table:

    python -m gamesmanmpi_amd.db DIR --game GAME_FILE [POSITION ...]

prints `<position>: <VALUE> in <r> moves` for each position (a Python
literal evaluated against nothing but literals, e.g. 4 or '...'), or for the
game's initial position when none is given.  Descriptor-solved tables are
keyed by the packed u64 key (GameSpec.key_of); graph-solved tables (game
files without a descriptor) by str(position).
"""
import argparse
import ast
import glob
import json
import os
import sys

import numpy as np

NAMES = ("WIN", "LOSS", "TIE", "DRAW")


class SolutionDB:
    def __init__(self, root):
        ranks = sorted(glob.glob(os.path.join(root, "stats", "*", "solution.npz")))
        if not ranks:
            raise FileNotFoundError("no stats/<rank>/solution.npz under %r" % root)
        keys, names, val, rem, metas = [], [], [], [], []
        for path in ranks:
            with np.load(path) as z:  # allow_pickle stays False
                if "keys" in z.files:
                    keys.append(z["keys"].astype(np.uint64))
                else:
                    names.append(z["names"])
                val.append(z["value"].astype(np.uint8))
                rem.append(z["remoteness"].astype(np.uint32))
            with open(os.path.join(os.path.dirname(path), "meta.json")) as f:
                metas.append(json.load(f))
        if keys and names:
            raise ValueError("mixed keyed and graph tables under %r" % root)
        self.meta = metas[0]
        self.ranks = len(ranks)
        self.value = np.concatenate(val)
        self.remoteness = np.concatenate(rem)
        if keys:
            self.by = "key"
            k = np.concatenate(keys)
            order = np.argsort(k, kind="stable")
            self.keys = k[order]
            if len(self.keys) > 1 and (np.diff(self.keys) == 0).any():
                raise ValueError("a position appears in two rank files")
            self.value, self.remoteness = self.value[order], self.remoteness[order]
        else:
            self.by = "name"
            self.index = {str(n): i for i, n in enumerate(np.concatenate(names))}

    def __len__(self):
        return len(self.value)

    def lookup_key(self, key):
        i = int(np.searchsorted(self.keys, np.uint64(key)))
        if i == len(self.keys) or int(self.keys[i]) != int(key):
            return None
        return int(self.value[i]), int(self.remoteness[i])

    def lookup_name(self, name):
        i = self.index.get(name)
        return None if i is None else (int(self.value[i]), int(self.remoteness[i]))

    def lookup(self, pos, spec=None):
        """(value, remoteness) of a game position, or None if unreachable."""
        if self.by == "name":
            return self.lookup_name(str(pos))
        if spec is None:
            raise ValueError("a keyed table needs the game's GameSpec")
        key = spec.key_of(pos)
        if "symmetry=1" in self.meta.get("params", "").split(","):
            # a symmetric solve stored orbit representatives (gm_symmetry)
            from .games import GameSpec
            key = int(GameSpec(spec.name, self.meta["params"]).symmetry(
                np.array([key], np.uint64))[0])
        return self.lookup_key(key)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="gamesmanmpi_amd.db")
    ap.add_argument("statsdir")
    ap.add_argument("--game", required=True, help="the game file that was solved")
    ap.add_argument("positions", nargs="*")
    args = ap.parse_intermixed_args(argv)
    from .solver_launcher import ensure_src_utils, load_game
    ensure_src_utils()
    mod = load_game(args.game)
    db = SolutionDB(args.statsdir)
    spec = None
    if db.by == "key":
        from .games import spec_for_module
        spec = spec_for_module(mod, os.path.splitext(os.path.basename(args.game))[0])
    todo = [ast.literal_eval(p) for p in args.positions] or [mod.initial_position()]
    rc = 0
    for pos in todo:
        r = db.lookup(pos, spec)
        if r is None:
            print("%s: not reachable" % (pos,))
            rc = 1
        else:
            print("%s: %s in %d moves" % (pos, NAMES[r[0]], r[1]))
    return rc


if __name__ == "__main__":
    sys.exit(main())
