"""Game specs: the pairing of a reference-API game module with its device
descriptor.

A game module (initial_position / gen_moves / do_move / primitive,
README.md:28-88) is identified by its file stem -- the same name the
reference's launcher loads it under (solver_launcher.py:41) -- plus the
module-level parameters the reference's game files read at call time
(length/height of the bitstring games, HEAPS of the synthetic sum game, the
start of Four-To-One).  ``GameSpec.verify`` replays the module's own
functions on sampled positions and checks the descriptor against them, so a
modified game file is refused instead of silently solved with stale rules.
"""
import os
import random

import numpy as np

from .. import _lib

# file stem -> how the module's positions map to canonical bytes
_INT_GAMES = ("four_to_one", "sum_four_to_one")
_BITSTRING_GAMES = ("toot_and_otto_bitstring", "othello_bit_new")
KNOWN = _INT_GAMES + _BITSTRING_GAMES + ("tic_tac_toe_np", "mttt")


class GameSpec:
    """One game instance known to the device library."""

    def __init__(self, name, params=""):
        L = _lib.load()
        self.name, self.params = name, params or ""
        gid = _lib.ctypes.c_int()
        _lib.check(L.gm_game_lookup(name.encode(), self.params.encode(),
                                    _lib.ctypes.byref(gid)))
        self.id = gid.value
        b = _lib.ctypes.c_uint64()
        t = _lib.ctypes.c_uint32()
        kb = _lib.ctypes.c_uint32()
        _lib.check(L.gm_game_info(self.id, _lib.ctypes.byref(b),
                                  _lib.ctypes.byref(t), _lib.ctypes.byref(kb)))
        self.positions_bound, self.max_levels, self.key_bits = (
            b.value, t.value, kb.value)
        r = _lib.ctypes.c_uint64()
        _lib.check(L.gm_root(self.id, _lib.ctypes.byref(r)))
        self.root_key = r.value

    def __repr__(self):
        return "GameSpec(%r, %r)" % (self.name, self.params)

    # -- symmetry hooks (params "symmetry=1") ------------------------------
    @property
    def symmetric(self):
        return any(p.strip() == "symmetry=1" for p in self.params.split(","))

    def symmetry(self, keys, which=-1):
        """which=-1: canonical orbit representatives of `keys` (identity
        for specs without symmetry); which=i: the module's i-th symmetry
        function as a key map (include/gamesman.h gm_symmetry)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), np.uint64)
        _lib.check(_lib.load().gm_symmetry(self.id, int(which), keys.ctypes.data,
                                           len(keys), out.ctypes.data))
        return out

    # -- canonical bytes <-> keys ------------------------------------------
    def encode(self, canon):
        k = _lib.ctypes.c_uint64()
        _lib.check(_lib.load().gm_encode(self.id, bytes(canon), len(canon),
                                         _lib.ctypes.byref(k)))
        return k.value

    def decode(self, key):
        buf = _lib.ctypes.create_string_buffer(64)
        n = _lib.ctypes.c_size_t()
        _lib.check(_lib.load().gm_decode(self.id, int(key), buf, 64,
                                         _lib.ctypes.byref(n)))
        return buf.raw[:n.value]

    def encode_batch(self, canon, lens):
        """canon: u8[n, stride], lens: u8[n] -> keys u64[n]"""
        canon = np.ascontiguousarray(canon, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint8)
        keys = np.zeros(len(lens), np.uint64)
        _lib.check(_lib.load().gm_encode_batch(
            self.id, canon.ctypes.data, canon.shape[1], lens.ctypes.data,
            len(lens), keys.ctypes.data))
        return keys

    def decode_batch(self, keys, stride=24):
        """keys u64[n] -> (canon u8[n, stride], lens u8[n])"""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        canon = np.zeros((len(keys), stride), np.uint8)
        lens = np.zeros(len(keys), np.uint8)
        _lib.check(_lib.load().gm_decode_batch(
            self.id, keys.ctypes.data, len(keys), canon.ctypes.data, stride,
            lens.ctypes.data))
        return canon, lens

    def str_utf8(self, key):
        buf = _lib.ctypes.create_string_buffer(64)
        n = _lib.ctypes.c_size_t()
        _lib.check(_lib.load().gm_str_utf8(self.id, int(key), buf, 64,
                                           _lib.ctypes.byref(n)))
        return buf.raw[:n.value]

    # -- python positions <-> canonical bytes ------------------------------
    def to_canon(self, pos):
        if self.name in _INT_GAMES:
            return str(int(pos)).encode("ascii")
        if self.name == "tic_tac_toe_np":
            return np.asarray(pos, dtype=np.int8).tobytes()
        if self.name == "mttt":
            return pos.encode("ascii")
        return pos.encode("ISO-8859-1")

    def from_canon(self, canon):
        if self.name in _INT_GAMES:
            return int(canon)
        if self.name == "tic_tac_toe_np":
            return np.frombuffer(canon, dtype=np.int8).reshape(3, 3).copy()
        if self.name == "mttt":
            return canon.decode("ascii")
        return canon.decode("ISO-8859-1")

    def key_of(self, pos):
        return self.encode(self.to_canon(pos))

    def pos_of(self, key):
        return self.from_canon(self.decode(key))

    # -- host-side descriptor probes (parity tooling) ------------------------
    def host_expand(self, keys):
        """(prim u8[n], nchild u8[n], children u64[n, GM_MAXCHILD]) from the
        product's descriptor run on the host."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        n = len(keys)
        ch = np.zeros((n, _lib.GM_MAXCHILD), np.uint64)
        nc = np.zeros(n, np.uint8)
        pr = np.zeros(n, np.uint8)
        _lib.check(_lib.load().gm_host_expand(
            self.id, keys.ctypes.data, n, ch.ctypes.data, nc.ctypes.data,
            pr.ctypes.data))
        return pr, nc, ch

    def host_level(self, keys):
        """Tier of each key (int32[n]) from the descriptor, on the host."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), np.int32)
        _lib.check(_lib.load().gm_host_level(self.id, keys.ctypes.data,
                                             len(keys), out.ctypes.data))
        return out

    def owners_host(self, keys, world_size):
        """GameState.get_hash(world_size) (src/game_state.py:22-30)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), np.uint32)
        _lib.check(_lib.load().gm_owner_host(self.id, keys.ctypes.data,
                                             len(keys), int(world_size),
                                             out.ctypes.data))
        return out

    def shard_info(self, rank, world):
        """Geometry of dense shard `rank` of `world` (DESIGN.md
        §Multi-GPU): dict B (block width in top-heap values), nblocks (over
        all ranks), nb (blocks of this rank: k = rank, rank + world, ...),
        rank, Z (prefixes per top value), E (top values), Wl (local
        prefixes per level), world."""
        out = (_lib.ctypes.c_uint64 * 8)()
        _lib.check(_lib.load().gm_shard_info(self.id, int(rank), int(world),
                                             out))
        return dict(zip(("B", "nblocks", "nb", "rank", "Z", "E", "Wl",
                         "world"), list(out)))

    # -- the drop-in guard -------------------------------------------------
    def verify(self, module, samples=200, seed=0):
        """Replay the module's own primitive/gen_moves/do_move on random
        playouts from initial_position() and require the descriptor to
        agree on every primitive value, child list (order included) and
        str(pos).  Raises ValueError on the first disagreement."""
        rng = random.Random(seed)
        root = module.initial_position()
        # a symmetric spec stores orbit representatives: compare canonically
        canon = (lambda ks: [int(x) for x in self.symmetry(np.array(ks, np.uint64))]) \
            if self.symmetric else (lambda ks: ks)
        if canon([self.key_of(root)])[0] != self.root_key:
            raise ValueError("initial_position() does not match descriptor "
                             "%r root" % (self,))
        checked = 0
        pos = root
        while checked < samples:
            key = self.key_of(pos)
            if self.str_utf8(key) != str(pos).encode("utf-8"):
                raise ValueError("str(pos) mismatch at %r" % (pos,))
            pr, nc, ch = self.host_expand(np.array(canon([key]), np.uint64))
            p = module.primitive(pos)
            if int(pr[0]) != int(p):
                raise ValueError("primitive mismatch at %r: module %r, "
                                 "descriptor %r" % (pos, p, int(pr[0])))
            checked += 1
            if p != 4:
                pos = root
                continue
            kids = [module.do_move(pos, m) for m in module.gen_moves(pos)]
            want = canon([self.key_of(c) for c in kids])
            got = [int(x) for x in ch[0, :nc[0]]]
            if self.symmetric:  # the representative's children are an image of pos's
                want, got = sorted(want), sorted(got)
            if want != got:
                raise ValueError("children mismatch at %r" % (pos,))
            pos = kids[rng.randrange(len(kids))]
        return checked

    def verify_symmetries(self, module, samples=200, seed=0):
        """The module's symmetry_functions() (othello_bit_new.py:224-226:
        [(player_flip, 2)]) must be the descriptor's key maps: for positions
        on random playouts, key(f(pos)) == gm_symmetry(i, key(pos)) and f
        applied `order` times is the identity."""
        funcs = list(module.symmetry_functions())
        rng = random.Random(seed)
        root = module.initial_position()
        pos, checked = root, 0
        while checked < samples:
            k = np.array([self.key_of(pos)], np.uint64)
            for i, (f, order) in enumerate(funcs):
                img = f(pos)
                if self.key_of(img) != int(self.symmetry(k, i)[0]):
                    raise ValueError("symmetry %d (%s) disagrees with the descriptor at %r"
                                     % (i, getattr(f, "__name__", f), pos))
                for _ in range(int(order) - 1):
                    img = f(img)
                if self.key_of(img) != int(k[0]):
                    raise ValueError("symmetry %d is not of order %d" % (i, order))
            checked += 1
            if module.primitive(pos) != 4:
                pos = root
                continue
            kids = [module.do_move(pos, m) for m in module.gen_moves(pos)]
            pos = kids[rng.randrange(len(kids))]
        return checked


def spec_for_module(module, stem=None):
    """Map a loaded game module to its GameSpec (raises if no descriptor)."""
    stem = stem or os.path.splitext(os.path.basename(
        getattr(module, "__file__", "") or ""))[0]
    if stem == "four_to_one":
        params = "start=%d" % int(module.initial_position())
    elif stem == "sum_four_to_one":
        params = "heaps=" + ":".join(str(int(h)) for h in module.HEAPS)
    elif stem in _BITSTRING_GAMES:
        params = "length=%d,height=%d" % (int(module.length),
                                          int(module.height))
    elif stem in ("tic_tac_toe_np", "mttt"):
        params = ""
    else:
        raise ValueError(
            "no device descriptor for game file %r (known: %s)"
            % (stem, ", ".join(KNOWN)))
    return GameSpec(stem, params)
