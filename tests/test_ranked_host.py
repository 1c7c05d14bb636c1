"""The RANKED layout's index map (gamesmanmpi_amd/csrc/gm_ranked.h) restated
on the host and checked against the oracle's reachable positions -- no GPU.

Every reachable toot-and-otto position (the oracle's solve, its canonical
bytes turned into device keys by the library's own codec) must land on a
distinct slot of its level's region, with hands inside [0, 6], the turn bit
and the hands that rk_key would rebuild -- the map the kernels' index
arithmetic and their `first mover = the reference's player 2` labelling
rest on.  The slot counts per level match gm_plan's table_slots."""
import itertools

import numpy as np
import pytest

HAND = 6


def _shape(C, H):
    """rank_shape: per level the height vectors in code order, blocks of
    8 x 2^L slots, levels padded to 512."""
    R = H + 1
    byl = {}
    for code in range(R ** C):
        hv = [(code // R ** x) % R for x in range(C)]
        byl.setdefault(sum(hv), []).append(code)
    base, lvstart, at = {}, [], 0
    for L in range(C * H + 1):
        lvstart.append(at)
        for j, code in enumerate(byl.get(L, [])):
            base[code] = at + j * (8 << L)
        at += (len(byl.get(L, [])) * (8 << L) + 511) // 512 * 512
    lvstart.append(at)
    return base, lvstart, at


def _slot(key, C, H, base):
    """rk_slot_of restated: key -> (slot, level) or None."""
    A = C * H
    full = (1 << A) - 1
    t, o = key & full, (key >> A) & full
    if t & o or key >> (2 * A + 13):
        return None
    occ = t | o
    code = pat = L = 0
    for x in range(C):
        h = 0
        while h < H and (occ >> (C * h + x)) & 1:
            h += 1
        if any((occ >> (C * y + x)) & 1 for y in range(h, H)):
            return None
        for y in range(h):
            pat |= ((t >> (C * y + x)) & 1) << (L + y)
        code += h * (H + 1) ** x
        L += h
    nT = bin(pat).count("1")
    sT, sO = (key >> (2 * A)) & 7, (key >> (2 * A + 3)) & 7          # player 1: the second mover
    fT, fO = (key >> (2 * A + 6)) & 7, (key >> (2 * A + 9)) & 7      # player 2: the first mover
    turn = (key >> (2 * A + 12)) & 1
    a = HAND - fT
    used = (a, (L + 1) // 2 - a, nT - a, L // 2 - (nT - a))
    if not all(0 <= u <= HAND for u in used):
        return None
    if (HAND - used[1], HAND - used[2], HAND - used[3]) != (fO, sT, sO) or turn != (L & 1):
        return None
    return base[code] + (a << L) + pat, L


@pytest.mark.parametrize("params,C,H", [("length=3,height=3", 3, 3), ("length=4,height=3", 4, 3),
                                        ("length=2,height=4", 2, 4)])
def test_ranked_index_covers_the_reachable_positions(params, C, H):
    from gamesmanmpi_amd.games import GameSpec
    from oracle.oracle import Game  # checker only
    spec = GameSpec("toot_and_otto_bitstring", params)
    sol = Game("toot_and_otto_bitstring", params).solve(1 << 22)
    canon, clen, _, _ = sol.dump(stride=24)
    keys = spec.encode_batch(canon, clen)
    base, lvstart, nslots = _shape(C, H)
    seen = set()
    per_level = np.zeros(C * H + 1, np.int64)
    for k in keys.tolist():
        r = _slot(k, C, H, base)
        assert r is not None, hex(k)
        s, L = r
        assert lvstart[L] <= s < lvstart[L + 1]
        assert s not in seen
        seen.add(s)
        per_level[L] += 1
    assert len(seen) == sol.count
    assert per_level[0] == 1  # the root: slot 0 of level 0
    assert _slot(int(spec.encode(sol.game.root())), C, H, base) == (0, 0)


@pytest.mark.parametrize("params,C,H", [("length=4,height=4", 4, 4), ("length=6,height=4", 6, 4)])
def test_ranked_plan_slots(params, C, H):
    """gm_plan's table_slots is the restated index space (levels padded to 512)."""
    import ctypes
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    p = _lib.gm_plan_t()
    _lib.check(_lib.load().gm_plan(GameSpec("toot_and_otto_bitstring", params).id, 0, 0, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_RANKED
    assert p.table_slots == _shape(C, H)[2]
    assert p.table_slots >= 8 * (2 ** (H + 1) - 1) ** C
