"""C-ABI checks that need no GPU: the library loads, exports every symbol the
header declares, and its HOST-side entry points (codec, the product's own
descriptors run on the host, md5 owners) agree with the reference's golden
vectors.  No kernel is launched here."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import ALL_CASES, CASES, GOLDEN, ROOT, load_table


def header_symbols():
    with open(os.path.join(ROOT, "include", "gamesman.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w ]+?\*?\s*\b(gm_\w+)\s*\(",
                                 text, re.M)))


def test_header_and_exports_agree():
    from gamesmanmpi_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 18
    assert sorted(_lib.EXPORTS) == syms
    lib = _lib.load()
    for s in syms:
        assert getattr(lib, s) is not None


def test_unknown_game_is_an_error():
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    with pytest.raises(_lib.GmError):
        GameSpec("chess")
    with pytest.raises(_lib.GmError):
        GameSpec("othello_bit_new", "length=4,height=3")  # non-square refused


@pytest.mark.parametrize("name", sorted(CASES))
def test_codec_roundtrip_on_golden_tables(name):
    from gamesmanmpi_amd.games import GameSpec
    t = load_table(name)
    if t is None:
        pytest.skip("sha-only fixture")
    spec = GameSpec(*CASES[name])
    keys = spec.encode_batch(t["canon"], t["clen"])
    assert len(np.unique(keys)) == len(keys)
    c, cl = spec.decode_batch(keys, stride=t["canon"].shape[1])
    np.testing.assert_array_equal(c, t["canon"])
    np.testing.assert_array_equal(cl, t["clen"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_product_descriptor_vs_reference_movegen(name):
    """The product's descriptors (run on the host) reproduce the reference
    modules' primitive() and ordered gen_moves/do_move children."""
    from gamesmanmpi_amd.games import GameSpec
    path = os.path.join(GOLDEN, "movegen", name + ".json")
    if not os.path.exists(path):
        pytest.skip("no vectors")
    spec = GameSpec(*CASES[name])
    with open(path) as f:
        rows = json.load(f)
    keys = np.array([spec.encode(bytes.fromhex(r["pos"])) for r in rows],
                    np.uint64)
    pr, nc, ch = spec.host_expand(keys)
    for i, row in enumerate(rows):
        assert pr[i] == row["primitive"], row["pos"]
        got = [spec.decode(k).hex() for k in ch[i, :nc[i]]]
        assert got == row["children"], row["pos"]
        assert spec.str_utf8(keys[i]).hex() == row["str_utf8"], row["pos"]


def test_root_keys_match_reference_initial_positions(golden_summary):
    from gamesmanmpi_amd.games import GameSpec
    for name, (stem, params) in CASES.items():
        spec = GameSpec(stem, params)
        root = bytes.fromhex(golden_summary[name]["root_canon_hex"])
        assert spec.decode(spec.root_key) == root, name


def test_md5_owner_vectors():
    """GameState.get_hash (src/game_state.py:22-30) owners for P=1..8, as
    computed by the reference itself."""
    from gamesmanmpi_amd.games import GameSpec
    with open(os.path.join(GOLDEN, "md5_owner.json")) as f:
        rows = json.load(f)
    specs = {n: GameSpec(*ALL_CASES[n]) for n in ALL_CASES}
    n = 0
    for row in rows:
        spec = specs[row["game"]]
        key = spec.encode(bytes.fromhex(row["canon"]))
        assert spec.str_utf8(key).hex() == row["str_utf8"]
        for P, owner in row["owners"].items():
            assert spec.owners_host(np.array([key], np.uint64),
                                    int(P))[0] == owner, (row, P)
        n += 1
    assert n > 100


def test_survey_md5_golden_values():
    """SURVEY Appendix A.5 spot values."""
    from gamesmanmpi_amd.games import GameSpec
    s = GameSpec("four_to_one", "start=4")
    k = np.array([4], np.uint64)
    assert [s.owners_host(k, P)[0] for P in (1, 2, 4, 5, 8)] == [0, 0, 0, 0, 4]
    o = GameSpec("othello_bit_new", "length=4,height=4")
    k = np.array([o.root_key], np.uint64)
    assert [o.owners_host(k, P)[0] for P in (2, 4, 5, 8)] == [0, 2, 1, 6]
    t = GameSpec("toot_and_otto_bitstring", "length=6,height=4")
    k = np.array([t.root_key], np.uint64)
    assert t.str_utf8(t.root_key).hex() == "0000000000006666c280"
    assert [t.owners_host(k, P)[0] for P in (2, 4, 5, 8)] == [1, 1, 0, 5]


def test_plan_sizes():
    import ctypes
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    s = GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31")
    assert s.positions_bound == 1 << 30
    assert s.max_levels == 187
    p = _lib.gm_plan_t()
    _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_FORCE_HASHED, 0,
                                   ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_HASHED
    assert p.table_slots == 1 << 31 and p.level_capacity >= 1 << 30
    assert p.table_bytes == 16 << 31
    # default: PLANES, one 8-bit word per position (natural rank order, no
    # holes) + a reach map of one bit per 32-position row
    _lib.check(_lib.load().gm_plan(s.id, 0, 0, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_PLANES
    assert p.table_slots == 1 << 30
    assert p.table_bytes == (1 << 30) + (1 << 30) // 256
    _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_WORDS16, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_PLANES and p.table_bytes == (2 << 30) + (1 << 30) // 256
    # the level-major DENSE table on request
    _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_LEVEL_MAJOR, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_DENSE
    assert p.table_slots == 187 * 32 ** 5
    # 8-bit order-form words (one-GPU, remoteness < 255) + reach bitmap
    assert p.table_bytes == 1 * 187 * 32 ** 5 + 187 * 32 ** 5 // 8
    # the kernel-family flags plan 16- or 32-bit words (and the environment
    # does not: no knob is read from it)
    _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_WORDS16 | _lib.GM_F_LEVEL_MAJOR, 0, ctypes.byref(p)))
    assert p.table_bytes == 2 * 187 * 32 ** 5 + 187 * 32 ** 5 // 8
    for f in (_lib.GM_F_WORDS32, _lib.GM_F_RESOLVE_SCALAR):
        _lib.check(_lib.load().gm_plan(s.id, 0, f, 0, ctypes.byref(p)))
        assert p.table_bytes == 4 * 187 * 32 ** 5 + 187 * 32 ** 5 // 8
    os.environ["GM_WORDS32"] = "1"
    try:
        _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_LEVEL_MAJOR, 0, ctypes.byref(p)))
        assert p.table_bytes == 1 * 187 * 32 ** 5 + 187 * 32 ** 5 // 8
    finally:
        del os.environ["GM_WORDS32"]
    # remoteness past 254 keeps 16-bit words (heaps 127 + 127 + 7 = 261 levels)
    w = GameSpec("sum_four_to_one", "heaps=127:127:7")
    _lib.check(_lib.load().gm_plan(w.id, 0, 0, 0, ctypes.byref(p)))
    assert p.table_bytes == 2 * 262 * 128 * 8 + 262 * 128 * 8 // 8
    # a byte budget below the dense table falls back to the keyed table
    _lib.check(_lib.load().gm_plan(s.id, 0, 0, 1 << 30, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_HASHED
    t = GameSpec("toot_and_otto_bitstring", "length=4,height=4")
    _lib.check(_lib.load().gm_plan(t.id, 0, 0, 0, ctypes.byref(p)))
    # toot: positions at computed indices -- per level, its height vectors'
    # blocks of 8 x 2^L slots, levels padded to 512 (gm_ranked.h)
    assert p.mode == _lib.GM_MODE_RANKED
    import itertools
    per = [0] * 17
    for hv in itertools.product(range(5), repeat=4):
        per[sum(hv)] += 8 << sum(hv)
    slots = sum((n + 511) // 512 * 512 for n in per)
    assert slots >= 8 * 31 ** 4 and p.table_slots == slots
    assert p.table_bytes >= slots + 2 * slots // 8
    _lib.check(_lib.load().gm_plan(t.id, 0, _lib.GM_F_FORCE_HASHED, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_BUCKETED  # the keyed layout: every move one level
    assert p.level_capacity == 3468773 + 64 and p.table_slots == 9932808 + 1024
    _lib.check(_lib.load().gm_plan(t.id, 0, _lib.GM_F_HASH_TABLE, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_HASHED
    # step-2 games (sums) never take the bucketed layout
    _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_FORCE_HASHED, 0, ctypes.byref(p)))
    assert p.mode == _lib.GM_MODE_HASHED


@pytest.mark.parametrize("outer,bytes_per_word", [
    (191, 1),   # root digit sum 253: absolute 8-bit words
    (192, 1),   # 254: relative 8-bit words (gm_plane.h, word form 3)
    (443, 1),   # 505 = kPlaneRelMaxSum: the last relative one
    (444, 2),   # 506: 16-bit words
])
def test_planes_word_width_by_root_sum(outer, bytes_per_word):
    """PLANES words: 8-bit up to root digit sum 505 (absolute forms to 253,
    relative ones above), 16-bit beyond; GM_F_WORDS16 forces 16-bit."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    s = GameSpec("sum_four_to_one", "heaps=31:31:%d" % outer)
    p = _lib.gm_plan_t()
    _lib.check(_lib.load().gm_plan(s.id, 0, 0, 0, ctypes.byref(p)))
    n = 1024 * (outer + 1)
    assert p.mode == _lib.GM_MODE_PLANES and p.table_slots == n
    rup = lambda x: (x + 255) // 256 * 256  # noqa: E731
    assert p.table_bytes == rup(bytes_per_word * n) + rup(n // 256)
    _lib.check(_lib.load().gm_plan(s.id, 0, _lib.GM_F_WORDS16, 0, ctypes.byref(p)))
    assert p.table_bytes == rup(2 * n) + rup(n // 256)


@pytest.mark.parametrize("world,heaps", [(4, "31:31:31:31:31:127"), (8, "31:31:31:31:31:255")])
def test_planes_bench_shards_plan_8bit_words(world, heaps):
    """The 4- and 8-GPU bench shapes (root digit sums 281 / 409) plan 8-bit
    relative words: a 2^30-position shard's words are 1 GiB, not 2."""
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    s = GameSpec("sum_four_to_one", "heaps=" + heaps)
    for r in range(world):
        p = _lib.gm_plan_t()
        _lib.check(_lib.load().gm_plan_shard(s.id, r, world, 0, 0, ctypes.byref(p)))
        assert p.mode == _lib.GM_MODE_PLANES and p.table_slots == 1 << 30
        # 1 GiB of words + 4 MiB of reach bits (one per row) + the halo
        # slices (2 x 2^15 planes each way, 8-bit): 16-bit words alone would
        # be 2 GiB
        halo = (1 << 25) * ((r > 0) + (r + 1 < world))
        assert p.table_bytes == (1 << 30) + (1 << 22) + 2 * halo


def test_product_library_reads_no_lab_knob():
    """The measurement labs' A/B environment knobs (some of them write wrong
    words on purpose, e.g. GM_RK_DBG) and the failure tests' fault injector
    are compiled into the LAB build only (-DGM_LAB=1,
    libgamesman_hip_lab.so): the shipped library does not even hold their
    names, so no environment can select them."""
    knobs = [b"GM_RK_DBG", b"GM_RK_ORDER", b"GM_RK_SLICED", b"GM_FAULT_STAGED", b"GM_PLANE_STAGE_K",
             b"GM_PLANE_GRAPH", b"GM_PLANE_SPIN", b"GM_PLANE_FWD_FIRST", b"GM_PLANE_FWD", b"GM_PLANE_FLOW",
             b"GM_FAULT_FLOW", b"GM_PLANE_PAIR_RUNS", b"GM_PLANE_PAIR_MAX"]
    with open(os.path.join(ROOT, "gamesmanmpi_amd", "libgamesman_hip.so"), "rb") as f:
        prod = f.read()
    for k in knobs:
        assert k not in prod, k
    lab = os.path.join(ROOT, "gamesmanmpi_amd", "libgamesman_hip_lab.so")
    if os.path.exists(lab):
        with open(lab, "rb") as f:
            data = f.read()
        for k in (b"GM_RK_DBG", b"GM_FAULT_STAGED"):
            assert k in data, k
