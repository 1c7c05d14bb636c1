"""Pin the CPU oracle to the reference: every golden table (generated from the
reference's own game modules), the ordered move-generation vectors, and the
root lines printed by the reference's own job loop (src/process.py:47-52)."""
import json
import os

import numpy as np
import pytest

from conftest import CASES, GOLDEN, load_table
from oracle.oracle import Game


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden_table(name, golden_summary):
    stem, params = CASES[name]
    info = golden_summary[name]
    sol = Game(stem, params).solve(max(1024, 2 * info["positions"]))
    assert sol.count == info["positions"]
    assert sol.edges == info["edges"]
    assert sol.root_line == info["root_line"]
    t = load_table(name)
    if t is None:  # large case: sha256 of the sorted table only
        if info["positions"] > 4_000_000:
            pytest.skip("too large")
        import hashlib
        c, cl, v, r = sol.dump(stride=t["canon"].shape[1] if t else 7)
        h = hashlib.sha256()
        h.update(c.tobytes())
        h.update(v.tobytes())
        h.update(r.tobytes())
        assert h.hexdigest() == info["table_sha256"]
        return
    c, cl, v, r = sol.dump(stride=t["canon"].shape[1])
    np.testing.assert_array_equal(c, t["canon"])
    np.testing.assert_array_equal(cl, t["clen"])
    np.testing.assert_array_equal(v, t["value"])
    np.testing.assert_array_equal(r, t["remoteness"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_movegen_vectors(name):
    path = os.path.join(GOLDEN, "movegen", name + ".json")
    if not os.path.exists(path):
        pytest.skip("no vectors")
    stem, params = CASES[name]
    g = Game(stem, params)
    with open(path) as f:
        rows = json.load(f)
    for row in rows:
        prim, kids = g.expand(bytes.fromhex(row["pos"]))
        assert prim == row["primitive"], row["pos"]
        assert [k.hex() for k in kids] == row["children"], row["pos"]


def test_reference_job_loop_root_lines():
    """Root lines the reference's own Process.run printed (fake-MPI harness,
    tests/golden/make_golden.py) equal the oracle's."""
    path = os.path.join(GOLDEN, "reference_runs.json")
    with open(path) as f:
        runs = json.load(f)
    want = {"four_to_one": Game("four_to_one", "start=4").solve().root_line,
            "mttt": Game("mttt").solve().root_line}
    seen = 0
    for key, run in runs.items():
        game = key.rsplit("_n", 1)[0]
        assert run["errors"] == [], run
        assert run["lines"] == [want[game]], (key, run["lines"])
        seen += 1
    assert seen >= 4


def test_fto_chain_closed_form():
    """Four-To-One KAT: LOSS iff x%3==0; rem(3k)=2k,
    rem(3k+1)=rem(3k+2)=2k+1."""
    g = Game("four_to_one", "start=300")
    sol = g.solve(4096)
    for x in range(0, 301):
        v, r = sol.lookup(str(x).encode())
        assert v == (1 if x % 3 == 0 else 0), x
        assert r == (2 * (x // 3) if x % 3 == 0 else 2 * (x // 3) + 1), x


# ---- multi-threaded restatements (oracle/oracle_mt.c) --------------------
@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_mt_levels_match_golden_table(name, golden_summary):
    """The tier-synchronous OpenMP solver reproduces every golden table
    position for position (it pins tests/golden/checksums.json)."""
    stem, params = CASES[name]
    info = golden_summary[name]
    t = load_table(name)
    if t is None and info["positions"] > 4_000_000:
        pytest.skip("too large")
    sol = Game(stem, params).solve_levels(keep=True)
    assert (sol.count, sol.edges, sol.root_line) == (
        info["positions"], info["edges"], info["root_line"])
    assert sol.stats["primitives"] == info["primitives"]
    if t is None:
        return
    for i in range(len(t["value"])):
        c = bytes(t["canon"][i, :t["clen"][i]])
        assert sol.lookup(c) == (t["value"][i], t["remoteness"][i]), c


@pytest.mark.parametrize("params", ["start=20", "start=301"])
def test_oracle_mt_rows_fto(params):
    """Row solver on the single-heap chain: counts, root and the closed
    form of every position."""
    g = Game("four_to_one", params)
    r = g.solve_rows()
    d = g.solve(4096)
    assert (r.count, r.edges, r.root_line) == (d.count, d.edges, d.root_line)
    n = int(params.split("=")[1])
    for x in range(n + 1):
        w = r.word(x)
        assert (w & 3) == (1 if x % 3 == 0 else 0)
        assert (w >> 2) == (2 * (x // 3) if x % 3 == 0 else 2 * (x // 3) + 1)


@pytest.mark.parametrize("heaps", ["3:3:3", "2:5:7", "6:9:4:11", "7:0:3", "15:15:15:15"])
def test_oracle_mt_rows_and_levels_agree(heaps):
    """Row solver == level solver == scalar DFS on sums of heaps, word for
    word, and the two multi-threaded checksums agree."""
    g = Game("sum_four_to_one", "heaps=" + heaps)
    r = g.solve_rows()
    st = r.refresh(True)
    lv = g.solve_levels(keep=True)
    d = g.solve(1 << 17)
    assert (r.count, r.edges, r.root_line) == (d.count, d.edges, d.root_line)
    assert (lv.count, lv.edges, lv.root_line) == (d.count, d.edges, d.root_line)
    assert st["checksum"] == lv.stats["checksum"]
    c, cl, v, m = d.dump(stride=24)
    for i in range(len(v)):
        rank = int(bytes(c[i, :cl[i]]))
        w = r.word(rank)
        assert (w & 3, w >> 2) == (v[i], m[i]), rank


def test_golden_checksums_small_cases_reproduce():
    """tests/golden/checksums.json entries the oracle recomputes in seconds
    (the large ones, toot 5x4 / 6x4 and 2^30 sums, are regenerated by
    tests/golden/make_checksums.py)."""
    with open(os.path.join(GOLDEN, "checksums.json")) as f:
        gold = json.load(f)
    done = 0
    for name in ("othello_4x4", "toot_4x4", "sum_15x5"):
        if name not in gold:
            continue
        e = gold[name]
        g = Game(e["game"], e["params"])
        if e["solver"].endswith("rows"):
            st = g.solve_rows().refresh(True)
        else:
            st = g.solve_levels(keep=False).stats
        assert "%016x" % st["checksum"] == e["checksum"], name
        assert st["positions"] == e["positions"] and st["edges"] == e["edges"]
        done += 1
    assert done >= 3


def test_golden_checksums_match_survey_appendix_b():
    """toot 5x4 / 6x4 fingerprints: counts, histogram and root line equal the
    survey's independent C++ probe."""
    with open(os.path.join(GOLDEN, "checksums.json")) as f:
        gold = json.load(f)
    want = {"toot_5x4": (70184763, 226547754, 36388900, 23833441, 9962422, "LOSS in 20 moves"),
            "toot_6x4": (1187212827, 4243234712, 659933325, 437913021, 89366481, "LOSS in 24 moves")}
    for name, (P, E, w, l, t, line) in want.items():
        if name not in gold:
            pytest.skip("%s not generated yet" % name)
        e = gold[name]
        assert (e["positions"], e["edges"], e["win"], e["loss"], e["tie"], e["root_line"]) == (P, E, w, l, t, line)
