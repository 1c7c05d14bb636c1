#!/usr/bin/env python3
"""Full-size validation of the real-game configs on one MI355X (writes one
JSON line per case).

  toot_and_otto_bitstring 5x4 (70,184,763 positions): GPU vs the oracle
      (oracle/, run on this host's CPU) by an order-independent checksum
      of every (canonical bytes, value, remoteness) row -- bit-exact parity
      at a size no committed fixture holds.
  toot_and_otto_bitstring 6x4 (1,187,212,827 positions, BASELINE config 3):
      counts, value histogram and root line vs SURVEY.md Appendix B (the
      survey's independent C++ probe); too large for the oracle here.
  othello_bit_new 4x4 (54,089): vs its golden table (also in pytest).

Usage: python tools/validate_games.py [toot54] [toot64] [othello44]
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")

SURVEY_B = {  # SURVEY.md Appendix B (positions, edges, W/L/T, root line)
    "5x4": (70184763, 226547754, (36388900, 23833441, 9962422), "LOSS in 20 moves"),
    "6x4": (1187212827, 4243234712, (659933325, 437913021, 89366481), "LOSS in 24 moves"),
}


def checksum(canon, lens, val, rem):
    """Order-independent 64-bit sum of a per-row mix of (bytes, value,
    remoteness); rows are (canon u8[n, w], lens, value, remoteness)."""
    n, w = canon.shape
    acc = np.zeros(n, np.uint64)
    for j in range(w):
        acc = (acc * np.uint64(0x100000001B3)) ^ canon[:, j].astype(np.uint64)
    acc ^= lens.astype(np.uint64) << np.uint64(56)
    acc = acc * np.uint64(0x9E3779B97F4A7C15) + (val.astype(np.uint64) << np.uint64(40)) + rem.astype(np.uint64)
    acc ^= acc >> np.uint64(29)
    acc *= np.uint64(0xBF58476D1CE4E5B9)
    acc ^= acc >> np.uint64(32)
    return int(acc.sum(dtype=np.uint64))


def gpu_solve(stem, params, positions=0):
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    spec = GameSpec(stem, params)
    s = Solver(spec, positions=positions)
    s.solve()  # warm-up (allocation, first-touch)
    t0 = time.perf_counter()
    r = s.solve()
    wall = time.perf_counter() - t0
    return spec, s, r, wall


def toot(L, H, with_oracle):
    key = "%dx%d" % (L, H)
    params = "length=%d,height=%d" % (L, H)
    spec, s, r, wall = gpu_solve("toot_and_otto_bitstring", params)
    out = {"case": "toot_" + key, "positions": r.positions, "edges": r.edges,
           "root": r.root_line, "gpu_solve_s": round(wall, 4),
           "gpu_ms_forward": r.ms_forward, "gpu_ms_backward": r.ms_backward,
           "positions_per_s": r.positions / wall}
    keys, val, rem = s.dump()
    out["value_hist_WLTD"] = [int((val == v).sum()) for v in range(4)]
    if key in SURVEY_B:
        P, E, hist, line = SURVEY_B[key]
        out["matches_survey_appendix_B"] = (r.positions == P and r.edges == E and
                                            tuple(out["value_hist_WLTD"][:3]) == hist
                                            and r.root_line == line)
    if with_oracle:
        canon, lens = spec.decode_batch(keys, stride=16)
        gsum = checksum(canon, lens, val, rem)
        del canon, lens
        from oracle.oracle import Game
        t0 = time.perf_counter()
        sol = Game("toot_and_otto_bitstring", params).solve(int(r.positions * 1.2))
        out["oracle_s"] = round(time.perf_counter() - t0, 2)
        c, cl, v, m = raw_dump(sol)
        osum = checksum(c, cl, v, m)
        out["oracle_positions"] = sol.count
        out["checksum_gpu"] = "%016x" % gsum
        out["checksum_oracle"] = "%016x" % osum
        out["bit_exact_vs_oracle"] = (gsum == osum and sol.count == r.positions
                                      and sol.root_line == r.root_line)
    print(json.dumps(out), flush=True)
    return out


def raw_dump(sol, stride=16):
    """Unsorted oracle dump (the checksum is order-independent)."""
    from oracle.oracle import lib
    n = sol.count
    canon = np.zeros((n, stride), np.uint8)
    clen = np.zeros(n, np.uint8)
    val = np.zeros(n, np.uint8)
    rem = np.zeros(n, np.uint32)
    rc = lib().or_dump(sol.h, canon.ctypes.data, stride, clen.ctypes.data,
                       val.ctypes.data, rem.ctypes.data)
    assert rc == 0
    return canon, clen, val, rem


def othello44():
    spec, s, r, wall = gpu_solve("othello_bit_new", "length=4,height=4")
    print(json.dumps({"case": "othello_4x4", "positions": r.positions,
                      "edges": r.edges, "root": r.root_line,
                      "gpu_solve_s": round(wall, 5)}), flush=True)


if __name__ == "__main__":
    todo = sys.argv[1:] or ["othello44", "toot54", "toot64"]
    for t in todo:
        if t == "toot54":
            toot(5, 4, with_oracle=True)
        elif t == "toot64":
            toot(6, 4, with_oracle=False)
        elif t == "othello44":
            othello44()
