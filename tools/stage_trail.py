#!/usr/bin/env python3
"""Pipeline model of the staged PLANES deal from kernel
traces of ONE-STREAM shard groups (tools/r05_session.sh stage: every key of
every shard alone on the GPU, so a launch's duration is what it costs on a
GPU of its own).

Per trace: the last solve's resolve launches of the LAST shard (a shard with a
predecessor: its geometry is the receiving ranks'), mapped to keys -- the
launch list is the key sequence with the narrow keys at both ends merged into
one-workgroup runs (k_plane_run), whose duration is split evenly over the keys
they hold.  Then, for rank r of N:

    T_r(K) = max(T_r(K - 1), wait_r(K)) + d(K)
    wait_r(K) = T_{r-1}(K + B - 1) + lat + row_bytes(K / k) / bw   if K % k == 0 (row K/k's halo)

(rank r's key k s reads halo row s, final on rank r-1 after its key
B - 1 + k s; sent as one message of 2 x planes(s) KiB).  In the real run the
receiver's narrow keys cannot merge across a halo wait: they pay their own
launch, `floor`.  The step is T_{N-1}(last key).  Not a measurement of an
N-GPU run: RCCL's transfers are priced by --lat / --bw.

  python tools/stage_trail.py gpurun_out/r05g [--lat 15e-6] [--bw 50e9] [--floor 5.5e-6]
"""
import argparse
import csv
import glob
import json
import os
import re

import numpy as np

B = 32


def classes(ndig=3, base=32):
    c = np.ones(1)
    for _ in range(ndig):
        c = np.convolve(c, np.ones(base))
    return c


def key_widths(k, R):
    cls = classes()
    K = B - 1 + k * (R - 1) + 1
    w = np.zeros(K)
    for s in range(R):
        for o in range(B):
            w[o + k * s] += cls[s]
    return w


def last_solve_launches(trace):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fin = [i for i, r in enumerate(rows) if "k_plane_finish" in r["Kernel_Name"]]
    # the last solve: between the previous solve's finish kernels (one per
    # shard, back to back) and its own
    first = [i for j, i in enumerate(fin) if j == 0 or fin[j - 1] != i - 1]
    lo = fin[fin.index(first[-1]) - 1] + 1 if len(first) > 1 else 0
    seq = [r for r in rows[lo:first[-1]] if "k_plane_resolve" in r["Kernel_Name"] or "k_plane_run" in r["Kernel_Name"]]
    return [((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9, "k_plane_run" in r["Kernel_Name"]) for r in seq]


def per_key(launches, k, world, narrow=32):
    """d(K) of the last shard of the one-stream group (shard after shard on
    the stream)."""
    R = 94
    w = key_widths(k, R)
    K = len(w)
    # the last shard: from its head run (in the one-stream group nothing
    # waits, so its narrow head keys merge) to its tail run (it sends no rows)
    runs = [i for i, (_, r) in enumerate(launches) if r]
    mine = launches[runs[-2]:]
    lo = 0
    while lo < K and w[lo] <= narrow:
        lo += 1
    hi = K
    while hi > 0 and w[hi - 1] <= narrow:
        hi -= 1
    # runs: the narrow head (if merged) and tail
    d = np.zeros(K)
    i = 0
    key = 0
    if mine[0][1]:  # head run
        d[:lo] = mine[0][0] / lo
        key, i = lo, 1
    for dur, run in mine[i:]:
        if run:  # tail run
            d[key:] = dur / (K - key)
            key = K
            break
        d[key] = dur
        key += 1
    if key != K:
        raise ValueError("launches do not map onto %d keys (k=%d): ended at %d" % (K, k, key))
    return d, w, (lo, hi)


def model(d, w, k, N, lat, bw, floor, narrow_head, narrow_tail):
    cls = classes()
    K = len(d)
    T = np.zeros((N, K))
    for r in range(N):
        prev = 0.0
        for key in range(K):
            dk = d[key]
            if (r > 0 and key < narrow_head) or (r < N - 1 and key >= narrow_tail):
                dk = max(dk, floor)  # no run across halo waits / row sends: a launch each
            start = prev
            if r > 0 and key % k == 0 and key // k < len(cls):
                s = key // k
                start = max(start, T[r - 1][min(key + B - 1, K - 1)] + lat + 2 * cls[s] * 1024 / bw)
            T[r][key] = start + dk
            prev = T[r][key]
    return float(T[N - 1][-1])


def row_deal(trace, world, lat, bw):
    """The row deal (heap 1 in 32-row slabs): keys = plane levels, rank r's
    level l waits for rank r - 1's level l and its two-row halo (n(l) x 64 B):
        T_r(l) = max(T_r(l - 1), T_{r-1}(l) + lat + 64 n(l) / bw) + d(l)
    d(l): the last shard's launches (one per level, no runs) of the one-stream
    group."""
    L = last_solve_launches(trace)
    n = len(L) // world
    d = np.array([x for x, _ in L[-n:]])
    cls = np.ones(1)
    for _ in range(4):
        cls = np.convolve(cls, np.ones(32))
    if len(d) != len(cls):
        raise ValueError("%d launches per shard, %d levels" % (len(d), len(cls)))
    out = {}
    for N in (2, 4, 8):
        T = np.zeros((N, len(d)))
        for r in range(N):
            prev = 0.0
            for l in range(len(d)):
                start = prev if r == 0 else max(prev, T[r - 1][l] + lat + 64 * cls[l] / bw)
                T[r][l] = start + d[l]
                prev = T[r][l]
        out[N] = float(T[N - 1][-1]) * 1e3
    return d, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--lat", type=float, default=15e-6)
    ap.add_argument("--bw", type=float, default=50e9)
    ap.add_argument("--floor", type=float, default=5.5e-6)
    a = ap.parse_args()
    out = []
    for t in sorted(glob.glob(os.path.join(a.root, "rows_w*", "run_kernel_trace.csv"))):
        world = int(re.search(r"rows_w(\d+)", t).group(1))
        d, step = row_deal(t, world, a.lat, a.bw)
        rec = {"deal": "rows", "world": world, "keys": len(d), "sweep_ms": d.sum() * 1e3,
               "max_level_ms": d.max() * 1e3, "step_ms": step, "lat_us": a.lat * 1e6, "bw_GBps": a.bw / 1e9,
               "trace": t}
        out.append(rec)
        print(json.dumps(rec))
    for t in sorted(glob.glob(os.path.join(a.root, "stage_w*_k*", "run_kernel_trace.csv"))):
        m = re.search(r"stage_w(\d+)_k(\d+)", t)
        world, k = int(m.group(1)), int(m.group(2))
        d, w, (lo, hi) = per_key(last_solve_launches(t), k, world)
        win = max(d[i:i + B].sum() for i in range(len(d) - B + 1))
        rec = {"world": world, "k": k, "keys": len(d), "sweep_ms": d.sum() * 1e3, "window32_ms": win * 1e3,
               "step_ms": {N: model(d, w, k, N, a.lat, a.bw, a.floor, lo, hi) * 1e3 for N in (2, 4, 8)},
               "lat_us": a.lat * 1e6, "bw_GBps": a.bw / 1e9, "trace": t}
        out.append(rec)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
