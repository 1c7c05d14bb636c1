"""Model of one PLANES shard's backward at N GPUs: the
level-synchronous deal (blocks of 8 top values dealt over the ranks, one
halo exchange per plane level on the critical path) against the staged
pipeline (one block of E/N top values per rank, planes resolved by key
o + k s with no level barrier, halo rows streamed to rank + 1).

Inputs are measured one-GPU figures: c = device time per plane at full
occupancy (k_plane_resolve 16-bit words: 2.77 ms / 2^20 planes), floor =
the time of a narrow launch (profiles/r03g_plane_ab.txt level times), link =
xGMI bandwidth per direction, lat = one RCCL transfer's latency.  Not a
measurement: it picks k and states the expected weak-scaling step time.

  python tools/stage_model.py [--c 2.64e-9] [--floor 5e-6] [--bw 70e9] [--lat 12e-6]
"""
import argparse

import numpy as np


def classes(ndig=3, base=32):
    d = np.ones(base)
    c = np.ones(1)
    for _ in range(ndig):
        c = np.convolve(c, d)
    return c  # c[s] = planes of lower-digit sum s per top value


def level_sync(N, c, floor, bw, lat, B=8, pb=2048):
    cls = classes()
    E = 32 * N
    S = E - 1 + len(cls) - 1
    work = np.zeros((N, S + 1))
    send = np.zeros((N, S + 1))
    for b in range(E // B):
        r = b % N
        for o in range(B):
            t = b * B + o
            work[r, t:t + len(cls)] += cls
            if o >= B - 2 and b + 1 < E // B:
                send[r, t:t + len(cls)] += cls
    comp = work.max(axis=0) * c + 2 * floor
    link = send.max(axis=0) * pb / bw + lat
    return float(np.maximum(comp, link).sum())


def staged(N, k, c, floor, lat, B=32):
    cls = classes()
    R = len(cls)
    K = B - 1 + k * (R - 1) + 1
    w = np.zeros(K)
    for s in range(R):
        for o in range(B):
            w[o + k * s] += cls[s]
    dur = np.maximum(w * c, floor)
    T = np.zeros((N, K))
    for r in range(N):
        prev = 0.0
        for key in range(K):
            start = prev
            if r > 0 and key % k == 0:  # row key/k of the previous rank: final after its key B-1+key
                start = max(start, T[r - 1][min(key + B - 1, K - 1)] + lat)
            T[r][key] = start + dur[key]
            prev = T[r][key]
    return float(T[N - 1][-1]), float(dur.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c", type=float, default=2.64e-9)
    ap.add_argument("--floor", type=float, default=5e-6)
    ap.add_argument("--bw", type=float, default=70e9)
    ap.add_argument("--lat", type=float, default=12e-6)
    a = ap.parse_args()
    for N in (2, 4, 8):
        ls = level_sync(N, a.c, a.floor, a.bw, a.lat)
        best = min((staged(N, k, a.c, a.floor, a.lat + 30e-6)[0], k) for k in range(1, 13))
        print("N=%d  level-sync %.2f ms   staged %.2f ms at k=%d" % (N, ls * 1e3, best[0] * 1e3, best[1]))
        print("      staged by k: " + "  ".join("%d:%.2f" % (k, staged(N, k, a.c, a.floor, a.lat + 30e-6)[0] * 1e3)
                                             for k in (2, 3, 4, 5, 6, 7, 8, 10)))


if __name__ == "__main__":
    main()
