#!/usr/bin/env python3
"""Load balance of sharded dense solves: for the bench's
weak-scaling shape 31^5 x (32N-1), the critical path of a level-synchronous
solve is sum over levels of the busiest rank's positions, relative to one
rank's share.  Compares one contiguous block per rank with round-robin
blocks of B top values.

    python tools/shard_balance.py
"""
import numpy as np


def level_hist(heaps):
    d = np.array([1.0])
    for h in heaps:
        d = np.convolve(d, np.ones(h + 1))
    return d


def critical_path(base, world, owner):
    top = len(owner)
    per = np.zeros((world, len(base) + top - 1))
    for t in range(top):
        per[owner[t], t:t + len(base)] += base
    return per.max(axis=0).sum() / per.sum(axis=1).mean()


def main():
    base = level_hist([31] * 5)
    for n in (2, 4, 8):
        top = 32 * n
        rows = {"contiguous x32": critical_path(base, n, [t // 32 for t in range(top)])}
        for b in (16, 8, 4):
            rows["round-robin x%d" % b] = critical_path(base, n, [(t // b) % n for t in range(top)])
        print("N=%d  " % n + "  ".join("%s: %.2f" % kv for kv in rows.items()))


if __name__ == "__main__":
    main()
