#!/usr/bin/env python3
"""Step model of toot's md5 shards of the RANKED layout (gm_ranked_shard.h)
at N GPUs, from a kernel trace of the N-shard group solved on ONE stream of
one GPU (tools/rk_shard_run.py N ... one: every kernel alone on the GPU, so
its duration is what it costs on a GPU of its own).

Per rank: its share of every kernel of the last solve (the trace holds all N
shards' launches: sums / N), plus the level exchange, which the one-GPU group
does as device copies and N GPUs do over xGMI: every rank sends its level
pack (~1/N of the level's words) to each of the N - 1 others, one link per
peer on a fully connected node, all links at once, per level
    xfer(L) = lat + (words(L) / N) / bw
Summed over the levels that is 25 lat + positions / (N bw).  The backward
levels run one after another (level L - 1 reads level L's exchanged words).

  python tools/rk_shard_model.py gpurun_out/r05r_rk8 N [--lat 20e-6] [--bw 50e9] [--positions 1187212827]
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_kernel(trace):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last solve: everything after the last group's set-up (k_rko_owner:
    # rk_shard_run.py builds the group anew for every solve)
    lo = max(i for i, r in enumerate(rows) if "k_rko_owner" in r["Kernel_Name"]) + 1
    t = collections.defaultdict(float)
    n = collections.Counter()
    for r in rows[lo:]:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        k = k.split("<")[0] + ("<OWN>" if "true>" in k else "")
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        n[k] += 1
    return t, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("world", type=int)
    ap.add_argument("--lat", type=float, default=20e-6)
    ap.add_argument("--bw", type=float, default=50e9)
    ap.add_argument("--positions", type=float, default=1187212827)
    ap.add_argument("--levels", type=int, default=25)
    ap.add_argument("--one_gpu_ms", type=float, default=12.2)
    a = ap.parse_args()
    trace = glob.glob(os.path.join(a.root, "**", "run_kernel_trace.csv"), recursive=True)[0]
    t, n = per_kernel(trace)
    N = a.world
    setup = {"k_rko_owner"}
    share = {k: v / N * 1e3 for k, v in t.items() if k not in setup and "copyBuffer" not in k}
    xfer = (a.levels * a.lat + a.positions / (N * a.bw)) * 1e3
    step = sum(share.values()) + xfer
    out = {"world": N, "per_rank_kernel_ms": {k: round(v, 3) for k, v in sorted(share.items(), key=lambda x: -x[1])},
           "kernels_ms": round(sum(share.values()), 3), "xfer_ms": round(xfer, 3), "lat_us": a.lat * 1e6,
           "bw_GBps_per_link": a.bw / 1e9, "step_ms": round(step, 3), "one_gpu_ms": a.one_gpu_ms,
           "speedup": round(a.one_gpu_ms / step, 3), "trace": trace}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
