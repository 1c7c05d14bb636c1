#!/usr/bin/env python3
"""Throughput of the md5 owner rule on the device (gm_owner: the register-
resident MD5 of str(pos) mod P) over N synthetic keys of a game:
    python tools/owner_rate.py [GAME] [PARAMS] [N_LOG2] [P]"""
import ctypes
import json
import sys
import time

sys.path.insert(0, ".")


def main():
    import torch
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    game = sys.argv[1] if len(sys.argv) > 1 else "toot_and_otto_bitstring"
    params = sys.argv[2] if len(sys.argv) > 2 else "length=6,height=4"
    n = 1 << (int(sys.argv[3]) if len(sys.argv) > 3 else 28)
    P = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    spec = GameSpec(game, params)
    keys = torch.randint(0, 1 << 60, (n,), dtype=torch.int64, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    L = _lib.load()
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(L.gm_owner(spec.id, keys.data_ptr(), n, P, out.data_ptr(), None))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(json.dumps({"game": game, "params": params, "keys": n, "P": P, "ms": dt * 1e3, "owners_per_s": n / dt,
                      "hist": torch.bincount(out.long(), minlength=P).tolist()}))


if __name__ == "__main__":
    main()
