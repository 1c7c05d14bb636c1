"""Diagnostic: read a dense solve's reach bitmap and word table back and
check them against the closed-form state space (valid slots, counts)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from gamesmanmpi_amd.games import GameSpec
from gamesmanmpi_amd.solver import Solver

params = sys.argv[1] if len(sys.argv) > 1 else "heaps=7:7:7:7"
heaps = [int(h) for h in params.split("=")[1].split(":")]
spec = GameSpec("sum_four_to_one", params)
s = Solver(spec, layout="dense")
r = s.solve()
table = s._tensors[0].cpu().numpy()
T = sum(heaps) + 1
base = [h + 1 for h in heaps]
W = int(np.prod(base[1:]))
Wb = (W + 63) // 64 * 64
words_bytes = (T * W * 4 + 255) // 256 * 256
bits = np.unpackbits(table[words_bytes:words_bytes + T * Wb // 8].view(np.uint8), bitorder="little").reshape(T, Wb)[:, :W]
words = table[:T * W * 4].view(np.uint32).reshape(T, W)
p = np.arange(W)
s_p = np.zeros(W, np.int64)
rest = p.copy()
for b in base[1:]:
    s_p += rest % b
    rest //= b
tot_valid = 0
for L in range(T):
    S = sum(heaps) - L
    valid = (s_p <= S) & (S - s_p <= heaps[0])
    nb = int(bits[L].sum()); nv = int(valid.sum()); bad = int((bits[L].astype(bool) & ~valid).sum())
    miss = int((~bits[L].astype(bool) & valid).sum())
    tot_valid += nv
    if bad or miss:
        print("level", L, "bits", nb, "valid", nv, "set-on-hole", bad, "valid-unset", miss)
print("result positions", r.positions, "edges", r.edges, "bit total", int(bits.sum()), "valid total", tot_valid)
