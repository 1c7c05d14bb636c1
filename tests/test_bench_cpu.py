"""bench.py's host logic (no GPU): the weak-scaling shapes, the closed forms
every step is checked against (against the oracle on small sums), the
roofline byte model and the kernel names the roofline line reports."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_weak_scaling_shapes_hold_2_30_positions_per_gpu():
    for n in (1, 2, 4, 8):
        heaps = bench.heaps_for(n)
        P, E, _ = bench.expected(heaps)
        assert P == n << 30
    assert bench.heaps_for(1) == [31] * 6
    with pytest.raises(SystemExit):
        bench.heaps_for(3)


@pytest.mark.parametrize("heaps", [[3, 3, 3], [2, 5, 7], [4, 4, 4], [6, 6, 6, 6], [1, 1], [0, 5]])
def test_closed_forms_match_the_oracle(heaps):
    from oracle.oracle import Game  # checker only
    P, E, root = bench.expected(heaps)
    sol = Game("sum_four_to_one", "heaps=" + ":".join(map(str, heaps))).solve(1 << 20)
    assert (sol.count, sol.edges, sol.root_line.split()[0]) == (P, E, root)


def test_roofline_byte_model():
    fwd, bwd = bench.algorithmic_bytes(1000, 10000, "dense", word_bytes=2)
    assert fwd == (10000 + 1000) / 8 and bwd == 2.125 * 1000 + 2 * 10000
    fwd, bwd = bench.algorithmic_bytes(1000, 10000, "dense")
    assert bwd == 4.125 * 1000 + 4 * 10000
    assert bench.algorithmic_bytes(10, 100, "hashed") == (24 * 10 + 8 * 100, 12 * 10 + 12 * 100)
    assert bench.model_8d_bytes(10, 100) == 36 * 10 + 20 * 100


def test_roofline_kernel_names(monkeypatch):
    for k in ("GM_DENSE_RESOLVE", "GM_DENSE_SWEEP", "GM_DENSE_PIPE"):
        monkeypatch.delenv(k, raising=False)
    assert bench.dense_resolve_kernel(16) == "k_dense_resolve8p"
    assert bench.dense_resolve_kernel(16, world=4) == "k_dense_resolve8c"
    assert bench.dense_resolve_kernel(32) == "k_dense_resolve4p"
    monkeypatch.setenv("GM_DENSE_PIPE", "0")
    assert bench.dense_resolve_kernel(32) == "k_dense_resolve4"
