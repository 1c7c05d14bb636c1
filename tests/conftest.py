import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def has_reference():
    return os.path.isdir(os.path.join(REFERENCE, "test_games"))


@pytest.fixture(scope="session")
def golden_summary():
    import json
    with open(os.path.join(GOLDEN, "summary.json")) as f:
        return json.load(f)


# fixture name -> (game file stem, params) for both oracle and product
CASES = {
    "four_to_one": ("four_to_one", "start=4"),
    "four_to_one_20": ("four_to_one", "start=20"),
    "four_to_one_64": ("four_to_one", "start=64"),
    "mttt": ("mttt", ""),
    "tic_tac_toe_np": ("tic_tac_toe_np", ""),
    "othello_4x4": ("othello_bit_new", "length=4,height=4"),
    "toot_3x3": ("toot_and_otto_bitstring", "length=3,height=3"),
    "toot_4x3": ("toot_and_otto_bitstring", "length=4,height=3"),
    "toot_3x4": ("toot_and_otto_bitstring", "length=3,height=4"),
    "toot_4x4": ("toot_and_otto_bitstring", "length=4,height=4"),
    "sum_fto_3_3_3": ("sum_four_to_one", "heaps=3:3:3"),
    "sum_fto_4_4_4": ("sum_four_to_one", "heaps=4:4:4"),
    "sum_fto_2_5_7": ("sum_four_to_one", "heaps=2:5:7"),
    "sum_fto_6_6_6_6": ("sum_four_to_one", "heaps=6:6:6:6"),
}

# fixtures pinned by SAMPLES only (no full table): md5_owner.json rows and
# movegen vectors of BASELINE config 3 at its own size (test_toot_6x4_fixtures)
SAMPLED_CASES = {
    "toot_6x4": ("toot_and_otto_bitstring", "length=6,height=4"),
}
ALL_CASES = dict(CASES, **SAMPLED_CASES)


def load_table(name):
    import numpy as np
    path = os.path.join(GOLDEN, "tables", name + ".npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


def collect_workers(q, procs, world, limit=200):
    """The workers' results; fails at once when a worker dies (its peers
    would wait in a collective until the limit)."""
    import queue
    import time
    out, t0 = [], time.time()
    while len(out) < world:
        try:
            out.append(q.get(timeout=2))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > limit:
                for p in procs:
                    p.kill()
                pytest.fail("worker exit codes %s after %.0f s" % ([p.exitcode for p in procs], time.time() - t0))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])
