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


def load_table(name):
    import numpy as np
    path = os.path.join(GOLDEN, "tables", name + ".npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)  # allow_pickle=False (default)
    return {k: z[k] for k in z.files}
