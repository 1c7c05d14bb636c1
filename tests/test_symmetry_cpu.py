"""Symmetry hooks on the host (include/gamesman.h gm_symmetry; SURVEY.md
§8f rank 4): the descriptor's player_flip is a level-preserving involution,
canonical keys are orbit minima, games without symmetry_functions() refuse
the hook, and -- where the reference is mounted -- the reference module's
own symmetry_functions() agree with the descriptor's key maps."""
import os

import numpy as np
import pytest

from conftest import CASES, REFERENCE, has_reference, load_table


def test_flip_is_a_level_preserving_involution():
    from gamesmanmpi_amd.games import GameSpec
    spec = GameSpec("othello_bit_new", "length=4,height=4,symmetry=1")
    plain = GameSpec(*CASES["othello_4x4"])
    t = load_table("othello_4x4")
    keys = plain.encode_batch(t["canon"], t["clen"])
    f = spec.symmetry(keys, 0)
    assert (f != keys).all()
    np.testing.assert_array_equal(spec.symmetry(f, 0), keys)
    np.testing.assert_array_equal(plain.host_level(f), plain.host_level(keys))
    c = spec.symmetry(keys)
    np.testing.assert_array_equal(c, np.minimum(keys, f))
    np.testing.assert_array_equal(spec.symmetry(c), c)  # idempotent
    np.testing.assert_array_equal(plain.symmetry(keys), keys)  # no hook: identity
    root_flip = int(spec.symmetry(np.array([plain.root_key], np.uint64), 0)[0])
    assert spec.root_key == min(plain.root_key, root_flip)


def test_games_without_symmetry_functions_refuse_the_hook():
    from gamesmanmpi_amd import _lib
    from gamesmanmpi_amd.games import GameSpec
    for name, params in (("tic_tac_toe_np", "symmetry=1"),
                         ("sum_four_to_one", "heaps=3:3,symmetry=1")):
        with pytest.raises(_lib.GmError):
            GameSpec(name, params)


@pytest.mark.skipif(not has_reference(), reason="reference not mounted")
def test_reference_symmetry_functions_match_descriptor():
    from test_launcher import _load
    from gamesmanmpi_amd.games import GameSpec
    mod = _load(os.path.join(REFERENCE, "test_games", "othello_bit_new.py"),
                "gm_sym_test", length=4, height=4)
    spec = GameSpec("othello_bit_new", "length=4,height=4,symmetry=1")
    assert spec.verify_symmetries(mod, samples=150) == 150
    assert spec.verify(mod, samples=150) == 150
