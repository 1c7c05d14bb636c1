"""Synthetic benchmark game: a disjunctive SUM of K Four-To-One heaps, written
against the reference's game-module API (README.md:28-88;
docs/source/game_modules.rst:11-33) so the reference's own solvers could load
it.  Each heap follows test_games/four_to_one.py:7-22 exactly: from a heap of
1 the only move is -1, otherwise -1 or -2; a move changes ONE heap.  The
position with every heap at 0 is the only primitive, a LOSS for the player to
move (four_to_one.py:19-22), so K=1 is four_to_one itself.

A position is the mixed-radix rank sum(h_i * prod_{j<i}(HEAPS[j]+1)) as a
plain int, hashable and str()-stable like four_to_one's int positions.  Heap
0 is the least-significant digit.  HEAPS (the start heights) may be edited
before solving, like the reference games' "Feel free to edit" constants.
SURVEY.md §8d: HEAPS=(31,)*6 gives 32**6 = 2**30 positions, 187 levels,
11.4375 moves per position on average.
"""
import src.utils

HEAPS = (31, 31, 31, 31, 31, 31)


def _strides():
    s, out = 1, []
    for h in HEAPS:
        out.append(s)
        s *= h + 1
    return out


def heaps_of(pos):
    out = []
    for h in HEAPS:
        out.append(pos % (h + 1))
        pos //= h + 1
    return out


def initial_position():
    return sum(h * s for h, s in zip(HEAPS, _strides()))


def gen_moves(pos):
    moves = []
    for i, h in enumerate(heaps_of(pos)):
        if h >= 1:
            moves.append((i, -1))
        if h >= 2:
            moves.append((i, -2))
    return moves


def do_move(pos, move):
    i, d = move
    return pos + d * _strides()[i]


def primitive(pos):
    if pos == 0:
        return src.utils.LOSS
    return src.utils.UNDECIDED
