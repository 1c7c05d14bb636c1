"""Tic-tac-toe on a 3x3 int8 grid, written for these tests against the
game-module API (README.md:28-88) with the rules of the reference's
test_games/tic_tac_toe_np.py:7-61: 0 empty, 1 moves
first, then 2; a completed line of one player's marks is a LOSS for the
player to move, else a full board is a TIE.  It has no device descriptor
under this file name, so the launcher solves it through the host-enumerated
graph path (gamesmanmpi_amd/generic.py).  Positions are numpy arrays, whose
str() is the position identity, as in the reference's own file."""
import numpy as np

import src.utils

LINES = [[(r, 0), (r, 1), (r, 2)] for r in range(3)] + \
        [[(0, c), (1, c), (2, c)] for c in range(3)] + \
        [[(0, 0), (1, 1), (2, 2)], [(0, 2), (1, 1), (2, 0)]]


def initial_position():
    return np.zeros((3, 3), dtype=np.int8)


def _to_move(grid):
    ones = int((grid == 1).sum())
    twos = int((grid == 2).sum())
    return 2 if ones > twos else 1


def gen_moves(grid):
    who = _to_move(grid)
    return [(who, (r, c)) for r in range(3) for c in range(3) if grid[r, c] == 0]


def do_move(grid, move):
    who, (r, c) = move
    nxt = grid.copy()
    nxt[r, c] = who
    return nxt


def primitive(grid):
    for line in LINES:
        a, b, c = (int(grid[p]) for p in line)
        if a != 0 and a == b == c:
            return src.utils.LOSS
    if not (grid == 0).any():
        return src.utils.TIE
    return src.utils.UNDECIDED
