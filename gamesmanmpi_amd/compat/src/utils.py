"""Constants and helpers game modules import as ``src.utils``.

Values and behaviour match the reference's src/utils.py:3-48 exactly (game
files return these codes from primitive()); ``game_module`` is set by the
launcher like solver_launcher.py:41-42 does."""
from functools import reduce as _reduce

WIN, LOSS, TIE, DRAW, UNDECIDED = range(5)
PRIMITIVES = (WIN, LOSS, TIE, DRAW)
PRIMITIVE_REMOTENESS = 0
UNKNOWN_REMOTENESS = -1
game_module = None

_NAMES = ("WIN", "LOSS", "TIE", "DRAW", "UNDECIDED")
STATE_MAP = {code: name.lower() for code, name in enumerate(_NAMES)}


def negate(state):
    """WIN <-> LOSS; every other code is its own negation."""
    if state == WIN:
        return LOSS
    if state == LOSS:
        return WIN
    return state


def to_str(state):
    return _NAMES[state]


def reduce_singleton(function, data):
    """reduce() that also accepts one element (called as function(x, None))."""
    if len(data) == 1:
        return function(data[0], None)
    return _reduce(function, data)
