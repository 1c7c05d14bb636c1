"""A three-position game whose two non-root positions move to each other
forever: no position on the cycle ever resolves (the reference's job loop
never finishes on it); the graph path must report it instead of hanging."""
import src.utils


def initial_position():
    return 0


def gen_moves(pos):
    return [1]


def do_move(pos, move):
    return 1 if pos != 1 else 2


def primitive(pos):
    return src.utils.UNDECIDED
