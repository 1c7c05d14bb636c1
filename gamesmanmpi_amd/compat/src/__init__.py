"""Importable stand-in for the reference's ``src`` package, so game files
written against the reference (``import src.utils``, e.g.
test_games/four_to_one.py:5) load unchanged under this solver."""
