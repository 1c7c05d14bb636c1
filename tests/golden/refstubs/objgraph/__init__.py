"""Stand-in for ``objgraph`` (imported unconditionally by src/debug.py:2).
Fixture-generation infrastructure only."""


def get_leaking_objects():
    return []
