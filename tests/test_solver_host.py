"""Host logic of Solver and checkpoint that needs no GPU: layout="auto"
falls back to the hashed table when a bucketed plan hits GM_ELIMIT (once,
and only for "auto"), and a checkpoint restore rebuilds the layout the
checkpoint was planned with when "auto" resolves differently in this build.
The C-ABI calls are replaced by stand-ins; no kernel runs."""
import types

import pytest

from gamesmanmpi_amd import _lib
from gamesmanmpi_amd import solver as solver_mod


class _Dev:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _fake_solver(layout, mode, errors):
    """A Solver whose _alloc records the planned layout and whose library
    raises `errors` (a list, consumed in order) from gm_solver_solve."""
    s = object.__new__(solver_mod.Solver)
    s.layout = layout
    s._planned_layout = layout
    s.world = 1
    s.positions_hint = 1000
    s.device = "cuda:0"
    s.torch = types.SimpleNamespace(cuda=types.SimpleNamespace(device=lambda d: _Dev()))
    s._h = object()
    s.plan = types.SimpleNamespace(mode=mode)
    s.allocs = []

    def alloc(positions):
        s.allocs.append((s._planned_layout, positions))
        s.plan = types.SimpleNamespace(mode=_lib.GM_MODE_HASHED if s._planned_layout == "hashed" else mode)
    s._alloc = alloc
    s._result = lambda r: "solved as %s" % s._planned_layout
    lib = types.SimpleNamespace()

    def solve(h, r):
        if errors:
            return errors.pop(0)
        return 0
    lib.gm_solver_solve = solve
    return s, lib


def _run(monkeypatch, s, lib, msg="limit"):
    monkeypatch.setattr(_lib, "load", lambda: lib)
    monkeypatch.setattr(_lib, "check", lambda rc: (_ for _ in ()).throw(_lib.LayoutLimit(rc, msg)) if rc == _lib.GM_ELIMIT
                        else (_ for _ in ()).throw(_lib.TableFull(rc, msg)) if rc == _lib.GM_EFULL else None)
    return s.solve()


def test_auto_bucketed_limit_falls_back_to_hashed(monkeypatch):
    s, lib = _fake_solver("auto", _lib.GM_MODE_BUCKETED, [_lib.GM_ELIMIT])
    assert _run(monkeypatch, s, lib) == "solved as hashed"
    assert s.allocs == [("hashed", 1000)]
    assert s.layout == "auto"  # the request is unchanged; the plan is hashed


def test_auto_falls_back_only_once(monkeypatch):
    s, lib = _fake_solver("auto", _lib.GM_MODE_BUCKETED, [_lib.GM_ELIMIT, _lib.GM_ELIMIT])
    with pytest.raises(_lib.LayoutLimit):
        _run(monkeypatch, s, lib)
    assert s.allocs == [("hashed", 1000)]


def test_explicit_bucketed_keeps_the_limit(monkeypatch):
    s, lib = _fake_solver("bucketed", _lib.GM_MODE_BUCKETED, [_lib.GM_ELIMIT])
    with pytest.raises(_lib.LayoutLimit):
        _run(monkeypatch, s, lib)
    assert s.allocs == []


def test_table_full_still_regrows(monkeypatch):
    s, lib = _fake_solver("auto", _lib.GM_MODE_HASHED, [_lib.GM_EFULL, _lib.GM_EFULL])
    assert _run(monkeypatch, s, lib) == "solved as auto"
    assert s.allocs == [("auto", 2000), ("auto", 4000)]


def test_checkpoint_restore_uses_the_resolved_layout(monkeypatch, tmp_path):
    from gamesmanmpi_amd import checkpoint
    plan = {"mode": _lib.GM_MODE_DENSE, "table_bytes": 10, "table_slots": 1, "level_capacity": 1,
            "scratch_bytes": 1, "max_levels": 3}
    made = []

    class FakeSolver:
        def __init__(self, spec, positions, device, layout, max_table_bytes, flags):
            made.append(layout)
            mode = _lib.GM_MODE_DENSE if layout == "dense" else _lib.GM_MODE_PLANES
            self.plan = types.SimpleNamespace(mode=mode, table_bytes=10, table_slots=1, level_capacity=1,
                                              scratch_bytes=1, max_levels=3)
            self.buffers = ()
            self.device = device

        def _free(self):  # the first table goes before the second is made
            made.append("free")

    monkeypatch.setattr(checkpoint, "Solver", FakeSolver)
    monkeypatch.setattr(checkpoint, "GameSpec", lambda g, p: (g, p))
    monkeypatch.setattr(checkpoint, "latest", lambda d: d)
    import torch
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    for meta_layout in ({"layout_resolved": "dense"}, {}):  # new checkpoints, and older ones (plan mode)
        made.clear()
        meta = dict(format=checkpoint.FORMAT, game="sum_four_to_one", params="heaps=31:31:3", layout="auto",
                    positions_hint=0, max_table_bytes=0, flags=0, plan=plan, step=4, steps=6, **meta_layout)
        monkeypatch.setattr(checkpoint, "read_meta", lambda d, m=meta: m)
        s, step = checkpoint.restore(str(tmp_path))
        assert made == ["auto", "free", "dense"] and step == 4
        assert int(s.plan.mode) == _lib.GM_MODE_DENSE
