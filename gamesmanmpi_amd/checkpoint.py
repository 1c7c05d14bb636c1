"""Level-granular checkpoint / resume of one-GPU solves (SURVEY.md §8f
rank 2).

The reference's only persistence is its write-through shelve files
(src/cache_dict.py:38-60): a rank that dies loses its job queue and pending
counters, so a run restarts from the root.  Here a solve is 2T steps
(forward levels 0..T-1, backward levels T-1..0; include/gamesman.h
gm_solver_set_steps) and the whole of its state lives in three caller-owned
device buffers -- table, level store, scratch.  A checkpoint is those
buffers written to a directory after some step, plus the plan they were
sized by; resuming loads them into a fresh solver of the same plan and runs
the remaining steps.  The solution itself is identical to an uninterrupted
solve (tests/test_gpu_checkpoint.py).

    save(solver, directory, step)          # after solve_steps(.., step) stopped
    solver, step = restore(directory)      # a fresh Solver holding the state
    result = solve_checkpointed(solver, directory, every=16)

Layout of `directory`: meta.json, table.bin, levels.bin, scratch.bin (raw
bytes of the buffers).  save() writes into `directory`.tmp and renames, so
a crash mid-write leaves the previous checkpoint intact.
"""
import json
import os
import shutil

import numpy as np

from . import _lib
from .games import GameSpec
from .solver import Solver

FORMAT = 1
_NAMES = ("table", "levels", "scratch")


def _plan_dict(solver):
    p = solver.plan
    return {"mode": int(p.mode), "table_bytes": int(p.table_bytes),
            "table_slots": int(p.table_slots),
            "level_capacity": int(p.level_capacity),
            "scratch_bytes": int(p.scratch_bytes),
            "max_levels": int(p.max_levels)}


def save(solver, directory, step):
    """Write `solver`'s buffers after step `step` (its last solve_steps call
    stopped there) to `directory`."""
    if solver.world != 1:
        raise ValueError("checkpoints cover one-GPU solves")
    solver.torch.cuda.synchronize(solver.device)
    tmp = directory.rstrip("/") + ".tmp"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    for name, t in zip(_NAMES, solver.buffers):
        t.cpu().numpy().view(np.uint8).tofile(os.path.join(tmp, name + ".bin"))
    meta = {"format": FORMAT, "game": solver.spec.name,
            "params": solver.spec.params, "layout": solver.layout,
            "positions_hint": solver.positions_hint,
            "max_table_bytes": solver.max_table_bytes,
            "plan": _plan_dict(solver), "step": int(step),
            "steps": solver.steps}
    with open(os.path.join(tmp, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    old = directory.rstrip("/") + ".old"
    shutil.rmtree(old, ignore_errors=True)
    if os.path.isdir(directory):
        os.replace(directory, old)
    os.replace(tmp, directory)
    shutil.rmtree(old, ignore_errors=True)


def read_meta(directory):
    with open(os.path.join(directory, "meta.json")) as fh:
        meta = json.load(fh)
    if meta.get("format") != FORMAT:
        raise ValueError("unknown checkpoint format %r" % meta.get("format"))
    return meta


def restore(directory, device=None):
    """A fresh Solver holding the checkpointed state, and the step to
    resume at."""
    import torch
    meta = read_meta(directory)
    spec = GameSpec(meta["game"], meta["params"])
    solver = Solver(spec, positions=meta["positions_hint"], device=device,
                    layout=meta["layout"],
                    max_table_bytes=meta["max_table_bytes"])
    if _plan_dict(solver) != meta["plan"]:
        raise ValueError("checkpoint plan %r does not match this build's %r"
                         % (meta["plan"], _plan_dict(solver)))
    for name, t in zip(_NAMES, solver.buffers):
        raw = np.fromfile(os.path.join(directory, name + ".bin"), dtype=np.uint8)
        dst = t.view(torch.uint8).reshape(-1)
        if raw.size != dst.numel():
            raise ValueError("%s.bin holds %d bytes, the plan %d"
                             % (name, raw.size, dst.numel()))
        dst.copy_(torch.from_numpy(raw))
    torch.cuda.synchronize(solver.device)
    return solver, int(meta["step"])


def solve_checkpointed(solver, directory, every, first=0, keep=False):
    """Run `solver` from step `first` to the end, checkpointing into
    `directory` every `every` steps; removes the checkpoint when the solve
    completes unless keep=True."""
    if every < 1:
        raise ValueError("every must be >= 1")
    step, total = int(first), solver.steps
    while True:
        stop = step + every
        r = solver.solve_steps(step, stop if stop < total else 0)
        if r is not None:
            if not keep:
                shutil.rmtree(directory, ignore_errors=True)
            return r
        save(solver, directory, stop)
        step = stop
