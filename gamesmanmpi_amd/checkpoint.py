"""Level-granular checkpoint / resume of one-GPU solves (SURVEY.md §8f
rank 2).

The reference's only persistence is its write-through shelve files
(src/cache_dict.py:38-60): a rank that dies loses its job queue and pending
counters, so a run restarts from the root.  Here a solve is 2T steps
(forward levels 0..T-1, backward levels T-1..0; include/gamesman.h
gm_solver_set_steps) and the whole of its state lives in three caller-owned
device buffers -- table, level store, scratch.  A checkpoint is those
buffers written to a directory after some step, plus the plan and the
kernel-family flags they were sized by; resuming loads them into a fresh
solver of the same plan and runs the remaining steps.  The solution is the
oracle's (tests/test_gpu_checkpoint.py).

    save(solver, directory, step)          # after solve_steps(.., step) stopped
    solver, step = restore(directory)      # a fresh Solver holding the state
    result = solve_checkpointed(solver, directory, every=16)

Layout of `directory`: meta.json, table.bin, levels.bin, scratch.bin (raw
bytes of the buffers).  Safety rules:
  * a directory that exists and holds anything but a checkpoint of ours
    (meta.json with our format, our .bin files) is refused, never touched;
  * save() writes `directory`.tmp, then moves the previous checkpoint to
    `directory`.old and the new one into place; only our own files are ever
    removed.  A crash between the two moves leaves the previous checkpoint
    in `directory`.old, which restore() and latest() fall back to;
  * buffers stream to and from disk in fixed-size chunks through one pinned
    host buffer: a checkpoint of a 200+ GB table needs no host copy of it.
"""
import json
import os

import numpy as np

from . import _lib
from .games import GameSpec
from .solver import Solver

FORMAT = 2
_NAMES = ("table", "levels", "scratch")
_OURS = {"meta.json"} | {n + ".bin" for n in _NAMES}
CHUNK = 256 << 20  # bytes per host staging chunk


class NotACheckpoint(ValueError):
    """The directory exists and is not a checkpoint this module wrote."""


def _plan_dict(solver):
    p = solver.plan
    return {"mode": int(p.mode), "table_bytes": int(p.table_bytes),
            "table_slots": int(p.table_slots),
            "level_capacity": int(p.level_capacity),
            "scratch_bytes": int(p.scratch_bytes),
            "max_levels": int(p.max_levels)}


def is_checkpoint(directory):
    """True if `directory` holds a checkpoint of this format."""
    try:
        read_meta(directory)
        return True
    except (OSError, ValueError):
        return False


def check_target(directory):
    """Refuse a directory that exists, is not empty and is not one of our
    checkpoints (raises NotACheckpoint; nothing is modified)."""
    if not os.path.exists(directory):
        return
    if not os.path.isdir(directory):
        raise NotACheckpoint("%s exists and is not a directory" % directory)
    names = set(os.listdir(directory))
    if not names:
        return
    if not is_checkpoint(directory) or not names <= _OURS:
        raise NotACheckpoint("%s exists and holds files that are not a gamesmanmpi_amd "
                             "checkpoint; refusing to overwrite it" % directory)


def check_scratch_dir(directory):
    """Refuse a save()'s own scratch directory (`directory`.tmp / .old) if
    it holds anything but checkpoint files.  Unlike check_target it needs no
    meta.json: save() writes meta.json last, so a crash while the .bin
    files stream out leaves a .tmp without one, and the next save() must
    be able to reuse it."""
    if not os.path.exists(directory):
        return
    if not os.path.isdir(directory):
        raise NotACheckpoint("%s exists and is not a directory" % directory)
    if not set(os.listdir(directory)) <= _OURS:
        raise NotACheckpoint("%s holds files that are not a gamesmanmpi_amd checkpoint's; "
                             "refusing to overwrite it" % directory)


def _remove_ours(directory):
    """Delete only the files a checkpoint consists of, then the directory if
    that left it empty."""
    if not os.path.isdir(directory):
        return
    for n in _OURS:
        try:
            os.remove(os.path.join(directory, n))
        except FileNotFoundError:
            pass
    try:
        os.rmdir(directory)
    except OSError:
        pass


def _stream_out(t, path, torch):
    """Device tensor -> file, CHUNK bytes at a time through pinned memory."""
    flat = t.view(torch.uint8).reshape(-1)
    n = flat.numel()
    stage = torch.empty(min(CHUNK, max(n, 1)), dtype=torch.uint8, pin_memory=True)
    with open(path, "wb") as fh:
        for a in range(0, n, CHUNK):
            b = min(n, a + CHUNK)
            stage[:b - a].copy_(flat[a:b])
            fh.write(stage[:b - a].numpy().tobytes())


def _stream_in(t, path, torch):
    flat = t.view(torch.uint8).reshape(-1)
    n = flat.numel()
    if os.path.getsize(path) != n:
        raise ValueError("%s holds %d bytes, the plan %d" % (path, os.path.getsize(path), n))
    stage = torch.empty(min(CHUNK, max(n, 1)), dtype=torch.uint8, pin_memory=True)
    view = stage.numpy()  # the pinned chunk as a writable host array: read straight into it
    with open(path, "rb") as fh:
        for a in range(0, n, CHUNK):
            b = min(n, a + CHUNK)
            if fh.readinto(memoryview(view[:b - a])) != b - a:
                raise ValueError("%s ended early" % path)
            flat[a:b].copy_(stage[:b - a])


def save(solver, directory, step):
    """Write `solver`'s buffers after step `step` (its last solve_steps call
    stopped there) to `directory`."""
    if solver.world != 1:
        raise ValueError("checkpoints cover one-GPU solves")
    directory = directory.rstrip("/")
    check_target(directory)
    torch = solver.torch
    torch.cuda.synchronize(solver.device)
    tmp, old = directory + ".tmp", directory + ".old"
    check_scratch_dir(tmp)
    check_scratch_dir(old)
    _remove_ours(tmp)
    os.makedirs(tmp)
    for name, t in zip(_NAMES, solver.buffers):
        _stream_out(t, os.path.join(tmp, name + ".bin"), torch)
    plan = _plan_dict(solver)
    meta = {"format": FORMAT, "game": solver.spec.name,
            "params": solver.spec.params, "layout": solver.layout,
            # what "auto" resolved to in this build: a later build may
            # resolve "auto" differently, and restore() falls back to this
            "layout_resolved": _lib.MODE_NAMES[plan["mode"]],
            "positions_hint": solver.positions_hint,
            "max_table_bytes": solver.max_table_bytes,
            "flags": solver.flags,
            "plan": plan, "step": int(step),
            "steps": solver.steps}
    with open(os.path.join(tmp, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    _remove_ours(old)
    if os.path.isdir(directory) and os.listdir(directory):
        os.replace(directory, old)
    elif os.path.isdir(directory):
        os.rmdir(directory)
    os.replace(tmp, directory)
    _remove_ours(old)


def read_meta(directory):
    with open(os.path.join(directory, "meta.json")) as fh:
        meta = json.load(fh)
    if meta.get("format") != FORMAT:
        raise ValueError("unknown checkpoint format %r" % meta.get("format"))
    return meta


def latest(directory):
    """The directory holding the newest complete checkpoint: `directory`,
    or `directory`.old when a save was interrupted between its two moves;
    None if neither holds one."""
    directory = directory.rstrip("/")
    for d in (directory, directory + ".old"):
        if is_checkpoint(d):
            return d
    return None


def restore(directory, device=None):
    """A fresh Solver holding the checkpointed state, and the step to
    resume at.  The plan and the kernel-family flags come from meta.json,
    not from the environment."""
    import torch
    src = latest(directory)
    if src is None:
        raise FileNotFoundError("no checkpoint in %s (or %s.old)" % (directory, directory.rstrip("/")))
    meta = read_meta(src)
    spec = GameSpec(meta["game"], meta["params"])

    def make(layout):
        return Solver(spec, positions=meta["positions_hint"], device=device,
                      layout=layout, max_table_bytes=meta["max_table_bytes"],
                      flags=meta.get("flags", 0))
    solver = make(meta["layout"])
    if _plan_dict(solver) != meta["plan"] and meta["layout"] == "auto":
        # "auto" resolves differently in this build: rebuild the layout the
        # checkpoint was planned with (older checkpoints: from its plan mode)
        resolved = meta.get("layout_resolved") or _lib.MODE_NAMES.get(int(meta["plan"]["mode"]))
        if resolved:
            # free the first table before the second is allocated: both at
            # once would peak at, e.g., toot 6x4's RANKED plus BUCKETED tables
            solver._free()
            del solver
            torch.cuda.empty_cache()
            solver = make(resolved)
    if _plan_dict(solver) != meta["plan"]:
        raise ValueError("checkpoint plan %r does not match this build's %r"
                         % (meta["plan"], _plan_dict(solver)))
    for name, t in zip(_NAMES, solver.buffers):
        _stream_in(t, os.path.join(src, name + ".bin"), torch)
    torch.cuda.synchronize(solver.device)
    return solver, int(meta["step"])


def solve_checkpointed(solver, directory, every, first=0, keep=False, max_regrow=4):
    """Run `solver` from step `first` to the end, checkpointing into
    `directory` every `every` steps; removes the checkpoint's files when the
    solve completes unless keep=True.  A keyed table that fills during the
    forward pass (positions_hint too small) is regrown and the solve
    restarted from step 0, as Solver.solve() does.  That includes a resumed
    solve (first > 0) whose checkpoint was taken with a plan that is too
    small: the stale checkpoint is dropped as soon as the buffers regrow
    (a later restore would otherwise rebuild the small plan and fail at the
    same level on every resume), and the solve restarts from the root."""
    if every < 1:
        raise ValueError("every must be >= 1")
    check_target(directory)
    step, total = int(first), solver.steps
    grown = 0
    while True:
        stop = step + every
        try:
            r = solver.solve_steps(step, stop if stop < total else 0)
        except _lib.TableFull:
            if grown >= max_regrow:
                raise
            grown += 1
            solver.positions_hint *= 2
            solver._alloc(solver.positions_hint)
            _remove_ours(directory.rstrip("/"))
            _remove_ours(directory.rstrip("/") + ".old")
            step = 0
            continue
        if r is not None:
            if not keep:
                _remove_ours(directory.rstrip("/"))
                _remove_ours(directory.rstrip("/") + ".old")
            return r
        save(solver, directory, stop)
        step = stop
