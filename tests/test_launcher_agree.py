"""Under torchrun every rank must take the same multi-GPU path
(solver_launcher.agreed_ranked): a rank whose GPU cannot hold the
replicated RANKED table must not go to the md5 keyed path alone while its
peers solve RANKED -- their collectives would never match.  Two gloo ranks on
the CPU, ranked_fits monkeypatched to differ between them."""
import socket
import types

import pytest

from conftest import collect_workers


def _worker(rank, world, port, q, fits, layout):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gamesmanmpi_amd import solver_launcher as sl
        sl.ranked_fits = lambda spec, local, *a: fits[rank]
        spec = types.SimpleNamespace(name="toot_and_otto_bitstring")
        try:
            q.put((rank, "ranked" if sl.agreed_ranked(spec, layout, 0) else "keyed"))
        except SystemExit as e:
            q.put((rank, "exit: %s" % e))
    finally:
        dist.destroy_process_group()


def _run(fits, layout):
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, len(fits), port, q, fits, layout)) for r in range(len(fits))]
    for p in procs:
        p.start()
    return [c for _, c in collect_workers(q, procs, len(fits), limit=120)]


@pytest.mark.parametrize("fits,want", [((True, True), "ranked"), ((True, False), "keyed"),
                                       ((False, True), "keyed"), ((False, False), "keyed")])
def test_ranks_agree_on_the_path(fits, want):
    assert _run(fits, "auto") == [want, want]


def test_explicit_ranked_that_does_not_fit_everywhere_is_an_error():
    got = _run((True, False), "ranked")
    assert all(c.startswith("exit: --layout ranked") for c in got), got
    assert "this rank: fits" in got[0] and "this rank: does not fit" in got[1]


def test_other_layouts_skip_the_vote():
    # no collective at all: a layout that never takes the RANKED path
    assert _run((True, True), "bucketed") == ["keyed", "keyed"]
