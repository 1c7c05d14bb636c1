"""Host enqueue cost of a one-table PLANES solve, and blocking vs queued
steps (tools/, diagnostic).  python3 tools/async_probe.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from gamesmanmpi_amd.games import GameSpec
    from gamesmanmpi_amd.solver import Solver
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    s = Solver(GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31"))
    for _ in range(3):
        s.solve()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        r = s.solve()
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t0) / K * 1e3
    print("blocking: %.4f ms/step (last solve host wall %.4f ms, device backward %.4f)" % (tb, r.ms_total, r.ms_backward))
    for depth in (1, 2, 4, 8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tickets, enq, res = [], [], []
        for _ in range(K):
            if len(tickets) == depth:
                res.append(s.collect(tickets.pop(0)))
            a = time.perf_counter()
            tickets.append(s.solve_async())
            enq.append(time.perf_counter() - a)
        for t in tickets:
            res.append(s.collect(t))
        torch.cuda.synchronize()
        tq = (time.perf_counter() - t0) / K * 1e3
        enq.sort()
        spans = sorted(x.ms_total for x in res)
        print("queued depth %d: %.4f ms/step; host enqueue per solve median %.4f ms max %.4f; device span median %.4f ms"
              % (depth, tq, enq[len(enq) // 2] * 1e3, enq[-1] * 1e3, spans[len(spans) // 2]))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
