"""Fake ``mpi4py.MPI``: per-rank Comm objects over pickled thread queues.

The reference calls: Get_rank/Get_size (solver_launcher.py:76-84),
Barrier (solver_launcher.py:45,98), send(obj, dest) (src/process.py:160,185),
probe(source=ANY_SOURCE) (src/process.py:172), recv(source=ANY_SOURCE)
(src/process.py:174) and Abort() (src/process.py:53)."""
import pickle
import queue
import threading

ANY_SOURCE = -1


class _Aborted(BaseException):
    """Raised inside every rank thread once some rank called Abort()."""


class World:
    def __init__(self, size):
        self.size = size
        self.queues = [queue.Queue() for _ in range(size)]
        self.aborted = threading.Event()
        self.messages = 0
        self._lock = threading.Lock()
        self.barrier = threading.Barrier(size)


class Comm:
    def __init__(self, world, rank):
        self.world = world
        self.rank = rank
        self._stash = None

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.world.size

    def Barrier(self):
        if self.world.size > 1:
            self.world.barrier.wait()

    def send(self, obj, dest):
        if self.world.aborted.is_set():
            raise _Aborted()
        with self.world._lock:
            self.world.messages += 1
        self.world.queues[dest].put(pickle.dumps(obj))

    def probe(self, source=ANY_SOURCE):
        if self._stash is not None:
            return True
        while True:
            if self.world.aborted.is_set():
                raise _Aborted()
            try:
                self._stash = self.world.queues[self.rank].get(timeout=0.05)
                return True
            except queue.Empty:
                continue

    def recv(self, source=ANY_SOURCE):
        if self._stash is None:
            self.probe(source)
        msg, self._stash = self._stash, None
        return pickle.loads(msg)

    def Abort(self, errorcode=0):
        self.world.aborted.set()
        raise _Aborted()


COMM_WORLD = None  # the generator builds per-rank Comm objects explicitly
