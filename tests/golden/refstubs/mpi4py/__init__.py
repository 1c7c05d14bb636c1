"""In-process fake of ``mpi4py`` so the reference job loop (src/process.py)
runs in THIS container for fixture generation.  One thread per rank; messages
are pickled into per-rank queues (what mpi4py's lowercase API does on the
wire).  Fixture-generation infrastructure only; never shipped."""
from . import MPI  # noqa: F401
