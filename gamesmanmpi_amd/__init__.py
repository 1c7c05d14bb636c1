"""gamesmanmpi_amd -- MI355X-native strong solver for two-player abstract
strategy games, driven by game modules written against the GamesmanMPI
game-module API (initial_position / gen_moves / do_move / primitive).

The solve runs as hand-written HIP kernels for gfx950 behind the C-ABI in
include/gamesman.h (libgamesman_hip.so); PyTorch-ROCm only allocates the HBM
buffers and provides torch.distributed (RCCL) for multi-GPU runs.
"""
__version__ = "0.1.0"

WIN, LOSS, TIE, DRAW, UNDECIDED = 0, 1, 2, 3, 4


def __getattr__(name):  # lazy: importing the package must not need a GPU
    if name in ("Solver", "SolveResult", "solve"):
        from . import solver
        return getattr(solver, name)
    if name in ("GameSpec", "spec_for_module"):
        from . import games
        return getattr(games, name)
    raise AttributeError(name)
