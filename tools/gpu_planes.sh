# PLANES layout: parity tests + a timing probe on the GPU box
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_planes.py -x -v --timeout 300 --timeout-method thread 2>&1 | tee gpurun_out/planes_tests.log
timeout -k 10 300 python -u - <<'PY' 2>&1 | tee gpurun_out/planes_time.log
import time, torch, sys
sys.path.insert(0, ".")
from gamesmanmpi_amd.games import GameSpec
from gamesmanmpi_amd.solver import Solver
s = Solver(GameSpec("sum_four_to_one", "heaps=31:31:31:31:31:31"))
for i in range(3): s.solve()
torch.cuda.synchronize(); t0 = time.perf_counter()
for i in range(10): r = s.solve()
torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 10
print("2^30 solve %.3f ms, %.3g pos/s" % (dt * 1e3, r.positions / dt), r.root_line, r.extra, r.ms_forward, r.ms_backward)
s.set_kernel_timing(True); r = s.solve()
print("kernels: reach %.3f ms, resolve %.3f ms over %d launches" % (r.ms_expand_kernels, r.ms_resolve_kernels, r.n_resolve_launches))
PY
