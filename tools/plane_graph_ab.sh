cd $GRAFT_REPO_ROOT
for i in 1 2; do
for g in 1 0; do  # GM_PLANE_GRAPH: whole-solve graph replay vs plain launches
  GM_PLANE_GRAPH=$g timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-keyed --steps 20 --warmup 3 > gpurun_out/r05ae_g$g.log 2>&1 || exit 1
  echo "graph=$g $(grep '"metric"' gpurun_out/r05ae_g$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["phase_ms"])')"
done; done
