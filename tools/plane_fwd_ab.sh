# A/B of the forward's enqueue order (GM_PLANE_FWD_FIRST: 1 = before the backward's first launch), PLANES bench
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
for v in 0 1; do
  GM_PLANE_FWD_FIRST=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-keyed --steps 20 --warmup 3 > gpurun_out/r05aw_f$v.log 2>&1 || exit 1
  echo "fwd_first=$v $(grep '"metric"' gpurun_out/r05aw_f$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phase_ms"]; print(round(d["ms_per_step"],4), round(p["solve_wall"],4), round(p["backward"],4))')"
done; done
