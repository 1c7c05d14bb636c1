# A/B of the end-of-solve wait (GM_PLANE_SPIN: poll vs hipStreamSynchronize), PLANES bench, twice each
cd $GRAFT_REPO_ROOT
for i in 1 2; do
for v in 1 0; do
  GM_PLANE_SPIN=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-keyed --steps 20 --warmup 3 > gpurun_out/r05au_s$v.log 2>&1 || exit 1
  echo "spin=$v $(grep '"metric"' gpurun_out/r05au_s$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phase_ms"]; print(round(d["ms_per_step"],4), round(p["solve_wall"],4), round(p["backward"],4))')"
done; done
