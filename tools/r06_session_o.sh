#!/bin/bash
# full -m gpu suite + smoke on the k_plane_flow tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r06al
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -3 $out/smoke.txt
POISON=1 REPS=10 timeout -k 10 250 python3 tools/flow_check.py heaps=31:31:1:127 heaps=31:31:3:63 heaps=31:31:1:1:63 heaps=31:31:7:7:7:7 > $out/stress.txt 2>&1 || { cat $out/stress.txt; exit 1; }
echo "stress: $(grep -c 'bad words 0 ' $out/stress.txt) clean of $(grep -c 'bad words' $out/stress.txt)"
for i in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-keyed --no-cpu-baseline > $out/bench$i.json 2> $out/bench$i.err || { tail $out/bench$i.err; exit 1; }
python3 -c "import json;d=json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], round(d['phase_ms']['resolve_kernels'],4), d['roofline']['frac'])"
done
