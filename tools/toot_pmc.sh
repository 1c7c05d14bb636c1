# Kernel stats + PMC passes (HBM bytes, L2 hits, atomics) of one hashed
# toot 6x4 solve (BASELINE config 3): bash tools/toot_pmc.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/toot_pmc}
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" hashed)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- "${cmd[@]}" > "$out/stats.log" 2>&1 || exit 1
echo stats ok
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- "${cmd[@]}" > "$out/fetch.log" 2>&1 || exit 1
echo fetch ok
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- "${cmd[@]}" > "$out/write.log" 2>&1 || exit 1
echo write ok
timeout -s KILL 300 rocprofv3 --pmc TCC_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/atomic" -o run -- "${cmd[@]}" > "$out/atomic.log" 2>&1 || exit 1
echo atomic ok
