#!/bin/bash
# Process-count sweep in the shape of the reference's testing.sh:6-38:
#   tools/testing.sh GAME_FILE FROM TO REPS [-l]
# runs the launcher under torchrun with FROM..TO processes (one per GPU),
# REPS times each, appending wall times to profile/time_results.txt and the
# printed root lines to profile/solve_results.txt.  -l also runs the
# single-process solve (the counterpart of solve_local.py) and then checks
# that every run printed the same root line -- the comparison the
# reference's -l run was for (its solve_local.py prints "Draw" for every
# game, SURVEY §0.1, so there it never matched).
set -u
game=$1; from=$2; to=$3; reps=$4; local_run=${5:-}
mkdir -p profile
echo "Beginning testing for $game from $from to $to, $reps tests each" > profile/time_results.txt
echo "Beginning testing for $game from $from to $to, $reps tests each" > profile/solve_results.txt
for i in $(seq "$from" "$to"); do
  for j in $(seq 1 "$reps"); do
    for f in profile/time_results.txt profile/solve_results.txt; do
      printf '\nTesting with %s processes\n---------\n' "$i" >> "$f"
    done
    start=$(date +%s.%N)
    timeout -k 10 1200 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$i" \
      --master-addr 127.0.0.1 --master-port $((29500 + i)) \
      -m gamesmanmpi_amd.solver_launcher "$game" >> profile/solve_results.txt 2>> profile/time_results.txt
    end=$(date +%s.%N)
    echo "real $(python3 -c "print(round($end - $start, 3))")s" >> profile/time_results.txt
  done
done
echo Done testing distributed solver
if [ "$local_run" = "-l" ]; then
  echo Testing with local solver
  for f in profile/time_results.txt profile/solve_results.txt; do
    printf '\nTesting with local, non-distributed solver\n---------\n' >> "$f"
  done
  start=$(date +%s.%N)
  timeout -k 10 1200 python -m gamesmanmpi_amd.solver_launcher "$game" >> profile/solve_results.txt 2>> profile/time_results.txt
  end=$(date +%s.%N)
  echo "real $(python3 -c "print(round($end - $start, 3))")s" >> profile/time_results.txt
  lines=$(grep -E '^(WIN|LOSS|TIE|DRAW) in [0-9]+ moves$' profile/solve_results.txt | sort -u | wc -l)
  if [ "$lines" = "1" ]; then
    echo "All runs agree: $(grep -E '^(WIN|LOSS|TIE|DRAW) in' profile/solve_results.txt | head -1)"
  else
    echo "Runs DISAGREE:"; grep -E '^(WIN|LOSS|TIE|DRAW) in' profile/solve_results.txt | sort | uniq -c
    exit 1
  fi
fi
echo Done with all tests
