#!/bin/bash
# A/B of the first-chunk scorers: bench.py with $PITT_LANE_SCORE = 0 / 1, alternating, plus a rocprof
# kernel trace of each (k_score per-launch durations).  Each run has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-ab}
for rep in 1 2; do
  for m in 0 1; do
    PITT_LANE_SCORE=$m timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline \
        > "$OUT/${TAG}_lane${m}_${rep}.json" 2> "$OUT/${TAG}_lane${m}_${rep}.err" || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  PITT_LANE_SCORE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof${m}" -o p -f csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --no-extras --no-cpu-baseline > "$OUT/${TAG}_prof${m}.log" 2>&1 || exit $?
done
