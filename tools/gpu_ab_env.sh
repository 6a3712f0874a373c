#!/bin/bash
# A/B of a runtime knob read from the environment when a context is created:
#   tools/gpu_ab_env.sh TAG VAR "v1 v2 ..." [extra bench args]
# bench.py per value (two alternating rounds), then a rocprof kernel trace per value at pipeline 1
# (each kernel alone on the chip).  Every GPU step has its own time limit; the script stops at the
# first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=$1; VAR=$2; VALS=$3; shift 3
for rep in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline "$@" \
        > "$OUT/${TAG}_${v}_${rep}.json" 2> "$OUT/${TAG}_${v}_${rep}.err" || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for v in $VALS; do
  export "$VAR=$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof${v}" -o p -f csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --pipeline 1 --no-extras --no-cpu-baseline \
      > "$OUT/${TAG}_prof${v}.log" 2>&1 || exit $?
done
