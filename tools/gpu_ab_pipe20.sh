#!/bin/bash
# The driver's bench command (--steps 20 --warmup 5) at pipeline depth 3 and 4 (8 queues), three
# alternating rounds, timed pass only.  Each step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-p20}
for rep in 1 2 3; do
  for p in 3 4; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --pipeline $p --no-extras --no-cpu-baseline \
        > "$OUT/${TAG}_p${p}_$rep.json" 2> "$OUT/${TAG}_p${p}_$rep.err" || exit $?
  done
done
