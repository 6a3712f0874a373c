#!/bin/bash
# Steady-state A/B of refinement knobs at the bench default (4 in flight, 8 queues), two alternating
# rounds: the default; two producers; the chain without its adds (PITT_REFINE_MODE=6, results wrong:
# what the chain's issue costs); the A6 fast mode for scale.  Each step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-abr}
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_def_$rep.json" 2>/dev/null || exit $?
  PITT_REFINE_PRODUCERS=2 timeout -k 10 200 python3 bench.py --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_p2_$rep.json" 2>/dev/null || exit $?
  PITT_REFINE_MODE=6 timeout -k 10 200 python3 bench.py --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_noadd_$rep.json" 2>/dev/null || exit $?
done
