#!/bin/bash
# A/B of variant builds with the driver's bench command (--steps 20 --warmup 5), timed pass only,
# three alternating rounds.  Usage: gpu_ab_variants20.sh TAG "v1 v2 ..." ("-" = the in-tree library).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=$1; VARS=$2
lib() { if [ "$1" = "-" ]; then echo ""; else echo "$GRAFT_REPO_ROOT/variants/$1/libpitt_seg.so"; fi; }
for rep in 1 2 3; do
  for v in $VARS; do
    PITT_LIB_PATH=$(lib $v) timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
        > "$OUT/${TAG}_${v}_$rep.json" 2> "$OUT/${TAG}_${v}_$rep.err" || exit $?
  done
done
