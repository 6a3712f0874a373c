#!/bin/bash
# Parity of a variant build (plane + shortcut suites), then a steady-state A/B of variant builds at
# the bench default, two alternating rounds.  Usage: gpu_ab_variants.sh TAG "parity_variant" "v1 v2 ..."
# ("-" = the in-tree library).  Each step has its own time limit; the script stops at a failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=$1; PV=$2; VARS=$3
lib() { if [ "$1" = "-" ]; then echo ""; else echo "$GRAFT_REPO_ROOT/variants/$1/libpitt_seg.so"; fi; }
for v in $PV; do
  PITT_LIB_PATH=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py tests/test_shortcuts_gpu.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/${TAG}_parity_$v.log" 2>&1 || exit $?
done
for rep in 1 2; do
  for v in $VARS; do
    PITT_LIB_PATH=$(lib $v) timeout -k 10 200 python3 bench.py --steps 40 --no-extras --no-cpu-baseline \
        > "$OUT/${TAG}_${v}_$rep.json" 2> "$OUT/${TAG}_${v}_$rep.err" || exit $?
  done
done
