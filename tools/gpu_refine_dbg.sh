#!/bin/bash
# k_refine per-role cycles ($PITT_REFINE_DEBUG) for a list of "tag:lib:producers:mode" variants, at
# pipeline 1 (k_refine alone on the chip).  lib "-" = the in-tree library, otherwise a variants/ dir.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
for v in "$@"; do
  IFS=: read -r tag lib p m <<< "$v"
  if [ "$lib" = "-" ]; then unset PITT_LIB_PATH; else export PITT_LIB_PATH="$GRAFT_REPO_ROOT/variants/$lib/libpitt_seg.so"; fi
  PITT_REFINE_MODE=$m PITT_REFINE_DEBUG=1 PITT_REFINE_PRODUCERS=$p timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 \
      --pipeline 1 --no-extras --no-cpu-baseline > "$OUT/dbg_$tag.json" 2> "$OUT/dbg_$tag.err" || exit $?
done
