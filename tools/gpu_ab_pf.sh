#!/bin/bash
# The chain's block-boundary prefetch (PITT_REFINE_MODE=10) against the default (2): parity of the
# plane suites under mode 10, per-role cycles at pipeline 1, then the driver's bench command, three
# alternating rounds.  Each step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-pf}
timeout -k 10 300 python -u -m pytest tests/test_score_paths_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "refine_mode10" > "$OUT/${TAG}_pytest.log" 2>&1 || exit $?
for m in 2 10; do
  PITT_REFINE_MODE=$m PITT_REFINE_DEBUG=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --pipeline 1 --no-extras \
      --no-cpu-baseline > "$OUT/${TAG}_dbg_m$m.json" 2> "$OUT/${TAG}_dbg_m$m.err" || exit $?
done
for rep in 1 2 3; do
  for m in 2 10; do
    PITT_REFINE_MODE=$m timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
        > "$OUT/${TAG}_m${m}_$rep.json" 2> "$OUT/${TAG}_m${m}_$rep.err" || exit $?
  done
done
