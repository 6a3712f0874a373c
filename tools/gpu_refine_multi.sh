#!/bin/bash
# k_refine_multi: the plane parity suite under every refinement variant, then the steady-state A/B
# of frames per refine block (1, 2, 3) at the bench default, two alternating rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-rm}
timeout -k 10 600 python -u -m pytest tests/test_score_paths_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "frames" > "$OUT/${TAG}_pytest.log" 2>&1 || exit $?
for rep in 1 2; do
  for F in 1 2 3; do
    PITT_REFINE_FRAMES=$F timeout -k 10 200 python3 bench.py --steps 40 --no-extras --no-cpu-baseline \
        > "$OUT/${TAG}_f${F}_$rep.json" 2> "$OUT/${TAG}_f${F}_$rep.err" || exit $?
  done
done
