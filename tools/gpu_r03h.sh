#!/bin/bash
# Round-3 re-entry check: the -m gpu suite and smoke on the rebuilt library, the A/B of k_score's
# inside-slab shortcut (PITT_INSIDE_CULL 0/1: bench lines + a rocprof kernel trace each at pipeline
# 1), then the pipeline depth x hardware queue sweep at the driver's 20 steps.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG=${1:-r03h}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $?
bash tools/gpu_ab_env.sh "${TAG}_ins" PITT_INSIDE_CULL "0 1" || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
for f in "$OUT/${TAG}_ins"_*_*.json; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['kernels']['k_score.first']['avg_launch_us'])" "$f")"
done
[ "${SWEEP:-1}" = 1 ] && bash tools/gpu_pipe_sweep.sh "$TAG" 20 "4 8" "5 8" "5 16" "6 16" "4 8" "5 16" "6 16"
exit 0
