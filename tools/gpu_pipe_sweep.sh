#!/bin/bash
# Pipeline depth x hardware queues sweep of bench.py (batches in flight).  Each run has its own time
# limit; the chain stops at the first failure.
#   tools/gpu_pipe_sweep.sh TAG STEPS "depth queues" ...   (default: 40 steps, the round-3 grid)
# With C5=1 a kernel + HIP API trace of config 5 follows.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-pipe}; STEPS=${2:-40}
shift 2 2>/dev/null
CFGS=("$@"); [ ${#CFGS[@]} -eq 0 ] && CFGS=("3 4" "4 4" "4 8" "5 8" "6 8")
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps $STEPS --warmup 5 --no-extras --no-cpu-baseline --pipeline $1 --hw-queues $2 \
      > "$OUT/${TAG}_s${STEPS}_p$1_q$2.json" 2> "$OUT/${TAG}_s${STEPS}_p$1_q$2.err" || exit $?
  echo "$cfg: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" "$OUT/${TAG}_s${STEPS}_p$1_q$2.json")"
done
if [ "${C5:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/${TAG}_c5" -o c5 -f csv -- \
      python3 "$GRAFT_REPO_ROOT/tools/config5_run.py" 3 > "$OUT/${TAG}_c5.log" 2>&1 || exit $?
fi
