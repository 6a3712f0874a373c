#!/bin/bash
# The driver's bench command (20 steps, 5 warm-up) with each step's batch whole (4 in flight, 8 queues)
# against the batch fanned out over contexts (--parts), alternating.  Each run has its own time limit;
# the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-parts}
for rep in ${REPS:-1 2}; do
  for cfg in "4 1 8" "2 4 16" "3 4 16" "1 4 8"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
        --pipeline $1 --parts $2 --hw-queues $3 > "$OUT/${TAG}_p$1_x$2_q$3_$rep.json" 2> "$OUT/${TAG}_p$1_x$2_q$3_$rep.err" || exit $?
    echo "$cfg rep $rep: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" "$OUT/${TAG}_p$1_x$2_q$3_$rep.json")"
  done
done
