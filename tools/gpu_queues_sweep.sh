#!/bin/bash
# bench.py pipeline sweep with more hardware queues per process: gpurun_out/qs_q<Q>_p<N>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for q in 8; do
    for p in 3 4 6; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 3 --pipeline $p --no-cpu-baseline \
            > "gpurun_out/qs_q${q}_p$p.json" 2> "gpurun_out/qs_q${q}_p$p.err" || exit $?
    done
done
