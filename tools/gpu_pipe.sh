#!/bin/bash
# Headline throughput vs batches in flight (contexts) and hardware queues.
set -o pipefail
TAG=${1:-r05p}
mkdir -p gpurun_out
for cfg in "4 8" "6 8" "8 8" "8 16" "6 16" "12 16"; do
    set -- $cfg
    timeout -k 10 240 python bench.py --no-extras --no-cpu-baseline --steps 30 --pipeline $1 --hw-queues $2 \
        > gpurun_out/${TAG}_p$1_q$2.json 2> gpurun_out/${TAG}_p$1_q$2.err || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_p$1_q$2.json').read().strip().splitlines()[-1]); print('p$1 q$2', d['value'], d['ms_per_step'])"
done
