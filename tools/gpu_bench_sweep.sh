#!/bin/bash
# bench.py at several pipeline depths (no CPU baseline): gpurun_out/sweep_p<N>.json/.err
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for p in "$@"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --pipeline "$p" --no-cpu-baseline \
        > "gpurun_out/sweep_p$p.json" 2> "gpurun_out/sweep_p$p.err" || exit $?
done
