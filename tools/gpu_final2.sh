#!/bin/bash
# Tests + smoke + bench (tools/gpu_round.sh), then the preprocess / primitive-services bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh || exit $?
timeout -k 10 400 python tools/bench_preprocess.py > gpurun_out/preprocess.json 2> gpurun_out/preprocess.err || exit $?
exit 0
