#!/bin/bash
# k_refine diagnosis: the chain loop in isolation (tools/microbench/chain_rate), per-role cycles of
# k_refine at pipeline 1 ($PITT_REFINE_DEBUG, producers 1 and 2), and the pipeline depth x hardware
# queue points that matter for the steady state.  Each GPU step has its own time limit; the script
# stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-probe}
timeout -k 10 120 tools/microbench/build/chain_rate > "$OUT/${TAG}_chain_rate.txt" 2>&1 || exit $?
for p in 1 2; do
  PITT_REFINE_DEBUG=1 PITT_REFINE_PRODUCERS=$p timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 \
      --pipeline 1 --no-extras --no-cpu-baseline > "$OUT/${TAG}_dbg_p$p.json" 2> "$OUT/${TAG}_dbg_p$p.err" || exit $?
done
for cfg in "3 0" "4 8" "3 8" "4 0"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline --pipeline $1 --hw-queues $2 \
      > "$OUT/${TAG}_pipe_p$1_q$2.json" 2> "$OUT/${TAG}_pipe_p$1_q$2.err" || exit $?
done
