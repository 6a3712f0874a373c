#!/bin/bash
# rocprofv3 passes over bench.py on the GPU box: kernel trace + stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), restricted to k_score.
# Outputs land in gpurun_out/prof_<tag>_*; tools/summarize_profiles.py turns them into profiles/.
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=${1:-r01}
STEPS=${2:-5}
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
BENCH="$ROOTDIR/bench.py --steps $STEPS --warmup 1 --settle-steps 0 --no-cpu-baseline --no-extras"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}_trace" -o trace -f csv -- python3 $BENCH \
    > "$OUT/prof_${TAG}_trace.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_score' -d "$OUT/prof_${TAG}_fetch" -o fetch -f csv \
    -- python3 $BENCH > "$OUT/prof_${TAG}_fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_score' -d "$OUT/prof_${TAG}_write" -o write -f csv \
    -- python3 $BENCH > "$OUT/prof_${TAG}_write.log" 2>&1 || exit $?
echo done > "$OUT/prof_${TAG}_done"
