#!/bin/bash
# Round-4 profile pass on the GPU box: (1) rocprofv3 kernel trace + stats of the default bench at 40 steps
# (the pipelined window for tools/trace_timeline.py and the roofline pass for tools/summarize_profiles.py),
# (2) the k_score PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs), (3) a kernel trace of config 5.
#   bash tools/gpu_prof_r04.sh <tag>
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=${1:-r04p}
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
BENCH="$ROOTDIR/bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}_trace" -o trace -f csv -- python3 $BENCH \
    > "$OUT/prof_${TAG}_trace.log" 2>&1 || exit $?
echo trace done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_score' -d "$OUT/prof_${TAG}_fetch" -o fetch -f csv \
    -- python3 $BENCH > "$OUT/prof_${TAG}_fetch.log" 2>&1 || exit $?
echo fetch done
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_score' -d "$OUT/prof_${TAG}_write" -o write -f csv \
    -- python3 $BENCH > "$OUT/prof_${TAG}_write.log" 2>&1 || exit $?
echo write done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}_c5" -o c5 -f csv -- python3 "$ROOTDIR/tools/config5_run.py" \
    > "$OUT/prof_${TAG}_c5.log" 2>&1 || exit $?
echo config5 done
