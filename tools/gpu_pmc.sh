#!/bin/bash
# PMC counters for one kernel over a short one-batch-in-flight bench.py run, one rocprofv3 pass per
# counter set.
#   bash tools/gpu_pmc.sh <tag> <kernel-regex> "<counters pass 1>" ["<counters pass 2>" ...]
# Output: gpurun_out/pmc_<tag>_<i>/ per pass.
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=$1
KRE=$2
shift 2
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
i=0
for set in "$@"; do
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "$KRE" -d "$OUT/pmc_${TAG}_$i" -o p -f csv -- \
        python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 --pipeline 1 --no-cpu-baseline > "$OUT/pmc_${TAG}_$i.log" 2>&1 || exit $?
    i=$((i + 1))
done
