#!/bin/bash
# Timing experiments: rebuild libpitt_seg.so with each -D variant and record a rocprofv3 kernel
# trace of a short bench.py run per variant.
#   bash tools/gpu_exp.sh "-DPITT_SCORE_EXP=0" "-DPITT_SCORE_EXP=1" ...
# Output: gpurun_out/exp_<i>/ (trace) and gpurun_out/exp_<i>.log; the last build is restored to
# the default flags.
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
i=0
for flags in "$@"; do
    make -s -C "$ROOTDIR/pitt_object_table_segmentation_amd/csrc" -B -j16 EXTRA="$flags" > "$OUT/exp_${i}_build.log" 2>&1 || exit 3
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/exp_$i" -o t -f csv -- \
        python3 "$ROOTDIR/bench.py" --steps 3 --warmup 1 --pipeline 1 --no-cpu-baseline) > "$OUT/exp_$i.log" 2>&1 || exit $?
    echo "$flags" > "$OUT/exp_$i.flags"
    i=$((i + 1))
done
