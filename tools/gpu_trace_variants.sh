#!/bin/bash
# Per -D variant: rebuild, then a rocprofv3 kernel trace of the pipelined bench (3 in flight).
#   bash tools/gpu_trace_variants.sh "-DX=1" ...  -> gpurun_out/tv_<i>/ (+ tv_<i>.flags)
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
i=0
for flags in "$@"; do
    make -s -C "$ROOTDIR/pitt_object_table_segmentation_amd/csrc" -B -j16 EXTRA="$flags" > "$OUT/tv_${i}_build.log" 2>&1 || exit 3
    echo "$flags" > "$OUT/tv_$i.flags"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tv_$i" -o t -f csv -- \
        python3 "$ROOTDIR/bench.py" --steps 20 --warmup 3 --pipeline 3 --no-cpu-baseline) > "$OUT/tv_$i.log" 2>&1 || exit $?
    i=$((i + 1))
done
make -s -C "$ROOTDIR/pitt_object_table_segmentation_amd/csrc" -B -j16 > /dev/null 2>&1
