#!/bin/bash
# k_score ablations: rebuild libpitt_seg.so per -D variant, bench (pipeline 1, no CPU baseline), then
# restore the default build.  bash tools/gpu_exp_variants.sh "-DX" "-DY" ... -> gpurun_out/ev_<i>.*
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for flags in "$@"; do
    make -s -C pitt_object_table_segmentation_amd/csrc -B -j16 EXTRA="$flags" > "gpurun_out/ev_${i}_build.log" 2>&1 || exit 3
    echo "$flags" > "gpurun_out/ev_${i}.flags"
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --pipeline 1 --no-cpu-baseline \
        > "gpurun_out/ev_${i}.json" 2> "gpurun_out/ev_${i}.err" || exit $?
    i=$((i + 1))
done
