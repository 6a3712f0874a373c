#!/bin/bash
# Rebuild libpitt_seg.so per -D variant and run bench.py (pipeline 1 and 3, no CPU baseline):
#   bash tools/gpu_variants_bench.sh "-DX=1" "-DX=2" ...  -> gpurun_out/vb_<i>_p<N>.json/.err
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for flags in "$@"; do
    make -s -C pitt_object_table_segmentation_amd/csrc -B -j16 EXTRA="$flags" > "gpurun_out/vb_${i}_build.log" 2>&1 || exit 3
    echo "$flags" > "gpurun_out/vb_${i}.flags"
    for p in 1 3; do
        timeout -k 10 300 python bench.py --steps 20 --warmup 3 --pipeline $p --no-cpu-baseline \
            > "gpurun_out/vb_${i}_p$p.json" 2> "gpurun_out/vb_${i}_p$p.err" || exit $?
    done
    i=$((i + 1))
done
make -s -C pitt_object_table_segmentation_amd/csrc -B -j16 > /dev/null 2>&1
