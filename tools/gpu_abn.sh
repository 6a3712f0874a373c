#!/bin/bash
# A/B/n of library builds on one box: bench.py with each library in turn ($PITT_LIB_PATH), ROUNDS times,
# alternating.  Libraries: abl/<name>/libpitt_seg.so (built in-tree by tools/build_variant.sh); "base" is
# the in-tree product library.  Output: gpurun_out/abn_<tag>_<name>_<i>.json
#   bash tools/gpu_abn.sh <tag> <rounds> "<name> <name> ..." [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; ROUNDS=$2; NAMES=$3; shift 3
for i in $(seq 1 $ROUNDS); do
  for n in $NAMES; do
    if [ "$n" = base ]; then lib=""; else lib="$PWD/abl/$n/libpitt_seg.so"; fi
    PITT_LIB_PATH=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-extras "$@" \
        > gpurun_out/abn_${TAG}_${n}_$i.json 2> gpurun_out/abn_${TAG}_${n}_$i.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abn_${TAG}_${n}_$i.json')); k=d['kernels']; print('$n', $i, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], k.get('k_score.first',{}).get('avg_launch_us'))"
  done
done
