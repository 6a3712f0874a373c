#!/bin/bash
# One parametrised A/B driver (replaces the per-experiment tools/gpu_*.sh scripts).
#   bash tools/gpu_ab.sh [-t "<pytest files>"] [-r ROUNDS] [-b "<bench.py args>"] NAME...
# NAME "cur" is the in-tree product library, "ab" the in-tree A/B build, any other NAME abv/libpitt_seg_<NAME>.so
# (built by tools/build_variant.sh); NAME+VAR=VALUE runs that library with VAR=VALUE in the environment.  With -t, the listed GPU tests run first under the in-tree library;
# then ROUNDS alternating bench runs per library, each printing value, roofline frac and the
# first scoring chunk's average launch.  Every GPU step has its own time limit; the script stops
# at the first failure.
set -o pipefail
TESTS=""; ROUNDS=2; BARGS="--no-extras --no-cpu-baseline"
while getopts "t:r:b:" o; do case $o in t) TESTS=$OPTARG;; r) ROUNDS=$OPTARG;; b) BARGS=$OPTARG;; *) exit 2;; esac; done
shift $((OPTIND - 1))
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    # NAME = LIB[+VAR=VALUE...]: LIB cur (in-tree product), ab (in-tree A/B build) or abv/libpitt_seg_LIB.so;
    # the +VAR=VALUE parts are set in the bench's environment (knobs of the A/B build)
    IFS='+' read -r -a parts <<< "$lib"
    base=${parts[0]}
    if [ "$base" = cur ]; then unset PITT_LIB_PATH
    elif [ "$base" = ab ]; then export PITT_LIB_PATH=$PWD/pitt_object_table_segmentation_amd/libpitt_seg_ab.so
    else export PITT_LIB_PATH=$PWD/abv/libpitt_seg_$base.so; fi
    tag=$(echo "$lib" | tr '+=' '__')
    timeout -k 10 300 env "${parts[@]:1}" python bench.py $BARGS > gpurun_out/ab_${tag}_$r.json 2> gpurun_out/ab_${tag}_$r.err || { tail -20 gpurun_out/ab_${tag}_$r.err; exit 1; }
    python - "$lib" "gpurun_out/ab_${tag}_$r.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
f = k.get("k_score.first", {}).get("avg_launch_us")
print(sys.argv[1], round(d["value"]), d["roofline"]["frac"], d["roofline"]["avg_launch_us"], f,
      d.get("steady_state"), {n: round(v.get("us_per_batch", 0), 1) for n, v in k.items()})
PY
  done
done
