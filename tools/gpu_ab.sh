#!/bin/bash
# A/B of two builds of libpitt_seg.so on the same box: bench.py alternately with the in-tree library
# (A) and exp_libs/<B>/libpitt_seg.so, ROUNDS times each.  Output: gpurun_out/ab_<tag>_{A,B}<i>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; B=$2; ROUNDS=${3:-2}; shift 3
for i in $(seq 1 $ROUNDS); do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/ab_${TAG}_A$i.json \
        2> gpurun_out/ab_${TAG}_A$i.err || exit $?
    PITT_LIB_PATH=$PWD/exp_libs/$B/libpitt_seg.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras "$@" \
        > gpurun_out/ab_${TAG}_B$i.json 2> gpurun_out/ab_${TAG}_B$i.err || exit $?
done
