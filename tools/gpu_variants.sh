#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/var_$tag.json 2> gpurun_out/var_$tag.err || exit $?; }
run p1 --pipeline 1
run p1np --pipeline 1 --no-prof
run p2lib --pipeline 2
run p2libnp --pipeline 2 --no-prof
run p2torch --pipeline 2 --torch-streams
run p3libnp --pipeline 3 --no-prof
