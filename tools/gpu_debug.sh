#!/bin/bash
# One debugging script on the GPU box under a time limit: bash tools/gpu_debug.sh <tag> <python script> [args]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u "$@" > gpurun_out/${TAG}.log 2>&1
rc=$?
tail -40 gpurun_out/${TAG}.log
exit $rc
