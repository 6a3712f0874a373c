#!/bin/bash
set -o pipefail
PITT_LIB_PATH=$PWD/abtmp/libpitt_seg_elmprof.so timeout -k 10 120 python tools/classify_run.py 1 > gpurun_out/lmprof.log 2>&1 || exit 1
grep PITT_ELM_PROF gpurun_out/lmprof.log | grep "m 1320" | head -1
