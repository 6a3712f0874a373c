#!/bin/bash
set -o pipefail
for r in 1 2; do
  for v in 1 4 8; do
    if [ $v = 4 ]; then unset PITT_LIB_PATH; else export PITT_LIB_PATH=$PWD/abtmp/libpitt_seg_xr$v.so; fi
    echo "split $v: $(timeout -k 10 120 python tools/config2_run.py 40)" || exit 1
  done
done
