#!/bin/bash
# A/B of classification knobs, alternating runs of tools/classify_run.py on one box.
set -o pipefail
for r in 1 2 3; do
  for cfg in "1 1" "0 1" "1 0" "0 0"; do
    set -- $cfg
    echo "prio=$1 stage=$2: $(PITT_AUX_LOW_PRIO=$1 PITT_STAGE_KERNEL=$2 timeout -k 10 60 python tools/classify_run.py 20 | cut -c1-22)" || exit 1
  done
done
