#!/bin/bash
# Early refinement (PITT_EARLY_REFINE, default on) against off: the plane / schedule / graph parity tests
# with it on, then alternating bench runs at 200 steps and at the driver's 20 (hardware queues 8 and 16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_plane_gpu.py tests/test_golden.py tests/test_schedule_gpu.py tests/test_graphs_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/er_tests.log 2>&1 || { tail -30 gpurun_out/er_tests.log; exit 1; }
tail -1 gpurun_out/er_tests.log
for r in 1 2; do
  for q in 8 16; do
    for er in 0 1; do
      for k in 200 20; do
        PITT_EARLY_REFINE=$er timeout -k 10 200 python bench.py --steps $k --warmup 5 --hw-queues $q --no-extras --no-cpu-baseline > gpurun_out/er_${er}_q${q}_${k}_$r.json 2> gpurun_out/er_${er}_q${q}_${k}_$r.err || exit 1
        python -c "import json; d=json.load(open('gpurun_out/er_${er}_q${q}_${k}_$r.json')); print('er=$er q=$q k=$k', d['value'], d['ms_per_step'])"
      done
    done
  done
done
