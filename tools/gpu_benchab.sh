#!/bin/bash
# bench.py against bench_prev.py, alternating, at the driver's 20 steps.  bench_prev.py is a copy of the earlier
# bench.py made before the call (e.g. `git show <rev>:bench.py > bench_prev.py`; not kept in the tree).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for b in prev cur; do
    f=bench.py; [ $b = prev ] && f=bench_prev.py
    timeout -k 10 200 python $f --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/bab_${b}_$r.json 2> gpurun_out/bab_${b}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/bab_${b}_$r.json')); print('$b', d['value'], d['ms_per_step'], d['kernels']['k_hypothesize']['us_per_batch'])"
  done
done
