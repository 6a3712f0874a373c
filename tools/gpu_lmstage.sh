#!/bin/bash
# The LM's staged QR chains: the LM / primitive / classification parity tests, the per-phase cycles of
# the classification frame's longest job (PITT_ELM_PROF build in abv/), and the classification time.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pcl_lm.py tests/test_sphere.py tests/test_cylinder.py tests/test_cone.py tests/test_classify_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lmstage_tests.log 2>&1 || { tail -30 gpurun_out/lmstage_tests.log; exit 1; }
tail -1 gpurun_out/lmstage_tests.log
PITT_LIB_PATH=$PWD/abv/libpitt_seg_elmprof.so timeout -k 10 120 python tools/classify_run.py 1 > gpurun_out/lmstage_prof.log 2>&1 || exit 1
grep PITT_ELM_PROF gpurun_out/lmstage_prof.log | grep "m 1320" | head -1
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --settle-steps 0 --no-cpu-baseline > gpurun_out/lmstage_bench.json 2> gpurun_out/lmstage_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/lmstage_bench.json')); print('classify', d['classify']); print('config5', d['config5']['gpu_ms_per_scene'])"
