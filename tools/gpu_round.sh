#!/bin/bash
# A round's GPU pass: the whole -m gpu suite, then the default bench line.  Every step under its own time
# limit.  Test failures (pytest exit 1) still let the bench run, unless the log holds a GPU fault; a
# fault, time limit, crash or abort stops the script there (nothing more runs on the GPU).
#   bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r06a}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
    > $OUT/${TAG}_pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/${TAG}_pytest_gpu.log | head -30
tail -3 $OUT/${TAG}_pytest_gpu.log
if grep -qiE "illegal memory access|memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" $OUT/${TAG}_pytest_gpu.log; then
    echo "GPU fault in the test run: stopping"; exit 3
fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.log || { tail -30 $OUT/${TAG}_bench.log; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config5',{}).get('gpu_ms_per_scene'), d.get('classify',{}).get('ms_per_frame'))"
exit $rc
