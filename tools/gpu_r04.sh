#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite (graphs from one frame up, the default since round 4), then the
# default bench line.  Every step under its own time limit; the chain stops at the first
# failure.
#   bash tools/gpu_r04.sh <tag>
set -o pipefail
TAG=${1:-r04a}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
    > $OUT/${TAG}_pytest_gpu.log 2>&1 || { tail -30 $OUT/${TAG}_pytest_gpu.log; exit 1; }
tail -3 $OUT/${TAG}_pytest_gpu.log
timeout -k 10 400 python -u bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.log || { tail -30 $OUT/${TAG}_bench.log; exit 1; }
cat $OUT/${TAG}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
