#!/bin/bash
# Round-5 pass: the whole -m gpu suite, the default bench line, then kernel traces of config 5,
# classification and config 2 (tools/gpu_prof_r05.sh).  A fault or time limit stops the script.
set -o pipefail
TAG=${1:-r05c}
bash tools/gpu_r05.sh $TAG || exit $?
bash tools/gpu_prof_r05.sh $TAG
