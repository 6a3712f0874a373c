#!/bin/bash
# End-of-round GPU pass: tests + smoke + bench (tools/gpu_round.sh), then the rocprofv3 trace + PMC
# passes (tools/gpu_profile.sh <tag>).  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_round.sh || exit $?
bash tools/gpu_profile.sh ${1:-final} 5 || exit $?
exit 0
