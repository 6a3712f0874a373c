#!/bin/bash
# k_score inside-slab shortcut: its parity tests (both settings on every plane case, the adversarial
# inside-slab scene), then the bench A/B of PITT_INSIDE_CULL 0/1 with a rocprof kernel trace each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG=${1:-r03j}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_score_paths_gpu.py tests/test_shortcuts_gpu.py tests/test_plane_gpu.py \
    -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "inside or INSIDE or not paths" \
    > "$OUT/${TAG}_pytest_ins.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_pytest_ins.log"
bash tools/gpu_ab_env.sh "${TAG}_ins" PITT_INSIDE_CULL "0 1" || exit $?
for f in "$OUT/${TAG}_ins"_*_*.json; do
  echo "$f $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['kernels']['k_score.first']['avg_launch_us'])" "$f")"
done
