"""BASELINE config 2 in a loop for rocprofv3 traces: one 640x480 cloud through the single-cloud ABI
(pitt_plane_segment: PointXYZ host array in, inliers and coefficients back), then the same frame as a
device-resident one-frame batch.

    python tools/config2_run.py [reps] [--json]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import pitt_object_table_segmentation_amd as pitt  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
x, y, z = pitt.synth_frame(0, 1000)
cloud = np.stack([x, y, z, np.ones_like(x)], 1).astype(np.float32)
# $C2_BUSY=k: first run k other contexts' 256-frame batches (the bench's state when it reaches config 2)
busy = []
for k in range(int(os.environ.get("C2_BUSY", "0"))):
    bc = pitt.Context(0)
    fb = pitt.FrameBatch.from_host([pitt.synth_frame(0, 1000 + i) for i in range(256)], device="cuda")
    bo = torch.empty(fb.capacity, dtype=torch.int32, device="cuda")
    bc.plane_segment_batch(fb, pitt.sac_params(), bo)
    busy.append((bc, fb, bo))
with pitt.Context(0) as ctx:
    ctx.plane_segment(cloud)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.plane_segment(cloud)
        ts.append((time.perf_counter() - t) * 1e3)
    b = pitt.FrameBatch.from_host([(x, y, z)], device="cuda")
    out = torch.empty(b.capacity, dtype=torch.int32, device="cuda")
    ctx.plane_segment_batch(b, pitt.sac_params(), out)
    td = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.plane_segment_batch(b, pitt.sac_params(), out)
        td.append((time.perf_counter() - t) * 1e3)
    m = ctx.plane_segment(cloud)
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(reps):
        ctx.plane_segment_batch(b, pitt.sac_params(), out)
    kern = {k: round(ctx.profile_get(k)[1] / reps * 1e3, 1) for k in ("k_score", "k_refine:xsum", "k_sel_mark")}
    ctx.profile(False)
if "--json" in sys.argv:  # for bench.py, which runs this in a child process
    import json
    print(json.dumps({"host_ms": round(float(np.median(ts)), 3), "device_ms": round(float(np.median(td)), 3),
                      "inliers": int(len(m.inliers)), "inliers_sum": int(np.asarray(m.inliers, np.int64).sum()),
                      "coefficients": [float(c) for c in m.coefficients]}))
else:
    print(f"config2 host ABI {np.median(ts):.3f} ms, device-resident batch {np.median(td):.3f} ms (medians of {reps}); "
          f"kernels us {kern}")
