"""BASELINE config 2 in a loop for rocprofv3 traces: one 640x480 cloud through the single-cloud ABI
(pitt_plane_segment: PointXYZ host array in, inliers and coefficients back), then the same frame as a
device-resident one-frame batch.

    python tools/config2_run.py [reps]"""
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
print(f"config2 host ABI {np.median(ts):.3f} ms, device-resident batch {np.median(td):.3f} ms (medians of {reps})")
