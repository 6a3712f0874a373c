"""BASELINE config 5 on one GPU: find_supports + euclidean_clusters on the 1.2M-point fused scene,
repeated, for rocprofv3 kernel traces (tools/gpu_r03.sh) and quick timing: the device-resident
scene path (pitt_segment_objects_dev) and the host-array service path.

    python tools/config5_run.py [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pitt_object_table_segmentation_amd as pitt  # noqa: E402


def main(reps=5, dev_only=False):
    import torch
    x, y, z = pitt.synth_fused(1000, 4)
    dx, dy, dz = (torch.from_numpy(a).cuda() for a in (x, y, z))
    with pitt.Context(0) as ctx:
        ts = []
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            n_on, sizes = ctx.segment_objects_dev(dx, dy, dz, copy=False)
            if r:
                ts.append((time.perf_counter() - t) * 1e3)
        print(f"config5 device path: {len(n_on)} supports, {len(sizes)} clusters; {np.median(ts):.2f} ms "
              f"(median of {reps})", flush=True)
        if dev_only:
            return
        ts = []
        for r in range(reps + 1):
            t = time.perf_counter()
            sups = ctx.find_supports(x, y, z)
            t1 = time.perf_counter()
            ncl = 0
            for s in sups:
                n = len(s.on_support_cloud)
                if n >= 30:
                    ncl += len(ctx.euclidean_clusters(*s.on_support_cloud.T, tolerance=0.03,
                                                      min_size=int(np.floor(n * 0.01 + 0.5)),
                                                      max_size=int(np.floor(n * 0.99 + 0.5))))
            t2 = time.perf_counter()
            if r:
                ts.append(((t1 - t) * 1e3, (t2 - t1) * 1e3))
        sup_ms = np.median([a for a, _ in ts])
        cl_ms = np.median([b for _, b in ts])
        print(f"config5 host path: {len(sups)} supports, {ncl} clusters; find_supports {sup_ms:.2f} ms, "
              f"clusters {cl_ms:.2f} ms (median of {reps})")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5, "--dev-only" in sys.argv)
