"""VoxelGrid (PCL order) on the 16 distinct 640x480 bench frames of tools/bench_preprocess.py, one frame
per call as PCManager::downSampling runs it: per-frame wall time (each call synchronised) and the mean,
for a rocprofv3 --kernel-trace --stats run to attribute to the introsort kernels.

    python tools/voxel_run.py [--reps 4] [--check]

--check compares every frame's centroids with the oracle (bit-exact), on the first rep.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pitt_object_table_segmentation_amd as pitt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    frames = [pitt.synth_frame(2 if f % 4 == 3 else 0, 1000 + f) for f in range(16)]
    dev = [tuple(torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda() for a in fr) for fr in frames]
    per = np.zeros((args.reps, 16))
    ok = None
    with pitt.Context(0) as ctx:
        for fr in dev:  # warm-up (scratch buffers)
            ctx.voxel_grid(*fr)
        torch.cuda.synchronize()
        for r in range(args.reps):
            for f, fr in enumerate(dev):
                t0 = time.perf_counter()
                (vx, vy, vz), _ = ctx.voxel_grid(*fr)
                torch.cuda.synchronize()
                per[r, f] = (time.perf_counter() - t0) * 1e3
                if args.check and r == 0:
                    import oracle_binding as orc
                    o, _ = orc.voxel_grid(*(np.asarray(a, np.float32) for a in frames[f]))
                    same = all(np.array_equal(np.ascontiguousarray(o[:, k]).view(np.int32), d.cpu().numpy().view(np.int32))
                               for k, d in enumerate((vx, vy, vz)))
                    ok = same if ok is None else (ok and same)
            print(f"rep {r}: mean {per[r].mean():.3f} ms", flush=True)
    med = np.median(per, 0)
    print(json.dumps({"ms_per_frame_mean": round(float(per.mean()), 4), "ms_per_frame_median_of_reps": [round(float(v), 3) for v in med],
                      "matches_oracle": ok}))


if __name__ == "__main__":
    main()
