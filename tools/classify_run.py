"""Batched primitive classification in a loop (bench.py's ten-cluster frame), for rocprofv3 traces:
   rocprofv3 --kernel-trace --hip-trace --stats -d gpurun_out/cls -o p -f csv -- python3 tools/classify_run.py"""
import importlib.util
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import pitt_object_table_segmentation_amd as pitt  # noqa: E402

spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)

ctx = pitt.Context(0)
srv = pitt.Services(ctx)
cl = bench.synth_clusters(0)
cnt = np.array([len(c) for c in cl], np.int64)
off = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
xyz = np.concatenate(cl)
d = [torch.from_numpy(np.ascontiguousarray(xyz[:, k])).cuda() for k in range(3)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
srv.classify_clusters(*d, off, cnt)
t = time.perf_counter()
for _ in range(reps):
    got = srv.classify_clusters(*d, off, cnt)
print(f"{(time.perf_counter() - t) / reps * 1e3:.2f} ms per frame", [g["shape"] for g in got], [g["inliers"] for g in got])
srv.close()
ctx.close()
