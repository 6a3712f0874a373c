"""Host-side cost of the pipelined headline loop: time spent inside plane_segment_batch_async (enqueue)
and inside wait() per batch, 4 contexts round robin as bench.py's timed pass.

    python tools/host_enqueue.py [steps] [pipeline]"""
import os
import sys
import time

import numpy as np

os.environ["GPU_MAX_HW_QUEUES"] = "8"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import pitt_object_table_segmentation_amd as pitt  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
B = 256
frames = [pitt.synth_frame(pitt.SCENE_TABLE, 1000 + i) for i in range(B)]
batches = [pitt.FrameBatch.from_host(frames, device="cuda") for _ in range(P)]
outs = [torch.empty(b.capacity, dtype=torch.int32, device="cuda") for b in batches]
ctxs = [pitt.Context(0) for _ in range(P)]
prm = pitt.sac_params()
for i in range(P):
    ctxs[i].plane_segment_batch(batches[i], prm, outs[i])
torch.cuda.synchronize()
pend = [False] * P
te, tw = [], []
t0 = time.perf_counter()
for s in range(steps):
    i = s % P
    if pend[i]:
        a = time.perf_counter()
        ctxs[i].wait()
        tw.append(time.perf_counter() - a)
    a = time.perf_counter()
    ctxs[i].plane_segment_batch_async(batches[i], prm, outs[i])
    te.append(time.perf_counter() - a)
    pend[i] = True
for i in range(P):
    ctxs[i].wait()
tt = time.perf_counter() - t0
print(f"pipeline {P}: {tt / steps * 1e3:.3f} ms per batch; enqueue median {np.median(te) * 1e3:.3f} ms "
      f"(max {np.max(te) * 1e3:.3f}), wait median {np.median(tw) * 1e3:.3f} ms")
