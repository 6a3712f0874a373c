"""pitt_sort_pairs against the oracle's std::sort on small arrays (the one-block introsort finish):
prints each case's result; used with the PITT_IS_WATCHDOG build to diagnose the block queue."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_binding as orc  # noqa: E402
import pitt_object_table_segmentation_amd as pitt  # noqa: E402

with pitt.Context(0) as ctx:
    for n, keys in [(17, 3), (40, 5), (100, 10), (500, 50), (2000, 2), (2000, 300), (2048, 2048), (5000, 100),
                    (8192, 300), (8193, 7), (8000, 8000), (30000, 40), (65536, 500), (65537, 900), (70000, 3)]:
        rng = np.random.default_rng(n + keys)
        k = rng.integers(0, keys, n).astype(np.uint32)
        v = rng.permutation(n).astype(np.uint32)
        want = orc.sort_pairs(k, v)
        tk = torch.from_numpy(k.view(np.int32)).cuda()
        tv = torch.from_numpy(v.view(np.int32)).cuda()
        ctx.sort_pairs(tk, tv, -1)
        torch.cuda.synchronize()
        ok = np.array_equal(tk.cpu().numpy().view(np.uint32), want[0]) and np.array_equal(tv.cpu().numpy().view(np.uint32), want[1])
        print(n, keys, "ok" if ok else "MISMATCH", flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "--voxel":  # one bench frame (the watchdog build prints per-block counters)
        x, y, z = pitt.synth_frame(0, 1000)
        ctx.voxel_grid(*(torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda() for a in (x, y, z)))
        torch.cuda.synchronize()
