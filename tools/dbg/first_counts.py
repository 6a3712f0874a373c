"""Debug: per-hypothesis counts of the first chunk against the oracle (one batch of test frames)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
import oracle_binding as orc
import pitt_object_table_segmentation_amd as pitt

frames = [pitt.synth_frame(s, seed) for s, seed in ((0, 1000), (0, 1001), (0, 1002), (1, 1000))]
with pitt.Context(0) as ctx:
    b = pitt.FrameBatch.from_host(frames)
    inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda")
    res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
    for i, f in enumerate(frames):
        o = orc.plane_segment(*f)
        got = ctx.hypothesis_counts(i, 32)
        print(i, "T", res[i]["hypotheses"], o.hypotheses, "n", len(f[0]))
        print("  got", got[:12].tolist())
        print("  ref", o.hyp_counts[:12].tolist())
