"""Dump the GPU neighbour lists of one voxelized frame for offline comparison with the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle_binding as orc  # noqa: E402
import pitt_object_table_segmentation_amd as pitt  # noqa: E402

scene, seed = int(sys.argv[1]), int(sys.argv[2])
x, y, z = pitt.synth_frame(scene, seed)
v, _ = orc.voxel_grid(x, y, z)
with pitt.Context(0) as ctx:
    t = [torch.from_numpy(np.ascontiguousarray(v[:, i])).cuda() for i in range(3)]
    nx, ny, nz, cv, (nn, cnt) = ctx.normal_estimation(*t, neighbours=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"nrm_{scene}_{seed}.npz"), v=v, nn=nn.cpu().numpy(),
                        cnt=cnt.cpu().numpy(), n=torch.stack([nx, ny, nz, cv], 1).cpu().numpy())
print("ok")
