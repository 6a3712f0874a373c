"""World-size-2 `gloo` test of the frame-sharded gather (the multi-GPU path's only collective):
each rank holds the result records of its contiguous shard; after gather_results every rank sees
all frames in frame order, equal to the single-process list."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import pitt_object_table_segmentation_amd as pitt
from pitt_object_table_segmentation_amd import distributed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(n):
    rng = np.random.default_rng(123)
    rec = np.zeros(n, pitt.RESULT_DTYPE)
    rec["coefficients"] = rng.normal(size=(n, 4)).astype(np.float32)
    rec["n_inliers"] = rng.integers(0, 307200, n)
    rec["hypotheses"] = rng.integers(1, 1002, n)
    rec["n_coeff"] = 4
    return rec


def _worker(rank, world, port, n_frames, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        allrec = _records(n_frames)
        s, e = distributed.shard_range(n_frames, world, rank)
        got = distributed.gather_results(allrec[s:e], s, n_frames, device="cpu")
        out_q.put((rank, got.tobytes() == allrec.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [16, 13])
def test_gloo_world2_gather(n_frames):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
