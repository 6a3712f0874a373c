"""Frame-parallel multi-GPU plumbing: contiguous frame shards, one process per
GPU, and a single gather of fixed-size per-frame result records to rank 0.

The data path has no collective: every rank segments its own frames with its own context.  The
only exchange is the result gather.  RCCL has no native gather, so it is an all_gather of
equal-size records (the `nccl` backend of torch.distributed is RCCL over xGMI on MI355X); with
the `gloo` backend the same code runs on CPU tensors (tests).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .api import RESULT_DTYPE

RECORD_BYTES = RESULT_DTYPE.itemsize


def shard_range(n_frames: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [start, end) of rank `rank`: GPU g gets frames [g*B/G, (g+1)*B/G)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(n_frames, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def pack_records(results: np.ndarray, frame_ids: np.ndarray, slots: int) -> np.ndarray:
    """Fixed-size byte records [slots, 8 + RECORD_BYTES]: (frame id int64, result record)."""
    out = np.zeros((slots, 8 + RECORD_BYTES), np.uint8)
    ids = np.full(slots, -1, np.int64)
    ids[:len(frame_ids)] = frame_ids
    out[:, :8] = ids.view(np.uint8).reshape(slots, 8)
    if len(results):
        out[:len(results), 8:] = np.ascontiguousarray(results, RESULT_DTYPE).view(np.uint8).reshape(len(results), -1)
    return out


def unpack_records(buf: np.ndarray, n_frames: int) -> np.ndarray:
    """Inverse of pack_records over the gathered buffer; returns results ordered by frame id.

    Vectorised: the frame ids index the output directly (fancy indexing, no per-record Python
    loop), and np.bincount checks that every frame arrived exactly once."""
    buf = np.ascontiguousarray(buf, np.uint8).reshape(-1, 8 + RECORD_BYTES)
    ids = np.ascontiguousarray(buf[:, :8]).view(np.int64).reshape(-1)
    recs = np.ascontiguousarray(buf[:, 8:]).view(RESULT_DTYPE).reshape(-1)
    live = ids >= 0
    ids, recs = ids[live], recs[live]
    if len(ids) and (ids.max() >= n_frames):
        raise RuntimeError(f"gather carried frame ids beyond the batch: {ids[ids >= n_frames][:8]}")
    seen = np.bincount(ids, minlength=n_frames)
    if not (seen == 1).all():
        lost, dup = np.nonzero(seen == 0)[0], np.nonzero(seen > 1)[0]
        raise RuntimeError(f"gather lost frames {lost[:8]} / duplicated frames {dup[:8]}")
    out = np.empty(n_frames, RESULT_DTYPE)
    out[ids] = recs
    return out


def gather_results(results: np.ndarray, frame_start: int, n_frames: int, device=None):
    """Gather every rank's per-frame results to all ranks (rank 0 consumes them).

    results: this rank's RESULT_DTYPE records for frames [frame_start, frame_start+len).
    device: torch device for the collective buffer ('cuda:k' with nccl/RCCL, cpu with gloo).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    slots = -(-n_frames // world)  # equal-size records per rank
    local = pack_records(results, np.arange(frame_start, frame_start + len(results), dtype=np.int64), slots)
    src = torch.from_numpy(local.reshape(-1)).to(device)
    dst = torch.empty(world * src.numel(), dtype=torch.uint8, device=src.device)
    dist.all_gather_into_tensor(dst, src)
    return unpack_records(dst.cpu().numpy(), n_frames)


def gather_inliers(inliers: np.ndarray, counts: np.ndarray, device=None):
    """Gather every rank's final inlier lists (optional part of config 4's exchange).

    inliers: this rank's frames' ascending inlier indices, concatenated in frame order (int32);
    counts:  inliers per frame of this rank (int64).  Returns (all_inliers, all_counts) over the
    whole batch in frame order.  Two equal-size all_gathers (lengths, then zero-padded lists),
    since RCCL has no variable-size gather.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    inliers = np.ascontiguousarray(inliers, np.int32)
    counts = np.ascontiguousarray(counts, np.int64)
    meta = torch.tensor([len(inliers), len(counts)], dtype=torch.int64, device=device)
    metas = torch.empty(world * 2, dtype=torch.int64, device=meta.device)
    dist.all_gather_into_tensor(metas, meta)
    metas = metas.cpu().numpy().reshape(world, 2)
    lmax, fmax = int(metas[:, 0].max()), int(metas[:, 1].max())
    pad_i = np.zeros(max(lmax, 1), np.int32)
    pad_i[:len(inliers)] = inliers
    pad_c = np.zeros(max(fmax, 1), np.int64)
    pad_c[:len(counts)] = counts
    src_i = torch.from_numpy(pad_i).to(device)
    src_c = torch.from_numpy(pad_c).to(device)
    dst_i = torch.empty(world * src_i.numel(), dtype=torch.int32, device=src_i.device)
    dst_c = torch.empty(world * src_c.numel(), dtype=torch.int64, device=src_c.device)
    dist.all_gather_into_tensor(dst_i, src_i)
    dist.all_gather_into_tensor(dst_c, src_c)
    all_i = dst_i.cpu().numpy().reshape(world, -1)
    all_c = dst_c.cpu().numpy().reshape(world, -1)
    out_i = np.concatenate([all_i[r, :metas[r, 0]] for r in range(world)]) if world else np.zeros(0, np.int32)
    out_c = np.concatenate([all_c[r, :metas[r, 1]] for r in range(world)]) if world else np.zeros(0, np.int64)
    return out_i, out_c


class AsyncRecordGather:
    """The per-step result gather of config 4, taken off the ranks' critical path.

    post() packs a finished batch's records into a staging slot and enqueues the all_gather
    without waiting (async_op); collect() completes a posted gather and unpacks it.  The bench
    posts batch i's records as soon as batch i is done and collects them one step later, so the
    exchange runs while the next batch is being enqueued.  Staging slots rotate (one per posted,
    uncollected gather), so a slot is never rewritten while its copy or collective is in flight.

    device: 'cuda:k' for the nccl (= RCCL over xGMI) backend -- the records go through a pinned
    host slot and a non-blocking H2D copy -- or 'cpu' for gloo.
    """

    def __init__(self, n_frames: int, frame_start: int, n_local: int, slots: int = 4, device="cpu"):
        import torch
        import torch.distributed as dist

        self.world = dist.get_world_size()
        self.n_frames = n_frames
        self.per_rank = -(-n_frames // self.world)
        self.ids = np.arange(frame_start, frame_start + n_local, dtype=np.int64)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        nb = self.per_rank * (8 + RECORD_BYTES)
        self.host = [torch.empty(nb, dtype=torch.uint8, pin_memory=self.cuda) for _ in range(slots)]
        self.src = [h.to(self.device) if self.cuda else h for h in self.host]
        self.dst = [torch.empty(self.world * nb, dtype=torch.uint8, device=self.device) for _ in range(slots)]
        self.next = 0
        self.busy = [False] * slots
        self.seconds = 0.0  # host time spent in post() + collect()
        self.posted = 0

    def post(self, results: np.ndarray):
        import time
        import torch.distributed as dist

        t = time.perf_counter()
        k = self.next
        if self.busy[k]:
            raise RuntimeError("AsyncRecordGather: every staging slot is in flight (collect first)")
        self.next = (k + 1) % len(self.host)
        self.busy[k] = True
        self.host[k].numpy()[:] = pack_records(results, self.ids, self.per_rank).reshape(-1)
        if self.cuda:
            self.src[k].copy_(self.host[k], non_blocking=True)
        work = dist.all_gather_into_tensor(self.dst[k], self.src[k], async_op=True)
        self.posted += 1
        self.seconds += time.perf_counter() - t
        return (k, work)

    def collect(self, handle) -> np.ndarray:
        import time

        t = time.perf_counter()
        k, work = handle
        work.wait()
        out = unpack_records(self.dst[k].cpu().numpy(), self.n_frames)
        self.busy[k] = False
        self.seconds += time.perf_counter() - t
        return out
