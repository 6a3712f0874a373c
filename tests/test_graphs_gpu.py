"""HIP-graph replay of the plane pipeline ("HIP graphs" and "Graph replays and direct work").

A batch layout seen twice is captured into a graph whose nodes hold device-arena and pinned-host
addresses (the result / chunk-stat copy nodes write pinned host blocks).  A graph replays only while
every address it holds is live (any arena or pinned block that moves bumps the arena generation, part
of the key) and while no direct work ran on its context since it last ran (the direct epoch): a
one-frame graph replayed after the primitive services' launches on the same stream faulted, in round 3
and again in round 4 with the floor at one frame, so batches below 64 frames launch directly and a graph
is captured afresh after direct work.  These tests hold replays, recaptures and direct launches to the
same bits."""
import os

import numpy as np
import pytest
import torch

import pitt_object_table_segmentation_amd as pitt
import test_plane_gpu as P
from test_sphere import sphere_scene

pytestmark = pytest.mark.gpu


def _ctx(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return pitt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_hip_graph_replay_bit_exact():
    """Repeated batch layouts are captured into a HIP graph (second sight) and replayed (third on):
    the replays give the same records and inlier lists as direct launches ($PITT_GRAPHS=0) and the
    oracle (pipelining)."""
    frames = [pitt.synth_frame(s, seed, 320, 240) for s, seed in ((0, 7000), (1, 7001), (2, 7002), (0, 7003))]
    b = pitt.FrameBatch.from_host(frames, device="cuda:0")
    direct = _ctx(PITT_GRAPHS=0)
    graphed = _ctx(PITT_GRAPHS=1, PITT_GRAPH_MIN_FRAMES=1)  # graphs for this 4-frame layout
    try:
        ref_inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
        ref = direct.plane_segment_batch(b, pitt.sac_params(), ref_inl)
        inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")  # one output buffer: one layout key
        for k in range(4):
            inl.fill_(-7)
            res = graphed.plane_segment_batch(b, pitt.sac_params(), inl)
            assert res.tobytes() == ref.tobytes(), k
            for o, r in zip(b.offsets, ref):
                assert torch.equal(inl[o:o + r["n_inliers"]], ref_inl[o:o + r["n_inliers"]]), k
        captures, replays = graphed.graph_stats()
        assert captures == 1 and replays == 3
        assert direct.graph_stats() == (0, 0)
        P._check(graphed, frames, ref, [ref_inl.cpu().numpy()[o:o + r["n_inliers"]] for o, r in zip(b.offsets, ref)])
    finally:
        direct.close()
        graphed.close()


def _run(ctx, b, inl):
    inl.fill_(-7)
    res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
    return res, inl.cpu().numpy().copy()


def _frames(n, seed, w=160, h=120):
    return [pitt.synth_frame(s % 3, seed + s, w, h) for s in range(n)]


def test_graph_survives_arena_and_pinned_growth():
    """A 64-frame layout captured into a graph, then batches that grow the pinned result / chunk-stat
    blocks and the device arena, then the 64-frame layout again: the stale graph is not replayed (the
    arena generation moved, so the key is new: first sight launches directly, the second recaptures), and
    every result stays bit-exact."""
    small = _frames(64, 7100)
    big = _frames(160, 7200)  # 160 records > one 4 KB pinned block
    b1 = pitt.FrameBatch.from_host(small, device="cuda:0")
    bb = pitt.FrameBatch.from_host(big, device="cuda:0")
    inl1 = torch.empty(b1.capacity, dtype=torch.int32, device="cuda:0")
    inlb = torch.empty(bb.capacity, dtype=torch.int32, device="cuda:0")
    ctx = _ctx(PITT_GRAPHS=1)
    try:
        ref, ref_inl = _run(ctx, b1, inl1)               # first sight: direct
        for _ in range(2):                               # capture, then replay
            r, i = _run(ctx, b1, inl1)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl)
        assert ctx.graph_stats() == (1, 2)
        # grows "results_h" (160 x 56 B > 4096 B), the device arena (tiles x frames), "meta_h" ...
        res_b = ctx.plane_segment_batch(bb, pitt.sac_params(), inlb)
        # ... and more iterations per frame: more chunks, a larger "cstat_h" and larger hypothesis buffers
        res_c = ctx.plane_segment_batch(bb, pitt.sac_params(max_iterations=5000), inlb)
        caps, reps = ctx.graph_stats()
        r, i = _run(ctx, b1, inl1)                       # the arena moved: a new key's first sight (direct)
        assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl)
        c1, r1 = ctx.graph_stats()
        assert (c1, r1) == (caps, reps), "a graph from before the arena moved was replayed"
        for k in range(2):                               # capture, replay
            r, i = _run(ctx, b1, inl1)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl), k
        assert ctx.graph_stats() == (caps + 1, reps + 2)
        # per-hypothesis counts are read from the context's last batch: b1 ran last here
        sample = [0, 1, 2, 33, 63]
        P._check(ctx, [small[f] for f in sample], ref[sample],
                 [ref_inl[b1.offsets[f]:b1.offsets[f] + ref[f]["n_inliers"]] for f in sample], frame_ids=sample)
        # run the 160-frame layout again so that its counts are the last batch's, then check a sample of it
        res_c2 = ctx.plane_segment_batch(bb, pitt.sac_params(max_iterations=5000), inlb)
        assert res_c2.tobytes() == res_c.tobytes()
        ib = inlb.cpu().numpy()
        sample = [0, 1, 2, 77, 159]
        P._check(ctx, [big[f] for f in sample], res_c[sample],
                 [ib[bb.offsets[f]:bb.offsets[f] + res_c[f]["n_inliers"]] for f in sample], frame_ids=sample,
                 max_iterations=5000)
        assert res_b["hypotheses"].min() > 0
    finally:
        ctx.close()


def test_graph_recaptured_after_service_calls():
    """Service calls between two batches of a graphed layout are direct work on the context: the next
    batch captures the graph afresh instead of replaying it, the one after replays, and every result
    equals a graph-free context's.  The services' one-frame plane batches launch directly (below the
    64-frame floor) and never capture."""
    ctx = _ctx(PITT_GRAPHS=1)
    ref_ctx = _ctx(PITT_GRAPHS=0)
    srv, ref_srv = pitt.Services(ctx), pitt.Services(ref_ctx)
    try:
        frames = _frames(64, 7300)
        b = pitt.FrameBatch.from_host(frames, device="cuda:0")
        inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
        ref, ref_inl = _run(ref_ctx, b, inl)
        for _ in range(3):                                 # direct, capture, replay
            r, i = _run(ctx, b, inl)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl)
        assert ctx.graph_stats() == (1, 2)
        for k, n in enumerate((300, 1200, 4000)):
            cloud = sphere_scene(n, n // 5, 900 + k).astype(np.float32)
            caps, reps = ctx.graph_stats()
            a = srv.ransac_sphere(cloud)
            c = srv.ransac_plane(cloud)                    # one frame: direct, no capture
            assert ctx.graph_stats() == (caps, reps)
            assert a[0] == ref_srv.ransac_sphere(cloud)[0]
            d = ref_srv.ransac_plane(cloud)
            assert c[0] == d[0] and np.array_equal(c[1], d[1]) and np.array_equal(c[2].view(np.int32), d[2].view(np.int32))
            # after direct work the old graph never replays: the batch is captured afresh (or, when the
            # services' scratch grew and moved the arena, launched directly as a new key's first sight)
            r, i = _run(ctx, b, inl)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl), k
            c1, r1 = ctx.graph_stats()
            assert c1 - caps == r1 - reps and c1 - caps <= 1, (k, caps, reps, c1, r1)
            for _ in range(2):                             # nothing in between: capture / replay
                r, i = _run(ctx, b, inl)
                assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl), k
            c2, r2 = ctx.graph_stats()
            assert c2 == caps + 1 and r2 == r1 + 2, (k, caps, reps, c2, r2)
    finally:
        srv.close()
        ref_srv.close()
        ctx.close()
        ref_ctx.close()
