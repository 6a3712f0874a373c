"""HIP-graph replay of the plane pipeline ("HIP graphs" and "The round-3 graph fault").

A batch layout seen twice is captured into a graph whose nodes hold device-arena and pinned-host
addresses (the result / chunk-stat copy nodes write pinned host blocks).  A graph may only replay
while every address it holds is live: any arena or pinned block that moves bumps the context's
arena generation, which is part of the graph key.  The round-3 fault was a one-frame graph replayed
after a larger batch on the same context had grown the pinned result block (`pinned()` freed the old
block without bumping the generation before c6cc7e9): the replay's copy node wrote to freed host
memory.  These tests drive exactly that sequence -- one-frame graphs, interleaved with batches and
service calls that grow the arena and the pinned blocks -- with the graph floor at one frame, and hold
every result to direct launches and the oracle."""
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


def _one(ctx, b, inl):
    inl.fill_(-7)
    res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
    return res, inl[:int(res[0]["n_inliers"])].cpu().numpy()


def test_one_frame_graph_survives_arena_and_pinned_growth():
    """The round-3 fault's sequence: a one-frame layout captured into a graph, then batches that grow
    the pinned result / chunk-stat blocks and the device arena, then the one-frame layout again.  The
    stale graph must not replay (the arena generation moved, so the key is new: first sight launches
    directly, the second recaptures), and every result stays bit-exact."""
    frame = [pitt.synth_frame(0, 7100, 160, 120)]
    big = [pitt.synth_frame(s % 3, 7200 + s, 160, 120) for s in range(160)]  # 160 records > one 4 KB pinned block
    b1 = pitt.FrameBatch.from_host(frame, device="cuda:0")
    bb = pitt.FrameBatch.from_host(big, device="cuda:0")
    inl1 = torch.empty(b1.capacity, dtype=torch.int32, device="cuda:0")
    inlb = torch.empty(bb.capacity, dtype=torch.int32, device="cuda:0")
    ctx = _ctx(PITT_GRAPHS=1, PITT_GRAPH_MIN_FRAMES=1)
    try:
        ref, ref_inl = _one(ctx, b1, inl1)               # first sight: direct
        for _ in range(2):                               # capture, then replay
            r, i = _one(ctx, b1, inl1)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl)
        assert ctx.graph_stats() == (1, 1)
        # grows "results_h" (160 x 48 B > 4096 B), the device arena (tiles x frames), "meta_h" ...
        res_b = ctx.plane_segment_batch(bb, pitt.sac_params(), inlb)
        # ... and more iterations per frame: more chunks, a larger "cstat_h" and larger hypothesis buffers
        res_c = ctx.plane_segment_batch(bb, pitt.sac_params(max_iterations=5000), inlb)
        caps, reps = ctx.graph_stats()
        for k in range(3):                               # new generation: direct, capture, replay
            r, i = _one(ctx, b1, inl1)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl), k
        assert ctx.graph_stats() == (caps + 1, reps + 1), "a graph from before the arena moved was replayed"
        P._check(ctx, frame, ref, [ref_inl])
        ib = inlb.cpu().numpy()
        sample = [0, 1, 2, 77, 159]
        P._check(ctx, [big[f] for f in sample], res_c[sample],
                 [ib[bb.offsets[f]:bb.offsets[f] + res_c[f]["n_inliers"]] for f in sample], max_iterations=5000)
        assert res_b["hypotheses"].min() > 0
    finally:
        ctx.close()


def test_one_frame_graphs_between_service_calls():
    """One-frame plane graphs replayed between the primitive services' direct launches on the same
    context and stream (the round-3 setting), with clusters of growing size so that every service
    grows its scratch between replays: the plane results equal a graph-free context's."""
    ctx = _ctx(PITT_GRAPHS=1, PITT_GRAPH_MIN_FRAMES=1)
    ref_ctx = _ctx(PITT_GRAPHS=0)
    srv, ref_srv = pitt.Services(ctx), pitt.Services(ref_ctx)
    try:
        frame = [pitt.synth_frame(0, 7300, 160, 120)]
        b1 = pitt.FrameBatch.from_host(frame, device="cuda:0")
        inl1 = torch.empty(b1.capacity, dtype=torch.int32, device="cuda:0")
        ref, ref_inl = _one(ref_ctx, b1, inl1)
        replays0 = ctx.graph_stats()[1]
        for k, n in enumerate((300, 300, 1200, 1200, 4000, 9000, 300)):
            cloud = sphere_scene(n, n // 5, 900 + k).astype(np.float32)
            a = srv.ransac_sphere(cloud)
            c = srv.ransac_plane(cloud)     # a one-frame batch through the single-cloud ABI (pinned staging)
            assert a[0] == ref_srv.ransac_sphere(cloud)[0]
            d = ref_srv.ransac_plane(cloud)
            assert c[0] == d[0] and np.array_equal(c[1], d[1]) and np.array_equal(c[2].view(np.int32), d[2].view(np.int32))
            r, i = _one(ctx, b1, inl1)
            assert r.tobytes() == ref.tobytes() and np.array_equal(i, ref_inl), k
        assert ctx.graph_stats()[1] > replays0  # some of those one-frame batches did replay a graph
    finally:
        srv.close()
        ref_srv.close()
        ctx.close()
        ref_ctx.close()
