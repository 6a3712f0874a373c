"""The first scoring chunk has two implementations: the survivor-list scorer
(compaction, v_cmp -> s_bcnt1 -> v_writelane per surviving (group, hypothesis) pair) and the
lane-counter scorer (k_score LANE: every surviving pair with full-rate VALU only, |d| - t sign bits
added into lane-private counters).  Either way a pair whose group box lies certainly inside the slab
may count the group's non-NaN points without scoring them ($PITT_INSIDE_CULL, off by default).  $PITT_LANE_SCORE picks one when a context is created; the other
is run here on the bit-exact parity tests of the plane path, so both stay exact.  Likewise k_refine's
producer count ($PITT_REFINE_PRODUCERS, 1..4 waves selecting steps in parallel and appending in
step order): every count must give the same ascending inlier stream, hence the same floats.  The
refinement itself has two paths: k_refine's serial chain (default) and k_xrefine's binade runs
($PITT_XREFINE=1, with k_refine as the fallback for frames it hands back: $PITT_XREFINE=2 hands back
every frame, so the fallback launch is covered too).  k_refine_multi ($PITT_REFINE_FRAMES = 2, 3) runs
2 or 3 frames per block with one chain wave for all of them: per frame the same sums in the same
order, so the same bits."""
import os

import pytest

import pitt_object_table_segmentation_amd as pitt
import test_plane_gpu as P
import test_shortcuts_gpu as S

pytestmark = pytest.mark.gpu


VARIANTS = [{"PITT_LANE_SCORE": "0"}, {"PITT_LANE_SCORE": "1"}, {"PITT_REFINE_PRODUCERS": "1"},
            {"PITT_REFINE_PRODUCERS": "2"}, {"PITT_REFINE_PRODUCERS": "4"}, {"PITT_XREFINE": "1"},
            {"PITT_XREFINE": "2"}, {"PITT_REFINE_FRAMES": "1"}, {"PITT_REFINE_FRAMES": "2"},
            {"PITT_REFINE_FRAMES": "3"}, {"PITT_REFINE_MODE": "10"}, {"PITT_INSIDE_CULL": "0"},
            {"PITT_INSIDE_CULL": "1"}]


@pytest.fixture(scope="module", params=VARIANTS, ids=lambda v: "-".join(f"{k[5:].lower()}{x}" for k, x in v.items()))
def path_ctx(request):
    old = {k: os.environ.get(k) for k in request.param}
    os.environ.update(request.param)
    try:
        c = pitt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    yield c
    c.close()


CASES = [P.test_full_size_frames_bit_exact, P.test_support_service_parameters, P.test_ragged_batch_and_edge_frames,
         P.test_no_optimize_and_thresholds, S.test_inliers_confined_to_one_tile, S.test_infinite_and_nan_coordinates]
CASES += [getattr(S, n) for n in dir(S) if n.startswith("test_") and getattr(S, n) not in CASES
          and getattr(S, n).__code__.co_argcount == 1]


@pytest.mark.parametrize("case", CASES, ids=[c.__name__ for c in CASES])
def test_both_scoring_paths_bit_exact(path_ctx, case):
    case(path_ctx)


def test_both_paths_reduce_orders(path_ctx):
    for order in (pitt.REDUCE_SSE2, pitt.REDUCE_HADD, pitt.REDUCE_SEQ):
        P.test_reduce_orders_and_division_modes(path_ctx, order, pitt.DIV_EIGEN32)


def test_hip_graph_replay_bit_exact():
    """Repeated batch layouts are captured into a HIP graph (second sight) and replayed (third on):
    the replays give the same records and inlier lists as direct launches ($PITT_GRAPHS=0) and the
    oracle (pipelining)."""
    import numpy as np
    import torch
    frames = [pitt.synth_frame(s, seed, 320, 240) for s, seed in ((0, 7000), (1, 7001), (2, 7002), (0, 7003))]
    b = pitt.FrameBatch.from_host(frames, device="cuda:0")
    old = {k: os.environ.get(k) for k in ("PITT_GRAPHS", "PITT_GRAPH_MIN_FRAMES")}
    try:
        os.environ["PITT_GRAPHS"] = "0"
        direct = pitt.Context(0)
        os.environ["PITT_GRAPHS"] = "1"
        os.environ["PITT_GRAPH_MIN_FRAMES"] = "1"  # graphs for this 4-frame layout (default: 64 frames and up)
        graphed = pitt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
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
