"""The first scoring chunk has two implementations: the survivor-list scorer
(compaction, v_cmp -> s_bcnt1 -> v_writelane per surviving (group, hypothesis) pair) and the
lane-counter scorer (k_score LANE: every surviving pair with full-rate VALU only, |d| - t sign bits
added into lane-private counters).  Either way a pair whose group box lies certainly inside the slab
may count the group's non-NaN points without scoring them ($PITT_INSIDE_CULL, off by default).  $PITT_LANE_SCORE picks one when a context is created (A/B
build only); the other is run here on the bit-exact parity tests of the plane path, so both stay exact.  Likewise k_refine's
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
from pitt_object_table_segmentation_amd import _lib
import test_plane_gpu as P
import test_shortcuts_gpu as S

# The variants exist only in the A/B build (libpitt_seg_ab.so, `make ab`); the product library ignores
# their environment knobs.  tests/test_variants_gpu.py runs this module under the A/B build.
AB_BUILD = bool(_lib.lib.pitt_build_flags() & _lib.PITT_BUILD_AB_VARIANTS)
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not AB_BUILD, reason="A/B variants: run under libpitt_seg_ab.so "
                                                                          "(tests/test_variants_gpu.py)")]


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
