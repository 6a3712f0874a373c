"""optimizeModelCoefficients' nine float sums by the block-parallel exact walk (csrc/xsum.hpp, DESIGN.md
s3d), the refinement of batches of up to 8 frames ($PITT_XS_MAX_FRAMES): bit-exact with the oracle's
sequential float chain and with k_refine's serial chain ($PITT_XS_MAX_FRAMES=0), on clouds built to
defeat the walk's predictions -- sums that cross zero at every point, dyadic coordinates (exact ties
on every grid), sums that land on powers of two, coordinates near 1000 m, tiny and denormal-scale
coordinates -- and on table / clutter / NaN frames."""
import os

import numpy as np
import pytest
import torch

import pitt_object_table_segmentation_amd as pitt
import test_plane_gpu as P
from test_xrefine_gpu import _frames

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


@pytest.fixture(scope="module")
def adversarial():
    return _frames()


def _run(ctx, frames):
    b = pitt.FrameBatch.from_host(frames, device="cuda:0")
    inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
    res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
    h = inl.cpu().numpy()
    return res, [h[o:o + r["n_inliers"]] for o, r in zip(b.offsets, res)]


def test_walk_equals_chain_and_oracle_on_adversarial_sums(adversarial):
    walk, chain = _ctx(), _ctx(PITT_XS_MAX_FRAMES=0)
    try:
        rw, iw = _run(walk, adversarial)
        rc, ic = _run(chain, adversarial)
        assert rw.tobytes() == rc.tobytes()
        assert all(np.array_equal(a, b) for a, b in zip(iw, ic))
        P._check(walk, adversarial, rw, iw)
    finally:
        walk.close()
        chain.close()


@pytest.mark.parametrize("order,div", [(pitt.REDUCE_SSE2, pitt.DIV_EIGEN32), (pitt.REDUCE_HADD, pitt.DIV_TRUE),
                                       (pitt.REDUCE_SEQ, pitt.DIV_EIGEN32)])
def test_walk_single_frames_and_orders(ctx, order, div):
    """One 640x480 frame at a time (the single-cloud service's batch), every reduction order."""
    for scene, seed in ((pitt.SCENE_TABLE, 9100), (pitt.SCENE_TABLE_NAN, 9101), (pitt.SCENE_CLUTTER, 9102)):
        fr = [pitt.synth_frame(scene, seed, 640, 480)]
        b =pitt.FrameBatch.from_host(fr, device="cuda:0")
        inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
        res = ctx.plane_segment_batch(b, pitt.sac_params(reduce_order=order, div_mode=div), inl)
        h = inl.cpu().numpy()
        P._check(ctx, fr, res, [h[:res[0]["n_inliers"]]], reduce_order=order, div_mode=div)
