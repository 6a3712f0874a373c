"""k_xrefine: optimizeModelCoefficients' nine exact-order float sums by binade runs (DESIGN.md s3,
"Binade runs").  Bar: bit-exact with the oracle's sequential float chain (and with k_refine's serial
chain, $PITT_XREFINE=0) on clouds built to break the run logic: sums that cross zero at every point,
dyadic coordinates (exact ties on the run grid at every binade), sums that land on powers of two,
huge coordinates (run grids coarser than the values), and tiny ones (denormal products).  Also the
forced hand-back path ($PITT_XREFINE=2: every frame refined again by the serial chain) and the
hand-back count on table frames."""
import os

import numpy as np
import pytest
import torch

import pitt_object_table_segmentation_amd as pitt
from pitt_object_table_segmentation_amd import _lib
import test_plane_gpu as P

# k_xrefine is an A/B variant: compiled only into libpitt_seg_ab.so (tests/test_variants_gpu.py)
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not (_lib.lib.pitt_build_flags() & _lib.PITT_BUILD_AB_VARIANTS),
                                                  reason="A/B variant: run under libpitt_seg_ab.so")]


def _ctx(xrefine):
    old = os.environ.get("PITT_XREFINE")
    os.environ["PITT_XREFINE"] = str(xrefine)
    try:
        return pitt.Context(0)
    finally:
        if old is None:
            del os.environ["PITT_XREFINE"]
        else:
            os.environ["PITT_XREFINE"] = old


def _frames():
    n = 60000
    i = np.arange(n, dtype=np.float64)
    rng = np.random.default_rng(11)
    out = []
    # x alternates sign: the x, xy, xz sums cross zero at every point
    x = ((-1.0) ** i) * (0.25 + 0.5 * rng.random(n))
    y = i * 1e-4 - 3.0
    z = 1.0 + 0.002 * np.sin(i * 0.7)
    out.append((x, y, z))
    # dyadic coordinates: products and sums are short binary fractions, ties at every grid
    x = rng.integers(-512, 513, n) / 256.0
    y = rng.integers(-512, 513, n) / 64.0
    z = np.full(n, 1.5) + rng.integers(-2, 3, n) / 1024.0
    out.append((x, y, z))
    # x = 1 + tiny: the x sum walks through every power of two exactly
    x = 1.0 + (i % 7) * 2.0 ** -20
    y = (i // 7) * 2.0 ** -10
    z = np.full(n, 3.0) + (i % 3) * 2.0 ** -12
    out.append((x, y, z))
    # far from the origin: sums around 1e10, run grids of thousands
    x = 1000.0 + rng.random(n)
    y = -2000.0 + rng.random(n)
    z = 1500.0 + 0.001 * rng.random(n)
    out.append((x, y, z))
    # small coordinates: run grids near 2^-90
    x = (rng.random(n) - 0.3) * 1e-15
    y = (rng.random(n) - 0.6) * 1e-15
    z = np.full(n, 0.25) + 0.001 * rng.random(n)
    out.append((x, y, z))
    # tiny coordinates: denormal products (the covariance degenerates to a NaN plane in PCL too)
    x = (rng.random(n) - 0.3) * 1e-19
    y = (rng.random(n) - 0.6) * 1e-19
    z = np.full(n, 0.25) + 0.001 * rng.random(n)
    out.append((x, y, z))
    # a table frame with the plane's sums crossing zero mid-frame (camera centred on the table)
    x, y, z = pitt.synth_frame(0, 1000, 320, 240)
    out.append((x - np.float32(np.median(x)), y - np.float32(np.median(y)), z))
    return [tuple(np.ascontiguousarray(a, np.float32) for a in f) for f in out]


@pytest.fixture(scope="module")
def frames():
    return _frames()


@pytest.mark.parametrize("mode", [1, 2, 0])
def test_adversarial_sums_bit_exact(frames, mode):
    ctx = _ctx(mode)
    try:
        res, inls = P._run_batch(ctx, frames)
        P._check(ctx, frames, res, inls)
        batches, handed_back = ctx.refine_stats()
        if mode == 0:
            assert (batches, handed_back) == (0, 0)
        else:
            assert batches == 1
            if mode == 2:
                assert handed_back == sum(1 for r in res if r["n_coeff"] == 4)
    finally:
        ctx.close()


def test_runs_equal_serial_chain_on_table_batch():
    """64 table / clutter frames: k_xrefine's records and inlier lists equal the serial chain's, and it
    hands back (almost) no frame."""
    frames = [pitt.synth_frame(s, 3000 + j, 640, 480) for j, s in enumerate([0] * 56 + [1] * 4 + [2] * 4)]
    b = pitt.FrameBatch.from_host(frames, device="cuda:0")
    outs = []
    for mode in (1, 0):
        ctx = _ctx(mode)
        try:
            inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
            res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
            outs.append((res, inl.cpu().numpy(), ctx.refine_stats()))
        finally:
            ctx.close()
    (r1, i1, st1), (r0, i0, _) = outs
    assert r1.tobytes() == r0.tobytes()
    for o, r in zip(b.offsets, r0):
        assert np.array_equal(i1[o:o + r["n_inliers"]], i0[o:o + r["n_inliers"]])
    assert st1[0] == 1 and st1[1] <= 1, st1
