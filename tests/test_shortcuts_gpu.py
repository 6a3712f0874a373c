"""Adversarial cases for the exact shortcuts of the plane path: the per-frame
hypothesis limit, pass-1 tile skipping by the winning hypothesis' per-tile counts, and pass-2 tile
skipping by tile bounding boxes against the refined plane's slab.  Each frame is compared with
the oracle bit for bit (counts, winning hypothesis, inlier indices, coefficients)."""
import numpy as np
import pytest

import pitt_object_table_segmentation_amd as pitt
from test_plane_gpu import _check, _run_batch

pytestmark = pytest.mark.gpu

TILE = 2048


def _plane_scene(rng, n_tiles, plane_tiles, noise=0.002, far=5.0, nan_tiles=()):
    """Tiles of sparse volumetric clutter far from z = 0, with a noisy z = 0 plane patch filling
    `plane_tiles` and all-NaN tiles at `nan_tiles`."""
    n = n_tiles * TILE
    x = rng.uniform(-5, 5, n).astype(np.float32)
    y = rng.uniform(-5, 5, n).astype(np.float32)
    z = rng.uniform(far, far + 20, n).astype(np.float32)
    for t in plane_tiles:
        s = slice(t * TILE, (t + 1) * TILE)
        z[s] = rng.normal(0, noise, TILE).astype(np.float32)
    for t in nan_tiles:
        s = slice(t * TILE, (t + 1) * TILE)
        x[s] = y[s] = z[s] = np.nan
    return x, y, z


def test_inliers_confined_to_one_tile(ctx):
    """Only the plane tile holds inliers of the winning hypothesis: pass 1 skips every other tile
    by its count, pass 2 by its box (clutter boxes lie far off the slab, NaN tiles are empty)."""
    rng = np.random.default_rng(11)
    frames = [_plane_scene(rng, 5, [p]) for p in (0, 2, 4)]
    frames.append(_plane_scene(rng, 40, [17], nan_tiles=[t for t in range(40) if t not in (3, 17, 30, 39)]))
    res, inls = _run_batch(ctx, frames)
    _check(ctx, frames, res, inls)


def test_infinite_and_nan_coordinates(ctx):
    rng = np.random.default_rng(12)
    frames = []
    for k in range(3):
        x, y, z = _plane_scene(rng, 30, range(5, 20))
        idx = rng.choice(len(x), 300, replace=False)
        x[idx[:100]] = np.inf
        y[idx[100:200]] = -np.inf
        z[idx[200:]] = np.nan
        # a whole tile of NaN (empty box) and one of infinities (never skipped)
        x[2 * TILE:3 * TILE] = np.nan
        z[25 * TILE:26 * TILE] = np.inf if k != 1 else -np.inf
        frames.append((x, y, z))
    res, inls = _run_batch(ctx, frames, max_iterations=300)
    _check(ctx, frames, res, inls, max_iterations=300)


def _ulps(v, k):
    """v moved by k ulps (float32)."""
    v = np.float32(v)
    for _ in range(abs(k)):
        v = np.nextafter(v, np.float32(np.inf) if k > 0 else np.float32(-np.inf))
    return np.float32(v)


def test_points_straddling_the_threshold(ctx):
    """Exact z = 0 plane patch (the refined plane is z = 0 up to rounding) plus isolated points in
    otherwise empty (NaN) tiles at |z| = t +- a few ulps: those tiles' boxes sit right at the slab
    edge, so pass 2's box test must keep them (the refined plane's tilt decides each point)."""
    rng = np.random.default_rng(13)
    for th in (0.007, 0.00700001, 0.02):
        t = pitt.float_threshold(th)
        x, y, z = _plane_scene(rng, 32, range(8, 20), noise=0.0, nan_tiles=range(21, 31))
        for k, tile in enumerate(range(21, 31)):
            j = tile * TILE + 17 * k
            sign = np.float32(1 if k % 2 else -1)
            for u in range(-3, 4):
                x[j + u + 3], y[j + u + 3] = rng.uniform(-5, 5, 2).astype(np.float32)
                z[j + u + 3] = sign * _ulps(t, u)
        frames = [(x, y, z)]
        res, inls = _run_batch(ctx, frames, threshold=th, max_iterations=100)
        _check(ctx, frames, res, inls, threshold=th, max_iterations=100)


def test_groups_inside_the_slab(ctx):
    """k_score's inside shortcut ($PITT_INSIDE_CULL, off by default): a (64-point group, hypothesis) pair
    whose box lies certainly inside the slab counts the group's points with three non-NaN coordinates.
    Thin planes (noise far below t) give many such pairs; their groups carry points with one NaN
    coordinate (x, y or z alone: they never widen the box and never count), all-NaN groups, and
    groups whose box reaches t - a few ulps (not certified: scored point by point)."""
    rng = np.random.default_rng(15)
    frames = []
    for k in range(4):
        x, y, z = _plane_scene(rng, 24, range(2, 22), noise=0.0002 if k < 2 else 0.0)
        n = len(x)
        idx = rng.choice(np.arange(2 * TILE, 22 * TILE), 3000, replace=False)
        x[idx[:1000]] = np.nan
        y[idx[1000:2000]] = np.nan
        z[idx[2000:]] = np.nan
        g = (5 + k) * TILE + 64 * 3  # one whole group of NaN points
        x[g:g + 64] = y[g:g + 64] = z[g:g + 64] = np.nan
        if k >= 2:  # exact z = 0 plane with groups whose extreme point sits at +-t - u ulps
            t = pitt.float_threshold(0.007)
            for j, u in enumerate(range(1, 9)):
                q = (10 + j) * TILE + 64 * j + 5
                z[q] = np.float32((-1) ** j) * _ulps(t, -u)
        frames.append((x, y, z))
    assert n == 24 * TILE
    res, inls = _run_batch(ctx, frames, max_iterations=200)
    _check(ctx, frames, res, inls, max_iterations=200)


def test_later_chunks_and_hypothesis_limit(ctx):
    """Low-inlier-ratio frames run many chunks (the per-frame limit applies from chunk 1 on);
    mixed with easy frames so chunk work lists shrink unevenly."""
    rng = np.random.default_rng(14)
    frames = [_plane_scene(rng, 24, [3, 4], noise=0.003), pitt.synth_frame(1, 3001, 320, 240),
              _plane_scene(rng, 24, range(24), noise=0.001), pitt.synth_frame(0, 3002, 320, 240)]
    res, inls = _run_batch(ctx, frames)
    _check(ctx, frames, res, inls)


def test_lazy_hypothesis_generation_across_windows(ctx):
    """Hypotheses are generated in windows of 256 sampler attempts, only as far as the chunks
    need them.  Mostly-collinear clouds (exact line x = t, y = 2t, z = 3t: every all-line sample is
    rejected) spread the good samples over many windows, put runs of rejections across window
    borders, and at 99.9 % on the line hit getSamples' 1000-rejection cut-off mid-stream."""
    rng = np.random.default_rng(15)
    frames = []
    for frac, n in ((0.95, 20000), (0.99, 20000), (0.999, 30000), (0.8, 5000)):
        t = (rng.integers(0, 4000, n) * 0.25).astype(np.float32)
        x, y, z = t.copy(), np.float32(2) * t, np.float32(3) * t
        off = rng.random(n) >= frac
        k = int(off.sum())
        x[off] = rng.uniform(-50, 50, k).astype(np.float32)
        y[off] = rng.uniform(-50, 50, k).astype(np.float32)
        z[off] = rng.uniform(-50, 50, k).astype(np.float32)
        frames.append((x, y, z))
    kw = dict(max_iterations=150, sampler_slack=7000)
    res, inls = _run_batch(ctx, frames, **kw)
    _check(ctx, frames, res, inls, max_iterations=150)
