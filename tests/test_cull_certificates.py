"""The two box certificates of k_score (csrc/plane_ransac.hip: box_clear, box_inside), restated in
numpy and checked for soundness on CPU against PCL's float evaluation of every point
(SampleConsensusModelPlane::countWithinDistance, sample_consensus/impl/sac_model_plane.hpp in PCL 1.7,
called at plane_segmentation_srv.cpp:67 through RandomSampleConsensus::computeModel).

box_clear  -- every point of the group certainly fails |c . (p, 1)| < t: the pair is culled (counts 0);
box_inside -- every point certainly passes: the pair counts the group's points with no NaN coordinate
              (PITT_INSIDE_CULL).

Both use the group's float axis-aligned box (centre 0.5 (lo + hi), half extent 0.5 (hi - lo)) and a
margin of 1e-5 S, S = (|a| + |b| + |c|) M + |d|, M the box's largest |coordinate|.  The device
evaluates the bounds with FMAs; here they are evaluated in float64 and rounded to float32, which differs
from the device by a few float32 ulps of S -- far inside the margin, which is what this test pins: no
certified pair may contain a point whose PCL-order float32 distance decides the other way, in any of
the three reduce orders (A3)."""
import warnings

import numpy as np
import pytest

F = np.float32


def _red4(a0, a1, a2, a3, order):
    if order == 1:
        return (a0 + a1) + (a2 + a3)
    if order == 2:
        return ((a0 + a1) + a2) + a3
    return (a0 + a2) + (a1 + a3)


def _pcl_dist(c, x, y, z, order):
    """|VectorXf(4).dot(Vector4f(x, y, z, 1))| in float32, in the given reduce order (no FMA)."""
    with np.errstate(invalid="ignore", over="ignore"):
        return np.abs(_red4(F(c[0]) * x, F(c[1]) * y, F(c[2]) * z, F(c[3]), order))


def _certificates(G, c, t):
    """(clear, inside) for groups G (n, 64, 3) float32 against coefficients c (float32 x4)."""
    with np.errstate(invalid="ignore", over="ignore"), warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)  # all-NaN groups: an empty (NaN) box
        lo = np.nanmin(G, axis=1)
        hi = np.nanmax(G, axis=1)
        cen = (F(0.5) * (lo + hi)).astype(F)
        h = (F(0.5) * (hi - lo)).astype(F)
        m = np.max(np.abs(np.concatenate([lo, hi], axis=1)), axis=1).astype(F)
        c64 = c.astype(np.float64)
        n1 = F(abs(c[0]) + abs(c[1]) + abs(c[2]))
        s = F(np.float64(n1) * m + (abs(c64[3]) + 1e-25))
        dc = F(cen.astype(np.float64) @ c64[:3] + c64[3])
        rr = F(h.astype(np.float64) @ np.abs(c64[:3]))
        clear = np.abs(dc) - rr > F(1e-5 * np.float64(s) + t)
        inside = np.abs(dc) + rr < F(-1e-5 * np.float64(s) + t)
    return clear, inside


def _groups(rng, n, scale, spread, nan_rate):
    """n groups of 64 points near a random plane patch: offsets of a few thresholds, random tilt."""
    centre = rng.uniform(-scale, scale, (n, 1, 3))
    pts = centre + rng.normal(0, spread, (n, 64, 3)) * rng.uniform(0.05, 1.0, (n, 1, 3))
    G = pts.astype(F)
    if nan_rate:
        mask = rng.random((n, 64, 3)) < nan_rate
        G[mask] = np.nan
    return G


@pytest.mark.parametrize("order", [0, 1, 2])
@pytest.mark.parametrize("scale,spread,t", [(1.0, 0.01, 0.007), (3.0, 0.003, 0.007), (0.5, 0.02, 0.02),
                                            (100.0, 0.05, 0.007), (1e-3, 1e-5, 1e-5)])
def test_certificates_are_sound(order, scale, spread, t):
    rng = np.random.default_rng(int(scale * 1000) + order * 7 + int(t * 1e6))
    t = F(t)
    n_in = n_clear = 0
    for _ in range(40):
        G = _groups(rng, 256, scale, spread, nan_rate=0.02)
        # a hypothesis through a random group's centre, tilted, shifted by a few thresholds
        k = rng.integers(len(G))
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            p0 = np.nan_to_num(np.nanmean(G[k].astype(np.float64), axis=0))
        nrm = rng.normal(0, 1, 3)
        nrm /= np.linalg.norm(nrm)
        c = np.empty(4)
        c[:3] = nrm
        c[3] = -(nrm @ p0) + rng.normal(0, 3) * float(t)
        c = c.astype(F)
        # half the groups flattened towards the plane (distances shrunk to 0-2 thresholds), so both
        # certificates and the undecided band between them are populated
        G64 = G[:128].astype(np.float64)
        dist = G64 @ c[:3].astype(np.float64) + np.float64(c[3])
        keep = rng.uniform(0, 2, (128, 1)) * float(t) / np.maximum(np.nanmax(np.abs(dist), axis=1, keepdims=True), 1e-30)
        G[:128] = (G64 - (dist * (1 - np.minimum(keep, 1)))[..., None] * c[:3].astype(np.float64)).astype(F)
        clear, inside = _certificates(G, c, t)
        assert not np.any(clear & inside)
        d = _pcl_dist(c, G[..., 0], G[..., 1], G[..., 2], order)
        with np.errstate(invalid="ignore"):
            passes = d < t  # NaN distances never pass
        # culled: no point passes; inside: every point with three non-NaN coordinates passes
        assert not np.any(passes[clear]), "box_clear culled a group holding an inlier"
        finite = ~np.isnan(G).any(axis=2)
        assert np.array_equal(passes[inside], finite[inside]), "box_inside certified a group holding an outlier"
        n_in += int(inside.sum())
        n_clear += int(clear.sum())
    assert n_clear > 0  # the cull fired on every scene
    # the inside certificate too, except 100 m out: its margin (1e-5 S ~ 1 mm) plus a tilted 5 cm
    # patch's box depth leave no room below t there
    assert n_in > 0 or scale >= 100


def test_certificates_refuse_nan_and_infinite_boxes():
    G = np.zeros((3, 64, 3), F)
    G[0, :, :] = np.nan  # all-NaN group: an empty box
    G[1, 5, 0] = np.inf
    G[2, 7, 2] = -np.inf
    c = np.array([0, 0, 1, 0], F)
    clear, inside = _certificates(G, c, F(0.007))
    assert not clear.any() and not inside.any()


def test_points_at_the_threshold_are_not_certified():
    """Groups whose extreme point sits a few ulps inside or outside t are left to the exact scorer."""
    t = F(0.007)
    G = np.zeros((16, 64, 3), F)
    G[..., 0] = np.linspace(-1, 1, 64, dtype=F)
    for i in range(16):
        v = t
        for _ in range(i - 8):
            v = np.nextafter(v, F(np.inf))
        for _ in range(8 - i):
            v = np.nextafter(v, F(-np.inf))
        G[i, 0, 2] = v
    clear, inside = _certificates(G, np.array([0, 0, 1, 0], F), t)
    assert not clear.any() and not inside.any()
