"""The cylinder / cone services' post-processing: the cloud projected on the
fitted axis and the O(n^2) search for the two projected points farthest apart
(cylinder_segmentation_srv.cpp:129-189, cone_segmentation_srv.cpp:129-189; helpers :53-79).

CPU: the oracle's restatement against an independent numpy float32 restatement (same operation
order, vectorised over all pairs) -- projection, height, pair and centroid bit-exact -- and the edge
cases the reference's loops define (no pair, duplicate points, ties, NaN points).
GPU: pitt_axis_height against the oracle, bit-exact, both modes.
"""
import numpy as np
import pytest

import oracle_binding as orc

F = np.float32


def cylinder_cloud(n, seed, radius=0.04, h=0.15, noise=0.002, axis=(0.1, 0.2, 1.0), base=(0.3, -0.1, 0.9)):
    """Points on a cylinder surface around `axis` through `base` (a fitted model's axis), with noise."""
    rng = np.random.default_rng(seed)
    a = np.asarray(axis, np.float64)
    a /= np.linalg.norm(a)
    u = np.cross(a, [1.0, 0.0, 0.0])
    u /= np.linalg.norm(u)
    v = np.cross(a, u)
    t = rng.uniform(0, h, n)
    phi = rng.uniform(0, 2 * np.pi, n)
    p = np.asarray(base) + t[:, None] * a + radius * (np.cos(phi)[:, None] * u + np.sin(phi)[:, None] * v)
    p += rng.normal(0, noise, p.shape)
    coef = np.array(list(base) + list(np.asarray(axis) * 0.7) + [radius], np.float32)  # unnormalised axis
    return p.astype(np.float32), coef


def numpy_axis_height(p, coef, mode):
    """Independent restatement: float32 numpy in the reference's operation order."""
    c = coef.astype(F)
    norm = np.sqrt(c[3] * c[3] + c[4] * c[4] + c[5] * c[5], dtype=F)
    d = np.array([c[3] / norm, c[4] / norm, c[5] / norm], F)
    a1 = np.array([c[k] + d[k] * F(-1.0) for k in range(3)], F)
    a2 = np.array([c[k] + d[k] * F(1.0) for k in range(3)], F)
    u = (a2 - a1).astype(F)
    gdiv = F(u[0] * u[0] + u[1] * u[1] + u[2] * u[2])
    v = (p - a1).astype(F)
    g = ((v[:, 0] * u[0] + v[:, 1] * u[1] + v[:, 2] * u[2]) / gdiv).astype(F)
    q = np.stack([a1[k] + g * u[k] for k in range(3)], 1).astype(F)
    n = len(p)
    h, i1, i2 = F(-1.0), -1, -1
    if n >= 2:
        ex = q[:, None, 0] - q[None, :, 0]
        ey = q[:, None, 1] - q[None, :, 1]
        ez = q[:, None, 2] - q[None, :, 2]
        dist = np.sqrt(ex * ex + ey * ey + ez * ez).astype(F)
        dist[np.triu_indices(n)] = np.nan  # only i > j
        if not np.all(np.isnan(dist)):
            m = np.nanmax(dist)
            ii, jj = np.nonzero(dist == m)
            k = np.lexsort((jj, ii))[0]  # first in (i, j) loop order
            h, i1, i2 = m, int(ii[k]), int(jj[k])
    if mode == 0:
        cen = (q[i1] + q[i2]) / F(2) if i1 >= 0 else np.full(3, np.nan, F)
    else:
        cen = np.array([c[k] + F(3.0 / 4.0) * h * d[k] for k in range(3)], F)
    return F(h), i1, i2, cen.astype(F), q


def same(a, b):
    a, b = np.asarray(a, F), np.asarray(b, F)
    return np.array_equal(a.view(np.int32), b.view(np.int32)) or (np.isnan(a).all() and np.isnan(b).all())


@pytest.mark.parametrize("n,seed,mode", [(2, 1, 0), (3, 2, 1), (200, 3, 0), (777, 4, 1), (1500, 5, 0)])
def test_oracle_axis_height_matches_numpy(n, seed, mode):
    p, coef = cylinder_cloud(n, seed)
    h, i1, i2, cen, q = orc.axis_height(*p.T, coef, mode)
    wh, wi1, wi2, wcen, wq = numpy_axis_height(p, coef, mode)
    assert same(q, wq)
    assert same(h, wh) and (i1, i2) == (wi1, wi2)
    assert same(cen, wcen)


def test_oracle_axis_height_edges():
    coef = np.array([0, 0, 0, 0, 0, 2], np.float32)
    # no pair
    for n in (0, 1):
        p = np.full((n, 3), 0.5, np.float32)
        h, i1, i2, cen, _ = orc.axis_height(*p.T, coef, 0)
        assert h == -1.0 and (i1, i2) == (-1, -1) and np.isnan(cen).all()
        h, i1, i2, cen, _ = orc.axis_height(*p.T, coef, 1)
        assert h == -1.0 and np.array_equal(cen, np.array([0, 0, -0.75], np.float32))
    # duplicates: height 0 at the first pair (1, 0)
    p = np.full((5, 3), 0.25, np.float32)
    h, i1, i2, _, _ = orc.axis_height(*p.T, coef, 0)
    assert h == 0.0 and (i1, i2) == (1, 0)
    # ties: points at z = -1, 1, -1, 1 -> the first maximal pair in loop order is (1, 0)
    p = np.array([[0, 0, -1], [0, 0, 1], [1, 0, -1], [1, 1, 1]], np.float32)
    h, i1, i2, cen, _ = orc.axis_height(*p.T, coef, 0)
    assert h == 2.0 and (i1, i2) == (1, 0) and np.array_equal(cen, np.zeros(3, np.float32))
    # NaN points never win
    p = np.array([[0, 0, 0.1], [np.nan, 0, 5], [0, 0, 0.4]], np.float32)
    h, i1, i2, _, _ = orc.axis_height(*p.T, coef, 0)
    wh = numpy_axis_height(p, coef, 0)[0]
    assert (i1, i2) == (2, 0) and same(h, wh) and abs(h - 0.3) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,mode", [(2, 11, 0), (3, 12, 1), (255, 13, 0), (256, 14, 1), (257, 15, 0),
                                         (1000, 16, 1), (4097, 17, 0), (20000, 18, 1), (30000, 19, 0)])
def test_hip_axis_height_matches_oracle(ctx, n, seed, mode):
    import torch
    p, coef = cylinder_cloud(n, seed)
    t = [torch.from_numpy(np.ascontiguousarray(p[:, k])).cuda() for k in range(3)]
    h, i1, i2, cen, (px, py, pz) = ctx.axis_height(*t, coef, mode, projected=True)
    wh, wi1, wi2, wcen, wq = orc.axis_height(*p.T, coef, mode)
    assert same(np.stack([px.cpu().numpy(), py.cpu().numpy(), pz.cpu().numpy()], 1), wq)
    assert same(h, wh) and (i1, i2) == (wi1, wi2)
    assert same(cen, wcen)


@pytest.mark.gpu
def test_hip_axis_height_edges(ctx):
    import torch
    coef = np.array([0, 0, 0, 0, 0, 2], np.float32)
    cases = [np.zeros((0, 3), np.float32), np.full((1, 3), 0.5, np.float32), np.full((600, 3), 0.25, np.float32),
             np.array([[0, 0, -1], [0, 0, 1], [1, 0, -1], [1, 1, 1]], np.float32),
             np.array([[0, 0, 0.1], [np.nan, 0, 5], [0, 0, 0.4]], np.float32)]
    rng = np.random.default_rng(7)
    tie = rng.choice([-1.0, 1.0], (3000, 1)).astype(np.float32) * np.array([[0, 0, 1]], np.float32)
    tie[:, 0] = rng.uniform(-1, 1, 3000)  # many pairs at the maximal distance 2
    cases.append(tie)
    for p in cases:
        for mode in (0, 1):
            t = [torch.from_numpy(np.ascontiguousarray(p[:, k])).cuda() for k in range(3)]
            got = ctx.axis_height(*t, coef, mode)
            want = orc.axis_height(*p.T, coef, mode)
            assert same(got[0], want[0]) and got[1:3] == want[1:3], (len(p), mode, got, want[:3])
            assert same(got[3], want[3])
