"""The cone service's seg.segment (cone_segmentation_srv.cpp:111-127):
SampleConsensusModelCone with normals, RANSAC with the opening-angle limits, the eps angle and the
normal-weighted distance, the least-squares refinement and the final selection; then the axis "height"
(test_axis_height, PITT_AXIS_CONE).

CPU: the oracle's computeModelCoefficients recovers an analytic cone from three exact samples; its
restatement recovers a noisy synthetic cone among clutter, and its refinement is scipy's float64
least-squares optimum of OptimizationFunctor's residual (sqrPointToLineDistance - (tan(angle) |apex -
proj|)^2) over the same inliers.  PCL and Eigen are not in the image: the float order of the Vector4f
arithmetic follows their published source ("parity unpinned" against a PCL build); PCL's refinement is
Eigen's float Levenberg-Marquardt, matched within tolerance.
GPU: pitt_cone_segment against the oracle: the RANSAC stage (hypothesis count, model, inliers)
bit-exact, the refined apex / axis / angle within tolerance, inliers equal except points at the threshold.
"""
import numpy as np
import pytest

import oracle_binding as orc


def _frame(axis):
    a = np.asarray(axis, float)
    a /= np.linalg.norm(a)
    u = np.cross(a, [1, 0, 0])
    u /= np.linalg.norm(u)
    return a, u, np.cross(a, u)


def cone_scene(n, n_out, seed, half_deg=25.0, h=0.15, axis=(0.1, 0.2, 1.0), apex=(0.3, -0.1, 1.1), noise=0.0005):
    """Points on the lateral surface of a cone (apex, axis, half opening angle) from 0.03 to h along the axis,
    with outward surface normals, plus uniform clutter with random normals."""
    rng = np.random.default_rng(seed)
    half = np.deg2rad(half_deg)
    a, u, v = _frame(axis)
    t = rng.uniform(0.03, h, n)
    ph = rng.uniform(0, 2 * np.pi, n)
    radial = np.cos(ph)[:, None] * u + np.sin(ph)[:, None] * v
    p = np.asarray(apex) + t[:, None] * a + (t * np.tan(half))[:, None] * radial + rng.normal(0, noise, (n, 3))
    nrm = np.cos(half) * radial - np.sin(half) * a + rng.normal(0, 0.01, (n, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    o = np.asarray(apex) + rng.uniform(-0.2, 0.2, (n_out, 3))
    on = rng.normal(size=(n_out, 3))
    on /= np.linalg.norm(on, axis=1)[:, None]
    P, N = np.concatenate([p, o]), np.concatenate([nrm, on])
    perm = rng.permutation(len(P))
    return P[perm].astype(np.float32), N[perm].astype(np.float32), a


def same_cone(c1, c2, pos=1e-5, ang=1e-8, opening=1e-6):
    """Two (apex, direction, opening angle) cones: same apex, same axis up to sign, same opening angle
    (the angle taken against the direction's sign: a flipped axis gives pi - angle)."""
    d1, d2 = c1[3:6] / np.linalg.norm(c1[3:6]), c2[3:6] / np.linalg.norm(c2[3:6])
    dot = float(np.dot(d1, d2))
    a2 = c2[6] if dot > 0 else np.pi - c2[6]
    return (np.linalg.norm(c1[:3] - c2[:3]) < pos and 1 - abs(dot) < ang
            and abs(np.tan(c1[6]) ** 2 - np.tan(a2) ** 2) < opening)


def test_oracle_cone_from3_analytic():
    apex, half = np.array([0.2, 0.1, 0.9]), np.deg2rad(30.0)
    a, u, v = _frame((0.0, 0.3, 1.0))
    ph = np.array([0.3, 2.2, 4.4])
    t = np.array([0.05, 0.08, 0.11])
    radial = np.cos(ph)[:, None] * u + np.sin(ph)[:, None] * v
    p = apex + t[:, None] * a + (t * np.tan(half))[:, None] * radial
    nrm = np.cos(half) * radial - np.sin(half) * a
    ok, c = orc.cone_from3(p, nrm)
    assert ok
    assert np.allclose(c[:3], apex, atol=1e-5)
    assert abs(abs(np.dot(c[3:6], a)) - 1) < 1e-6
    ang = c[6] if np.dot(c[3:6], a) > 0 else np.pi - c[6]
    assert abs(ang - half) < 1e-5
    # the opening-angle limits reject it (computeModelCoefficients returns false)
    assert not orc.cone_from3(p, nrm, min_angle=np.deg2rad(40), max_angle=np.deg2rad(170))[0]


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_cone_recovers_and_refines(seed):
    from scipy.optimize import least_squares
    P, N, a = cone_scene(3000, 1000, seed)
    with orc.lm_mode(orc.LM_OPTIMUM):
        res = orc.cone_segment(P, N)
    assert res["ok"] and len(res["inliers"]) > 2500
    c = res["coef"].astype(np.float64)
    assert same_cone(c, np.r_[0.3, -0.1, 1.1, a, np.deg2rad(25.0)], pos=3e-3, ang=1e-3, opening=5e-3)
    # the refinement: scipy's optimum of the functor's residual over the pre-refinement inliers
    b = res["best"].astype(np.float64)
    q = P.astype(np.float64)
    sel = orc.cone_segment(P, N, orc.cone_params(optimize=False))["inliers"]

    def f(v):
        d = v[3:6]
        w = np.cross(d, v[:3] - q[sel])
        k = (q[sel] - v[:3]) @ d / np.dot(d, d)
        hgt = np.abs(k) * np.linalg.norm(d)
        return (w * w).sum(1) / np.dot(d, d) - (np.tan(v[6]) * hgt) ** 2
    fit = least_squares(f, b, xtol=1e-15, ftol=1e-15, gtol=1e-15)
    assert same_cone(c, fit.x, pos=1e-5, ang=1e-8, opening=1e-6)


def test_oracle_cone_edges():
    P = np.zeros((2, 3), np.float32)
    assert not orc.cone_segment(P, P)["ok"]  # fewer than 3 points
    P, N, _ = cone_scene(1500, 200, 3)
    # Eigen >= 3.3: the eps check against the zero axis sees pi/2 > 0.4, so every model counts 0
    res = orc.cone_segment(P, N, orc.cone_params(eigen33=1, max_iterations=50))
    assert res["ok"] and len(res["inliers"]) == 0 and res["hypotheses"] == 51
    # an axis given (setAxis) within eps of the cone's keeps it
    res = orc.cone_segment(P, N, orc.cone_params(eigen33=1, axis=(0.1, 0.2, 1.0)))
    assert res["ok"] and len(res["inliers"]) > 1200


# the least-squares optimum against PCL's float LM stopping point: apex (m), axis
# 1 - |cos|, tan^2 of the opening angle (measured envelope in tests/test_pcl_lm.py, with margin)
CONE_PCL_TOL = dict(pos=1e-4, ang=1e-7, opening=1e-4)


def _optimum(fn, *a):
    """The oracle in its least-squares-optimum refinement mode (a double LM to the optimum)."""
    with orc.lm_mode(orc.LM_OPTIMUM):
        return fn(*a)


def _gpu(ctx, P, N, **kw):
    import torch
    t = [torch.from_numpy(np.ascontiguousarray(a[:, k])).cuda() for a in (P, N) for k in range(3)]
    inl, coef, hyp = ctx.cone_segment(*t, **kw)
    return inl.cpu().numpy(), coef, hyp


def _oracle_kw(kw):
    return orc.cone_params(**kw)


@pytest.mark.gpu
@pytest.mark.parametrize("n,n_out,seed,half", [(3000, 1000, 1, 25.0), (800, 3000, 2, 40.0), (20000, 4000, 3, 15.0),
                                               (300, 60, 4, 60.0)])
def test_hip_cone_matches_oracle(ctx, n, n_out, seed, half):
    P, N, _ = cone_scene(n, n_out, seed, half_deg=half)
    raw = orc.cone_segment(P, N, orc.cone_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False)
    assert hyp == raw["hypotheses"]
    assert np.array_equal(coef.view(np.int32), raw["coef"].view(np.int32))
    assert np.array_equal(inl, raw["inliers"])
    # refined by PCL's float Eigen LM on the device (elm.hpp): bit-exact with the oracle's restatement
    pcl = orc.cone_segment(P, N)
    inl, coef, hyp = _gpu(ctx, P, N)
    assert hyp == pcl["hypotheses"]
    assert np.array_equal(coef.view(np.int32), pcl["coef"].view(np.int32)), (coef, pcl["coef"])
    assert np.array_equal(inl, pcl["inliers"])
    # the float LM's stop against the least-squares optimum: within its envelope (tests/test_pcl_lm.py)
    want = _optimum(orc.cone_segment, P, N)
    assert same_cone(coef.astype(np.float64), want["coef"].astype(np.float64), **CONE_PCL_TOL)


@pytest.mark.gpu
def test_hip_cone_edges(ctx):
    P = np.zeros((2, 3), np.float32)
    inl, coef, hyp = _gpu(ctx, P, P)
    assert coef is None and len(inl) == 0
    P, N, _ = cone_scene(1500, 200, 3)
    for kw in (dict(eigen33=1, max_iterations=50), dict(eigen33=1, axis=(0.1, 0.2, 1.0), optimize=False),
               dict(min_angle_deg=60.0, max_angle_deg=120.0, optimize=False, max_iterations=40)):
        want = orc.cone_segment(P, N, _oracle_kw(kw))
        inl, coef, hyp = _gpu(ctx, P, N, **kw)
        assert (coef is not None) == want["ok"] and hyp == want["hypotheses"]
        assert np.array_equal(inl, want["inliers"])
        if coef is not None and kw.get("optimize", True) is False:
            assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32))
    # identical points with identical normals: the apex is 0 / 0 (NaN), every model passes the limits and
    # counts no point
    P = np.full((50, 3), 0.3, np.float32)
    N = np.tile(np.array([[0, 0, 1]], np.float32), (50, 1))
    want = orc.cone_segment(P, N, orc.cone_params(optimize=False, max_iterations=20))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False, max_iterations=20)
    assert (coef is not None) == want["ok"] and hyp == want["hypotheses"] and len(inl) == len(want["inliers"]) == 0
    # fewer than 7 inliers: the model is kept, only the direction normalised
    P, N, _ = cone_scene(5, 0, 5)
    want = orc.cone_segment(P, N)
    inl, coef, hyp = _gpu(ctx, P, N)
    assert (coef is not None) == want["ok"] and hyp == want["hypotheses"]
    if coef is not None:
        assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32))
        assert np.array_equal(inl, want["inliers"])


@pytest.mark.gpu
@pytest.mark.parametrize("what", ["points", "normals"])
def test_hip_cone_nan_inputs(ctx, what):
    """NaN coordinates or normals (a camera cloud's invalid pixels): NaN distances never count, a sample that
    draws one gives a NaN model that counts no point; the RANSAC stage stays bit-exact."""
    P, N, _ = cone_scene(3000, 800, 9)
    rng = np.random.default_rng(9)
    bad = rng.random(len(P)) < 0.05
    (P if what == "points" else N)[bad] = np.nan
    raw = orc.cone_segment(P, N, orc.cone_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False)
    assert hyp == raw["hypotheses"] and (coef is not None) == raw["ok"]
    assert np.array_equal(coef.view(np.int32), raw["coef"].view(np.int32))
    assert np.array_equal(inl, raw["inliers"]) and not bad[inl].any()
    want = orc.cone_segment(P, N)
    inl, coef, hyp = _gpu(ctx, P, N)
    assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32)), (coef, want["coef"])
    assert np.array_equal(inl, want["inliers"])
