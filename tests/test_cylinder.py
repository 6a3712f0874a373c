"""The cylinder service's seg.segment (cylinder_segmentation_srv.cpp:110-126):
SampleConsensusModelCylinder with normals, RANSAC with the radius limits and the normal-weighted
distance, the least-squares refinement and the final selection; then the axis "height" (test_axis_height).

CPU: the oracle's restatement recovers a noisy synthetic cylinder among clutter, and its refinement is
scipy's float64 least-squares optimum of OptimizationFunctor's residual (sqrPointToLineDistance - r^2)
over the same inliers (compared as a line: axis direction, distance between the axes, radius).  PCL and
Eigen are not in the image: the float order of the Vector4f arithmetic follows their published source
("parity unpinned" against a PCL build); PCL's refinement is Eigen's float Levenberg-Marquardt, matched
within tolerance.
GPU: pitt_cylinder_segment against the oracle: the RANSAC stage (hypothesis count, model, inliers)
bit-exact, the refined axis / radius within tolerance, inliers equal except points at the threshold.
"""
import numpy as np
import pytest

import oracle_binding as orc


def cylinder_scene(n, n_out, seed, r=0.04, h=0.15, axis=(0.1, 0.2, 1.0), base=(0.3, -0.1, 0.9), noise=0.001):
    rng = np.random.default_rng(seed)
    a = np.asarray(axis, float)
    a /= np.linalg.norm(a)
    u = np.cross(a, [1, 0, 0])
    u /= np.linalg.norm(u)
    v = np.cross(a, u)
    t = rng.uniform(0, h, n)
    ph = rng.uniform(0, 2 * np.pi, n)
    radial = np.cos(ph)[:, None] * u + np.sin(ph)[:, None] * v
    p = np.asarray(base) + t[:, None] * a + r * radial + rng.normal(0, noise, (n, 3))
    nrm = radial + rng.normal(0, 0.02, (n, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    o = np.asarray(base) + rng.uniform(-0.2, 0.2, (n_out, 3))
    on = rng.normal(size=(n_out, 3))
    on /= np.linalg.norm(on, axis=1)[:, None]
    P, N = np.concatenate([p, o]), np.concatenate([nrm, on])
    perm = rng.permutation(len(P))
    return P[perm].astype(np.float32), N[perm].astype(np.float32), a


def same_line(c1, c2, ang=1e-4, dist=1e-5, rad=1e-5):
    """Two (point, direction, radius) cylinders describe the same axis and radius."""
    d1, d2 = c1[3:6] / np.linalg.norm(c1[3:6]), c2[3:6] / np.linalg.norm(c2[3:6])
    cosang = abs(float(np.dot(d1, d2)))
    off = np.cross(d1, c2[:3].astype(np.float64) - c1[:3].astype(np.float64))
    return 1 - cosang < ang and np.linalg.norm(off) < dist and abs(abs(c1[6]) - abs(c2[6])) < rad


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_cylinder_recovers_and_refines(seed):
    from scipy.optimize import least_squares
    P, N, a = cylinder_scene(3000, 1000, seed)
    res = _optimum(orc.cylinder_segment, P, N)
    assert res["ok"] and len(res["inliers"]) > 2500
    c = res["coef"]
    assert abs(abs(np.dot(c[3:6], a)) - 1) < 1e-3 and abs(c[6] - 0.04) < 1e-3
    # the refinement: scipy's optimum of |u x (c - p)|^2 / |u|^2 - r^2 over the pre-refinement inliers
    b = res["best"].astype(np.float64)
    q = P.astype(np.float64)
    sel = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False))["inliers"]

    def f(v):
        w = np.cross(v[3:6], v[:3] - q[sel])
        return (w * w).sum(1) / np.dot(v[3:6], v[3:6]) - v[6] ** 2
    fit = least_squares(f, b, xtol=1e-15, ftol=1e-15, gtol=1e-15)
    assert same_line(c.astype(np.float64), fit.x, ang=1e-8, dist=1e-6, rad=1e-6)


def test_oracle_cylinder_edges():
    P = np.zeros((1, 3), np.float32)
    assert not orc.cylinder_segment(P, P)["ok"]  # fewer than 2 points
    P, N, _ = cylinder_scene(800, 0, 3, r=0.8)  # outside the 0.5 m radius limit: no model can form
    res = orc.cylinder_segment(P, N)
    assert not res["ok"] or len(res["inliers"]) == 0


# the least-squares optimum against PCL's float LM stopping point: axis 1 - |cos|,
# distance between the axis lines (m), radius (m) (measured envelope in tests/test_pcl_lm.py)
CYL_PCL_TOL = dict(ang=1e-7, dist=5e-5, rad=5e-5)


def _optimum(fn, *a):
    """The oracle in its least-squares-optimum refinement mode (a double LM to the optimum)."""
    with orc.lm_mode(orc.LM_OPTIMUM):
        return fn(*a)


def _gpu(ctx, P, N, **kw):
    import torch
    t = [torch.from_numpy(np.ascontiguousarray(a[:, k])).cuda() for a in (P, N) for k in range(3)]
    inl, coef, hyp = ctx.cylinder_segment(*t, **kw)
    return inl.cpu().numpy(), coef, hyp


@pytest.mark.gpu
@pytest.mark.parametrize("n,n_out,seed", [(3000, 1000, 1), (800, 3000, 2), (20000, 4000, 3), (300, 60, 4)])
def test_hip_cylinder_matches_oracle(ctx, n, n_out, seed):
    P, N, _ = cylinder_scene(n, n_out, seed)
    raw = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False)
    assert hyp == raw["hypotheses"]
    assert np.array_equal(coef.view(np.int32), raw["coef"].view(np.int32))
    assert np.array_equal(inl, raw["inliers"])
    # refined by PCL's float Eigen LM on the device (elm.hpp): bit-exact with the oracle's restatement
    pcl = orc.cylinder_segment(P, N)
    inl, coef, hyp = _gpu(ctx, P, N)
    assert hyp == pcl["hypotheses"]
    assert np.array_equal(coef.view(np.int32), pcl["coef"].view(np.int32)), (coef, pcl["coef"])
    assert np.array_equal(inl, pcl["inliers"])
    # the float LM's stop against the least-squares optimum: the same line and radius within its envelope
    want = _optimum(orc.cylinder_segment, P, N)
    assert same_line(coef.astype(np.float64), want["coef"].astype(np.float64), **CYL_PCL_TOL)


@pytest.mark.gpu
def test_hip_cylinder_edges(ctx):
    P = np.zeros((1, 3), np.float32)
    inl, coef, hyp = _gpu(ctx, P, P)
    assert coef is None and len(inl) == 0
    P, N, _ = cylinder_scene(800, 0, 3, r=0.8)
    want = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False)
    assert (coef is not None) == want["ok"] and hyp == want["hypotheses"]
    # identical points: every sample is skipped
    P = np.full((50, 3), 0.3, np.float32)
    N = np.tile(np.array([[0, 0, 1]], np.float32), (50, 1))
    want = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False, max_iterations=20))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False, max_iterations=20)
    assert (coef is not None) == want["ok"] and hyp == want["hypotheses"]


@pytest.mark.gpu
def test_hip_cylinder_few_inliers(ctx):
    """Fewer than 7 inliers: Eigen's LM refuses m < n, the model stays and only the direction is normalised."""
    P, N, _ = cylinder_scene(5, 0, 5)
    want = orc.cylinder_segment(P, N)
    inl, coef, hyp = _gpu(ctx, P, N)
    assert (coef is not None) == want["ok"] and hyp == want["hypotheses"]
    if coef is not None:
        assert len(want["inliers"]) < 7
        assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32))
        assert np.array_equal(inl, want["inliers"])


@pytest.mark.gpu
@pytest.mark.parametrize("what", ["points", "normals"])
def test_hip_cylinder_nan_inputs(ctx, what):
    """NaN coordinates or normals: NaN distances never count; the RANSAC stage stays bit-exact."""
    P, N, _ = cylinder_scene(3000, 800, 9)
    rng = np.random.default_rng(9)
    bad = rng.random(len(P)) < 0.05
    (P if what == "points" else N)[bad] = np.nan
    raw = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False)
    assert hyp == raw["hypotheses"] and (coef is not None) == raw["ok"]
    assert np.array_equal(coef.view(np.int32), raw["coef"].view(np.int32))
    assert np.array_equal(inl, raw["inliers"]) and not bad[inl].any()
    want = orc.cylinder_segment(P, N)
    inl, coef, hyp = _gpu(ctx, P, N)
    assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32)), (coef, want["coef"])
    assert np.array_equal(inl, want["inliers"])


def _zero_normals(seed):
    P, N, _ = cylinder_scene(3000, 600, seed)
    rng = np.random.default_rng(seed)
    zero = rng.random(len(P)) < 0.2
    N[zero] = 0.0
    return P, N, zero


def test_oracle_cylinder_zero_normals_eigen_conventions():
    """A zero normal (the ROS adapter's fill for a cloud without normal fields): Eigen 3.2's
    normalized() gives NaN, so the point never counts; Eigen >= 3.3 keeps it zero (angle pi/2), and
    with the 0.001 normal weight such points can count (the cylinder follows the cone)."""
    P, N, zero = _zero_normals(21)
    e32 = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False, eigen33=0))
    e33 = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False, eigen33=1))
    assert e32["ok"] and e33["ok"]
    assert not zero[e32["inliers"]].any()
    assert zero[e33["inliers"]].any()


@pytest.mark.gpu
@pytest.mark.parametrize("eigen33", [0, 1])
def test_hip_cylinder_zero_normals(ctx, eigen33):
    P, N, _ = _zero_normals(21)
    raw = orc.cylinder_segment(P, N, orc.cylinder_params(optimize=False, eigen33=eigen33))
    inl, coef, hyp = _gpu(ctx, P, N, optimize=False, eigen33=eigen33)
    assert hyp == raw["hypotheses"] and (coef is not None) == raw["ok"]
    assert np.array_equal(coef.view(np.int32), raw["coef"].view(np.int32))
    assert np.array_equal(inl, raw["inliers"])
