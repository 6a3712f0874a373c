"""The sphere service's seg.segment (sphere_segmentation_srv.cpp:57-73):
SampleConsensusModelSphere RANSAC with the radius limits, then the least-squares refinement and the
final selection.

CPU: the oracle's restatement against analytic spheres (computeModelCoefficients recovers a sphere
from 4 of its points; RANSAC finds a noisy sphere among outliers) and its refinement against scipy's
float64 least squares on the same inliers; the edge cases (fewer than 4 points, coplanar samples,
radius limits).  PCL and Eigen are not in the image: the float order of the determinants (Eigen
3.2's 4 x 4 expansion) follows the library's published source ("parity unpinned" against a PCL
build), and PCL's own refinement is Eigen's float Levenberg-Marquardt, matched within tolerance.
GPU: pitt_sphere_segment against the oracle -- the RANSAC stage (hypothesis count, best model) bit-
exact, the refined coefficients within 2e-6 relative, the final inliers equal except points within
1e-5 m of the threshold shell.
"""
import numpy as np
import pytest

import oracle_binding as orc


def sphere_scene(n_sphere, n_out, seed, centre=(0.3, -0.2, 1.1), radius=0.05, noise=0.001, box=0.3):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n_sphere, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    d[:, 2] = -np.abs(d[:, 2])  # the camera sees one hemisphere
    pts = np.asarray(centre) + radius * d + rng.normal(0, noise, (n_sphere, 3))
    out = np.asarray(centre) + rng.uniform(-box, box, (n_out, 3))
    p = np.concatenate([pts, out])
    p = p[rng.permutation(len(p))]
    return p.astype(np.float32)


def test_oracle_sphere_from4_recovers_the_sphere():
    rng = np.random.default_rng(3)
    for _ in range(20):
        c = rng.uniform(-0.5, 0.5, 3)
        r = rng.uniform(0.05, 0.4)
        d = rng.normal(size=(4, 3))
        d /= np.linalg.norm(d, axis=1)[:, None]
        ok, coef = orc.sphere_from4((c + r * d).astype(np.float32))
        assert ok
        # float Cramer determinants cancel heavily (PCL's own accuracy): the geometry, not the digits
        assert np.allclose(coef[:3], c, atol=3e-2 * r) and abs(coef[3] - r) < 3e-2 * r
    # four coplanar points: m11 == 0 (the points don't define a sphere)
    ok, _ = orc.sphere_from4(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]], np.float32))
    assert not ok


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_sphere_ransac_and_refinement(seed):
    from scipy.optimize import least_squares
    p = sphere_scene(3000, 1500, seed)
    with orc.lm_mode(orc.LM_OPTIMUM):
        res = orc.sphere_segment(*p.T)
    assert res["ok"] and len(res["inliers"]) > 2500
    c = res["coef"]
    assert np.allclose(c[:3], (0.3, -0.2, 1.1), atol=1e-3) and abs(c[3] - 0.05) < 1e-3
    # the optimum mode's refinement is the float64 least-squares optimum over the pre-refinement inliers
    b = res["best"]
    q = p.astype(np.float64)
    d = q - b[:3].astype(np.float64)
    pre = np.nonzero(np.abs(np.sqrt((d * d).sum(1)).astype(np.float32) - b[3]) < 0.007)[0]
    fit = least_squares(lambda v: np.sqrt(((q[pre] - v[:3]) ** 2).sum(1)) - v[3], b.astype(np.float64),
                        xtol=1e-15, ftol=1e-15, gtol=1e-15)
    assert np.allclose(c, fit.x, rtol=0, atol=1e-6)
    # the counts are the hypotheses' inlier counts in RANSAC order; the best is the first maximum
    assert res["hypotheses"] >= 1 and len(res["counts"]) == res["hypotheses"]


def test_oracle_sphere_edges():
    p = np.zeros((3, 3), np.float32)
    assert not orc.sphere_segment(*p.T)["ok"]  # fewer than 4 points
    # radius limits: a 1 m sphere is outside [0.005, 0.5] -> every model counts 0
    big = sphere_scene(2000, 0, 4, radius=1.0)
    res = orc.sphere_segment(*big.T)
    assert res["ok"] and len(res["inliers"]) == 0 or not res["ok"]
    res = orc.sphere_segment(*big.T, orc.sphere_params(radius_max=2.0))
    assert res["ok"] and len(res["inliers"]) > 1500


# |least-squares optimum - PCL's float LM| on sphere coefficients (metres): the float LM stops at
# Eigen's sqrt(FLT_EPSILON) tolerances; measured <= 1.7e-6 (tests/test_pcl_lm.py)
SPHERE_PCL_ATOL = 5e-6


def _gpu(ctx, p, **kw):
    import torch
    t = [torch.from_numpy(np.ascontiguousarray(p[:, k])).cuda() for k in range(3)]
    inl, coef, hyp = ctx.sphere_segment(*t, **kw)
    return inl.cpu().numpy(), coef, hyp


def _shell_distance(p, c):
    d = p.astype(np.float64) - c[:3].astype(np.float64)
    return np.abs(np.abs(np.sqrt((d * d).sum(1)) - c[3]) - 0.007)


@pytest.mark.gpu
@pytest.mark.parametrize("n_s,n_o,seed", [(3000, 1500, 1), (800, 4000, 2), (20000, 5000, 3), (200, 50, 4)])
def test_hip_sphere_matches_oracle(ctx, n_s, n_o, seed):
    p = sphere_scene(n_s, n_o, seed)
    pcl = orc.sphere_segment(*p.T)  # PCL's float Eigen LM (the reference's refinement, oracle/eigen_lm.hpp)
    # RANSAC stage (optimize off): bit-exact
    raw = orc.sphere_segment(*p.T, orc.sphere_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, p, optimize=False)
    assert hyp == raw["hypotheses"]
    assert np.array_equal(coef.view(np.int32), raw["coef"].view(np.int32))
    assert np.array_equal(inl, raw["inliers"])
    # refined by the device's port of the same float LM (elm.hpp): bit-exact, and so the final inliers
    inl, coef, hyp = _gpu(ctx, p)
    assert hyp == pcl["hypotheses"]
    assert np.array_equal(coef.view(np.int32), pcl["coef"].view(np.int32)), (coef, pcl["coef"])
    assert np.array_equal(inl, pcl["inliers"])
    # and the float LM's stop is close to the least-squares optimum (the envelope of tests/test_pcl_lm.py)
    with orc.lm_mode(orc.LM_OPTIMUM):
        want = orc.sphere_segment(*p.T)
    assert np.allclose(coef, want["coef"], rtol=0, atol=SPHERE_PCL_ATOL)


@pytest.mark.gpu
def test_hip_sphere_edges(ctx):
    import torch
    p = np.zeros((3, 3), np.float32)
    inl, coef, hyp = _gpu(ctx, p)
    assert coef is None and len(inl) == 0
    big = sphere_scene(2000, 0, 4, radius=1.0)
    for kw, okw in (({}, {}), ({"radius_max": 2.0}, {"radius_max": 2.0})):
        want = orc.sphere_segment(*big.T, orc.sphere_params(optimize=False, **okw))
        inl, coef, hyp = _gpu(ctx, big, optimize=False, **kw)
        assert (coef is not None) == want["ok"] and hyp == want["hypotheses"]
        if want["ok"]:
            assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32))
            assert np.array_equal(inl, want["inliers"])
    # a flat patch: coplanar samples (m11 == 0 or huge spheres outside the limits)
    flat = np.zeros((500, 3), np.float32)
    flat[:, :2] = np.random.default_rng(5).uniform(-0.1, 0.1, (500, 2))
    want = orc.sphere_segment(*flat.T, orc.sphere_params(optimize=False))
    inl, coef, hyp = _gpu(ctx, flat, optimize=False)
    assert hyp == want["hypotheses"] and (coef is not None) == want["ok"]
    if want["ok"]:
        assert np.array_equal(inl, want["inliers"])
    del torch
