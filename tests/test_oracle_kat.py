"""Pin the oracle (CPU restatement of the reference's PCL path) before trusting it.

The reference ships no tests or fixtures, so the pins are: the C++ standard's
mt19937 known answer, the reference's rnd() draws for seed 12345, an independent Python
restatement of drawIndexSample, and analytic known-answer cases for every stage."""
import numpy as np
import pytest

import oracle_binding as orc


def test_mt19937_standard_kat():
    # [rand.predef]: the 10000th consecutive invocation of a default-constructed mt19937
    assert orc.mt19937(5489, 10000)[-1] == 4123659995


def test_reference_rnd_draws_seed_12345():
    # boost::uniform_int<>(0, INT_MAX) over mt19937(12345) == mt() >> 1
    assert list(orc.mt19937(12345, 3) >> 1) == [1996335345, 1911592690, 679411342]


@pytest.mark.parametrize("n", [3, 4, 7, 1000, 307200])
def test_sampler_matches_python_restatement(n):
    attempts = 400
    draws = (orc.mt19937(12345, 3 * attempts) >> 1).astype(np.int64)
    shuffled = {}
    exp = []
    k = 0
    for _ in range(attempts):  # SampleConsensusModel::drawIndexSample, sparse shuffled_indices_
        for i in range(3):
            j = i + int(draws[k]) % (n - i)
            k += 1
            vi, vj = shuffled.get(i, i), shuffled.get(j, j)
            shuffled[i], shuffled[j] = vj, vi
        exp.append([shuffled.get(0, 0), shuffled.get(1, 1), shuffled.get(2, 2)])
    assert np.array_equal(orc.sampler_table(n, attempts), np.array(exp, np.int32))


def test_plane_from_three_points_exact():
    ok, c = orc.plane_coefficients([0, 0, 1], [1, 0, 1], [0, 1, 1])
    assert ok and np.array_equal(c, np.array([0, 0, 1, -1], np.float32))


def test_collinear_sample_rejected():
    ok, _ = orc.plane_coefficients([0, 0, 0], [1, 1, 1], [2, 2, 2])
    assert not ok


def test_count_within_threshold_is_strict_and_double():
    # |d| < 0.007 (double): a point at exactly float(0.007) above the plane is outside because
    # float(0.007) > 0.007; one ulp below is inside.
    t = np.float32(0.007)
    z = np.array([1 + 0, 1 + 0.0069, np.float32(1.0) + t, np.nextafter(t, np.float32(0)) + np.float32(1.0)],
                 np.float32)
    d = z - np.float32(1.0)
    x = np.zeros(4, np.float32)
    n = orc.count_within(x, x, d, [0, 0, 1, 0], 0.007)
    assert n == int(np.sum(np.abs(d).astype(np.float64) < 0.007))


def test_eigen33_diagonal_known_answer():
    ev, v = orc.eigen33(np.diag([3.0, 2.0, 0.5]).astype(np.float32))
    assert abs(ev - 0.5) < 1e-6
    assert np.allclose(np.abs(v), [0, 0, 1], atol=1e-6)


def test_eigen33_libm_and_cr_agree_on_plane_like_covariances():
    rng = np.random.default_rng(3)
    diff = 0
    for _ in range(300):
        a = rng.normal(size=(3, 3)).astype(np.float32)
        cov = (a @ a.T * np.float32(0.01)).astype(np.float32)
        cov[2, :] *= np.float32(1e-3)
        cov[:, 2] *= np.float32(1e-3)
        _, v1 = orc.eigen33(cov, orc.TRIG_CR)
        _, v2 = orc.eigen33(cov, orc.TRIG_LIBM)
        diff += int(not np.array_equal(v1, v2))
        assert np.allclose(v1, v2, atol=1e-5)
    # the documented envelope of A7: libm vs correctly-rounded trig rarely changes the vector bits
    assert diff < 300


def test_noise_free_plane_known_answer():
    g = np.stack(np.meshgrid(np.arange(50) * 0.01, np.arange(40) * 0.01), -1).reshape(-1, 2).astype(np.float32)
    rng = np.random.default_rng(7)
    out = rng.uniform(-1, 1, (500, 3)).astype(np.float32)
    out[:, 2] += 2.0
    xyz = np.concatenate([np.c_[g, np.full(len(g), 0.5, np.float32)], out])
    r = orc.plane_segment(*xyz.T)
    assert len(r.inliers) == 2000 and np.array_equal(r.inliers, np.arange(2000))
    c = r.coefficients / np.sign(r.coefficients[2])
    assert np.allclose(c, [0, 0, 1, -0.5], atol=1e-6)


def test_too_few_points_and_zero_iterations_give_no_model():
    x = np.array([0, 1], np.float32)
    assert orc.plane_segment(x, x, x).coefficients.size == 0
    g = np.random.default_rng(1).normal(size=(100, 3)).astype(np.float32)
    # setMaxIterations(0): max_skip = 0, the RANSAC loop never runs
    assert orc.plane_segment(*g.T, max_iterations=0).coefficients.size == 0


def test_collinear_cloud_gives_no_model():
    t = np.arange(2000, dtype=np.float32) * np.float32(0.25)
    r = orc.plane_segment(t, 2 * t, 3 * t)  # every sample collinear: 1000 rejections, no model
    assert r.coefficients.size == 0 and r.hypotheses == 0 and r.rejected_samples == 1000


def _blob(center, n_side=6, step=0.01):
    g = np.stack(np.meshgrid(*(np.arange(n_side) * step,) * 3), -1).reshape(-1, 3)
    return (g + np.asarray(center)).astype(np.float32)


def test_clusters_known_answer_order_and_centroid():
    a = _blob([0, 0, 0], 6)      # 216 points
    b = _blob([0.3, 0, 0], 5)    # 125
    c = _blob([0, 0.3, 0], 7)    # 343
    xyz = np.concatenate([b, a, c])
    cl = orc.euclidean_clusters(*xyz.T)
    assert [len(k["inliers"]) for k in cl] == [343, 216, 125]  # size-descending
    assert np.array_equal(cl[0]["inliers"], np.arange(341, 684))
    s = xyz[cl[0]["inliers"]].astype(np.float32)
    exp = np.array([np.float32(np.add.reduce(s[:, i], dtype=np.float32)) / np.float32(344) for i in range(3)])
    assert np.allclose(cl[0]["centroid"], exp, rtol=1e-5)  # Q7: divided by n + 1


def test_clusters_size_filter_and_min_input():
    xyz = np.concatenate([_blob([0, 0, 0], 6), _blob([1, 1, 1], 2)])  # 216 + 8
    cl = orc.euclidean_clusters(*xyz.T)  # min = round(224 * 0.01) = 2: both kept
    assert [len(k["inliers"]) for k in cl] == [216, 8]
    cl = orc.euclidean_clusters(*xyz.T, min_rate=0.05)  # min 11: the 8-point blob is dropped
    assert [len(k["inliers"]) for k in cl] == [216]
    assert orc.euclidean_clusters(*xyz[:20].T) == []  # < 30 points: skipped (:54)


def test_supports_table_with_object_known_answer():
    # a horizontal table (z = 0.75, 1 cm grid) and a box standing on it: one support, the box on it
    g = np.stack(np.meshgrid(np.arange(80) * 0.01, np.arange(60) * 0.01), -1).reshape(-1, 2)
    table = np.c_[g, np.full(len(g), 0.75)]
    bg = np.stack(np.meshgrid(np.arange(6) * 0.01 + 0.3, np.arange(6) * 0.01 + 0.3, np.arange(6) * 0.01 + 0.8),
                  -1).reshape(-1, 3)
    xyz = np.concatenate([table, bg]).astype(np.float32)
    sup = orc.find_supports(*xyz.T)
    assert len(sup) == 1
    s = sup[0]
    assert len(s["support_cloud"]) == len(table)
    assert len(s["on_support_cloud"]) == len(bg)
    assert np.all(s["idx_map"][:len(table)] == -2)
    assert np.array_equal(s["idx_map"][len(table):], np.arange(len(bg)))


# --- preprocessing (deep_filter_srv.cpp:27-44, obj_segmentation.cpp:248) ---------------------------
def test_service_float_param_sentinels():
    """srv_manager.h:163-167: >= 0 is used as given; -1 and NaN select the default."""
    assert orc.service_float_param(-1.0, 3.0) == 3.0
    assert orc.service_float_param(float("nan"), 3.0) == 3.0
    assert orc.service_float_param(0.0, 3.0) == 0.0
    assert orc.service_float_param(2.5, 3.0) == 2.5


def test_deep_filter_known_answer():
    x = np.arange(7, dtype=np.float32)
    y = x + 10
    z = np.array([1.0, np.nan, 3.5, 3.0, -1.0, np.inf, 2.9999998], np.float32)
    closer, further = orc.deep_filter(x, y, z, 3.0)
    assert closer[:, 0].tolist() == [0, 3, 4, 6]      # z <= 3 (ties closer), input order
    assert further[:, 0].tolist() == [2, 5]           # z > 3, +inf included; NaN z dropped
    assert np.array_equal(closer[:, 2], z[[0, 3, 4, 6]])


def test_transform_known_answers():
    rng = np.random.default_rng(3)
    x, y, z = rng.normal(size=(3, 1000)).astype(np.float32)
    ident = np.eye(4, dtype=np.float32)
    assert np.array_equal(orc.transform_cloud(x, y, z, ident), np.stack([x, y, z], 1))
    # the published float order, restated in numpy float32 (IEEE single ops, no FMA)
    m = rng.normal(size=(4, 4)).astype(np.float32)
    ref = np.stack([((m[k, 0] * x + m[k, 1] * y) + m[k, 2] * z) + m[k, 3] for k in range(3)], 1)
    assert np.array_equal(orc.transform_cloud(x, y, z, m), ref)
    # a 90-degree turn about z plus a translation is exact
    rot = np.array([[0, -1, 0, 1], [1, 0, 0, 2], [0, 0, 1, 3], [0, 0, 0, 1]], np.float32)
    assert np.array_equal(orc.transform_cloud(x, y, z, rot), np.stack([-y + 1, x + 2, z + 3], 1))


def test_transform_non_dense_copies_non_finite():
    x = np.array([1.0, np.nan, 2.0], np.float32)
    y = np.array([1.0, 1.0, np.inf], np.float32)
    z = np.array([1.0, 1.0, 1.0], np.float32)
    m = np.eye(4, dtype=np.float32)
    m[:3, 3] = 5
    out = orc.transform_cloud(x, y, z, m, dense=False)
    assert out[0].tolist() == [6, 6, 6]
    assert np.isnan(out[1, 0]) and out[1, 1:].tolist() == [1, 1]   # copied, not transformed
    assert out[2, 0] == 2 and np.isinf(out[2, 1]) and out[2, 2] == 1
    dense = orc.transform_cloud(x, y, z, m, dense=True)
    assert np.isnan(dense[1]).all()                                 # dense: NaN propagates
