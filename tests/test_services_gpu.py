"""The service mirror (pitt_srv.h) keeps the reference handlers' semantics on top of the HIP path:
parameter resolution, sentinels, the normals size check and the post-processing quirks."""
import numpy as np
import pytest

import oracle_binding as orc
import pitt_object_table_segmentation_amd as pitt

pytestmark = pytest.mark.gpu

PLANE_TH = "/pitt/srv/plane_segmentation/distance_th"
PLANE_IT = "/pitt/srv/plane_segmentation/max_iter_limit"
CL_TOL = "/pitt/srv/cluster_segmentation/tolerance"
CL_MIN = "/pitt/srv/cluster_segmentation/min_rate"


@pytest.fixture(scope="module")
def srv(ctx):
    s = pitt.Services(ctx)
    yield s
    s.close()


def _cloud(seed=1000, w=160, h=120, scene=0):
    return np.stack(pitt.synth_frame(scene, seed, w, h), 1)


def test_plane_handler_drops_index_zero_and_keeps_centroid_zero(srv):
    xyz = _cloud()
    ok, inl, coef, centroid = srv.ransac_plane(xyz)
    o = orc.plane_segment(*xyz.T)
    assert ok
    assert np.array_equal(inl, o.inliers[o.inliers != 0])        # Q1
    assert np.array_equal(coef, o.coefficients)
    assert np.array_equal(centroid, np.zeros(3, np.float32))      # Q3
    # a cloud whose plane contains point 0: the response loses it
    plane = np.c_[np.random.default_rng(0).uniform(size=(500, 2)), np.zeros(500)].astype(np.float32)
    ok, inl, coef, _ = srv.ransac_plane(plane)
    assert ok and len(inl) == 499 and 0 not in inl


def test_plane_handler_params_and_normals_check(srv):
    xyz = _cloud(1001)
    srv.set_param(PLANE_TH, 0.002)
    srv.set_param(PLANE_IT, 50)
    try:
        ok, inl, coef, _ = srv.ransac_plane(xyz)
        o = orc.plane_segment(*xyz.T, threshold=0.002, max_iterations=50)
        assert np.array_equal(inl, o.inliers[o.inliers != 0]) and np.array_equal(coef, o.coefficients)
    finally:
        srv.erase_param(PLANE_TH)
        srv.erase_param(PLANE_IT)
    # SACSegmentationFromNormals: normals of the wrong size => PCL clears the outputs (A1)
    ok, inl, coef, _ = srv.ransac_plane(xyz, n_normals=len(xyz) - 1)
    assert ok and len(inl) == 0 and len(coef) == 0


def test_ros_int_param_from_double_is_rounded(srv):
    xyz = _cloud(1002)
    srv.set_param(PLANE_IT, 10.6)   # roscpp getParam(int&) on a double: rounds (-> 11)
    try:
        _, _, coef, _ = srv.ransac_plane(xyz)
        assert np.array_equal(coef, orc.plane_segment(*xyz.T, max_iterations=11).coefficients)
    finally:
        srv.erase_param(PLANE_IT)


def test_support_handler_sentinels_and_used_fields(srv):
    xyz = np.stack(pitt.synth_fused(31, 2, 160, 120), 1)
    ok, sups, used = srv.find_supports(xyz)
    ref = orc.find_supports(*xyz.T)
    assert ok and len(sups) == len(ref)
    for s, r in zip(sups, ref):
        assert np.array_equal(s["inliers"], r["idx_map"])
        assert np.array_equal(s["coefficients"], r["coefficients"])
        assert np.array_equal(s["on_support_cloud"], r["on_support_cloud"])
    assert np.allclose(used, [0.03, 0.03, 0.09, -0.09, 10, 0.02, 0.9, 0, 0, -1, 0.02, 0.02, 0.005])
    # explicit request values (>= 0, 3-vectors) override; malformed arrays fall back
    ok, sups, used = srv.find_supports(xyz, ransac_max_iteration_threshold=25, horizontal_axis=[0, 0, 1],
                                       support_edge_remove_offset=[0.1, 0.1])
    assert used[4] == 25 and list(used[7:10]) == [0, 0, 1] and np.allclose(used[10:], [0.02, 0.02, 0.005])
    ref = orc.find_supports(*xyz.T, ransac_max_iterations=25, horizontal_axis=(0, 0, 1))
    assert len(sups) == len(ref)
    # input normals of the wrong size: the first RANSAC fails, no supports
    ok, sups, _ = srv.find_supports(xyz, n_normals=3)
    assert ok and sups == []


def test_cluster_handler_centroid_and_min_input_quirk(srv):
    rng = np.random.default_rng(4)
    g = np.stack(np.meshgrid(*(np.arange(5) * 0.01,) * 3), -1).reshape(-1, 3)
    xyz = np.concatenate([g + [0, 0, 0], g + [0.5, 0, 0], g[:40] + [0, 0.5, 0]]).astype(np.float32)
    ok, cl = srv.clusterize(xyz)
    ref = orc.euclidean_clusters(*xyz.T)
    assert ok and [len(c["inliers"]) for c in cl] == [125, 125, 40]
    for a, b in zip(cl, ref):
        assert np.array_equal(a["inliers"], b["inliers"])
        assert np.array_equal(a["centroid"], b["centroid"])      # Q7: sum / (n + 1)
        assert np.array_equal(a["cloud"], xyz[a["inliers"]])
    small = xyz[:29]
    assert srv.clusterize(small)[1] == []                        # < 30 points (default)
    # Q6: min input size is read from the TOLERANCE name; a double there rounds to 0 => no skip
    srv.set_param(CL_TOL, 0.03)
    try:
        ok, cl = srv.clusterize(small)
        assert len(cl) == 1
    finally:
        srv.erase_param(CL_TOL)
    srv.set_param(CL_MIN, 0.5)
    try:
        ok, cl = srv.clusterize(xyz)
        assert cl == []                                          # min = round(290 * 0.5) = 145
    finally:
        srv.erase_param(CL_MIN)
    _ = rng


def test_segment_objects_glue(srv):
    xyz = np.stack(pitt.synth_fused(41, 2, 160, 120), 1)
    outs = srv.segment_objects(xyz)
    ref = orc.find_supports(*xyz.T)
    exp = []
    for r in ref:
        cl = orc.euclidean_clusters(*r["on_support_cloud"].T)
        if cl:
            exp.append(cl)
    assert len(outs) == len(exp)
    for o, e in zip(outs, exp):
        assert [list(c["inliers"]) for c in o] == [list(c["inliers"]) for c in e]
        assert all(np.array_equal(c["centroid"], d["centroid"]) for c, d in zip(o, e))


def test_call_ransac_plane_client(srv):
    """callRansacPlaneSegmentation (ransac_segmentation.cpp:175-199): accepted iff the handler's response
    holds > 0 inliers (Q2), with the handler's response; a normals-size mismatch gives no model."""
    xyz = _cloud(1002)
    ok, inl, coef = srv.call_ransac_plane(xyz)
    h_ok, h_inl, h_coef, _ = srv.ransac_plane(xyz)
    assert ok and h_ok and np.array_equal(inl, h_inl) and np.array_equal(coef, h_coef)
    ok, inl, coef = srv.call_ransac_plane(xyz, n_normals=len(xyz) - 1)
    assert not ok and len(inl) == 0 and len(coef) == 0
    # the only inlier is point 0, which the handler drops (Q1): the client rejects the empty response
    two = np.array([[0, 0, 0], [1, 1, 1]], np.float32)
    ok, inl, _ = srv.call_ransac_plane(two)
    assert not ok and len(inl) == 0


def test_sphere_handler(srv):
    """ransacSphereDetection (sphere_segmentation_srv.cpp:29-96): params, Q1, centroid = centre."""
    from test_sphere import sphere_scene
    xyz = sphere_scene(1500, 800, 9)
    ok, inl, coef, centroid = srv.ransac_sphere(xyz)
    want = orc.sphere_segment(*xyz.T)  # PCL's float Eigen LM refinement
    assert ok and want["ok"] and len(coef) == 4
    assert np.array_equal(coef.view(np.int32), want["coef"].view(np.int32))
    assert np.array_equal(centroid, coef[:3])
    ref = want["inliers"][want["inliers"] != 0]
    assert np.array_equal(inl, ref) and 0 not in inl
    # radius limits from the parameter server: a 0.05 m sphere outside [0.1, 0.5] has no inliers
    srv.set_param("/pitt/srv/sphere_segmentation/min_radius_limit", 0.1)
    try:
        ok, inl, coef, centroid = srv.ransac_sphere(xyz)
        want = orc.sphere_segment(*xyz.T, orc.sphere_params(radius_min=0.1))
        ref = want["inliers"][want["inliers"] != 0]
        assert ok and np.array_equal(inl, ref)
    finally:
        srv.erase_param("/pitt/srv/sphere_segmentation/min_radius_limit")
    # normals of the wrong size: PCL clears the outputs
    ok, inl, coef, centroid = srv.ransac_sphere(xyz, n_normals=len(xyz) - 1)
    assert ok and len(inl) == 0 and len(coef) == 0 and not centroid.any()


def test_cylinder_handler(srv):
    """ransacCylinderDetaction (cylinder_segmentation_srv.cpp:82-216): the model, then the axis height
    pushed after the 7 coefficients and the centroid of the farthest projected pair (:129-200)."""
    from test_cylinder import cylinder_scene
    P, N, _ = cylinder_scene(1500, 500, 11)
    ok, inl, coef, centroid = srv.ransac_cylinder(P, N)
    want = orc.cylinder_segment(P, N)
    assert ok and want["ok"] and len(coef) == 8
    assert np.array_equal(coef[:7].view(np.int32), want["coef"].view(np.int32))
    # the post-processing on the handler's own coefficients: bit-exact against the restatement
    h, i1, i2, cen, _ = orc.axis_height(*P.T, coef[:6], 0)
    assert np.float32(coef[7]).view(np.int32) == np.float32(h).view(np.int32)
    assert np.array_equal(centroid.view(np.int32), cen.view(np.int32))
    ref = want["inliers"][want["inliers"] != 0]
    assert np.array_equal(inl, ref) and 0 not in inl
    # normals of the wrong size: PCL clears the outputs; the height stays -1 (:132, :195)
    ok, inl, coef, centroid = srv.ransac_cylinder(P, N, n_normals=len(P) - 1)
    assert ok and len(inl) == 0 and list(coef) == [-1.0] and not centroid.any()


def test_cone_handler(srv):
    """ransacConeDetaction (cone_segmentation_srv.cpp:83-216): the parameter-server defaults (:24-31, the
    opening angles converted at :124), the model, then the axis height pushed after the 7 coefficients and
    the centroid apex + 3/4 height along the axis (:129-200)."""
    from test_cone import cone_scene
    P, N, _ = cone_scene(1500, 500, 11)
    ok, inl, coef, centroid = srv.ransac_cone(P, N)
    want = orc.cone_segment(P, N)
    assert ok and want["ok"] and len(coef) == 8
    assert np.array_equal(coef[:7].view(np.int32), want["coef"].view(np.int32))
    # the post-processing on the handler's own coefficients: bit-exact against the restatement
    h, i1, i2, cen, _ = orc.axis_height(*P.T, coef[:6], 1)
    assert np.float32(coef[7]).view(np.int32) == np.float32(h).view(np.int32)
    assert np.array_equal(centroid.view(np.int32), cen.view(np.int32))
    ref = want["inliers"][want["inliers"] != 0]
    assert np.array_equal(inl, ref) and 0 not in inl
    # a parameter on the server reaches the model: opening angles 60-120 degrees exclude this 25-degree cone
    srv.set_param("/pitt/srv/cone_segmentation/min_opening_angle_deg", 60.0)
    srv.set_param("/pitt/srv/cone_segmentation/max_opening_angle_deg", 120.0)
    try:
        ok, inl, coef, centroid = srv.ransac_cone(P, N)
        want = orc.cone_segment(P, N, orc.cone_params(min_angle_deg=60.0, max_angle_deg=120.0))
        ref = want["inliers"][want["inliers"] != 0]
        assert ok and np.array_equal(inl, ref)
    finally:
        srv.erase_param("/pitt/srv/cone_segmentation/min_opening_angle_deg")
        srv.erase_param("/pitt/srv/cone_segmentation/max_opening_angle_deg")
    # normals of the wrong size: PCL clears the outputs; the height stays -1 (:132, :195)
    ok, inl, coef, centroid = srv.ransac_cone(P, N, n_normals=len(P) - 1)
    assert ok and len(inl) == 0 and list(coef) == [-1.0] and not centroid.any()


def test_handlers_refill_their_responses_in_place(srv):
    """The flat ABI keeps one response per service object and the handlers refill it in place (assign /
    resize on the existing vectors): a scene after a larger or smaller one must leave nothing stale."""
    scenes = [np.stack(pitt.synth_fused(s, v, 160, 120), 1) for s, v in ((51, 2), (52, 1), (51, 2), (53, 4))]
    for xyz in scenes:
        ok, sups, _ = srv.find_supports(xyz)
        ref = orc.find_supports(*xyz.T)
        assert ok and len(sups) == len(ref)
        for s, r in zip(sups, ref):
            assert np.array_equal(s["inliers"], r["idx_map"])
            assert np.array_equal(s["coefficients"], r["coefficients"])
            assert np.array_equal(s["on_support_cloud"], r["on_support_cloud"])
            assert np.array_equal(s["support_cloud"], r["support_cloud"])
        for r in ref:
            on = np.ascontiguousarray(r["on_support_cloud"], np.float32)
            if len(on) < 30:
                continue
            ok, cl = srv.clusterize(on)
            exp = orc.euclidean_clusters(*on.T)
            assert ok and [list(c["inliers"]) for c in cl] == [list(c["inliers"]) for c in exp]
            for c, e in zip(cl, exp):
                assert np.array_equal(c["centroid"], e["centroid"])
                assert np.array_equal(c["cloud"], on[c["inliers"]])
