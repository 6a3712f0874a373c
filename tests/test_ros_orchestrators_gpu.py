"""The two orchestrator nodes (adapters/ros/obj_segmentation_node.cpp, ransac_segmentation_node.cpp) run
end to end on the MI355X through the ROS stand-ins: tests/ros_stub/orchestrator_harness.cpp delivers
one message to the node's subscriber, runs the node's own main loop, and records what it publishes.

obj_segmentation: a Kinect-like PointCloud2 (padded fields) -> the node's device chain (unpack, 1 cm
VoxelGrid, deep filter, the arm filter service round trip, world transform, supports, clusters per
support) against the oracle's chain of the same stages (obj_segmentation.cpp:229-312): every published
ClustersOutput's member indices, points and centroids bit for bit.

ransac_segmentation: a frame of ten tracked clusters -> one TrackedShapes whose tags, coefficients and
estimated centroids equal the per-cluster service calls of clustersAcquisition (:230-328), as
test_classify_gpu holds the batched classification to them.

The harness binaries are built on the CPU beforehand (make -C tests/ros_stub, run by
__graft_entry__.build()); a missing binary fails the test."""
import os
import subprocess

import numpy as np
import pytest

import oracle_binding as orc
import pitt_object_table_segmentation_amd as pitt
from test_preprocess_gpu import _pc2, _pose

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "ros_stub", "_build")


def _harness(name):
    exe = os.path.join(BUILD, f"{name}_harness")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} missing: run make -C tests/ros_stub (part of __graft_entry__.build())")
    return exe


def _run(name, mode, inp, out, *opts):
    p = subprocess.run([_harness(name), mode, str(inp), str(out), *opts], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    return p.stderr


class _Reader:
    def __init__(self, path):
        self.b = open(path, "rb").read()
        self.o = 0

    def take(self, dtype, n=1):
        a = np.frombuffer(self.b, dtype, n, self.o)
        self.o += a.nbytes
        return a

    def i64(self):
        return int(self.take(np.int64)[0])


def _read_clusters_outputs(path):
    r = _Reader(path)
    msgs = []
    for _ in range(r.i64()):
        cl = []
        for _ in range(r.i64()):
            idx = r.take(np.int32, r.i64()).copy()
            cen = r.take(np.float32, 3).copy()
            pts = r.take(np.float32, 3 * r.i64()).reshape(-1, 3).copy()
            cl.append((idx, cen, pts))
        msgs.append(cl)
    return msgs


def _write_cloud(path, xyz, rng, point_step=32, row_pad=16, width=640, height=480):
    offsets = (0, 4, 8)
    buf, row_step = _pc2(xyz, point_step, row_pad, offsets, width, height, rng)
    hdr = np.array([width, height, point_step, row_step, *offsets], np.int64)
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(buf.tobytes())


def _oracle_chain(x, y, z, pose, deep=-1.0, crop=None, **support):
    """depthAcquisition's stages on the oracle: VoxelGrid -> deep filter -> arm filter -> transform ->
    supports -> clusters of every support with >= 30 on-support points (obj_segmentation.cpp:238-312)."""
    v, _ = orc.voxel_grid(x, y, z)
    closer, _ = orc.deep_filter(*v.T, orc.service_float_param(deep, 3.0))
    if crop is not None:
        closer = closer[closer[:, 0] <= np.float32(crop)]
    w = orc.transform_cloud(*closer.T, pose)
    if len(w) <= 30:
        return []
    msgs = []
    for s in orc.find_supports(*w.T, **support):
        on = s["on_support_cloud"]
        cl = orc.euclidean_clusters(*on.T) if len(on) >= 30 else []
        if cl:
            msgs.append([(c["inliers"], c["centroid"], on[c["inliers"]]) for c in cl])
    return msgs


def _same(got, want):
    assert len(got) == len(want) and len(want) >= 1
    for gm, wm in zip(got, want):
        assert len(gm) == len(wm)
        for (gi, gc, gp), (wi, wc, wp) in zip(gm, wm):
            assert np.array_equal(gi, wi)
            assert np.array_equal(gc.view(np.int32), np.asarray(wc, np.float32).view(np.int32))
            assert np.array_equal(gp.view(np.int32), np.ascontiguousarray(wp, np.float32).view(np.int32))


def _pose_arg(m):
    return ",".join(repr(float(v)) for v in np.asarray(m, np.float32)[:3].reshape(-1))


@pytest.mark.parametrize("seed", [2100, 2101])
def test_obj_segmentation_node_matches_oracle_chain(tmp_path, seed):
    x, y, z = pitt.synth_frame(pitt.SCENE_TABLE_NAN, seed, 640, 480)
    pose = _pose(0.0, 35.0, (0.0, 0.0, 1.35))
    _write_cloud(tmp_path / "cloud.bin", np.stack([x, y, z], 1), np.random.default_rng(seed))
    log = _run("obj_segmentation", "obj", tmp_path / "cloud.bin", tmp_path / "out.bin", "--pose", _pose_arg(pose))
    got = _read_clusters_outputs(tmp_path / "out.bin")
    _same(got, _oracle_chain(x, y, z, pose))
    assert "raw clusters data" in log


def test_obj_segmentation_node_parameters_and_arm_filter(tmp_path):
    """The deep-filter threshold and support parameters from the parameter server, and an arm filter
    service that crops the cloud: the node's result follows each, as the reference's does."""
    x, y, z = pitt.synth_frame(pitt.SCENE_TABLE, 2102, 640, 480)
    pose = _pose(0.0, 35.0, (0.0, 0.0, 1.35))
    _write_cloud(tmp_path / "cloud.bin", np.stack([x, y, z], 1), np.random.default_rng(7), point_step=16, row_pad=0)
    opts = ["--pose", _pose_arg(pose), "--arm", "crop:0.3",
            "--param", "/pitt/service/deep_filter/z_threshold=dbl:2.2",
            "--param", "/pitt/srv/supports_segmentation/max_iter=int:25",
            "--param", "/pitt/srv/supports_segmentation/in_shape_distance_th=dbl:0.015"]
    _run("obj_segmentation", "obj", tmp_path / "cloud.bin", tmp_path / "out.bin", *opts)
    got = _read_clusters_outputs(tmp_path / "out.bin")
    want = _oracle_chain(x, y, z, pose, deep=2.2, crop=0.3, ransac_max_iterations=25,
                         ransac_distance_threshold=np.float32(0.015))
    _same(got, want)


def test_obj_segmentation_node_arm_filter_missing_or_disabled(tmp_path):
    """callArmFilter fails when no arm_filter_srv answers: the frame is dropped and nothing is published
    (:244).  With ~arm_filter false the node skips the call and publishes the unfiltered chain."""
    x, y, z = pitt.synth_frame(pitt.SCENE_TABLE, 2103, 640, 480)
    pose = _pose(0.0, 35.0, (0.0, 0.0, 1.35))
    _write_cloud(tmp_path / "cloud.bin", np.stack([x, y, z], 1), np.random.default_rng(8))
    _run("obj_segmentation", "obj", tmp_path / "cloud.bin", tmp_path / "o1.bin", "--pose", _pose_arg(pose),
         "--arm", "missing")
    assert _read_clusters_outputs(tmp_path / "o1.bin") == []
    _run("obj_segmentation", "obj", tmp_path / "cloud.bin", tmp_path / "o2.bin", "--pose", _pose_arg(pose),
         "--arm", "none")
    _same(_read_clusters_outputs(tmp_path / "o2.bin"), _oracle_chain(x, y, z, pose))


def _write_clusters(path, clusters):
    with open(path, "wb") as f:
        f.write(np.int64(len(clusters)).tobytes())
        for j, P in enumerate(clusters):
            f.write(np.int32(100 + j).tobytes())
            f.write(np.asarray(P.mean(0) if len(P) else np.zeros(3), np.float32).tobytes())
            f.write(np.int64(len(P)).tobytes())
            f.write(np.ascontiguousarray(P, np.float32).tobytes())


def _read_tracked_shapes(path):
    r = _Reader(path)
    msgs = []
    for _ in range(r.i64()):
        shapes = []
        for _ in range(r.i64()):
            oid = int(r.take(np.int32)[0])
            pc = r.take(np.float32, 3).copy()
            tag = r.take(np.uint8, r.i64()).tobytes().decode()
            est = r.take(np.float32, 3).copy()
            coef = r.take(np.float32, r.i64()).copy()
            shapes.append(dict(object_id=oid, pc=pc, tag=tag, est=est, coef=coef))
        msgs.append(shapes)
    return msgs


def test_ransac_segmentation_node_matches_per_cluster_services(tmp_path):
    from test_classify_gpu import _per_cluster, frame_clusters
    clusters = frame_clusters(4) + [np.zeros((0, 3), np.float32)]
    _write_clusters(tmp_path / "cl.bin", clusters)
    log = _run("ransac_segmentation", "ransac", tmp_path / "cl.bin", tmp_path / "out.bin")
    msgs = _read_tracked_shapes(tmp_path / "out.bin")
    assert len(msgs) == 1 and len(msgs[0]) == len(clusters)
    names = {pitt.SHAPE_UNKNOWN: "unknown", pitt.SHAPE_PLANE: "plane", pitt.SHAPE_SPHERE: "sphere",
             pitt.SHAPE_CONE: "cone", pitt.SHAPE_CYLINDER: "cylinder"}
    src = {pitt.SHAPE_SPHERE: 0, pitt.SHAPE_CYLINDER: 1, pitt.SHAPE_CONE: 2, pitt.SHAPE_PLANE: 3}
    with pitt.Context(0) as ctx:
        srv = pitt.Services(ctx)
        try:
            for j, (P, s) in enumerate(zip(clusters, msgs[0])):
                assert s["object_id"] == 100 + j
                assert np.array_equal(s["pc"], np.asarray(P.mean(0) if len(P) else np.zeros(3), np.float32))
                if len(P) == 0:
                    assert s["tag"] == "unknown" and len(s["coef"]) == 0
                    continue
                want, counts, tag = _per_cluster(ctx, srv, P)
                assert s["tag"] == names[tag], (j, s["tag"], counts)
                if tag in src:
                    ok, inl, coef, centroid = want[src[tag]]
                    assert np.array_equal(s["coef"].view(np.int32), np.asarray(coef, np.float32).view(np.int32))
                    assert np.array_equal(s["est"].view(np.int32), np.asarray(centroid, np.float32).view(np.int32))
        finally:
            srv.close()
    assert len({s["tag"] for s in msgs[0]}) >= 2
    assert log.count("#INLIER") == len(clusters)


def test_srv_segment_objects_dev_equals_host_service():
    """pitt_srv_segment_objects_dev (the obj_segmentation node's entry point) against the host-side
    segmentObjects mirror (the reference's service calls, held to the oracle in test_services_gpu):
    the same clusters per support, under the defaults and under parameter-server overrides, which
    both read the same way (callSupportFilter's -1 sentinels, clusterize's Q6)."""
    import torch
    x, y, z = pitt.synth_fused(1300, 2, 320, 240)
    cloud = np.stack([x, y, z], 1)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (x, y, z)]
    with pitt.Context(0) as ctx:
        srv = pitt.Services(ctx)
        try:
            for params in ({}, {"/pitt/srv/supports_segmentation/max_iter": 25,
                                "/pitt/srv/supports_segmentation/horizontal_axis": [0.0, 0.0, -1.0],
                                "/pitt/srv/cluster_segmentation/min_rate": 0.02}):
                for k, v in params.items():
                    srv.set_param(k, v)
                sp, cp = srv.resolved_params()
                if params:
                    assert sp.ransac_max_iterations == 25 and cp.min_rate == 0.02
                else:
                    assert sp.ransac_max_iterations == 10 and abs(cp.tolerance - 0.03) < 1e-12
                host = srv.segment_objects(cloud)
                dev = srv.segment_objects_dev(*d)
                assert len(host) == len(dev) >= 1
                for hm, dm in zip(host, dev):
                    assert len(hm) == len(dm)
                    for a, b in zip(hm, dm):
                        assert np.array_equal(a["inliers"], b["inliers"])
                        assert np.array_equal(a["centroid"].view(np.int32), b["centroid"].view(np.int32))
                for k in params:
                    srv.erase_param(k)
        finally:
            srv.close()
