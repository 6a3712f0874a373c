"""The ROS nodes of adapters/ros, checked without ROS: every node compiles
with g++ against the minimal stand-in headers in tests/ros_stub (syntax, types and the C-ABI
calls), and the PointCloud2 conversions reject malformed payloads the way the device unpack
(pitt_unpack_pointcloud2) does instead of reading past the buffer."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "ros_stub")
INC = ["-I" + STUB, "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "adapters", "ros"),
       "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
NODES = sorted(glob.glob(os.path.join(ROOT, "adapters", "ros", "*.cpp")))


def test_nine_nodes_present():
    """Seven service nodes and the two orchestrators (obj_segmentation, ransac_segmentation)."""
    assert len(NODES) == 9


@pytest.mark.parametrize("src", NODES, ids=[os.path.basename(n) for n in NODES])
def test_ros_node_compiles(src):
    p = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror"] + INC + [src],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]


def test_pointcloud2_layout_checks(tmp_path):
    exe = str(tmp_path / "layout_check")
    p = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-fsanitize=address,undefined"] + INC +
                       [os.path.join(STUB, "layout_check.cpp"), "-o", exe], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    got = {ln.split()[0]: [float(v) for v in ln.split()[1:]] for ln in r.stdout.splitlines()}
    # well-formed: point i at byte 16 i -> floats 4 i, 4 i + 1, 4 i + 2, pad 1.0
    assert got["ok"][0] == 24 and got["ok"][1:9] == [0, 1, 2, 1, 4, 5, 6, 1]
    assert got["ok_padded_rows"][0] == 24 and got["ok_padded_rows"][1:5] == [0, 1, 2, 1]
    for bad in ("short_payload", "row_step_small", "field_beyond_step", "big_endian", "no_fields"):
        assert got[bad] == [0], bad
    assert got["normals_ok"] == [6, 0, 1, 2, 4, 5, 6]
    assert got["normals_short"] == [0]
    assert got["normals_missing"] == [6, 0, 0, 0, 0, 0, 0]
    assert "rejected" in r.stderr


def test_orchestrator_harness_links(tmp_path):
    """The two orchestrator nodes link against libpitt_seg.so in their harness (every C-ABI symbol they
    call is exported); running them needs the GPU (tests/test_ros_orchestrators_gpu.py)."""
    lib = os.path.join(ROOT, "pitt_object_table_segmentation_amd", "libpitt_seg.so")
    if not os.path.exists(lib):
        pytest.skip("libpitt_seg.so not built")
    p = subprocess.run(["make", "-C", STUB, "OUT=" + str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    for n in ("obj_segmentation_harness", "ransac_segmentation_harness"):
        assert os.access(str(tmp_path / n), os.X_OK)


# ---- the orchestrator nodes' own code on the CPU, over a host emulation of the C ABI ------------------
# tests/ros_stub/abi_host_emu.cpp stands in for libpitt_seg.so (the oracle underneath, hipMalloc over
# malloc); the nodes' argument handling, TF, parameter forwarding, arm filter round trip and message
# assembly run unchanged.  The same nodes run on the MI355X in tests/test_ros_orchestrators_gpu.py.
@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    out = tmp_path_factory.mktemp("emu")
    p = subprocess.run(["make", "-C", STUB, "OUT=" + str(out), "emu"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    return out


def _emu_run(emu, node, mode, inp, outp, *opts):
    p = subprocess.run([str(emu / f"{node}_emu"), mode, str(inp), str(outp), *opts], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return p.stderr


def test_obj_segmentation_node_on_host_emulation(emu, tmp_path):
    """depthAcquisition's chain through the node (padded PointCloud2, TF pose, the arm filter service, deep
    threshold and support parameters from the parameter server) equals the oracle's chain of the same
    stages; without an arm_filter_srv the frame is dropped; with ~arm_filter false the call is skipped."""
    import numpy as np
    import pitt_object_table_segmentation_amd as pitt
    from test_preprocess_gpu import _pose
    from test_ros_orchestrators_gpu import _oracle_chain, _pose_arg, _read_clusters_outputs, _same, _write_cloud
    x, y, z = pitt.synth_frame(pitt.SCENE_TABLE_NAN, 2100, 640, 480)
    pose = _pose(0.0, 35.0, (0.0, 0.0, 1.35))
    _write_cloud(tmp_path / "c.bin", np.stack([x, y, z], 1), np.random.default_rng(1))
    log = _emu_run(emu, "obj_segmentation", "obj", tmp_path / "c.bin", tmp_path / "o.bin", "--pose", _pose_arg(pose))
    _same(_read_clusters_outputs(tmp_path / "o.bin"), _oracle_chain(x, y, z, pose))
    assert "raw clusters data" in log and "0, 0, 0, " in log
    # parameters and a cropping arm filter
    x, y, z = pitt.synth_frame(pitt.SCENE_TABLE, 2102, 640, 480)
    pose = _pose(0.0, 35.0, (0.0, 0.0, 1.35))
    _write_cloud(tmp_path / "c2.bin", np.stack([x, y, z], 1), np.random.default_rng(2), point_step=16, row_pad=0)
    _emu_run(emu, "obj_segmentation", "obj", tmp_path / "c2.bin", tmp_path / "o2.bin", "--pose", _pose_arg(pose),
             "--arm", "crop:0.3", "--param", "/pitt/service/deep_filter/z_threshold=dbl:2.2",
             "--param", "/pitt/srv/supports_segmentation/max_iter=int:25",
             "--param", "/pitt/srv/supports_segmentation/in_shape_distance_th=dbl:0.015")
    _same(_read_clusters_outputs(tmp_path / "o2.bin"),
          _oracle_chain(x, y, z, pose, deep=2.2, crop=0.3, ransac_max_iterations=25,
                        ransac_distance_threshold=np.float32(0.015)))
    # no arm filter service: the frame is dropped (obj_segmentation.cpp:244); ~arm_filter false: skipped
    _emu_run(emu, "obj_segmentation", "obj", tmp_path / "c2.bin", tmp_path / "o3.bin", "--pose", _pose_arg(pose),
             "--arm", "missing")
    assert _read_clusters_outputs(tmp_path / "o3.bin") == []
    _emu_run(emu, "obj_segmentation", "obj", tmp_path / "c2.bin", tmp_path / "o4.bin", "--pose", _pose_arg(pose),
             "--arm", "none")
    _same(_read_clusters_outputs(tmp_path / "o4.bin"), _oracle_chain(x, y, z, pose))


def test_ransac_segmentation_node_on_host_emulation(emu, tmp_path):
    """clustersAcquisition's publication (ransac_segmentation.cpp:315-328) from the classification
    result: one TrackedShape per cluster in input order, the cluster's id and point-cloud centroid, the
    tag's name, and for a known shape the chosen service's coefficients (its n_coef values) and centroid."""
    import numpy as np
    from test_ros_orchestrators_gpu import _read_tracked_shapes, _write_clusters
    rng = np.random.default_rng(3)
    sizes = [0, 1, 7, 12, 33, 64, 100, 101, 102, 103]
    clusters = [rng.normal(0, 0.1, (n, 3)).astype(np.float32) for n in sizes]
    _write_clusters(tmp_path / "cl.bin", clusters)
    log = _emu_run(emu, "ransac_segmentation", "ransac", tmp_path / "cl.bin", tmp_path / "o.bin")
    msgs = _read_tracked_shapes(tmp_path / "o.bin")
    assert len(msgs) == 1 and len(msgs[0]) == len(clusters)
    names = ["unknown", "plane", "sphere", "cone", "cylinder"]
    ncoef = {"sphere": 4, "cylinder": 8, "cone": 8, "plane": 4}
    qof = {"sphere": 0, "cylinder": 1, "cone": 2, "plane": 3}
    for c, (P, s) in enumerate(zip(clusters, msgs[0])):
        assert s["object_id"] == 100 + c
        assert np.array_equal(s["pc"], np.asarray(P.mean(0) if len(P) else np.zeros(3), np.float32))
        tag = names[len(P) % 5]
        assert s["tag"] == tag, (c, s["tag"])
        if tag == "unknown":
            assert len(s["coef"]) == 0 and not s["est"].any()
        else:
            q = qof[tag]
            assert s["coef"].tolist() == [float(10 * c + k) + 0.25 * q for k in range(ncoef[tag])]
            assert s["est"].tolist() == [c + 0.5 * k for k in range(3)]
    assert log.count("#INLIER") == len(clusters) and "selected: cylinder" in log
