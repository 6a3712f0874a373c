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
