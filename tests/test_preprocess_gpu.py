"""Parity of the device preprocessing steps in front of findSupports with the
oracle restatement: deepFiltering (deep_filter_srv.cpp:27-44) and pcl::transformPointCloud as
called at obj_segmentation.cpp:248.  Both are exact float / order-preserving byte work, so every
output must be bit-equal.  PCL 1.7's transforms.hpp is absent here: the transform's float order is
the published expression (oracle/pitt_oracle.cpp orc_transform_cloud), pinned by the analytic cases
in tests/test_oracle_kat.py."""
import numpy as np
import pytest
import torch

import oracle_binding as orc
import pitt_object_table_segmentation_amd as pitt

pytestmark = pytest.mark.gpu


def _dev(*arrays):
    return [torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda() for a in arrays]


def _host(planes):
    return np.stack([p.cpu().numpy() for p in planes], 1) if planes is not None else None


def _same(a, b):
    """Bit-equality of float arrays (NaN payloads included)."""
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _pose(yaw_deg, pitch_deg, cam):
    """Camera optical frame -> z-up world frame (tools' synthetic look_at), row-major 4x4 float."""
    yaw, pitch = np.radians(yaw_deg), np.radians(pitch_deg)
    f = np.array([np.sin(yaw) * np.cos(pitch), np.cos(yaw) * np.cos(pitch), -np.sin(pitch)])
    r = np.array([np.cos(yaw), -np.sin(yaw), 0.0])
    d = np.cross(f, r)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = r, d, f, cam
    return m.astype(np.float32)


@pytest.mark.parametrize("scene,seed,th", [(0, 1000, -1.0), (0, 1001, 1.2), (2, 1002, -1.0), (2, 1003, 0.9),
                                           (1, 1004, 2.0), (0, 1005, 0.0), (0, 1006, 100.0),
                                           (0, 1007, float("nan"))])
def test_deep_filter_matches_oracle(ctx, scene, seed, th):
    x, y, z = pitt.synth_frame(scene, seed)
    closer, further, used = ctx.deep_filter(*_dev(x, y, z), deep_threshold=th)
    assert used == orc.service_float_param(th, 3.0)
    rc, rf = orc.deep_filter(x, y, z, used)
    assert _same(_host(closer), rc) and _same(_host(further), rf)
    assert len(rc) + len(rf) == int(np.sum(~np.isnan(z)))


@pytest.mark.parametrize("n", [0, 1, 2047, 2048, 2049, 5000, 1228800])
def test_deep_filter_ragged_and_large(ctx, n):
    rng = np.random.default_rng(n)
    x, y = rng.normal(size=(2, n)).astype(np.float32)
    z = rng.uniform(0.0, 6.0, n).astype(np.float32)
    z[rng.uniform(size=n) < 0.1] = np.nan
    z[rng.uniform(size=n) < 0.05] = np.float32(3.0)  # ties at the default threshold stay closer
    x[rng.uniform(size=n) < 0.05] = np.nan           # a NaN x with a finite z is kept
    closer, further, used = ctx.deep_filter(*_dev(x, y, z))
    rc, rf = orc.deep_filter(x, y, z, used)
    assert _same(_host(closer), rc) and _same(_host(further), rf)


def test_deep_filter_single_output(ctx):
    x, y, z = pitt.synth_frame(0, 1010)
    closer, further, used = ctx.deep_filter(*_dev(x, y, z), deep_threshold=1.5, further=False)
    assert further is None
    rc, _ = orc.deep_filter(x, y, z, used)
    assert _same(_host(closer), rc)


@pytest.mark.parametrize("dense", [True, False])
@pytest.mark.parametrize("scene,seed", [(0, 1100), (2, 1101)])
def test_transform_matches_oracle(ctx, scene, seed, dense):
    x, y, z = pitt.synth_frame(scene, seed)
    m = _pose(3.7, 35.2, (0.013, -0.021, 1.37))
    out = ctx.transform_cloud(*_dev(x, y, z), m, dense=dense)
    ref = orc.transform_cloud(x, y, z, m, dense=dense)
    assert _same(_host(out), ref)
    if not dense:  # non-finite points are copied unchanged
        bad = ~(np.isfinite(x) & np.isfinite(y) & np.isfinite(z))
        assert _same(ref[bad], np.stack([x, y, z], 1)[bad])


def test_transform_random_matrices(ctx):
    rng = np.random.default_rng(7)
    n = 100003
    x, y, z = (rng.normal(scale=3.0, size=(3, n))).astype(np.float32)
    x[:5] = [np.inf, -np.inf, np.nan, 0.0, -0.0]
    for _ in range(4):
        m = rng.normal(size=(4, 4)).astype(np.float32)
        for dense in (True, False):
            out = ctx.transform_cloud(*_dev(x, y, z), m, dense=dense)
            assert _same(_host(out), orc.transform_cloud(x, y, z, m, dense=dense))
    # planes that are not 16-byte aligned take the scalar kernel
    dx, dy, dz = (a[1:] for a in _dev(x, y, z))
    out = ctx.transform_cloud(dx, dy, dz, m)
    assert _same(_host(out), orc.transform_cloud(x[1:], y[1:], z[1:], m))


def test_preprocessing_chain_into_supports(ctx):
    """deepFiltering -> transformPointCloud -> findSupports (obj_segmentation.cpp:241-260, minus the
    out-of-scope VoxelGrid and arm filter), device chain against the oracle chain."""
    x, y, z = pitt.synth_frame(0, 1200, 320, 240)
    closer, _, used = ctx.deep_filter(*_dev(x, y, z), further=False)
    m = _pose(0.0, 35.0, (0.0, 0.0, 1.35))
    wx, wy, wz = ctx.transform_cloud(*closer, m)
    w = np.stack([a.cpu().numpy() for a in (wx, wy, wz)], 1)
    rc, _ = orc.deep_filter(x, y, z, used)
    rw = orc.transform_cloud(*rc.T, m)
    assert _same(w, rw)
    dev = ctx.find_supports(*w.T)
    ref = orc.find_supports(*rw.T)
    assert len(dev) == len(ref)
    for d, r in zip(dev, ref):
        assert np.array_equal(d.idx_map, r["idx_map"])
        assert np.array_equal(d.coefficients, r["coefficients"])



def _pc2(xyz, point_step, row_pad, offsets, width, height, rng):
    """A PointCloud2 payload with random bytes in the unused fields and row padding."""
    row_step = width * point_step + row_pad
    buf = rng.integers(0, 256, size=height * row_step, dtype=np.uint8)
    for k in range(3):
        col = np.frombuffer(xyz[:, k].astype("<f4").tobytes(), np.uint8).reshape(-1, 4)
        for r in range(height):
            base = r * row_step + offsets[k]
            idx = base + np.arange(width)[:, None] * point_step + np.arange(4)[None, :]
            buf[idx] = col[r * width:(r + 1) * width]
    return buf, row_step


@pytest.mark.parametrize("point_step,row_pad,offsets", [(16, 0, (0, 4, 8)), (32, 0, (0, 4, 8)), (16, 16, (0, 4, 8)),
                                                        (20, 8, (8, 12, 16)), (12, 4, (0, 4, 8))])
def test_unpack_pointcloud2_matches_oracle(ctx, point_step, row_pad, offsets):
    rng = np.random.default_rng(point_step * 100 + row_pad)
    width, height = 160, 120
    x, y, z = pitt.synth_frame(2, 1300, width, height)  # NaN pixels included
    xyz = np.stack([x, y, z], 1)
    buf, row_step = _pc2(xyz, point_step, row_pad, offsets, width, height, rng)
    dx, dy, dz = ctx.unpack_pointcloud2(torch.from_numpy(buf).cuda(), width, height, point_step, row_step, offsets)
    ref = orc.unpack_pointcloud2(buf, width, height, point_step, row_step, offsets)
    assert _same(_host((dx, dy, dz)), ref)
    assert _same(ref, xyz.astype(np.float32))


def test_unpack_pointcloud2_full_frame(ctx):
    """640x480 PointXYZ (point_step 16): the 16-byte load path."""
    rng = np.random.default_rng(5)
    x, y, z = pitt.synth_frame(0, 1301)
    xyz = np.stack([x, y, z], 1)
    buf = np.zeros((len(x), 4), np.float32)
    buf[:, :3] = xyz
    buf[:, 3] = rng.normal(size=len(x))
    dx, dy, dz = ctx.unpack_pointcloud2(torch.from_numpy(buf.view(np.uint8).reshape(-1)).cuda(), 640, 480, 16, 640 * 16)
    assert _same(_host((dx, dy, dz)), xyz)


def test_unpack_pointcloud2_rejects_bad_layout(ctx):
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(pitt.PittError):
        ctx.unpack_pointcloud2(buf, 2, 1, 16, 32, (0, 4, 14))   # field past point_step
    with pytest.raises(pitt.PittError):
        ctx.unpack_pointcloud2(buf, 2, 2, 16, 16, (0, 4, 8))    # row_step shorter than a row
    with pytest.raises(pitt.PittError):
        ctx.unpack_pointcloud2(buf, 5, 1, 16, 80, (0, 4, 8))    # 5 points need 76 B, the payload has 64
    with pytest.raises(pitt.PittError):
        ctx.unpack_pointcloud2(buf, 2, 2, 16, 40, (0, 4, 8))    # second row ends at byte 68
    x, y, z = ctx.unpack_pointcloud2(buf, 4, 1, 16, 64, (0, 4, 8))  # exactly fits: 60 B needed
    assert x.numel() == 4


def test_unpack_pointcloud2_payload_ends_after_last_z(ctx):
    """a PointXYZ payload that ends right after the last point's z (width * 16 - 4 bytes)
    is valid; the 16-byte load path would read 4 bytes past it, so the scalar path must take it."""
    rng = np.random.default_rng(6)
    n = 4099
    xyz = rng.normal(size=(n, 3)).astype(np.float32)
    buf = np.zeros((n, 4), np.float32)
    buf[:, :3] = xyz
    raw = buf.view(np.uint8).reshape(-1)[:n * 16 - 4].copy()
    dx, dy, dz = ctx.unpack_pointcloud2(torch.from_numpy(raw).cuda(), n, 1, 16, n * 16)
    assert _same(_host((dx, dy, dz)), xyz)


def test_preprocessed_frames_through_plane_batch(ctx):
    """PointCloud2 payloads -> unpack -> deep filter -> world transform on the device, then the frames
    (now of different sizes) through the batched plane RANSAC; every stage and the RANSAC results
    against the oracle chain."""
    rng = np.random.default_rng(11)
    m = _pose(2.0, 36.0, (0.01, 0.0, 1.36))
    frames, ref_frames = [], []
    for k, scene in enumerate((0, 2, 0, 1)):
        x, y, z = pitt.synth_frame(scene, 1400 + k, 320, 240)
        xyz = np.stack([x, y, z], 1)
        buf, row_step = _pc2(xyz, 16, 0, (0, 4, 8), 320, 240, rng)
        ux, uy, uz = ctx.unpack_pointcloud2(torch.from_numpy(buf).cuda(), 320, 240, 16, row_step)
        closer, _, used = ctx.deep_filter(ux, uy, uz, deep_threshold=2.5 if k % 2 else -1.0, further=False)
        wx, wy, wz = ctx.transform_cloud(*closer, m)
        frames.append(tuple(a.cpu().numpy() for a in (wx, wy, wz)))
        rc, _ = orc.deep_filter(*orc.unpack_pointcloud2(buf, 320, 240, 16, row_step).T, used)
        ref_frames.append(tuple(orc.transform_cloud(*rc.T, m).T))
    for f, r in zip(frames, ref_frames):
        assert _same(np.stack(f, 1), np.stack(r, 1))
    b = pitt.FrameBatch.from_host(frames)
    inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda")
    res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
    inl = inl.cpu().numpy()
    for i, (f, r) in enumerate(zip(ref_frames, res)):
        o = orc.plane_segment(*f)
        assert r["hypotheses"] == o.hypotheses and r["best_count"] == o.best_count
        assert np.array_equal(inl[b.offsets[i]:b.offsets[i] + r["n_inliers"]], o.inliers)
        assert np.array_equal(r["coefficients"][:r["n_coeff"]], o.coefficients)
