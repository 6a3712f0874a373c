"""NormalEstimation<PointXYZ, Normal>, KdTree, setKSearch(50) (pc_manager.cpp:68-78).

CPU: the oracle's restatement against scipy's cKDTree neighbour sets (independent exact kNN) and
analytic planes.  GPU: pitt_normal_estimation against the oracle bit for bit -- neighbour lists in
summation order, normals and curvature -- on voxel-downsampled camera frames (the reference's input,
obj_segmentation.cpp:238-253), a raw organised frame, NaN points, duplicates (index-ordered ties) and
clouds with fewer than k or 3 points.
"""
import numpy as np
import pytest

import oracle_binding as orc


def frame(scene, seed, w=640, h=480):
    from pitt_object_table_segmentation_amd import api
    return api.synth_frame(scene, seed, w, h)


def voxelized(scene, seed):
    v, _ = orc.voxel_grid(*frame(scene, seed))
    return v[:, 0].copy(), v[:, 1].copy(), v[:, 2].copy()


# ---- oracle -------------------------------------------------------------------------------------
def test_oracle_neighbours_match_ckdtree():
    from scipy.spatial import cKDTree
    x, y, z = voxelized(0, 1000)
    _, _, (nn, cnt) = orc.normal_estimation(x, y, z, neighbours=True)
    p = np.stack([x, y, z], 1).astype(np.float64)
    d, i = cKDTree(p).query(p, k=51)
    # sets are compared where the 50th and 51st float64 distances are apart (no float ordering doubt)
    clear = (d[:, 50] - d[:, 49]) > 1e-6 * np.maximum(d[:, 50], 1e-9)
    assert clear.mean() > 0.95 and np.all(cnt == 50)
    same = [set(a) == set(b) for a, b, c in zip(nn, i[:, :50], clear) if c]
    assert all(same)
    # the list is in ascending distance
    dd = np.take_along_axis(((p[nn] - p[:, None, :]) ** 2).sum(-1), np.arange(50)[None, :], 1)
    assert np.all(np.diff(dd, axis=1) >= -1e-9)


def test_oracle_plane_normals_and_flip():
    g = np.stack(np.meshgrid(np.arange(30) * 0.01, np.arange(30) * 0.01), -1).reshape(-1, 2)
    pts = np.c_[g, np.full(len(g), 0.7)].astype(np.float32)
    nrm, cur = orc.normal_estimation(*pts.T)
    assert np.allclose(np.abs(nrm[:, 2]), 1.0, atol=1e-6) and np.all(cur < 1e-6)
    assert np.all(nrm[:, 2] < 0)  # flipped towards the origin (below the plane)
    nrm2, _ = orc.normal_estimation(*pts.T, viewpoint=(0.0, 0.0, 2.0))
    assert np.all(nrm2[:, 2] > 0)


def test_oracle_small_and_nan():
    nrm, cur = orc.normal_estimation(np.zeros(2, np.float32), np.ones(2, np.float32), np.arange(2, dtype=np.float32))
    assert np.all(np.isnan(nrm)) and np.all(np.isnan(cur))  # fewer than 3 points
    rng = np.random.default_rng(1)
    p = rng.uniform(0, 1, (200, 3)).astype(np.float32)
    p[::9, 0] = np.nan
    nrm, cur, (nn, cnt) = orc.normal_estimation(*p.T, neighbours=True)
    bad = np.isnan(p).any(1)
    assert np.all(np.isnan(nrm[bad])) and not np.isnan(nrm[~bad]).any()
    assert np.all(cnt[~bad] == 50) and not np.isin(nn[~bad], np.nonzero(bad)[0]).any()


# ---- HIP path -----------------------------------------------------------------------------------
def _gpu(ctx, x, y, z, k=50, viewpoint=(0.0, 0.0, 0.0)):
    import torch
    t = [torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda() for a in (x, y, z)]
    nx, ny, nz, cv, (nn, cnt) = ctx.normal_estimation(*t, k=k, viewpoint=viewpoint, neighbours=True)
    return (np.stack([nx.cpu().numpy(), ny.cpu().numpy(), nz.cpu().numpy()], 1), cv.cpu().numpy(),
            nn.cpu().numpy(), cnt.cpu().numpy())


def _check(ctx, x, y, z, k=50, viewpoint=(0.0, 0.0, 0.0)):
    nrm, cur, nn, cnt = _gpu(ctx, x, y, z, k, viewpoint)
    rn, rc, (rnn, rcnt) = orc.normal_estimation(x, y, z, k, viewpoint, neighbours=True)
    assert np.array_equal(cnt, rcnt)
    for i in np.nonzero(cnt)[0][:: max(1, len(cnt) // 20000)]:
        assert np.array_equal(nn[i, :cnt[i]], rnn[i, :rcnt[i]]), i
    assert np.array_equal(nrm, rn, equal_nan=True)
    assert np.array_equal(cur, rc, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("scene,seed", [(0, 1000), (2, 1001), (1, 1003)])
def test_hip_normals_voxelized_frames(ctx, scene, seed):
    _check(ctx, *voxelized(scene, seed))


@pytest.mark.gpu
def test_hip_normals_raw_frame(ctx):
    _check(ctx, *frame(0, 1004, 160, 120))


@pytest.mark.gpu
def test_hip_normals_edges(ctx):
    rng = np.random.default_rng(2)
    p = rng.uniform(-0.2, 0.2, (3000, 3)).astype(np.float32)
    p[::11, 2] = np.nan
    p[5] = p[6]  # an exact duplicate: tied distances go by index
    p[7] = p[6]
    _check(ctx, *p.T)
    _check(ctx, *p.T, k=7, viewpoint=(0.0, 0.0, 1.0))
    far = np.concatenate([p[:500], np.array([[5.0, 5.0, 5.0], [-4.0, 3.0, 9.0]], np.float32)])
    _check(ctx, *far.T)  # isolated points: the ring grows to the whole grid
    _check(ctx, *p[:20].T)  # fewer points than k
    _check(ctx, *p[:2].T)   # fewer than 3: NaN
    _check(ctx, *np.zeros((0, 3), np.float32).T)
