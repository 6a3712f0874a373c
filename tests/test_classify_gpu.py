"""Batched primitive classification of a frame's clusters (pitt_classify_clusters).

clustersAcquisition (ransac_segmentation.cpp:230-302) runs, per cluster, PCManager::estimateNormal (k = 50),
the sphere, cylinder, cone and plane services and the arbitration on their response sizes.  The batched
entry point runs all clusters through every stage together; each stage runs the per-cluster service's
kernels on the same values, so its counts, coefficients, heights, centroids and tags must equal the
per-cluster services' (pitt_srv_ransac_*, themselves held to the oracle in test_services_gpu.py) bit for
bit."""
import numpy as np
import pytest

import pitt_object_table_segmentation_amd as pitt
from test_cone import cone_scene
from test_cylinder import cylinder_scene
from test_pcl_lm import _box
from test_sphere import sphere_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = pitt.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def srv(ctx):
    s = pitt.Services(ctx)
    yield s
    s.close()


def frame_clusters(seed=0):
    """Ten table-top clusters of the four kinds and mixed sizes (normals are re-estimated, as the
    reference does, so the generators' normals are dropped)."""
    rng = np.random.default_rng(seed)
    cl = [sphere_scene(900, 150, 41 + seed), cylinder_scene(1200, 200, 42 + seed)[0],
          cone_scene(1000, 150, 43 + seed, half_deg=25.0)[0], _box(1500, 44 + seed),
          sphere_scene(300, 40, 45 + seed, radius=0.03), cylinder_scene(600, 60, 46 + seed, r=0.03)[0],
          _box(400, 47 + seed), cone_scene(2500, 300, 48 + seed, half_deg=35.0)[0],
          sphere_scene(2000, 500, 49 + seed, radius=0.08), cylinder_scene(3000, 600, 50 + seed, r=0.05)[0]]
    return [np.ascontiguousarray(c.astype(np.float32)[rng.permutation(len(c))]) for c in cl]


def _layout(clusters, gap=37):
    """One SoA with the clusters at unaligned offsets and junk between them."""
    offs, n = [], gap
    for c in clusters:
        offs.append(n)
        n += len(c) + gap
    xyz = np.full((n, 3), 7.0, np.float32)
    for o, c in zip(offs, clusters):
        xyz[o:o + len(c)] = c
    return xyz, np.array(offs, np.int64), np.array([len(c) for c in clusters], np.int64)


def _per_cluster(ctx, srv, P):
    """clustersAcquisition's body for one cluster through the per-cluster services."""
    import torch
    d = [torch.from_numpy(np.ascontiguousarray(P[:, k])).cuda() for k in range(3)]
    nx, ny, nz, _ = ctx.normal_estimation(*d, k=50)
    N = torch.stack([nx, ny, nz], 1).cpu().numpy()
    out = []
    out.append(srv.ransac_sphere(P))
    out.append(srv.ransac_cylinder(P, N))
    out.append(srv.ransac_cone(P, N))
    out.append(srv.ransac_plane(P))
    counts = [len(r[1]) if r[0] else 0 for r in out]
    tag = pitt.Services.arbitrate(*counts)
    return out, counts, tag


def _bits(a):
    return np.asarray(a, np.float32).view(np.int32)


def _check_against_services(ctx, srv, clusters, got):
    for P, g in zip(clusters, got):
        want, counts, tag = _per_cluster(ctx, srv, P)
        assert g["n_points"] == len(P)
        assert g["inliers"] == counts, (g["inliers"], counts)
        assert g["tag"] == tag
        for q in range(4):
            ok, inl, coef, centroid = want[q]
            assert np.array_equal(_bits(g["coefficients"][q]), _bits(coef)), (q, g["coefficients"][q], coef)
            assert np.array_equal(_bits(g["centroid"][q]), _bits(centroid)), (q, g["centroid"][q], centroid)
        src = {pitt.SHAPE_SPHERE: 0, pitt.SHAPE_CYLINDER: 1, pitt.SHAPE_CONE: 2, pitt.SHAPE_PLANE: 3}.get(tag)
        if src is not None:
            assert np.array_equal(_bits(g["est_centroid"]), _bits(want[src][3]))


def test_batch_equals_per_cluster_services(ctx, srv):
    """Ten clusters (device SoA, unaligned offsets): every service's response size, coefficients (with
    the cylinder / cone heights) and centroid, and the arbitration, as the per-cluster services."""
    import torch
    clusters = frame_clusters(0)
    xyz, offs, cnt = _layout(clusters)
    d = [torch.from_numpy(np.ascontiguousarray(xyz[:, k])).cuda() for k in range(3)]
    got = srv.classify_clusters(*d, offs, cnt)
    _check_against_services(ctx, srv, clusters, got)
    # the clusters are not all classified alike, and each service finds models
    assert len({g["tag"] for g in got}) >= 3
    assert all(sum(g["status"][q] == pitt.PITT_OK for g in got) >= 5 for q in range(4))
    # the context-level entry point with the services' defaults gives the same
    got2 = ctx.classify_clusters(*d, offs, cnt)
    for a, b in zip(got, got2):
        assert a["inliers"] == b["inliers"] and a["tag"] == b["tag"]
        assert all(np.array_equal(_bits(x), _bits(y)) for x, y in zip(a["coefficients"], b["coefficients"]))


def test_host_memory_and_repeated_calls(ctx, srv):
    """Host SoA in; a second call (scratch reused) gives the same bits."""
    clusters = frame_clusters(1)[:4]
    xyz, offs, cnt = _layout(clusters, gap=5)
    a = ctx.classify_clusters(xyz[:, 0], xyz[:, 1], xyz[:, 2], offs, cnt)
    b = ctx.classify_clusters(xyz[:, 0], xyz[:, 1], xyz[:, 2], offs, cnt)
    for x, y in zip(a, b):
        assert x["inliers"] == y["inliers"] and x["tag"] == y["tag"]
        assert all(np.array_equal(_bits(u), _bits(v)) for u, v in zip(x["coefficients"], y["coefficients"]))
    _check_against_services(ctx, srv, clusters, a)


def test_degenerate_clusters(ctx, srv):
    """Empty, 1-, 2-, 3- and 5-point clusters and one with NaN points, beside a normal one: each service
    answers as the per-cluster handler does (no model below its sample size; index 0 dropped)."""
    rng = np.random.default_rng(5)
    nanc = sphere_scene(400, 50, 61).astype(np.float32)
    nanc[rng.choice(len(nanc), 40, replace=False)] = np.nan
    clusters = [np.zeros((0, 3), np.float32), rng.normal(0, 0.01, (1, 3)).astype(np.float32),
                rng.normal(0, 0.01, (2, 3)).astype(np.float32), rng.normal(0, 0.01, (3, 3)).astype(np.float32),
                (rng.normal(0, 0.01, (5, 3)) + 1).astype(np.float32), nanc, _box(600, 62)]
    xyz, offs, cnt = _layout(clusters, gap=3)
    got = srv.classify_clusters(xyz[:, 0], xyz[:, 1], xyz[:, 2], offs, cnt)
    assert got[0]["n_points"] == 0 and got[0]["tag"] == pitt.SHAPE_UNKNOWN and got[0]["inliers"] == [0, 0, 0, 0]
    _check_against_services(ctx, srv, clusters[1:], got[1:])


def test_service_parameters_reach_the_batch(ctx, srv):
    """A parameter-server override (the cone's opening angles) changes the batch as it changes the service."""
    clusters = frame_clusters(2)[:4]
    xyz, offs, cnt = _layout(clusters)
    srv.set_param("/pitt/srv/cone_segmentation/min_opening_angle_deg", 60.0)
    srv.set_param("/pitt/srv/cone_segmentation/max_opening_angle_deg", 120.0)
    try:
        got = srv.classify_clusters(xyz[:, 0], xyz[:, 1], xyz[:, 2], offs, cnt)
        _check_against_services(ctx, srv, clusters, got)
    finally:
        srv.erase_param("/pitt/srv/cone_segmentation/min_opening_angle_deg")
        srv.erase_param("/pitt/srv/cone_segmentation/max_opening_angle_deg")


def test_batch_time_per_frame(ctx):
    """The bench's figure (ms per frame of ten clusters), and fewer host round trips than the per-cluster
    loop: stage-wise synchronisation is what the batch is for."""
    import time
    import torch
    clusters = frame_clusters(3)
    xyz, offs, cnt = _layout(clusters)
    d = [torch.from_numpy(np.ascontiguousarray(xyz[:, k])).cuda() for k in range(3)]
    ctx.classify_clusters(*d, offs, cnt)
    t0 = time.perf_counter()
    for _ in range(3):
        ctx.classify_clusters(*d, offs, cnt)
    ms = (time.perf_counter() - t0) / 3 * 1e3
    print(f"classify: {ms:.2f} ms per frame of {len(clusters)} clusters")
    assert ms < 1000.0


def test_sampler_table_memo_across_iteration_limits(ctx, srv):
    """The sampler-table memo (prim_ransac.hpp): a batch at max_iterations X, then one at Y < X
    whose first cloud is too small to sample (its slot is skipped while later slots are written at the
    Y stride, over the X layout's slot 0), then the first batch again: the repeat must not reuse slot 0's
    overwritten table.  Equal to the first call and to the per-cluster services at X."""
    clusters = frame_clusters(4)[:3]
    tiny = np.random.default_rng(9).normal(0, 0.01, (2, 3)).astype(np.float32)
    names = ["/pitt/srv/sphere_segmentation/max_iter_limit", "/pitt/srv/cylinder_segmentation/max_iter_limit",
             "/pitt/srv/cone_segmentation/max_iter_limit"]

    def run(cl, iters):
        for n in names:
            srv.set_param(n, iters)
        xyz, offs, cnt = _layout(cl, gap=11)
        return srv.classify_clusters(xyz[:, 0], xyz[:, 1], xyz[:, 2], offs, cnt)

    try:
        first = run(clusters, 300)
        run([tiny] + clusters[1:], 40)
        again = run(clusters, 300)
        for a, b in zip(first, again):
            assert a["inliers"] == b["inliers"] and a["tag"] == b["tag"]
            assert all(np.array_equal(_bits(x), _bits(y)) for x, y in zip(a["coefficients"], b["coefficients"]))
        _check_against_services(ctx, srv, clusters, again)
    finally:
        for n in names:
            srv.erase_param(n)
