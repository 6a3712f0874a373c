"""VoxelGrid<PointXYZ> downsampling (pc_manager.cpp:55-67, leaf 0.01 m; obj_segmentation.cpp:238).

CPU: the oracle's restatement of PCL 1.7 applyFilter against analytic cases and an independent numpy
restatement of the leaf indices (integer work, exact) and of the stable-order centroids.
GPU: pitt_voxel_grid against the oracle -- in PCL order (the default; libstdc++'s introsort permutation
reproduced on the device) bit-exact against the oracle's std::sort; in stable order bit-exact against
the stable restatement and within the float reordering bound of PCL's centroids.  pitt_sort_pairs
against std::sort and, with a forced depth limit, against the oracle's restatement (heapsort path).
"""
import numpy as np
import pytest

import oracle_binding as orc

U = 2.0 ** -24  # float unit roundoff


def leaf_keys(x, y, z, leaf=(0.01, 0.01, 0.01)):
    """Independent numpy restatement of applyFilter's leaf index (float32 arithmetic, int32 wrap):
    returns (finite point indices, idx) in input order."""
    x, y, z = (np.asarray(a, np.float32) for a in (x, y, z))
    fin = np.nonzero(np.isfinite(x) & np.isfinite(y) & np.isfinite(z))[0]
    if len(fin) == 0:
        return fin, np.zeros(0, np.int64)
    inv = np.float32(1) / np.asarray(leaf, np.float32)
    c = [a[fin] for a in (x, y, z)]
    mn = np.array([v.min() for v in c], np.float32)
    mx = np.array([v.max() for v in c], np.float32)
    min_b = np.floor(mn * inv).astype(np.int64)
    max_b = np.floor(mx * inv).astype(np.int64)
    div = max_b - min_b + 1
    mul = np.array([1, div[0], div[0] * div[1]], np.int64)
    ijk = [(np.floor(c[k] * inv[k]) - np.float32(min_b[k])).astype(np.int64) for k in range(3)]
    return fin, ijk[0] * mul[0] + ijk[1] * mul[1] + ijk[2] * mul[2]


def stable_centroids(x, y, z, leaf=(0.01, 0.01, 0.01)):
    """Leaves in ascending idx; each leaf's points summed in ascending point order in float32, then
    times 1/n (Eigen 3.2 `/=`).  Also returns per-leaf counts and sum of |p| (for the order bound)."""
    fin, idx = leaf_keys(x, y, z, leaf)
    order = np.lexsort((fin, idx))
    fin, idx = fin[order], idx[order]
    starts = np.r_[0, np.nonzero(np.diff(idx))[0] + 1] if len(idx) else np.zeros(0, np.int64)
    ends = np.r_[starts[1:], len(idx)]
    pts = np.stack([x, y, z], 1).astype(np.float32)
    out = np.empty((len(starts), 3), np.float32)
    mag = np.empty((len(starts), 3), np.float64)
    for v, (a, b) in enumerate(zip(starts, ends)):
        p = pts[fin[a:b]]
        out[v] = np.cumsum(p, axis=0, dtype=np.float32)[-1] * (np.float32(1) / np.float32(b - a))
        mag[v] = np.abs(p.astype(np.float64)).sum(0)
    return out, ends - starts, mag


def reorder_bound(counts, mag):
    """|difference| of a float sum of n terms evaluated in two orders, after the 1/n multiply."""
    n = counts[:, None].astype(np.float64)
    return 2.0 * (n - 1) * U * mag / n + 4 * U * mag / n + 1e-30


def frame(scene, seed, w=640, h=480):
    from pitt_object_table_segmentation_amd import api
    return api.synth_frame(scene, seed, w, h)


# ---- oracle ----------------------------------------------------------------------------------------
def test_oracle_voxel_analytic():
    # three leaves: (0,0,0) gets 3 points, (1,0,0) 1 point, (0,2,1) 2 points; one NaN point dropped
    pts = np.array([[0.001, 0.002, 0.003], [0.012, 0.001, 0.004], [0.004, 0.005, 0.006], [0.002, 0.021, 0.013],
                    [np.nan, 0.0, 0.0], [0.009, 0.009, 0.009], [0.008, 0.028, 0.019]], np.float32)
    out, flag = orc.voxel_grid(*pts.T)
    assert flag == 0 and out.shape == (3, 3)
    first = pts[[0, 2, 5]]
    want0 = np.cumsum(first, 0, dtype=np.float32)[-1] * (np.float32(1) / np.float32(3))
    assert np.array_equal(out[0], want0)
    assert np.array_equal(out[1], pts[1])
    assert np.array_equal(out[2], np.cumsum(pts[[3, 6]], 0, dtype=np.float32)[-1] * np.float32(0.5))


def test_oracle_voxel_overflow_copies_input():
    pts = np.array([[0, 0, 0], [100, 100, 100], [np.inf, 0, 0]], np.float32)
    out, flag = orc.voxel_grid(*pts.T, leaf=(1e-4, 1e-4, 1e-4))
    assert flag == 1 and out.shape == pts.shape
    assert np.array_equal(out[:2], pts[:2]) and np.isinf(out[2, 0])


@pytest.mark.parametrize("n,keys", [(17, 3), (5000, 50), (300000, 90000), (50000, 2)])
def test_oracle_introsort_restatement_is_the_library(n, keys):
    """The oracle's introsort restatement (used to check the device's heapsort path) equals this
    image's std::sort, and at depth 0 its heapsort equals std::partial_sort."""
    import ctypes
    rng = np.random.default_rng(n)
    k = rng.integers(0, keys, n).astype(np.uint32)
    v = np.arange(n, dtype=np.uint32)
    a, b = orc.sort_pairs(k, v), orc.sort_pairs(k, v, -1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    orc.O.orc_partial_sort_pairs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    hk, hv = k.copy(), v.copy()
    orc.O.orc_partial_sort_pairs(hk.ctypes.data, hv.ctypes.data, n)
    c = orc.sort_pairs(k, v, 0)
    assert np.array_equal(hk, c[0]) and np.array_equal(hv, c[1])


def test_oracle_voxel_empty_and_all_nan():
    out, flag = orc.voxel_grid(np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.float32))
    assert flag == 0 and out.shape == (0, 3)
    nan = np.full(10, np.nan, np.float32)
    out, flag = orc.voxel_grid(nan, nan, nan)
    assert out.shape == (0, 3)


@pytest.mark.parametrize("scene,seed", [(0, 1000), (2, 1001)])
def test_oracle_voxel_vs_numpy(scene, seed):
    x, y, z = frame(scene, seed)
    want, counts, mag = stable_centroids(x, y, z)
    stable, _ = orc.voxel_grid(x, y, z, sort_mode=orc.SORT_STABLE)
    pcl, _ = orc.voxel_grid(x, y, z)
    assert np.array_equal(stable, want)  # integer leaf work + the stable float sums, bit for bit
    assert pcl.shape == want.shape
    assert np.all(np.abs(pcl.astype(np.float64) - want) <= reorder_bound(counts, mag))
    # the two orders really differ somewhere (PCL's introsort moves equal keys)
    assert (pcl != stable).any()


# ---- HIP path --------------------------------------------------------------------------------------
def _gpu_voxel(ctx, x, y, z, leaf=(0.01, 0.01, 0.01), order=0):
    import torch
    t = [torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda() for a in (x, y, z)]
    (ox, oy, oz), flags = ctx.voxel_grid(*t, leaf=leaf, order=order)
    return np.stack([ox.cpu().numpy(), oy.cpu().numpy(), oz.cpu().numpy()], 1), flags


@pytest.mark.gpu
@pytest.mark.parametrize("scene,seed", [(0, 1000), (1, 1003), (2, 1001)])
def test_hip_voxel_frames(ctx, scene, seed):
    """PCL order (default): bit-exact against the oracle's std::sort; stable order: bit-exact against
    the stable restatement and within the reordering bound of PCL's centroids."""
    x, y, z = frame(scene, seed)
    got, flags = _gpu_voxel(ctx, x, y, z)
    pcl, _ = orc.voxel_grid(x, y, z)
    assert flags == 0 and np.array_equal(got, pcl)
    got_s, _ = _gpu_voxel(ctx, x, y, z, order=1)
    stable, _ = orc.voxel_grid(x, y, z, sort_mode=orc.SORT_STABLE)
    _, counts, mag = stable_centroids(x, y, z)
    assert np.array_equal(got_s, stable)
    assert np.all(np.abs(got_s.astype(np.float64) - pcl) <= reorder_bound(counts, mag))


@pytest.mark.gpu
def test_hip_voxel_fused_1p2m(ctx):
    from pitt_object_table_segmentation_amd import api
    x, y, z = api.synth_fused(1000, 4)
    got, _ = _gpu_voxel(ctx, x, y, z)
    pcl, _ = orc.voxel_grid(x, y, z)
    assert np.array_equal(got, pcl)


@pytest.mark.gpu
@pytest.mark.parametrize("n,keys,depth", [(17, 3, -1), (1000, 7, -1), (300000, 90000, -1), (50000, 2, -1),
                                          (20000, 50, 0), (20000, 50, 2), (5000, 5, 3), (4096, 4096, 1),
                                          (2048, 100, -1), (2049, 100, -1), (100000, 3, -1), (200000, 1000, 9),
                                          (1000000, 500000, -1), (1000000, 100, 14),
                                          (26624, 1000, 0), (26625, 7, 0), (60000, 60000, 1),
                                          (8192, 300, -1), (8193, 300, -1), (8192, 50, 3), (8000, 8000, -1),
                                          (30000, 40, -1), (65536, 500, -1), (65537, 900, -1), (65536, 30, 4),
                                          (70000, 3, 5)])
def test_hip_sort_pairs_is_std_sort(ctx, n, keys, depth):
    """pitt_sort_pairs reproduces std::sort's permutation of equal keys (the library's own sort at
    the default depth; the oracle's restatement, validated against the library, with a forced
    small depth limit that reaches the heapsort fallback)."""
    import torch
    rng = np.random.default_rng(n + keys)
    k = rng.integers(0, keys, n).astype(np.uint32)
    v = rng.permutation(n).astype(np.uint32)
    want = orc.sort_pairs(k, v) if depth < 0 else orc.sort_pairs(k, v, depth)
    tk = torch.from_numpy(k.view(np.int32)).cuda()
    tv = torch.from_numpy(v.view(np.int32)).cuda()
    ctx.sort_pairs(tk, tv, depth)
    assert np.array_equal(tk.cpu().numpy().view(np.uint32), want[0])
    assert np.array_equal(tv.cpu().numpy().view(np.uint32), want[1])


@pytest.mark.gpu
def test_hip_voxel_edges(ctx):
    rng = np.random.default_rng(3)
    p = rng.uniform(-0.3, 0.3, (5000, 3)).astype(np.float32)
    p[::7, 1] = np.nan
    p[3, 2] = np.inf
    for leaf in [(0.01, 0.01, 0.01), (0.05, 0.02, 0.013), (1.0, 1.0, 1.0)]:
        got, flags = _gpu_voxel(ctx, *p.T, leaf=leaf)
        want, _ = orc.voxel_grid(*p.T, leaf=leaf)
        assert flags == 0 and np.array_equal(got, want), leaf
    # overflow: the input comes back unchanged (non-finite points included)
    big = np.array([[0, 0, 0], [100, 100, 100], [np.nan, 1, 1]], np.float32)
    got, flags = _gpu_voxel(ctx, *big.T, leaf=(1e-4, 1e-4, 1e-4))
    assert flags == 1 and got.shape == (3, 3) and np.array_equal(got[:2], big[:2]) and np.isnan(got[2, 0])
    # empty, single point, all NaN
    assert _gpu_voxel(ctx, *np.zeros((0, 3), np.float32).T)[0].shape == (0, 3)
    one = np.array([[0.1234, -0.5, 2.0]], np.float32)
    assert np.array_equal(_gpu_voxel(ctx, *one.T)[0], one)
    assert _gpu_voxel(ctx, *np.full((9, 3), np.nan, np.float32).T)[0].shape == (0, 3)
