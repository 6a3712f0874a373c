"""Hand-built scenes for the independent pins (tools/make_independent_golden.py, test_independent.py).

Deterministic numpy (PCG64) clouds in the body frame of the support service (horizontal axis
(0, 0, -1), so a support plane is z = const):

  q4_scene   table (horizontal), then a wall (vertical), then a shelf (horizontal) -- in that
             RANSAC order -- so createNewIdxMap runs with level -1 between two supports and the
             table's -2 tags are overwritten (quirk Q4, supports_segmentation_srv.cpp:145,332)
  q5_scene   a table whose first cloud point is its minimum-x (and minimum-y) point, plus object
             points just inside the true edge: getPointOnPlane's `else if` bbox (Q5, :192-200)
             never lets a running-max point lower xMin, so those objects fall outside
  cluster_cloud  separated blobs of distinct sizes plus sparse clutter, with no point pair within
             1e-6 m of the clustering radius (so `<` versus `<=` cannot matter)
"""
import math

import numpy as np


def _plane_patch(rng, n, x, y, z, noise=0.002):
    p = np.empty((n, 3), np.float64)
    p[:, 0] = rng.uniform(*x, n) if isinstance(x, tuple) else x + rng.normal(0, noise, n)
    p[:, 1] = rng.uniform(*y, n) if isinstance(y, tuple) else y + rng.normal(0, noise, n)
    p[:, 2] = rng.uniform(*z, n) if isinstance(z, tuple) else z + rng.normal(0, noise, n)
    return p


def _box(rng, n, lo, hi):
    return rng.uniform(lo, hi, (n, 3))


def q4_scene(seed=5):
    rng = np.random.default_rng(seed)
    table = _plane_patch(rng, 9000, (0.0, 1.0), (-0.5, 0.5), 0.70)
    wall = _plane_patch(rng, 6000, 1.30, (-0.6, 0.6), (0.0, 1.6))
    shelf = _plane_patch(rng, 3000, (0.2, 0.9), (-0.45, 0.45), 1.25)
    objs = np.concatenate([_box(rng, 500, (0.3, 0.72, 0.0), (0.4, 0.85, 0.1)) @ np.eye(3)[[0, 2, 1]],
                           _box(rng, 400, (0.6, -0.2, 0.72), (0.7, -0.1, 0.85))])
    pts = np.concatenate([table, wall, shelf, objs])
    pts = pts[rng.permutation(len(pts))].astype(np.float32)
    return pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()


def q5_scene(seed=5):
    rng = np.random.default_rng(seed)
    table = _plane_patch(rng, 6000, (0.0, 1.0), (-0.5, 0.5), 0.70, noise=0.001)
    # first table point: the minimum x and minimum y of the table
    table[0] = (-0.01, -0.51, 0.70)
    # objects just inside the true x / y edges (inside x > xmin + 0.02), away from the far edges
    near = _box(rng, 300, (0.015, 0.0, 0.73), (0.04, 0.3, 0.80))
    near_y = _box(rng, 300, (0.3, -0.485, 0.73), (0.6, -0.47, 0.80))
    mid = _box(rng, 500, (0.4, 0.0, 0.73), (0.55, 0.15, 0.85))
    pts = np.concatenate([table, near, near_y, mid]).astype(np.float32)
    return pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()


def cluster_cloud(seed, radius=0.03, n_blobs=7):
    """Blobs of distinct sizes (far apart) plus sparse clutter.  One point of every pair whose
    distance lies within 1e-6 of the radius is dropped (removing points changes no other distance)."""
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    parts = []
    sizes = rng.choice(np.arange(150, 1500, 37), n_blobs, replace=False)
    for b, s in enumerate(sizes):
        c = np.array([0.6 * (b % 4), 0.6 * (b // 4), 1.0 + 0.05 * b])
        parts.append(c + rng.normal(0, 0.025, (s, 3)))
    parts.append(rng.uniform((-0.3, -0.3, 0.5), (2.2, 1.4, 1.8), (400, 3)))
    pts = np.concatenate(parts)
    pts = pts[rng.permutation(len(pts))].astype(np.float32)
    t = cKDTree(pts.astype(np.float64))
    shell = t.query_pairs(radius + 1e-6) - t.query_pairs(radius - 1e-6)
    drop = np.zeros(len(pts), bool)
    for i, j in sorted(shell):
        if not (drop[i] or drop[j]):
            drop[j] = True
    pts = pts[~drop]
    return pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy()


def plain_bbox_on_support(x, y, z, support, idx_map, level, offset=(0.02, 0.02, 0.005), quirk=True):
    """getPointOnPlane (supports_segmentation_srv.cpp:187-238) restated in numpy.  quirk=True is the
    reference's `else if` running bbox (Q5); quirk=False an ordinary min/max bbox, for contrast."""
    sx, sy, sz = (support[:, k].astype(np.float64) for k in range(3))

    def bounds(v):
        if not quirk:
            return float(v.max()), float(v.min())
        prev = np.maximum.accumulate(np.concatenate([[-np.inf], v[:-1]]))
        lows = v[v <= prev]  # not a new running max: the `else if` branch may lower xMin
        return float(v.max()), float(lows.min()) if len(lows) else np.inf

    xmax, xmin = bounds(sx)
    ymax, ymin = bounds(sy)
    off = np.asarray(offset, np.float32).astype(np.float64)
    xmax -= off[0]
    xmin += off[0]
    ymax -= off[1]
    ymin += off[1]
    zmed = math.fsum(sz) / len(sz) + off[2]  # the sequential double sum is exact here (Q10)
    keep = (idx_map != level) & (x > xmin) & (x < xmax) & (z > zmed) & (y > ymin) & (y < ymax)
    return np.stack([x[keep], y[keep], z[keep]], 1)
