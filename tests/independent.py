"""Independent restatements used to pin the oracle from outside (TEST INFRASTRUCTURE ONLY).

Nothing here calls the oracle: numpy float32 restatements of PCL 1.7's plane distance test and
covariance, float64 eigen-solves, and scipy graph components for Euclidean clustering.

  select(x, y, z, c)          SampleConsensusModelPlane::selectWithinDistance / countWithinDistance
                              (sac_model_plane.hpp): |c . (p, 1)| < th with the 4-lane dot summed in
                              SSE2 predux order (c0 x + c2 z) + (c1 y + c3) (A3), float32, th as double
  covariance32(...)           computeMeanAndCovarianceMatrix (centroid.hpp): nine float accumulators,
                              sequential in inlier order (np.cumsum is sequential), accu *= 1/n (A9)
  plane_expectations(...)     eig64 / lsq64 planes and their tolerances (tools/make_independent_golden.py)
  cluster_labels(...)         cKDTree.query_pairs + connected_components, clusterize's size filter
"""
import numpy as np

TH = 0.007


def select(x, y, z, c, th=TH):
    c = np.asarray(c, np.float32)
    d = (c[0] * x + c[2] * z) + (c[1] * y + c[3])  # float32 throughout, no FMA in numpy
    return np.nonzero(np.abs(d).astype(np.float64) < th)[0].astype(np.int32)


def covariance32(x, y, z, idx):
    X, Y, Z = x[idx], y[idx], z[idx]
    acc = np.array([np.cumsum(v, dtype=np.float32)[-1] for v in (X * X, X * Y, X * Z, Y * Y, Y * Z, Z * Z, X, Y, Z)],
                   np.float32)
    acc = acc * (np.float32(1) / np.float32(len(idx)))
    mx, my, mz = acc[6], acc[7], acc[8]
    c = np.empty((3, 3), np.float32)
    c[0, 0], c[0, 1], c[0, 2] = acc[0] - mx * mx, acc[1] - mx * my, acc[2] - mx * mz
    c[1, 1], c[1, 2], c[2, 2] = acc[3] - my * my, acc[4] - my * mz, acc[5] - mz * mz
    c[1, 0], c[2, 0], c[2, 1] = c[0, 1], c[0, 2], c[1, 2]
    return c, np.array([mx, my, mz], np.float64)


def covariance64(x, y, z, idx):
    p = np.stack([x[idx], y[idx], z[idx]], 1).astype(np.float64)
    m = p.mean(0)
    return (p - m).T @ (p - m) / len(idx), m


def _plane(cov, centroid):
    w, v = np.linalg.eigh(np.asarray(cov, np.float64))
    n = v[:, 0]
    return np.r_[n, -n @ centroid], w


def plane_distance(a, b):
    """Max abs difference of two planes after scaling both to a unit normal and aligning signs."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    a, b = a / np.linalg.norm(a[:3]), b / np.linalg.norm(b[:3])
    return float(np.abs(a - np.sign(a[:3] @ b[:3]) * b).max())


def plane_expectations(x, y, z, best_coef):
    idx = select(x, y, z, best_coef)
    out = {"best_count": np.array([len(idx)])}
    if len(idx) < 4:  # optimizeModelCoefficients keeps the hypothesis
        c = np.asarray(best_coef, np.float64)
        out.update(eig64=c, lsq64=c, tol_eig=np.array([1e-6]), tol_lsq=np.array([1e-6]))
        return out
    c32, m32 = covariance32(x, y, z, idx)
    c64, m64 = covariance64(x, y, z, idx)
    eig, w = _plane(c32, m32)
    lsq, _ = _plane(c64, m64)
    gap = max(w[1] - w[0], 1e-30)
    scale = 1.0 + float(np.abs(m32).max())  # d = -n . centroid carries the normal's error
    # PCL's eigen33 clamps the smallest root to 0 (computeRoots2) when the scaled determinant is
    # below FLT_EPSILON or the float covariance came out indefinite; otherwise it solves the cubic
    s32 = c32.astype(np.float64) / max(float(np.abs(c32).max()), 1e-30)
    clamped = w[0] <= 0 or abs(np.linalg.det(s32)) < np.finfo(np.float32).eps
    tol_eig = (1e-5 + (2.0 * abs(w[0]) / gap if clamped else 0.0)) * scale
    dc = np.linalg.norm(c32.astype(np.float64) - c64, 2)
    tol_lsq = tol_eig + 2.0 * dc / gap * scale
    out.update(eig64=eig, lsq64=lsq, tol_eig=np.array([tol_eig]), tol_lsq=np.array([tol_lsq]))
    return out


def cluster_labels(x, y, z, radius=0.03, min_rate=0.01, max_rate=0.99):
    """Components of the radius graph, kept when round(n min_rate) <= size <= round(n max_rate),
    labelled 0.. by decreasing size; -1 for points in no kept cluster."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    from scipy.spatial import cKDTree
    p = np.stack([x, y, z], 1).astype(np.float64)
    n = len(p)
    pairs = cKDTree(p).query_pairs(radius, output_type="ndarray")
    g = coo_matrix((np.ones(len(pairs)), (pairs[:, 0], pairs[:, 1])), shape=(n, n))
    _, comp = connected_components(g, directed=False)
    sizes = np.bincount(comp)
    lo, hi = int(np.floor(n * min_rate + 0.5)), int(np.floor(n * max_rate + 0.5))
    kept = [c for c in np.argsort(-sizes, kind="stable") if lo <= sizes[c] <= hi]
    if len({int(sizes[c]) for c in kept}) != len(kept):
        raise ValueError("cluster sizes must be distinct for an order-independent fixture")
    lab = np.full(n, -1, np.int32)
    for rank, c in enumerate(kept):
        lab[comp == c] = rank
    return lab


def labels_from_clusters(n, clusters):
    lab = np.full(n, -1, np.int32)
    for rank, idx in enumerate(clusters):
        lab[np.asarray(idx)] = rank
    return lab
