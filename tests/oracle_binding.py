"""ctypes binding of oracle/build/libpitt_oracle.so -- the CPU restatement of the reference's PCL
path.  TEST INFRASTRUCTURE ONLY (the checker), never the product."""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libpitt_oracle.so")

REDUCE_SSE2, REDUCE_HADD, REDUCE_SEQ = 0, 1, 2
TRIG_CR, TRIG_LIBM = 0, 1
DIV_EIGEN32, DIV_TRUE = 0, 1


class OrcSacParams(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32),
                ("probability", ctypes.c_double), ("seed", ctypes.c_uint32), ("optimize", ctypes.c_int32),
                ("reduce_order", ctypes.c_int32), ("trig_mode", ctypes.c_int32), ("div_mode", ctypes.c_int32)]


class OrcPlaneResult(ctypes.Structure):
    _fields_ = [("coefficients", ctypes.c_float * 4), ("n_coeff", ctypes.c_int32), ("hypotheses", ctypes.c_int32),
                ("n_inliers", ctypes.c_int64), ("best_hypothesis", ctypes.c_int32),
                ("rejected_samples", ctypes.c_int32), ("best_count", ctypes.c_int64),
                ("best_coefficients", ctypes.c_float * 4)]


class OrcSupportParams(ctypes.Structure):
    _fields_ = [("min_iterative_cloud_percentage", ctypes.c_float),
                ("min_iterative_plane_percentage", ctypes.c_float),
                ("horizontal_variance_threshold", ctypes.c_float), ("ransac_distance_threshold", ctypes.c_float),
                ("ransac_max_iterations", ctypes.c_int32), ("horizontal_axis", ctypes.c_float * 3),
                ("edge_remove_offset", ctypes.c_float * 3), ("reduce_order", ctypes.c_int32),
                ("trig_mode", ctypes.c_int32), ("div_mode", ctypes.c_int32)]


_fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
_ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))  # noqa: E731


def load():
    if not os.path.exists(ORACLE_SO):
        raise FileNotFoundError(f"{ORACLE_SO} missing: run `make -C oracle`")
    return ctypes.CDLL(ORACLE_SO)


O = load()
O.orc_count_within.restype = ctypes.c_int64
O.orc_select_within.restype = ctypes.c_int64
O.orc_find_supports.restype = ctypes.c_void_p
O.orc_support_count.argtypes = [ctypes.c_void_p]
O.orc_support_get.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p]
O.orc_support_cloud.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p]
O.orc_support_free.argtypes = [ctypes.c_void_p]
O.orc_euclidean_clusters.restype = ctypes.c_void_p
O.orc_euclidean_clusters.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int32]
O.orc_cluster_count.argtypes = [ctypes.c_void_p]
O.orc_cluster_size.argtypes = [ctypes.c_void_p, ctypes.c_int32]
O.orc_cluster_size.restype = ctypes.c_int64
O.orc_cluster_get.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
O.orc_cluster_free.argtypes = [ctypes.c_void_p]


def mt19937(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    O.orc_mt19937(ctypes.c_uint32(seed), ctypes.c_int64(n), out.ctypes.data_as(ctypes.c_void_p))
    return out


def sampler_table(n: int, attempts: int, seed: int = 12345) -> np.ndarray:
    out = np.zeros(3 * attempts, np.int32)
    O.orc_sampler_table(ctypes.c_int64(n), ctypes.c_uint32(seed), ctypes.c_int64(attempts), _ip(out))
    return out.reshape(attempts, 3)


def plane_coefficients(p0, p1, p2, reduce_order=REDUCE_SSE2, div_mode=DIV_EIGEN32):
    a, b, c = (np.asarray(v, np.float32) for v in (p0, p1, p2))
    out = np.zeros(4, np.float32)
    ok = O.orc_plane_coefficients(_fp(a), _fp(b), _fp(c), reduce_order, div_mode, _fp(out))
    return bool(ok), out


def eigen33(cov, trig_mode=TRIG_CR):
    c = np.ascontiguousarray(cov, np.float32).reshape(9)
    ev = ctypes.c_float()
    vec = np.zeros(3, np.float32)
    O.orc_eigen33(_fp(c), trig_mode, 0, ctypes.byref(ev), _fp(vec))
    return ev.value, vec


@dataclass
class OracleSegment:
    inliers: np.ndarray
    coefficients: np.ndarray
    hypotheses: int
    best_hypothesis: int
    best_count: int
    rejected_samples: int
    best_coefficients: np.ndarray
    hyp_counts: np.ndarray


def plane_segment(x, y, z, threshold=0.007, max_iterations=1000, probability=0.99, seed=12345, optimize=True,
                  reduce_order=REDUCE_SSE2, trig_mode=TRIG_CR, div_mode=DIV_EIGEN32) -> OracleSegment:
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    p = OrcSacParams(threshold, max_iterations, probability, seed, 1 if optimize else 0, reduce_order, trig_mode,
                     div_mode)
    r = OrcPlaneResult()
    inl = np.zeros(max(n, 1), np.int32)
    hc = np.zeros(max(max_iterations + 1, 1), np.int32)
    O.orc_plane_segment(_fp(x), _fp(y), _fp(z), ctypes.c_int64(n), ctypes.byref(p), _ip(inl), ctypes.byref(r),
                        _ip(hc))
    return OracleSegment(inl[:r.n_inliers].copy(), np.array(list(r.coefficients)[:r.n_coeff], np.float32),
                         r.hypotheses, r.best_hypothesis, r.best_count, r.rejected_samples,
                         np.array(list(r.best_coefficients), np.float32), hc[:r.hypotheses].copy())


def count_within(x, y, z, coeff, threshold, reduce_order=REDUCE_SSE2) -> int:
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    c = np.asarray(coeff, np.float32)
    return int(O.orc_count_within(_fp(x), _fp(y), _fp(z), ctypes.c_int64(len(x)), _fp(c),
                                  ctypes.c_double(threshold), reduce_order))


def find_supports(x, y, z, reduce_order=REDUCE_SSE2, trig_mode=TRIG_CR, div_mode=DIV_EIGEN32, **kw):
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    p = OrcSupportParams(kw.get("min_iterative_cloud_percentage", 0.03), kw.get("min_iterative_plane_percentage", 0.03),
                         kw.get("horizontal_variance_threshold", 0.09), kw.get("ransac_distance_threshold", 0.02),
                         kw.get("ransac_max_iterations", 10),
                         (ctypes.c_float * 3)(*kw.get("horizontal_axis", (0.0, 0.0, -1.0))),
                         (ctypes.c_float * 3)(*kw.get("edge_remove_offset", (0.02, 0.02, 0.005))),
                         reduce_order, trig_mode, div_mode)
    h = O.orc_find_supports(_fp(x), _fp(y), _fp(z), ctypes.c_int64(n), ctypes.byref(p))
    out = []
    try:
        for s in range(O.orc_support_count(h)):
            idx = np.zeros(max(n, 1), np.int32)
            co = np.zeros(4, np.float32)
            a, b = ctypes.c_int64(), ctypes.c_int64()
            O.orc_support_get(h, s, idx.ctypes.data_as(ctypes.c_void_p), co.ctypes.data_as(ctypes.c_void_p),
                              ctypes.byref(a), ctypes.byref(b))
            clouds = []
            for which, m in ((0, a.value), (1, b.value)):
                cx, cy, cz = (np.zeros(max(m, 1), np.float32) for _ in range(3))
                O.orc_support_cloud(h, s, which, cx.ctypes.data_as(ctypes.c_void_p),
                                    cy.ctypes.data_as(ctypes.c_void_p), cz.ctypes.data_as(ctypes.c_void_p))
                clouds.append(np.stack([cx[:m], cy[:m], cz[:m]], 1))
            out.append(dict(idx_map=idx[:n].copy(), coefficients=co, support_cloud=clouds[0],
                            on_support_cloud=clouds[1]))
    finally:
        O.orc_support_free(h)
    return out


def euclidean_clusters(x, y, z, tolerance=0.03, min_rate=0.01, max_rate=0.99, min_input_size=30):
    """Handler-level (clusterize): sizes from rates, centroid = sum / (n + 1)."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    h = O.orc_euclidean_clusters(x.ctypes.data_as(ctypes.c_void_p), y.ctypes.data_as(ctypes.c_void_p),
                                 z.ctypes.data_as(ctypes.c_void_p), len(x), tolerance, min_rate, max_rate,
                                 min_input_size)
    out = []
    try:
        for c in range(O.orc_cluster_count(h)):
            m = O.orc_cluster_size(h, c)
            idx = np.zeros(max(m, 1), np.int32)
            ce = np.zeros(3, np.float32)
            O.orc_cluster_get(h, c, idx.ctypes.data_as(ctypes.c_void_p), ce.ctypes.data_as(ctypes.c_void_p))
            out.append(dict(inliers=idx[:m].copy(), centroid=ce))
    finally:
        O.orc_cluster_free(h)
    return out


O.orc_service_float_param.restype = ctypes.c_float
O.orc_service_float_param.argtypes = [ctypes.c_float, ctypes.c_float]
O.orc_deep_filter.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_float] + [ctypes.c_void_p] * 8
O.orc_transform_cloud.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32] + \
    [ctypes.c_void_p] * 3


def service_float_param(value: float, default: float) -> float:
    """srv_manager.h:163-167 getServiceFloatParameter."""
    return float(O.orc_service_float_param(value, default))


def deep_filter(x, y, z, threshold: float):
    """deep_filter_srv.cpp:37-44 at an already-resolved float threshold: (closer Nx3, further Nx3)."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    c = np.empty((3, max(n, 1)), np.float32)
    f = np.empty((3, max(n, 1)), np.float32)
    nc, nf = ctypes.c_int64(), ctypes.c_int64()
    O.orc_deep_filter(_fp(x), _fp(y), _fp(z), n, threshold, _fp(c[0]), _fp(c[1]), _fp(c[2]), ctypes.byref(nc),
                      _fp(f[0]), _fp(f[1]), _fp(f[2]), ctypes.byref(nf))
    return c[:, :nc.value].T.copy(), f[:, :nf.value].T.copy()


def transform_cloud(x, y, z, matrix, dense: bool = True):
    """pcl::transformPointCloud(cloud, out, Matrix4f) restated (obj_segmentation.cpp:248): Nx3."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    m = np.ascontiguousarray(np.asarray(matrix, np.float32).reshape(16))
    n = len(x)
    o = np.empty((3, max(n, 1)), np.float32)
    O.orc_transform_cloud(_fp(x), _fp(y), _fp(z), n, _fp(m), 1 if dense else 0, _fp(o[0]), _fp(o[1]), _fp(o[2]))
    return o[:, :n].T.copy()


O.orc_unpack_pointcloud2.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 3


def unpack_pointcloud2(data: np.ndarray, width, height, point_step, row_step, offsets=(0, 4, 8)):
    """fromROSMsg XYZ restated (pc_manager.cpp:94-104): Nx3 float32, row-major."""
    data = np.ascontiguousarray(data, np.uint8)
    n = width * height
    o = np.empty((3, max(n, 1)), np.float32)
    O.orc_unpack_pointcloud2(data.ctypes.data, width, height, point_step, row_step, *offsets,
                             _fp(o[0]), _fp(o[1]), _fp(o[2]))
    return o[:, :n].T.copy()


O.orc_voxel_grid.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                     ctypes.c_int32] + [ctypes.c_void_p] * 4
SORT_PCL, SORT_STABLE = 0, 1


def voxel_grid(x, y, z, leaf=(0.01, 0.01, 0.01), sort_mode=SORT_PCL):
    """VoxelGrid<PointXYZ>::applyFilter restated (pc_manager.cpp:61-67): (Nx3 centroids, overflow flag)."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    o = np.empty((3, max(n, 1)), np.float32)
    m = ctypes.c_int64()
    rc = O.orc_voxel_grid(_fp(x), _fp(y), _fp(z), n, *leaf, sort_mode, _fp(o[0]), _fp(o[1]), _fp(o[2]),
                          ctypes.byref(m))
    return o[:, :m.value].T.copy(), rc


O.orc_normal_estimation.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int32] + [ctypes.c_void_p] * 7


def normal_estimation(x, y, z, k=50, viewpoint=(0.0, 0.0, 0.0), neighbours=False):
    """NormalEstimation<PointXYZ, Normal>, KdTree, setKSearch(k) restated (pc_manager.cpp:68-78):
    (normals Nx3, curvature N) [, (neighbour lists N x k, counts N)]."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    vp = np.asarray(viewpoint, np.float32)
    o = np.empty((4, max(n, 1)), np.float32)
    nn = np.full((max(n, 1), k), -1, np.int32) if neighbours else None
    cnt = np.zeros(max(n, 1), np.int32)
    O.orc_normal_estimation(_fp(x), _fp(y), _fp(z), n, k, _fp(vp), _fp(o[0]), _fp(o[1]), _fp(o[2]), _fp(o[3]),
                            None if nn is None else _ip(nn), _ip(cnt))
    out = (o[:3, :n].T.copy(), o[3, :n].copy())
    return out + ((nn[:n], cnt[:n]),) if neighbours else out


O.orc_std_sort_pairs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
O.orc_introsort_pairs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]


def sort_pairs(keys, vals, depth_limit=None):
    """std::sort of (key, value) pairs by key (this image's libstdc++), or, with depth_limit, the
    oracle's restatement of its introsort (-1: the library's limit)."""
    k = np.ascontiguousarray(keys, np.uint32).copy()
    v = np.ascontiguousarray(vals, np.uint32).copy()
    if depth_limit is None:
        O.orc_std_sort_pairs(k.ctypes.data, v.ctypes.data, len(k))
    else:
        O.orc_introsort_pairs(k.ctypes.data, v.ctypes.data, len(k), depth_limit)
    return k, v


O.orc_axis_height.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32] + \
    [ctypes.c_void_p] * 7
O.orc_axis_height.restype = None


def axis_height(x, y, z, coef, mode=0):
    """The cylinder (mode 0) / cone (mode 1) height post-processing restated
    (cylinder_segmentation_srv.cpp:129-189): (height, idx1, idx2, centroid[3], projected Nx3)."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    c = np.ascontiguousarray(np.asarray(coef, np.float32)[:6])
    p = np.empty((3, max(n, 1)), np.float32)
    h = ctypes.c_float()
    i1, i2 = ctypes.c_int32(), ctypes.c_int32()
    cen = np.zeros(3, np.float32)
    O.orc_axis_height(_fp(x), _fp(y), _fp(z), n, _fp(c), mode, _fp(p[0]), _fp(p[1]), _fp(p[2]), ctypes.byref(h),
                      ctypes.byref(i1), ctypes.byref(i2), _fp(cen))
    return h.value, i1.value, i2.value, cen, p[:, :n].T.copy()


class SphereParams(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32), ("optimize", ctypes.c_int32),
                ("probability", ctypes.c_double), ("radius_min", ctypes.c_double), ("radius_max", ctypes.c_double),
                ("seed", ctypes.c_uint32), ("pad", ctypes.c_int32)]


def sphere_params(threshold=0.007, max_iterations=1000, optimize=True, radius_min=0.005, radius_max=0.5,
                  probability=0.99, seed=12345):
    """sphere_segmentation_srv.cpp:19-27 defaults (distance 0.007, 1000 iterations, radius 0.005-0.5)."""
    return SphereParams(threshold, max_iterations, int(optimize), probability, radius_min, radius_max, seed, 0)


O.orc_sphere_segment.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.POINTER(SphereParams)] + \
    [ctypes.c_void_p] * 6 + [ctypes.c_int32, ctypes.c_void_p]
O.orc_sphere_from4.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def sphere_from4(p4):
    c = np.zeros(4, np.float32)
    ok = O.orc_sphere_from4(_fp(np.ascontiguousarray(p4, np.float32)), _fp(c))
    return bool(ok), c


def sphere_segment(x, y, z, params=None, counts_cap=20000):
    """The sphere service's seg.segment restated: dict(ok, inliers, coef, best, hypotheses, counts)."""
    x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
    n = len(x)
    p = params or sphere_params()
    inl = np.empty(max(n, 1), np.int32)
    ni = ctypes.c_int64()
    coef, best = np.zeros(4, np.float32), np.zeros(4, np.float32)
    hyp, nc = ctypes.c_int32(), ctypes.c_int32()
    cnt = np.zeros(counts_cap, np.int32)
    ok = O.orc_sphere_segment(_fp(x), _fp(y), _fp(z), n, ctypes.byref(p), _ip(inl), ctypes.byref(ni), _fp(coef),
                              _fp(best), ctypes.byref(hyp), _ip(cnt), counts_cap, ctypes.byref(nc))
    return {"ok": bool(ok), "inliers": inl[:ni.value].copy(), "coef": coef, "best": best, "hypotheses": hyp.value,
            "counts": cnt[:min(nc.value, counts_cap)].copy()}


class CylinderParams(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32), ("optimize", ctypes.c_int32),
                ("probability", ctypes.c_double), ("radius_min", ctypes.c_double), ("radius_max", ctypes.c_double),
                ("normal_distance_weight", ctypes.c_double), ("seed", ctypes.c_uint32), ("eigen33", ctypes.c_int32)]


def cylinder_params(threshold=0.008, max_iterations=1000, optimize=True, radius_min=0.005, radius_max=0.5,
                    normal_distance_weight=0.001, probability=0.99, seed=12345, eigen33=0):
    """cylinder_segmentation_srv.cpp:23-30 defaults."""
    return CylinderParams(threshold, max_iterations, int(optimize), probability, radius_min, radius_max,
                          normal_distance_weight, seed, eigen33)


O.orc_cylinder_segment.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.POINTER(CylinderParams)] + \
    [ctypes.c_void_p] * 5


def cylinder_segment(xyz, nrm, params=None):
    """The cylinder service's seg.segment restated: dict(ok, inliers, coef[7], best[7], hypotheses)."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    nrm = np.ascontiguousarray(nrm, np.float32)
    cols = [np.ascontiguousarray(a[:, k]) for a in (xyz, nrm) for k in range(3)]
    n = len(xyz)
    p = params or cylinder_params()
    inl = np.empty(max(n, 1), np.int32)
    ni = ctypes.c_int64()
    coef, best = np.zeros(7, np.float32), np.zeros(7, np.float32)
    hyp = ctypes.c_int32()
    ok = O.orc_cylinder_segment(*(_fp(c) for c in cols), n, ctypes.byref(p), _ip(inl), ctypes.byref(ni), _fp(coef),
                                _fp(best), ctypes.byref(hyp))
    return {"ok": bool(ok), "inliers": inl[:ni.value].copy(), "coef": coef, "best": best, "hypotheses": hyp.value}


class ConeParams(ctypes.Structure):
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32), ("optimize", ctypes.c_int32),
                ("probability", ctypes.c_double), ("normal_distance_weight", ctypes.c_double),
                ("min_angle", ctypes.c_double), ("max_angle", ctypes.c_double), ("eps_angle", ctypes.c_double),
                ("axis", ctypes.c_float * 3), ("eigen33", ctypes.c_int32), ("seed", ctypes.c_uint32),
                ("pad", ctypes.c_int32)]


def cone_params(threshold=0.0055, max_iterations=1000, optimize=True, normal_distance_weight=0.0006,
                min_angle_deg=10.0, max_angle_deg=170.0, eps_angle=0.4, axis=(0.0, 0.0, 0.0), eigen33=0,
                probability=0.99, seed=12345):
    """cone_segmentation_srv.cpp:24-31 defaults; the angles converted as :124 does (deg / 180 * M_PI)."""
    return ConeParams(threshold, max_iterations, int(optimize), probability, normal_distance_weight,
                      min_angle_deg / 180.0 * np.pi, max_angle_deg / 180.0 * np.pi, eps_angle,
                      (ctypes.c_float * 3)(*axis), eigen33, seed, 0)


O.orc_cone_segment.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.POINTER(ConeParams)] + \
    [ctypes.c_void_p] * 5
O.orc_cone_from3.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]


def cone_from3(p3, n3, min_angle=-np.finfo(np.float64).max, max_angle=np.finfo(np.float64).max):
    c = np.zeros(7, np.float32)
    ok = O.orc_cone_from3(_fp(np.ascontiguousarray(p3, np.float32)), _fp(np.ascontiguousarray(n3, np.float32)),
                          min_angle, max_angle, _fp(c))
    return bool(ok), c


def cone_segment(xyz, nrm, params=None):
    """The cone service's seg.segment restated: dict(ok, inliers, coef[7], best[7], hypotheses)."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    nrm = np.ascontiguousarray(nrm, np.float32)
    cols = [np.ascontiguousarray(a[:, k]) for a in (xyz, nrm) for k in range(3)]
    n = len(xyz)
    p = params or cone_params()
    inl = np.empty(max(n, 1), np.int32)
    ni = ctypes.c_int64()
    coef, best = np.zeros(7, np.float32), np.zeros(7, np.float32)
    hyp = ctypes.c_int32()
    ok = O.orc_cone_segment(*(_fp(c) for c in cols), n, ctypes.byref(p), _ip(inl), ctypes.byref(ni), _fp(coef),
                            _fp(best), ctypes.byref(hyp))
    return {"ok": bool(ok), "inliers": inl[:ni.value].copy(), "coef": coef, "best": best, "hypotheses": hyp.value}


# ---- primitive refinement: PCL's float Eigen LM (default) vs the least-squares optimum -------------
LM_PCL, LM_OPTIMUM = 0, 1
MODEL_SPHERE, MODEL_CYLINDER, MODEL_CONE = 0, 1, 2
O.orc_set_lm_mode.argtypes = [ctypes.c_int32]
O.orc_get_lm_mode.restype = ctypes.c_int32
O.orc_lm_refine.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]


def set_lm_mode(mode):
    O.orc_set_lm_mode(mode)


def get_lm_mode():
    return O.orc_get_lm_mode()


def lm_refine(model, xyz, inliers, coef, mode=LM_PCL):
    """optimizeModelCoefficients alone (orc_lm_refine): returns (coefficients, Eigen status, nfev)."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    cols = [np.ascontiguousarray(xyz[:, k]) for k in range(3)]
    inl = np.ascontiguousarray(inliers, np.int32)
    cin = np.ascontiguousarray(coef, np.float32)
    out = np.zeros(len(cin), np.float32)
    st, nf = ctypes.c_int32(), ctypes.c_int32()
    O.orc_lm_refine(model, *(_fp(c) for c in cols), _ip(inl), len(inl), _fp(cin), _fp(out), mode, ctypes.byref(st),
                    ctypes.byref(nf))
    return out, st.value, nf.value


O.orc_elm_fit64.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]


def elm_fit64(model, xyz, inliers, coef):
    """The Eigen LM restatement instantiated in double (orc_elm_fit64): (x, status, njac, trials)."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    cols = [np.ascontiguousarray(xyz[:, k]) for k in range(3)]
    inl = np.ascontiguousarray(inliers, np.int32)
    cin = np.ascontiguousarray(coef, np.float64)
    out = np.zeros(len(cin), np.float64)
    st, nj, tr = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    O.orc_elm_fit64(model, *(c.ctypes.data for c in cols), inl.ctypes.data, len(inl), cin.ctypes.data,
                    out.ctypes.data, ctypes.byref(st), ctypes.byref(nj), ctypes.byref(tr))
    return out, st.value, nj.value, tr.value


class lm_mode:
    """with orc.lm_mode(orc.LM_OPTIMUM): ... -- the oracle's refinement mode inside the block."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.saved = get_lm_mode()
        set_lm_mode(self.mode)
        return self

    def __exit__(self, *exc):
        set_lm_mode(self.saved)
