"""ctypes binding of the C ABI in include/pitt_seg.h (libpitt_seg.so, built in-tree).

The library is the product: every segmentation call in this package goes through it.  If the
shared object is missing or cannot be loaded, import fails loudly -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


# PITT_LIB_PATH: an alternative build of the same library (A/B experiments, tools/ only)
LIB_PATH = os.environ.get("PITT_LIB_PATH") or os.path.join(_HERE, "libpitt_seg.so")

PITT_OK = 0
PITT_NO_MODEL = 1
PITT_E_INVALID = -1
PITT_E_HIP = -2
PITT_E_NOMEM = -3
PITT_E_SAMPLER = -4
PITT_E_NODEVICE = -5
PITT_TILE_POINTS = 2048
PITT_BUILD_AB_VARIANTS = 1
PITT_FLAG_K_NEAR_INTEGER = 1
PITT_VOXEL_OVERFLOW_COPY = 1
PITT_VOXEL_ORDER_PCL, PITT_VOXEL_ORDER_STABLE = 0, 1
PITT_AXIS_CYLINDER, PITT_AXIS_CONE = 0, 1

REDUCE_SSE2, REDUCE_HADD, REDUCE_SEQ = 0, 1, 2
DIV_EIGEN32, DIV_TRUE = 0, 1
COV_EXACT, COV_FAST = 0, 1
SCENE_TABLE, SCENE_CLUTTER, SCENE_TABLE_NAN = 0, 1, 2


class SacParams(ctypes.Structure):
    _fields_ = [
        ("threshold", ctypes.c_double),
        ("max_iterations", ctypes.c_int32),
        ("probability", ctypes.c_double),
        ("seed", ctypes.c_uint32),
        ("optimize", ctypes.c_int32),
        ("reduce_order", ctypes.c_int32),
        ("div_mode", ctypes.c_int32),
        ("sampler_slack", ctypes.c_int32),
        ("cov_mode", ctypes.c_int32),
        ("pad", ctypes.c_int32),
    ]


class PlaneResult(ctypes.Structure):
    _fields_ = [
        ("coefficients", ctypes.c_float * 4),
        ("n_coeff", ctypes.c_int32),
        ("status", ctypes.c_int32),
        ("n_inliers", ctypes.c_int64),
        ("hypotheses", ctypes.c_int32),
        ("best_hypothesis", ctypes.c_int32),
        ("best_count", ctypes.c_int64),
        ("rejected_samples", ctypes.c_int32),
        ("flags", ctypes.c_int32),
    ]


class Frames(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("z", ctypes.c_void_p),
        ("offsets", ctypes.POINTER(ctypes.c_int64)),
        ("counts", ctypes.POINTER(ctypes.c_int64)),
        ("n_frames", ctypes.c_int32),
        ("capacity", ctypes.c_int64),
    ]


class SphereParams(ctypes.Structure):
    """pitt_sphere_params (include/pitt_seg.h)."""
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32), ("optimize", ctypes.c_int32),
                ("probability", ctypes.c_double), ("radius_min", ctypes.c_double), ("radius_max", ctypes.c_double),
                ("seed", ctypes.c_uint32), ("pad", ctypes.c_int32)]


class CylinderParams(ctypes.Structure):
    """pitt_cylinder_params (include/pitt_seg.h)."""
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32), ("optimize", ctypes.c_int32),
                ("probability", ctypes.c_double), ("radius_min", ctypes.c_double), ("radius_max", ctypes.c_double),
                ("normal_distance_weight", ctypes.c_double), ("seed", ctypes.c_uint32), ("eigen33", ctypes.c_int32)]


class ConeParams(ctypes.Structure):
    """pitt_cone_params (include/pitt_seg.h)."""
    _fields_ = [("threshold", ctypes.c_double), ("max_iterations", ctypes.c_int32), ("optimize", ctypes.c_int32),
                ("probability", ctypes.c_double), ("normal_distance_weight", ctypes.c_double),
                ("min_angle", ctypes.c_double), ("max_angle", ctypes.c_double), ("eps_angle", ctypes.c_double),
                ("axis", ctypes.c_float * 3), ("eigen33", ctypes.c_int32), ("seed", ctypes.c_uint32),
                ("pad", ctypes.c_int32)]


class ClassifyParams(ctypes.Structure):
    """pitt_classify_params (include/pitt_seg.h)."""
    _fields_ = [("k", ctypes.c_int32), ("viewpoint", ctypes.c_float * 3), ("plane", SacParams),
                ("sphere", SphereParams), ("cylinder", CylinderParams), ("cone", ConeParams),
                ("cone_over_cylinder", ctypes.c_float), ("pad", ctypes.c_int32)]


class ClusterShape(ctypes.Structure):
    """pitt_cluster_shape (include/pitt_seg.h)."""
    _fields_ = [("n_points", ctypes.c_int64), ("tag", ctypes.c_int32), ("inliers", ctypes.c_int32 * 4),
                ("status", ctypes.c_int32 * 4), ("hypotheses", ctypes.c_int32 * 4), ("n_coef", ctypes.c_int32 * 4),
                ("sphere", ctypes.c_float * 4), ("cylinder", ctypes.c_float * 8), ("cone", ctypes.c_float * 8),
                ("plane", ctypes.c_float * 4), ("centroid", (ctypes.c_float * 3) * 4),
                ("est_centroid", ctypes.c_float * 3), ("pad", ctypes.c_int32)]


SHAPE_UNKNOWN, SHAPE_PLANE, SHAPE_SPHERE, SHAPE_CONE, SHAPE_CYLINDER = 0, 1, 2, 3, 4
SRV_SPHERE, SRV_CYLINDER, SRV_CONE, SRV_PLANE = 0, 1, 2, 3


class SupportParams(ctypes.Structure):
    _fields_ = [
        ("min_iterative_cloud_percentage", ctypes.c_float),
        ("min_iterative_plane_percentage", ctypes.c_float),
        ("horizontal_variance_threshold", ctypes.c_float),
        ("ransac_distance_threshold", ctypes.c_float),
        ("ransac_max_iterations", ctypes.c_int32),
        ("horizontal_axis", ctypes.c_float * 3),
        ("edge_remove_offset", ctypes.c_float * 3),
        ("reduce_order", ctypes.c_int32),
        ("div_mode", ctypes.c_int32),
    ]


class Support(ctypes.Structure):
    _fields_ = [
        ("n_points", ctypes.c_int32),
        ("idx_map", ctypes.POINTER(ctypes.c_int32)),
        ("coefficients", ctypes.c_float * 4),
        ("n_support", ctypes.c_int64),
        ("support_xyz", ctypes.POINTER(ctypes.c_float)),
        ("n_on_support", ctypes.c_int64),
        ("on_support_xyz", ctypes.POINTER(ctypes.c_float)),
    ]


class SupportList(ctypes.Structure):
    _fields_ = [
        ("n_supports", ctypes.c_int32),
        ("supports", ctypes.POINTER(Support)),
        ("iterations", ctypes.c_int32),
    ]


class Cluster(ctypes.Structure):
    _fields_ = [
        ("size", ctypes.c_int64),
        ("indices", ctypes.POINTER(ctypes.c_int32)),
        ("sum_xyz", ctypes.c_float * 3),
    ]


class ClusterList(ctypes.Structure):
    _fields_ = [
        ("n_clusters", ctypes.c_int32),
        ("clusters", ctypes.POINTER(Cluster)),
    ]


class SupportDev(ctypes.Structure):
    """pitt_support_dev: device pointers (ints), host coefficients."""
    _fields_ = [
        ("n_points", ctypes.c_int32),
        ("idx_map", ctypes.c_void_p),
        ("coefficients", ctypes.c_float * 4),
        ("n_support", ctypes.c_int64),
        ("support_xyz", ctypes.c_void_p),
        ("n_on_support", ctypes.c_int64),
        ("on_support_xyz", ctypes.c_void_p),
        ("stride", ctypes.c_int64),
    ]


class SupportListDev(ctypes.Structure):
    _fields_ = [("n_supports", ctypes.c_int32), ("supports", ctypes.POINTER(SupportDev)), ("iterations", ctypes.c_int32)]


class ClusterDev(ctypes.Structure):
    _fields_ = [("size", ctypes.c_int64), ("offset", ctypes.c_int64), ("sum_xyz", ctypes.c_float * 3),
                ("pad", ctypes.c_float)]


class ClusterListDev(ctypes.Structure):
    _fields_ = [("n_clusters", ctypes.c_int32), ("clusters", ctypes.POINTER(ClusterDev)), ("indices", ctypes.c_void_p)]


class ClusterParams(ctypes.Structure):
    _fields_ = [("tolerance", ctypes.c_double), ("min_rate", ctypes.c_double), ("max_rate", ctypes.c_double),
                ("min_input_size", ctypes.c_int32), ("pad", ctypes.c_int32)]


class SceneObject(ctypes.Structure):
    _fields_ = [("support", ctypes.c_int32), ("pad", ctypes.c_int32), ("size", ctypes.c_int64),
                ("offset", ctypes.c_int64), ("sum_xyz", ctypes.c_float * 3), ("pad2", ctypes.c_float)]


class Scene(ctypes.Structure):
    _fields_ = [("supports", SupportListDev), ("n_objects", ctypes.c_int32), ("objects", ctypes.POINTER(SceneObject)),
                ("indices", ctypes.c_void_p)]


_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); every symbol declared in include/pitt_seg.h
PITT_ABI_VERSION = 4  # include/pitt_seg.h

SIGNATURES = {
    "pitt_abi_version": (_i32, []),
    "pitt_build_flags": (_i32, []),
    "pitt_schedule_stats": (_i32, [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)]),
    "pitt_sac_params_default": (None, [ctypes.POINTER(SacParams)]),
    "pitt_create": (_i32, [ctypes.POINTER(_vp), _i32]),
    "pitt_destroy": (None, [_vp]),
    "pitt_set_stream": (_i32, [_vp, _vp]),
    "pitt_get_stream": (_vp, [_vp]),
    "pitt_last_error": (ctypes.c_char_p, [_vp]),
    "pitt_plane_segment": (_i32, [_vp, _f32p, _i64, _i32, ctypes.POINTER(SacParams), _i32p, _i64p,
                                  _f32p, _i32p]),
    "pitt_plane_segment_batch": (_i32, [_vp, ctypes.POINTER(Frames), ctypes.POINTER(SacParams),
                                        ctypes.POINTER(PlaneResult), _vp]),
    "pitt_plane_segment_batch_async": (_i32, [_vp, ctypes.POINTER(Frames), ctypes.POINTER(SacParams),
                                              ctypes.POINTER(PlaneResult), _vp]),
    "pitt_wait": (_i32, [_vp]),
    "pitt_multi_create": (_i32, [ctypes.POINTER(_vp), _i32p, _i32]),
    "pitt_multi_destroy": (None, [_vp]),
    "pitt_multi_devices": (_i32, [_vp]),
    "pitt_multi_context": (_vp, [_vp, _i32]),
    "pitt_multi_last_error": (ctypes.c_char_p, [_vp]),
    "pitt_plane_segment_batch_multi": (_i32, [_vp, ctypes.POINTER(Frames), ctypes.POINTER(SacParams),
                                              ctypes.POINTER(PlaneResult), _i32p]),
    "pitt_last_hypothesis_counts": (_i32, [_vp, _i32, _i32p, _i32]),
    "pitt_extract_indices": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _i64, _i32, _vp, _vp, _vp, _i64p]),
    "pitt_deep_filter": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.c_float, _vp, _vp, _vp, _i64p, _vp, _vp, _vp,
                                _i64p, _f32p]),
    "pitt_transform_cloud": (_i32, [_vp, _vp, _vp, _vp, _i64, _f32p, _i32, _vp, _vp, _vp]),
    "pitt_unpack_pointcloud2": (_i32, [_vp, _vp, _i64, _i32, _i32, _i32, _i64, _i32, _i32, _i32, _vp, _vp, _vp]),
    "pitt_normal_estimation": (_i32, [_vp, _vp, _vp, _vp, _i64, _i32, _f32p, _vp, _vp, _vp, _vp, _vp, _vp]),
    "pitt_voxel_grid": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.c_float, ctypes.c_float, ctypes.c_float, _i32, _vp,
                               _vp, _vp, _i64p, _i32p]),
    "pitt_sort_pairs": (_i32, [_vp, _vp, _vp, _i64, _i32]),
    "pitt_sphere_segment_host": (_i32, [_vp, _f32p, _i64, ctypes.POINTER(SphereParams), _i32p, _i64p, _f32p, _i32p]),
    "pitt_cylinder_segment": (_i32, [_vp] * 7 + [_i64, ctypes.POINTER(CylinderParams), _vp, _i64p, _f32p, _i32p]),
    "pitt_sphere_segment": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.POINTER(SphereParams), _vp, _i64p, _f32p, _i32p]),
    "pitt_axis_height": (_i32, [_vp, _vp, _vp, _vp, _i64, _f32p, _i32, _vp, _vp, _vp, _f32p, _i32p, _i32p, _f32p]),
    "pitt_support_params_default": (None, [ctypes.POINTER(SupportParams)]),
    "pitt_find_supports": (_i32, [_vp, _f32p, _f32p, _f32p, _i64, ctypes.POINTER(SupportParams),
                                  ctypes.POINTER(SupportList)]),
    "pitt_euclidean_clusters": (_i32, [_vp, _f32p, _f32p, _f32p, _i64, ctypes.c_double, _i32, _i32,
                                       ctypes.POINTER(ClusterList)]),
    "pitt_find_supports_aos": (_i32, [_vp, _f32p, _i64, _i32, ctypes.POINTER(SupportParams),
                                      ctypes.POINTER(SupportList)]),
    "pitt_euclidean_clusters_aos": (_i32, [_vp, _f32p, _i64, _i32, ctypes.c_double, _i32, _i32,
                                           ctypes.POINTER(ClusterList)]),
    "pitt_find_supports_dev": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.POINTER(SupportParams),
                                      ctypes.POINTER(SupportListDev)]),
    "pitt_euclidean_clusters_dev": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.c_double, _i32, _i32,
                                           ctypes.POINTER(ClusterListDev)]),
    "pitt_cluster_params_default": (None, [ctypes.POINTER(ClusterParams)]),
    "pitt_memcpy": (_i32, [_vp, _vp, _vp, _i64]),
    "pitt_refine_stats": (_i32, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "pitt_segment_objects_dev": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.POINTER(SupportParams),
                                        ctypes.POINTER(ClusterParams), ctypes.POINTER(Scene)]),
    "pitt_synth_frame": (_i32, [_i32, ctypes.c_uint64, _i32, _i32, _f32p, _f32p, _f32p]),
    "pitt_synth_fused": (_i32, [ctypes.c_uint64, _i32, _i32, _i32, _f32p, _f32p, _f32p]),
    "pitt_sampler_table": (_i32, [_i64, ctypes.c_uint32, _i64, _i32p]),
    "pitt_float_threshold": (ctypes.c_float, [ctypes.c_double]),
    "pitt_profile_enable": (_i32, [_vp, _i32]),
    "pitt_profile_get": (_i32, [_vp, ctypes.c_char_p, _i64p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double)]),
    "pitt_profile_reset": (_i32, [_vp]),
    "pitt_classify_params_default": (None, [ctypes.POINTER(ClassifyParams)]),
    "pitt_classify_clusters": (_i32, [_vp, _vp, _vp, _vp, _i64p, _i64p, _i32, ctypes.POINTER(ClassifyParams),
                                      ctypes.POINTER(ClusterShape)]),
}


class SrvSupportRequest(ctypes.Structure):
    _fields_ = [
        ("min_iterative_cloud_percentual_size", ctypes.c_float),
        ("min_iterative_plane_percentual_size", ctypes.c_float),
        ("variance_threshold_for_horizontal", ctypes.c_float),
        ("ransac_distance_point_in_shape_threshold", ctypes.c_float),
        ("ransac_model_normal_distance_weigth", ctypes.c_float),
        ("ransac_max_iteration_threshold", ctypes.c_int32),
        ("n_horizontal_axis", ctypes.c_int32),
        ("horizontal_axis", ctypes.c_float * 8),
        ("n_edge_remove_offset", ctypes.c_int32),
        ("edge_remove_offset", ctypes.c_float * 8),
    ]


# include/pitt_srv.h
SIGNATURES.update({
    "pitt_srv_create": (_vp, [_vp]),
    "pitt_srv_destroy": (None, [_vp]),
    "pitt_srv_param_set_int": (_i32, [_vp, ctypes.c_char_p, _i32]),
    "pitt_srv_param_set_double": (_i32, [_vp, ctypes.c_char_p, ctypes.c_double]),
    "pitt_srv_param_set_list": (_i32, [_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), _i32]),
    "pitt_srv_param_erase": (_i32, [_vp, ctypes.c_char_p]),
    "pitt_srv_ransac_plane": (_i32, [_vp, _f32p, _i64, _i64, _i32p, _i64p, _f32p, _i32p, _f32p]),
    "pitt_srv_ransac_cone": (_i32, [_vp, _f32p, _i64, _f32p, _i64, _i32p, _i64p, _f32p, _i32p, _f32p]),
    "pitt_srv_ransac_cylinder": (_i32, [_vp, _f32p, _i64, _f32p, _i64, _i32p, _i64p, _f32p, _i32p, _f32p]),
    "pitt_cylinder_segment_host": (_i32, [_vp, _f32p, _f32p, _i64, ctypes.POINTER(CylinderParams), _i32p, _i64p, _f32p,
                                          _i32p]),
    "pitt_cone_segment": (_i32, [_vp] * 7 + [_i64, ctypes.POINTER(ConeParams), _vp, _i64p, _f32p, _i32p]),
    "pitt_cone_segment_host": (_i32, [_vp, _f32p, _f32p, _i64, ctypes.POINTER(ConeParams), _i32p, _i64p, _f32p, _i32p]),
    "pitt_axis_height_host": (_i32, [_vp, _f32p, _i64, _f32p, _i32, _f32p, _i32p, _i32p, _f32p]),
    "pitt_srv_ransac_sphere": (_i32, [_vp, _f32p, _i64, _i64, _i32p, _i64p, _f32p, _i32p, _f32p]),
    "pitt_srv_call_ransac_plane": (_i32, [_vp, _f32p, _i64, _i64, _i32p, _i64p, _f32p, _i32p]),
    "pitt_srv_arbitrate": (_i32, [_i64, _i64, _i64, _i64]),
    "pitt_srv_find_supports": (_i32, [_vp, _f32p, _i64, _i64, ctypes.POINTER(SrvSupportRequest), _i32p, _f32p]),
    "pitt_srv_support_get": (_i32, [_vp, _i32, _i32p, _f32p, _i64p, _i64p]),
    "pitt_srv_support_cloud": (_i32, [_vp, _i32, _i32, _f32p]),
    "pitt_srv_clusterize": (_i32, [_vp, _f32p, _i64, _i32p]),
    "pitt_srv_cluster_get": (_i32, [_vp, _i32, _i32p, _i64p, _f32p, _f32p]),
    "pitt_srv_segment_objects": (_i32, [_vp, _f32p, _i64, _i64, _i32p]),
    "pitt_srv_output_size": (_i32, [_vp, _i32, _i32p]),
    "pitt_srv_output_cluster": (_i32, [_vp, _i32, _i32, _i32p, _i64p, _f32p]),
    "pitt_srv_classify_clusters": (_i32, [_vp, _vp, _vp, _vp, _i64p, _i64p, _i32, ctypes.POINTER(ClusterShape)]),
    "pitt_srv_segment_objects_dev": (_i32, [_vp, _vp, _vp, _vp, _i64, ctypes.POINTER(Scene)]),
    "pitt_srv_resolved_params": (_i32, [_vp, ctypes.POINTER(SupportParams), ctypes.POINTER(ClusterParams)]),
})


def _preload_torch_hip_runtime() -> None:
    """Make libpitt_seg.so bind to the HIP runtime torch uses (same SONAME libamdhip64.so.7),
    so a process that also uses torch holds exactly one HIP runtime."""
    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        return
    rt = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(rt):
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    _preload_torch_hip_runtime()
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the structs below are laid out for this ABI: a library of another ABI would read or write past
    # them (pitt_seg.h: callers check pitt_abi_version() at load)
    if lib.pitt_abi_version() != PITT_ABI_VERSION:
        raise ImportError(f"{path} implements ABI {lib.pitt_abi_version()}, this binding ABI {PITT_ABI_VERSION}")
    return lib


lib = load()
