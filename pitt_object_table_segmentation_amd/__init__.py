"""MI355X-native RANSAC-plane / support / Euclidean-cluster path of
TheEngineRoom-UniGe/pitt_object_table_segmentation, behind the C ABI in include/pitt_seg.h.

Importing this package loads libpitt_seg.so (hand-written HIP kernels for gfx950); it fails
loudly when the library is missing -- there is no CPU fallback.
"""
from . import _lib
from ._lib import (COV_EXACT, COV_FAST, DIV_EIGEN32, DIV_TRUE, PITT_E_SAMPLER, PITT_NO_MODEL, PITT_OK, PITT_TILE_POINTS,
                   REDUCE_HADD, REDUCE_SEQ, REDUCE_SSE2, SCENE_CLUTTER, SCENE_TABLE, SCENE_TABLE_NAN, SHAPE_CONE,
                   SHAPE_CYLINDER, SHAPE_PLANE, SHAPE_SPHERE, SHAPE_UNKNOWN)
from .api import (RESULT_DTYPE, ClusterResult, Context, FrameBatch, MultiContext, PittError, PlaneModel, Services,
                  SupportResult, classify_params, float_threshold, padded_offsets, sac_params, sampler_table,
                  support_params, synth_frame, synth_fused)

__all__ = [
    "Context", "MultiContext", "Services", "FrameBatch", "PlaneModel", "SupportResult", "ClusterResult", "PittError",
    "RESULT_DTYPE", "sac_params", "support_params", "synth_frame", "synth_fused", "sampler_table",
    "float_threshold", "padded_offsets", "REDUCE_SSE2", "REDUCE_HADD", "REDUCE_SEQ", "DIV_EIGEN32",
    "DIV_TRUE", "SCENE_TABLE", "SCENE_CLUTTER", "SCENE_TABLE_NAN", "PITT_OK", "PITT_NO_MODEL",
    "PITT_E_SAMPLER", "PITT_TILE_POINTS", "COV_EXACT", "COV_FAST", "classify_params", "SHAPE_UNKNOWN",
    "SHAPE_PLANE", "SHAPE_SPHERE", "SHAPE_CONE", "SHAPE_CYLINDER",
]
