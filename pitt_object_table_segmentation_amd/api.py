"""Python surface of the MI355X path: a thin, typed layer over libpitt_seg.so.

Every call crosses the C ABI (include/pitt_seg.h, include/pitt_srv.h); nothing here computes a
segmentation result.  Device memory comes from torch (plumbing only); host arrays are numpy.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L

lib = L.lib

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def _ip(a: np.ndarray):
    return a.ctypes.data_as(_i32p)


def _host_copy(ptr, shape, dtype) -> np.ndarray:
    """A numpy copy of `shape` elements at a host address the library returned (one memmove:
    np.ctypeslib.as_array builds a ctypes array type per call, which costs milliseconds here)."""
    out = np.empty(shape, dtype)
    if out.size:
        ctypes.memmove(out.ctypes.data, ctypes.cast(ptr, ctypes.c_void_p).value, out.nbytes)
    return out


class PittError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"pitt error {code}: {msg}")
        self.code = code


def sac_params(threshold: float = 0.007, max_iterations: int = 1000, probability: float = 0.99,
               seed: int = 12345, optimize: bool = True, reduce_order: int = L.REDUCE_SSE2,
               div_mode: int = L.DIV_EIGEN32, sampler_slack: int = 1000,
               cov_mode: int = 0) -> L.SacParams:
    """SACSegmentation parameters (defaults: plane_segmentation_srv.cpp:19-21)."""
    p = L.SacParams()
    lib.pitt_sac_params_default(ctypes.byref(p))
    p.threshold = threshold
    p.max_iterations = max_iterations
    p.probability = probability
    p.seed = seed
    p.optimize = 1 if optimize else 0
    p.reduce_order = reduce_order
    p.div_mode = div_mode
    p.sampler_slack = sampler_slack
    p.cov_mode = cov_mode
    return p


def support_params(**kw) -> L.SupportParams:
    """findSupports parameters (defaults: supports_segmentation_srv.cpp:30-39)."""
    p = L.SupportParams()
    lib.pitt_support_params_default(ctypes.byref(p))
    for k, v in kw.items():
        if k in ("horizontal_axis", "edge_remove_offset"):
            getattr(p, k)[:] = [float(t) for t in v]
        else:
            setattr(p, k, v)
    return p


RESULT_DTYPE = np.dtype([("coefficients", np.float32, 4), ("n_coeff", np.int32), ("status", np.int32),
                         ("n_inliers", np.int64), ("hypotheses", np.int32), ("best_hypothesis", np.int32),
                         ("best_count", np.int64), ("rejected_samples", np.int32), ("flags", np.int32)])
assert RESULT_DTYPE.itemsize == ctypes.sizeof(L.PlaneResult)


@dataclass
class PlaneModel:
    inliers: np.ndarray                 # int32, ascending (exact PCL semantics, index 0 kept)
    coefficients: np.ndarray            # float32[4], or empty when no model
    status: int = L.PITT_OK


@dataclass
class SupportResult:
    idx_map: np.ndarray                 # int32[n]: Support::inliers
    coefficients: np.ndarray            # float32[4] (refined)
    support_cloud: np.ndarray           # float32[m, 3]
    on_support_cloud: np.ndarray        # float32[k, 3]


@dataclass
class ClusterResult:
    indices: np.ndarray                 # int32, ascending
    sum_xyz: np.ndarray                 # float32[3], float sums in index order


def synth_frame(scene: int = L.SCENE_TABLE, seed: int = 1000, width: int = 640, height: int = 480):
    """Deterministic synthetic organised cloud (camera optical frame), SoA float32."""
    n = width * height
    x, y, z = (np.empty(n, np.float32) for _ in range(3))
    rc = lib.pitt_synth_frame(scene, ctypes.c_uint64(seed), width, height, _fp(x), _fp(y), _fp(z))
    if rc != L.PITT_OK:
        raise PittError(rc, "pitt_synth_frame")
    return x, y, z


def synth_fused(seed: int = 1000, views: int = 4, width: int = 640, height: int = 480):
    """`views` views of one table scene in a z-up world frame, concatenated (config 5)."""
    n = views * width * height
    x, y, z = (np.empty(n, np.float32) for _ in range(3))
    rc = lib.pitt_synth_fused(ctypes.c_uint64(seed), views, width, height, _fp(x), _fp(y), _fp(z))
    if rc != L.PITT_OK:
        raise PittError(rc, "pitt_synth_fused")
    return x, y, z


def sampler_table(n: int, attempts: int, seed: int = 12345) -> np.ndarray:
    out = np.empty(3 * attempts, np.int32)
    rc = lib.pitt_sampler_table(n, seed, attempts, _ip(out))
    if rc != L.PITT_OK:
        raise PittError(rc, "pitt_sampler_table")
    return out.reshape(attempts, 3)


def float_threshold(th: float) -> np.float32:
    return np.float32(lib.pitt_float_threshold(th))


def padded_offsets(counts: Sequence[int], tile: int = L.PITT_TILE_POINTS):
    """Frame offsets for a packed batch where every frame starts on a tile boundary; returns
    (offsets, capacity)."""
    offs, o = [], 0
    for c in counts:
        offs.append(o)
        o += max(tile, -(-int(c) // tile) * tile)
    return np.asarray(offs, np.int64), o


class FrameBatch:
    """Device-resident SoA batch (torch tensors on the context's device)."""

    def __init__(self, x, y, z, offsets: np.ndarray, counts: np.ndarray, capacity: int):
        self.x, self.y, self.z = x, y, z
        self.offsets = np.ascontiguousarray(offsets, np.int64)
        self.counts = np.ascontiguousarray(counts, np.int64)
        self.capacity = int(capacity)

    @property
    def n_frames(self) -> int:
        return len(self.counts)

    @classmethod
    def from_host(cls, frames: Sequence[tuple], device="cuda"):
        import torch
        counts = np.asarray([len(f[0]) for f in frames], np.int64)
        offsets, cap = padded_offsets(counts)
        planes = []
        for c in range(3):
            h = np.full(cap, np.nan, np.float32)
            for f, o, n in zip(frames, offsets, counts):
                h[o:o + n] = f[c]
            planes.append(torch.from_numpy(h).to(device))
        return cls(planes[0], planes[1], planes[2], offsets, counts, cap)

    def abi(self) -> L.Frames:
        self._keep = (self.offsets, self.counts)
        return L.Frames(self.x.data_ptr(), self.y.data_ptr(), self.z.data_ptr(),
                        self.offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                        self.counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                        self.n_frames, self.capacity)


class Context:
    """One pitt_ctx: a device, a stream and its scratch arena.  Not thread-safe."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        rc = lib.pitt_create(ctypes.byref(h), device)
        if rc != L.PITT_OK:
            raise PittError(rc, "pitt_create (needs a gfx950 device)")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib.pitt_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> int:
        if rc < 0:
            raise PittError(rc, f"{what}: {lib.pitt_last_error(self.h).decode()}")
        return rc

    def set_stream(self, stream) -> None:
        if getattr(self, "_inflight", None) is not None:  # finish the batch on the stream it was queued on
            self.wait()
        handle = getattr(stream, "cuda_stream", stream)
        self._check(lib.pitt_set_stream(self.h, ctypes.c_void_p(handle or 0)), "pitt_set_stream")

    # ---- plane -----------------------------------------------------------------------------
    def plane_segment(self, cloud: np.ndarray, params: Optional[L.SacParams] = None) -> PlaneModel:
        """seg.segment() on one host cloud: (n, 3) or (n, 4) float32 (PCL PointXYZ)."""
        cloud = np.ascontiguousarray(cloud, np.float32)
        n = cloud.shape[0]
        stride = 4 * cloud.shape[1] if cloud.ndim == 2 else 12
        p = params or sac_params()
        inl = np.empty(max(n, 1), np.int32)
        ni = ctypes.c_int64()
        co = np.zeros(4, np.float32)
        nc = ctypes.c_int32()
        rc = self._check(lib.pitt_plane_segment(self.h, _fp(cloud), n, stride, ctypes.byref(p), _ip(inl),
                                                ctypes.byref(ni), _fp(co), ctypes.byref(nc)), "pitt_plane_segment")
        return PlaneModel(inl[:ni.value], co[:nc.value].copy(), rc)

    def plane_segment_batch(self, batch: FrameBatch, params: Optional[L.SacParams] = None,
                            inliers_out=None) -> np.ndarray:
        """Batched seg.segment(); returns a RESULT_DTYPE record per frame.  inliers_out: optional
        int32 device tensor of batch.capacity entries (frame f at batch.offsets[f])."""
        p = params or sac_params()
        res = np.zeros(batch.n_frames, RESULT_DTYPE)
        fr = batch.abi()
        ptr = ctypes.c_void_p(inliers_out.data_ptr()) if inliers_out is not None else ctypes.c_void_p()
        self._check(lib.pitt_plane_segment_batch(self.h, ctypes.byref(fr), ctypes.byref(p),
                                                 res.ctypes.data_as(ctypes.POINTER(L.PlaneResult)), ptr),
                    "pitt_plane_segment_batch")
        return res

    def plane_segment_batch_async(self, batch: FrameBatch, params: Optional[L.SacParams] = None,
                                  inliers_out=None) -> np.ndarray:
        """Enqueue a batch on this context's stream and return immediately; the returned record
        array is filled by wait().  One batch in flight per context."""
        p = params or sac_params()
        # the previous batch completes into its own record array first (the C side would finish it
        # inside the call below; doing it here keeps that array alive while it is written)
        if getattr(self, "_inflight", None) is not None:
            self.wait()
        res = np.zeros(batch.n_frames, RESULT_DTYPE)
        fr = batch.abi()
        ptr = ctypes.c_void_p(inliers_out.data_ptr()) if inliers_out is not None else ctypes.c_void_p()
        self._check(lib.pitt_plane_segment_batch_async(self.h, ctypes.byref(fr), ctypes.byref(p),
                                                       res.ctypes.data_as(ctypes.POINTER(L.PlaneResult)), ptr),
                    "pitt_plane_segment_batch_async")
        self._inflight = (res, fr, p, batch)  # keep the buffers alive until wait()
        return res

    def wait(self) -> None:
        try:
            self._check(lib.pitt_wait(self.h), "pitt_wait")
        finally:
            self._inflight = None

    def hypothesis_counts(self, frame: int, cap: int) -> np.ndarray:
        out = np.zeros(cap, np.int32)
        self._check(lib.pitt_last_hypothesis_counts(self.h, frame, _ip(out), cap), "hypothesis_counts")
        return out

    # ---- ExtractIndices ---------------------------------------------------------------------
    def extract_indices(self, x, y, z, indices, negative: bool):
        """Device tensors in/out; returns (ox, oy, oz) trimmed to the output size."""
        import torch
        n = x.numel()
        m = indices.numel()
        size = m if not negative else n
        ox, oy, oz = (torch.empty(max(size, 1), dtype=torch.float32, device=x.device) for _ in range(3))
        nout = ctypes.c_int64()
        self._check(lib.pitt_extract_indices(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), n,
                                             indices.data_ptr() if m else None, m, 1 if negative else 0,
                                             ox.data_ptr(), oy.data_ptr(), oz.data_ptr(), ctypes.byref(nout)),
                    "pitt_extract_indices")
        k = nout.value
        return ox[:k], oy[:k], oz[:k]

    # ---- preprocessing (deep_filter_srv.cpp:27-44, obj_segmentation.cpp:248) ----------------
    def deep_filter(self, x, y, z, deep_threshold: float = -1.0, closer: bool = True, further: bool = True):
        """deepFiltering on device tensors: returns (closer (x, y, z), further (x, y, z), used_threshold);
        a cloud not asked for comes back as None (it is only counted)."""
        import torch
        n = x.numel()

        def planes(want):
            return [torch.empty(max(n, 1), dtype=torch.float32, device=x.device) for _ in range(3)] if want else None

        c, f = planes(closer), planes(further)
        nc, nf = ctypes.c_int64(), ctypes.c_int64()
        used = ctypes.c_float()

        def ptrs(p):
            return (None, None, None) if p is None else tuple(a.data_ptr() for a in p)

        self._check(lib.pitt_deep_filter(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), n, float(deep_threshold),
                                         *ptrs(c), ctypes.byref(nc), *ptrs(f), ctypes.byref(nf), ctypes.byref(used)),
                    "pitt_deep_filter")
        cout = None if c is None else tuple(a[:nc.value] for a in c)
        fout = None if f is None else tuple(a[:nf.value] for a in f)
        return cout, fout, used.value

    def transform_cloud(self, x, y, z, matrix, dense: bool = True):
        """pcl::transformPointCloud with a row-major 4x4 float matrix; device tensors in and out."""
        import torch
        m = np.ascontiguousarray(np.asarray(matrix, np.float32).reshape(16))
        ox, oy, oz = (torch.empty_like(a) for a in (x, y, z))
        self._check(lib.pitt_transform_cloud(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), x.numel(), _fp(m),
                                             1 if dense else 0, ox.data_ptr(), oy.data_ptr(), oz.data_ptr()),
                    "pitt_transform_cloud")
        return ox, oy, oz

    def unpack_pointcloud2(self, data, width: int, height: int, point_step: int, row_step: int,
                           offsets=(0, 4, 8)):
        """fromROSMsg of the XYZ fields: `data` a device uint8 tensor holding the PointCloud2 payload;
        returns device (x, y, z) of width * height points, row-major."""
        import torch
        n = width * height
        x, y, z = (torch.empty(max(n, 1), dtype=torch.float32, device=data.device) for _ in range(3))
        self._check(lib.pitt_unpack_pointcloud2(self.h, data.data_ptr(), data.numel() * data.element_size(), width,
                                                height, point_step, row_step,
                                                offsets[0], offsets[1], offsets[2], x.data_ptr(), y.data_ptr(),
                                                z.data_ptr()), "pitt_unpack_pointcloud2")
        return x[:n], y[:n], z[:n]

    def voxel_grid(self, x, y, z, leaf=(0.01, 0.01, 0.01), order: int = L.PITT_VOXEL_ORDER_PCL):
        """VoxelGrid<PointXYZ> downsampling (pc_manager.cpp:55-67) on device tensors: returns device
        (x, y, z) of the leaf centroids in ascending leaf index, and the flags (PITT_VOXEL_OVERFLOW_COPY).
        order: PCL's std::sort order inside a leaf (default, bit-exact) or stable (faster)."""
        import torch
        n = x.numel()
        ox, oy, oz = (torch.empty(max(n, 1), dtype=torch.float32, device=x.device) for _ in range(3))
        m, fl = ctypes.c_int64(), ctypes.c_int32()
        self._check(lib.pitt_voxel_grid(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), n, float(leaf[0]),
                                        float(leaf[1]), float(leaf[2]), int(order), ox.data_ptr(), oy.data_ptr(),
                                        oz.data_ptr(), ctypes.byref(m), ctypes.byref(fl)), "pitt_voxel_grid")
        k = m.value
        return (ox[:k], oy[:k], oz[:k]), fl.value

    def normal_estimation(self, x, y, z, k: int = 50, viewpoint=(0.0, 0.0, 0.0), neighbours: bool = False):
        """NormalEstimation with KdTree + setKSearch(k) (pc_manager.cpp:68-78) on device tensors:
        returns device (nx, ny, nz, curvature) [and (neighbour lists n x k, counts n)]."""
        import torch
        n = x.numel()
        out = [torch.empty(max(n, 1), dtype=torch.float32, device=x.device) for _ in range(4)]
        nn = torch.full((max(n, 1), k), -1, dtype=torch.int32, device=x.device) if neighbours else None
        cnt = torch.zeros(max(n, 1), dtype=torch.int32, device=x.device) if neighbours else None
        vp = np.asarray(viewpoint, np.float32)
        self._check(lib.pitt_normal_estimation(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), n, int(k), _fp(vp),
                                               *(o.data_ptr() for o in out), None if nn is None else nn.data_ptr(),
                                               None if cnt is None else cnt.data_ptr()), "pitt_normal_estimation")
        res = tuple(o[:n] for o in out)
        return res + ((nn[:n], cnt[:n]),) if neighbours else res

    def sort_pairs(self, key, val, depth_limit: int = -1):
        """std::sort's permutation of (key, val) uint32 pairs by key, in place on device int32 tensors."""
        self._check(lib.pitt_sort_pairs(self.h, key.data_ptr(), val.data_ptr(), key.numel(), int(depth_limit)),
                    "pitt_sort_pairs")

    def sphere_segment(self, x, y, z, threshold: float = 0.007, max_iterations: int = 1000, optimize: bool = True,
                       radius_min: float = 0.005, radius_max: float = 0.5, probability: float = 0.99,
                       seed: int = 12345):
        """The sphere service's seg.segment (sphere_segmentation_srv.cpp:57-73; defaults :19-27) on device
        tensors: (inliers device int32, coefficients [cx, cy, cz, r] or None, hypotheses)."""
        import torch
        n = x.numel()
        prm = L.SphereParams(threshold, max_iterations, int(optimize), probability, radius_min, radius_max, seed, 0)
        inl = torch.empty(max(n, 1), dtype=torch.int32, device=x.device)
        ni = ctypes.c_int64()
        coef = np.zeros(4, np.float32)
        hyp = ctypes.c_int32()
        rc = lib.pitt_sphere_segment(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), n, ctypes.byref(prm),
                                     inl.data_ptr(), ctypes.byref(ni), _fp(coef), ctypes.byref(hyp))
        if rc == L.PITT_NO_MODEL:
            return inl[:0], None, hyp.value
        self._check(rc, "pitt_sphere_segment")
        return inl[:ni.value], coef, hyp.value

    def cylinder_segment(self, x, y, z, nx, ny, nz, threshold: float = 0.008, max_iterations: int = 1000,
                         optimize: bool = True, radius_min: float = 0.005, radius_max: float = 0.5,
                         normal_distance_weight: float = 0.001, probability: float = 0.99, seed: int = 12345,
                         eigen33: int = 0):
        """The cylinder service's seg.segment (cylinder_segmentation_srv.cpp:110-126; defaults :23-30) on
        device tensors (points and normals): (inliers device int32, coefficients[7] or None, hypotheses)."""
        import torch
        n = x.numel()
        prm = L.CylinderParams(threshold, max_iterations, int(optimize), probability, radius_min, radius_max,
                               normal_distance_weight, seed, eigen33)
        inl = torch.empty(max(n, 1), dtype=torch.int32, device=x.device)
        ni = ctypes.c_int64()
        coef = np.zeros(7, np.float32)
        hyp = ctypes.c_int32()
        rc = lib.pitt_cylinder_segment(self.h, *(t.data_ptr() for t in (x, y, z, nx, ny, nz)), n, ctypes.byref(prm),
                                       inl.data_ptr(), ctypes.byref(ni), _fp(coef), ctypes.byref(hyp))
        if rc == L.PITT_NO_MODEL:
            return inl[:0], None, hyp.value
        self._check(rc, "pitt_cylinder_segment")
        return inl[:ni.value], coef, hyp.value

    def cone_segment(self, x, y, z, nx, ny, nz, threshold: float = 0.0055, max_iterations: int = 1000,
                     optimize: bool = True, normal_distance_weight: float = 0.0006, min_angle_deg: float = 10.0,
                     max_angle_deg: float = 170.0, eps_angle: float = 0.4, axis=(0.0, 0.0, 0.0), eigen33: int = 0,
                     probability: float = 0.99, seed: int = 12345):
        """The cone service's seg.segment (cone_segmentation_srv.cpp:111-127; defaults :24-31, the angles
        converted as :124 does) on device tensors (points and normals): (inliers device int32,
        coefficients[7] = apex, axis, opening angle, or None, hypotheses)."""
        import torch
        n = x.numel()
        prm = L.ConeParams(threshold, max_iterations, int(optimize), probability, normal_distance_weight,
                           min_angle_deg / 180.0 * np.pi, max_angle_deg / 180.0 * np.pi, eps_angle,
                           (ctypes.c_float * 3)(*axis), eigen33, seed, 0)
        inl = torch.empty(max(n, 1), dtype=torch.int32, device=x.device)
        ni = ctypes.c_int64()
        coef = np.zeros(7, np.float32)
        hyp = ctypes.c_int32()
        rc = lib.pitt_cone_segment(self.h, *(t.data_ptr() for t in (x, y, z, nx, ny, nz)), n, ctypes.byref(prm),
                                   inl.data_ptr(), ctypes.byref(ni), _fp(coef), ctypes.byref(hyp))
        if rc == L.PITT_NO_MODEL:
            return inl[:0], None, hyp.value
        self._check(rc, "pitt_cone_segment")
        return inl[:ni.value], coef, hyp.value

    def axis_height(self, x, y, z, coefficients, mode: int = L.PITT_AXIS_CYLINDER, projected: bool = False):
        """The cylinder / cone services' post-processing (cylinder_segmentation_srv.cpp:129-189,
        cone_segmentation_srv.cpp:129-189) on device tensors: (height, idx1, idx2, centroid[3])
        [, (px, py, pz) the cloud projected on the axis]."""
        import torch
        n = x.numel()
        coef = np.ascontiguousarray(np.asarray(coefficients, np.float32)[:6])
        if coef.size != 6:
            raise ValueError("coefficients: the axis point and direction (6 values) are needed")
        proj = [torch.empty(max(n, 1), dtype=torch.float32, device=x.device) for _ in range(3)] if projected else None
        h = ctypes.c_float()
        i1, i2 = ctypes.c_int32(), ctypes.c_int32()
        cen = np.zeros(3, np.float32)
        self._check(lib.pitt_axis_height(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), n, _fp(coef), int(mode),
                                         *((p.data_ptr() for p in proj) if proj else (None, None, None)),
                                         ctypes.byref(h), ctypes.byref(i1), ctypes.byref(i2), _fp(cen)),
                    "pitt_axis_height")
        res = (h.value, i1.value, i2.value, cen)
        return res + (tuple(p[:n] for p in proj),) if projected else res

    # ---- supports ---------------------------------------------------------------------------
    def find_supports(self, x, y, z, params: Optional[L.SupportParams] = None) -> List[SupportResult]:
        x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
        p = params or support_params()
        out = L.SupportList()
        self._check(lib.pitt_find_supports(self.h, _fp(x), _fp(y), _fp(z), len(x), ctypes.byref(p),
                                           ctypes.byref(out)), "pitt_find_supports")
        res = []
        for i in range(out.n_supports):
            s = out.supports[i]
            # the clouds come back as SoA planes: an (m, 3) view of a (3, m) copy (its .T rows are the
            # contiguous x, y, z planes the other entry points take)
            sup = _host_copy(s.support_xyz, (3, s.n_support), np.float32).T
            on = _host_copy(s.on_support_xyz, (3, s.n_on_support), np.float32).T
            res.append(SupportResult(_host_copy(s.idx_map, (s.n_points,), np.int32),
                                     np.array(list(s.coefficients), np.float32), sup, on))
        return res

    # ---- clusters ---------------------------------------------------------------------------
    def euclidean_clusters(self, x, y, z, tolerance: float = 0.03, min_size: int = 1,
                           max_size: int = 2 ** 31 - 1) -> List[ClusterResult]:
        x, y, z = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
        out = L.ClusterList()
        self._check(lib.pitt_euclidean_clusters(self.h, _fp(x), _fp(y), _fp(z), len(x), tolerance, min_size,
                                                max_size, ctypes.byref(out)), "pitt_euclidean_clusters")
        if out.n_clusters == 0:
            return []
        # the members of every cluster are one contiguous block (size-descending order): one copy
        cl = [out.clusters[i] for i in range(out.n_clusters)]
        total = sum(c.size for c in cl)
        allm = _host_copy(cl[0].indices, (total,), np.int32)
        res, o = [], 0
        for c in cl:
            res.append(ClusterResult(allm[o:o + c.size], np.array(list(c.sum_xyz), np.float32)))
            o += c.size
        return res

    def schedule_stats(self):
        """(batches finished by a continuation past their scheduled chunks, chunks the last batch launched
        up front) of the adaptive chunk schedule on this context."""
        c, k = ctypes.c_int64(0), ctypes.c_int32(0)
        self._check(lib.pitt_schedule_stats(self.h, ctypes.byref(c), ctypes.byref(k)), "pitt_schedule_stats")
        return c.value, k.value

    def refine_stats(self):
        """(batches refined by k_xrefine, frames it handed back to k_refine's serial chain)."""
        b, f = ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(lib.pitt_refine_stats(self.h, ctypes.byref(b), ctypes.byref(f)), "pitt_refine_stats")
        return b.value, f.value

    # ---- device-resident support / cluster path (pitt_*_dev) ---------------------------------
    def _dev_copy(self, ptr, n: int, dtype, device):
        """A fresh device tensor holding n elements copied from a device address of the arena."""
        import torch
        t = torch.empty(max(n, 1), dtype=dtype, device=device)
        if n:
            # the caching allocator may hand back a block that kernels still queued on torch's stream
            # use; pitt_memcpy writes on the context's stream, so let torch's stream drain first
            torch.cuda.current_stream(t.device).synchronize()
            self._check(lib.pitt_memcpy(self.h, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr),
                                        n * t.element_size()), "pitt_memcpy")
        return t[:n]

    def _planes_copy(self, ptr, n: int, stride: int, device):
        import torch
        if n == 0:
            return torch.zeros((0, 3), dtype=torch.float32, device=device)
        return torch.stack([self._dev_copy(ptr + 4 * k * stride, n, torch.float32, device) for k in range(3)], 1)

    def find_supports_dev(self, x, y, z, params: Optional[L.SupportParams] = None):
        """pitt_find_supports_dev on device tensors: a list of dicts of device tensors (idx_map,
        support_cloud, on_support_cloud as (m, 3)) and host coefficients."""
        p = params or support_params()
        out = L.SupportListDev()
        self._check(lib.pitt_find_supports_dev(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), x.numel(),
                                               ctypes.byref(p), ctypes.byref(out)), "pitt_find_supports_dev")
        return [self._support_dev(out.supports[i], x.device) for i in range(out.n_supports)]

    def _support_dev(self, s, device):
        import torch
        return {"idx_map": self._dev_copy(s.idx_map, s.n_points, torch.int32, device),
                "coefficients": np.array(list(s.coefficients), np.float32),
                "support_cloud": self._planes_copy(s.support_xyz, s.n_support, s.stride, device),
                "on_support_cloud": self._planes_copy(s.on_support_xyz, s.n_on_support, s.stride, device)}

    def euclidean_clusters_dev(self, x, y, z, tolerance: float = 0.03, min_size: int = 1, max_size: int = 2 ** 31 - 1):
        """pitt_euclidean_clusters_dev on device tensors: [(device int32 members, host sums)]."""
        import torch
        out = L.ClusterListDev()
        self._check(lib.pitt_euclidean_clusters_dev(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), x.numel(),
                                                    tolerance, min_size, max_size, ctypes.byref(out)),
                    "pitt_euclidean_clusters_dev")
        total = sum(out.clusters[i].size for i in range(out.n_clusters))
        idx = self._dev_copy(out.indices or 0, total, torch.int32, x.device)
        return [(idx[out.clusters[i].offset:out.clusters[i].offset + out.clusters[i].size],
                 np.array(list(out.clusters[i].sum_xyz), np.float32)) for i in range(out.n_clusters)]

    def segment_objects_dev(self, x, y, z, support: Optional[L.SupportParams] = None,
                            tolerance: float = 0.03, min_rate: float = 0.01, max_rate: float = 0.99,
                            min_input_size: int = 30, copy: bool = True):
        """pitt_segment_objects_dev (obj_segmentation.cpp:261-312 on the device): (supports, objects)
        with objects = [(support index, device members, host sums)]; copy=False returns only the
        sizes (what crosses the boundary when nothing is read back)."""
        import torch
        sp = support or support_params()
        cp = L.ClusterParams(tolerance, min_rate, max_rate, min_input_size, 0)
        out = L.Scene()
        self._check(lib.pitt_segment_objects_dev(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), x.numel(),
                                                 ctypes.byref(sp), ctypes.byref(cp), ctypes.byref(out)),
                    "pitt_segment_objects_dev")
        if not copy:
            return ([out.supports.supports[i].n_on_support for i in range(out.supports.n_supports)],
                    [out.objects[i].size for i in range(out.n_objects)])
        sups = [self._support_dev(out.supports.supports[i], x.device) for i in range(out.supports.n_supports)]
        total = sum(out.objects[i].size for i in range(out.n_objects))
        idx = self._dev_copy(out.indices or 0, total, torch.int32, x.device)
        objs = [(out.objects[i].support, idx[out.objects[i].offset:out.objects[i].offset + out.objects[i].size],
                 np.array(list(out.objects[i].sum_xyz), np.float32)) for i in range(out.n_objects)]
        return sups, objs

    # ---- primitive classification -----------------------------------------------------------
    def classify_clusters(self, x, y, z, offsets, counts, params: Optional[L.ClassifyParams] = None):
        """pitt_classify_clusters (ransac_segmentation.cpp:230-302 for all of a frame's clusters in one
        pass): device (or host) SoA, cluster c = [offsets[c], offsets[c] + counts[c]).  Returns one dict
        per cluster: tag, inliers / status / hypotheses / coefficients / centroid per service (sphere,
        cylinder, cone, plane) and the chosen primitive's est_centroid."""
        offsets = np.ascontiguousarray(np.asarray(offsets, np.int64))
        counts = np.ascontiguousarray(np.asarray(counts, np.int64))
        nc = len(counts)
        prm = params or classify_params()
        out = (L.ClusterShape * max(nc, 1))()
        ptr = (lambda a: a.data_ptr()) if hasattr(x, "data_ptr") else (lambda a: np.ascontiguousarray(a, np.float32).ctypes.data)
        keep = [x, y, z] if hasattr(x, "data_ptr") else [np.ascontiguousarray(a, np.float32) for a in (x, y, z)]
        self._check(lib.pitt_classify_clusters(self.h, *(ptr(a) for a in keep), _i64(offsets), _i64(counts), nc,
                                               ctypes.byref(prm), out), "pitt_classify_clusters")
        return [_shape_dict(out[c]) for c in range(nc)]

    # ---- profiling --------------------------------------------------------------------------
    def profile(self, on: bool = True) -> None:
        lib.pitt_profile_enable(self.h, 1 if on else 0)

    def profile_reset(self) -> None:
        lib.pitt_profile_reset(self.h)

    def profile_get(self, kernel: str):
        n, ms, b = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        self._check(lib.pitt_profile_get(self.h, kernel.encode(), ctypes.byref(n), ctypes.byref(ms), ctypes.byref(b)),
                    "pitt_profile_get")
        return n.value, ms.value, b.value


def classify_params(**kw) -> L.ClassifyParams:
    """pitt_classify_params_default (the four services' handler defaults, k = 50), fields overridden by
    keyword (e.g. k=50, cone_over_cylinder=0.9)."""
    p = L.ClassifyParams()
    lib.pitt_classify_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


SERVICE_NAMES = ("sphere", "cylinder", "cone", "plane")
SHAPE_NAMES = {L.SHAPE_UNKNOWN: "unknown", L.SHAPE_PLANE: "plane", L.SHAPE_SPHERE: "sphere", L.SHAPE_CONE: "cone",
               L.SHAPE_CYLINDER: "cylinder"}  # returnPrimitiveNameFromTag, ransac_segmentation.cpp:210-218


def _i64(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def _shape_dict(o) -> dict:
    coef = [np.array(o.sphere[:o.n_coef[0]], np.float32), np.array(o.cylinder[:o.n_coef[1]], np.float32),
            np.array(o.cone[:o.n_coef[2]], np.float32), np.array(o.plane[:o.n_coef[3]], np.float32)]
    return dict(n_points=o.n_points, tag=o.tag, shape=SHAPE_NAMES.get(o.tag, "unknown"),
                inliers=list(o.inliers), status=list(o.status), hypotheses=list(o.hypotheses), coefficients=coef,
                centroid=np.array([list(c) for c in o.centroid], np.float32),
                est_centroid=np.array(list(o.est_centroid), np.float32))


def _cloud16(xyz: np.ndarray) -> np.ndarray:
    """(n, 3) -> PCL PointXYZ layout (n, 4) with the pad = 1.0f."""
    xyz = np.asarray(xyz, np.float32)
    if xyz.ndim == 2 and xyz.shape[1] == 4:
        return np.ascontiguousarray(xyz)
    out = np.ones((xyz.shape[0], 4), np.float32)
    out[:, :3] = xyz
    return out


class MultiContext:
    """pitt_multi: one context per listed device, frame-sharded plane batches from host memory
    (include/pitt_seg.h; the in-process multi-device path of a C++ host).  A device may be listed
    more than once (several contexts on it: how the path is exercised on a one-GPU box)."""

    def __init__(self, devices: Sequence[int]):
        devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
        h = ctypes.c_void_p()
        rc = lib.pitt_multi_create(ctypes.byref(h), devs, len(devices))
        if rc != L.PITT_OK:
            raise PittError(rc, "pitt_multi_create (needs gfx950 devices)")
        self.h = h
        self.devices = list(devices)

    def close(self):
        if self.h:
            lib.pitt_multi_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plane_segment_batch(self, frames: Sequence[tuple], params: Optional[L.SacParams] = None):
        """frames: host (x, y, z) float32 arrays.  Returns (RESULT_DTYPE records, [ascending inliers])
        gathered in frame order from the devices' shards."""
        counts = np.array([len(f[0]) for f in frames], np.int64)
        offs, cap = padded_offsets(counts)
        planes = [np.zeros(max(cap, 1), np.float32) for _ in range(3)]
        for o, n, f in zip(offs, counts, frames):
            for k in range(3):
                planes[k][o:o + n] = f[k]
        inl = np.empty(max(cap, 1), np.int32)
        res = np.zeros(len(frames), RESULT_DTYPE)
        fr = L.Frames(planes[0].ctypes.data, planes[1].ctypes.data, planes[2].ctypes.data,
                      offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                      counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(frames), cap)
        p = params or sac_params()
        rc = lib.pitt_plane_segment_batch_multi(self.h, ctypes.byref(fr), ctypes.byref(p),
                                                res.ctypes.data_as(ctypes.POINTER(L.PlaneResult)), _ip(inl))
        if rc < 0:
            raise PittError(rc, f"pitt_plane_segment_batch_multi: {lib.pitt_multi_last_error(self.h).decode()}")
        return res, [inl[o:o + r["n_inliers"]].copy() for o, r in zip(offs, res)]


class Services:
    """The reference's three service handlers + obj_segmentation glue (C++ mirror, pitt_srv.h)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.h = lib.pitt_srv_create(ctx.h)
        if not self.h:
            raise PittError(L.PITT_E_INVALID, "pitt_srv_create")

    def close(self):
        if self.h:
            lib.pitt_srv_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_param(self, name: str, value) -> None:
        if isinstance(value, bool) or isinstance(value, int):
            lib.pitt_srv_param_set_int(self.h, name.encode(), int(value))
        elif isinstance(value, float):
            lib.pitt_srv_param_set_double(self.h, name.encode(), value)
        else:
            arr = (ctypes.c_double * len(value))(*[float(v) for v in value])
            lib.pitt_srv_param_set_list(self.h, name.encode(), arr, len(value))

    def erase_param(self, name: str) -> None:
        lib.pitt_srv_param_erase(self.h, name.encode())

    def _rc(self, rc: int, what: str) -> bool:
        if rc < 0:
            raise PittError(rc, f"{what}: {lib.pitt_last_error(self.ctx.h).decode()}")
        return rc == 1

    def ransac_plane(self, cloud: np.ndarray, n_normals: Optional[int] = None):
        """ransacPlaneDetaction: returns (ok, inliers (index 0 dropped), coefficients, centroid)."""
        c = _cloud16(cloud)
        n = c.shape[0]
        inl = np.empty(max(n, 1), np.int32)
        ni, nc = ctypes.c_int64(), ctypes.c_int32()
        co = np.zeros(4, np.float32)
        ce = np.zeros(3, np.float32)
        ok = self._rc(lib.pitt_srv_ransac_plane(self.h, _fp(c), n, n if n_normals is None else n_normals, _ip(inl),
                                                ctypes.byref(ni), _fp(co), ctypes.byref(nc), _fp(ce)), "ransac_plane")
        return ok, inl[:ni.value].copy(), co[:nc.value].copy(), ce

    def ransac_sphere(self, cloud: np.ndarray, n_normals: Optional[int] = None):
        """ransacSphereDetection (sphere_segmentation_srv.cpp:29-96): (ok, inliers (index 0 dropped),
        coefficients [cx, cy, cz, r] or empty, centroid = the centre)."""
        c = _cloud16(cloud)
        n = c.shape[0]
        inl = np.empty(max(n, 1), np.int32)
        ni, nc = ctypes.c_int64(), ctypes.c_int32()
        co = np.zeros(4, np.float32)
        ce = np.zeros(3, np.float32)
        ok = self._rc(lib.pitt_srv_ransac_sphere(self.h, _fp(c), n, n if n_normals is None else n_normals, _ip(inl),
                                                 ctypes.byref(ni), _fp(co), ctypes.byref(nc), _fp(ce)), "ransac_sphere")
        return ok, inl[:ni.value].copy(), co[:nc.value].copy(), ce

    def ransac_cylinder(self, cloud: np.ndarray, normals: np.ndarray, n_normals: Optional[int] = None):
        """ransacCylinderDetaction (cylinder_segmentation_srv.cpp:82-216): (ok, inliers (index 0 dropped),
        coefficients (7 model values, then the height), centroid)."""
        c = _cloud16(cloud)
        n = c.shape[0]
        nrm = np.ascontiguousarray(np.asarray(normals, np.float32).reshape(-1, 3))
        inl = np.empty(max(n, 1), np.int32)
        ni, nc = ctypes.c_int64(), ctypes.c_int32()
        co = np.zeros(8, np.float32)
        ce = np.zeros(3, np.float32)
        ok = self._rc(lib.pitt_srv_ransac_cylinder(self.h, _fp(c), n, _fp(nrm), n if n_normals is None else n_normals,
                                                   _ip(inl), ctypes.byref(ni), _fp(co), ctypes.byref(nc), _fp(ce)),
                      "ransac_cylinder")
        return ok, inl[:ni.value].copy(), co[:nc.value].copy(), ce

    def ransac_cone(self, cloud: np.ndarray, normals: np.ndarray, n_normals: Optional[int] = None):
        """ransacConeDetaction (cone_segmentation_srv.cpp:83-216): (ok, inliers (index 0 dropped),
        coefficients (apex, axis, opening angle, then the height), centroid)."""
        c = _cloud16(cloud)
        n = c.shape[0]
        nrm = np.ascontiguousarray(np.asarray(normals, np.float32).reshape(-1, 3))
        inl = np.empty(max(n, 1), np.int32)
        ni, nc = ctypes.c_int64(), ctypes.c_int32()
        co = np.zeros(8, np.float32)
        ce = np.zeros(3, np.float32)
        ok = self._rc(lib.pitt_srv_ransac_cone(self.h, _fp(c), n, _fp(nrm), n if n_normals is None else n_normals,
                                               _ip(inl), ctypes.byref(ni), _fp(co), ctypes.byref(nc), _fp(ce)),
                      "ransac_cone")
        return ok, inl[:ni.value].copy(), co[:nc.value].copy(), ce

    def call_ransac_plane(self, cloud: np.ndarray, n_normals: Optional[int] = None):
        """callRansacPlaneSegmentation (ransac_segmentation.cpp:175-199): (accepted, inliers, coefficients)."""
        c = _cloud16(cloud)
        n = len(c)
        inl = np.empty(max(n, 1), np.int32)
        ni, nc = ctypes.c_int64(), ctypes.c_int32()
        co = np.zeros(4, np.float32)
        rc = lib.pitt_srv_call_ransac_plane(self.h, _fp(c), n, n if n_normals is None else n_normals, _ip(inl),
                                            ctypes.byref(ni), _fp(co), ctypes.byref(nc))
        return self._rc(rc, "pitt_srv_call_ransac_plane"), inl[:ni.value].copy(), co[:nc.value].copy()

    @staticmethod
    def arbitrate(sphere: int, cylinder: int, cone: int, plane: int) -> int:
        """The primitive arbitration of ransac_segmentation.cpp:265-302 (tags :42-46)."""
        rc = lib.pitt_srv_arbitrate(sphere, cylinder, cone, plane)
        if rc < 0:
            raise PittError(rc, "pitt_srv_arbitrate")
        return rc

    def classify_clusters(self, x, y, z, offsets, counts):
        """clustersAcquisition's loop (ransac_segmentation.cpp:230-302) for all clusters in one pass, with
        the parameters the four handlers read (pitt_srv_classify_clusters); as Context.classify_clusters."""
        offsets = np.ascontiguousarray(np.asarray(offsets, np.int64))
        counts = np.ascontiguousarray(np.asarray(counts, np.int64))
        nc = len(counts)
        out = (L.ClusterShape * max(nc, 1))()
        keep = [x, y, z] if hasattr(x, "data_ptr") else [np.ascontiguousarray(a, np.float32) for a in (x, y, z)]
        ptrs = [a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data for a in keep]
        rc = lib.pitt_srv_classify_clusters(self.h, *ptrs, _i64(offsets), _i64(counts), nc, out)
        if rc < 0:
            raise PittError(rc, f"classify_clusters: {lib.pitt_last_error(self.ctx.h).decode()}")
        return [_shape_dict(out[c]) for c in range(nc)]

    def find_supports(self, cloud: np.ndarray, n_normals: Optional[int] = None, **req):
        c = _cloud16(cloud)
        n = c.shape[0]
        r = L.SrvSupportRequest()
        r.min_iterative_cloud_percentual_size = req.get("min_iterative_cloud_percentual_size", -1.0)
        r.min_iterative_plane_percentual_size = req.get("min_iterative_plane_percentual_size", -1.0)
        r.variance_threshold_for_horizontal = req.get("variance_threshold_for_horizontal", -1.0)
        r.ransac_distance_point_in_shape_threshold = req.get("ransac_distance_point_in_shape_threshold", -1.0)
        r.ransac_model_normal_distance_weigth = req.get("ransac_model_normal_distance_weigth", -1.0)
        r.ransac_max_iteration_threshold = req.get("ransac_max_iteration_threshold", -1)
        ax = list(req.get("horizontal_axis", [-1.0]))
        of = list(req.get("support_edge_remove_offset", [-1.0]))
        r.n_horizontal_axis = len(ax)
        r.horizontal_axis[:len(ax)] = ax
        r.n_edge_remove_offset = len(of)
        r.edge_remove_offset[:len(of)] = of
        ns = ctypes.c_int32()
        used = np.zeros(13, np.float32)
        ok = self._rc(lib.pitt_srv_find_supports(self.h, _fp(c), n, n if n_normals is None else n_normals,
                                                 ctypes.byref(r), ctypes.byref(ns), _fp(used)), "find_supports")
        sups = []
        for s in range(ns.value):
            idx = np.empty(max(n, 1), np.int32)
            co = np.zeros(4, np.float32)
            a, b = ctypes.c_int64(), ctypes.c_int64()
            lib.pitt_srv_support_get(self.h, s, _ip(idx), _fp(co), ctypes.byref(a), ctypes.byref(b))
            sc = np.empty((max(a.value, 1), 4), np.float32)
            oc = np.empty((max(b.value, 1), 4), np.float32)
            lib.pitt_srv_support_cloud(self.h, s, 0, _fp(sc))
            lib.pitt_srv_support_cloud(self.h, s, 1, _fp(oc))
            sups.append(dict(inliers=idx[:n].copy(), coefficients=co, support_cloud=sc[:a.value, :3].copy(),
                             on_support_cloud=oc[:b.value, :3].copy()))
        return ok, sups, used

    def clusterize(self, cloud: np.ndarray):
        c = _cloud16(cloud)
        n = c.shape[0]
        nc = ctypes.c_int32()
        ok = self._rc(lib.pitt_srv_clusterize(self.h, _fp(c), n, ctypes.byref(nc)), "clusterize")
        out = []
        for k in range(nc.value):
            size = ctypes.c_int64()
            lib.pitt_srv_cluster_get(self.h, k, None, ctypes.byref(size), None, None)
            idx = np.empty(max(size.value, 1), np.int32)
            ce = np.zeros(3, np.float32)
            cl = np.empty((max(size.value, 1), 4), np.float32)
            lib.pitt_srv_cluster_get(self.h, k, _ip(idx), ctypes.byref(size), _fp(ce), _fp(cl))
            out.append(dict(inliers=idx[:size.value].copy(), centroid=ce, cloud=cl[:size.value, :3].copy()))
        return ok, out

    def resolved_params(self):
        """(SupportParams, ClusterParams) that segment_objects_dev would use with the current parameters."""
        sp, cp = L.SupportParams(), L.ClusterParams()
        self._rc(lib.pitt_srv_resolved_params(self.h, ctypes.byref(sp), ctypes.byref(cp)), "resolved_params")
        return sp, cp

    def segment_objects_dev(self, x, y, z):
        """pitt_srv_segment_objects_dev: segment_objects with the world cloud in HBM (device tensors), the
        parameters from the parameter server.  Returns one list per support with at least one cluster, of
        dicts (inliers = on-support indices, centroid = sum / (size + 1)), as segment_objects."""
        out = L.Scene()
        rc = lib.pitt_srv_segment_objects_dev(self.h, x.data_ptr(), y.data_ptr(), z.data_ptr(), x.numel(),
                                              ctypes.byref(out))
        self._rc(rc, "segment_objects_dev")
        total = max([out.objects[i].offset + out.objects[i].size for i in range(out.n_objects)], default=0)
        idx = np.empty(max(total, 1), np.int32)
        if total:
            self.ctx._check(lib.pitt_memcpy(self.ctx.h, _ip(idx), ctypes.c_void_p(out.indices), total * 4),
                            "pitt_memcpy")
        outs = []
        for s in range(out.supports.n_supports):
            objs = []
            for i in range(out.n_objects):
                o = out.objects[i]
                if o.support == s:
                    sums = np.array(list(o.sum_xyz), np.float32)
                    objs.append(dict(inliers=idx[o.offset:o.offset + o.size].copy(),
                                     centroid=sums / np.float32(o.size + 1)))
            if objs:
                outs.append(objs)
        return outs

    def segment_objects(self, cloud: np.ndarray, n_normals: Optional[int] = None):
        c = _cloud16(cloud)
        n = c.shape[0]
        no = ctypes.c_int32()
        self._rc(lib.pitt_srv_segment_objects(self.h, _fp(c), n, n if n_normals is None else n_normals,
                                              ctypes.byref(no)), "segment_objects")
        outs = []
        for o in range(no.value):
            k = ctypes.c_int32()
            lib.pitt_srv_output_size(self.h, o, ctypes.byref(k))
            objs = []
            for c_ in range(k.value):
                size = ctypes.c_int64()
                lib.pitt_srv_output_cluster(self.h, o, c_, None, ctypes.byref(size), None)
                idx = np.empty(max(size.value, 1), np.int32)
                ce = np.zeros(3, np.float32)
                lib.pitt_srv_output_cluster(self.h, o, c_, _ip(idx), ctypes.byref(size), _fp(ce))
                objs.append(dict(inliers=idx[:size.value].copy(), centroid=ce))
            outs.append(objs)
        return outs
