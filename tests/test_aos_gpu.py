"""The strided PointXYZ entry points (pitt_find_supports_aos, pitt_euclidean_clusters_aos; ABI 4): a
host cloud in the layout a ROS node holds (pcl::PointXYZ, 16 bytes, or packed 12-byte xyz) goes up in
one copy and is deinterleaved on the device.  Their outputs must be byte-equal to the SoA entry points'
on the same points (which the oracle tests pin), including NaN points and an empty cloud."""
import ctypes

import numpy as np
import pytest

import pitt_object_table_segmentation_amd as pitt
from pitt_object_table_segmentation_amd import _lib as L
from pitt_object_table_segmentation_amd.api import _host_copy

pytestmark = pytest.mark.gpu


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _aos(x, y, z, stride):
    a = np.zeros((len(x), stride // 4), np.float32)
    a[:, 0], a[:, 1], a[:, 2] = x, y, z
    if stride == 16:
        a[:, 3] = 1.0
    return a


def _supports_aos(ctx, x, y, z, stride):
    a = _aos(x, y, z, stride)
    out = L.SupportList()
    rc = L.lib.pitt_find_supports_aos(ctx.h, _fp(a), len(x), stride, ctypes.byref(pitt.support_params()),
                                      ctypes.byref(out))
    assert rc == 0, L.lib.pitt_last_error(ctx.h)
    res = []
    for i in range(out.n_supports):
        s = out.supports[i]
        res.append((_host_copy(s.idx_map, (s.n_points,), np.int32), np.array(list(s.coefficients), np.float32),
                    _host_copy(s.support_xyz, (3, s.n_support), np.float32),
                    _host_copy(s.on_support_xyz, (3, s.n_on_support), np.float32)))
    return res


@pytest.mark.parametrize("stride", [16, 12])
def test_find_supports_aos_equals_soa(ctx, stride):
    x, y, z = pitt.synth_fused(61, 2, 160, 120)
    x = x.copy()
    x[::97] = np.nan  # NaN points ride along as they lie
    want = ctx.find_supports(x, y, z)
    got = _supports_aos(ctx, x, y, z, stride)
    assert len(got) == len(want) > 0
    for g, w in zip(got, want):
        assert np.array_equal(g[0], w.idx_map)
        assert np.array_equal(g[1], w.coefficients)
        assert np.array_equal(g[2], w.support_cloud.T, equal_nan=True)
        assert np.array_equal(g[3], w.on_support_cloud.T, equal_nan=True)


@pytest.mark.parametrize("stride", [16, 12])
def test_euclidean_clusters_aos_equals_soa(ctx, stride):
    sup = ctx.find_supports(*pitt.synth_fused(62, 1, 160, 120))
    on = np.ascontiguousarray(sup[0].on_support_cloud.T)
    n = on.shape[1]
    want = ctx.euclidean_clusters(*on, tolerance=0.03, min_size=int(n * 0.01), max_size=int(n * 0.99))
    a = _aos(*on, stride)
    out = L.ClusterList()
    rc = L.lib.pitt_euclidean_clusters_aos(ctx.h, _fp(a), n, stride, 0.03, int(n * 0.01), int(n * 0.99),
                                           ctypes.byref(out))
    assert rc == 0
    assert out.n_clusters == len(want) > 0
    for i, w in enumerate(want):
        c = out.clusters[i]
        assert np.array_equal(_host_copy(c.indices, (c.size,), np.int32), w.indices)
        assert np.array_equal(np.array(list(c.sum_xyz), np.float32), w.sum_xyz)


def test_aos_entry_points_reject_bad_strides_and_take_empty_clouds(ctx):
    a = np.zeros((8, 4), np.float32)
    out, cl = L.SupportList(), L.ClusterList()
    p = pitt.support_params()
    assert L.lib.pitt_find_supports_aos(ctx.h, _fp(a), 8, 8, ctypes.byref(p), ctypes.byref(out)) == L.PITT_E_INVALID
    assert L.lib.pitt_euclidean_clusters_aos(ctx.h, _fp(a), 8, 10, 0.03, 1, 100, ctypes.byref(cl)) == L.PITT_E_INVALID
    assert L.lib.pitt_find_supports_aos(ctx.h, _fp(a), 0, 16, ctypes.byref(p), ctypes.byref(out)) == 0
    assert out.n_supports == 0
    assert L.lib.pitt_euclidean_clusters_aos(ctx.h, _fp(a), 0, 16, 0.03, 1, 100, ctypes.byref(cl)) == 0
    assert cl.n_clusters == 0
