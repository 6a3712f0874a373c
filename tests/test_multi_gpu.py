"""The C++ host's multi-device path (pitt_multi_*, include/pitt_seg.h).

One host process, one context per listed device, contiguous frame shards, results and inlier lists
gathered on the host in frame order.  On a one-GPU box the devices are the same GPU listed several times
(several contexts on device 0, each shard driven by its own host thread): the gathered records and
inlier lists must be byte-equal to one single-context batch over the same frames, and the frames match
the oracle (test_plane_gpu._check)."""
import ctypes

import numpy as np
import pytest
import torch

import pitt_object_table_segmentation_amd as pitt
from pitt_object_table_segmentation_amd import _lib as L

pytestmark = pytest.mark.gpu


def _frames():
    w, h = 320, 240
    fr = [pitt.synth_frame(s, 3000 + i, w, h) for i, s in enumerate((0, 0, 1, 2, 0, 1, 0))]
    fr.insert(3, tuple(np.zeros(0, np.float32) for _ in range(3)))   # an empty frame
    fr.append(tuple(a[:2049].copy() for a in pitt.synth_frame(0, 3100, w, h)))  # a ragged one
    return fr


def _single(frames):
    with pitt.Context(0) as ctx:
        b = pitt.FrameBatch.from_host(frames, device="cuda:0")
        inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
        res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
        h = inl.cpu().numpy()
        return res, [h[o:o + r["n_inliers"]].copy() for o, r in zip(b.offsets, res)]


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_batch_equals_one_batch(devices):
    frames = _frames()
    want_res, want_inl = _single(frames)
    with pitt.MultiContext(devices) as m:
        assert L.lib.pitt_multi_devices(m.h) == len(devices)
        res, inl = m.plane_segment_batch(frames)
        assert res.tobytes() == want_res.tobytes()
        assert all(np.array_equal(a, b) for a, b in zip(inl, want_inl))
        # a second call on the same contexts (scratch reused, shards re-uploaded)
        res2, inl2 = m.plane_segment_batch(frames[::-1])
        want2, wantl2 = _single(frames[::-1])
        assert res2.tobytes() == want2.tobytes()
        assert all(np.array_equal(a, b) for a, b in zip(inl2, wantl2))


def test_multi_device_against_the_oracle():
    import test_plane_gpu as P
    frames = [pitt.synth_frame(s, 3200 + i) for i, s in enumerate((0, 1, 2, 0))]
    with pitt.MultiContext([0, 0]) as m:
        res, inl = m.plane_segment_batch(frames)
        # the last shard's context holds the last two frames' per-hypothesis counts (its local frames 0, 1)
        ctx1 = pitt.Context.__new__(pitt.Context)
        ctx1.h, ctx1.device = ctypes.c_void_p(L.lib.pitt_multi_context(m.h, 1)), 0
        try:
            P._check(ctx1, frames[2:], res[2:], inl[2:])
        finally:
            ctx1.h = None  # owned by the pitt_multi


def test_multi_device_rejects_overlapping_frames():
    x = np.zeros(8192, np.float32)
    offs = np.array([0, 4], np.int64)
    cnt = np.array([100, 100], np.int64)
    fr = L.Frames(x.ctypes.data, x.ctypes.data, x.ctypes.data, offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                  cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), 2, 8192)
    res = np.zeros(2, pitt.RESULT_DTYPE)
    p = pitt.sac_params()
    with pitt.MultiContext([0, 0]) as m:
        rc = L.lib.pitt_plane_segment_batch_multi(m.h, ctypes.byref(fr), ctypes.byref(p),
                                                  res.ctypes.data_as(ctypes.POINTER(L.PlaneResult)), None)
        assert rc == L.PITT_E_INVALID
        assert b"non-overlapping" in L.lib.pitt_multi_last_error(m.h)
