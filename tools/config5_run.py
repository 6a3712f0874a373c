"""BASELINE config 5 on one GPU: find_supports + euclidean_clusters on the 1.2M-point fused scene,
repeated, for rocprofv3 kernel traces (tools/gpu_r03.sh) and quick timing: the device-resident
scene path (pitt_segment_objects_dev) and the host-array service path.

    python tools/config5_run.py [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pitt_object_table_segmentation_amd as pitt  # noqa: E402


def main(reps=5, dev_only=False):
    import torch
    x, y, z = pitt.synth_fused(1000, 4)
    dx, dy, dz = (torch.from_numpy(a).cuda() for a in (x, y, z))
    with pitt.Context(0) as ctx:
        ts = []
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            n_on, sizes = ctx.segment_objects_dev(dx, dy, dz, copy=False)
            if r:
                ts.append((time.perf_counter() - t) * 1e3)
        print(f"config5 device path: {len(n_on)} supports, {len(sizes)} clusters; {np.median(ts):.2f} ms "
              f"(median of {reps})", flush=True)
        if dev_only:
            return
        ts = []
        for r in range(reps + 1):
            t = time.perf_counter()
            sups = ctx.find_supports(x, y, z)
            t1 = time.perf_counter()
            ncl = 0
            for s in sups:
                n = len(s.on_support_cloud)
                if n >= 30:
                    ncl += len(ctx.euclidean_clusters(*s.on_support_cloud.T, tolerance=0.03,
                                                      min_size=int(np.floor(n * 0.01 + 0.5)),
                                                      max_size=int(np.floor(n * 0.99 + 0.5))))
            t2 = time.perf_counter()
            if r:
                ts.append(((t1 - t) * 1e3, (t2 - t1) * 1e3))
        sup_ms = np.median([a for a, _ in ts])
        cl_ms = np.median([b for _, b in ts])
        print(f"config5 host path: {len(sups)} supports, {ncl} clusters; find_supports {sup_ms:.2f} ms, "
              f"clusters {cl_ms:.2f} ms (median of {reps})")
        # the C entry point alone (no Python conversion of its outputs), and the service handler
        import ctypes
        from pitt_object_table_segmentation_amd import _lib as L
        xs, ys, zs = (np.ascontiguousarray(a, np.float32) for a in (x, y, z))
        fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
        out, p = L.SupportList(), pitt.support_params()
        raw = []
        for r in range(reps + 1):
            t = time.perf_counter()
            assert L.lib.pitt_find_supports(ctx.h, fp(xs), fp(ys), fp(zs), len(xs), ctypes.byref(p),
                                            ctypes.byref(out)) == 0
            if r:
                raw.append((time.perf_counter() - t) * 1e3)
        print(f"config5 pitt_find_supports (C ABI call only): {np.median(raw):.2f} ms (median of {reps})")
        ons = [np.ascontiguousarray(s.on_support_cloud.T) for s in sups]
        craw = []
        cout = L.ClusterList()
        for r in range(reps + 1):
            t = time.perf_counter()
            for o in ons:
                n = o.shape[1]
                if n >= 30:
                    assert L.lib.pitt_euclidean_clusters(ctx.h, fp(o[0]), fp(o[1]), fp(o[2]), n, 0.03,
                                                         int(np.floor(n * 0.01 + 0.5)), int(np.floor(n * 0.99 + 0.5)),
                                                         ctypes.byref(cout)) == 0
            if r:
                craw.append((time.perf_counter() - t) * 1e3)
        print(f"config5 pitt_euclidean_clusters (C ABI calls only, {[o.shape[1] for o in ons]} points): "
              f"{np.median(craw):.2f} ms (median of {reps})")
        cloud = np.stack([xs, ys, zs], 1)
        srv = pitt.Services(ctx)
        try:
            # the C++ handler alone, as a ROS node calls it (SegmentationServices::findSupports through the
            # flat ABI on a PointXYZ-layout cloud prepared once; its outputs stay in the service object)
            c16 = np.zeros((len(xs), 4), np.float32)
            c16[:, 0], c16[:, 1], c16[:, 2] = xs, ys, zs
            req = L.SrvSupportRequest()
            for fld in ("min_iterative_cloud_percentual_size", "min_iterative_plane_percentual_size",
                        "variance_threshold_for_horizontal", "ransac_distance_point_in_shape_threshold",
                        "ransac_model_normal_distance_weigth"):
                setattr(req, fld, -1.0)
            req.ransac_max_iteration_threshold = -1
            req.n_horizontal_axis, req.n_edge_remove_offset = 1, 1
            req.horizontal_axis[0] = req.edge_remove_offset[0] = -1.0
            ns, used = ctypes.c_int32(), np.zeros(13, np.float32)
            hv = []
            for r in range(reps + 1):
                t = time.perf_counter()
                rc = L.lib.pitt_srv_find_supports(srv.h, fp(c16), len(xs), len(xs), ctypes.byref(req), ctypes.byref(ns),
                                                  fp(used))
                if r:
                    hv.append((time.perf_counter() - t) * 1e3)
                assert rc >= 0
            print(f"config5 findSupports service handler (C++ SegmentationServices::findSupports, flat ABI call "
                  f"only): {np.median(hv):.2f} ms, {ns.value} supports (median of {reps})")
            sv = []
            for r in range(reps + 1):
                t = time.perf_counter()
                _, res, _ = srv.find_supports(cloud)
                if r:
                    sv.append((time.perf_counter() - t) * 1e3)
            print(f"config5 findSupports service (pitt_srv_find_supports + Python): {np.median(sv):.2f} ms, "
                  f"{len(res)} supports (median of {reps})")
        finally:
            srv.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5, "--dev-only" in sys.argv)
