"""Throughput of the device preprocessing steps on one GPU: PointCloud2
unpacking, deepFiltering and transformPointCloud over a 256-frame batch of synthetic 640x480 camera clouds concatenated into one
78.6M-point cloud, resident in HBM.  Prints one JSON line: per-kernel average duration (HIP events),
algorithmic bytes and the fraction of the 8 TB/s HBM peak, plus a CPU (oracle) sample for scale.

    python tools/bench_preprocess.py [--frames 256] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pitt_object_table_segmentation_amd as pitt  # noqa: E402

PEAK = 8000.0  # GB/s, MI355X HBM3E spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    n1 = 640 * 480
    x = np.empty(args.frames * n1, np.float32)
    y = np.empty_like(x)
    z = np.empty_like(x)
    for f in range(min(args.frames, 16)):  # 16 distinct frames, cycled
        fx, fy, fz = pitt.synth_frame(2 if f % 4 == 3 else 0, 1000 + f)
        x[f * n1:(f + 1) * n1], y[f * n1:(f + 1) * n1], z[f * n1:(f + 1) * n1] = fx, fy, fz
    for f in range(16, args.frames):
        s = f % 16
        x[f * n1:(f + 1) * n1], y[f * n1:(f + 1) * n1], z[f * n1:(f + 1) * n1] = (
            x[s * n1:(s + 1) * n1], y[s * n1:(s + 1) * n1], z[s * n1:(s + 1) * n1])
    n = len(x)
    dx, dy, dz = (torch.from_numpy(a).cuda() for a in (x, y, z))
    m = np.eye(4, dtype=np.float32)
    m[:3, :3] = [[0.9986, -0.0523, 0.0], [-0.0300, -0.5726, -0.8192], [0.0428, 0.8181, -0.5736]]
    m[:3, 3] = [0.01, -0.02, 1.37]
    aos = torch.stack([dx, dy, dz, torch.zeros_like(dx)], 1).contiguous().view(torch.uint8).reshape(-1)
    with pitt.Context(0) as ctx:
        ux, uy, uz = ctx.unpack_pointcloud2(aos, n1, n // n1, 16, n1 * 16)  # PointXYZ payload -> SoA
        assert all(torch.equal(u.view(torch.int32), d.view(torch.int32)) for u, d in ((ux, dx), (uy, dy), (uz, dz)))
        closer, further, used = ctx.deep_filter(dx, dy, dz)  # warm-up (buffers)
        ctx.transform_cloud(dx, dy, dz, m)
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(args.reps):
            ctx.unpack_pointcloud2(aos, n1, n // n1, 16, n1 * 16)
            closer, further, used = ctx.deep_filter(dx, dy, dz)
            ctx.transform_cloud(dx, dy, dz, m)
        torch.cuda.synchronize()
        kept = len(closer[0]) + len(further[0])
        res = {}
        for k, extra in (("k_unpack_pc2", 0.0), ("k_deep_count", 0.0), ("k_scan_pair", 0.0),
                         ("k_deep_write", 12.0 * kept), ("k_transform", 0.0)):
            launches, ms, algo = ctx.profile_get(k)
            per = ms / launches * 1e3
            byts = algo / launches + extra
            res[k] = {"avg_us": round(per, 1), "algorithmic_bytes": byts,
                      "GB_s": round(byts / per / 1e3, 1), "frac": round(byts / per / 1e3 / PEAK, 3)}
        ctx.profile(False)
        # VoxelGrid 1 cm, one 640x480 frame per call as downSampling runs it (16 distinct frames)
        frames = [tuple(t[f * n1:(f + 1) * n1] for t in (dx, dy, dz)) for f in range(min(16, args.frames))]
        for fr in frames:
            ctx.voxel_grid(*fr)
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        vox_reps = 4
        for _ in range(vox_reps):
            for fr in frames:
                (vx, _, _), _ = ctx.voxel_grid(*fr)
        torch.cuda.synchronize()
        vox_ms = (time.perf_counter() - t0) * 1e3 / (vox_reps * len(frames))
        vox = {"ms_per_frame_wall": round(vox_ms, 4), "leaves_last_frame": int(vx.numel()), "kernels": {}}
        for k in ("k_vox_minmax", "k_vox_keys", "vox_introsort", "vox_radix_sort", "k_vox_runs", "k_vox_centroid"):
            launches, ms, algo = ctx.profile_get(k)
            if launches:
                vox["kernels"][k] = {"avg_us": round(ms / launches * 1e3, 1)}
        ctx.profile(False)
        # the same frames in stable order (PITT_VOXEL_ORDER_STABLE: no introsort partitions)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(vox_reps):
            for fr in frames:
                ctx.voxel_grid(*fr, order=pitt._lib.PITT_VOXEL_ORDER_STABLE)
        torch.cuda.synchronize()
        vox["stable_order_ms_per_frame_wall"] = round((time.perf_counter() - t0) * 1e3 / (vox_reps * len(frames)), 4)
        # NormalEstimation k = 50 on the voxelized frames (estimateNormal's input, obj_segmentation.cpp:253)
        vframes = [ctx.voxel_grid(*fr)[0] for fr in frames]
        for vf in vframes[:2]:
            ctx.normal_estimation(*vf)
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        for vf in vframes:
            ctx.normal_estimation(*vf)
        torch.cuda.synchronize()
        nrm = {"ms_per_frame_wall": round((time.perf_counter() - t0) * 1e3 / len(vframes), 4),
               "points_per_frame": int(vframes[0][0].numel()), "k": 50, "kernels": {}}
        for kname in ("k_nrm_grid", "k_knn", "k_normals"):
            launches, ms, algo = ctx.profile_get(kname)
            if launches:
                nrm["kernels"][kname] = {"avg_us": round(ms / launches * 1e3, 1)}
        ctx.profile(False)
        # cylinder / cone post-processing: the O(n^2) axis "height" search on object-sized clusters
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_axis_height import cylinder_cloud
        axis = {}
        for na in (5000, 50000):
            pa, coef = cylinder_cloud(na, na)
            ta = [torch.from_numpy(np.ascontiguousarray(pa[:, k])).cuda() for k in range(3)]
            ctx.axis_height(*ta, coef)
            torch.cuda.synchronize()
            ctx.profile(True)
            ctx.profile_reset()
            t0 = time.perf_counter()
            for _ in range(5):
                ctx.axis_height(*ta, coef)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3 / 5
            pairs = na * (na - 1) / 2
            e = {"ms_per_call_wall": round(wall, 3), "pairs": pairs, "kernels": {}}
            for kname in ("k_axis_project", "k_pair_max", "k_pair_first"):
                launches, ms, algo = ctx.profile_get(kname)
                if launches:
                    us = ms / launches * 1e3
                    e["kernels"][kname] = {"avg_us": round(us, 1)}
                    if kname == "k_pair_max":  # 8 VALU ops per pair (3 sub, 3 mul, 2 add; + 1 max) vs 78.6 Tops/s
                        e["kernels"][kname]["valu_frac"] = round(pairs * 8 / (us * 1e-6) / 78.6e12, 3)
            ctx.profile(False)
            axis[str(na)] = e
        # sphere service: RANSAC (radius limits) + refinement on object-sized clusters with clutter
        from test_sphere import sphere_scene
        sph = {}
        for ns, no in ((4000, 1000), (40000, 10000)):
            ps = sphere_scene(ns, no, 7)
            ts = [torch.from_numpy(np.ascontiguousarray(ps[:, k])).cuda() for k in range(3)]
            ctx.sphere_segment(*ts)
            torch.cuda.synchronize()
            ctx.profile(True)
            ctx.profile_reset()
            t0 = time.perf_counter()
            for _ in range(5):
                inl_s, coef_s, hyp_s = ctx.sphere_segment(*ts)
            torch.cuda.synchronize()
            e = {"ms_per_call_wall": round((time.perf_counter() - t0) * 1e3 / 5, 3), "points": ns + no,
                 "hypotheses": hyp_s, "inliers": int(inl_s.numel()), "kernels": {}}
            for kname in ("k_sph_model", "k_sph_count", "k_sph_lm"):
                launches, ms, algo = ctx.profile_get(kname)
                if launches:
                    e["kernels"][kname] = {"launches_per_call": launches / 5, "avg_us": round(ms / launches * 1e3, 1)}
            ctx.profile(False)
            sph[str(ns + no)] = e
        # cylinder / cone services: RANSAC with normals + refinement on object-sized clusters with clutter
        from test_cylinder import cylinder_scene
        from test_cone import cone_scene
        prim = {}
        for name, scene, fn, knames in (
                ("cylinder_segment", cylinder_scene, ctx.cylinder_segment, ("k_cyl_model", "k_cyl_count", "k_cyl_lm")),
                ("cone_segment", cone_scene, ctx.cone_segment, ("k_cone_model", "k_cone_count", "k_cone_lm"))):
            prim[name] = {}
            for ns, no in ((4000, 1000), (40000, 10000)):
                P, N, _ = scene(ns, no, 7)
                ts = [torch.from_numpy(np.ascontiguousarray(a[:, k])).cuda() for a in (P, N) for k in range(3)]
                fn(*ts)
                torch.cuda.synchronize()
                ctx.profile(True)
                ctx.profile_reset()
                t0 = time.perf_counter()
                for _ in range(5):
                    inl_c, coef_c, hyp_c = fn(*ts)
                torch.cuda.synchronize()
                e = {"ms_per_call_wall": round((time.perf_counter() - t0) * 1e3 / 5, 3), "points": ns + no,
                     "hypotheses": hyp_c, "inliers": int(inl_c.numel()), "kernels": {}}
                for kname in knames:
                    launches, ms, algo = ctx.profile_get(kname)
                    if launches:
                        e["kernels"][kname] = {"launches_per_call": launches / 5,
                                               "avg_us": round(ms / launches * 1e3, 1)}
                ctx.profile(False)
                prim[name][str(ns + no)] = e
    import oracle_binding as orc
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < 3.0:
        sl = slice((k % 16) * n1, (k % 16 + 1) * n1)
        rc, rf = orc.deep_filter(x[sl], y[sl], z[sl], used)
        orc.transform_cloud(*rc.T, m)
        k += 1
    cpu = k * n1 / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for f in range(4):
        orc.voxel_grid(*(a[f * n1:(f + 1) * n1] for a in (x, y, z)))
    vox["cpu_oracle_ms_per_frame_1thread"] = round((time.perf_counter() - t0) * 1e3 / 4, 2)
    v0, _ = orc.voxel_grid(x[:n1], y[:n1], z[:n1])
    t0 = time.perf_counter()
    orc.normal_estimation(*v0.T)
    nrm["cpu_oracle_ms_per_frame_1thread"] = round((time.perf_counter() - t0) * 1e3, 1)
    pa, coef = cylinder_cloud(5000, 5000)
    t0 = time.perf_counter()
    orc.axis_height(*pa.T, coef)
    axis["5000"]["cpu_oracle_ms_1thread"] = round((time.perf_counter() - t0) * 1e3, 1)
    ps = sphere_scene(4000, 1000, 7)
    t0 = time.perf_counter()
    orc.sphere_segment(*ps.T)
    sph["5000"]["cpu_oracle_ms_1thread"] = round((time.perf_counter() - t0) * 1e3, 1)
    for name, scene, fn in (("cylinder_segment", cylinder_scene, orc.cylinder_segment),
                            ("cone_segment", cone_scene, orc.cone_segment)):
        for ns, no in ((4000, 1000), (40000, 10000)):
            P, N, _ = scene(ns, no, 7)
            t0 = time.perf_counter()
            fn(P, N)
            prim[name][str(ns + no)]["cpu_oracle_ms_1thread"] = round((time.perf_counter() - t0) * 1e3, 1)
    print(json.dumps({"workload": f"{args.frames} x 640x480 synthetic camera clouds ({n} points), deep filter "
                                  f"(th {used}) + transform, PointXYZ unpack, {args.reps} reps", "points": n, "kept": kept,
                      "kernels": res, "cpu_oracle_points_per_s_1thread": round(cpu), "voxel_grid": vox, "normal_estimation": nrm,
                      "axis_height": axis, "sphere_segment": sph, **prim,
                      "gpu_points_per_s": round(n / (sum(r["avg_us"] for r in res.values()) * 1e-6))}))


if __name__ == "__main__":
    main()
