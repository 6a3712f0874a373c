"""Generate the committed golden fixtures under tests/golden/ from the oracle (CPU restatement of
the reference's PCL path).  Inputs are deterministic synthetic clouds plus hand-built analytic
cases; expected outputs are the oracle's.  Re-run only when the oracle semantics change:

    python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_binding as orc  # noqa: E402
from pitt_object_table_segmentation_amd import api  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def plane_cases():
    cases = {}
    # small organised synthetic clouds (80x60 = 4800 points)
    for name, scene, seed in (("table_a", 0, 1000), ("table_b", 0, 1007), ("clutter", 1, 1003), ("table_nan", 2, 1001)):
        cases[name] = api.synth_frame(scene, seed, 80, 60)
    # analytic: 2000 points exactly on z = 0.5 (a grid) + 500 far outliers
    g = np.stack(np.meshgrid(np.arange(50) * 0.01, np.arange(40) * 0.01), -1).reshape(-1, 2).astype(np.float32)
    rng = np.random.default_rng(7)
    out = rng.uniform(-1, 1, (500, 3)).astype(np.float32)
    out[:, 2] += 2.0
    xyz = np.concatenate([np.c_[g, np.full(len(g), 0.5, np.float32)], out])
    perm = rng.permutation(len(xyz))
    xyz = xyz[perm]
    cases["analytic_plane"] = (xyz[:, 0].copy(), xyz[:, 1].copy(), xyz[:, 2].copy())
    # duplicates: many identical points force isSampleGood rejections (0/0 ratios are NaN = good,
    # exact duplicates of a pair with a third distinct point give 0 ratios = rejected)
    base = rng.uniform(0, 1, (60, 3)).astype(np.float32)
    dup = np.repeat(base, 8, axis=0)
    cases["duplicates"] = (dup[:, 0].copy(), dup[:, 1].copy(), dup[:, 2].copy())
    return cases


def main():
    os.makedirs(OUT, exist_ok=True)
    arrays = {}
    for name, (x, y, z) in plane_cases().items():
        for order in (orc.REDUCE_SSE2, orc.REDUCE_HADD):
            r = orc.plane_segment(x, y, z, reduce_order=order)
            key = f"{name}_o{order}"
            arrays[f"{key}_inliers"] = r.inliers
            arrays[f"{key}_coefficients"] = r.coefficients
            arrays[f"{key}_stats"] = np.array([r.hypotheses, r.best_hypothesis, r.best_count, r.rejected_samples],
                                              np.int64)
            arrays[f"{key}_hyp_counts"] = r.hyp_counts
        arrays[f"{name}_x"], arrays[f"{name}_y"], arrays[f"{name}_z"] = x, y, z
    np.savez_compressed(os.path.join(OUT, "plane_golden.npz"), **arrays)

    # supports + clusters on a small fused scene (2 views of 96x72)
    x, y, z = api.synth_fused(2024, 2, 96, 72)
    sup = orc.find_supports(x, y, z)
    arr = dict(x=x, y=y, z=z, n_supports=np.array([len(sup)]))
    for i, s in enumerate(sup):
        arr[f"s{i}_idx_map"] = s["idx_map"]
        arr[f"s{i}_coefficients"] = s["coefficients"]
        arr[f"s{i}_support"] = s["support_cloud"]
        arr[f"s{i}_on"] = s["on_support_cloud"]
        cl = orc.euclidean_clusters(*s["on_support_cloud"].T)
        arr[f"s{i}_n_clusters"] = np.array([len(cl)])
        for j, c in enumerate(cl):
            arr[f"s{i}_c{j}_inliers"] = c["inliers"]
            arr[f"s{i}_c{j}_centroid"] = c["centroid"]
    np.savez_compressed(os.path.join(OUT, "support_golden.npz"), **arr)
    for f in ("plane_golden.npz", "support_golden.npz"):
        print(f, os.path.getsize(os.path.join(OUT, f)), "bytes")


if __name__ == "__main__":
    main()
