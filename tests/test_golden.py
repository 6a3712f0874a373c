"""Committed golden fixtures (tests/golden/, made by tools/make_golden.py from the oracle):
the oracle must keep reproducing them (CPU), and the HIP path must match them (GPU)."""
import os

import numpy as np
import pytest

import oracle_binding as orc

HERE = os.path.dirname(os.path.abspath(__file__))
PLANE = np.load(os.path.join(HERE, "golden", "plane_golden.npz"))
SUP = np.load(os.path.join(HERE, "golden", "support_golden.npz"))
CASES = sorted({k[:-2] for k in PLANE.files if k.endswith("_x")})


def _cloud(name):
    return PLANE[f"{name}_x"], PLANE[f"{name}_y"], PLANE[f"{name}_z"]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("order", [0, 1])
def test_oracle_reproduces_plane_golden(name, order):
    r = orc.plane_segment(*_cloud(name), reduce_order=order)
    key = f"{name}_o{order}"
    assert np.array_equal(r.inliers, PLANE[f"{key}_inliers"])
    assert np.array_equal(r.coefficients, PLANE[f"{key}_coefficients"])
    assert np.array_equal(r.hyp_counts, PLANE[f"{key}_hyp_counts"])
    assert [r.hypotheses, r.best_hypothesis, r.best_count, r.rejected_samples] == list(PLANE[f"{key}_stats"])


def test_oracle_reproduces_support_golden():
    x, y, z = SUP["x"], SUP["y"], SUP["z"]
    sup = orc.find_supports(x, y, z)
    assert len(sup) == int(SUP["n_supports"][0])
    for i, s in enumerate(sup):
        assert np.array_equal(s["idx_map"], SUP[f"s{i}_idx_map"])
        assert np.array_equal(s["on_support_cloud"], SUP[f"s{i}_on"])
        cl = orc.euclidean_clusters(*s["on_support_cloud"].T)
        assert len(cl) == int(SUP[f"s{i}_n_clusters"][0])
        for j, c in enumerate(cl):
            assert np.array_equal(c["inliers"], SUP[f"s{i}_c{j}_inliers"])


@pytest.mark.gpu
@pytest.mark.parametrize("order", [0, 1])
def test_hip_path_matches_plane_golden(ctx, order):
    import torch
    import pitt_object_table_segmentation_amd as pitt
    frames = [_cloud(n) for n in CASES]
    b = pitt.FrameBatch.from_host(frames)
    inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda")
    res = ctx.plane_segment_batch(b, pitt.sac_params(reduce_order=order), inl)
    inl = inl.cpu().numpy()
    for f, name in enumerate(CASES):
        key = f"{name}_o{order}"
        stats = list(PLANE[f"{key}_stats"])
        assert [res[f]["hypotheses"], res[f]["best_hypothesis"], res[f]["best_count"],
                res[f]["rejected_samples"]] == stats, name
        got = inl[b.offsets[f]:b.offsets[f] + res[f]["n_inliers"]]
        assert np.array_equal(got, PLANE[f"{key}_inliers"]), name
        assert np.array_equal(res[f]["coefficients"][:res[f]["n_coeff"]], PLANE[f"{key}_coefficients"]), name
        assert np.array_equal(ctx.hypothesis_counts(f, stats[0]), PLANE[f"{key}_hyp_counts"]), name


@pytest.mark.gpu
def test_hip_path_matches_support_golden(ctx):
    x, y, z = SUP["x"], SUP["y"], SUP["z"]
    sup = ctx.find_supports(x, y, z)
    assert len(sup) == int(SUP["n_supports"][0])
    for i, s in enumerate(sup):
        assert np.array_equal(s.idx_map, SUP[f"s{i}_idx_map"])
        assert np.array_equal(s.coefficients, SUP[f"s{i}_coefficients"])
        assert np.array_equal(s.support_cloud, SUP[f"s{i}_support"])
        assert np.array_equal(s.on_support_cloud, SUP[f"s{i}_on"])
        n = len(s.on_support_cloud)
        cl = ctx.euclidean_clusters(*s.on_support_cloud.T, 0.03, int(np.floor(n * 0.01 + 0.5)),
                                    int(np.floor(n * 0.99 + 0.5))) if n >= 30 else []
        assert len(cl) == int(SUP[f"s{i}_n_clusters"][0])
        for j, c in enumerate(cl):
            assert np.array_equal(c.indices, SUP[f"s{i}_c{j}_inliers"])
            assert np.array_equal(c.sum_xyz / np.float32(c.indices.size + 1), SUP[f"s{i}_c{j}_centroid"])
