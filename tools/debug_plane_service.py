"""Plane service on the classification test's clusters under each plane-path setting (graphs, adaptive
chunk schedule, exact-walk refinement), against the oracle: isolates which setting changes a result.

    python tools/debug_plane_service.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_binding as orc  # noqa: E402
import pitt_object_table_segmentation_amd as pitt  # noqa: E402
from test_classify_gpu import frame_clusters  # noqa: E402


def ctx_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return pitt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    cl = frame_clusters(0)
    want = []
    for P in cl:
        o = orc.plane_segment(*(np.ascontiguousarray(P[:, k]) for k in range(3)))
        want.append((len(o.inliers), o.coefficients.view(np.int32).tolist(), o.hypotheses))
    configs = {"default": {}, "no-adaptive": {"PITT_ADAPTIVE_CHUNKS": "0"}, "no-xs": {"PITT_XS_MAX_FRAMES": "0"},
               "no-graphs": {"PITT_GRAPHS": "0"},
               "none": {"PITT_ADAPTIVE_CHUNKS": "0", "PITT_XS_MAX_FRAMES": "0", "PITT_GRAPHS": "0"}}
    for name, env in configs.items():
        ctx = ctx_with(env)
        srv = pitt.Services(ctx)
        line = []
        for i, P in enumerate(cl):
            ok, inl, coef, _ = srv.ransac_plane(P)
            r = ctx.plane_segment(np.c_[P, np.zeros(len(P), np.float32)])
            got = (len(r.inliers), r.coefficients.view(np.int32).tolist())
            line.append(f"{i}:{'ok' if got[0] == want[i][0] and got[1] == want[i][1] else 'BAD'}({got[0]}/{want[i][0]},"
                        f" srv {len(inl) if ok else 'none'}, stats {ctx.schedule_stats()})")
        print(name, " ".join(line), flush=True)
        srv.close()
        ctx.close()


if __name__ == "__main__":
    main()
