"""Summarise tools/gpu_ab.sh: frames/s and per-kernel us/batch of A (in-tree) vs B per round.
    python tools/ab_report.py <tag>"""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
for side in "AB":
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"ab_{tag}_{side}*.json"))):
        d = json.load(open(f))
        k = d.get("kernels", {})
        ks = " ".join(f"{n}={v['us_per_batch']}" for n, v in k.items() if n in ("k_score.first", "k_refine", "k_sel_mark"))
        print(f"{side} {os.path.basename(f):20s} {d['value']:10.1f} frames/s  {d['ms_per_step']:.4f} ms  frac {d['roofline']['frac']}  {ks}")
