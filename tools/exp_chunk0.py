"""Chunk-0 k_score durations (the first k_score after each k_hypothesize: every frame active)
per tools/gpu_exp.sh experiment directory.

    python tools/exp_chunk0.py
"""
import csv
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "exp_[0-9]*")), key=lambda p: int(re.findall(r"\d+", p)[-1])):
    if not os.path.isdir(d):
        continue
    tr = glob.glob(os.path.join(d, "**", "t_kernel_trace.csv"), recursive=True)
    if not tr:
        continue
    rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    c0, seen = [], False
    for r in rows:
        if "k_hypothesize" in r["Kernel_Name"]:
            seen = True
        elif "k_score" in r["Kernel_Name"] and seen:
            c0.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            seen = False
    flags = open(d + ".flags").read().strip() if os.path.exists(d + ".flags") else "?"
    print(f"{os.path.basename(d)} [{flags}] chunk-0 k_score us: {[round(x, 1) for x in c0]}")
