"""Summary of tools/gpu_trace_variants.sh: per variant, the median chunk-0 k_score duration in the
pipelined timed pass, its median overlap with k_refine, and the k_refine median."""
import csv
import glob
import os
import re
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = os.path.join(ROOT, "gpurun_out")
for d in sorted(glob.glob(os.path.join(g, "tv_[0-9]*")), key=lambda p: int(re.findall(r"tv_(\d+)", p)[0])):
    if not os.path.isdir(d):
        continue
    tr = glob.glob(os.path.join(d, "**", "t_kernel_trace.csv"), recursive=True)
    if not tr:
        continue
    rows = list(csv.DictReader(open(tr[0])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ev = ev[len(ev) // 5: len(ev) * 3 // 5]  # middle of the run: the timed, pipelined pass
    sc = [(s, e) for s, e, n in ev if "k_score" in n and "true" in n]
    refs = [(s, e) for s, e, n in ev if "k_refine" in n]

    def overl(s, e):
        return sum(max(0, min(e, b) - max(s, a)) for a, b in refs)

    flags = open(d + ".flags").read().strip()
    print(f"{os.path.basename(d)} [{flags}] chunk0 k_score median {statistics.median([(e - s) / 1e3 for s, e in sc]):.0f} us, "
          f"refine overlap {statistics.median([overl(s, e) / 1e3 for s, e in sc]):.0f} us, "
          f"k_refine median {statistics.median([(e - s) / 1e3 for s, e in refs]):.0f} us")
