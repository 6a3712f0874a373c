"""Per-kernel durations from tools/gpu_exp.sh traces: first k_score launch (chunk 0, every frame
active) and totals per kernel name, one column per experiment.

    python tools/exp_report.py
"""
import csv
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    g = os.path.join(ROOT, "gpurun_out")
    for d in sorted(glob.glob(os.path.join(g, "exp_[0-9]*")), key=lambda p: int(re.findall(r"\d+", p)[-1])):
        if not os.path.isdir(d):
            continue
        tr = glob.glob(os.path.join(d, "**", "t_kernel_trace.csv"), recursive=True)
        if not tr:
            continue
        flags = open(d + ".flags").read().strip() if os.path.exists(d + ".flags") else "?"
        rows = list(csv.DictReader(open(tr[0])))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        per = {}
        for r in rows:
            name = re.sub(r"^void ", "", r["Kernel_Name"]).split("(")[0].split("<")[0].replace("pitt::", "")
            per.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        sc = per.get("k_score", [])
        big = sorted(sc, reverse=True)[:6]
        print(f"{os.path.basename(d)} [{flags}] k_score top6 us: {[round(x, 1) for x in big]}")
        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            print(f"    {k:18s} n={len(v):4d} total={sum(v) / 1e3:8.3f} ms avg={sum(v) / len(v):8.1f} us")


if __name__ == "__main__":
    main()
