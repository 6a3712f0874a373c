"""Per-launch durations of the last batches in a rocprofv3 kernel trace (one batch in flight).

    python tools/batch_seq.py gpurun_out/<tag>_p1 [batches]
"""
import csv
import glob
import os
import re
import sys


def main(d, nb=2):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    seq = []
    for r in rows:
        n = re.sub(r"^void ", "", r["Kernel_Name"]).split("(")[0].replace("pitt::", "")
        if n.startswith("__amd"):
            continue
        d_us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if n.startswith("k_hyp"):
            seq.append([])
        if seq:
            seq[-1].append(f"{n.split('(')[0][:22]} {d_us:.1f}")
    for s in seq[-nb:]:
        print(" | ".join(s))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
