"""Per-dispatch SQ counters of tools/gpu_sq.sh runs: the largest dispatch of the kernel (the first
scoring chunk for k_score), its instruction mix and issue utilisation.

    python tools/sq_report.py <tag> [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(tag, part, kern):
    fs = glob.glob(os.path.join(ROOT, "gpurun_out", f"sq_{tag}_{part}", "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(dict)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            key = int(r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            per[key]["_grid"] = int(r.get("Grid_Size", 0) or 0)
    return per


def main(tag, kern="k_score"):
    a, b = load(tag, "a", kern), load(tag, "b", kern)
    c = load(tag, "c", kern)
    # the dispatch with the most waves in pass b, matched in pass a by grid size and order
    big_b = max(b.values(), key=lambda d: d.get("SQ_WAVES", 0))
    big_a = max(a.values(), key=lambda d: d.get("SQ_WAVE_CYCLES", 0))
    d = dict(big_a)
    d.update(big_b)
    if c:
        big_c = max(c.values(), key=lambda d: d.get("SQ_WAVE_CYCLES", 0))
        d.update({k + ("" if k not in d else "_c"): v for k, v in big_c.items()})
    for k in sorted(d):
        print(f"  {k:24s} {d[k]:16.0f}")
    cu = 256
    gui = d.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over 8 XCDs
    if gui:
        print(f"  kernel cycles (GRBM_GUI_ACTIVE/8)   {gui:.0f}")
        print(f"  VALU issue share per SIMD          {d['SQ_INSTS_VALU'] * 2 / (cu * 4) / gui:.3f}  (2 cycles per wave64 VALU)")
        print(f"  SALU issue share per CU            {d['SQ_INSTS_SALU'] / cu / gui:.3f}  (1 per cycle per CU)")
        print(f"  SQ_ACTIVE_INST_VALU/WAVE_CYCLES    {d.get('SQ_ACTIVE_INST_VALU', 0) / max(1, d.get('SQ_WAVE_CYCLES', 1)):.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
