"""Summary of tools/gpu_variants_bench.sh results."""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = os.path.join(ROOT, "gpurun_out")
for f in sorted(glob.glob(os.path.join(g, "vb_*.flags")), key=lambda p: int(re.findall(r"vb_(\d+)", p)[0])):
    i = re.findall(r"vb_(\d+)", f)[0]
    out = [open(f).read().strip()]
    for p in (1, 3):
        try:
            line = [x for x in open(os.path.join(g, f"vb_{i}_p{p}.json")) if x.startswith("{")][-1]
            d = json.loads(line)
            out.append(f"p{p}: {d['value']:.0f} fr/s score avg {d['roofline']['avg_launch_us']} us frac {d['roofline']['frac']}")
        except (OSError, IndexError):
            out.append(f"p{p}: -")
    print(" | ".join(out))
