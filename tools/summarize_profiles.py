"""Turn the rocprofv3 outputs of tools/gpu_profile.sh (merged into gpurun_out/) into the committed
summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_summary.json       per-kernel averages; k_score over bench.py's roofline pass
  profiles/pmc_k_score.json         HBM bytes per k_score launch from the PMC passes:
                                    FETCH_SIZE * 1024 * 2 (gfx950 reports 1/2 of a wide coalesced
                                    stream, MI355X_MICROARCH.md s HBM) + WRITE_SIZE * 1024

bench.py runs a timed pass (batches overlapped on several streams) and then a roofline pass of
`launches` k_score dispatches with one batch in flight; the roofline figures use the last
`launches` k_score dispatches of the trace.

    python tools/summarize_profiles.py r01
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(tag):
    g = os.path.join(ROOT, "gpurun_out")
    trace_dir = os.path.join(g, f"prof_{tag}_trace")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    shutil.copy(os.path.join(trace_dir, "trace_kernel_stats.csv"),
                os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    bench = None
    with open(os.path.join(g, f"prof_{tag}_trace.log")) as f:
        for line in f:
            if line.startswith("{") and '"metric"' in line:
                bench = json.loads(line)
    n_roof = bench["roofline"]["launches"]
    n_empty = bench["roofline"].get("empty_launches", 0)
    tr = rows(os.path.join(trace_dir, "trace_kernel_trace.csv"))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    score = [r for r in tr if "k_score" in r["Kernel_Name"]]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in score]
    # the roofline pass's dispatches; the chunks with no active frame (bench.py lists them apart)
    # are its n_empty shortest
    last = dur[-(n_roof + n_empty):]
    roof = sorted(last)[n_empty:]
    stats = {}
    for r in rows(os.path.join(trace_dir, "trace_kernel_stats.csv")):
        name = r["Name"].split("(")[0].replace("void ", "")
        stats[name] = dict(calls=int(r["Calls"]), avg_us=float(r["AverageNs"]) / 1e3,
                           total_ms=float(r["TotalDurationNs"]) / 1e6, pct=float(r["Percentage"]))
    out = dict(tag=tag, bench=bench, kernels=stats,
               k_score_roofline_pass=dict(launches=len(roof), avg_us=sum(roof) / max(1, len(roof)),
                                          bench_avg_us=bench["roofline"]["avg_launch_us"]),
               k_score_all_dispatches=dict(launches=len(dur), avg_us=sum(dur) / max(1, len(dur))))
    pmc = {}
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(g, f"prof_{tag}_{kind}", f"{kind}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        vals = [float(r["Counter_Value"]) for r in rows(p) if r["Counter_Name"] == counter]
        pmc[counter] = vals[-(n_roof + n_empty):]
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:  # drop the empty chunks (the smallest fetches)
        keep = sorted(range(len(pmc["FETCH_SIZE"])), key=lambda i: pmc["FETCH_SIZE"][i])[n_empty:]
        pmc = {k: [v[i] for i in sorted(keep)] for k, v in pmc.items()}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        per = [f * 1024 * 2 + w * 1024 for f, w in zip(pmc["FETCH_SIZE"], pmc["WRITE_SIZE"])]
        hbm = sum(per) / len(per)
        out["k_score_pmc"] = dict(launches=len(per), fetch_size_kb_avg=sum(pmc["FETCH_SIZE"]) / len(per),
                                  write_size_kb_avg=sum(pmc["WRITE_SIZE"]) / len(per), hbm_bytes_per_launch=hbm,
                                  algorithmic_bytes_per_launch=bench["roofline"]["algorithmic_bytes_per_launch"],
                                  correction="FETCH_SIZE x 1024 x 2 (gfx950 half-count) + WRITE_SIZE x 1024")
        with open(os.path.join(ROOT, "profiles", "pmc_k_score.json"), "w") as f:
            # stamped with the library the passes ran (bench.py prints its sha256): bench.py reports
            # this traffic only for that same build
            json.dump(dict(tag=tag, hbm_bytes_per_launch=round(hbm, 1), launches=len(per),
                           algorithmic_bytes_per_launch=bench["roofline"]["algorithmic_bytes_per_launch"],
                           library_sha16=bench.get("library_sha16")), f, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "bench"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
