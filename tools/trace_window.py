"""The timed window of bench.py's pipelined pass from a rocprofv3 kernel trace (tools/gpu_trace.sh):
which batches overlap, each batch's kernels and latency, and how many kernels run at once.

    python tools/trace_window.py <trace_kernel_trace.csv> --skip S --steps K [--out profiles/x.json]

S = k_hypothesize launches before the timed steps (setup 2 per context + the oracle spot check's 1 +
settle + warm-up steps), K = timed steps.  Batch j's kernels are those on its queue from its
k_hypothesize to the next k_hypothesize on that queue."""
import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_timeline import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, required=True)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    ks = load(a.csv)
    hyp = [i for i, k in enumerate(ks) if k["name"] == "k_hypothesize"]
    T = hyp[a.skip:a.skip + a.steps]
    t0 = ks[T[0]]["s"]
    batches = []
    for j, hi in enumerate(T):
        q = ks[hi]["q"]
        seq = []
        for k in ks[hi:]:
            if k["q"] != q:
                continue
            if k["name"] == "k_hypothesize" and seq:
                break
            if k["name"].startswith("__amd_rocclr_fill"):  # the next batch's first memset on this queue
                break
            seq.append(k)
        batches.append(dict(batch=j, queue=q, start_us=round((seq[0]["s"] - t0) / 1e3, 1),
                            end_us=round((seq[-1]["e"] - t0) / 1e3, 1),
                            latency_us=round((seq[-1]["e"] - seq[0]["s"]) / 1e3, 1),
                            kernels=[[k["name"], round((k["s"] - t0) / 1e3, 1), round((k["e"] - k["s"]) / 1e3, 1)]
                                     for k in seq]))
    t1 = t0 + 1e3 * max(b["end_us"] for b in batches)
    body = [k for k in ks if k["s"] >= t0 and k["e"] <= t1]
    ev = sorted([(k["s"], 1) for k in body] + [(k["e"], -1) for k in body])
    hist = collections.Counter()
    n, last = 0, ev[0][0]
    for t, d in ev:
        hist[n] += t - last
        n += d
        last = t
    tot = sum(hist.values())
    starts = [b["start_us"] for b in batches]
    out = {
        "window_us": round((t1 - t0) / 1e3, 1),
        "steps": a.steps,
        "ms_per_step_window": round((t1 - t0) / 1e6 / a.steps, 4),
        "batch_period_us_mean": round((starts[-1] - starts[0]) / (len(starts) - 1), 1),
        "last_batch_latency_us": batches[-1]["latency_us"],
        "queues": sorted({b["queue"] for b in batches}),
        "concurrency_share": {str(k): round(v / tot, 3) for k, v in sorted(hist.items())},
        "batches": batches,
    }
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "batches"}, indent=1))


if __name__ == "__main__":
    main()
