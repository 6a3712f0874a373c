"""Timeline analysis of a rocprofv3 --kernel-trace of bench.py's pipelined pass.

    python tools/trace_timeline.py gpurun_out/prof_<tag>/.../trace_kernel_trace.csv [--steps K]

Batches are delimited by their k_hypothesize launches (one per batch).  For the window of the last
K + pipeline batches of the pipelined pass (before the one-batch roofline pass) it reports:
  * per queue: the batch latency (k_hypothesize start -> k_finalize end) and the idle gaps between a
    batch's kernels and between batches (the host's turnaround);
  * per kernel: launches, mean duration under overlap, and the share of the window it is running;
  * chip: the share of the window with 0, 1, 2, ... kernels running.
"""
import argparse
import collections
import csv
import json
import statistics


def load(path):
    with open(path) as f:
        rows = list(csv.DictReader(f))
    out = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip().split("::")[-1]
        q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
        out.append(dict(name=name, q=q, s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"])))
    out.sort(key=lambda k: k["s"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--batches", type=int, default=24, help="batches of the window (the last of the pipelined pass)")
    ap.add_argument("--skip-tail", type=int, default=10, help="k_hypothesize launches of the roofline pass to skip")
    args = ap.parse_args()
    ks = load(args.csv)
    hyp = [i for i, k in enumerate(ks) if k["name"] == "k_hypothesize"]
    # the pipelined pass's last batches: drop the roofline pass's batches at the end
    cut = hyp[-args.skip_tail] if args.skip_tail else len(ks)
    starts = [i for i in hyp if i < cut][-args.batches:]
    t0 = ks[starts[0]]["s"]
    # window end: the last kernel before the roofline pass
    body = [k for k in ks[starts[0]:cut]]
    t1 = max(k["e"] for k in body)
    # batches: per queue, from a k_hypothesize to the next k_hypothesize on that queue
    perq = collections.defaultdict(list)
    for k in body:
        perq[k["q"]].append(k)
    lat, inner_gap, turn = [], [], []
    for q, seq in perq.items():
        cur = None
        for k in seq:
            if k["name"] == "k_hypothesize":
                if cur:
                    lat.append((cur[-1]["e"] - cur[0]["s"]) / 1e3)
                    turn.append((k["s"] - cur[-1]["e"]) / 1e3)
                cur = [k]
            elif cur is not None:
                inner_gap.append((k["s"] - cur[-1]["e"]) / 1e3)
                cur.append(k)
    # per kernel busy share
    per = collections.defaultdict(lambda: [0, 0.0])
    for k in body:
        per[k["name"]][0] += 1
        per[k["name"]][1] += (k["e"] - k["s"]) / 1e3
    span = (t1 - t0) / 1e3
    # concurrency histogram
    ev = []
    for k in body:
        ev.append((k["s"], 1))
        ev.append((k["e"], -1))
    ev.sort()
    hist = collections.Counter()
    n, last = 0, ev[0][0]
    for t, d in ev:
        hist[n] += t - last
        n += d
        last = t
    tot = sum(hist.values())
    out = {
        "window_us": round(span, 1), "batches": len(starts), "queues": len(perq),
        "us_per_batch": round(span / max(1, len(starts)), 1),
        "batch_latency_us": dict(mean=round(statistics.mean(lat), 1), max=round(max(lat), 1)) if lat else None,
        "gap_between_kernels_of_a_batch_us": dict(mean=round(statistics.mean(inner_gap), 2),
                                                  sum_per_batch=round(sum(inner_gap) / max(1, len(lat)), 1))
        if inner_gap else None,
        "host_turnaround_us": dict(mean=round(statistics.mean(turn), 1), max=round(max(turn), 1)) if turn else None,
        "kernels": {name: dict(launches=c, mean_us=round(t / c, 1), busy_share=round(t / span, 3))
                    for name, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])},
        "concurrency_share": {str(k): round(v / tot, 3) for k, v in sorted(hist.items())},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
