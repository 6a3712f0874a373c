"""Timeline analysis of a rocprofv3 kernel trace of bench.py's timed pass (several streams):
per-queue busy time, overlap, and per-kernel totals inside a window.

    python tools/timeline.py gpurun_out/prof_<tag>/.../trace_kernel_trace.csv [t0_frac t1_frac]
"""
import csv
import re
import sys


def main(path, f0=0.3, f1=0.7):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        name = re.sub(r"^void ", "", r["Kernel_Name"]).split("(")[0].split("<")[0].replace("pitt::", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", "?"))))
    ev.sort()
    t_begin, t_end = ev[0][0], max(e[1] for e in ev)
    w0 = t_begin + (t_end - t_begin) * f0
    w1 = t_begin + (t_end - t_begin) * f1
    win = [(max(s, w0), min(e, w1), n, q) for s, e, n, q in ev if e > w0 and s < w1]
    span = w1 - w0
    per = {}
    for s, e, n, q in win:
        per[n] = per.get(n, 0) + (e - s)
    # union of busy time (any kernel running)
    busy = 0
    cur_s, cur_e = None, None
    for s, e, n, q in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    # time with a k_score running
    sc = sorted((s, e) for s, e, n, q in win if n == "k_score")
    sbusy = 0
    cs, ce = None, None
    for s, e in sc:
        if ce is None or s > ce:
            if ce is not None:
                sbusy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        sbusy += ce - cs
    print(f"window {span / 1e6:.3f} ms: any-kernel busy {busy / span:.1%}, k_score running {sbusy / span:.1%}")
    for n, t in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {n:16s} {t / 1e6:8.3f} ms summed ({t / span:6.1%} of window)")
    qs = sorted(set(q for *_, q in win))
    print("queues:", qs)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(float(x) for x in a[1:3]))
