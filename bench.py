"""Benchmark of the MI355X RANSAC-plane path (BASELINE.json metric).

One step = one batch of synthetic 640x480 table-scene clouds per GPU (256 by default, BASELINE
config 3) through pitt_plane_segment_batch: hypotheses, adaptive RANSAC scoring, refinement and
the final ascending inlier list, results on the host; with N > 1 ranks the per-frame result
records are gathered over RCCL (config 4).  Inputs are resident in HBM before the timed region;
each in-flight context segments its own batch (distinct frames, no cross-batch cache reuse).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-gpu B] [--settle-steps S]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

The K timed steps are bracketed by a barrier and torch.cuda.synchronize() on both sides and timed as
the max over ranks.  The same K-step window is timed twice: first after only the W warm-up steps (the
GPU from idle: `value_without_settle`), then after S untimed pipelined settle steps (default 300,
~0.2 s) and the W warm-up steps again (`value`): the first tens of milliseconds of pipelined work after
an idle GPU run ~10 % slower per step.  `untimed_steps` counts every pipelined step
run before the timed window.

Prints ONE JSON line on rank 0.  Besides the headline value it carries (rank 0, N = 1):
  roofline      k_score, the inlier-scoring kernel: algorithmic bytes (12 B per point of every
                (active frame, tile) a launch reads) / its average launch time, HIP events on its
                stream over a pass with one batch in flight
  kernels       every kernel of the batch with the bytes it actually moved (device-counted for
                the data-dependent ones) and its launch time
  clutter       a clutter-scene batch (T = 1001 hypotheses per frame) against the VALU roof
  pcie_fed      frames/s when every batch starts in pinned host memory (H2D copy in the step)
  streaming     every step's buffers receive new frames (a clutter-bearing batch among them): frames/s,
                continuations per 100 batches
  config2       one cloud through the single-cloud ABI (host in, host out), median latency
  config5       find_supports + euclidean_clusters on the 1.2M-point fused scene, GPU vs oracle
  cpu_baseline  the oracle (CPU restatement of PCL's path) on the host: frame-parallel on the
                host's CPU share, and single-core per-frame medians (config 1)
  steady_state  (K < 200) the same pipelined step over 200 timed steps right after the headline's
"""
import argparse
import concurrent.futures as cf
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "RANSAC frames/sec on 307k-pt clouds @1/2/4/8 GPU; inlier-kernel HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
# non-FMA f32 VALU ops/s: 256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz (157.3 TFLOPS counts an FMA as 2)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
W, H = 640, 480
KERNELS = ("k_hypothesize", "k_score", "k_score.first", "k_score:empty", "k_replay", "k_refine", "k_sel_mark",
           "k_sel_write")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpus():
    """CPUs of this host and the share this process may use: sched affinity, the cgroup CPU quota,
    and OMP_NUM_THREADS (the GPU box sets it to the box's CPU share)."""
    info = {"affinity": len(os.sched_getaffinity(0))}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("CPU(s):"):
                info["lscpu"] = int(ln.split(":")[1])
            elif ln.startswith("Model name:"):
                info["model"] = ln.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError, ValueError):
        pass
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_quota"] = round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    share = info["affinity"]
    if "cgroup_quota" in info:
        share = min(share, max(1, math.floor(info["cgroup_quota"])))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        share = min(share, int(os.environ["OMP_NUM_THREADS"]))
    info["share"] = max(1, share)
    return info


def make_frames(ids, threads, scene=None):
    import pitt_object_table_segmentation_amd as pitt
    scene = pitt.SCENE_TABLE if scene is None else scene
    with cf.ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL
        return list(ex.map(lambda i: pitt.synth_frame(scene, 1000 + int(i), W, H), ids))


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_binding as orc
    return orc


def cpu_baseline(frames, clutter_frame, cpus, budget_s):
    """The oracle (CPU restatement of the reference's PCL path): frame-parallel over the host's CPU
    share for ~budget_s, then single-core per-frame medians of 5 repeats after 1 warm-up."""
    orc = oracle()
    threads = cpus["share"]
    done = 0
    t0 = time.perf_counter()

    def one(k):
        orc.plane_segment(*frames[k % len(frames)])
        return 1

    with cf.ThreadPoolExecutor(threads) as ex:
        k = 0
        while time.perf_counter() - t0 < budget_s:
            done += sum(ex.map(one, range(k, k + threads * 4)))
            k += threads * 4
    dt = time.perf_counter() - t0

    def median_ms(fr, reps=5):
        orc.plane_segment(*fr)
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            o = orc.plane_segment(*fr)
            ts.append((time.perf_counter() - t) * 1e3)
        return round(float(np.median(ts)), 2), o.hypotheses

    table_ms, table_t = median_ms(frames[0])
    clutter_ms, clutter_t = median_ms(clutter_frame)
    return dict(value=round(done / dt, 2), unit="frames/s", cores=threads, kind="port",
                sample=f"{done} frames cycled over the first {len(frames)} synthetic 640x480 table frames, "
                       f"{dt:.1f} s wall, frame-parallel over {threads} threads = the host's CPU share "
                       f"(oracle/pitt_oracle.cpp, g++ -O2, PCL-equivalent single-threaded segment() per frame)",
                single_core={"config1_table_ms_per_frame": table_ms, "table_hypotheses": int(table_t),
                             "clutter_ms_per_frame": clutter_ms, "clutter_hypotheses": int(clutter_t),
                             "statistic": "median of 5 after 1 warm-up, one thread"},
                host=cpus)


def library_sha16():
    """sha256 (16 hex) of the libpitt_seg.so this process runs: the stamp that ties a PMC summary to
    the build it measured."""
    import hashlib
    from pitt_object_table_segmentation_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_traffic(lib_sha):
    """Per-launch HBM bytes of k_score from the committed rocprofv3 PMC summary, when that summary was
    measured on this very library build (its `library_sha16` stamp); otherwise (None, reason)."""
    path = os.path.join(ROOT, "profiles", "pmc_k_score.json")
    if not os.path.exists(path):
        return None, "no PMC summary (profiles/pmc_k_score.json)"
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"unreadable PMC summary: {e}"
    stamp = pmc.get("library_sha16")
    if stamp != lib_sha:
        return None, (f"PMC summary {pmc.get('tag')} measured library {stamp}, this run's library is {lib_sha}: "
                      "not this build's traffic")
    return pmc.get("hbm_bytes_per_launch"), f"PMC summary {pmc.get('tag')}, same library build"


def kernel_table(ctx, batches):
    out = {}
    for k in KERNELS:
        n, ms, b = ctx.profile_get(k)
        if n == 0:
            continue
        out[k] = {"launches_per_batch": round(n / batches, 2), "us_per_batch": round(ms / batches * 1e3, 1),
                  "avg_launch_us": round(ms / n * 1e3, 1), "GBps": round(b / max(1e-9, ms) / 1e6, 1)}
    return out


def clutter_pass(pitt, ctx, dev, threads, frames_n=64, steps=3):
    """BASELINE sec. 3: the clutter scene (table on ~8 % of pixels) runs all 1001 hypotheses per frame;
    algorithmic VALU work = 1001 x 7 ops (3 mul, 3 add, compare) x 307,200 points per frame."""
    import torch
    frames = make_frames(range(frames_n), threads, pitt.SCENE_CLUTTER)
    b = pitt.FrameBatch.from_host(frames, device=dev)
    out = torch.empty(b.capacity, dtype=torch.int32, device=dev)
    p = pitt.sac_params()
    res = ctx.plane_segment_batch(b, p, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = ctx.plane_segment_batch(b, p, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    hyps = float(np.mean(res["hypotheses"]))
    ops = hyps * 7 * W * H
    achieved = ops * frames_n / dt / 1e12
    return frames, {"frames": frames_n, "frames_per_s": round(frames_n / dt, 1),
                    "ms_per_batch": round(dt * 1e3, 3), "hypotheses_per_frame_mean": round(hyps, 1),
                    "valu_roof": {"ops_per_frame": round(ops), "achieved_Tops": round(achieved, 2),
                                  "peak_Tops": round(VALU_PEAK_TOPS, 1), "frac": round(achieved / VALU_PEAK_TOPS, 4),
                                  "note": "algorithmic ops (every point x every hypothesis); the kernel culls "
                                          "(group, hypothesis) pairs by certified box tests, so it executes fewer"}}


def cov_fast_pass(pitt, ctx, batches, outs, params, step, drain, steps, frames_per_batch):
    """SURVEY A6's fast covariance mode (PITT_COV_FAST: tree-reduced double sums instead of PCL's
    nine sequential float chains), reported beside the exact-order headline: frames/s over the same
    pipelined steps, and on batch 0 the max |coefficient difference| and the final-inlier differences
    against the exact mode.  Exact order stays the default and the parity path."""
    import torch
    fast = pitt.sac_params(cov_mode=pitt.COV_FAST)
    # every context sees the fast layout twice before timing (arena and chunk hint settle), as the
    # main pass primes its contexts
    for _ in range(2 * len(batches)):
        step(fast)
    drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(fast)
    drain()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    b = batches[0]
    out_e = torch.empty(b.capacity, dtype=torch.int32, device=b.x.device)
    out_f = torch.empty(b.capacity, dtype=torch.int32, device=b.x.device)
    re = ctx.plane_segment_batch(b, params, out_e)
    rf = ctx.plane_segment_batch(b, fast, out_f)
    he, hf = out_e.cpu().numpy(), out_f.cpu().numpy()
    xor = [len(np.setxor1d(he[o:o + a], hf[o:o + c])) for o, a, c in zip(b.offsets, re["n_inliers"], rf["n_inliers"])]
    return {"frames_per_s": round(frames_per_batch * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 4),
            "max_abs_dcoef_vs_exact": float(np.max(np.abs(re["coefficients"] - rf["coefficients"]))),
            "frames_coef_bit_equal": int(np.sum(np.all(re["coefficients"] == rf["coefficients"], axis=1))),
            "frames_inliers_differ": int(np.count_nonzero(xor)), "max_inlier_xor": int(max(xor)),
            "frames": int(len(re)), "note": "not the parity path: the headline value is exact order"}


def pcie_pass(pitt, ctxs, host_batches, dev, params, steps):
    """Every step's batch starts in pinned host memory: H2D copy on the context's stream, then the
    batch; the copy of one batch overlaps the kernels of the others."""
    import torch
    streams = [torch.cuda.Stream(device=dev) for _ in ctxs]
    dev_planes = []
    for hb in host_batches:
        dev_planes.append([torch.empty_like(t, device=dev) for t in (hb.x, hb.y, hb.z)])
    outs = [torch.empty(hb.capacity, dtype=torch.int32, device=dev) for hb in host_batches]
    for c, s in zip(ctxs, streams):
        c.set_stream(s)
    pending = [False] * len(ctxs)

    def step(i):
        j = i % len(ctxs)
        c, s, hb = ctxs[j], streams[j], host_batches[j]
        if pending[j]:
            c.wait()
        with torch.cuda.stream(s):
            for d, h in zip(dev_planes[j], (hb.x, hb.y, hb.z)):
                d.copy_(h, non_blocking=True)
        b = pitt.FrameBatch(dev_planes[j][0], dev_planes[j][1], dev_planes[j][2], hb.offsets, hb.counts, hb.capacity)
        c.plane_segment_batch_async(b, params, outs[j])
        pending[j] = True

    for i in range(len(ctxs)):
        step(i)
    for j, c in enumerate(ctxs):
        c.wait()
        pending[j] = False
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    for j, c in enumerate(ctxs):
        if pending[j]:
            c.wait()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for c in ctxs:
        c.set_stream(None)
    frames = sum(hb.n_frames for hb in host_batches) // len(host_batches)
    nbytes = sum(t.numel() * 4 for t in (host_batches[0].x, host_batches[0].y, host_batches[0].z))
    return {"frames_per_s": round(frames * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
            "h2d_bytes_per_batch": nbytes, "h2d_GBps": round(nbytes * steps / dt / 1e9, 1), "steps": steps}


def streaming_pass(pitt, ctxs, batches, dev, threads, params, steps, clutter_per_batch=8, pool_n=5):
    """The streaming case a drop-in sees: every step's batch buffers receive new
    frames.  A pool of `pool_n` distinct batches is staged in HBM; pool batch 0 holds `clutter_per_batch`
    clutter frames (T = 1001) among its table frames, the others table frames only, so 1 batch in
    `pool_n` needs the whole chunk schedule.  Step i copies pool batch i % pool_n into the buffers of
    context i % len(ctxs) (a device-to-device copy on that context's stream, ahead of its batch), so a
    context's buffers hold new content at every use.  Reported: frames/s with the copies inside the
    steps, the copies' own time (a copy-only pass), continuations per 100 batches."""
    import torch
    B = batches[0].n_frames
    rng = np.random.default_rng(77)
    clutter_at = set(rng.choice(B, clutter_per_batch, replace=False).tolist())
    pool = []
    for q in range(pool_n):
        ids = range(20000 + q * B, 20000 + (q + 1) * B)
        fr = make_frames(ids, threads)
        if q == 0:
            cl = make_frames([20000 + q * B + f for f in sorted(clutter_at)], threads, pitt.SCENE_CLUTTER)
            for f, c in zip(sorted(clutter_at), cl):
                fr[f] = c
        pool.append(pitt.FrameBatch.from_host(fr, device=dev))
    assert all(p.capacity == batches[0].capacity and list(p.offsets) == list(batches[0].offsets) for p in pool)
    streams = [torch.cuda.Stream(device=dev) for _ in ctxs]
    outs = [torch.empty(b.capacity, dtype=torch.int32, device=dev) for b in batches]
    for c, st in zip(ctxs, streams):
        c.set_stream(st)
    pending = [False] * len(ctxs)

    def step(i, run=True):
        j = i % len(ctxs)
        if pending[j]:
            ctxs[j].wait()
            pending[j] = False
        src = pool[i % pool_n]
        with torch.cuda.stream(streams[j]):
            for d, h in zip((batches[j].x, batches[j].y, batches[j].z), (src.x, src.y, src.z)):
                d.copy_(h, non_blocking=True)
        if run:
            ctxs[j].plane_segment_batch_async(batches[j], params, outs[j])
            pending[j] = True

    def drain():
        for j, c in enumerate(ctxs):
            if pending[j]:
                c.wait()
                pending[j] = False
        torch.cuda.synchronize()

    for i in range(2 * len(ctxs) * pool_n):  # every context sees every pool batch (the chunk hint settles)
        step(i)
    drain()
    cont0 = sum(c.schedule_stats()[0] for c in ctxs)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    drain()
    dt = time.perf_counter() - t0
    cont = sum(c.schedule_stats()[0] for c in ctxs) - cont0
    t1 = time.perf_counter()
    for i in range(steps):
        step(i, run=False)
    drain()
    dc = time.perf_counter() - t1
    # the last batch of every context against its pool batch, through the oracle on one frame each
    ok = True
    for j in range(len(ctxs)):
        i = steps - len(ctxs) + j
        if i < 0:
            continue
        src = pool[i % pool_n]
        res = ctxs[i % len(ctxs)].plane_segment_batch(src, params, outs[i % len(ctxs)])
        f = min(clutter_at) if i % pool_n == 0 else 0
        o = oracle().plane_segment(*(t[int(src.offsets[f]):int(src.offsets[f]) + int(src.counts[f])].cpu().numpy()
                                     for t in (src.x, src.y, src.z)))
        ok &= bool(res[f]["hypotheses"] == o.hypotheses and np.array_equal(res[f]["coefficients"], o.coefficients))
    for c in ctxs:
        c.set_stream(None)
    nbytes = sum(t.numel() * 4 for t in (pool[0].x, pool[0].y, pool[0].z))
    return {"frames_per_s": round(B * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps,
            "copy_ms_per_step": round(dc / steps * 1e3, 4), "copy_bytes_per_step": nbytes,
            "frames_per_s_copies_excluded": round(B * steps / max(1e-9, dt - dc), 1),
            "clutter_frames": f"{clutter_per_batch} of {B} in 1 of {pool_n} pool batches",
            "continuations_per_100_batches": round(100.0 * cont / steps, 2),
            "spot_check_vs_oracle": ok,
            "note": "a step = a device-to-device copy of new frames into the context's buffers, then its batch"}


ORIG_HW_QUEUES = None  # the caller's GPU_MAX_HW_QUEUES, before main() raises it for the pipelined pass


def config2_pass(pitt, ctx, frame, reps=200):
    """BASELINE config 2: one 640x480 cloud through the single-cloud ABI (pitt_plane_segment: PointXYZ
    host array in, inliers and coefficients back on the host -- the service handler's path, PCIe
    included), median latency of `reps` after 1 warm-up, checked against the oracle."""
    cloud = np.zeros((len(frame[0]), 4), np.float32)
    for k in range(3):
        cloud[:, k] = frame[k]
    r = ctx.plane_segment(cloud)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        r = ctx.plane_segment(cloud)
        ts.append((time.perf_counter() - t) * 1e3)
    o = oracle().plane_segment(*frame)
    # where the time goes: the same frame as a device-resident one-frame batch (no PCIe, no AoS -> SoA),
    # and that batch's kernels by the library's HIP-event profiler
    import torch
    b = pitt.FrameBatch.from_host([frame], device="cuda")
    out = torch.empty(b.capacity, dtype=torch.int32, device="cuda")
    ctx.plane_segment_batch(b, pitt.sac_params(), out)
    td = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.plane_segment_batch(b, pitt.sac_params(), out)
        td.append((time.perf_counter() - t) * 1e3)
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(reps):
        ctx.plane_segment_batch(b, pitt.sac_params(), out)
    kern = {}
    for k in ("k_hypothesize", "k_score", "k_replay", "k_refine:xsum", "k_refine", "k_sel_mark", "k_sel_write"):
        n, ms, _ = ctx.profile_get(k)
        if n:
            kern[k] = round(ms / reps * 1e3, 1)
    ctx.profile(False)
    res = {"ms_per_frame_in_bench_process": round(float(np.median(ts)), 3),
           "statistic": f"median of {reps} after 1 warm-up",
           "inliers": int(len(r.inliers)), "matches_oracle": bool(np.array_equal(r.inliers, o.inliers) and
                                                                np.array_equal(r.coefficients, o.coefficients)),
           "device_resident_ms_per_frame": round(float(np.median(td)), 3),
           "device_kernels_us": kern}
    # The service's own process: the same call in a child process with the caller's environment (this
    # process runs the headline with 8 hardware queues and four contexts' arenas, which cost the one-cloud
    # call ~10 and ~7 us, tools/gpu_c2c.sh); its result must equal the oracle-checked one above.
    env = dict(os.environ)
    if ORIG_HW_QUEUES is None:
        env.pop("GPU_MAX_HW_QUEUES", None)
    else:
        env["GPU_MAX_HW_QUEUES"] = ORIG_HW_QUEUES
    try:
        cp = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "config2_run.py"), str(reps), "--json"],
                            env=env, capture_output=True, text=True, timeout=300)
        c = json.loads(cp.stdout.strip().splitlines()[-1])
        same = (c["inliers"] == len(r.inliers) and c["inliers_sum"] == int(np.asarray(r.inliers, np.int64).sum())
                and np.array_equal(np.asarray(c["coefficients"], np.float32), r.coefficients))
        res["ms_per_frame"] = c["host_ms"] if same else None
        res["service_process"] = {"ms_per_frame": c["host_ms"], "device_resident_ms_per_frame": c["device_ms"],
                                  "same_result": bool(same), "how": "tools/config2_run.py in a child process"}
    except Exception as e:  # noqa: BLE001 -- reported, the in-process figure stands
        res["ms_per_frame"] = res["ms_per_frame_in_bench_process"]
        res["service_process"] = {"error": repr(e)[:200]}
    return res


def config5_pass(pitt, ctx, threads, reps=5):
    """BASELINE config 5: find_supports (th 0.02f, 10 iterations) on the 1.2M-point fused scene, then
    euclidean_clusters (0.03 m, 1 % / 99 %) on every support's on-support cloud
    (obj_segmentation.cpp:261-312).  Timed through pitt_segment_objects_dev with the scene resident
    in HBM (nothing read back but sizes, coefficients and sums), median of `reps` after 1 warm-up.
    Beside it, the host-array path a C++ caller of the drop-in ABI takes (pitt_find_supports, then
    pitt_euclidean_clusters on each support's on-support cloud straight from the pointers it returned:
    H2D of the scene, D2H of every output into the library's pinned blocks), and the same through the
    Python wrappers (which copy every output into fresh numpy arrays).  Results vs the oracle once."""
    import ctypes
    import torch
    from pitt_object_table_segmentation_amd import _lib as L
    orc = oracle()
    x, y, z = pitt.synth_fused(1000, 4)
    dx, dy, dz = (torch.from_numpy(a).cuda() for a in (x, y, z))
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    sp = pitt.support_params()

    def dev_once():
        return ctx.segment_objects_dev(dx, dy, dz, copy=False)

    def host_abi_once():
        out, cout = L.SupportList(), L.ClusterList()
        assert L.lib.pitt_find_supports(ctx.h, fp(x), fp(y), fp(z), len(x), ctypes.byref(sp), ctypes.byref(out)) == 0
        shape = []
        for i in range(out.n_supports):
            s = out.supports[i]
            m = s.n_on_support
            if m < 30:
                shape.append((int(s.n_support), m, []))
                continue
            a = ctypes.cast(s.on_support_xyz, ctypes.c_void_p).value
            pl = [ctypes.cast(a + 4 * m * k, ctypes.POINTER(ctypes.c_float)) for k in range(3)]
            assert L.lib.pitt_euclidean_clusters(ctx.h, pl[0], pl[1], pl[2], m, 0.03, int(np.floor(m * 0.01 + 0.5)),
                                                 int(np.floor(m * 0.99 + 0.5)), ctypes.byref(cout)) == 0
            shape.append((int(s.n_support), m, [int(cout.clusters[c].size) for c in range(cout.n_clusters)]))
        return shape

    def host_once():
        sups = ctx.find_supports(x, y, z)
        cl = []
        for s in sups:
            n = len(s.on_support_cloud)
            cl.append(ctx.euclidean_clusters(*s.on_support_cloud.T, tolerance=0.03,
                                             min_size=int(np.floor(n * 0.01 + 0.5)),
                                             max_size=int(np.floor(n * 0.99 + 0.5))) if n >= 30 else [])
        return sups, cl

    def median_ms(fn):
        fn()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t) * 1e3)
        return round(float(np.median(ts)), 2)

    dev_ms = median_ms(dev_once)
    host_ms = median_ms(host_abi_once)
    py_ms = median_ms(host_once)
    sups, objs = ctx.segment_objects_dev(dx, dy, dz)
    # the host paths found the same supports and clusters as the device path
    hsups, hcl = host_once()
    host_same = (host_abi_once() == [(int(s["support_cloud"].shape[0]), int(s["on_support_cloud"].shape[0]),
                                      [int(o[1].numel()) for o in objs if o[0] == k]) for k, s in enumerate(sups)]
                 and len(hsups) == len(sups)
                 and all(np.array_equal(a.idx_map, b["idx_map"].cpu().numpy()) for a, b in zip(hsups, sups))
                 and [len(c.indices) for cl in hcl for c in cl] == [int(o[1].numel()) for o in objs])
    t = time.perf_counter()
    rs = orc.find_supports(x, y, z)
    rcl = [(k, c) for k, s in enumerate(rs) if len(s["on_support_cloud"]) >= 30
           for c in orc.euclidean_clusters(*s["on_support_cloud"].T)]
    cpu_ms = (time.perf_counter() - t) * 1e3
    same = (len(rs) == len(sups) and
            all(np.array_equal(a["idx_map"].cpu().numpy(), b["idx_map"]) for a, b in zip(sups, rs)) and
            len(objs) == len(rcl) and
            all(k == kr and np.array_equal(i.cpu().numpy(), c["inliers"]) for (k, i, _), (kr, c) in zip(objs, rcl)))
    return {"points": int(len(x)), "supports": len(sups), "clusters": len(objs),
            "gpu_ms_per_scene": dev_ms, "gpu_statistic": f"median of {reps} after 1 warm-up",
            "gpu_path": "pitt_segment_objects_dev (device-resident: scene in HBM, sizes/coefficients/sums back)",
            "host_api_ms_per_scene": host_ms,
            "host_api": "C ABI from host arrays: pitt_find_supports + pitt_euclidean_clusters per support on the "
                        "returned on-support planes (every output copied to the library's pinned host blocks)",
            "python_api_ms_per_scene": py_ms,
            "host_paths_match_device_path": bool(host_same),
            "cpu_ms_per_scene": round(cpu_ms, 1), "cpu": "oracle, one thread, O(N) restatement of the loop",
            "matches_oracle": bool(same)}


def synth_clusters(seed=0):
    """Ten table-top clusters of mixed kinds and sizes (300-3,600 points, 10-20 % clutter): spheres,
    cylinders, cones and boxes with 1 mm noise -- the shapes clustersAcquisition classifies."""
    rng = np.random.default_rng(seed)

    def clutter(n, c):
        return rng.uniform(-0.12, 0.12, (n, 3)) + c

    def sphere(n, c, r):
        d = rng.normal(size=(n, 3))
        return d / np.linalg.norm(d, axis=1)[:, None] * r + c

    def frame(axis):
        a = np.asarray(axis, float) / np.linalg.norm(axis)
        u = np.cross(a, [1.0, 0.0, 0.0] if abs(a[0]) < 0.9 else [0.0, 1.0, 0.0])
        u /= np.linalg.norm(u)
        return a, u, np.cross(a, u)

    def cylinder(n, c, r, h, axis=(0.1, 0.2, 1.0)):
        a, u, v = frame(axis)
        t, ph = rng.uniform(0, h, n), rng.uniform(0, 2 * np.pi, n)
        return c + t[:, None] * a + r * (np.cos(ph)[:, None] * u + np.sin(ph)[:, None] * v)

    def cone(n, c, half_deg, h, axis=(0.1, 0.2, 1.0)):
        a, u, v = frame(axis)
        t, ph = rng.uniform(0.03, h, n), rng.uniform(0, 2 * np.pi, n)
        r = t * np.tan(np.radians(half_deg))
        return c + t[:, None] * a + r[:, None] * (np.cos(ph)[:, None] * u + np.sin(ph)[:, None] * v)

    def box(n, c):
        face = rng.integers(0, 3, n)
        q = rng.uniform(-0.05, 0.05, (n, 2))
        p = np.zeros((n, 3))
        p[face == 0] = np.c_[q, np.full(n, 0.05)][face == 0]
        p[face == 1] = np.c_[q[:, 0], np.full(n, -0.05), q[:, 1]][face == 1]
        p[face == 2] = np.c_[np.full(n, 0.05), q][face == 2]
        return p + c

    specs = [(sphere, 900, (0.3, -0.2, 1.1), 0.05), (cylinder, 1200, (0.3, -0.1, 0.9), 0.04, 0.15),
             (cone, 1000, (0.3, -0.1, 1.1), 25.0, 0.15), (box, 1500, (0.3, -0.1, 1.0)),
             (sphere, 300, (0.1, 0.2, 1.2), 0.03), (cylinder, 600, (0.0, 0.1, 0.8), 0.03, 0.12),
             (box, 400, (-0.2, 0.1, 1.0)), (cone, 2500, (-0.1, -0.2, 1.0), 35.0, 0.15),
             (sphere, 2000, (0.2, 0.3, 1.3), 0.08), (cylinder, 3000, (-0.3, 0.0, 0.9), 0.05, 0.2)]
    out = []
    for f, n, c, *a in specs:
        pts = np.concatenate([f(n, np.asarray(c), *a), clutter(n // 6, np.asarray(c))])
        pts += rng.normal(0, 0.001, pts.shape)
        out.append(pts[rng.permutation(len(pts))].astype(np.float32))
    return out


def classify_pass(pitt, ctx, reps=5):
    """clustersAcquisition (ransac_segmentation.cpp:230-302) on a frame of ten clusters: normals (k = 50),
    the sphere / cylinder / cone / plane services and the arbitration, batched through
    pitt_srv_classify_clusters (one host synchronisation per stage for the frame), against the
    reference's per-cluster loop through the per-cluster services on the same device (median of `reps`
    after 1 warm-up; counts and tags compared)."""
    import torch
    srv = pitt.Services(ctx)
    cl = synth_clusters(0)
    cnt = np.array([len(c) for c in cl], np.int64)
    off = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
    xyz = np.concatenate(cl)
    d = [torch.from_numpy(np.ascontiguousarray(xyz[:, k])).cuda() for k in range(3)]

    def batched():
        return srv.classify_clusters(*d, off, cnt)

    def loop():
        res = []
        for P in cl:
            dd = [torch.from_numpy(np.ascontiguousarray(P[:, k])).cuda() for k in range(3)]
            nx, ny, nz, _ = ctx.normal_estimation(*dd, k=50)
            N = torch.stack([nx, ny, nz], 1).cpu().numpy()
            r = [srv.ransac_sphere(P), srv.ransac_cylinder(P, N), srv.ransac_cone(P, N), srv.ransac_plane(P)]
            counts = [len(q[1]) if q[0] else 0 for q in r]
            res.append((counts, pitt.Services.arbitrate(*counts)))
        return res

    def median_ms(fn):
        out = fn()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t) * 1e3)
        return round(float(np.median(ts)), 2), out

    b_ms, got = median_ms(batched)
    l_ms, ref = median_ms(loop)
    same = all(g["inliers"] == c and g["tag"] == t for g, (c, t) in zip(got, ref))
    srv.close()
    return {"clusters": len(cl), "points": int(cnt.sum()), "ms_per_frame": b_ms,
            "statistic": f"median of {reps} after 1 warm-up",
            "path": "pitt_srv_classify_clusters (device SoA in, one pass for all clusters)",
            "per_cluster_loop_ms": l_ms, "per_cluster_loop": "normals + 4 service calls per cluster (the reference's loop)",
            "tags": [g["shape"] for g in got], "matches_per_cluster_services": bool(same)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-gpu", type=int, default=256)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the clutter / PCIe / config-5 passes")
    ap.add_argument("--no-inliers", action="store_true", help="skip writing the final inlier lists")
    # 4 batches in flight, each context's stream on its own hardware queue (profiles/r03p_*: 370.8k
    # frames/s against 355.2k at 3 in flight on the box's default 4 queues; 4 in flight sharing 4
    # queues measured 287.4k)
    ap.add_argument("--pipeline", type=int, default=4, help="contexts/streams with batches in flight")
    ap.add_argument("--settle-steps", type=int, default=300,
                    help="untimed pipelined steps before the warm-up steps (GPU clocks settle; DESIGN.md s6)")
    ap.add_argument("--parts", type=int, default=1,
                    help="world 1: each step's batch split over this many contexts (the same frames and work per "
                         "step, several steps in flight); the roofline and extra passes keep whole batches")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (0: leave the environment's); set before HIP starts")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for world > 1 (nccl = RCCL over xGMI; gloo: tests)")
    ap.add_argument("--all-ranks-device", type=int, default=-1,
                    help="test only: every rank on this device (rehearses world > 1 on a 1-GPU box)")
    ap.add_argument("--dump-records", default="",
                    help="rank 0 writes the (gathered) records of batch slot 0's last step to this .npy")
    args = ap.parse_args()
    global ORIG_HW_QUEUES
    ORIG_HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")
    if args.hw_queues > 0:  # hardware queues per process (one per in-flight context's stream); before HIP init
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    gpu = local if args.all_ranks_device < 0 else args.all_ranks_device
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    backend = None
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        backend = dist.get_backend()
        log(f"[rank {rank}] torch.distributed backend {backend}"
            f"{' (RCCL)' if backend == 'nccl' else ''}, world size {dist.get_world_size()}, device {gpu}")

    import pitt_object_table_segmentation_amd as pitt
    from pitt_object_table_segmentation_amd import distributed

    cpus = host_cpus()
    threads = cpus["share"]
    B = args.frames_per_gpu
    total = B * world
    start, end = distributed.shard_range(total, world, rank)
    t_gen = time.perf_counter()
    # one distinct batch per in-flight context: batch j holds frames start + j * total + [0, B)
    batches, frames0 = [], None
    parts = args.parts if world == 1 else 1
    pbatches = []  # parts > 1: slot j's frames as `parts` contiguous part batches (slot-major)
    for j in range(args.pipeline):
        fr = make_frames(range(start + j * total, end + j * total), threads)
        if j == 0:
            frames0 = fr
        batches.append(pitt.FrameBatch.from_host(fr, device=dev))
        if parts > 1:
            ps = (len(fr) + parts - 1) // parts
            pbatches += [pitt.FrameBatch.from_host(fr[q * ps:(q + 1) * ps], device=dev) for q in range(parts)]
    log(f"[rank {rank}] {args.pipeline} x {len(frames0)} frames generated + uploaded in "
        f"{time.perf_counter() - t_gen:.1f} s")

    # Several contexts, each on its own library-created stream (own HW queue): batch i+1 is enqueued
    # before batch i completes, so the latency-bound covariance chain of one batch overlaps the
    # HBM-bound kernels of the next.
    ctxs = [pitt.Context(gpu) for _ in range(args.pipeline)]
    outs = [None if args.no_inliers else torch.empty(b.capacity, dtype=torch.int32, device=dev) for b in batches]
    pending = [None] * len(ctxs)
    torch.cuda.synchronize()
    params = pitt.sac_params()
    counter = [0]
    # config 4: the records of a finished batch are gathered asynchronously (posted when the batch
    # completes, collected one step later), so the exchange overlaps the next batch's enqueue
    gather = (distributed.AsyncRecordGather(total, start, end - start, slots=args.pipeline + 2,
                                            device=dev if backend == "nccl" else "cpu") if world > 1 else None)
    posted = []                         # (ctx slot, gather handle), oldest first
    records = [None] * len(ctxs)        # the last completed (gathered) records of each slot

    def collect(keep):
        while len(posted) > keep:
            i, h = posted.pop(0)
            records[i] = gather.collect(h)

    def finish(i):
        ctxs[i].wait()
        if gather is None:
            records[i] = pending[i]
        else:
            posted.append((i, gather.post(pending[i])))
        pending[i] = None

    def step(prm=params):
        i = counter[0] % len(ctxs)
        counter[0] += 1
        if pending[i] is not None:
            finish(i)
        pending[i] = ctxs[i].plane_segment_batch_async(batches[i], prm, outs[i])
        if gather is not None:
            collect(1)

    def drain():
        for i in range(len(ctxs)):
            if pending[i] is not None:
                finish(i)
        if gather is not None:
            collect(0)
        return records[(counter[0] - 1) % len(ctxs)]

    timed_step, timed_drain = step, drain  # the timed pass; the extra passes always use whole batches
    if parts > 1:
        # one context per part: a step enqueues its batch's parts on `parts` contexts at once
        pctxs = [pitt.Context(gpu) for _ in pbatches]
        pouts = [None if args.no_inliers else torch.empty(b.capacity, dtype=torch.int32, device=dev)
                 for b in pbatches]
        ppending, precords = [None] * len(pctxs), [None] * len(pctxs)
        pcounter = [0]
        for k in range(len(pctxs)):
            for _ in range(2):
                pctxs[k].plane_segment_batch(pbatches[k], params, pouts[k])

        def parts_step():
            i = pcounter[0] % args.pipeline
            pcounter[0] += 1
            for k in range(i * parts, (i + 1) * parts):
                if ppending[k] is not None:
                    pctxs[k].wait()
                    precords[k] = ppending[k]
                ppending[k] = pctxs[k].plane_segment_batch_async(pbatches[k], params, pouts[k])

        def parts_drain():
            for k in range(len(pctxs)):
                if ppending[k] is not None:
                    pctxs[k].wait()
                    precords[k] = ppending[k]
                    ppending[k] = None
            for j in range(args.pipeline):  # slot j's records: its parts' records, in frame order
                if all(precords[k] is not None for k in range(j * parts, (j + 1) * parts)):
                    records[j] = np.concatenate([precords[k] for k in range(j * parts, (j + 1) * parts)])
            return records[(pcounter[0] - 1) % args.pipeline]

        timed_step, timed_drain = parts_step, parts_drain

    ctx = ctxs[0]
    # setup, not steps: every context runs its batch twice, so that its scratch arena is allocated
    # and its chunk hint learnt before any timed step; otherwise contexts the warm-up steps never
    # reach pay for that inside the timed region
    for i in range(len(ctxs)):
        for _ in range(2):
            ctxs[i].plane_segment_batch(batches[i], params, outs[i])
    # parity spot check outside the timed region (first frame of this rank vs the oracle), before the
    # warm-up steps: the oracle's CPU time leaves the GPU idle, and the timed region should start on
    # the clocks the warm-up steps brought up, not on an idle GPU's
    if rank == 0:
        res0 = ctx.plane_segment_batch(batches[0], params, outs[0])
        o = oracle().plane_segment(*frames0[0])
        ok = (np.array_equal(res0[0]["coefficients"], o.coefficients) and res0[0]["n_inliers"] == len(o.inliers)
              and res0[0]["hypotheses"] == o.hypotheses)
        log(f"[rank 0] parity frame 0 vs oracle: {'bit-exact' if ok else 'MISMATCH'} "
            f"(T={int(res0[0]['hypotheses'])}, inliers={int(res0[0]['n_inliers'])})")
    if world > 1:
        dist.barrier()

    def timed_window(steps):
        """K pipelined steps bracketed by a barrier + synchronize on both sides; the max over ranks."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            timed_step()
        r = timed_drain()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        d = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([d], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d = float(t.item())
        return d, r

    # ---- the same K-step window with only the W warm-up steps before it (no settle steps): the GPU
    # comes from the setup's serial batches and the oracle's CPU time, as a bench without settling
    # would time it.  Reported beside `value` as `value_without_settle`, never instead of it. ----
    for _ in range(args.warmup):
        timed_step()
    timed_drain()
    dt_cold, _ = timed_window(args.steps)
    # settle, then warm up: --settle-steps pipelined untimed steps before the W warm-up steps.  After
    # the setup's serial batches and the oracle's CPU time the GPU has been idle or lightly loaded, and
    # the first tens of milliseconds of pipelined work run slower per step (clocks and power settling):
    # 20 timed steps measured 358-362k frames/s after 5 warm-up steps, 382-391k after 50 and 394-396k
    # after 300.  The timed steps are unchanged; every untimed pipelined step before them
    # is counted in the line's `untimed_steps`.
    for _ in range(args.settle_steps):
        timed_step()
    for _ in range(args.warmup):
        timed_step()
    timed_drain()

    # ---- timed throughput pass: K steps, batches overlapped on the contexts' streams ----
    if gather is not None:
        gather.seconds, gather.posted = 0.0, 0
    dt, res = timed_window(args.steps)
    rec_dump = None if records[0] is None else records[0].copy()  # before the extra passes reuse the slots
    # the same pipelined step over 200 timed steps right after the headline's (1 GPU, default extras, when
    # fewer steps were asked): the steady state beside the short window's fill and drain; never `value`
    steady = None
    if world == 1 and not args.no_extras and args.steps < 200:
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(200):
            timed_step()
        timed_drain()
        torch.cuda.synchronize()
        dts = time.perf_counter() - ts
        steady = {"steps": 200, "frames_per_s": round(total * 200 / dts, 1), "ms_per_step": round(dts / 200 * 1e3, 4),
                  "note": "the headline's pipelined step timed over 200 steps right after it (fill and drain "
                          "amortised); reported beside `value`, not instead of it"}
        log(f"[rank 0] steady state: {steady}")

    # ---- roofline pass: one batch at a time, HIP events around every launch on the launch stream
    # (a concurrent batch would share HBM and stretch the kernel's duration) ----
    roof_steps = max(1, min(args.steps, 10))
    # every batch layout once on this context first (unprofiled): the adaptive chunk schedule learns per
    # layout, and a layout's first batch launches every chunk
    for k in range(len(batches)):
        ctx.plane_segment_batch(batches[k], params, outs[k])
    ctx.profile(True)
    ctx.profile_reset()
    for k in range(roof_steps):
        ctx.plane_segment_batch(batches[k % len(batches)], params, outs[k % len(batches)])
    launches, ms, nbytes = ctx.profile_get("k_score")
    n_empty, ms_empty, _ = ctx.profile_get("k_score:empty")
    kernels = kernel_table(ctx, roof_steps)
    if rank == 0:
        for k, v in kernels.items():
            log(f"[rank 0] {k:15s} launches/batch {v['launches_per_batch']:5.1f}  {v['us_per_batch']:8.1f} us/batch  "
                f"avg {v['avg_launch_us']:8.1f} us  {v['GBps']:8.1f} GB/s")
    ctx.profile(False)
    hyps = res["hypotheses"]

    line = None
    if rank == 0:
        lib_sha = library_sha16()
        traffic, traffic_note = pmc_traffic(lib_sha)
        avg_ms = ms / max(1, launches)
        achieved = (nbytes / max(1, launches)) / (avg_ms * 1e-3) / 1e9 if launches else 0.0
        line = {
            "metric": METRIC,
            "value": round(total * args.steps / dt, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            # every pipelined step run before the timed K (untimed): the W warm-up steps before the
            # no-settle window, that window's K steps, the settle steps and the W warm-up steps again
            "untimed_steps": 2 * args.warmup + args.steps + args.settle_steps,
            "value_without_settle": round(total * args.steps / dt_cold, 2),
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic 640x480 organised table-scene clouds, scene_seed = 1000 + frame id, "
                    f"{args.pipeline} distinct batches in flight",
            "config": {
                "workload": f"batch of {B} synthetic 307k-pt clouds per GPU (BASELINE config 3"
                            f"{'; config 4: frame-sharded, RCCL all_gather of per-frame records' if world > 1 else ''}),"
                            " PCL plane RANSAC th 0.007 / 1000 iters / seed 12345 / optimize, final inlier lists",
                "frames_per_gpu": B,
                "points_per_frame": W * H,
                "parallelism": f"frame-sharded x{world}, {args.pipeline} batches in flight per GPU"
                               + (f", each split over {parts} contexts" if parts > 1 else ""),
                "untimed_before_timed": {"warmup_steps": args.warmup, "no_settle_window_steps": args.steps,
                                         "settle_steps": args.settle_steps, "warmup_steps_again": args.warmup,
                                         "note": "value_without_settle = the same K-step window timed after only "
                                                 "the W warm-up steps (the GPU from idle); value = the K-step "
                                                 "window after the settle steps"},
                "hypotheses_per_frame_mean": round(float(np.mean(hyps)), 2),
                "world_size_seen": world,
                "collective": (f"{backend} all_gather_into_tensor of per-frame records, async (collected one "
                               "step later)" if world > 1 else None),
                "gather_us_per_step": (round(gather.seconds / args.steps * 1e6, 1) if gather is not None else None),
                "gathers": (gather.posted if gather is not None else None),
                # runtime knobs of the exact kernel variants (read when a context is created)
                "knobs": {k: os.environ[k] for k in sorted(os.environ) if k.startswith("PITT_")} or None,
            },
            "roofline": {
                "kernel": "k_score",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_note,
                "launches": launches,
                "measured": f"HIP events on k_score's stream over a separate {roof_steps}-batch pass with one "
                            "batch in flight (the timed pass overlaps batches on several streams); launches "
                            "that score at least one tile (chunks with no active frame are listed apart)",
                "empty_launches": n_empty,
                "empty_us_per_batch": round(ms_empty / roof_steps * 1e3, 1),
                "avg_launch_us": round(avg_ms * 1e3, 2),
                "algorithmic_bytes_per_launch": round(nbytes / max(1, launches), 1),
            },
            "kernels": kernels,
            "library_sha16": lib_sha,
        }
        if steady is not None:
            line["steady_state"] = steady
    if rank == 0 and world == 1 and not args.no_extras:
        line["cov_fast"] = cov_fast_pass(pitt, ctx, batches, outs, params, step, drain, args.steps, B)
        log(f"[rank 0] cov_fast: {line['cov_fast']}")
        clutter_frames, line["clutter"] = clutter_pass(pitt, ctx, dev, threads)
        log(f"[rank 0] clutter: {line['clutter']}")
        host = [pitt.FrameBatch(b.x.cpu().pin_memory(), b.y.cpu().pin_memory(), b.z.cpu().pin_memory(), b.offsets,
                                b.counts, b.capacity) for b in batches]
        line["pcie_fed"] = pcie_pass(pitt, ctxs, host, dev, params, max(3, min(args.steps, 10)))
        log(f"[rank 0] pcie_fed: {line['pcie_fed']}")
        line["streaming"] = streaming_pass(pitt, ctxs, batches, dev, threads, params, max(20, args.steps))
        log(f"[rank 0] streaming: {line['streaming']}")
        line["config2"] = config2_pass(pitt, ctx, frames0[0])
        log(f"[rank 0] config2: {line['config2']}")
        line["config5"] = config5_pass(pitt, ctx, threads)
        log(f"[rank 0] config5: {line['config5']}")
        line["classify"] = classify_pass(pitt, ctx)
        log(f"[rank 0] classify: {line['classify']}")
    else:
        clutter_frames = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cl = clutter_frames[0] if clutter_frames else make_frames([0], 1, pitt.SCENE_CLUTTER)[0]
        line["cpu_baseline"] = cpu_baseline(frames0, cl, cpus, args.cpu_budget)
    if rank == 0 and args.dump_records:
        np.save(args.dump_records, rec_dump)
    if rank == 0:
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
