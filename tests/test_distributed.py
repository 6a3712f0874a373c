"""World-size-2 `gloo` tests of the frame-sharded path (config 4).  CPU: the gather of fixed-size
records and of variable-length inlier lists (the multi-GPU path's only collectives).  GPU: the
whole shard -> segment -> gather path on the HIP kernels, byte-equal to one single-batch run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import pitt_object_table_segmentation_amd as pitt
from pitt_object_table_segmentation_amd import distributed


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _records(n):
    rng = np.random.default_rng(123)
    rec = np.zeros(n, pitt.RESULT_DTYPE)
    rec["coefficients"] = rng.normal(size=(n, 4)).astype(np.float32)
    rec["n_inliers"] = rng.integers(0, 307200, n)
    rec["hypotheses"] = rng.integers(1, 1002, n)
    rec["n_coeff"] = 4
    return rec


def _worker(rank, world, port, n_frames, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        allrec = _records(n_frames)
        s, e = distributed.shard_range(n_frames, world, rank)
        got = distributed.gather_results(allrec[s:e], s, n_frames, device="cpu")
        rng = np.random.default_rng(7)
        cnt = rng.integers(0, 50, n_frames)
        lists = [np.sort(rng.choice(1000, c, replace=False)).astype(np.int32) for c in cnt]
        gi, gc = distributed.gather_inliers(np.concatenate(lists[s:e] + [np.zeros(0, np.int32)]), cnt[s:e], device="cpu")
        ok_inl = gi.tobytes() == np.concatenate(lists).tobytes() and np.array_equal(gc, cnt)
        out_q.put((rank, got.tobytes() == allrec.tobytes() and ok_inl))
    finally:
        dist.destroy_process_group()


def _async_worker(rank, world, port, n_frames, out_q):
    """AsyncRecordGather as bench.py drives it: several gathers posted before the oldest is collected."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = distributed.shard_range(n_frames, world, rank)
        g = distributed.AsyncRecordGather(n_frames, s, e - s, slots=3, device="cpu")
        recs = [_records(n_frames) for _ in range(4)]
        for k in range(4):
            recs[k]["hypotheses"] += k  # distinct per step
        handles, got = [], []
        for k in range(4):
            handles.append(g.post(recs[k][s:e]))
            if len(handles) > 2:
                got.append(g.collect(handles.pop(0)))
        got += [g.collect(h) for h in handles]
        out_q.put((rank, all(a.tobytes() == b.tobytes() for a, b in zip(got, recs)) and g.posted == 4))
    except Exception as ex:
        out_q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("n_frames", [16, 13])
def test_gloo_world2_async_gather(n_frames):
    """bench.py's config-4 exchange: gathers posted asynchronously and collected later, in order."""
    assert _spawn(_async_worker, 2, n_frames) == {0: True, 1: True}


def test_unpack_records_vectorised_checks():
    rec = _records(6)
    buf = np.concatenate([distributed.pack_records(rec[:3], np.arange(3), 4),
                          distributed.pack_records(rec[3:], np.arange(3, 6), 4)])
    assert distributed.unpack_records(buf, 6).tobytes() == rec.tobytes()
    # a permuted buffer unpacks to the same frame order
    assert distributed.unpack_records(buf[::-1].copy(), 6).tobytes() == rec.tobytes()
    with pytest.raises(RuntimeError, match="lost"):
        distributed.unpack_records(buf[:4], 6)
    dup = buf.copy()
    dup[1] = dup[0]
    with pytest.raises(RuntimeError, match="duplicated"):
        distributed.unpack_records(dup, 6)


@pytest.mark.parametrize("n_frames", [16, 13])
def test_gloo_world2_gather(n_frames):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


# ---- config 4 on the HIP path: shard -> segment (own context per rank) -> gather ----------------
def _sharded_frames(n_frames):
    frames = []
    for f in range(n_frames):
        scene = (pitt.SCENE_TABLE, pitt.SCENE_CLUTTER, pitt.SCENE_TABLE_NAN)[f % 3]
        w, h = ((320, 240), (160, 120), (640, 480))[f % 3]
        frames.append(pitt.synth_frame(scene, 2000 + f, w, h))
    return frames


def _hip_worker(rank, world, port, n_frames, out_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = _sharded_frames(n_frames)
        s, e = distributed.shard_range(n_frames, world, rank)
        with pitt.Context(0) as ctx:
            b = pitt.FrameBatch.from_host(frames[s:e], device="cuda:0")
            inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
            res = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
            inl = inl.cpu().numpy()
            mine = np.concatenate([inl[o:o + r["n_inliers"]] for o, r in zip(b.offsets, res)] + [np.zeros(0, np.int32)])
        got = distributed.gather_results(res, s, n_frames, device="cpu")
        all_inl, all_cnt = distributed.gather_inliers(mine, res["n_inliers"].astype(np.int64), device="cpu")
        out_q.put((rank, got.tobytes(), all_inl.tobytes(), all_cnt.tobytes()))
    except Exception as ex:  # report instead of hanging the parent
        out_q.put((rank, repr(ex), b"", b""))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_config4_sharded_hip_path_equals_single_batch(ctx):
    """SURVEY s4 / BASELINE config 4 on one GPU: the frame set split by shard_range over a gloo
    world of 2, each rank segmenting its shard through its own Context on the HIP path, then the
    per-frame records and the inlier lists gathered -- byte-equal to one plane_segment_batch over
    every frame (and so to the oracle, which test_plane_gpu pins frame by frame)."""
    import torch
    n_frames, world = 7, 2
    frames = _sharded_frames(n_frames)
    b = pitt.FrameBatch.from_host(frames, device="cuda:0")
    inl = torch.empty(b.capacity, dtype=torch.int32, device="cuda:0")
    ref = ctx.plane_segment_batch(b, pitt.sac_params(), inl)
    inl = inl.cpu().numpy()
    ref_inl = np.concatenate([inl[o:o + r["n_inliers"]] for o, r in zip(b.offsets, ref)])
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_hip_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, recs, ginl, gcnt in got:
        assert isinstance(recs, bytes), recs
        assert recs == ref.tobytes(), f"rank {rank}: gathered records differ"
        assert ginl == ref_inl.tobytes(), f"rank {rank}: gathered inlier lists differ"
        assert gcnt == ref["n_inliers"].astype(np.int64).tobytes()
    assert sorted(r for r, *_ in got) == [0, 1]


# ---- bench.py's own world > 1 branch, rehearsed on the 1-GPU box -------------------------------
def _run_bench(world, frames_per_gpu, dump, port, steps=4, pipeline=2, extra=()):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--steps", str(steps), "--warmup", "1", "--settle-steps", "0", "--pipeline", str(pipeline), "--frames-per-gpu",
              str(frames_per_gpu), "--no-extras", "--no-cpu-baseline", "--dump-records", dump] + list(extra)
    if world == 1:
        cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "1"] + common
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
               "--gpus", str(world), "--dist-backend", "gloo", "--all-ranks-device", "0"] + common
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_world2_gloo_equals_world1(tmp_path):
    """bench.py's world > 1 branch (shards, async record gather, barriers, max
    over ranks) runs at world 2 -- gloo, both ranks on device 0 -- and the gathered records of 2 x B
    frames are byte-equal to a world-1 run over the same 2 B frames."""
    B = 4
    one = _run_bench(1, 2 * B, str(tmp_path / "w1.npy"), _free_port())
    two = _run_bench(2, B, str(tmp_path / "w2.npy"), _free_port())
    assert one["config"]["world_size_seen"] == 1 and two["config"]["world_size_seen"] == 2
    assert two["n_gpus"] == 2 and two["config"]["gather_us_per_step"] is not None
    assert two["config"]["gathers"] == 4 and "gloo" in two["config"]["collective"]
    r1, r2 = np.load(tmp_path / "w1.npy"), np.load(tmp_path / "w2.npy")
    assert r1.dtype == pitt.RESULT_DTYPE and len(r1) == 2 * B
    assert r1.tobytes() == r2.tobytes()


@pytest.mark.gpu
def test_bench_world8_config4_2048_frames(tmp_path):
    """VERDICT r3 next #2 -- BASELINE config 4 at its workload, rehearsed on the 1-GPU box: bench.py at
    world 8 (torchrun, gloo, every rank on device 0, one batch in flight, the box's default hardware
    queues) segments 8 x 256 synthetic 640x480 frames, and the 2048 gathered records are byte-equal to
    a world-1 run over the same 2048 frames; a sample is checked against the oracle.  (RCCL refuses
    two ranks on one GPU, so the 8-rank rehearsal uses gloo; the RCCL branch of the gather is covered
    by test_async_record_gather_rccl_world1.)"""
    import oracle_binding as orc
    B, world = 256, 8
    extra = ("--all-ranks-device", "0", "--hw-queues", "0")
    one = _run_bench(1, world * B, str(tmp_path / "w1.npy"), _free_port(), steps=2, pipeline=1, extra=extra)
    eight = _run_bench(world, B, str(tmp_path / "w8.npy"), _free_port(), steps=2, pipeline=1, extra=extra)
    assert one["config"]["world_size_seen"] == 1 and eight["config"]["world_size_seen"] == world
    assert eight["n_gpus"] == world and eight["config"]["gathers"] == 2
    r1, r8 = np.load(tmp_path / "w1.npy"), np.load(tmp_path / "w8.npy")
    assert r1.dtype == pitt.RESULT_DTYPE and len(r1) == world * B
    assert r1.tobytes() == r8.tobytes()
    for f in (0, 255, 256, 1023, 1500, 2047):  # frame ids of both ranks' shards; bench's scene seed 1000 + id
        o = orc.plane_segment(*pitt.synth_frame(pitt.SCENE_TABLE, 1000 + f, 640, 480))
        assert r8[f]["hypotheses"] == o.hypotheses and r8[f]["n_inliers"] == len(o.inliers), f
        assert np.array_equal(r8[f]["coefficients"].view(np.int32), o.coefficients.view(np.int32)), f
    print(f"config 4 rehearsal: world 8 gather_us_per_step {eight['config']['gather_us_per_step']} "
          f"(gloo, host records), ms_per_step {eight['ms_per_step']}, frames/s {eight['value']}; "
          f"world 1 x 2048 frames: ms_per_step {one['ms_per_step']}, frames/s {one['value']}")


def _rccl_worker(port, n_frames, out_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            assert dist.get_backend() == "nccl"
            g = distributed.AsyncRecordGather(n_frames, 0, n_frames, slots=3, device="cuda:0")
            assert g.cuda and g.host[0].is_pinned() and g.dst[0].is_cuda
            recs = [_records(n_frames) for _ in range(5)]
            for k in range(5):
                recs[k]["hypotheses"] += k
            handles, got = [], []
            for k in range(5):
                handles.append(g.post(recs[k]))
                if len(handles) > 2:  # three in flight at most: every staging slot in use
                    got.append(g.collect(handles.pop(0)))
            got += [g.collect(h) for h in handles]
            ok = all(a.tobytes() == b.tobytes() for a, b in zip(got, recs)) and g.posted == 5
            ok = ok and distributed.gather_results(recs[0], 0, n_frames, device="cuda:0").tobytes() == recs[0].tobytes()
            out_q.put(ok)
        finally:
            dist.destroy_process_group()
    except Exception as ex:
        out_q.put(repr(ex))


@pytest.mark.gpu
@pytest.mark.parametrize("n_frames", [256, 13])
def test_async_record_gather_rccl_world1(n_frames):
    """AsyncRecordGather's device branch (distributed.py: pinned staging slot, non-blocking H2D copy, RCCL
    all_gather_into_tensor) on a world-1 nccl (= RCCL) process group: several gathers in flight,
    collected in order, byte-equal to what was posted."""
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    p = mctx.Process(target=_rccl_worker, args=(_free_port(), n_frames, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res is True, res
