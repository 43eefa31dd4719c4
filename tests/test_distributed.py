"""CPU test of the multi-rank plumbing bench.py uses (gloo, world_size 2): the frame-to-rank split, the broadcast
of the shared initial frame (config 3), max-over-ranks timing and the per-frame keypoint-count
all-gather -- the same bench.py functions the GPU run calls, with a CPU stub in place of the extraction."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch

    import bench

    w, r, _ = bench.dist_env()
    dist = bench.dist_init(w, "gloo")
    t = bench.max_over_ranks(dist, 1.0 + r)
    counts = torch.arange(4, dtype=torch.int32) + 100 * r
    g = bench.allgather_counts(dist, counts, w)
    q.put((r, t, g.tolist()))
    dist.destroy_process_group()


def test_gloo_world2_allgather_and_max():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=120) for _ in range(2))
    [p.join(timeout=60) for p in ps]
    for r, t, g in res:
        assert t == 2.0
        assert g == [0, 1, 2, 3, 100, 101, 102, 103]


def _stub_extract(img):
    """CPU stand-in for ORB extraction: a deterministic 'record' of the frame (count + bytes)."""
    import numpy as np

    rng = np.random.default_rng(int(img.sum()) % (2 ** 32))
    n = int(rng.integers(100, 200))
    return np.concatenate([np.array([n], np.int32).view(np.uint8), rng.integers(0, 256, 60 * n, np.uint8)])


def _worker_share(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    import bench
    from orbslam2_with_quadrics_amd import synthetic

    w, r, _ = bench.dist_env()
    dist = bench.dist_init(w, "gloo")
    B = 5
    f1, frames = bench._frames(synthetic, 64, 96, B, r)  # the real frame generator, tiny frames
    start, count = bench.shard_range(w * B, w, r)
    record = {}
    size = 4 + 60 * 200
    buf = torch.zeros(size, dtype=torch.uint8)

    def pack(b):
        rec = _stub_extract(f1)  # only the source rank extracts F1
        b.zero_()
        b[:len(rec)] = torch.from_numpy(rec)
        record["f1"] = b.clone()

    def unpack(b):
        record["f1"] = b.clone()

    bench.broadcast_record(dist, r, buf, pack, unpack)
    # config 5: the local map (world points) built on rank 0 and broadcast as one byte record
    import numpy as np

    kp = np.zeros(50, [("x", "<f4"), ("y", "<f4"), ("octave", "<i4")])
    kp["x"], kp["y"], kp["octave"] = np.arange(50) * 3.0 + 10 * (r == 0), 40.0, np.arange(50) % 8
    mp = bench.local_map(kp, np.full((50, 32), r, np.uint8), 64, 7, 96, 64, 1.2 ** np.arange(8))
    mrec = torch.from_numpy(bench.pack_map(mp).copy())
    bench.broadcast_record(dist, r, mrec, lambda b: None, lambda b: None)
    record["map"] = mrec.numpy().tobytes()
    counts = torch.tensor([int(_stub_extract(f)[:4].view(np.int32)[0]) for f in frames], dtype=torch.int32)
    g = bench.allgather_counts(dist, counts, w)
    q.put((r, start, count, __import__("hashlib").sha256(f1.tobytes()).hexdigest(), record["f1"].numpy().tobytes(),
           g.tolist(), counts.tolist(), record["map"]))
    dist.destroy_process_group()


def test_gloo_world2_shared_initial_frame_split_and_gather():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_share, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=180) for _ in range(2))
    [p.join(timeout=60) for p in ps]
    (r0, s0, c0, h0, rec0, g0, n0, m0), (r1, s1, c1, h1, rec1, g1, n1, m1) = res
    assert (s0, c0, s1, c1) == (0, 5, 5, 5)      # the global frame set [0, 10) split without overlap
    assert h0 == h1                              # every rank renders the same initial frame
    assert rec0 == rec1 and any(rec0)            # rank 1 holds rank 0's record after the broadcast
    assert g0 == g1 == n0 + n1                   # all-gathered keypoint counts, rank order
    assert n0 != n1                              # the ranks' frames differ (per-rank sensor noise)
    assert m0 == m1                              # rank 1 holds rank 0's local map (it built a different one)


def _worker_steady(rank, world, port, q):
    """The real bench.multi_rank_step over 5 steady-state steps with stub contexts: count the host synchronisations
    and the collectives each step issues."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as tdist

    import bench

    w, r, _ = bench.dist_env()
    dist = bench.dist_init(w, "gloo")
    calls = {"broadcast": 0, "all_gather": 0, "sync": 0, "after": 0, "work": 0}

    class Dist:  # torch.distributed with the collectives counted
        def __getattr__(self, name):
            return getattr(tdist, name)

        def broadcast(self, *a, **k):
            calls["broadcast"] += 1
            return tdist.broadcast(*a, **k)

        def all_gather_into_tensor(self, *a, **k):
            calls["all_gather"] += 1
            return tdist.all_gather_into_tensor(*a, **k)

    class Ctx:
        def synchronize(self):
            calls["sync"] += 1

    exs = [Ctx(), Ctx()]
    per = 3  # frames per context
    counts = torch.zeros(len(exs) * per, dtype=torch.int32)
    src = {}

    def work():
        calls["work"] += 1
        for s_ in range(len(exs)):
            src[s_] = torch.arange(per, dtype=torch.int32) + 1000 * r + 100 * s_ + 10 * calls["work"]

    def copy_counts(s_, e):
        counts[s_ * per:(s_ + 1) * per] = src[s_]

    def after(s_, e):
        calls["after"] += 1

    per_step, gathered = [], []
    D = Dist()
    for _ in range(5):
        before = dict(calls)
        bench.multi_rank_step(work, exs, D, w, counts, copy_counts, after)
        per_step.append({k: calls[k] - before[k] for k in calls})
        gathered.append(bench.allgather_counts(D, counts, w).tolist())
    q.put((r, per_step, gathered))
    dist.destroy_process_group()


def test_gloo_world2_steady_step_has_one_host_sync_and_no_broadcast():
    """Verdict r02 item 3: the N > 1 step adds no host synchronisation and no broadcast beyond N = 1's per-step
    context synchronisation; its only collective is the keypoint-count all-gather (the shared initial frame and the
    local map are broadcast once, at set-up)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_steady, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=180) for _ in range(2))
    [p.join(timeout=60) for p in ps]
    for r, per_step, gathered in res:
        for k, d in enumerate(per_step):
            assert d == {"broadcast": 0, "all_gather": 1, "sync": 2, "after": 2, "work": 1}, (r, k, d)
        for k, g in enumerate(gathered):
            step = k + 1
            want = [1000 * rr + 100 * s_ + 10 * step + i for rr in range(2) for s_ in range(2) for i in range(3)]
            assert g == want


def test_single_rank_step_is_collective_free():
    sys.path.insert(0, ROOT)
    import bench

    n = {"sync": 0, "copy": 0, "work": 0}

    class Ctx:
        def synchronize(self):
            n["sync"] += 1

    bench.multi_rank_step(lambda: n.__setitem__("work", n["work"] + 1), [Ctx(), Ctx()], None, 1, None,
                          lambda s, e: n.__setitem__("copy", n["copy"] + 1), None)
    assert n == {"sync": 2, "copy": 0, "work": 1}


def test_map_record_fields_are_16_byte_aligned():
    """every local-map field starts on a 16-byte boundary for any point count."""
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench

    for M in (1, 3, 5, 4999, 5000, 5001):
        offs = bench.map_offsets(M)
        assert all(o % 16 == 0 for o in offs.values())
        mp = dict(pos=np.arange(3 * M, dtype=np.float32).reshape(M, 3), normal=np.ones((M, 3), np.float32),
                  max_dist=np.full(M, 2, np.float32), min_dist=np.full(M, 1, np.float32),
                  is_bad=np.zeros(M, np.uint8), n_obs=np.arange(M, dtype=np.int32),
                  desc=np.full((M, 32), 7, np.uint8))
        rec = bench.pack_map(mp)
        assert len(rec) == offs["_end"]
        assert np.array_equal(rec[offs["n_obs"]:offs["n_obs"] + 4 * M].view(np.int32), mp["n_obs"])
        assert np.array_equal(rec[offs["pos"]:offs["pos"] + 12 * M].view(np.float32), mp["pos"].reshape(-1))


def test_shard_range_partitions():
    sys.path.insert(0, ROOT)
    import bench

    for n in (0, 1, 7, 512, 1000):
        for w in (1, 2, 3, 8):
            got = [bench.shard_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in got) == n
            assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(w - 1))


def test_rccl_refuses_more_ranks_than_gpus():
    """Under RCCL (the default backend) every rank needs its own GPU: more ranks on a node than GPUs is refused before
    any device call, with a message; gloo keeps the round-robin rehearsal."""
    sys.path.insert(0, ROOT)
    import bench

    assert [bench.pick_device(r, 8, 8, "nccl") for r in range(8)] == list(range(8))
    assert bench.pick_device(0, 1, 1, "nccl") == 0
    for local, lw, n in ((1, 2, 1), (0, 2, 1), (4, 8, 4), (8, 8, 8)):
        with pytest.raises(SystemExit, match="one GPU per rank"):
            bench.pick_device(local, lw, n, "nccl")
    assert [bench.pick_device(r, 4, 1, "gloo") for r in range(4)] == [0, 0, 0, 0]
    assert [bench.pick_device(r, 4, 2, "gloo") for r in range(4)] == [0, 1, 0, 1]
    with pytest.raises(SystemExit, match="no GPU"):
        bench.pick_device(0, 1, 0, "gloo")


def test_single_rank_is_collective_free():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.dist_init(1, "gloo") is None
    assert bench.max_over_ranks(None, 3.5) == 3.5


def test_stage_bytes_formula():
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench

    inv = np.array([1.0, 0.8333333, 0.6944444, 0.57870364, 0.48225302, 0.40187752, 0.3348979, 0.27908158],
                   np.float32)
    P = bench.level_pixels(1920, 1080, inv)
    assert P[0] == 1920 * 1080 and P[1] == 1600 * 900
    assert sum(P) == pytest.approx(6_419_321, abs=2000)


def test_interval_union():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.interval_union([]) == 0.0
    assert bench.interval_union([(0.0, 2.0), (1.0, 3.0)]) == 3.0
    assert bench.interval_union([(5.0, 6.0), (0.0, 1.0), (0.5, 0.75)]) == 2.0
    assert bench.interval_union([(-1.0, 1.0), (1.0, 2.0)]) == 3.0


def test_gpus_flag_plans_the_launch():
    """`bench.py --gpus N` runs N ranks by itself.  Without WORLD_SIZE, N > 1 starts
    torch.distributed.run as a child (one process per GPU, 127.0.0.1 rendezvous) with the same arguments; under
    torch.distributed.run (WORLD_SIZE set) the process is a rank; a mismatch is refused."""
    sys.path.insert(0, ROOT)
    import bench

    argv = ["--gpus", "8", "--steps", "20", "--warmup", "2"]
    how, cmd = bench.plan_launch(8, {}, argv, port=29511, python="/usr/bin/python3")
    assert how == "spawn"
    assert cmd == ["/usr/bin/python3", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
                   "--master-addr=127.0.0.1", "--master-port=29511", os.path.join(ROOT, "bench.py")] + argv
    assert bench.plan_launch(1, {}, []) == ("run", 1)
    assert bench.plan_launch(None, {}, []) == ("run", 1)
    assert bench.plan_launch(8, {"WORLD_SIZE": "8"}, argv) == ("run", 8)
    assert bench.plan_launch(None, {"WORLD_SIZE": "4"}, []) == ("run", 4)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.plan_launch(8, {"WORLD_SIZE": "2"}, argv)
    with pytest.raises(SystemExit, match="WORLD_SIZE=8"):
        bench.plan_launch(1, {"WORLD_SIZE": "8"}, [])
    with pytest.raises(SystemExit, match=">= 1"):
        bench.plan_launch(0, {}, [])


def test_gpus_flag_spawns_ranks_without_touching_the_gpu():
    """The real `python bench.py --gpus 2` on this GPU-less host: the parent starts two ranks through
    torch.distributed.run, each rank gets as far as its device pick (no GPU here, so each refuses), and the parent exits
    with the job's failing status -- the parent itself never imports torch."""
    import subprocess

    import torch

    if torch.cuda.is_available():
        pytest.skip("CPU-host test (on a GPU box the ranks would run the bench)")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--batch", "2", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert "launching the ranks:" in r.stderr and "--nproc-per-node=2" in r.stderr
    assert r.stderr.count("no GPU visible") >= 2, r.stderr[-3000:]
    assert r.stdout == ""


def test_roofline_record_names_the_binding_resource():
    """with the PMC VALU count the line's bound is the VALU pipe (frac = 4-cycle busy fraction) and
    the HBM figure -- FAST's pixel bytes of SURVEY.md §8(d), candidates reported separately -- sits beside it."""
    sys.path.insert(0, ROOT)
    import bench

    P = [100, 50]
    assert bench.stage_bytes("fast", 4, P, 10, 0) == 4 * 150
    assert bench.candidate_bytes("fast", 10) == 80 and bench.candidate_bytes("describe", 10) == 0
    valu = {"insts_per_launch": 2_633_533_273, "busy_frac_if_4cyc": 0.8381}
    r = bench.roofline_record("fast", 3_286_692_352, 277_000_000, 5.1146, 5.1146, 5_241_057_176, valu)
    assert r["bound"] == "valu" and r["kernel"] == "fast"
    assert r["frac"] == pytest.approx(0.8381, abs=2e-4)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert r["hbm"]["frac"] == pytest.approx(3_286_692_352 / 5.1146e-3 / 8e12, rel=1e-4)
    assert r["hbm"]["candidate_bytes_per_launch"] == 277_000_000
    assert r["traffic"] == r["hbm"]["traffic"] == 5_241_057_176
    h = bench.roofline_record("fast", 3_286_692_352, 0, 5.1146, 5.1146, None, None)
    assert h["bound"] == "hbm" and h["frac"] == h["hbm"]["frac"] and h["unit"] == "GB/s"
