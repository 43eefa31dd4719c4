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


def test_shard_range_partitions():
    sys.path.insert(0, ROOT)
    import bench

    for n in (0, 1, 7, 512, 1000):
        for w in (1, 2, 3, 8):
            got = [bench.shard_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in got) == n
            assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(w - 1))


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
