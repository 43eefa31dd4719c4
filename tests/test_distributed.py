"""CPU test of the multi-rank plumbing bench.py uses (gloo, world_size 2): max-over-ranks timing and
the per-frame keypoint-count all-gather (the path's only collective)."""
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
