"""bench.py -- frames/s of ORB extract + match @1920x1080, 2000 features (BASELINE.json metric).

One step = one batch of B synthetic 1920x1080 frames already resident in HBM, per GPU:
  * extract the B new frames (ORBextractor::operator(), src/ORBextractor.cc:1043-1105) -- pyramid, FAST cells,
    octree, orientation, blur + rBRIEF, grid -- against the initial frame F1 (Tracking::mInitialFrame);
  * vbPrevMatched := F1 keypoints (src/Tracking.cc:573-575) and SearchForInitialization(F1, F_b) for every
    frame b (src/ORBmatcher.cc:405-520; window 100, ratio 0.9, orientation check, src/Tracking.cc:599-600);
  * F1 is extracted once at set-up, as Tracking extracts its initial frame once (src/Tracking.cc:571); with N > 1
    rank 0 extracts it and broadcasts it once (RCCL, one ~120 KB record) to the other ranks, which match their own
    frames against it; every step ends with the RCCL all-gather of the per-frame keypoint counts,
    stream-ordered against the next step's count copies (no host synchronisation beyond the per-step one).
Frames are independent, so N GPUs run N frame shards ("scaling": "weak"; value = all frames / max time).
Within a GPU the B frames are split over S extractor contexts (--streams, one HIP stream each) whose
kernels run concurrently (default: 1 context, 2 for the tracking workload, DEFAULT_STREAMS).

python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--streams S]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match @1920×1080, 2000 feat; 1/2/4/8 MI355X"
VALU_CLK_HZ = 2.4e9
VALU_SIMDS = 1024
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------------
# distributed plumbing (kept free of GPU specifics so tests can run it on gloo)
# ------------------------------------------------------------------------------------------------
def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def plan_launch(gpus, environ, argv, port=None, python=None):
    """How this process runs `bench.py --gpus N` (decided before torch is imported or any HIP call is made):
      ("run", N)     -- this process is one of the N ranks: WORLD_SIZE is set by torch.distributed.run and equals N
                        (or --gpus was not given), or N == 1 without WORLD_SIZE;
      ("spawn", cmd) -- N > 1 and no WORLD_SIZE: start N ranks as `python -m torch.distributed.run` on this node, one
                        process per GPU, as a child process (this one never touches the GPU and never execs);
    and SystemExit when WORLD_SIZE and --gpus disagree."""
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if gpus is not None and int(ws) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (launched with {ws} ranks); "
                             f"pass --gpus {ws} or launch {gpus} ranks")
        return "run", int(ws)
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n} must be >= 1")
    if n == 1:
        return "run", 1
    cmd = [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port if port is not None else free_port()}",
           os.path.abspath(__file__)] + list(argv)
    return "spawn", cmd


def spawn_ranks(cmd) -> int:
    """Run the N-rank job as a child process with this process's stdout/stderr (rank 0's JSON line comes through
    unchanged); SIGTERM/SIGINT are passed on to it.  Returns its exit code."""
    import signal
    import subprocess

    log(f"launching the ranks: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, env=dict(os.environ, ORBGPU_BENCH_LAUNCHER="bench.py --gpus"))

    def fwd(sig, _frame):
        p.send_signal(sig)

    old = {s: signal.signal(s, fwd) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        rc = p.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def dist_init(world: int, backend: str):
    if world <= 1:
        return None
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group(backend=backend)
    return dist


def pick_device(local: int, local_world: int, device_count: int, backend: str) -> int:
    """The GPU of local rank `local`: one rank per GPU.  RCCL ("nccl", the default backend) cannot run two ranks on
    one GPU, so more ranks on a node than it has GPUs is refused here, before any device or process-group call,
    instead of failing inside RCCL.  ORBGPU_BENCH_BACKEND=gloo rehearses the multi-rank path with more ranks than
    GPUs: ranks then share the devices round-robin."""
    if device_count < 1:
        raise SystemExit("bench.py: no GPU visible (torch.cuda.device_count() == 0)")
    if backend == "nccl" and max(local_world, local + 1) > device_count:
        raise SystemExit(f"bench.py: {max(local_world, local + 1)} ranks on this node but {device_count} GPU(s): "
                         f"RCCL needs one GPU per rank (use ORBGPU_BENCH_BACKEND=gloo to rehearse with shared GPUs)")
    return local % device_count


def max_over_ranks(dist, value: float, device=None) -> float:
    if dist is None:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def per_rank_values(dist, value: float, device=None):
    """Every rank's value (all-gather); [value] on a single rank."""
    if dist is None:
        return [value]
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def shard_range(n_total: int, world: int, rank: int):
    """Contiguous frame-to-rank split of a step's global frame set: (first global frame, frame count) of `rank`."""
    base, rem = divmod(n_total, world)
    return rank * base + min(rank, rem), base + (1 if rank < rem else 0)


def broadcast_record(dist, rank: int, buf, pack, unpack, src: int = 0):
    """A frame extracted once and shared by every rank (config 3: the initial frame F1 that every new frame is
    matched against, src/Tracking.cc:563-635): the source rank packs it into `buf`, one broadcast (RCCL on the
    GPU), the other ranks unpack it.  No-op on a single rank."""
    if dist is None:
        return
    if rank == src:
        pack(buf)
    dist.broadcast(buf, src=src)
    if rank != src:
        unpack(buf)


def multi_rank_step(work, exs, dist, world: int, counts, copy_counts, after_gather, ncount=None):
    """One timed step: enqueue the workload on every context, copy each context's per-frame keypoint counts into
    `counts` on that context's stream, synchronise every context once (the step's only host synchronisation: it
    also reads the contexts' capacity-guard flags), then all-gather the counts over RCCL (north_star).  The
    all-gather is left in flight; after_gather(s, e) orders context s's next count copy after it on the GPU.
    Single rank: no copies, no collective.  ncount: the first ncount contexts hold the counts (config 4: the left
    extractors; the right ones are synchronised but count nothing); default all."""
    work()
    owners = exs if ncount is None else exs[:ncount]
    if dist is not None:
        for s_, e in enumerate(owners):
            copy_counts(s_, e)
    for e in exs:
        e.synchronize()
    if dist is not None:
        allgather_counts(dist, counts, world)
        for s_, e in enumerate(owners):
            after_gather(s_, e)


def allgather_counts(dist, counts, world: int):
    """All-gather of per-frame keypoint counts (int32 tensor); returns the gathered tensor."""
    if dist is None:
        return counts
    import torch

    out = torch.empty(world * counts.numel(), dtype=counts.dtype, device=counts.device)
    dist.all_gather_into_tensor(out, counts)
    return out


# ------------------------------------------------------------------------------------------------
# algorithmic bytes
# ------------------------------------------------------------------------------------------------
def level_pixels(cols, rows, inv_scale):
    return [int(np.rint(np.float32(cols) * s)) * int(np.rint(np.float32(rows) * s)) for s in inv_scale]


def stage_bytes(stage, B, P, cand_total, kp_total, mappoints=0):
    """Algorithmic HBM bytes of one launch of `stage` for a batch of B frames."""
    if stage == "pyramid":  # read levels 0..L-2, write levels 1..L-1
        return B * (sum(P[:-1]) + sum(P[1:]))
    if stage == "fast":  # every pyramid pixel once; the candidates it writes: candidate_bytes
        return B * sum(P)
    if stage == "octree":  # candidates read once + 5 B per selected keypoint written
        return 8 * cand_total + 5 * kp_total
    if stage == "describe":  # 43x43 raw neighbourhood per keypoint + 28 B keypoint + 32 B descriptor
        return kp_total * (43 * 43 + 60)
    if stage == "grid":
        return kp_total * (28 + 4) + B * 3073 * 4
    if stage == "search_init":  # F2 keypoints + descriptors + grid, F1 once
        return kp_total * 60 + B * 3073 * 4
    if stage == "search_proj":  # map-point snapshot (58 B per point) + keypoints + descriptors + grid
        return B * mappoints * 58 + kp_total * 60 + B * 3073 * 4
    if stage == "frustum":  # the shared map's geometry (33 B per point) once + 21 B of track fields per (frame, point)
        return mappoints * 33 + B * mappoints * 21
    if stage == "stereo":  # left and right keypoints + descriptors, the 11x11 left window and 11x21 right band of
        # each left keypoint, uRight / depth / SAD out (kp_total = left keypoints; right ones taken as many)
        return kp_total * (2 * 60 + 121 + 231 + 12)
    return 0


def candidate_bytes(stage, cand_total):
    """Bytes a launch writes beside stage_bytes' algorithmic ones: FAST's packed candidates, 8 B each (reported beside
    the roofline, not in it)."""
    return 8 * cand_total if stage == "fast" else 0


def roofline_record(dom, dom_bytes, cand_bytes, dom_ms, dom_ms_span, traffic, valu):
    """The bench line's roofline object.  `bound` names the resource that binds the dominant kernel: the VALU issue
    pipe when the PMC VALU count is known (the FAST / resize / describe kernels issue ~0.84 of the pipe's 4-cycle
    slots while reading HBM at < 0.1 of its peak), and then `achieved` / `peak` / `frac` are VALU
    wave-instruction issue rates; the HBM figure (SURVEY.md §8(d) algorithmic bytes / launch time against 8 TB/s, and
    the PMC traffic) is always given under `hbm`.  Without PMC data the HBM figure is the top level."""
    ach = dom_bytes / (dom_ms * 1e-3) / 1e9
    hbm = {"achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
           "traffic": traffic, "algorithmic_bytes_per_launch": int(dom_bytes),
           "candidate_bytes_per_launch": int(cand_bytes),
           "traffic_over_algorithmic": round(traffic / dom_bytes, 3) if traffic and dom_bytes else None,
           "bytes": "SURVEY.md §8(d): every pyramid pixel once for FAST (candidate writes reported separately)"}
    out = {"kernel": dom, "avg_launch_ms": round(dom_ms, 4), "avg_launch_span_ms": round(dom_ms_span, 4),
           "launch_time": "union of the kernel's HIP-event intervals over the concurrent streams / launches"}
    if valu is not None:
        peak = VALU_SIMDS * VALU_CLK_HZ / 4 / 1e9  # G wave-instructions/s when every instruction is a 4-cycle form
        rate = valu["insts_per_launch"] / (dom_ms * 1e-3) / 1e9
        out.update(bound="valu", achieved=round(rate, 2), peak=round(peak, 1),
                   unit="G VALU wave-instructions/s (4-cycle issue: 1024 SIMDs x 2.4 GHz / 4)",
                   frac=round(rate / peak, 4), traffic=traffic, valu=valu, hbm=hbm)
    else:
        out.update(bound="hbm", achieved=hbm["achieved"], peak=HBM_PEAK_GBS, unit="GB/s", frac=hbm["frac"],
                   traffic=traffic, valu=None, hbm=hbm)
    return out


def interval_union(iv):
    """Total length of the union of [t0, t1) intervals."""
    tot, end = 0.0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


# ------------------------------------------------------------------------------------------------
# CPU baseline: the oracle (a plain-C restatement of the reference path) built with the reference's flags
# (-O3 -march=native, bit-identical to the checker build), on one pinned host core; median per frame after
# warm-up frames (the full >= 200-frame and all-cores runs: tools/cpu_baseline.py)
# ------------------------------------------------------------------------------------------------
def _oracle_fast():
    os.environ["ORB_ORACLE_FAST"] = "1"
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O

    O.build()
    return O


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def timed_cpu_frames(work, frame, seconds, warmup=10):
    """Median seconds per frame of work(frame(i)) on one pinned core (the lowest core this process may use)."""
    import statistics

    prev = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(prev)})
    try:
        for i in range(warmup):
            work(frame(i))
        ts, spent = [], 0.0
        i = warmup
        while spent < seconds or len(ts) < 3:
            f = frame(i)
            t = time.perf_counter()
            work(f)
            ts.append(time.perf_counter() - t)
            spent += ts[-1]
            i += 1
    finally:
        os.sched_setaffinity(0, prev)
    return statistics.median(ts), len(ts)


def cpu_record(med, n, warmup, what):
    return {"value": round(1.0 / med, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
            "sample": f"median of {n} frames after {warmup} warm-up frames, one pinned core: {what}; oracle built -O3 "
                      f"-march=native (plain C, scalar; OpenCV's SIMD build of the reference would be faster); the "
                      f"full plan (>= 200 frames, 16-core run): tools/cpu_baseline.py, profiles/r06_cpu_baseline.json",
            "full_plan": "profiles/r06_cpu_baseline.json"}


def cpu_baseline(rows, cols, nfeat, seconds):
    O = _oracle_fast()
    from orbslam2_with_quadrics_amd import synthetic

    ex = O.OracleExtractor(nfeat)
    scene = synthetic.make_scene(synthetic.SEED_BASE + 999, rows, cols)
    f1 = synthetic.render(scene, rows, cols, 0, 0, noise_seed=5)
    k1, d1 = ex(f1)
    sf = ex.tables()["scale"]
    F1 = O.OracleFrame(k1, d1, cols, rows, sf)
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)

    def work(f2):
        k2, d2 = ex(f2)
        O.search_for_initialization(F1, O.OracleFrame(k2, d2, cols, rows, sf), prev.copy(), 0.9, True, 100)

    med, n = timed_cpu_frames(work, lambda i: synthetic.render(scene, rows, cols, 3 + i % 9, 2 + i % 5,
                                                                noise_seed=100 + i), seconds)
    return cpu_record(med, n, 10, f"{cols}x{rows}, {nfeat} features, oracle extract + SearchForInitialization")


# ------------------------------------------------------------------------------------------------
# workloads: each sets up its contexts and device buffers and returns the timed step
# ------------------------------------------------------------------------------------------------
def _frames(synthetic, rows, cols, B, rank, seed_off=1000):
    """The initial frame (shared by all ranks) and this rank's B frames (global frames [rank*B, (rank+1)*B),
    shard_range): one scene seen under 32 shifts with per-rank sensor noise, repeating with period 32."""
    scene = synthetic.make_scene(synthetic.SEED_BASE + seed_off, rows, cols)
    nuniq = min(B, 32)
    uniq = [synthetic.render(scene, rows, cols, int(3 + 5 * (i % 8)), int(2 + 3 * (i // 8)),
                             noise_seed=rank * 100000 + 10 + i) for i in range(nuniq)]
    f1 = synthetic.render(scene, rows, cols, 0, 0, noise_seed=1)
    return f1, np.stack([uniq[i % nuniq] for i in range(B)])


def bench_golden(args, rank, name="bench_golden.json"):
    """Oracle hashes of this rank's frames (tests/golden/bench_golden.json for config 3, bench_extract_golden.json
    for config 2; tests/golden/make_golden.py), or None when the run's configuration is not the one the goldens
    were made for."""
    path = os.path.join(ROOT, "tests", "golden", name)
    if not os.path.exists(path):
        return None
    g = json.load(open(path))
    if (g["rows"], g["cols"], g["nfeatures"], g["semantics"]) != (args.rows, args.cols, args.nfeatures, args.semantics):
        return None
    return next((r for r in g["ranks"] if r["rank"] == rank), None)


def _sha(a) -> str:
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def pcie_peak(torch, dev, nbytes=256 << 20, reps=4):
    """Measured link peak: pinned host <-> device copies of 256 MB (H2D, D2H, and both directions at once on two
    streams), best of `reps`, GB/s.  The PCIe-inclusive bench line reports its transfer rate against these."""
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{dev}")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{dev}")
    s1, s2 = torch.cuda.Stream(device=f"cuda:{dev}"), torch.cuda.Stream(device=f"cuda:{dev}")
    out = {}
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h2.copy_(d2, non_blocking=True))):
        best = 0.0
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            with torch.cuda.stream(s1):
                fn()
            torch.cuda.synchronize()
            best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
        out[name + "_GBps"] = round(best, 2)
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, 2 * nbytes / (time.perf_counter() - t) / 1e9)
    out["bidir_GBps"] = round(best, 2)
    del h, h2, d, d2
    return out


def setup_mono_init(args, env):
    """config 3: extract the initial frame and B frames, SearchForInitialization of each against it.  The B frames
    are split over S contexts (streams) and, per context, K sequential launches (--chunks; one launch is fastest,
    profiles/sweeps/r01_stagger_chunks.txt)."""
    L, C_, _lib, ORBextractor, synthetic = env["L"], C, env["_lib"], env["ORBextractor"], env["synthetic"]
    rows, cols, B, NF, S, dev = args.rows, args.cols, args.batch, args.nfeatures, args.streams, env["dev"]
    K = args.chunks
    Bs = B // S
    if Bs % K:
        raise SystemExit(f"--batch/--streams = {Bs} frames per stream must be a multiple of --chunks {K}")
    Bc = Bs // K
    f1, frames = _frames(synthetic, rows, cols, B, env["rank"])
    ex_ref = ORBextractor(NF, 1.2, 8, 20, 7, device=dev, semantics=args.semantics)
    exs = [ORBextractor(NF, 1.2, 8, 20, 7, device=dev, semantics=args.semantics) for _ in range(S)]
    d_f1 = ex_ref.device_alloc(f1.nbytes)
    d_frames = exs[0].device_alloc(frames.nbytes)
    ex_ref.h2d(d_f1, f1)
    dist, rank = env["dist"], env["rank"]
    exs[0].h2d(d_frames, frames)
    fbytes = rows * cols
    grid = _lib.GridGeom()
    L.orbgpu_grid_geom_for_image(cols, rows, C_.byref(grid))
    # F1 (Tracking::mInitialFrame) is extracted once, at set-up (src/Tracking.cc:571); with N > 1 rank 0's F1 is
    # the one every rank matches against: it reaches the others as one frame record, also once.
    # Every rank runs the set-up extraction too: it plans the reference context for the frame geometry (the record
    # size and the buffers the record is unpacked into), and rank 0's record then replaces the result.
    ex_ref.extract_batch_device(d_f1, 1, cols, rows, cols, f1.nbytes)
    ex_ref.synchronize()
    if dist is not None:
        import torch

        rec = torch.empty(int(L.orbgpu_frame_record_bytes(ex_ref.ctx)), dtype=torch.uint8, device=f"cuda:{dev}")

        def pack(buf):
            _lib.check(ex_ref.ctx, L.orbgpu_frame_record_pack(ex_ref.ctx, 0, C_.c_void_p(buf.data_ptr())), "pack")
            ex_ref.synchronize()

        def unpack(buf):
            torch.cuda.current_stream().synchronize()  # the broadcast has landed
            _lib.check(ex_ref.ctx, L.orbgpu_frame_record_unpack(ex_ref.ctx, C_.c_void_p(buf.data_ptr())), "unpack")
            ex_ref.synchronize()

        broadcast_record(dist, rank, rec, pack, unpack)
        del rec
    for s_, e in enumerate(exs):
        e.extract_batch_device(d_frames + s_ * Bs * fbytes, Bc, cols, rows, cols, fbytes)
        e.synchronize()
    outs = [e.batch_outputs() for e in exs]
    cap = outs[0][3]
    d_prev = [e.device_alloc(Bc * cap * 2 * 4) for e in exs]
    d_m12 = [e.device_alloc(Bc * cap * 4) for e in exs]
    d_nm = [e.device_alloc(Bc * 4) for e in exs]
    d_cnt = [e.device_alloc(Bs * 4) for e in exs]  # per-frame keypoint counts of all K chunks (all-gathered)
    host = None
    if args.host_io:  # frames from pinned host memory, keypoints + descriptors back to pinned host memory
        import torch

        # the frames' device copy is a torch tensor (copied on a per-context side stream); d_frames stays the
        # device_alloc buffer of set-up and is not read in this mode
        dv = torch.empty(frames.nbytes, dtype=torch.uint8, device=f"cuda:{dev}")
        host = dict(frames=torch.from_numpy(frames.reshape(-1)).pin_memory(), dev=dv,
                    kps=[torch.empty(Bc * cap * 28, dtype=torch.uint8).pin_memory() for _ in exs],
                    desc=[torch.empty(Bc * cap * 32, dtype=torch.uint8).pin_memory() for _ in exs],
                    # chunk r+1's upload runs on a side stream while chunk r computes; the compute stream waits for
                    # the upload's event, and the next step's upload of a chunk waits for its compute to finish
                    cs=[torch.cuda.Stream(device=f"cuda:{dev}") for _ in exs],
                    xs=[torch.cuda.ExternalStream(e.stream(), device=f"cuda:{dev}") for e in exs],
                    up=[[torch.cuda.Event() for _ in range(K)] for _ in exs],
                    done=[[torch.cuda.Event() for _ in range(K)] for _ in exs])
        host["peak"] = pcie_peak(torch, dev)

    def step():
        for r in range(K):
            for s_, e in enumerate(exs):
                off = (s_ * Bs + r * Bc) * fbytes
                src = d_frames
                if host is not None:
                    import torch

                    cs, xs = host["cs"][s_], host["xs"][s_]
                    cs.wait_event(host["done"][s_][r])  # the previous step's compute of this chunk is done
                    with torch.cuda.stream(cs):
                        host["dev"][off:off + Bc * fbytes].copy_(host["frames"][off:off + Bc * fbytes],
                                                                 non_blocking=True)
                    host["up"][s_][r].record(cs)
                    xs.wait_event(host["up"][s_][r])
                    src = host["dev"].data_ptr()
                e.extract_batch_device(src + off, Bc, cols, rows, cols, fbytes)
                _lib.check(e.ctx, L.orbgpu_memcpy_d2d_async(e.ctx, C_.c_void_p(d_cnt[s_] + 4 * r * Bc),
                                                            C_.c_void_p(outs[s_][2]), Bc * 4), "d2d")
                _lib.check(e.ctx, L.orbgpu_prev_matched_from_frame(ex_ref.ctx, 0, e.ctx, C_.c_void_p(d_prev[s_])),
                           "prev")
                _lib.check(e.ctx, L.orbgpu_search_for_initialization_batch(ex_ref.ctx, 0, e.ctx, grid, 0.9, 1, 100,
                                                                             C_.c_void_p(d_prev[s_]),
                                                                             C_.c_void_p(d_m12[s_]),
                                                                             C_.c_void_p(d_nm[s_])), "search_init")
                if host is not None:  # mvKeys + mDescriptors of the chunk back to the host
                    _lib.check(e.ctx, L.orbgpu_memcpy_d2h_async(e.ctx, C_.c_void_p(host["kps"][s_].data_ptr()),
                                                                C_.c_void_p(outs[s_][0]), Bc * cap * 28), "d2h")
                    _lib.check(e.ctx, L.orbgpu_memcpy_d2h_async(e.ctx, C_.c_void_p(host["desc"][s_].data_ptr()),
                                                                C_.c_void_p(outs[s_][1]), Bc * cap * 32), "d2h")
                    host["done"][s_][r].record(host["xs"][s_])

    def verify():
        """Parity of the timed path itself: every frame of the last step's last chunk (and the initial frame)
        against the oracle's hashes of the same frame -- keypoints, descriptors, vnMatches12, nmatches and the
        updated vbPrevMatched (src/ORBmatcher.cc:405-520)."""
        g = bench_golden(args, env["rank"])
        if g is None:
            return {"status": "no oracle golden for this configuration/rank", "frames": 0, "mismatches": None}
        nuniq = min(B, 32)
        ex_ref.synchronize()
        o_ref = ex_ref.batch_outputs()
        n1 = np.zeros(1, np.int32)
        ex_ref.d2h(n1, o_ref[2])
        n1 = int(n1[0])
        k1 = np.zeros(n1 * 28, np.uint8)
        d1 = np.zeros(n1 * 32, np.uint8)
        ex_ref.d2h(k1, o_ref[0])
        ex_ref.d2h(d1, o_ref[1])
        bad = int(_sha(k1) != g["f1"]["kps_sha256"] or _sha(d1) != g["f1"]["desc_sha256"] or n1 != g["f1"]["n"])
        checked = 0
        for s_, e in enumerate(exs):
            e.synchronize()
            kp, de, cn, cap_ = outs[s_]
            kps = np.zeros(Bc * cap_ * 28, np.uint8)
            desc = np.zeros(Bc * cap_ * 32, np.uint8)
            cnt = np.zeros(Bc, np.int32)
            m12 = np.zeros(Bc * cap_, np.int32)
            prev = np.zeros(Bc * cap_ * 2, np.float32)
            nm = np.zeros(Bc, np.int32)
            for dst, src in ((kps, kp), (desc, de), (cnt, cn), (m12, d_m12[s_]), (prev, d_prev[s_]), (nm, d_nm[s_])):
                e.d2h(dst, src)
            for b in range(Bc):
                gf = g["frames"][(s_ * Bs + (K - 1) * Bc + b) % nuniq]
                n = int(cnt[b])
                ok = (n == gf["n"] and nm[b] == gf["nmatches"] and
                      _sha(kps[b * cap_ * 28:(b * cap_ + n) * 28]) == gf["kps_sha256"] and
                      _sha(desc[b * cap_ * 32:(b * cap_ + n) * 32]) == gf["desc_sha256"] and
                      _sha(m12[b * cap_:b * cap_ + n1]) == gf["matches12_sha256"] and
                      _sha(prev[2 * b * cap_:2 * (b * cap_ + n1)]) == gf["prev_sha256"])
                bad += int(not ok)
                checked += 1
        return {"status": "checked", "frames": checked + 1, "unique_frames": nuniq + 1, "mismatches": bad,
                "against": "oracle hashes of the same frames (tests/golden/bench_golden.json)"}

    def post():  # the last chunk of every context
        counts = np.zeros(Bc, np.int32)
        nm = np.zeros(Bc, np.int32)
        kp_all, nm_all = 0, 0
        for s_, e in enumerate(exs):
            e.d2h(counts, outs[s_][2])
            e.d2h(nm, d_nm[s_])
            kp_all += int(counts.sum())
            nm_all += int(nm.sum())
        extra = {"mean_keypoints_per_frame": round(kp_all / (Bc * S), 1),
                 "mean_init_matches_per_frame": round(nm_all / (Bc * S), 1),
                 "chunks_per_stream": K}
        if host is not None:
            extra["pcie"] = {"h2d_bytes_per_step": int(frames.nbytes), "d2h_bytes_per_step": int(B * cap * 60),
                             "link_peak": host["peak"],
                             "note": "frames H2D on a side stream per context, overlapped with the previous chunk's "
                                     "compute; keypoints + descriptors D2H on the compute stream"}
        return extra, kp_all / S

    def free():
        for s_, e in enumerate(exs):
            for p in (d_prev[s_], d_m12[s_], d_nm[s_], d_cnt[s_]):
                e.device_free(p)
        exs[0].device_free(d_frames)
        ex_ref.device_free(d_f1)

    metric = METRIC if host is None else METRIC + " (PCIe-inclusive: frames H2D, keypoints + descriptors D2H)"
    return dict(metric=metric, exs=exs, step=step, post=post, free=free, verify=verify, Bs=Bc,
                per_stream=Bs, frames_per_step=B,
                counts=d_cnt,
                workload=f"config 3: {cols}x{rows} mono, {NF} features, ORB extract + SearchForInitialization "
                         f"(window 100, ratio 0.9, checkOri) of every frame against an initial frame",
                cpu=lambda: cpu_baseline(rows, cols, NF, args.cpu_seconds))


def setup_extract(args, env):
    """config 2 (640x480, 1000 features by default): ORB extraction only."""
    _lib, ORBextractor, synthetic = env["_lib"], env["ORBextractor"], env["synthetic"]
    rows, cols, B, NF, S, dev = args.rows, args.cols, args.batch, args.nfeatures, args.streams, env["dev"]
    Bs = B // S
    _, frames = _frames(synthetic, rows, cols, B, env["rank"], 2000)
    exs = [ORBextractor(NF, 1.2, 8, 20, 7, device=dev, semantics=args.semantics) for _ in range(S)]
    d_frames = exs[0].device_alloc(frames.nbytes)
    exs[0].h2d(d_frames, frames)
    fbytes = rows * cols
    for s_, e in enumerate(exs):
        e.extract_batch_device(d_frames + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
        e.synchronize()
    outs = [e.batch_outputs() for e in exs]

    def step():
        for s_, e in enumerate(exs):
            e.extract_batch_device(d_frames + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)

    def post():
        counts = np.zeros(Bs, np.int32)
        kp_all = 0
        for s_, e in enumerate(exs):
            e.d2h(counts, outs[s_][2])
            kp_all += int(counts.sum())
        return {"mean_keypoints_per_frame": round(kp_all / B, 1)}, kp_all / S

    def verify():
        """Parity of the timed path: keypoints and descriptors of every frame of the last step against the
        oracle's hashes of the same frames (ORBextractor::operator(), src/ORBextractor.cc:1043-1105)."""
        g = bench_golden(args, env["rank"], "bench_extract_golden.json")
        if g is None:
            return {"status": "no oracle golden for this configuration/rank", "frames": 0, "mismatches": None}
        nuniq = min(B, 32)
        bad = checked = 0
        for s_, e in enumerate(exs):
            e.synchronize()
            kp, de, cn, cap_ = outs[s_]
            kps = np.zeros(Bs * cap_ * 28, np.uint8)
            desc = np.zeros(Bs * cap_ * 32, np.uint8)
            cnt = np.zeros(Bs, np.int32)
            for dst, src in ((kps, kp), (desc, de), (cnt, cn)):
                e.d2h(dst, src)
            for b in range(Bs):
                gf = g["frames"][(s_ * Bs + b) % nuniq]
                n = int(cnt[b])
                ok = (n == gf["n"] and _sha(kps[b * cap_ * 28:(b * cap_ + n) * 28]) == gf["kps_sha256"] and
                      _sha(desc[b * cap_ * 32:(b * cap_ + n) * 32]) == gf["desc_sha256"])
                bad += int(not ok)
                checked += 1
        return {"status": "checked", "frames": checked, "unique_frames": nuniq, "mismatches": bad,
                "against": "oracle hashes of the same frames (tests/golden/bench_extract_golden.json)"}

    return dict(metric=f"frames/sec ORB extract @{cols}×{rows}, {NF} feat", exs=exs, step=step, post=post, verify=verify,
                free=lambda: exs[0].device_free(d_frames), Bs=Bs, frames_per_step=B, counts=[o[2] for o in outs],
                workload=f"config 2: {cols}x{rows}, {NF} features, ORB extraction (ORBextractor::operator())",
                cpu=lambda: cpu_baseline_extract(rows, cols, NF, args.cpu_seconds))


def setup_stereo(args, env):
    """config 4 (KITTI 1241x376, 2000 features): left + right extraction and Frame::ComputeStereoMatches."""
    L, _lib, ORBextractor, synthetic = env["L"], env["_lib"], env["ORBextractor"], env["synthetic"]
    rows, cols, B, NF, S, dev = args.rows, args.cols, args.batch, args.nfeatures, args.streams, env["dev"]
    Bs = B // S
    nuniq = min(B, 16)
    pairs = [synthetic.stereo_pair(3000 + env["rank"] * 100 + i, rows, cols) for i in range(nuniq)]
    left = np.stack([pairs[i % nuniq][0] for i in range(B)])
    right = np.stack([pairs[i % nuniq][1] for i in range(B)])
    exL = [ORBextractor(NF, 1.2, 8, 20, 7, device=dev, semantics=args.semantics) for _ in range(S)]
    exR = [ORBextractor(NF, 1.2, 8, 20, 7, device=dev, semantics=args.semantics) for _ in range(S)]
    dL = exL[0].device_alloc(left.nbytes)
    dR = exL[0].device_alloc(right.nbytes)
    exL[0].h2d(dL, left)
    exL[0].h2d(dR, right)
    fbytes = rows * cols
    for s_ in range(S):
        exL[s_].extract_batch_device(dL + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
        exR[s_].extract_batch_device(dR + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
        exL[s_].synchronize()
        exR[s_].synchronize()
    outs = [e.batch_outputs() for e in exL]
    cap = outs[0][3]
    d_out = [e.device_alloc(Bs * cap * 8 + Bs * 4) for e in exL]
    mbf, mb = 386.1448, 386.1448 / 718.856  # Examples/Stereo/KITTI00-02.yaml

    # --serial-pairs (profiling): each right context's stream waits for its left context's extraction, so the L and
    # R launches of a pair do not overlap and rocprof's per-kernel durations are one context's own
    serial = None
    if args.serial_pairs:
        import torch

        serial = [(torch.cuda.ExternalStream(exL[s_].stream(), device=f"cuda:{dev}"),
                   torch.cuda.ExternalStream(exR[s_].stream(), device=f"cuda:{dev}"),
                   torch.cuda.Event()) for s_ in range(S)]

    def step():
        for s_ in range(S):
            exL[s_].extract_batch_device(dL + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
            if serial is not None:
                sl, sr, ev = serial[s_]
                ev.record(sl)
                sr.wait_event(ev)
            exR[s_].extract_batch_device(dR + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
        for s_ in range(S):
            o = d_out[s_]
            _lib.check(exL[s_].ctx, L.orbgpu_compute_stereo_matches_batch(
                exL[s_].ctx, exR[s_].ctx, mbf, mb, C.c_void_p(o), C.c_void_p(o + Bs * cap * 4),
                C.c_void_p(o + Bs * cap * 8)), "stereo")

    def post():
        counts = np.zeros(Bs, np.int32)
        nm = np.zeros(Bs, np.int32)
        kp_all, nm_all = 0, 0
        for s_ in range(S):
            exL[s_].d2h(counts, outs[s_][2])
            exL[s_].d2h(nm, d_out[s_] + Bs * cap * 8)
            kp_all += int(counts.sum())
            nm_all += int(nm.sum())
        return {"mean_left_keypoints_per_frame": round(kp_all / B, 1),
                "mean_stereo_matches_per_frame": round(nm_all / B, 1)}, kp_all / S

    def verify():
        """Parity of the timed path: every pair of the last step -- left keypoints and descriptors, the number of
        stereo matches and mvuRight / mvDepth as bit patterns (src/Frame.cc:466-640) -- against the oracle's hashes
        of the same pairs."""
        g = bench_golden(args, env["rank"], "bench_stereo_golden.json")
        if g is None:
            return {"status": "no oracle golden for this configuration/rank", "frames": 0, "mismatches": None}
        bad = checked = 0
        for s_ in range(S):
            exL[s_].synchronize()
            kp, de, cn, cap_ = outs[s_]
            kps = np.zeros(Bs * cap_ * 28, np.uint8)
            desc = np.zeros(Bs * cap_ * 32, np.uint8)
            cnt = np.zeros(Bs, np.int32)
            ur = np.zeros(Bs * cap_, np.float32)
            dp = np.zeros(Bs * cap_, np.float32)
            nm = np.zeros(Bs, np.int32)
            for dst, src in ((kps, kp), (desc, de), (cnt, cn), (ur, d_out[s_]), (dp, d_out[s_] + Bs * cap_ * 4),
                             (nm, d_out[s_] + Bs * cap_ * 8)):
                exL[s_].d2h(dst, src)
            for b in range(Bs):
                gp = g["pairs"][(s_ * Bs + b) % nuniq]
                n = int(cnt[b])
                ok = (n == gp["n"] and int(nm[b]) == gp["nmatches"] and
                      _sha(kps[b * cap_ * 28:(b * cap_ + n) * 28]) == gp["kps_sha256"] and
                      _sha(desc[b * cap_ * 32:(b * cap_ + n) * 32]) == gp["desc_sha256"] and
                      _sha(ur[b * cap_:b * cap_ + n]) == gp["uright_sha256"] and
                      _sha(dp[b * cap_:b * cap_ + n]) == gp["depth_sha256"])
                bad += int(not ok)
                checked += 1
        return {"status": "checked", "frames": checked, "unique_frames": nuniq, "mismatches": bad,
                "against": "oracle hashes of the same pairs (tests/golden/bench_stereo_golden.json)"}

    def free():
        for s_ in range(S):
            exL[s_].device_free(d_out[s_])
        exL[0].device_free(dL)
        exL[0].device_free(dR)

    return dict(metric=f"stereo frames/sec ORB extract L+R + ComputeStereoMatches @{cols}×{rows}, {NF} feat",
                exs=exL + exR, step=step, post=post, free=free, verify=verify, Bs=Bs, frames_per_step=B,
                counts=[o[2] for o in outs],
                workload=f"config 4: {cols}x{rows} rectified stereo pairs, {NF} features per image, "
                         f"left + right ORB extraction and Frame::ComputeStereoMatches (bf 386.1448)",
                cpu=lambda: cpu_baseline_stereo(rows, cols, NF, args.cpu_seconds))


MP_KEYS = ("track_in_view", "is_bad", "level", "view_cos", "proj_x", "proj_y", "proj_xr", "n_obs", "desc")


def tracking_mappoints(k, d, M, seed):
    """M local-map points sampled from the camera's own extraction -- descriptor bits
    flipped with p = 0.05, projection = keypoint + N(0, 1 px), level = octave, viewCos ~ U(0.9, 1), in view,
    2 observations, no right projection (th = 1)."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, len(k), M)
    return dict(track_in_view=np.ones(M, np.uint8), is_bad=np.zeros(M, np.uint8),
                level=k["octave"][src].astype(np.int32), view_cos=rng.uniform(0.9, 1.0, M).astype(np.float32),
                proj_x=(k["x"][src] + rng.normal(0, 1, M)).astype(np.float32),
                proj_y=(k["y"][src] + rng.normal(0, 1, M)).astype(np.float32),
                proj_xr=np.full(M, -1, np.float32), n_obs=np.full(M, 2, np.int32),
                desc=d[src] ^ np.packbits(rng.random((M, 256)) < 0.05, axis=1))


# config 5's camera model: a planar scene at depth RIG_DEPTH in front of pinhole cameras (fx = fy = RIG_F, principal
# point at the image centre, monocular); frame slot b of a rank sees it from camera translation (-dx, -dy) * depth / f,
# which moves every map point by the (dx, dy) pixel shift its synthetic frame was rendered with
RIG_F, RIG_DEPTH = 1200.0, 5.0


def frame_shift(i: int):
    """Pixel shift (dx, dy) of unique frame i of _frames (period 32)."""
    i %= 32
    return int(3 + 5 * (i % 8)), int(2 + 3 * (i // 8))


def rig_camera(cols, rows, dx, dy, scale_factor, nlevels):
    """orbgpu_camera / oracle camera dict of the camera that sees the planar map shifted by (dx, dy) pixels."""
    t = np.array([-dx * RIG_DEPTH / RIG_F, -dy * RIG_DEPTH / RIG_F, 0.0], np.float32)
    return dict(Rcw=np.eye(3, dtype=np.float32), tcw=t, Ow=-t, fx=RIG_F, fy=RIG_F, cx=cols / 2.0, cy=rows / 2.0, mbf=0.0,
                mb=0.0, scale_factor=float(scale_factor), nlevels=int(nlevels), cols=cols, rows=rows)


def local_map(k, d, M, seed, cols, rows, scale_factors):
    """SURVEY.md §8(d) config 5's local map as world points: M points sampled from the reference camera's extraction
    (identity pose), back-projected onto the plane at RIG_DEPTH with N(0, 1 px) jitter, descriptor bits flipped with
    p = 0.05; normal = viewing direction, mfMaxDistance = dist * scale^octave, mfMinDistance = max / scale^(L-1)
    (MapPoint::UpdateNormalAndDepth, src/MapPoint.cc:340-383)."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, len(k), M)
    u = (k["x"][src] + rng.normal(0, 1, M)).astype(np.float64)
    v = (k["y"][src] + rng.normal(0, 1, M)).astype(np.float64)
    pos = np.stack([(u - cols / 2.0) / RIG_F * RIG_DEPTH, (v - rows / 2.0) / RIG_F * RIG_DEPTH,
                    np.full(M, RIG_DEPTH)], 1).astype(np.float32)
    dist = np.linalg.norm(pos.astype(np.float64), axis=1).astype(np.float32)
    sf = np.asarray(scale_factors, np.float32)
    maxd = (dist * sf[k["octave"][src]]).astype(np.float32)
    return dict(pos=pos, normal=(pos / dist[:, None]).astype(np.float32), max_dist=maxd,
                min_dist=(maxd / sf[-1]).astype(np.float32), is_bad=np.zeros(M, np.uint8),
                n_obs=np.full(M, 2, np.int32), desc=d[src] ^ np.packbits(rng.random((M, 256)) < 0.05, axis=1))


MAP_FIELDS = (("pos", 12), ("normal", 12), ("max_dist", 4), ("min_dist", 4), ("is_bad", 1), ("n_obs", 4),
              ("desc", 32))


def map_offsets(M):
    """Byte offset of each field inside the local-map record: fields in MAP_FIELDS order, each starting on a 16-byte
    boundary (so the kernels' int32 / float loads stay aligned for any point count)."""
    offs, o = {}, 0
    for f, w in MAP_FIELDS:
        offs[f] = o
        o += (w * M + 15) & ~15
    offs["_end"] = o
    return offs


def pack_map(mp):
    """The local map as one byte record (the unit rank 0 broadcasts once, at set-up); fields at map_offsets."""
    M = len(mp["pos"])
    offs = map_offsets(M)
    rec = np.zeros(offs["_end"], np.uint8)
    for f, w in MAP_FIELDS:
        rec[offs[f]:offs[f] + w * M] = np.ascontiguousarray(mp[f]).view(np.uint8).reshape(-1)
    return rec


def cpu_baseline_tracking(rows, cols, nfeat, M, seconds):
    O = _oracle_fast()
    from orbslam2_with_quadrics_amd import synthetic

    ex = O.OracleExtractor(nfeat)
    sf = ex.tables()["scale"]
    scene = synthetic.make_scene(synthetic.SEED_BASE + 5000, rows, cols)
    k0, d0 = ex(synthetic.render(scene, rows, cols, 0, 0, noise_seed=1))
    mp = local_map(k0, d0, M, 7000, cols, rows, sf)

    def work(i):
        dx, dy = frame_shift(i)
        k, d = ex(synthetic.render(scene, rows, cols, dx, dy, noise_seed=10 + i))
        _, tr = O.is_in_frustum(rig_camera(cols, rows, dx, dy, 1.2, len(sf)), mp["pos"], mp["normal"],
                                mp["max_dist"], mp["min_dist"], 0.5)
        O.search_by_projection(O.OracleFrame(k, d, cols, rows, sf), dict(tr, is_bad=mp["is_bad"], n_obs=mp["n_obs"],
                                                                          desc=mp["desc"]), 0.8, 1.0)

    med, n = timed_cpu_frames(work, lambda i: i, seconds)
    return cpu_record(med, n, 10, f"{cols}x{rows}, {nfeat} features, oracle extraction + isInFrustum + "
                                 f"SearchByProjection vs a {M}-point local map (th 1)")


def setup_tracking(args, env):
    """config 5 (8-camera 1920x1080 rig, 4000 features): per camera frame, ORB extraction, Frame::isInFrustum of every
    local-map point for the camera's pose (src/Tracking.cc:1167-1180) and SearchByProjection(F, local map, th=1)
    (Tracking::SearchLocalPoints, :1184-1191).  The local map (world points) is built by rank 0 from
    its reference frame and broadcast to every rank once, at set-up; each rank's frames have their own
    camera poses."""
    import torch

    L, _lib, ORBextractor, synthetic = env["L"], env["_lib"], env["ORBextractor"], env["synthetic"]
    dist, rank = env["dist"], env["rank"]
    rows, cols, B, NF, S, dev = args.rows, args.cols, args.batch, args.nfeatures, args.streams, env["dev"]
    M = args.mappoints
    Bs = B // S
    f_ref, frames = _frames(synthetic, rows, cols, B, rank, 5000)
    exs = [ORBextractor(NF, 1.2, 8, 20, 7, device=dev, semantics=args.semantics) for _ in range(S)]
    sfac = exs[0].GetScaleFactors()
    # the local map: rank 0 extracts its reference frame and builds it; the byte record is broadcast every step
    k0, d0 = exs[0](f_ref)
    mp = local_map(k0, d0, M, 7000, cols, rows, sfac)
    d_frames = exs[0].device_alloc(frames.nbytes)
    exs[0].h2d(d_frames, frames)
    fbytes = rows * cols
    for s_, e in enumerate(exs):
        e.extract_batch_device(d_frames + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
        e.synchronize()
    outs = [e.batch_outputs() for e in exs]
    cap = outs[0][3]
    rec_h = pack_map(mp)
    rec = torch.from_numpy(rec_h).to(f"cuda:{dev}")
    # the local map from rank 0, once (before any frame is matched against it): rank 0's record overwrites the
    # other ranks' (they built theirs from their own reference frame only to size the buffer)
    broadcast_record(dist, rank, rec, lambda buf: None, lambda buf: torch.cuda.current_stream().synchronize())
    offs = {f: rec.data_ptr() + o for f, o in map_offsets(M).items() if f != "_end"}
    geom = _lib.MapPointGeomView(M, offs["pos"], offs["normal"], offs["max_dist"], offs["min_dist"])
    grid = _lib.GridGeom()
    L.orbgpu_grid_geom_for_image(cols, rows, C.byref(grid))
    # per stream: cameras of its frame slots (device), the track fields (Bs x M), owners
    per = []
    for s_, e in enumerate(exs):
        cams = np.zeros((Bs, 23), np.float32)
        for b in range(Bs):
            c = rig_camera(cols, rows, *frame_shift(s_ * Bs + b), 1.2, len(sfac))
            cams[b, :9] = c["Rcw"].reshape(9)
            cams[b, 9:12] = c["tcw"]
            cams[b, 12:15] = c["Ow"]
            cams[b, 15:22] = [c["fx"], c["fy"], c["cx"], c["cy"], c["mbf"], c["mb"], c["scale_factor"]]
            cams[b, 22] = np.array([c["nlevels"]], np.int32).view(np.float32)[0]
        d_cams = e.device_alloc(cams.nbytes)
        e.h2d(d_cams, cams)
        tr = {f: e.device_alloc(Bs * M * w) for f, w in (("iv", 1), ("px", 4), ("py", 4), ("pxr", 4), ("lv", 4),
                                                          ("vc", 4))}
        d_none = e.device_alloc(Bs * cap * 4)  # mvpMapPoints all NULL at SearchLocalPoints time
        e.h2d(d_none, np.full(Bs * cap, -1, np.int32))
        d_zero = e.device_alloc(Bs * cap * 4)  # ... so no owner has observations (the oracle's convention: 0)
        e.h2d(d_zero, np.zeros(Bs * cap, np.int32))
        view = _lib.MapPointsView(M, tr["iv"], offs["is_bad"], tr["lv"], tr["vc"], tr["px"], tr["py"], tr["pxr"],
                                  offs["n_obs"], offs["desc"])
        per.append(dict(cams=d_cams, tr=tr, none=d_none, zero=d_zero, own=e.device_alloc(Bs * cap * 4),
                        obs=e.device_alloc(Bs * cap * 4), nm=e.device_alloc(Bs * 4), view=view))

    def step():
        for s_, e in enumerate(exs):
            q = per[s_]
            e.extract_batch_device(d_frames + s_ * Bs * fbytes, Bs, cols, rows, cols, fbytes)
            tr = q["tr"]
            _lib.check(e.ctx, L.orbgpu_is_in_frustum_batch(e.ctx, C.c_void_p(q["cams"]), Bs, grid, C.byref(geom), 0.5,
                                                           M, C.c_void_p(tr["iv"]), C.c_void_p(tr["px"]),
                                                           C.c_void_p(tr["py"]), C.c_void_p(tr["pxr"]),
                                                           C.c_void_p(tr["lv"]), C.c_void_p(tr["vc"])), "frustum")
            _lib.check(e.ctx, L.orbgpu_memcpy_d2d_async(e.ctx, C.c_void_p(q["own"]), C.c_void_p(q["none"]),
                                                        Bs * cap * 4), "d2d")
            _lib.check(e.ctx, L.orbgpu_memcpy_d2d_async(e.ctx, C.c_void_p(q["obs"]), C.c_void_p(q["zero"]),
                                                        Bs * cap * 4), "d2d")
        for s_, e in enumerate(exs):
            q = per[s_]
            _lib.check(e.ctx, L.orbgpu_search_by_projection_batch_shared_map(
                e.ctx, C.byref(q["view"]), M, 0.8, 1.0, None, C.c_void_p(q["own"]), C.c_void_p(q["obs"]),
                C.c_void_p(q["nm"])), "search_proj")

    def post():
        counts = np.zeros(Bs, np.int32)
        nm = np.zeros(Bs, np.int32)
        kp_all, nm_all = 0, 0
        for s_, e in enumerate(exs):
            e.d2h(counts, outs[s_][2])
            e.d2h(nm, per[s_]["nm"])
            kp_all += int(counts.sum())
            nm_all += int(nm.sum())
        return {"mean_keypoints_per_frame": round(kp_all / B, 1), "map_points": M,
                "mean_projection_matches_per_frame": round(nm_all / B, 1),
                "local_map": "world points broadcast from rank 0 once at set-up; per-frame isInFrustum on the GPU"}, \
            kp_all / S

    def verify():
        """Parity of the timed path: every frame of the last step -- keypoints, descriptors, nmatches and the
        mvpMapPoints owner / observation vectors of SearchByProjection after isInFrustum (src/ORBmatcher.cc:45-137,
        src/Frame.cc:269-325) -- against the oracle's hashes of the same frames and cameras."""
        g = bench_golden(args, env["rank"], "bench_tracking_golden.json")
        if g is None or g.get("mappoints", M) != M:
            return {"status": "no oracle golden for this configuration/rank", "frames": 0, "mismatches": None}
        nuniq = min(B, 32)
        bad = checked = 0
        field_bad = {}
        for s_, e in enumerate(exs):
            e.synchronize()
            q = per[s_]
            kp, de, cn, cap_ = outs[s_]
            kps = np.zeros(Bs * cap_ * 28, np.uint8)
            desc = np.zeros(Bs * cap_ * 32, np.uint8)
            cnt = np.zeros(Bs, np.int32)
            own = np.zeros(Bs * cap_, np.int32)
            obs = np.zeros(Bs * cap_, np.int32)
            nm = np.zeros(Bs, np.int32)
            for dst, src in ((kps, kp), (desc, de), (cnt, cn), (own, q["own"]), (obs, q["obs"]), (nm, q["nm"])):
                e.d2h(dst, src)
            if os.environ.get("ORBGPU_BENCH_DUMP"):  # diagnostics: the downloaded arrays of this stream
                np.savez(os.environ["ORBGPU_BENCH_DUMP"] + f"_s{s_}.npz", kps=kps, desc=desc, cnt=cnt, own=own, obs=obs,
                         nm=nm, cap=cap_)
            for b in range(Bs):
                gf = g["frames"][(s_ * Bs + b) % nuniq]
                n = int(cnt[b])
                fields = dict(n=n == gf["n"], nmatches=int(nm[b]) == gf["nmatches"],
                              kps=_sha(kps[b * cap_ * 28:(b * cap_ + n) * 28]) == gf["kps_sha256"],
                              desc=_sha(desc[b * cap_ * 32:(b * cap_ + n) * 32]) == gf["desc_sha256"],
                              owner=_sha(own[b * cap_:b * cap_ + n]) == gf["owner_sha256"],
                              owner_obs=_sha(obs[b * cap_:b * cap_ + n]) == gf["owner_obs_sha256"])
                for k_, v in fields.items():
                    field_bad[k_] = field_bad.get(k_, 0) + int(not v)
                bad += int(not all(fields.values()))
                checked += 1
        if bad:
            log(f"tracking parity: mismatching frames per field {field_bad}")
        return {"status": "checked", "frames": checked, "unique_frames": nuniq, "mismatches": bad,
                "against": "oracle hashes of the same frames and cameras (tests/golden/bench_tracking_golden.json)"}

    def free():
        for s_, e in enumerate(exs):
            q = per[s_]
            for p in [q["cams"], q["none"], q["zero"], q["own"], q["obs"], q["nm"]] + list(q["tr"].values()):
                e.device_free(p)
        exs[0].device_free(d_frames)

    return dict(metric=f"frames/sec ORB extract + isInFrustum + SearchByProjection vs {M} map points "
                       f"@{cols}×{rows}, {NF} feat",
                exs=exs, step=step, post=post, free=free, verify=verify, Bs=Bs, frames_per_step=B,
                counts=[o[2] for o in outs], streams_state=per,
                # the map record's device memory is read by every step's kernels through raw pointers (offs): the
                # tensor must outlive set-up, or torch's caching allocator hands its memory to later tensors
                map_record=rec,
                workload=f"config 5: {cols}x{rows} camera frames, {NF} features, ORB extraction + isInFrustum + "
                         f"SearchByProjection (th 1, ratio 0.8) against a {M}-point local map shared by all cameras",
                cpu=lambda: cpu_baseline_tracking(rows, cols, NF, M, args.cpu_seconds))


WORKLOADS = {"mono_init": setup_mono_init, "extract": setup_extract, "stereo": setup_stereo, "tracking": setup_tracking}
DEFAULT_SHAPE = {"mono_init": (1080, 1920, 2000), "extract": (480, 640, 1000), "stereo": (376, 1241, 2000),
                 "tracking": (1080, 1920, 4000)}
# extractor contexts (HIP streams) per GPU by default: the faster of 1 and 2 per workload on MI355X, alternated A/B
# runs (profiles/sweeps/r05_streams_all.txt: one stream +0.2-1.2 % at config 3, +1.8 % at config 4, equal at config
# 2, -0.5 % at config 5)
DEFAULT_STREAMS = {"mono_init": 1, "extract": 1, "stereo": 1, "tracking": 2}


def cpu_baseline_extract(rows, cols, nfeat, seconds):
    O = _oracle_fast()
    from orbslam2_with_quadrics_amd import synthetic

    ex = O.OracleExtractor(nfeat)
    scene = synthetic.make_scene(synthetic.SEED_BASE + 998, rows, cols)
    med, n = timed_cpu_frames(lambda f: ex(f), lambda i: synthetic.render(scene, rows, cols, i % 9, i % 5,
                                                                          noise_seed=100 + i), seconds)
    return cpu_record(med, n, 10, f"{cols}x{rows}, {nfeat} features, oracle extraction")


def cpu_baseline_stereo(rows, cols, nfeat, seconds):
    O = _oracle_fast()
    from orbslam2_with_quadrics_amd import synthetic

    exL, exR = O.OracleExtractor(nfeat), O.OracleExtractor(nfeat)
    pairs = [synthetic.stereo_pair(900 + i, rows, cols) for i in range(4)]

    def work(p):
        kL, dL = exL(p[0])
        kR, dR = exR(p[1])
        O.stereo_matches(exL, exR, kL, dL, kR, dR, 386.1448, 386.1448 / 718.856)

    med, n = timed_cpu_frames(work, lambda i: pairs[i % 4], seconds)
    r = cpu_record(med, n, 10, f"{cols}x{rows} stereo pairs, {nfeat} features, oracle L+R extraction + "
                              f"ComputeStereoMatches")
    r["unit"] = "pairs/s"
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks, one process per GPU) on this node; N > 1 without torch.distributed.run's "
                         "WORLD_SIZE starts the N ranks itself (plan_launch); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=500)  # ~5 s timed: long enough for outside GPU-busy sampling
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="frames (pairs) per step per GPU")
    ap.add_argument("--streams", type=int, default=None,
                    help="concurrent extractor contexts (HIP streams) per GPU (default per workload, DEFAULT_STREAMS)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="mono_init",
                    help="mono_init = BASELINE.json's config 3 (the headline metric); extract = config 2; "
                         "stereo = config 4; tracking = config 5")
    ap.add_argument("--mappoints", type=int, default=5000, help="local-map points per camera (tracking)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="sequential launches per stream per step (mono_init; default 1, with --host-io 8: chunk r+1 "
                         "uploads while chunk r computes)")
    ap.add_argument("--host-io", action="store_true",
                    help="mono_init: frames come from pinned host memory and keypoints/descriptors go back to it "
                         "inside the timed step (the PCIe-inclusive rate; not the headline value)")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--nfeatures", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--semantics", type=lambda v: int(v, 0), default=0,
                    help="ORBGPU_SEM_* flags (include/orbgpu.h): which OpenCV/compiler behaviours to reproduce")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial-pairs", action="store_true",
                    help="stereo (profiling): the right extraction of a pair waits for the left one, so per-kernel "
                         "durations are not inflated by the overlapping L/R launches")
    ap.add_argument("--instrumented-steps", type=int, default=50,
                    help="steps of the separate stage-timed pass (per-stage times and the roofline's launch time)")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC per-stage summary (tools/pmc_summary.py) the roofline's traffic comes from; default "
                         "profiles/pmc_latest.json (mono_init) or profiles/pmc_latest_<workload>.json")
    args = ap.parse_args()
    how, what = plan_launch(args.gpus, os.environ, sys.argv[1:])
    if how == "spawn":  # before `import torch`: this process stays off the GPU
        sys.exit(spawn_ranks(what))
    if args.streams is None:
        args.streams = DEFAULT_STREAMS[args.workload]
    if args.chunks is None:
        args.chunks = 8 if args.host_io else 1
    r0, c0, n0 = DEFAULT_SHAPE[args.workload]
    args.rows = args.rows or r0
    args.cols = args.cols or c0
    args.nfeatures = args.nfeatures or n0
    if args.batch % args.streams:
        raise SystemExit(f"--batch {args.batch} must be a multiple of --streams {args.streams}")

    world, rank, local = dist_env()
    import torch  # noqa: F401  (imported before liborbgpu.so: one HIP runtime in the process)

    from orbslam2_with_quadrics_amd import ORBextractor, _lib, synthetic

    backend = os.environ.get("ORBGPU_BENCH_BACKEND", "nccl")
    dev = pick_device(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)), torch.cuda.device_count(), backend)
    torch.cuda.set_device(dev)  # before the process group: RCCL binds each rank's communicator to this device
    dist = dist_init(world, backend)
    env = dict(L=_lib.lib(), _lib=_lib, ORBextractor=ORBextractor, synthetic=synthetic, dev=dev, rank=rank,
               dist=dist, world=world)
    t = time.time()
    W = WORKLOADS[args.workload](args, env)
    log(f"rank {rank}: {args.workload} set up in {time.time() - t:.1f}s")
    exs, Bs, S, B = W["exs"], W["Bs"], args.streams, W["frames_per_step"]
    Bps = W.get("per_stream", Bs)  # frames per stream per step (Bs = frames per launch)
    counts_t = torch.zeros(B, dtype=torch.int32, device=f"cuda:{dev}")
    streams = [torch.cuda.ExternalStream(e.stream(), device=f"cuda:{dev}") for e in exs]

    def copy_counts(s_, e):
        _lib.check(e.ctx, _lib.lib().orbgpu_memcpy_d2d_async(
            e.ctx, C.c_void_p(counts_t.data_ptr() + 4 * s_ * Bps), C.c_void_p(W["counts"][s_]), Bps * 4), "d2d")

    def after_gather(s_, e):
        # the next step's copy into counts_t waits (on the GPU) for this step's all-gather, which reads it on the
        # collective's stream: a stream wait, not a host synchronisation
        streams[s_].wait_stream(torch.cuda.current_stream())

    def step():
        multi_rank_step(W["step"], exs, dist, world, counts_t, copy_counts, after_gather, len(W["counts"]))

    stage_acc = {}
    union_acc = {}  # stage -> total time with >= 1 launch of it running (union over the concurrent contexts)

    def collect():
        for e in exs:
            for name, ms in e.stage_times():
                a = stage_acc.setdefault(name, [0.0, 0])
                a[0] += ms
                a[1] += 1
        ivs = {}
        for e in exs:
            marks = e.stage_marks(exs[0])
            for (_, t0), (name, t1) in zip(marks, marks[1:]):
                ivs.setdefault(name, []).append((t0, t1))
        for name, iv in ivs.items():
            union_acc[name] = union_acc.get(name, 0.0) + interval_union(iv)

    for i in range(args.warmup):
        step()

    def timed(n, instrumented):
        # n steps bracketed by a barrier + device synchronisation on both sides; returns this rank's seconds.
        # instrumented: HIP-event stage timing on every context stream and the host reads the events after each
        # step (collect), so those steps carry the instrumentation; the headline loop runs without it
        for e in exs:
            e.set_stage_timing(instrumented)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            step()
            if instrumented:
                collect()
            if i == 0 or (i + 1) % 50 == 0:
                log(f"rank {rank}: {'instrumented' if instrumented else 'timed'} step {i + 1}/{n}")
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        dt_ = time.perf_counter() - t0
        for e in exs:
            e.set_stage_timing(False)
        return dt_

    # the per-stage breakdown and the roofline's launch time come from a separate instrumented pass before the
    # timed loop; `value` and `ms_per_step` come from the uninstrumented loop (extract + match + count all-gather)
    n_inst = max(1, min(args.steps, args.instrumented_steps))
    dt_inst = max_over_ranks(dist, timed(n_inst, True), device=f"cuda:{dev}")
    dt = timed(args.steps, False)
    dt_ranks = per_rank_values(dist, dt, device=f"cuda:{dev}")
    dt = max_over_ranks(dist, dt, device=f"cuda:{dev}")

    # ---- per-stage averages and the dominant kernel's roofline (per-launch quantities: one launch processes
    # one context's Bs frames)
    cand_total = sum(_lib.lib().orbgpu_batch_candidate_total(e.ctx) for e in exs) / len(exs)
    extra, kp_total = W["post"]()
    parity = W["verify"]() if "verify" in W else None
    if parity is not None and dist is not None:  # every rank joins the reduction, with or without goldens
        import torch

        has = parity["mismatches"] is not None
        t = torch.tensor([parity["frames"], parity["mismatches"] if has else 0, int(has)], dtype=torch.int64,
                         device=f"cuda:{dev}")
        dist.all_reduce(t)
        parity = dict(parity, frames=int(t[0]), mismatches=int(t[1]) if int(t[2]) else None, ranks=world,
                      ranks_checked=int(t[2]))
    P = level_pixels(args.cols, args.rows, exs[0].GetInverseScaleFactors())
    stages = {k: v[0] / max(v[1], 1) for k, v in stage_acc.items()}
    kernels = {k: v for k, v in stages.items()
               if k in ("pyramid", "fast", "octree", "describe", "grid", "search_init", "search_proj", "stereo",
                        "frustum")}
    dom = max(kernels, key=kernels.get)
    # effective launch duration: time the GPU has >= 1 launch of the kernel running, per launch.  With
    # concurrent streams a launch's own event span also covers the co-running launches; the union does
    # not (and equals the plain average when launches do not overlap, e.g. under the profiler).
    launches = stage_acc[dom][1]
    dom_ms = union_acc[dom] / max(launches, 1)
    dom_ms_span = kernels[dom]
    dom_bytes = stage_bytes(dom, Bs, P, cand_total, kp_total, args.mappoints)
    traffic = None
    valu = None
    pmc_json = args.pmc_json or os.path.join(ROOT, "profiles", "pmc_latest.json" if args.workload == "mono_init"
                                             else f"pmc_latest_{args.workload}.json")
    if os.path.exists(pmc_json):
        try:
            pmc = json.load(open(pmc_json))
            pk = pmc.get("kernels", {}).get(dom, {})
            scale = Bs / pmc["batch"] if pmc.get("batch", Bs) != Bs else 1.0  # per-frame linear in the batch
            traffic = pk.get("hbm_bytes_per_launch")
            if traffic is not None:
                traffic = int(traffic * scale)
            if pk.get("SQ_INSTS_VALU"):
                # VALU pipe occupancy, 256 CUs x 4 SIMDs at 2.4 GHz.  A wave64 VALU instruction holds its SIMD-32 for
                # 2 cycles (v_add_u32, v_and/or/xor, v_add/fma_f32, 16-bit v_max/min/add, v_mov) or 4 cycles (packed
                # 16-bit, 3-input, v_perm, v_mbcnt, v_cmp, 32-bit v_max/min, v_lshlrev, 24-bit multiplies), measured by
                # tools/micro/valu_rate.hip (profiles/r05_valu_issue_rates.txt): the two bounds bracket the kernel's mix
                insts = pk["SQ_INSTS_VALU"] * scale
                den = dom_ms * 1e-3 * VALU_CLK_HZ * VALU_SIMDS
                valu = {"insts_per_launch": int(insts),
                        "busy_frac_if_4cyc": round(insts * 4 / den, 4),
                        "busy_frac_if_2cyc": round(insts * 2 / den, 4),
                        "note": f"PMC SQ_INSTS_VALU ({os.path.relpath(pmc_json, ROOT)}) x 4 (or 2) cycles / "
                                "(avg_launch_ms x 2.4 GHz x 1024 SIMDs); the 4-cycle forms dominate the FAST, describe "
                                "and resize kernels, so the first is the closer one (DESIGN.md §6)"}
        except Exception:
            traffic = None
            valu = None

    total_frames = world * B * args.steps
    value = total_frames / dt
    out = {
        "metric": W["metric"],
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": dict({
            "workload": W["workload"],
            "frames_per_step_per_gpu": B,
            "streams_per_gpu": S,
            "frames_per_launch": Bs,
            **({"serial_pairs": True} if args.serial_pairs else {}),
            "resolution": f"{args.cols}x{args.rows}",
            "nfeatures": args.nfeatures,
            "semantics": _lib.semantics_name(args.semantics),
            "parallelism": f"frame-sharded x{world} GPUs, {S} streams per GPU (RCCL all-gather of keypoint "
                           f"counts only)",
        }, **extra),
        "roofline": roofline_record(dom, dom_bytes, candidate_bytes(dom, cand_total), dom_ms, dom_ms_span, traffic,
                                    valu),
        "parity": parity,
        # what the collectives ran on: the process group's own world size (RCCL = backend "nccl" on ROCm)
        "collective": {"backend": dist.get_backend() if dist is not None else None,
                       "world_size": dist.get_world_size() if dist is not None else 1,
                       "launcher": os.environ.get("ORBGPU_BENCH_LAUNCHER",
                                                  "torch.distributed.run" if world > 1 else "single process")},
        "stages_ms_per_launch": {k: round(v, 4) for k, v in stages.items()},
        "stages_busy_ms_per_step": {k: round(v / n_inst, 4) for k, v in union_acc.items()},
        # the pass the stages and the roofline's launch time come from (HIP-event stage timing on; not `value`)
        "instrumented": {"steps": n_inst, "ms_per_step": round(dt_inst / n_inst * 1e3, 3)},
    }
    if world > 1:  # each rank's own step time (the value above uses their maximum)
        out["per_rank_ms_per_step"] = [round(v / args.steps * 1e3, 3) for v in dt_ranks]
    if "pcie" in out["config"]:  # --host-io: the step's transfers against the measured link peak
        pc = out["config"].pop("pcie")
        step_s = dt / args.steps
        h2d = pc["h2d_bytes_per_step"] / step_s / 1e9
        both = (pc["h2d_bytes_per_step"] + pc["d2h_bytes_per_step"]) / step_s / 1e9
        out["pcie"] = dict(pc, achieved_h2d_GBps=round(h2d, 2), achieved_total_GBps=round(both, 2),
                           h2d_frac_of_peak=round(h2d / pc["link_peak"]["h2d_GBps"], 3),
                           total_frac_of_bidir_peak=round(both / pc["link_peak"]["bidir_GBps"], 3))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU baseline (oracle, 1 thread)")
        out["cpu_baseline"] = W["cpu"]()
    elif rank == 0:
        out["cpu_baseline"] = None
    W["free"]()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
