"""CPU baseline of BASELINE.md §2: the oracle (plain-C restatement of the reference path) built with the reference's
flags (-O3 -march=native, contractions explicit: bit-identical to the checker build), on this host's cores.

Per config: 10 warm-up frames, then >= 200 timed frames pinned to one core (os.sched_setaffinity, as taskset -c 0),
median and mean per frame; then an all-cores frame-parallel run (one worker process per core, each pinned, frames
dealt round-robin) whose throughput is total frames / wall time.  Records the CPU model and nproc.

    python tools/cpu_baseline.py [--frames 200] [--configs 2,3,4,5] [--out profiles/r02_cpu_baseline.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
os.environ["ORB_ORACLE_FAST"] = "1"

import numpy as np  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def make_config(cfg):
    """(per-frame work function, frame generator, description) of a BASELINE config on synthetic frames
    (SURVEY.md §8(d) recipes)."""
    import oracle_py as O
    from orbslam2_with_quadrics_amd import synthetic

    O.build()
    if cfg == 2:
        ex = O.OracleExtractor(1000)
        scene = synthetic.make_scene(synthetic.SEED_BASE + 998, 480, 640)

        def frame(i):
            return synthetic.render(scene, 480, 640, i % 9, i % 5, noise_seed=100 + i)

        return (lambda f: ex(f)), frame, "640x480, 1000 features: ORB extraction"
    if cfg == 3:
        ex = O.OracleExtractor(2000)
        scene = synthetic.make_scene(synthetic.SEED_BASE + 999, 1080, 1920)
        f1 = synthetic.render(scene, 1080, 1920, 0, 0, noise_seed=5)
        k1, d1 = ex(f1)
        sf = ex.tables()["scale"]
        F1 = O.OracleFrame(k1, d1, 1920, 1080, sf)
        prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)

        def work(f):
            k2, d2 = ex(f)
            O.search_for_initialization(F1, O.OracleFrame(k2, d2, 1920, 1080, sf), prev.copy(), 0.9, True, 100)

        def frame(i):
            return synthetic.render(scene, 1080, 1920, 3 + i % 9, 2 + i % 5, noise_seed=100 + i)

        return work, frame, "1920x1080, 2000 features: ORB extraction + SearchForInitialization (window 100, 0.9)"
    if cfg == 4:
        exL, exR = O.OracleExtractor(2000), O.OracleExtractor(2000)
        pairs = [synthetic.stereo_pair(900 + i, 376, 1241) for i in range(4)]

        def work(p):
            kL, dL = exL(p[0])
            kR, dR = exR(p[1])
            O.stereo_matches(exL, exR, kL, dL, kR, dR, 386.1448, 386.1448 / 718.856)

        return work, (lambda i: pairs[i % 4]), "1241x376 stereo pairs, 2000 features: L+R extraction + " \
                                              "ComputeStereoMatches"
    if cfg == 5:
        sys.path.insert(0, ROOT)
        import bench

        ex = O.OracleExtractor(4000)
        sf = ex.tables()["scale"]
        scene = synthetic.make_scene(synthetic.SEED_BASE + 997, 1080, 1920)
        cache = {}

        def frame(i):
            f = synthetic.render(scene, 1080, 1920, i % 9, i % 5, noise_seed=300 + i % 16)
            if i % 16 not in cache:
                k0, d0 = ex(f)
                cache[i % 16] = bench.tracking_mappoints(k0, d0, 5000, i % 16)
            return f, cache[i % 16]

        def work(fm):
            k, d = ex(fm[0])
            O.search_by_projection(O.OracleFrame(k, d, 1920, 1080, sf), fm[1], 0.8, 1.0)

        return work, frame, "1920x1080, 4000 features: ORB extraction + SearchByProjection vs 5000 map points (th 1)"
    raise ValueError(cfg)


def single_core(cfg, n, warm, core=None):
    prev = os.sched_getaffinity(0)
    core = min(prev) if core is None else core  # the lowest core this process may use (a box's cpuset may lack 0)
    os.sched_setaffinity(0, {core})
    try:
        work, frame, desc = make_config(cfg)
        frames = [frame(i) for i in range(warm + n)]
        for f in frames[:warm]:
            work(f)
        ts = []
        for f in frames[warm:]:
            t = time.perf_counter()
            work(f)
            ts.append(time.perf_counter() - t)
            if len(ts) % 50 == 0:
                print(f"config {cfg}: {len(ts)}/{n} frames on core {core}", file=sys.stderr, flush=True)
    finally:
        os.sched_setaffinity(0, prev)
    return desc, ts, core


def _worker(args):
    cfg, core, idx = args
    os.sched_setaffinity(0, {core})
    work, frame, _ = make_config(cfg)
    frames = [frame(i) for i in idx]
    work(frames[0])  # warm-up
    t = time.perf_counter()
    for f in frames:
        work(f)
    return time.perf_counter() - t, len(frames)


def all_cores(cfg, n, max_cores):
    from multiprocessing import get_context

    cores = sorted(os.sched_getaffinity(0))[:max_cores]
    per = max(1, n // len(cores))
    with get_context("spawn").Pool(len(cores)) as pool:
        t = time.perf_counter()
        res = pool.map(_worker, [(cfg, c, list(range(k * per, (k + 1) * per))) for k, c in enumerate(cores)])
        wall = time.perf_counter() - t
    busy = max(r[0] for r in res)
    tot = sum(r[1] for r in res)
    return {"cores": len(cores), "frames": tot, "frames_per_s": round(tot / busy, 3),
            "note": "per-worker timed loops after setup; throughput = all frames / slowest worker's loop time",
            "wall_incl_setup_s": round(wall, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--configs", default="2,3,4,5")
    ap.add_argument("--max-cores", type=int, default=16, help="workers of the all-cores run (the GPU box's CPU share)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_cpu_baseline.json"))
    args = ap.parse_args()
    out = {"cpu_model": cpu_model(), "nproc": os.cpu_count(), "oracle_build": "gcc -O3 -march=native "
           "-ffp-contract=off (oracle/Makefile liborb_oracle_fast.so; bit-identical to the checker build)",
           "kind": "port", "caveat": "the oracle's resize / FAST / GaussianBlur are scalar C; an OpenCV SIMD build of "
           "the reference would be faster", "configs": {}}
    for cfg in [int(c) for c in args.configs.split(",")]:
        desc, ts, core = single_core(cfg, args.frames, args.warmup)
        med = statistics.median(ts)
        entry = {"workload": desc, "single_core": {"frames": len(ts), "warmup": args.warmup,
                                                  "median_ms": round(med * 1e3, 3),
                                                  "mean_ms": round(statistics.mean(ts) * 1e3, 3),
                                                  "frames_per_s_median": round(1 / med, 3), "pinned_core": core}}
        entry["all_cores"] = all_cores(cfg, args.frames, args.max_cores)
        out["configs"][str(cfg)] = entry
        print(cfg, json.dumps(entry), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
