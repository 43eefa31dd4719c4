"""The headline timed path at its own shape (bench.py config 3): 1920x1080, 2000 features, 512 frames per step --
bench.py's default, one extractor context (HIP stream) x 512 frames per launch, and the two-context form, 2 x 256
frames on concurrently running streams -- SearchForInitialization of every frame against the initial frame.  Every
one of the 512 frames is checked against the oracle's hashes of the same frame (tests/golden/bench_golden.json, made
by tests/golden/make_golden.py from bench._frames), and the first, second, middle and last frame of each launch field
by field against a live oracle run.  Also bench.py itself: `--gpus 2` starting its own two ranks (gloo on the one
GPU), and the secondary workloads' timed parity."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("S,Bs", [(1, 512), (2, 256)], ids=["default_1x512", "two_streams_2x256"])
def test_bench_shape(gpu, oracle, S, Bs):
    import ctypes as C

    sys.path.insert(0, ROOT)
    import bench
    from orbslam2_with_quadrics_amd import _lib, synthetic
    from orbslam2_with_quadrics_amd.extractor import KP_DTYPE

    rows, cols, NF = 1080, 1920, 2000
    assert S == bench.DEFAULT_STREAMS["mono_init"] or S == 2
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_golden.json")))["ranks"][0]
    f1, frames = bench._frames(synthetic, rows, cols, S * Bs, 0)
    L = _lib.lib()
    ex_ref = gpu.ORBextractor(NF, 1.2, 8, 20, 7)
    exs = [gpu.ORBextractor(NF, 1.2, 8, 20, 7) for _ in range(S)]
    fb = rows * cols
    d_f1 = ex_ref.device_alloc(f1.nbytes)
    d_frames = exs[0].device_alloc(frames.nbytes)
    bufs = []
    try:
        ex_ref.h2d(d_f1, f1)
        exs[0].h2d(d_frames, frames)
        grid = _lib.GridGeom()
        L.orbgpu_grid_geom_for_image(cols, rows, C.byref(grid))
        ex_ref.extract_batch_device(d_f1, 1, cols, rows, cols, fb)
        for s, e in enumerate(exs):  # both streams enqueued before either is waited on: they run concurrently
            e.extract_batch_device(d_frames + s * Bs * fb, Bs, cols, rows, cols, fb)
        outs = [e.batch_outputs() for e in exs]
        cap = outs[0][3]
        for s, e in enumerate(exs):
            prev, m12, nm = (e.device_alloc(Bs * cap * 8), e.device_alloc(Bs * cap * 4), e.device_alloc(Bs * 4))
            bufs.append((e, prev, m12, nm))
            _lib.check(e.ctx, L.orbgpu_prev_matched_from_frame(ex_ref.ctx, 0, e.ctx, C.c_void_p(prev)), "prev")
            _lib.check(e.ctx, L.orbgpu_search_for_initialization_batch(ex_ref.ctx, 0, e.ctx, grid, 0.9, 1, 100,
                                                                         C.c_void_p(prev), C.c_void_p(m12),
                                                                         C.c_void_p(nm)), "search")
        for e in exs + [ex_ref]:
            e.synchronize()
        k1, d1 = ex_ref.batch_download(0)
        assert _sha(k1) == g["f1"]["kps_sha256"] and _sha(d1) == g["f1"]["desc_sha256"]
        n1 = len(k1)
        oe = oracle.OracleExtractor(NF)
        ko1, do1 = oe(f1)
        F1 = oracle.OracleFrame(ko1, do1, cols, rows, oe.tables()["scale"])
        bad = []
        for s, (e, prev, m12, nm) in enumerate(bufs):
            M = np.zeros(Bs * cap, np.int32)
            P = np.zeros(Bs * cap * 2, np.float32)
            NM = np.zeros(Bs, np.int32)
            e.d2h(M, m12)
            e.d2h(P, prev)
            e.d2h(NM, nm)
            for b in range(Bs):
                k, d = e.batch_download(b)
                gf = g["frames"][(s * Bs + b) % 32]
                m, p = M[b * cap:b * cap + n1], P[2 * b * cap:2 * (b * cap + n1)]
                if not (_sha(k) == gf["kps_sha256"] and _sha(d) == gf["desc_sha256"] and NM[b] == gf["nmatches"]
                        and _sha(m) == gf["matches12_sha256"] and _sha(p) == gf["prev_sha256"]):
                    bad.append((s, b))
                if b in (0, 1, Bs // 2, Bs - 1):  # field by field against the live oracle
                    ko, do = oe(frames[s * Bs + b])
                    assert len(k) == len(ko)
                    for f in FIELDS:
                        assert np.array_equal(k[f].view(np.int32), ko[f].view(np.int32)), (s, b, f)
                    assert np.array_equal(d, do)
                    prev0 = np.stack([ko1["x"], ko1["y"]], 1).astype(np.float32)
                    no, mo, po = oracle.search_for_initialization(
                        F1, oracle.OracleFrame(ko, do, cols, rows, oe.tables()["scale"]), prev0, 0.9, True, 100)
                    assert NM[b] == no and np.array_equal(m, mo) and np.array_equal(p.reshape(-1, 2), po), (s, b)
        assert not bad, bad[:10]
    finally:
        for e, prev, m12, nm in bufs:
            for q in (prev, m12, nm):
                e.device_free(q)
        exs[0].device_free(d_frames)
        ex_ref.device_free(d_f1)
    assert KP_DTYPE.itemsize == 28


def test_grid_csr_batch256_vs_oracle(gpu, oracle):
    """Frame::AssignFeaturesToGrid of a 256-frame 1080p batch compared array by array with the oracle's grid
    (cell starts and per-cell item lists, src/Frame.cc:230-245) -- the grid kernel's LDS sort at the batch size
    where its round-1 generic-pointer form faulted."""
    import ctypes as C

    sys.path.insert(0, ROOT)
    import bench
    from orbslam2_with_quadrics_amd import _lib, synthetic

    rows, cols, NF, B = 1080, 1920, 2000, 256
    _, frames = bench._frames(synthetic, rows, cols, B, 0)
    ex = gpu.ORBextractor(NF, 1.2, 8, 20, 7)
    d = ex.device_alloc(frames.nbytes)
    try:
        ex.h2d(d, frames)
        ex.extract_batch_device(d, B, cols, rows, cols, rows * cols)
        ex.synchronize()  # raises on a tripped range check (status bit 64)
        cap = ex.batch_outputs()[3]
        cs, ci = C.c_void_p(), C.c_void_p()
        _lib.check(ex.ctx, _lib.lib().orbgpu_batch_grid(ex.ctx, C.byref(cs), C.byref(ci)), "grid")
        CS = np.zeros(B * 3073, np.int32)
        CI = np.zeros(B * cap, np.int32)
        ex.d2h(CS, cs.value)
        ex.d2h(CI, ci.value)
        sf = ex.GetScaleFactors()
        for b in range(0, B, 17):
            k, dsc = ex.batch_download(b)
            of = oracle.OracleFrame(k, dsc, cols, rows, sf)
            s0 = CS[b * 3073:(b + 1) * 3073]
            assert np.array_equal(s0, of.cell_start), b
            assert np.array_equal(CI[b * cap:b * cap + s0[-1]], of.cell_items[:s0[-1]]), b
    finally:
        ex.device_free(d)


@pytest.mark.parametrize("workload", ["tracking", "stereo", "extract", "stereo --serial-pairs"])
def test_bench_workload_timed_parity(gpu, workload):
    """Each secondary bench workload end to end (bench.py as the driver runs it, a short run): the timed path's
    own parity check against the oracle goldens must report zero mismatches.  Catches state shared between set-up
    and the timed steps (e.g. the config-5 map record, read through raw pointers by every step)."""
    import subprocess

    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", *workload.split(), "--batch", "8",
                          "--streams", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["parity"]["status"] == "checked", line["parity"]
    assert line["parity"]["frames"] > 0 and line["parity"]["mismatches"] == 0, (line["parity"], out.stderr[-1000:])


def test_bench_gpus2_starts_its_own_ranks(gpu):
    """`python bench.py --gpus 2` (no torch.distributed.run around it) starts two ranks itself and
    reports n_gpus 2, both ranks' step times, the process group's world size, and the timed path's parity over both
    ranks' frames (each rank's own frames against its own oracle goldens).  gloo stands in for RCCL, so the two ranks
    can share the one GPU of the test box."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["ORBGPU_BENCH_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "8", "--steps", "2",
                          "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    assert len(line["per_rank_ms_per_step"]) == 2
    assert line["collective"] == {"backend": "gloo", "world_size": 2, "launcher": "bench.py --gpus"}
    p = line["parity"]
    assert p["status"] == "checked" and p["ranks"] == 2 and p["ranks_checked"] == 2, p
    assert p["frames"] == 2 * 9 and p["mismatches"] == 0, p
    assert line["value"] == pytest.approx(2 * 8 * 2 / (line["ms_per_step"] * 2e-3), rel=0.01)
