"""GPU parity tests of the matchers: SearchForInitialization and SearchByProjection (through the C
ABI) against the CPU oracle -- match indices, counts and updated state must be identical."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import synthetic

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pair(gpu, oracle, pid, rows, cols, nf, shift=(7, 3)):
    f1, f2 = synthetic.frame_pair(pid, rows, cols, shift)
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    k1, d1 = ex(f1)
    k2, d2 = ex(f2)
    return ex, k1, d1, k2, d2


@pytest.mark.parametrize("pid,rows,cols,nf", [(21, 1080, 1920, 2000), (22, 480, 640, 1000)])
def test_search_for_initialization_golden(gpu, oracle, pid, rows, cols, nf):
    ex, k1, d1, k2, d2 = _pair(gpu, oracle, pid, rows, cols, nf)
    sf = ex.GetScaleFactors()
    F1, F2 = gpu.Frame(k1, d1, cols, rows, sf), gpu.Frame(k2, d2, cols, rows, sf)
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
    m = gpu.ORBmatcher(0.9, True, context=ex)
    n, m12 = m.SearchForInitialization(F1, F2, prev, 100)
    g = {c["pair_id"]: c for c in json.load(open(os.path.join(ROOT, "tests/golden/match_golden.json")))["cases"]}
    assert n == g[pid]["nmatches"]
    assert hashlib.sha256(m12.astype(np.int32).tobytes()).hexdigest() == g[pid]["matches_sha256"]
    assert hashlib.sha256(prev.tobytes()).hexdigest() == g[pid]["prev_sha256"]


@pytest.mark.parametrize("seed", range(4))
def test_search_for_initialization_vs_oracle_variants(gpu, oracle, seed):
    rng = np.random.default_rng(seed)
    shift = (int(rng.integers(-20, 20)), int(rng.integers(-20, 20)))
    ex, k1, d1, k2, d2 = _pair(gpu, oracle, 50 + seed, 480, 640, 1000, shift)
    sf = ex.GetScaleFactors()
    # duplicate some F2 descriptors to force equal distances and steals
    d2 = d2.copy()
    d2[5:40:3] = d2[4:39:3]
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    win = int(rng.choice([10, 50, 100, 200]))
    ratio = float(rng.choice([0.6, 0.9]))
    ori = bool(seed % 2)
    G1, G2 = gpu.Frame(k1, d1, 640, 480, sf), gpu.Frame(k2, d2, 640, 480, sf)
    pg = np.ascontiguousarray(prev.copy())
    n, m12 = gpu.ORBmatcher(ratio, ori, context=ex).SearchForInitialization(G1, G2, pg, win)
    O1, O2 = oracle.OracleFrame(k1, d1, 640, 480, sf), oracle.OracleFrame(k2, d2, 640, 480, sf)
    no, mo, po = oracle.search_for_initialization(O1, O2, prev, ratio, ori, win)
    assert n == no
    assert np.array_equal(m12, mo)
    assert np.array_equal(pg, po)


def _mappoints(rng, k, d, M, levels_ok=True):
    src = rng.integers(0, len(k), M)
    desc = d[src].copy()
    flips = rng.random((M, 256)) < 0.05
    desc ^= np.packbits(flips, axis=1)
    return dict(track_in_view=np.ones(M, np.uint8), is_bad=np.zeros(M, np.uint8),
                level=k["octave"][src].astype(np.int32),
                view_cos=rng.uniform(0.9, 1.0, M).astype(np.float32),
                proj_x=(k["x"][src] + rng.normal(0, 1, M)).astype(np.float32),
                proj_y=(k["y"][src] + rng.normal(0, 1, M)).astype(np.float32),
                proj_xr=np.full(M, -1, np.float32), n_obs=np.full(M, 2, np.int32), desc=desc)


@pytest.mark.parametrize("th", [1.0, 3.0, 5.0])
def test_search_by_projection_vs_oracle(gpu, oracle, th):
    rng = np.random.default_rng(int(th * 10))
    img = synthetic.frame(60, 1080, 1920)
    ex = gpu.ORBextractor(4000, 1.2, 8, 20, 7)
    k, d = ex(img)
    mp = _mappoints(rng, k, d, 5000)
    mp["n_obs"][::7] = 0  # some points without observations: they do not block later points
    mp["track_in_view"][::11] = 0
    mp["is_bad"][::13] = 1
    sf = ex.GetScaleFactors()
    F = gpu.Frame(k, d, 1920, 1080, sf)
    n, own, obs = gpu.ORBmatcher(0.8, context=ex).SearchByProjection(F, mp, th)
    no, owo, obo = oracle.search_by_projection(oracle.OracleFrame(k, d, 1920, 1080, sf), mp, 0.8, th)
    assert n == no
    assert np.array_equal(own, owo)
    assert np.array_equal(obs, obo)


def _dense_frame(rng, Q=48, per=40, rows=1080, cols=1920):
    """Crafted keypoints: Q clusters of `per` level-0 keypoints within +-2 px, their descriptors 20-90 bits from the
    cluster's base descriptor, plus scattered background keypoints.  A map point projected on a cluster sees every
    keypoint of it inside its window with a distance <= TH_HIGH: far more than OG_PJ_K = 16 kept candidates."""
    from orbslam2_with_quadrics_amd import extractor as gx

    def at_distance(base, dist):
        bits = np.unpackbits(base)
        flip = rng.choice(256, dist, replace=False)
        bits[flip] ^= 1
        return np.packbits(bits)

    cx = rng.uniform(60, cols - 60, Q)
    cy = rng.uniform(60, rows - 60, Q)
    base = rng.integers(0, 256, (Q, 32), dtype=np.uint8)
    kl, dl = [], []
    for q in range(Q):
        for _ in range(per):
            kl.append((cx[q] + rng.uniform(-2, 2), cy[q] + rng.uniform(-2, 2)))
            dl.append(at_distance(base[q], int(rng.integers(20, 91))))
    nb = 600  # background
    for _ in range(nb):
        kl.append((rng.uniform(20, cols - 20), rng.uniform(20, rows - 20)))
        dl.append(rng.integers(0, 256, 32, dtype=np.uint8))
    k = np.zeros(len(kl), gx.KP_DTYPE)
    k["x"] = [p[0] for p in kl]
    k["y"] = [p[1] for p in kl]
    k["size"], k["octave"], k["class_id"], k["response"] = 31.0, 0, -1, 1.0
    k["angle"] = rng.uniform(0, 360, len(kl))
    return k, np.stack(dl), cx, cy, base


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_search_by_projection_dense_windows_and_forced_paths(gpu, oracle, flags):
    """the projection matcher's paths that ordinary frames never reach, pinned against the oracle.
    * Dense windows: every map point projected on a crafted cluster keeps ~40 candidates (> OG_PJ_K = 16), so the
      resolve re-enumerates those points in every round (and several points contest each cluster's keypoints,
      with and without observations, so the claim rounds iterate).
    * flags (orbgpu_debug_set_projection_paths): 1 = window enumeration from HBM geometry instead of the LDS copy,
      2 = claim rounds on the HBM slots instead of LDS-staged lists (the paths of frames too large for the LDS)."""
    from orbslam2_with_quadrics_amd import _lib

    rng = np.random.default_rng(55)
    rows, cols = 1080, 1920
    k, d, cx, cy, base = _dense_frame(rng)
    Q = len(cx)
    reps = 5
    M = Q * reps
    src = np.repeat(np.arange(Q), reps)
    desc = base[src] ^ np.packbits(rng.random((M, 256)) < 0.04, axis=1)
    mp = dict(track_in_view=np.ones(M, np.uint8), is_bad=np.zeros(M, np.uint8), level=np.zeros(M, np.int32),
              view_cos=rng.choice([0.95, 0.999], M).astype(np.float32),
              proj_x=(cx[src] + rng.normal(0, 0.3, M)).astype(np.float32),
              proj_y=(cy[src] + rng.normal(0, 0.3, M)).astype(np.float32),
              proj_xr=np.full(M, -1, np.float32), n_obs=np.where(rng.random(M) < 0.5, 0, 3).astype(np.int32),
              desc=desc)
    ex = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    sf = ex.GetScaleFactors()
    owner0 = np.full(len(k), -1, np.int32)
    obs0 = np.zeros(len(k), np.int32)
    owner0[::29] = M + 3  # claims made before the call
    obs0[::58] = 1
    _lib.check(ex.ctx, _lib.lib().orbgpu_debug_set_projection_paths(ex.ctx, flags), "debug paths")
    try:
        for th in (1.0, 3.0):
            F = gpu.Frame(k, d, cols, rows, sf)
            n, own, obs = gpu.ORBmatcher(0.8, context=ex).SearchByProjection(F, mp, th, owner=owner0.copy(),
                                                                             owner_obs=obs0.copy())
            no, owo, obo = oracle.search_by_projection(oracle.OracleFrame(k, d, cols, rows, sf), mp, 0.8, th,
                                                       owner0, obs0)
            # (few matches pass the ratio test: ~40 candidates per window at similar distances)
            assert n == no and n > 5, (flags, th, n, no)
            assert np.array_equal(own, owo), (flags, th)
            assert np.array_equal(obs, obo), (flags, th)
    finally:
        _lib.lib().orbgpu_debug_set_projection_paths(ex.ctx, 0)


def test_search_by_projection_stereo_and_preclaimed(gpu, oracle):
    rng = np.random.default_rng(3)
    img = synthetic.frame(61, 376, 1241)
    ex = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    k, d = ex(img)
    mp = _mappoints(rng, k, d, 1500)
    mp["proj_xr"] = (mp["proj_x"] - 30 + rng.normal(0, 2, len(mp["proj_x"]))).astype(np.float32)
    uright = np.where(rng.random(len(k)) < 0.5, k["x"] - 30, -1).astype(np.float32)
    owner0 = np.where(rng.random(len(k)) < 0.2, 7777, -1).astype(np.int32)
    obs0 = ((owner0 >= 0) & (rng.random(len(k)) < 0.5)).astype(np.int32)
    sf = ex.GetScaleFactors()
    F = gpu.Frame(k, d, 1241, 376, sf, uright=uright)
    n, own, obs = gpu.ORBmatcher(0.8, context=ex).SearchByProjection(F, mp, 3.0, owner0, obs0)
    no, owo, obo = oracle.search_by_projection(oracle.OracleFrame(k, d, 1241, 376, sf, uright=uright), mp, 0.8, 3.0,
                                               owner0, obs0)
    assert n == no
    assert np.array_equal(own, owo)
    assert np.array_equal(obs, obo)


def test_descriptor_distance(gpu, oracle):
    rng = np.random.default_rng(0)
    for _ in range(200):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        assert gpu.ORBmatcher.DescriptorDistance(a, b) == oracle.descriptor_distance(a, b)


@pytest.mark.parametrize("B", [5, 256])
def test_batch_search_for_initialization(gpu, oracle, B):
    """Device-resident batch: frame 0 of a reference context is F1 for every frame of a batch.  B = 256 is the
    bench's launch size (every kernel's grid at full width; frames 0, 1, 128 and 255 checked)."""
    import ctypes as C

    from orbslam2_with_quadrics_amd import _lib

    rows, cols = 480, 640
    scene = synthetic.make_scene(synthetic.SEED_BASE + 77, rows, cols)
    f1 = synthetic.render(scene, rows, cols, 0, 0, noise_seed=1)
    frames = np.stack([synthetic.render(scene, rows, cols, 3 * (b % 8), 2 * (b % 8), noise_seed=10 + b)
                       for b in range(B)])
    exr = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    exb = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    d1 = exr.device_alloc(f1.nbytes)
    db = exb.device_alloc(frames.nbytes)
    exr.h2d(d1, f1)
    exb.h2d(db, frames)
    exr.extract_batch_device(d1, 1, cols, rows, cols, f1.nbytes)
    exb.extract_batch_device(db, B, cols, rows, cols, rows * cols)
    k1, de1 = exr.batch_download(0)
    _, _, _, cap = exr.batch_outputs()
    prev = np.zeros((B, cap, 2), np.float32)
    prev[:, :len(k1), 0] = k1["x"]
    prev[:, :len(k1), 1] = k1["y"]
    d_prev = exb.device_alloc(prev.nbytes)
    d_m = exb.device_alloc(B * cap * 4)
    d_n = exb.device_alloc(B * 4)
    exb.h2d(d_prev, prev)
    g = _lib.GridGeom()
    _lib.lib().orbgpu_grid_geom_for_image(cols, rows, C.byref(g))
    rc = _lib.lib().orbgpu_search_for_initialization_batch(exr.ctx, 0, exb.ctx, g, 0.9, 1, 100,
                                                           C.c_void_p(d_prev), C.c_void_p(d_m), C.c_void_p(d_n))
    _lib.check(exb.ctx, rc, "batch")
    exb.synchronize()
    m_all = np.zeros((B, cap), np.int32)
    n_all = np.zeros(B, np.int32)
    p_all = np.zeros_like(prev)
    exb.d2h(m_all, d_m)
    exb.d2h(n_all, d_n)
    exb.d2h(p_all, d_prev)
    oe = oracle.OracleExtractor(1000)
    ko1, do1 = oe(f1)
    sf = exr.GetScaleFactors()
    O1 = oracle.OracleFrame(ko1, do1, cols, rows, sf)
    for b in (range(B) if B <= 8 else (0, 1, 128, B - 1)):
        k2, dd2 = oe(frames[b])
        O2 = oracle.OracleFrame(k2, dd2, cols, rows, sf)
        no, mo, po = oracle.search_for_initialization(O1, O2, np.stack([ko1["x"], ko1["y"]], 1), 0.9, True, 100)
        assert n_all[b] == no
        assert np.array_equal(m_all[b, :len(ko1)], mo)
        assert np.array_equal(p_all[b, :len(ko1)], po)
    for p in (d1, db):
        exr.device_free(p)
    for p in (d_prev, d_m, d_n):
        exb.device_free(p)


@pytest.mark.parametrize("ratio", [0.6, 0.75, 0.9, 1.0, 1.5])
def test_search_for_initialization_distance_bound(gpu, oracle, ratio):
    """Crafted candidates at Hamming distances around the pruning bound of og_init_keep_bound (d > 50 with
    50 < d * ratio): best 40-52, seconds 50-90, plus shared candidates that steal from each other."""
    rng = np.random.default_rng(int(ratio * 100))
    rows, cols, n1 = 480, 640, 300
    k1 = np.zeros(n1, gpu.KP_DTYPE)
    k1["x"] = rng.uniform(30, cols - 30, n1).astype(np.float32)
    k1["y"] = rng.uniform(30, rows - 30, n1).astype(np.float32)
    k1["angle"] = rng.uniform(0, 360, n1).astype(np.float32)
    k1["size"], k1["octave"], k1["class_id"] = 31.0, 0, -1
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)

    def at_distance(d, n):
        bits = np.unpackbits(d, bitorder="little")
        flip = rng.choice(256, n, replace=False)
        bits[flip] ^= 1
        return np.packbits(bits, bitorder="little")

    k2l, d2l = [], []
    for i in range(n1):
        for dist in (int(rng.integers(40, 53)), int(rng.integers(50, 91)), int(rng.integers(50, 91))):
            kp = np.zeros(1, gpu.KP_DTYPE)
            kp["x"] = k1["x"][i] + rng.uniform(-3, 3)
            kp["y"] = k1["y"][i] + rng.uniform(-3, 3)
            kp["angle"] = (k1["angle"][i] + rng.choice([0.0, 0.0, 0.0, 90.0])) % 360
            kp["size"], kp["octave"], kp["class_id"] = 31.0, 0, -1
            k2l.append(kp)
            d2l.append(at_distance(d1[i], dist))
    k2 = np.concatenate(k2l)
    d2 = np.stack(d2l)
    sf = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    prev = np.ascontiguousarray(np.stack([k1["x"], k1["y"]], 1).astype(np.float32))
    pg = prev.copy()
    n, m12 = gpu.ORBmatcher(ratio, True, context=ex).SearchForInitialization(
        gpu.Frame(k1, d1, cols, rows, sf), gpu.Frame(k2, d2, cols, rows, sf), pg, 12)
    no, mo, po = oracle.search_for_initialization(oracle.OracleFrame(k1, d1, cols, rows, sf),
                                                  oracle.OracleFrame(k2, d2, cols, rows, sf), prev, ratio, True, 12)
    assert n == no and n > 10
    assert np.array_equal(m12, mo)
    assert np.array_equal(pg, po)


def _mp_conflicts(rng, k, d, M):
    """Map points that fight over the same keypoints: each source keypoint is projected by several points with
    near-identical descriptors, mixed n_obs 0/2 (claims that do / do not block later points)."""
    src = np.repeat(rng.integers(0, len(k), M // 6), 6)[:M]
    mp = _mappoints(rng, k, d, len(src))
    mp["level"] = k["octave"][src].astype(np.int32)
    mp["proj_x"] = (k["x"][src] + rng.normal(0, 0.5, len(src))).astype(np.float32)
    mp["proj_y"] = (k["y"][src] + rng.normal(0, 0.5, len(src))).astype(np.float32)
    mp["desc"] = d[src] ^ np.packbits(rng.random((len(src), 256)) < 0.02, axis=1)
    mp["n_obs"] = np.where(rng.random(len(src)) < 0.4, 0, 2).astype(np.int32)
    return mp


@pytest.mark.parametrize("rows,cols,nf,M,conflicts", [(480, 640, 1000, 1500, False), (480, 640, 1000, 1800, True),
                                                      (1080, 1920, 4000, 5000, False)])
def test_search_by_projection_batch_vs_oracle(gpu, oracle, rows, cols, nf, M, conflicts):
    """orbgpu_search_by_projection_batch: B frames of a device batch, each against its own map-point snapshot
    (config 5 shape in the last case), with claims made before the call; per-frame owners and counts bit-exact."""
    import ctypes as C

    from orbslam2_with_quadrics_amd import _lib

    B = 3
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    imgs = np.stack([synthetic.frame(200 + b, rows, cols) for b in range(B)])
    dimg = ex.device_alloc(imgs.nbytes)
    bufs = [dimg]
    try:
        ex.h2d(dimg, imgs)
        ex.extract_batch_device(dimg, B, cols, rows, cols, rows * cols)
        _, _, _, cap = ex.batch_outputs()
        sf = ex.GetScaleFactors()
        rng = np.random.default_rng(M)
        frames, mps, owner0, obs0 = [], [], np.full((B, cap), -1, np.int32), np.zeros((B, cap), np.int32)
        for b in range(B):
            k, d = ex.batch_download(b)
            frames.append((k, d))
            mp = _mp_conflicts(rng, k, d, M) if conflicts else _mappoints(rng, k, d, M)
            mp["n_obs"][::7] = 0
            mp["track_in_view"][::11] = 0
            mp["is_bad"][::13] = 1
            mps.append(mp)
            owner0[b, :len(k)][::19] = M  # claims made before the call
            obs0[b, :len(k)][::38] = 1
        stride = M + 5
        dev = {}
        for key in ("track_in_view", "is_bad", "level", "view_cos", "proj_x", "proj_y", "proj_xr", "n_obs", "desc"):
            a0 = mps[0][key]
            arr = np.zeros((B, stride) + a0.shape[1:], a0.dtype)
            for b in range(B):
                arr[b, :M] = mps[b][key]
            p = ex.device_alloc(arr.nbytes)
            bufs.append(p)
            ex.h2d(p, arr)
            dev[key] = p
        d_own, d_obs, d_nm = (ex.device_alloc(B * cap * 4), ex.device_alloc(B * cap * 4), ex.device_alloc(B * 4))
        bufs += [d_own, d_obs, d_nm]
        ex.h2d(d_own, owner0)
        ex.h2d(d_obs, obs0)
        mv = _lib.MapPointsView(M, *[dev[k] for k in ("track_in_view", "is_bad", "level", "view_cos", "proj_x",
                                                        "proj_y", "proj_xr", "n_obs", "desc")])
        for th in (1.0, 3.0):
            ex.h2d(d_own, owner0)
            ex.h2d(d_obs, obs0)
            _lib.check(ex.ctx, _lib.lib().orbgpu_search_by_projection_batch(ex.ctx, C.byref(mv), stride, 0.8, th, None,
                                                                             C.c_void_p(d_own), C.c_void_p(d_obs),
                                                                             C.c_void_p(d_nm)), "sbp_batch")
            own = np.zeros((B, cap), np.int32)
            obs = np.zeros((B, cap), np.int32)
            nm = np.zeros(B, np.int32)
            ex.d2h(own, d_own)
            ex.d2h(obs, d_obs)
            ex.d2h(nm, d_nm)
            for b in range(B):
                k, d = frames[b]
                n = len(k)
                wn, wown, wobs = oracle.search_by_projection(oracle.OracleFrame(k, d, cols, rows, sf), mps[b], 0.8, th,
                                                             owner0[b, :n], obs0[b, :n])
                assert nm[b] == wn and wn > 50, (b, th)
                assert np.array_equal(own[b, :n], wown), (b, th)
                assert np.array_equal(obs[b, :n], wobs), (b, th)
    finally:
        for p in bufs:
            ex.device_free(p)


def test_golden_tracking_projection_and_stereo(gpu):
    """The GPU path against the committed oracle goldens (tests/golden/tracking_golden.json): config-5
    SearchByProjection through the host C ABI and through the batched device form, and KITTI-shape stereo."""
    import ctypes as C

    from orbslam2_with_quadrics_amd import _lib

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden

    g = json.load(open(os.path.join(ROOT, "tests/golden/tracking_golden.json")))
    for case in g["projection"]:
        rows, cols = case["rows"], case["cols"]
        ex = gpu.ORBextractor(case["nfeatures"], 1.2, 8, 20, 7)
        img = synthetic.frame(case["frame_id"], rows, cols)
        k, d = ex(img)
        mp = make_golden.config5_mappoints(k, d, case["mappoints"], case["mp_seed"])
        n, own, obs = gpu.ORBmatcher(0.8, context=ex).SearchByProjection(gpu.Frame(k, d, cols, rows,
                                                                                   ex.GetScaleFactors()),
                                                                         mp, case["th"])
        assert n == case["nmatches"]
        assert hashlib.sha256(own.astype(np.int32).tobytes()).hexdigest() == case["owner_sha256"]
        assert hashlib.sha256(obs.astype(np.int32).tobytes()).hexdigest() == case["owner_obs_sha256"]
        # batched device form, one frame
        d_img = ex.device_alloc(img.nbytes)
        bufs = [d_img]
        try:
            ex.h2d(d_img, img)
            ex.extract_batch_device(d_img, 1, cols, rows, cols, img.nbytes)
            _, _, _, cap = ex.batch_outputs()
            dev = {}
            for key in ("track_in_view", "is_bad", "level", "view_cos", "proj_x", "proj_y", "proj_xr", "n_obs", "desc"):
                a = np.ascontiguousarray(mp[key])
                dev[key] = ex.device_alloc(a.nbytes)
                bufs.append(dev[key])
                ex.h2d(dev[key], a)
            d_own, d_obs, d_nm = ex.device_alloc(cap * 4), ex.device_alloc(cap * 4), ex.device_alloc(4)
            bufs += [d_own, d_obs, d_nm]
            ex.h2d(d_own, np.full(cap, -1, np.int32))
            ex.h2d(d_obs, np.zeros(cap, np.int32))
            M = case["mappoints"]
            mv = _lib.MapPointsView(M, *[dev[kk] for kk in ("track_in_view", "is_bad", "level", "view_cos", "proj_x",
                                                              "proj_y", "proj_xr", "n_obs", "desc")])
            _lib.check(ex.ctx, _lib.lib().orbgpu_search_by_projection_batch(ex.ctx, C.byref(mv), M, 0.8, case["th"],
                                                                             None, C.c_void_p(d_own),
                                                                             C.c_void_p(d_obs), C.c_void_p(d_nm)),
                       "sbp_batch")
            bown = np.zeros(cap, np.int32)
            nm = np.zeros(1, np.int32)
            ex.d2h(bown, d_own)
            ex.d2h(nm, d_nm)
            assert nm[0] == case["nmatches"]
            assert hashlib.sha256(bown[:len(k)].tobytes()).hexdigest() == case["owner_sha256"]
        finally:
            for p in bufs:
                ex.device_free(p)
    for case in g["stereo"]:
        left, right, _ = synthetic.stereo_pair(case["pair_id"], case["rows"], case["cols"])
        exL, exR = gpu.ORBextractor(case["nfeatures"], 1.2, 8, 20, 7), gpu.ORBextractor(case["nfeatures"], 1.2, 8, 20, 7)
        exL(left)
        exR(right)
        ur, de, n = gpu.ComputeStereoMatches(exL, exR, case["mbf"], case["mb"])
        assert n == case["nmatches"]
        assert hashlib.sha256(ur.tobytes()).hexdigest() == case["uright_sha256"]
        assert hashlib.sha256(de.tobytes()).hexdigest() == case["depth_sha256"]
