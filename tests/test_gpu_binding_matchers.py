"""The matcher and stereo drop-in bindings EXECUTED (GPU): integration/ORBmatcher_perframe.cc and
integration/Frame_stereo.cc, compiled against the reference declarations restated in integration/refdecl (checked line
by line against the reference headers by tests/test_integration_compile.py) and linked with the extractor binding
integration/ORBextractor.cc (built against the reference's unchanged include/ORBextractor.h), the test cv shim
(tests/binding_run/cvmini.cc) and test-only definitions of the Frame / MapPoint / KeyFrame members they read
(tests/binding_run/refstubs.cc), into tests/binding_run/run_matchers.  Each case runs ORB-SLAM2's own call pattern:

* SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, 100) with ORBmatcher(0.9, true)
  (src/Tracking.cc:599-600), plus other ratios / windows / orientation settings;
* SearchByProjection(F, vpLocalMapPoints, th) with ORBmatcher(0.8), th 1 / 3 / 5 (src/Tracking.cc:1184-1191),
  with pre-claimed keypoints and a stereo frame;
* SearchByProjection(CurrentFrame, LastFrame, th, bMono) with ORBmatcher(0.9, true), th 7 / 14 mono and 15 / 30
  stereo (src/Tracking.cc:869-891);
* SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) with (10, 100) and (3, 64)
  (src/Tracking.cc:1433,1467, src/ORBmatcher.cc:1472-1599); the binding's PredictScale is the caller's;
* Frame::ComputeStereoMatches (src/Frame.cc:466-640) on the device pyramids of the two extractors.

Every output -- the extracted keypoints and descriptors, vnMatches12, the updated vbPrevMatched, the match counts,
F.mvpMapPoints (as map-point indices) and mvuRight / mvDepth (as bit patterns) -- is compared with the CPU oracle.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import KP_DTYPE, synthetic

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(ROOT, "tests", "binding_run", "run_matchers")


def _write_blob(path, arrays):
    with open(path, "wb") as f:
        for k, v in arrays.items():
            b = np.ascontiguousarray(v).tobytes()
            f.write(struct.pack("<I", len(k)) + k.encode() + struct.pack("<Q", len(b)) + b)


def _read_blob(path):
    buf = open(path, "rb").read()
    o, out = 0, {}
    while o < len(buf):
        (nl,) = struct.unpack_from("<I", buf, o)
        name = buf[o + 4:o + 4 + nl].decode()
        (nb,) = struct.unpack_from("<Q", buf, o + 4 + nl)
        o += 12 + nl
        out[name] = buf[o:o + nb]
        o += nb
    return out


def _run(tmp_path, mode, arrays):
    if not os.path.exists(RUNNER):
        pytest.fail("tests/binding_run/run_matchers was not built (build it where /root/reference exists: "
                    "python -c 'import __graft_entry__ as g; g.build()')")
    fin, fout = tmp_path / f"{mode}.in", tmp_path / f"{mode}.out"
    _write_blob(fin, arrays)
    r = subprocess.run([RUNNER, mode, str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return _read_blob(fout)


def _kps(out, tag):
    return np.frombuffer(out[tag + "_kps"], KP_DTYPE), np.frombuffer(out[tag + "_desc"], np.uint8).reshape(-1, 32)


def _same_extraction(out, tag, ko, do):
    k, d = _kps(out, tag)
    assert len(k) == len(ko) and k.tobytes() == ko.tobytes(), tag
    assert np.array_equal(d, do), tag


def _i32(out, k):
    return int(np.frombuffer(out[k], np.int32)[0])


def _pose(cam):
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = cam["Rcw"]
    T[:3, 3] = cam["tcw"]
    return T


def _poses(seed, cols, rows, tz=0.0):
    rng = np.random.default_rng(seed)
    R0 = synthetic.rotation(*rng.uniform(-0.05, 0.05, 3))
    t0 = rng.uniform(-0.3, 0.3, 3)
    dR = synthetic.rotation(*rng.uniform(-0.01, 0.01, 3))
    last = synthetic.camera(cols, rows, R0, t0)
    cur = synthetic.camera(cols, rows, dR @ R0, dR @ t0 + np.array([-0.02, -0.01, tz]))
    return last, cur


@pytest.mark.parametrize("pid,shape,nf", [(21, (1080, 1920), 2000), (23, (480, 640), 1000)])
def test_search_for_initialization_binding(gpu, oracle, tmp_path, pid, shape, nf):
    rows, cols = shape
    f1, f2 = synthetic.frame_pair(pid, rows, cols, (7, 3))
    cases = [(0.9, 100, 1), (0.6, 50, 0), (0.9, 10, 1)]  # the first is Tracking's call
    out = _run(tmp_path, "init", dict(params=np.array([cols, rows, nf], np.int32), img1=f1, img2=f2,
                                      ratio=np.array([c[0] for c in cases], np.float32),
                                      window=np.array([c[1] for c in cases], np.int32),
                                      check_ori=np.array([c[2] for c in cases], np.int32)))
    oe = oracle.OracleExtractor(nf)
    k1, d1 = oe(f1)
    k2, d2 = oe(f2)
    _same_extraction(out, "f1", k1, d1)
    _same_extraction(out, "f2", k2, d2)
    sf = oe.tables()["scale"]
    O1, O2 = oracle.OracleFrame(k1, d1, cols, rows, sf), oracle.OracleFrame(k2, d2, cols, rows, sf)
    prev0 = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    for c, (ratio, win, ori) in enumerate(cases):
        no, mo, po = oracle.search_for_initialization(O1, O2, prev0, ratio, bool(ori), win)
        assert _i32(out, f"n{c}") == no and no > 20
        assert np.array_equal(np.frombuffer(out[f"m12_{c}"], np.int32), mo)
        assert np.array_equal(np.frombuffer(out[f"prev_{c}"], np.float32).reshape(-1, 2), po)


@pytest.mark.parametrize("stereo", [False, True])
def test_search_by_projection_local_map_binding(gpu, oracle, tmp_path, stereo):
    rows, cols, nf, M = (376, 1241, 2000, 1500) if stereo else (1080, 1920, 4000, 5000)
    rng = np.random.default_rng(7 + stereo)
    img = synthetic.frame(60 + stereo, rows, cols)
    oe = oracle.OracleExtractor(nf)
    k, d = oe(img)
    src = rng.integers(0, len(k), M)
    desc = d[src] ^ np.packbits(rng.random((M, 256)) < 0.05, axis=1)
    mp = dict(track_in_view=(rng.random(M) >= 0.09).astype(np.uint8), is_bad=(rng.random(M) < 0.07).astype(np.uint8),
              level=k["octave"][src].astype(np.int32), view_cos=rng.uniform(0.9, 1.0, M).astype(np.float32),
              proj_x=(k["x"][src] + rng.normal(0, 1, M)).astype(np.float32),
              proj_y=(k["y"][src] + rng.normal(0, 1, M)).astype(np.float32),
              proj_xr=np.full(M, -1, np.float32), n_obs=np.where(rng.random(M) < 0.15, 0, 2).astype(np.int32),
              desc=np.ascontiguousarray(desc))
    uright = None
    if stereo:
        mp["proj_xr"] = (mp["proj_x"] - 30 + rng.normal(0, 2, M)).astype(np.float32)
        uright = np.where(rng.random(len(k)) < 0.5, k["x"] - 30, -1).astype(np.float32)
    claim = np.where(rng.random(len(k)) < 0.15, (rng.random(len(k)) < 0.5).astype(np.int32), -1).astype(np.int32)
    ths = [1.0, 3.0, 5.0]
    arrays = dict(params=np.array([cols, rows, nf], np.int32), img=img, claim=claim, th=np.array(ths, np.float32), **mp)
    if stereo:
        arrays["uright"] = uright
    out = _run(tmp_path, "proj", arrays)
    _same_extraction(out, "f", k, d)
    Fo = oracle.OracleFrame(k, d, cols, rows, oe.tables()["scale"], uright=uright)
    owner0 = np.where(claim >= 0, M, -1).astype(np.int32)
    obs0 = (claim == 1).astype(np.int32)
    for c, th in enumerate(ths):
        no, owo, _ = oracle.search_by_projection(Fo, mp, 0.8, th, owner0, obs0)
        assert _i32(out, f"n{c}") == no and no > 50
        assert np.array_equal(np.frombuffer(out[f"owner_{c}"], np.int32), owo), th


@pytest.mark.parametrize("seed,mono,tz", [(0, True, 0.0), (2, False, 0.0), (3, False, 0.8)])
def test_search_by_projection_last_frame_binding(gpu, oracle, tmp_path, seed, mono, tz):
    rows, cols, nf = 480, 640, 1000
    f1, f2 = synthetic.frame_pair(80 + seed, rows, cols, (5, 2))
    oe = oracle.OracleExtractor(nf)
    k1, d1 = oe(f1)
    k2, d2 = oe(f2)
    last, cur = _poses(seed, cols, rows, tz)
    lf = synthetic.last_frame_points(seed, k1, d1, last)
    rng = np.random.default_rng(seed)
    uright = None if mono else np.where(rng.random(len(k2)) < 0.5, k2["x"] - rng.uniform(1, 40, len(k2)),
                                        -1).astype(np.float32)
    claim = np.full(len(k2), -1, np.int32)
    claim[::17] = 0
    claim[::34] = 1
    ths = [7.0, 14.0] if mono else [15.0, 30.0]  # src/Tracking.cc:876-891
    arrays = dict(params=np.array([cols, rows, nf, int(mono), 1], np.int32), img_last=f1, img_cur=f2,
                  K=np.array([cur["fx"], cur["fy"], cur["cx"], cur["cy"]], np.float32),
                  Tcw_last=_pose(last), Tcw_cur=_pose(cur), mbf_mb=np.array([cur["mbf"], cur["mb"]], np.float32),
                  has_mp=lf["has_mp"], outlier=lf["outlier"], pos=lf["pos"], n_obs=lf["n_obs"], desc=lf["desc"],
                  claim=claim, th=np.array(ths, np.float32))
    if uright is not None:
        arrays["uright"] = uright
    out = _run(tmp_path, "last", arrays)
    _same_extraction(out, "last", k1, d1)
    _same_extraction(out, "cur", k2, d2)
    Fo = oracle.OracleFrame(k2, d2, cols, rows, oe.tables()["scale"], uright)
    owner0 = np.where(claim >= 0, len(k1), -1).astype(np.int32)
    obs0 = (claim == 1).astype(np.int32)
    for c, th in enumerate(ths):
        wn, wown, _ = oracle.search_by_projection_last(Fo, cur, last, lf, th, mono, True, owner0, obs0)
        assert _i32(out, f"n{c}") == wn and wn > 20
        assert np.array_equal(np.frombuffer(out[f"owner_{c}"], np.int32), wown), th


@pytest.mark.parametrize("seed,shape,nf", [(0, (480, 640), 1000), (2, (1080, 1920), 2000)])
def test_search_by_projection_keyframe_binding(gpu, oracle, tmp_path, seed, shape, nf):
    rows, cols = shape
    f1, f2 = synthetic.frame_pair(130 + seed, rows, cols, (4, -2))
    oe = oracle.OracleExtractor(nf)
    k1, d1 = oe(f1)
    k2, d2 = oe(f2)
    kfcam, cur = _poses(seed, cols, rows)
    kf = synthetic.keyframe_points(seed, k1, d1, kfcam)
    claim = np.full(len(k2), -1, np.int32)
    claim[::13] = 1
    cases = [(10.0, 100), (3.0, 64)]  # src/Tracking.cc:1433, :1467
    out = _run(tmp_path, "kf", dict(params=np.array([cols, rows, nf, 1], np.int32), img_kf=f1, img_cur=f2,
                                    K=np.array([cur["fx"], cur["fy"], cur["cx"], cur["cy"]], np.float32),
                                    Tcw_cur=_pose(cur), mbf_mb=np.array([cur["mbf"], cur["mb"]], np.float32),
                                    valid=kf["valid"], pos=kf["pos"], max_dist=kf["max_dist"], min_dist=kf["min_dist"],
                                    desc=kf["desc"], claim=claim, th=np.array([c[0] for c in cases], np.float32),
                                    orbdist=np.array([c[1] for c in cases], np.int32)))
    _same_extraction(out, "kf", k1, d1)
    _same_extraction(out, "cur", k2, d2)
    Fo = oracle.OracleFrame(k2, d2, cols, rows, oe.tables()["scale"])
    owner0 = np.where(claim >= 0, len(k1), -1).astype(np.int32)
    for c, (th, orbdist) in enumerate(cases):
        wn, wown = oracle.search_by_projection_kf(Fo, cur, kf, th, orbdist, True, owner0)
        assert _i32(out, f"n{c}") == wn and wn > 10
        assert np.array_equal(np.frombuffer(out[f"owner_{c}"], np.int32), wown), (th, orbdist)


@pytest.mark.parametrize("pid,shape,nf", [(0, (376, 1241), 2000), (3, (480, 640), 1000)])
def test_compute_stereo_matches_binding(gpu, oracle, tmp_path, pid, shape, nf):
    rows, cols = shape
    left, right, _ = synthetic.stereo_pair(pid, rows, cols)
    mbf, fx = 386.1448, 718.856  # Examples/Stereo/KITTI00-02.yaml:8,25
    mb = np.float32(np.float32(mbf) / np.float32(fx))
    out = _run(tmp_path, "stereo", dict(params=np.array([cols, rows, nf], np.int32), left=left, right=right,
                                        mbf_mb=np.array([mbf, mb], np.float32)))
    oL, oR = oracle.OracleExtractor(nf), oracle.OracleExtractor(nf)
    kl, dl = oL(left)
    kr, dr = oR(right)
    _same_extraction(out, "left", kl, dl)
    _same_extraction(out, "right", kr, dr)
    nso, uro, deo = oracle.stereo_matches(oL, oR, kl, dl, kr, dr, np.float32(mbf), mb)
    ur = np.frombuffer(out["uright"], np.float32)
    de = np.frombuffer(out["depth"], np.float32)
    assert len(ur) == len(kl) and nso > 100
    assert ur.tobytes() == uro.tobytes() and de.tobytes() == deo.tobytes()
