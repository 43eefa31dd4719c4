"""CPU tests: pin the oracle's pieces against everything that can be checked without the reference
binary (which needs OpenCV/Eigen/Pangolin and cannot be built here -- DESIGN.md §4)."""
import hashlib
import json
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import refpy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_scale_tables_match_survey(oracle):
    """src/ORBextractor.cc:410-470 -- per-level budgets quoted in SURVEY.md §8 and umax."""
    t = oracle.OracleExtractor(1000).tables()
    assert t["features_per_level"].tolist() == [217, 181, 151, 126, 105, 87, 73, 60]
    t2 = oracle.OracleExtractor(2000).tables()
    assert t2["features_per_level"].tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    t4 = oracle.OracleExtractor(4000).tables()
    assert t4["features_per_level"][0] == 869
    assert t["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    # float(float*double) chain of src/ORBextractor.cc:421 (double member scaleFactor)
    sf = [np.float32(1.0)]
    for _ in range(7):
        sf.append(np.float32(np.float64(sf[-1]) * np.float64(np.float32(1.2))))
    assert np.array_equal(t["scale"], np.array(sf, np.float32))


def test_gaussian_kernel_table():
    """cvRound(256 * getGaussianKernel(7, 2)) -> the 257-sum integer kernel the oracle/GPU use."""
    x = np.arange(7) - 3.0
    t = np.exp(-0.125 * x * x)
    k = (t / t.sum()).astype(np.float32)
    ik = [int(np.rint(np.float64(v) * 256)) for v in k]
    assert ik == [18, 34, 49, 55, 49, 34, 18]


def test_fast_score_matches_definition(oracle):
    """cornerScore<16> == largest threshold for which the segment test still passes."""
    rng = np.random.default_rng(1)
    checked = corners = 0
    for trial in range(1500):
        patch = rng.integers(0, 256, size=(7, 7)).astype(np.uint8)
        if trial % 3 == 0:  # force arcs so that corners are common
            s = rng.integers(0, 16)
            ln = rng.integers(8, 13)
            val = rng.integers(0, 256)
            for k in range(ln):
                dx, dy = refpy.CIRCLE[(s + k) % 16]
                patch[3 + dy, 3 + dx] = val
        img = np.zeros((13, 13), np.uint8)
        img[3:10, 3:10] = patch
        got = oracle.fast_score(img, 6, 6)
        want = refpy.fast_score_definition(patch)
        assert got == want, (patch, got, want)
        checked += 1
        corners += want >= 0
    assert corners > 300


def test_sincosf_restatement_exhaustive_sample(tmp_path):
    """oracle glibc-sincosf restatement vs this host's libm (every 61st float in [0, 8))."""
    exe = tmp_path / "verify_sincosf"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fopenmp",
                           os.path.join(ROOT, "tools", "verify_sincosf.c"), "-o", str(exe), "-lm"])
    out = subprocess.check_output([str(exe), "61"]).decode()
    assert out.strip().endswith("mismatches 0"), out


def test_logf_restatement_exhaustive_sample(tmp_path):
    """oracle glibc-logf restatement (PredictScale) vs this host's libm (every 7th positive float)."""
    exe = tmp_path / "verify_logf"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-fopenmp",
                           os.path.join(ROOT, "tools", "verify_logf.c"), "-o", str(exe), "-lm"])
    out = subprocess.check_output([str(exe), "7"]).decode()
    assert out.strip().endswith("mismatches 0"), out


def test_projection_contraction_probe(tmp_path):
    """GCC -O3 -march=native contracts the isInFrustum / SearchByProjection projections into the FMA
    forms the oracle pins (u = fma(fx*X, invz, cx), ur = fma(-mbf, invz, u))."""
    exe = tmp_path / "probe_proj"
    subprocess.check_call(["g++", "-O3", "-march=native", os.path.join(ROOT, "tools", "probe_contraction_proj.cc"),
                           "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().split()
    vals = dict(zip(out[2::2], out[3::2]))
    if "fma" not in open("/proc/cpuinfo").read():
        pytest.skip("host without FMA: the reference build would not contract")
    assert vals["u!=fma(fx*X,invz,cx)"] == "0" and vals["ur!=fma(-mbf,invz,u)"] == "0", out


def test_sincos_golden_vectors(oracle):
    """Golden (angle -> sin, cos) pairs produced by libm sincosf (tests/golden/make_golden.py)."""
    g = json.load(open(os.path.join(GOLDEN, "sincosf.json")))
    for a, s, c in g["vectors"]:
        gs, gc = oracle.sincos(np.float32(a))
        assert np.float32(gs) == np.float32(s) and np.float32(gc) == np.float32(c)


def test_fastatan2_accuracy_and_quadrants(oracle):
    assert oracle.fastatan2(0.0, 0.0) == 0.0
    assert oracle.fastatan2(1.0, 0.0) == 90.0
    assert oracle.fastatan2(0.0, -1.0) == 180.0
    assert oracle.fastatan2(-1.0, 0.0) == 270.0
    rng = np.random.default_rng(5)
    for _ in range(2000):
        y, x = (float(v) for v in rng.integers(-200000, 200000, 2))
        a = oracle.fastatan2(y, x)
        ref = math.degrees(math.atan2(y, x)) % 360.0
        d = abs(a - ref)
        assert min(d, 360 - d) < 0.02


@pytest.mark.skipif(not os.path.exists("/root/reference/src/ORBextractor.cc"), reason="reference absent")
def test_pattern_matches_reference_source():
    """The committed rBRIEF pattern equals bit_pattern_31_ (src/ORBextractor.cc:150-408)."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_orb_pattern

    ref = gen_orb_pattern.parse()
    for inc in ("oracle/orb_pattern.inc", "orbslam2_with_quadrics_amd/csrc/orb_pattern.inc"):
        txt = open(os.path.join(ROOT, inc)).read()
        body = txt[txt.index("{") + 1: txt.index("};")]
        vals = [int(v) for v in re.findall(r"-?\d+", body)]
        assert vals == ref, inc


def test_pattern_copies_identical():
    a = open(os.path.join(ROOT, "oracle/orb_pattern.inc")).read()
    b = open(os.path.join(ROOT, "orbslam2_with_quadrics_amd/csrc/orb_pattern.inc")).read()
    assert a == b


def _have_fma():
    try:
        return " fma " in open("/proc/cpuinfo").read().replace("\n", " ")
    except OSError:
        return False


@pytest.mark.skipif(not _have_fma(), reason="host CPU has no FMA: the reference build would not contract")
def test_descriptor_rotation_contraction_probe(tmp_path):
    """GCC -O3 -march=native fuses the rBRIEF sample rotation (src/ORBextractor.cc:118-120) as
    fma(x,b,y*a) / fma(x,a,-(y*b)); the oracle and the GPU write exactly those forms."""
    src = tmp_path / "probe.cc"
    src.write_text(open(os.path.join(ROOT, "tools", "probe_contraction.cc")).read())
    exe = tmp_path / "probe"
    subprocess.check_call(["g++", "-O3", "-march=native", "-std=c++11", str(src), "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode()
    assert "fused-first-product mismatches 0" in out, out


def test_oracle_golden_extraction(oracle):
    """Regression pin of the oracle on committed golden fixtures (hash of keypoints + descriptors)."""
    from orbslam2_with_quadrics_amd import synthetic

    g = json.load(open(os.path.join(GOLDEN, "extract_golden.json")))
    for case in g["cases"]:
        img = synthetic.frame(case["frame_id"], case["rows"], case["cols"])
        assert hashlib.sha256(img.tobytes()).hexdigest() == case["image_sha256"]
        k, d = oracle.OracleExtractor(case["nfeatures"], semantics=case.get("semantics", 0))(img)
        assert len(k) == case["n"]
        assert hashlib.sha256(k.tobytes()).hexdigest() == case["kps_sha256"]
        assert hashlib.sha256(d.tobytes()).hexdigest() == case["desc_sha256"]
        head = np.array(case["head"], np.float64)
        assert np.array_equal(np.stack([k["x"], k["y"], k["angle"], k["response"]], 1)[:len(head)]
                              .astype(np.float64), head)


def test_oracle_golden_tracking_and_stereo(oracle):
    """Regression pin of the oracle's SearchByProjection (config 5: 1080p, 4000 features, 5000 map points) and
    ComputeStereoMatches (KITTI shape) on the committed tracking_golden.json."""
    from orbslam2_with_quadrics_amd import synthetic

    sys.path.insert(0, GOLDEN)
    import make_golden

    g = json.load(open(os.path.join(GOLDEN, "tracking_golden.json")))
    for case in g["projection"]:
        img = synthetic.frame(case["frame_id"], case["rows"], case["cols"])
        ex = oracle.OracleExtractor(case["nfeatures"])
        k, d = ex(img)
        mp = make_golden.config5_mappoints(k, d, case["mappoints"], case["mp_seed"])
        n, own, obs = oracle.search_by_projection(oracle.OracleFrame(k, d, case["cols"], case["rows"],
                                                                     ex.tables()["scale"]), mp, 0.8, case["th"])
        assert n == case["nmatches"]
        assert hashlib.sha256(own.astype(np.int32).tobytes()).hexdigest() == case["owner_sha256"]
        assert hashlib.sha256(obs.astype(np.int32).tobytes()).hexdigest() == case["owner_obs_sha256"]
    for case in g["stereo"]:
        left, right, _ = synthetic.stereo_pair(case["pair_id"], case["rows"], case["cols"])
        exL, exR = oracle.OracleExtractor(case["nfeatures"]), oracle.OracleExtractor(case["nfeatures"])
        kl, dl = exL(left)
        kr, dr = exR(right)
        n, ur, de = oracle.stereo_matches(exL, exR, kl, dl, kr, dr, case["mbf"], case["mb"])
        assert n == case["nmatches"]
        assert hashlib.sha256(ur.tobytes()).hexdigest() == case["uright_sha256"]
        assert hashlib.sha256(de.tobytes()).hexdigest() == case["depth_sha256"]


# ---------------------------------------------------------------------------------------------------------
# OpenCV / compiler semantics variants (ORBGPU_SEM_*): each oracle form against an independent
# numpy restatement of the OpenCV code path it stands for
# ---------------------------------------------------------------------------------------------------------
SEM_BLUR_SSE2_257, SEM_BLUR_SCALAR_257, SEM_BLUR_BITEXACT_256, SEM_BLUR_BITEXACT_ED = (v << 2 for v in range(4))


def _resize_tables(n_src, n_dst):
    """resizeGeneric_ coefficient tables of one axis (float32 fx, cvFloor, clamps, cvRound(x * 2048))."""
    scale = 1.0 / (n_dst / n_src)
    ofs, a0, a1, vmax = [], [], [], n_dst
    for d in range(n_dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0), 0
        if s + 1 >= n_src:
            vmax = min(vmax, d)
            if s >= n_src - 1:
                f, s = np.float32(0), n_src - 1
        ofs.append(s)
        a0.append(int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048))))
        a1.append(int(np.rint(f * np.float32(2048))))
    return np.array(ofs), np.array(a0), np.array(a1), vmax


def _sat16(v):
    return np.clip(v, -32768, 32767)


def _resize_sse2(src, dw, dh):
    """cv::resize INTER_LINEAR 8U as OpenCV 3.x runs it on x86-64: HResizeLinear (exact int), then
    VResizeLinearVec_32s8u's instruction sequence srai(4) / packs_epi32 / mulhi_epi16 / adds_epi16 /
    adds(2) / srai(2) / packus_epi16, emulated lane by lane."""
    sh, sw = src.shape
    xo, xa0, xa1, xmax = _resize_tables(sw, dw)
    yo, yb0, yb1, _ = _resize_tables(sh, dh)
    S = src.astype(np.int64)
    nx = np.minimum(xo + 1, sw - 1)
    D = np.where(np.arange(dw) < xmax, S[:, xo] * xa0 + S[:, nx] * xa1, S[:, xo] * 2048)
    out = np.zeros((dh, dw), np.uint8)
    for y in range(dh):
        r0 = min(max(yo[y], 0), sh - 1)
        r1 = min(max(yo[y] + 1, 0), sh - 1)
        x0, x1 = _sat16(D[r0] >> 4), _sat16(D[r1] >> 4)
        m = _sat16(((x0 * yb0[y]) >> 16) + ((x1 * yb1[y]) >> 16))
        out[y] = np.clip(_sat16(m + 2) >> 2, 0, 255)
    return out


def test_resize_opencv_8u_form_vs_sse2_sequence(oracle):
    """Default resize semantics == OpenCV's SSE2 VResizeLinearVec_32s8u body over the whole row (its 8U
    VResizeLinear specialisation makes the scalar tail compute the same form); the FIXEDPT variant is the
    generic (b0*D0 + b1*D1 + 2^21) >> 22 and does differ from it."""
    from orbslam2_with_quadrics_amd import synthetic

    rng = np.random.default_rng(3)
    differs = 0
    for (h, w) in [(480, 640), (400, 533), (376, 1241), (1080, 1920), (97, 61)]:
        src = synthetic.frame(int(rng.integers(1000)), h, w) if h > 100 else rng.integers(0, 256, (h, w), np.uint8)
        dw, dh = int(np.rint(np.float32(w) / np.float32(1.2))), int(np.rint(np.float32(h) / np.float32(1.2)))
        got = oracle.resize_linear(src, dw, dh, 0)
        assert np.array_equal(got, _resize_sse2(src, dw, dh)), (h, w)
        differs += int((oracle.resize_linear(src, dw, dh, 0x01) != got).sum())
    assert differs > 0


def _gauss_kernels():
    """The integer 7x7 sigma-2 kernels of the three OpenCV generations, from the double-precision Gaussian."""
    x = np.arange(7) - 3.0
    g = np.exp(-0.125 * x * x)
    g = g / g.sum()
    legacy = [int(np.rint(np.float32(v) * 256)) for v in g.astype(np.float32)]   # cvRound(256 * float kernel)
    sides = [int(np.rint(v * 256)) for v in g[:3]]
    bitexact = sides + [256 - 2 * sum(sides)] + sides[::-1]                       # centre = 1 - sum(sides)
    ed, err = [], 0.0                                                            # error-diffused rounding
    for v in g[:3]:
        adj = v * 256 + err
        q = int(np.rint(adj))
        err = adj - q
        ed.append(q)
    ed = ed + [256 - 2 * sum(ed)] + ed[::-1]
    return legacy, bitexact, ed


def test_gaussian_kernel_tables_all_variants():
    legacy, bitexact, ed = _gauss_kernels()
    assert legacy == [18, 34, 49, 55, 49, 34, 18]
    assert bitexact == [18, 34, 49, 54, 49, 34, 18]
    assert ed == [18, 34, 48, 56, 48, 34, 18]


def _reflect101(i, n):
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)


def _blur_rows(img, k):
    h, w = img.shape
    I = img.astype(np.int64)
    xs = np.arange(w)
    return sum(k[t] * I[:, _reflect101(xs + t - 3, w)] for t in range(7))


def _blur_sse2(img):
    """OpenCV 3.0-3.4.1 GaussianBlur on x86-64 (no IPP): exact integer row sums (SymmRowSmallVec_8u32s), then
    SymmColumnVec_32s8u in float32 -- centre * f0 + (up_k + down_k) * f_k, f = k / 65536 -- rounded by cvtps2dq
    (half-to-even) for x < 4 * floor(w / 4); SymmColumnFilter's scalar tail (S + 2^15) >> 16 after that."""
    k = [18, 34, 49, 55, 49, 34, 18]
    h, w = img.shape
    R = _blur_rows(img, k)
    ys = np.arange(h)
    f = [np.float32(k[3 + t] / 65536.0) for t in range(4)]
    s = R[_reflect101(ys, h)].astype(np.float32) * f[0]
    for t in range(1, 4):
        pair = (R[_reflect101(ys - t, h)] + R[_reflect101(ys + t, h)]).astype(np.float32)
        s = (s + pair * f[t]).astype(np.float32)
    vec = np.clip(np.rint(s), 0, 255)
    S = sum(k[t] * R[_reflect101(ys + t - 3, h)] for t in range(7))
    tail = np.clip((S + (1 << 15)) >> 16, 0, 255)
    xs = np.arange(w)[None, :]
    return np.where(xs < (w & ~3), vec, tail).astype(np.uint8)


def _blur_fixed(img, k):
    h, w = img.shape
    R = _blur_rows(img, k)
    S = sum(k[t] * R[_reflect101(np.arange(h) + t - 3, h)] for t in range(7))
    return np.clip((S + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


def test_gaussian_variants_vs_restatements(oracle):
    """Each GaussianBlur variant of the oracle against an independent restatement of its OpenCV code path;
    binarised images make the half-to-even ties frequent, so the SSE2 and scalar variants do differ."""
    from orbslam2_with_quadrics_amd import synthetic

    legacy, bitexact, ed = _gauss_kernels()
    ties = 0
    for fid, (h, w) in enumerate([(480, 640), (313, 1034), (61, 43), (37, 41)]):
        img = synthetic.frame(fid + 50, h, w) if h > 100 else np.random.default_rng(fid).integers(0, 256, (h, w))
        img = (np.asarray(img, np.uint8) & 0x80) | 0x10 if fid % 2 == 0 else np.asarray(img, np.uint8)
        sse2 = oracle.gaussian7(img, SEM_BLUR_SSE2_257)
        assert np.array_equal(sse2, _blur_sse2(img)), (h, w)
        scalar = oracle.gaussian7(img, SEM_BLUR_SCALAR_257)
        assert np.array_equal(scalar, _blur_fixed(img, legacy))
        assert np.array_equal(oracle.gaussian7(img, SEM_BLUR_BITEXACT_256), _blur_fixed(img, bitexact))
        assert np.array_equal(oracle.gaussian7(img, SEM_BLUR_BITEXACT_ED), _blur_fixed(img, ed))
        ties += int((sse2 != scalar).sum())
    assert ties > 0


def test_semantics_constants_agree():
    """include/orbgpu.h ORBGPU_SEM_* and the oracle's OO_SEM_* use the same bits."""
    hdr = open(os.path.join(ROOT, "include", "orbgpu.h")).read()
    ora = open(os.path.join(ROOT, "oracle", "orb_oracle.h")).read()

    def val(txt, name):
        return int(re.search(r"#define " + name + r"\s+(0x[0-9a-fA-F]+|\d+)", txt).group(1), 0)

    assert val(hdr, "ORBGPU_SEM_RESIZE_FIXEDPT") == val(ora, "OO_SEM_RESIZE_FIXEDPT") == 0x01
    assert val(hdr, "ORBGPU_SEM_BLUR_SHIFT") == val(ora, "OO_SEM_BLUR_SHIFT") == 2
    assert val(hdr, "ORBGPU_SEM_BRIEF_NOFMA") == val(ora, "OO_SEM_BRIEF_NOFMA") == 0x20
    from orbslam2_with_quadrics_amd import _lib

    assert (_lib.SEM_RESIZE_FIXEDPT, _lib.SEM_BLUR_SHIFT, _lib.SEM_BRIEF_NOFMA) == (0x01, 2, 0x20)


def test_rbrief_fma_probe_golden(oracle):
    """tests/golden/semantics_probe.json (tools/find_fma_probe.py): an image on which the FMA and the non-FMA
    rBRIEF rotation give different descriptors; the oracle reproduces both committed hashes."""
    sys.path.insert(0, GOLDEN)
    import make_golden

    g = json.load(open(os.path.join(GOLDEN, "semantics_probe.json")))
    img = make_golden.fma_probe_image(g["seed"], g["mods"])
    ka, da = oracle.OracleExtractor(g["nfeatures"])(img)
    kb, db = oracle.OracleExtractor(g["nfeatures"], semantics=0x20)(img)
    assert hashlib.sha256(ka.tobytes()).hexdigest() == hashlib.sha256(kb.tobytes()).hexdigest() == g["kps_sha256"]
    assert hashlib.sha256(da.tobytes()).hexdigest() == g["desc_fma_sha256"]
    assert hashlib.sha256(db.tobytes()).hexdigest() == g["desc_nofma_sha256"]
    assert int((da != db).any(1).sum()) == g["descriptors_differing"] > 0


def test_rbrief_nofma_form_vs_restatement(oracle):
    """The non-FMA rotation recomputed in numpy float32 (two rounded products) from the oracle's own angle and
    blurred level reproduces the oracle's NOFMA descriptors on the probe image; the FMA form with refpy's exact
    fmaf reproduces the default ones."""
    sys.path.insert(0, GOLDEN)
    import make_golden

    g = json.load(open(os.path.join(GOLDEN, "semantics_probe.json")))
    img = make_golden.fma_probe_image(g["seed"], g["mods"])
    ex = oracle.OracleExtractor(g["nfeatures"], semantics=0x20)
    k, d_nofma = ex(img)
    _, d_fma = oracle.OracleExtractor(g["nfeatures"])(img)
    txt = open(os.path.join(ROOT, "oracle", "orb_pattern.inc")).read()
    pat = np.array([int(v) for v in re.findall(r"-?\d+", txt[txt.index("{") + 1:txt.index("};")])]).reshape(256, 4)
    blurred = oracle.gaussian7(ex.level(0), 0)
    F = np.float32
    rows = np.nonzero((d_nofma != d_fma).any(1) & (k["octave"] == 0))[0]
    assert len(rows) > 0
    for i in rows:
        s, c = oracle.sincos(F(F(k["angle"][i]) * F(3.14159265358979323846 / 180.0)))
        a, b = F(c), F(s)
        cx, cy = int(np.rint(k["x"][i])), int(np.rint(k["y"][i]))
        for form, want in (("nofma", d_nofma[i]), ("fma", d_fma[i])):
            bits = []
            for x0, y0, x1, y1 in pat:
                v = []
                for x, y in ((F(x0), F(y0)), (F(x1), F(y1))):
                    if form == "nofma":
                        r, q = F(F(x * b) + F(y * a)), F(F(x * a) - F(y * b))
                    else:
                        r, q = refpy.fmaf(x, b, F(y * a)), refpy.fmaf(x, a, -F(y * b))
                    v.append(int(blurred[cy + int(np.rint(r)), cx + int(np.rint(q))]))
                bits.append(v[0] < v[1])
            assert np.array_equal(np.packbits(np.array(bits, np.uint8), bitorder="little"), want), (form, i)


def test_oracle_bench_golden_sample(oracle):
    """tests/golden/bench_golden.json (the frames bench.py times): the oracle reproduces the initial frame and two
    frames of rank 0 and one of rank 5 from bench._frames."""
    from orbslam2_with_quadrics_amd import synthetic

    sys.path.insert(0, ROOT)
    import bench

    g = json.load(open(os.path.join(GOLDEN, "bench_golden.json")))
    for rank, idx in ((0, (0, 17)), (5, (3,))):
        gr = g["ranks"][rank]
        f1, frames = bench._frames(synthetic, g["rows"], g["cols"], 32, rank)
        ex = oracle.OracleExtractor(g["nfeatures"])
        k1, d1 = ex(f1)
        assert hashlib.sha256(k1.tobytes()).hexdigest() == gr["f1"]["kps_sha256"]
        for i in idx:
            k, d = ex(frames[i])
            assert hashlib.sha256(k.tobytes()).hexdigest() == gr["frames"][i]["kps_sha256"]
            assert hashlib.sha256(d.tobytes()).hexdigest() == gr["frames"][i]["desc_sha256"]


def test_oracle_bench_extract_golden_sample(oracle):
    """tests/golden/bench_extract_golden.json (the config-2 frames bench.py --workload extract times): the oracle
    reproduces frames of ranks 0 and 7 from bench._frames."""
    from orbslam2_with_quadrics_amd import synthetic

    sys.path.insert(0, ROOT)
    import bench

    g = json.load(open(os.path.join(GOLDEN, "bench_extract_golden.json")))
    for rank, idx in ((0, (0, 31)), (7, (9,))):
        gr = g["ranks"][rank]
        _, frames = bench._frames(synthetic, g["rows"], g["cols"], 32, rank, 2000)
        ex = oracle.OracleExtractor(g["nfeatures"])
        for i in idx:
            k, d = ex(frames[i])
            assert len(k) == gr["frames"][i]["n"]
            assert hashlib.sha256(k.tobytes()).hexdigest() == gr["frames"][i]["kps_sha256"]
            assert hashlib.sha256(d.tobytes()).hexdigest() == gr["frames"][i]["desc_sha256"]


def test_oracle_bench_stereo_golden_sample(oracle):
    """tests/golden/bench_stereo_golden.json (the config-4 pairs bench.py --workload stereo times): the oracle
    reproduces one pair of rank 0 and one of rank 6."""
    from orbslam2_with_quadrics_amd import synthetic

    g = json.load(open(os.path.join(GOLDEN, "bench_stereo_golden.json")))
    mbf, mb = 386.1448, 386.1448 / 718.856
    for rank, i in ((0, 5), (6, 12)):
        gp = g["ranks"][rank]["pairs"][i]
        left, right = synthetic.stereo_pair(3000 + rank * 100 + i, g["rows"], g["cols"])[:2]
        exL, exR = oracle.OracleExtractor(g["nfeatures"]), oracle.OracleExtractor(g["nfeatures"])
        kL, dL = exL(left)
        kR, dR = exR(right)
        n, ur, de = oracle.stereo_matches(exL, exR, kL, dL, kR, dR, mbf, mb)
        assert (len(kL), n) == (gp["n"], gp["nmatches"])
        assert hashlib.sha256(ur.astype(np.float32).tobytes()).hexdigest() == gp["uright_sha256"]
        assert hashlib.sha256(de.astype(np.float32).tobytes()).hexdigest() == gp["depth_sha256"]


def test_oracle_bench_tracking_golden_sample(oracle):
    """tests/golden/bench_tracking_golden.json (the config-5 frames bench.py --workload tracking times): the oracle
    reproduces one frame of rank 3 -- extraction, isInFrustum for its camera, SearchByProjection (th 1)."""
    from orbslam2_with_quadrics_amd import synthetic

    sys.path.insert(0, ROOT)
    import bench

    g = json.load(open(os.path.join(GOLDEN, "bench_tracking_golden.json")))
    rank, i = 3, 21
    rows, cols = g["rows"], g["cols"]
    f_ref, frames = bench._frames(synthetic, rows, cols, 32, rank, 5000)
    ex = oracle.OracleExtractor(g["nfeatures"])
    sf = ex.tables()["scale"]
    k0, d0 = ex(f_ref)
    mp = bench.local_map(k0, d0, g["mappoints"], 7000, cols, rows, sf)
    k, d = ex(frames[i])
    _, tr = oracle.is_in_frustum(bench.rig_camera(cols, rows, *bench.frame_shift(i), 1.2, len(sf)), mp["pos"],
                                 mp["normal"], mp["max_dist"], mp["min_dist"], 0.5)
    n, own, obs = oracle.search_by_projection(oracle.OracleFrame(k, d, cols, rows, sf),
                                              dict(tr, is_bad=mp["is_bad"], n_obs=mp["n_obs"], desc=mp["desc"]), 0.8, 1.0)
    gf = g["ranks"][rank]["frames"][i]
    assert (len(k), n) == (gf["n"], gf["nmatches"])
    assert hashlib.sha256(own.astype(np.int32).tobytes()).hexdigest() == gf["owner_sha256"]
    assert hashlib.sha256(obs.astype(np.int32).tobytes()).hexdigest() == gf["owner_obs_sha256"]


def test_libm_chunk_golden_matches_host_libm():
    """tests/golden/libm_chunks.json (the GPU pins' reference) re-derived from this host's libm on sample chunks."""
    sys.path.insert(0, GOLDEN)
    import make_golden

    g = json.load(open(os.path.join(GOLDEN, "libm_chunks.json")))
    cl = g["chunk_log2"]
    for fn, spec in g["functions"].items():
        for c in (0, len(spec["hashes"]) // 2, len(spec["hashes"]) - 1):
            lo = max(spec["begin"], ((spec["begin"] >> cl) + c) << cl)
            hi = min(spec["end"], ((spec["begin"] >> cl) + c + 1) << cl)
            assert make_golden.libm_chunk_hashes(fn, lo, hi, cl) == [spec["hashes"][c]], (fn, c)


def test_fast_oracle_build_is_bit_identical(tmp_path):
    """The -O3 -march=native oracle build (the CPU baseline's) gives the same keypoints, descriptors and matches
    as the -O2 checker build (FMAs are explicit, contraction is off in both)."""
    code = r'''
import hashlib, sys
sys.path[:0] = [%r, %r]
import numpy as np
import oracle_py as O
from orbslam2_with_quadrics_amd import synthetic
f1, f2 = synthetic.frame_pair(21, 480, 640)
ex = O.OracleExtractor(1000)
k1, d1 = ex(f1); k2, d2 = ex(f2)
sf = ex.tables()["scale"]
n, m, p = O.search_for_initialization(O.OracleFrame(k1, d1, 640, 480, sf), O.OracleFrame(k2, d2, 640, 480, sf),
                                      np.stack([k1["x"], k1["y"]], 1).astype(np.float32), 0.9, True, 100)
print(O.LIB_PATH, hashlib.sha256(k1.tobytes() + d1.tobytes() + k2.tobytes() + d2.tobytes() + m.tobytes()).hexdigest())
''' % (ROOT, os.path.join(ROOT, "oracle"))
    outs = []
    for fast in ("0", "1"):
        env = dict(os.environ, ORB_ORACLE_FAST=fast)
        outs.append(subprocess.check_output([sys.executable, "-c", code], env=env).decode().split())
    assert outs[0][0] != outs[1][0] and outs[0][1] == outs[1][1], outs


def test_fast_slot_division_exact():
    """The quotient trick trunc(fma(p, 1/H, 0.5/H)) in float32 (og_resize2_kernel's staging maps a chunk index to
    (row, chunk) this way, csrc/orb_extract.hip).  (p + 1/2)/H is at least 1/(2H) from an integer, far beyond the rounding of
    the correctly rounded 1/H and of the fma, so the quotient is exact: checked for every p < 2^14 and H <= 128
    (the kernels need p < 2^14).  The fma is evaluated exactly in float64 (a 24 x 24-bit product
    is exact there) and rounded once to float32, as the hardware fma rounds."""
    p = np.arange(0, 1 << 14, dtype=np.int64)
    for H in range(1, 129):
        rH = np.float32(1.0) / np.float32(H)
        hH = np.float32(0.5) * rH
        q = (p.astype(np.float64) * np.float64(rH) + np.float64(hH)).astype(np.float32)
        assert np.array_equal(np.trunc(q).astype(np.int64), p // H), H
