"""GPU parity tests: the gfx950 ORBextractor (through the C ABI) against the CPU oracle, bit-exact.

Integer/byte outputs (pyramid, candidates, octree order, octaves, descriptors) must be identical; the
float fields (x, y, size, angle, response) are computed with the reference's exact float operation
sequence and are compared bit-for-bit too.
"""
import numpy as np
import pytest

from orbslam2_with_quadrics_amd import synthetic

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def assert_same(k, d, ko, do):
    assert len(k) == len(ko)
    for f in FIELDS:
        bad = np.nonzero(k[f].view(np.int32) != ko[f].view(np.int32))[0]
        assert len(bad) == 0, (f, bad[:5], k[bad[:3]], ko[bad[:3]])
    assert np.array_equal(d, do)


@pytest.fixture(scope="module")
def ex1000(gpu):
    return gpu.ORBextractor(1000, 1.2, 8, 20, 7)


@pytest.fixture(scope="module")
def ex2000(gpu):
    return gpu.ORBextractor(2000, 1.2, 8, 20, 7)


@pytest.mark.parametrize("fid", [0, 1, 2, 3])
def test_extract_640x480(ex1000, oracle, fid):
    img = synthetic.frame(fid, 480, 640)
    k, d = ex1000(img)
    ko, do = oracle.OracleExtractor(1000)(img)
    assert_same(k, d, ko, do)


def test_extract_1080p(ex2000, oracle):
    img = synthetic.frame(7, 1080, 1920)
    k, d = ex2000(img)
    ko, do = oracle.OracleExtractor(2000)(img)
    assert_same(k, d, ko, do)


def test_extract_kitti_shape(ex2000, oracle):
    img = synthetic.frame(5, 376, 1241)
    k, d = ex2000(img)
    ko, do = oracle.OracleExtractor(2000)(img)
    assert_same(k, d, ko, do)


def test_pyramid_and_candidates(ex1000, oracle):
    img = synthetic.frame(11, 480, 640)
    ex1000(img)
    oe = oracle.OracleExtractor(1000)
    oe(img)
    for l in range(8):
        assert np.array_equal(ex1000.level(l), oe.level(l)), l
        c = ex1000.debug_candidates(0, l)
        g = set(zip((c & 0xFFFF).tolist(), ((c >> 16) & 0xFFFF).tolist(), ((c >> 32) & 0xFF).tolist()))
        xy, r = oe.candidates(l)
        o = set(zip(xy[:, 0].astype(int).tolist(), xy[:, 1].astype(int).tolist(), r.astype(int).tolist()))
        assert g == o, l


@pytest.mark.parametrize("shape", [(481, 643), (300, 211), (620, 500), (96, 130)])
def test_odd_and_small_shapes(gpu, oracle, shape):
    rows, cols = shape
    img = synthetic.frame(13, rows, cols)
    ok = True
    try:
        ex = gpu.ORBextractor(500, 1.2, 8, 20, 7)
        k, d = ex(img)
    except RuntimeError as e:  # levels smaller than a FAST cell: the reference divides by zero
        assert "smaller than one FAST cell" in str(e) or "initial octree" in str(e)
        ok = False
    if ok:
        ko, do = oracle.OracleExtractor(500)(img)
        assert_same(k, d, ko, do)


def test_flat_image_gives_no_keypoints(ex1000, oracle):
    img = synthetic.flat(480, 640, 90)
    k, d = ex1000(img)
    assert len(k) == 0 and d.shape == (0, 32)


def test_pure_noise_stresses_octree(ex2000, oracle):
    img = synthetic.pure_noise(17, 480, 640)
    k, d = ex2000(img)
    ko, do = oracle.OracleExtractor(2000)(img)
    assert_same(k, d, ko, do)


def test_dense_corners_candidate_sets(gpu, oracle):
    """Pure noise at thresholds (3, 1): nearly every pixel passes the quick test and a block keeps hundreds of NMS
    maxima, so FAST's compacted kept list (stage 3, written into the ROI buffer; bound: one strict 3x3 maximum per
    2x2 pixels of a cell, 1280 per block) runs near its densest.  The candidate sets of every level and the final
    keypoints/descriptors must equal the oracle's (src/ORBextractor.cc:789-829 + cv::FAST NMS)."""
    img = synthetic.pure_noise(23, 480, 640)
    params = (3000, 1.2, 8, 3, 1)
    ex = gpu.ORBextractor(*params)
    k, d = ex(img)
    oe = oracle.OracleExtractor(*params)
    ko, do = oe(img)
    assert_same(k, d, ko, do)
    dense = 0
    for l in range(8):
        c = ex.debug_candidates(0, l)
        g = set(zip((c & 0xFFFF).tolist(), ((c >> 16) & 0xFFFF).tolist(), ((c >> 32) & 0xFF).tolist()))
        xy, r = oe.candidates(l)
        o = set(zip(xy[:, 0].astype(int).tolist(), xy[:, 1].astype(int).tolist(), r.astype(int).tolist()))
        assert g == o, l
        dense = max(dense, len(g))
    assert dense > 20000  # (level 0: about one kept maximum per 10 pixels)


def test_threshold_fallback_and_other_params(gpu, oracle):
    img = synthetic.frame(19, 480, 640)
    for params in [(1500, 1.2, 8, 30, 10), (800, 1.3, 6, 12, 5), (4000, 1.2, 8, 20, 7)]:
        ex = gpu.ORBextractor(*params)
        k, d = ex(img)
        ko, do = oracle.OracleExtractor(*params)(img)
        assert_same(k, d, ko, do)


def test_empty_image_returns_untouched(ex1000):
    k, d = ex1000(np.zeros((0, 0), np.uint8))
    assert k is None and d is None


def test_getters_match_oracle(ex1000, oracle):
    t = oracle.OracleExtractor(1000).tables()
    assert ex1000.GetLevels() == 8
    assert np.float32(ex1000.GetScaleFactor()) == np.float32(1.2)
    assert np.array_equal(ex1000.GetScaleFactors(), t["scale"])
    assert np.array_equal(ex1000.GetInverseScaleFactors(), t["inv_scale"])
    assert np.array_equal(ex1000.GetScaleSigmaSquares(), t["sigma2"])
    assert np.array_equal(ex1000.GetInverseScaleSigmaSquares(), t["inv_sigma2"])
    assert np.array_equal(ex1000.features_per_level(), t["features_per_level"])


def test_batch_device_path_equals_per_frame(gpu, oracle):
    """B frames resident in HBM, one batched launch sequence == B single-frame oracle runs."""
    B, rows, cols = 6, 480, 640
    frames = np.stack([synthetic.frame(30 + b, rows, cols) for b in range(B)])
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    d_img = ex.device_alloc(frames.nbytes)
    try:
        ex.h2d(d_img, frames)
        ex.extract_batch_device(d_img, B, cols, rows, cols, rows * cols)
        ex.synchronize()
        oe = oracle.OracleExtractor(1000)
        for b in range(B):
            k, d = ex.batch_download(b)
            ko, do = oe(frames[b])
            assert_same(k, d, ko, do)
    finally:
        ex.device_free(d_img)


def test_two_contexts_interleaved(gpu, oracle):
    """Stereo runs two extractor instances concurrently (src/Frame.cc:78-81): contexts are independent."""
    import threading

    a = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    b = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    L = synthetic.frame(40, 376, 1241)
    R = synthetic.frame(41, 376, 1241)
    out = {}

    def run(name, ex, img):
        out[name] = ex(img)

    ts = [threading.Thread(target=run, args=("L", a, L)), threading.Thread(target=run, args=("R", b, R))]
    [t.start() for t in ts]
    [t.join() for t in ts]
    oe = oracle.OracleExtractor(2000)
    assert_same(*out["L"], *oe(L))
    assert_same(*out["R"], *oe(R))


@pytest.mark.parametrize("seed", range(12))
def test_random_parameters_vs_oracle(gpu, oracle, seed):
    """Randomised extractor parameters and image shapes (scale factor up to the 1.6 the fused pyramid's LDS is
    sized for, 1-8 levels, thresholds, odd widths and pitches): keypoints, descriptors and the whole pyramid
    bit-exact.  Configurations the reference itself cannot run (a level narrower than one FAST cell, or zero
    initial octree nodes) and levels of more than 2040 features must be rejected with ORBGPU_ERR_UNSUPPORTED."""
    rng = np.random.default_rng(1000 + seed)
    rows, cols = int(rng.integers(120, 1100)), int(rng.integers(160, 1300))
    scale = float(np.float32(rng.uniform(1.05, 1.6)))
    nlevels = int(rng.integers(1, 9))
    # level 0 takes nf * (1 - 1/s) / (1 - s^-L) features (src/ORBextractor.cc:435-446): up to 2000 of them (both
    # octree list capacities)
    f = 1.0 / scale
    share0 = (1 - f) / (1 - f ** nlevels) if nlevels > 1 else 1.0
    nf = int(rng.integers(100, max(101, int(2000 / share0))))
    ini = int(rng.integers(8, 40))
    mn = int(rng.integers(3, ini))
    img = synthetic.frame(300 + seed, rows, cols)
    if seed % 3 == 0:  # a wider pitch than the width (a view into a larger image)
        big = np.zeros((rows, cols + 13), np.uint8)
        big[:, :cols] = img
        img = big[:, :cols]
    try:
        ex = gpu.ORBextractor(nf, scale, nlevels, ini, mn)
        k, d = ex(img)
    except RuntimeError as e:
        # the reference's own impossibilities, or more than 2040 features on one level (the LDS octree's list
        # capacity): reported, never silently wrong
        assert any(m in str(e) for m in ("FAST cell", "initial octree", "octree capacity", "grid capacity")), str(e)
        return
    oe = oracle.OracleExtractor(nf, scale, nlevels, ini, mn)
    ko, do = oe(np.ascontiguousarray(img))
    assert_same(k, d, ko, do)
    for lvl in range(nlevels):
        assert np.array_equal(ex.level(lvl), oe.level(lvl)), (lvl, rows, cols, scale, nlevels)


@pytest.mark.parametrize("nf,shape", [(5000, (1080, 1920)), (8000, (1080, 1920)), (5000, (480, 640))])
def test_many_features_vs_oracle(gpu, oracle, nf, shape):
    """More than ~1016 features on one level: those levels run the 2048-node octree (two list nodes per thread,
    OG_OCT_MAXL_BIG), the rest the 1024-node one; keypoints and descriptors bit-exact at 5000 and 8000 features."""
    img = synthetic.frame(11, *shape)
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    assert ex.features_per_level()[0] > 1016
    k, d = ex(img)
    ko, do = oracle.OracleExtractor(nf)(img)
    assert_same(k, d, ko, do)


def test_level_capacity_is_reported(gpu):
    """More than 2040 features on one level exceeds the LDS octree list: ORBGPU_ERR_UNSUPPORTED with a message,
    never a silently different keypoint set."""
    ex = gpu.ORBextractor(12000, 1.2, 8, 20, 7)  # level 0 budget 2604
    with pytest.raises(RuntimeError, match="octree capacity"):
        ex(synthetic.frame(3, 480, 640))
