"""ORBGPU_SEM_SCORE_HARRIS option (include/orbgpu.h): the octree ranks FAST candidates by OpenCV ORB's Harris
response (features2d orb.cpp HarrisResponses, blockSize 7, k 0.04) instead of the FAST score.

ORB-SLAM2 itself never ranks by Harris (src/ORBextractor.cc:795-806), and OpenCV is absent from
/root/reference, so this option's parity is UNPINNED: the oracle (oracle/orb_oracle.c oo_harris_response) is a
restatement of the published algorithm, checked here against a second, numpy restatement; the GPU path is then
bit-exact against the oracle.  The default path (FAST score) is unchanged and covered by every other parity test.
"""
import numpy as np
import pytest

from orbslam2_with_quadrics_amd import _lib, synthetic

FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def harris_numpy(img, x, y):
    """Independent restatement: Sobel-form gradients by array slicing, the float tail in float32 steps."""
    p = img.astype(np.int64)
    win = p[y - 4:y + 5, x - 4:x + 5]
    ix = 2 * (win[1:-1, 2:] - win[1:-1, :-2]) + (win[:-2, 2:] - win[:-2, :-2]) + (win[2:, 2:] - win[2:, :-2])
    iy = 2 * (win[2:, 1:-1] - win[:-2, 1:-1]) + (win[2:, :-2] - win[:-2, :-2]) + (win[2:, 2:] - win[:-2, 2:])
    a, b, c = (int((ix * ix).sum()), int((iy * iy).sum()), int((ix * iy).sum()))
    f = np.float32
    scale = f(1.0) / f(4 * 7 * 255.0)
    s4 = f(f(f(scale * scale) * scale) * scale)
    fa, fb, fc = f(a), f(b), f(c)
    s = f(fa + fb)
    return float(f(f(f(fa * fb) - f(fc * fc)) - f(f(f(0.04) * s) * s)) * s4)


def test_oracle_harris_matches_numpy_restatement(oracle):
    rng = np.random.default_rng(7)
    img = synthetic.frame(3, 120, 160)
    noise = rng.integers(0, 256, (40, 40), dtype=np.uint8)
    for im in (img, noise, np.full((20, 20), 77, np.uint8)):
        h, w = im.shape
        for _ in range(60):
            x, y = int(rng.integers(4, w - 4)), int(rng.integers(4, h - 4))
            r = oracle.harris_response(im, x, y)
            assert np.float32(r).view(np.int32) == np.float32(harris_numpy(im, x, y)).view(np.int32), (x, y)
    assert oracle.harris_response(np.full((20, 20), 77, np.uint8), 9, 9) == 0.0  # flat: a = b = c = 0
    # a vertical step edge: Ix only, so a*b - c^2 = 0 and the response is -k a^2 scale^4 < 0
    step = np.zeros((20, 20), np.uint8)
    step[:, 10:] = 200
    assert oracle.harris_response(step, 10, 10) < 0


def test_harris_key_orders_like_float():
    from oracle_py import harris_key

    vals = np.array([-3e4, -1.0, -1e-30, 0.0, 1e-30, 0.5, 1.0, 7e5], np.float32)
    keys = [harris_key(float(v)) for v in vals]
    assert keys == sorted(keys) and len(set(keys)) == len(keys)
    assert harris_key(-0.0) == harris_key(0.0)


def test_oracle_harris_extraction_properties(oracle):
    """Harris ranking changes which keypoint each octree node keeps, not how many nodes there are; every kept
    keypoint's response is the Harris response at its level pixel, and it is the node maximum of its candidates."""
    img = synthetic.frame(3, 480, 640)
    base = oracle.OracleExtractor(1000)
    hk = oracle.OracleExtractor(1000, semantics=_lib.SEM_SCORE_HARRIS)
    k0, _ = base(img)
    k1, d1 = hk(img)
    assert len(k1) == len(k0)
    moved = 0
    for lvl in range(8):
        a, b = k0[k0["octave"] == lvl], k1[k1["octave"] == lvl]
        assert len(a) == len(b)
        lv = hk.level(lvl)
        s = base.tables()["scale"][lvl]
        for kp in b:
            x, y = (kp["x"], kp["y"]) if lvl == 0 else (kp["x"] / s, kp["y"] / s)
            xi, yi = int(round(float(x))), int(round(float(y)))
            assert kp["response"] == np.float32(oracle.harris_response(lv, xi, yi))
        moved += int((np.sort(a["x"]) != np.sort(b["x"])).any())
    assert moved > 0  # the option actually changes the selection on a natural frame


@pytest.mark.gpu
@pytest.mark.parametrize("shape,nf", [((480, 640), 1000), ((376, 1241), 2000), ((1080, 1920), 2000)])
def test_gpu_harris_vs_oracle(gpu, oracle, shape, nf):
    h, w = shape
    img = synthetic.frame(11, h, w)
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7, semantics=_lib.SEM_SCORE_HARRIS)
    oe = oracle.OracleExtractor(nf, semantics=_lib.SEM_SCORE_HARRIS)
    k, d = ex(img)
    ko, do = oe(img)
    assert len(k) == len(ko)
    for f in FIELDS:
        bad = np.nonzero(k[f].view(np.int32) != ko[f].view(np.int32))[0]
        assert len(bad) == 0, (f, bad[:5])
    assert np.array_equal(d, do)
    # the octree's response keys are the order-preserving image of the oracle's floats
    from oracle_py import harris_key
    for lvl in (0, 3):
        gx, gy, gr = ex.debug_octree(0, lvl)
        xy, resp = oe.candidates(lvl)
        assert len(gr) > 0
        assert set(int(r) for r in gr) <= set(harris_key(float(r)) for r in resp)


@pytest.mark.gpu
def test_gpu_harris_batch_and_default_unchanged(gpu, oracle):
    """A 16-frame batched launch under the option matches the oracle per frame; switching the option off again
    on the same context returns the FAST-score extraction bit for bit."""
    B, rows, cols = 16, 480, 640
    frames = np.stack([synthetic.frame(600 + b, rows, cols) for b in range(B)]).astype(np.uint8)
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7, semantics=_lib.SEM_SCORE_HARRIS)
    oe = oracle.OracleExtractor(1000, semantics=_lib.SEM_SCORE_HARRIS)
    d_img = ex.device_alloc(frames.nbytes)
    try:
        ex.h2d(d_img, frames)
        ex.extract_batch_device(d_img, B, cols, rows, cols, rows * cols)
        ex.synchronize()
        for b in range(B):
            k, d = ex.batch_download(b)
            ko, do = oe(frames[b])
            assert k.tobytes() == ko.tobytes() and np.array_equal(d, do), b
    finally:
        ex.device_free(d_img)
    ex.set_semantics(_lib.SEM_DEFAULT)
    k, d = ex(frames[0])
    ko, do = oracle.OracleExtractor(1000)(frames[0])
    assert k.tobytes() == ko.tobytes() and np.array_equal(d, do)
