"""GPU parity tests of Frame::ComputeStereoMatches (src/Frame.cc:466-640) through the C ABI against the
CPU oracle (oo_stereo_matches): mvuRight / mvDepth must be bit-identical, match counts equal.
KITTI-shape pairs (1241 x 376, bf = 386.1448, fx = 718.856 -- SURVEY.md §8 config 4)."""
import numpy as np
import pytest

from orbslam2_with_quadrics_amd import synthetic

pytestmark = pytest.mark.gpu

MBF = 386.1448
MB = MBF / 718.856


def _oracle_stereo(oracle, left, right, nf):
    exL = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
    exR = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
    kL, dL = exL(left)
    kR, dR = exR(right)
    n, ur, de = oracle.stereo_matches(exL, exR, kL, dL, kR, dR, MBF, MB)
    return kL, kR, n, ur, de


def _gpu_stereo(gpu, left, right, nf):
    exL = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    exR = gpu.ORBextractor(nf, 1.2, 8, 20, 7)
    kL, _ = exL(left)
    kR, _ = exR(right)
    ur, de, nm = gpu.ComputeStereoMatches(exL, exR, MBF, MB)
    return exL, exR, kL, kR, ur, de, nm


def _same_f32(a, b):
    np.testing.assert_array_equal(np.asarray(a, np.float32).view(np.uint32), np.asarray(b, np.float32).view(np.uint32))


@pytest.mark.parametrize("pid", range(4))
def test_stereo_kitti_shape_vs_oracle(gpu, oracle, pid):
    left, right, _ = synthetic.stereo_pair(100 + pid, 376, 1241)
    kL, kR, n, ur, de = _oracle_stereo(oracle, left, right, 2000)
    _, _, gkL, gkR, gur, gde, gn = _gpu_stereo(gpu, left, right, 2000)
    assert np.array_equal(gkL, kL) and np.array_equal(gkR, kR)
    assert gn == n and n > 100
    _same_f32(gur, ur)
    _same_f32(gde, de)


def test_stereo_identical_images_zero_disparity_branch(gpu, oracle):
    """left == right: disparities around 0 exercise the `disparity <= 0 -> 0.01` branch (:615-619)."""
    img = synthetic.frame(7, 376, 1241)
    kL, kR, n, ur, de = _oracle_stereo(oracle, img, img, 2000)
    _, _, _, _, gur, gde, gn = _gpu_stereo(gpu, img, img, 2000)
    assert gn == n
    _same_f32(gur, ur)
    _same_f32(gde, de)


@pytest.mark.parametrize("shape,nf", [((480, 640), 1000), ((720, 1280), 1500), ((1080, 1920), 2000)])
def test_stereo_other_sizes_vs_oracle(gpu, oracle, shape, nf):
    h, w = shape
    left, right, _ = synthetic.stereo_pair(200 + w, h, w, band=48, dmin=0, dmax=60)
    kL, kR, n, ur, de = _oracle_stereo(oracle, left, right, nf)
    _, _, _, _, gur, gde, gn = _gpu_stereo(gpu, left, right, nf)
    assert gn == n
    _same_f32(gur, ur)
    _same_f32(gde, de)


def test_stereo_empty_right_image(gpu, oracle):
    left, _, _ = synthetic.stereo_pair(3, 376, 1241)
    right = synthetic.flat(376, 1241)
    kL, kR, n, ur, de = _oracle_stereo(oracle, left, right, 2000)
    assert len(kR) == 0 and n == 0
    _, _, _, _, gur, gde, gn = _gpu_stereo(gpu, left, right, 2000)
    assert gn == 0
    assert np.all(gur == -1) and np.all(gde == -1) and len(gur) == len(kL)


def test_stereo_rejects_mismatched_extractors(gpu):
    left, right, _ = synthetic.stereo_pair(4, 376, 1241)
    exL = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    exR = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    exL(left)
    exR(right[:, :1200].copy())
    with pytest.raises(RuntimeError):
        gpu.ComputeStereoMatches(exL, exR, MBF, MB)


def test_stereo_batch_device_equals_oracle(gpu, oracle):
    """B rectified pairs resident in HBM: one batched stereo launch == B oracle runs."""
    import ctypes as C

    from orbslam2_with_quadrics_amd import _lib

    B, rows, cols = 5, 376, 1241
    pairs = [synthetic.stereo_pair(300 + b, rows, cols) for b in range(B)]
    exL = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    exR = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    dl = exL.device_alloc(B * rows * cols)
    dr = exR.device_alloc(B * rows * cols)
    try:
        exL.h2d(dl, np.stack([p[0] for p in pairs]))
        exR.h2d(dr, np.stack([p[1] for p in pairs]))
        exL.extract_batch_device(dl, B, cols, rows, cols, rows * cols)
        exR.extract_batch_device(dr, B, cols, rows, cols, rows * cols)
        _, _, _, fcap = exL.batch_outputs()
        d_out = exL.device_alloc(B * fcap * 8 + B * 4)
        d_ur, d_de, d_nm = d_out, d_out + B * fcap * 4, d_out + B * fcap * 8
        L = _lib.lib()
        _lib.check(exL.ctx, L.orbgpu_compute_stereo_matches_batch(exL.ctx, exR.ctx, MBF, MB, C.c_void_p(d_ur),
                                                                   C.c_void_p(d_de), C.c_void_p(d_nm)),
                   "stereo_batch")
        exL.synchronize()
        ur = np.zeros((B, fcap), np.float32)
        de = np.zeros((B, fcap), np.float32)
        nm = np.zeros(B, np.int32)
        exL.d2h(ur, d_ur)
        exL.d2h(de, d_de)
        exL.d2h(nm, d_nm)
        for b in range(B):
            kL, _, n, our, ode = _oracle_stereo(oracle, pairs[b][0], pairs[b][1], 2000)
            assert nm[b] == n
            _same_f32(ur[b, :len(kL)], our)
            _same_f32(de[b, :len(kL)], ode)
        exL.device_free(d_out)
    finally:
        exL.device_free(dl)
        exR.device_free(dr)
