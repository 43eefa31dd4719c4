"""Colour input (Tracking::GrabImage*'s cvtColor, src/Tracking.cc:169-255) and the config-1 TUM RGB-D path on
the GPU, bit-exact against the oracle: the batched conversion kernel, orbgpu_extract_color, and a synthetic
TUM sequence read from PNG files through tum.grab_image_rgbd (gray conversion, extraction, UndistortKeyPoints,
ComputeStereoFromRGBD)."""
import numpy as np
import pytest

from orbslam2_with_quadrics_amd import synthetic

from test_gpu_extract import assert_same
from test_tum import TUM1_YAML

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("code,rows,cols,B,pad", [(7, 480, 640, 3, 0), (6, 376, 1241, 2, 5), (11, 33, 7, 4, 3),
                                                 (10, 1080, 1920, 1, 0), (7, 5, 1, 2, 1)])
def test_cvt_color_batch_vs_oracle(gpu, oracle, code, rows, cols, B, pad):
    cn = 4 if code >= 10 else 3
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    rng = np.random.default_rng(rows * 7 + cols)
    imgs = rng.integers(0, 256, size=(B, rows, cols, cn), dtype=np.uint8)
    spitch = cols * cn + pad                   # odd pitches take the byte path
    sstride = spitch * rows + 3 * pad          # and odd frame strides
    dpitch, dstride = cols + pad, (cols + pad) * rows + pad
    host = np.zeros(sstride * B + 64, np.uint8)
    for b in range(B):
        v = host[b * sstride: b * sstride + spitch * rows].reshape(rows, spitch)
        v[:, :cols * cn] = imgs[b].reshape(rows, cols * cn)
    d_src = ex.device_alloc(host.nbytes)
    d_dst = ex.device_alloc(dstride * B + 64)
    try:
        ex.h2d(d_src, host)
        ex.cvt_color_to_gray_batch(d_src + pad, B, cols, rows, spitch, sstride, code, d_dst + pad, dpitch, dstride)
        out = np.zeros(dstride * B + 64, np.uint8)
        ex.d2h(out, d_dst)
    finally:
        ex.device_free(d_src)
        ex.device_free(d_dst)
    for b in range(B):
        # the kernel read from d_src + pad: shift the expected frame accordingly
        v = np.frombuffer(host[pad + b * sstride: pad + b * sstride + spitch * rows].tobytes(), np.uint8)
        src = v.reshape(rows, spitch)[:, :cols * cn].reshape(rows, cols, cn)
        want = oracle.cvt_gray(src, code)
        got = out[pad + b * dstride: pad + b * dstride + dpitch * rows].reshape(rows, dpitch)[:, :cols]
        assert np.array_equal(got, want), (b, np.argwhere(got != want)[:5])


def test_cvt_color_rejects_bad_codes(gpu):
    from orbslam2_with_quadrics_amd import _lib

    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    with pytest.raises(ValueError):
        ex.extract_color(np.zeros((48, 64, 3), np.uint8), _lib.COLOR_RGBA2GRAY)  # 3 channels for a 4-channel code
    L = _lib.lib()
    assert L.orbgpu_cvt_color_to_gray_batch(ex.ctx, None, 1, 8, 8, 24, 192, 7, None, 8, 64) == _lib.ERR_ARG
    d = ex.device_alloc(4096)
    try:
        import ctypes as C
        assert L.orbgpu_cvt_color_to_gray_batch(ex.ctx, C.c_void_p(d), 1, 8, 8, 24, 192, 8, C.c_void_p(d), 8,
                                                64) == _lib.ERR_ARG  # CV_BGRA2RGBA is not a gray conversion
        assert L.orbgpu_cvt_color_to_gray_batch(ex.ctx, C.c_void_p(d), 1, 8, 8, 23, 192, 7, C.c_void_p(d), 8,
                                                64) == _lib.ERR_ARG  # pitch < cols * 3
    finally:
        ex.device_free(d)


@pytest.mark.parametrize("code,shape", [(7, (480, 640)), (6, (376, 1241)), (11, (480, 640))])
def test_extract_color_vs_oracle(gpu, oracle, code, shape):
    rows, cols = shape
    img = synthetic.color_frame(40 + code, rows, cols, alpha=code >= 10)
    if code == 6:
        img = np.ascontiguousarray(img[..., ::-1])  # a BGR image
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    k, d = ex.extract_color(img, code)
    gray = oracle.cvt_gray(img, code)
    oe = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    ko, do = oe(gray)
    assert_same(k, d, ko, do)
    assert np.array_equal(ex.level(0), gray)  # mvImagePyramid[0] is the converted image
    assert np.array_equal(ex.level(3), oe.level(3))
    assert len(k) > 500


def test_tum_rgbd_sequence_vs_oracle(gpu, oracle, tmp_path):
    """Config 1 plumbing: a synthetic TUM RGB-D sequence (PNG colour + 16-bit depth + associations.txt) with the
    TUM1 settings, frame by frame as rgbd_tum.cc reads it, up to the RGB-D Frame."""
    pytest.importorskip("PIL")
    from orbslam2_with_quadrics_amd import tum

    assoc = synthetic.write_tum_rgbd_sequence(str(tmp_path / "seq"), 3)
    yml = tmp_path / "TUM1.yaml"
    yml.write_text(TUM1_YAML)
    fs = tum.read_settings(str(yml))
    K4, dist, mbf, factor, bRGB = tum.camera_from_settings(fs)
    ex = tum.extractor_from_settings(fs)
    oe = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    n = 0
    for t, imRGB, imD in tum.sequence_rgbd(str(tmp_path / "seq"), assoc):
        F = tum.grab_image_rgbd(ex, imRGB, imD, K4, dist, mbf, factor, bRGB)
        # oracle chain: cvtColor(RGB2GRAY) on the BGR data imread returned (the TUM yaml's Camera.RGB: 1), extract,
        # UndistortKeyPoints, convertTo(CV_32F, 1/5000), ComputeStereoFromRGBD
        gray = oracle.cvt_gray(imRGB, 7)
        ko, do = oe(gray)
        assert_same(F.mvKeys, F.mDescriptors, ko, do)
        ku = oracle.undistort_keypoints(K4, dist, ko)
        assert F.mvKeysUn.tobytes() == ku.tobytes()
        wur, wde = oracle.stereo_from_rgbd(ko, ku, oracle.depth_u16_to_f32(imD, float(factor)), float(mbf))
        assert F.mvuRight.tobytes() == wur.tobytes() and F.mvDepth.tobytes() == wde.tobytes()
        assert (F.mvDepth > 0).sum() > 100
        n += 1
    assert n == 3
