"""Config-1 plumbing on the CPU: the TUM formats (association / rgb.txt / settings / PNG) and the colour
conversion's oracle, pinned against an independent numpy restatement of OpenCV's RGB2Gray<uchar>."""
import os

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import synthetic, tum

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# the TUM1 settings (Examples/RGB-D/TUM1.yaml values) in OpenCV's FileStorage YAML dialect
TUM1_YAML = """%YAML:1.0
Camera.fx: 517.306408
Camera.fy: 516.469215
Camera.cx: 318.643040
Camera.cy: 255.313989
Camera.k1: 0.262383
Camera.k2: -0.953104
Camera.p1: -0.005358
Camera.p2: 0.002628
Camera.k3: 1.163314
Camera.width: 640
Camera.height: 480
Camera.fps: 30.0
Camera.bf: 40.0
Camera.RGB: 1
ThDepth: 40.0
DepthMapFactor: 5000.0
ORBextractor.nFeatures: 1000
ORBextractor.scaleFactor: 1.2
ORBextractor.nLevels: 8
ORBextractor.iniThFAST: 20
ORBextractor.minThFAST: 7
"""


def test_association_file_real_format():
    # first lines of the reference's Examples/RGB-D/associations/fr1_xyz.txt (data fixture)
    rgb, depth, ts = tum.load_images_rgbd(os.path.join(GOLDEN, "fr1_xyz_associations_head.txt"))
    assert len(rgb) == len(depth) == len(ts) == 13
    assert rgb[0] == "rgb/1305031102.175304.png" and depth[0] == "depth/1305031102.160407.png"
    assert ts[0] == 1305031102.175304
    assert all(r.startswith("rgb/") and d.startswith("depth/") for r, d in zip(rgb, depth))
    assert all(b > a for a, b in zip(ts, ts[1:]))


def test_association_edge_cases(tmp_path):
    p = tmp_path / "a.txt"
    p.write_text("\n1.5 rgb/a.png 1.4 depth/a.png\n\n2.5 rgb/b.png 2.4 depth/b.png")  # blank lines, no final \n
    assert tum.load_images_rgbd(str(p)) == (["rgb/a.png", "rgb/b.png"], ["depth/a.png", "depth/b.png"], [1.5, 2.5])
    p.write_text("3.0 rgb/c.png\n")  # a short line: the missing tokens stay empty (stringstream >> fails)
    assert tum.load_images_rgbd(str(p)) == (["rgb/c.png"], [""], [3.0])
    p.write_text("")
    assert tum.load_images_rgbd(str(p)) == ([], [], [])


def test_mono_rgb_txt(tmp_path):
    p = tmp_path / "rgb.txt"
    p.write_text("# color images\n# file: 'x.bag'\n# timestamp filename\n"
                 "1305031102.175304 rgb/1305031102.175304.png\n1305031102.211214 rgb/1305031102.211214.png\n")
    files, ts = tum.load_images_mono(str(p))
    assert files == ["rgb/1305031102.175304.png", "rgb/1305031102.211214.png"]
    assert ts == [1305031102.175304, 1305031102.211214]


def test_settings(tmp_path):
    p = tmp_path / "TUM1.yaml"
    p.write_text(TUM1_YAML)
    fs = tum.read_settings(str(p))
    K4, dist, mbf, factor, bRGB = tum.camera_from_settings(fs)
    assert K4.dtype == np.float32 and K4[0] == np.float32(517.306408)
    assert dist.size == 5 and dist[4] == np.float32(1.163314)  # k3 != 0 -> 5 coefficients
    assert mbf == np.float32(40.0) and bRGB
    assert factor == np.float32(np.float32(1.0) / np.float32(5000.0))
    fs["Camera.k3"] = 0.0
    fs["DepthMapFactor"] = 0.0
    _, dist, _, factor, _ = tum.camera_from_settings(fs)
    assert dist.size == 4 and factor == np.float32(1.0)  # |DepthMapFactor| < 1e-5 -> 1


def test_png_round_trip(tmp_path):
    pytest.importorskip("PIL")
    assoc = synthetic.write_tum_rgbd_sequence(str(tmp_path), 2, 48, 64)
    rgb, depth, ts = tum.load_images_rgbd(assoc)
    assert len(rgb) == 2
    for i, (t, im, d) in enumerate(tum.sequence_rgbd(str(tmp_path), assoc)):
        assert im.dtype == np.uint8 and im.shape == (48, 64, 3)
        assert (im[..., ::-1] == synthetic.color_frame(i, 48, 64)).all()  # imread order: BGR
        assert d.dtype == np.uint16 and (d == synthetic.depth_u16(synthetic.SEED_BASE + i, 48, 64)).all()


def _gray_ref(img, code):
    """Independent restatement: OpenCV RGB2Gray<uchar>, R2Y 4899, G2Y 9617, B2Y 1868, yuv_shift 14."""
    a = img.astype(np.int64)
    b, r = (a[..., 0], a[..., 2]) if code in (6, 10) else (a[..., 2], a[..., 0])
    return ((b * 1868 + a[..., 1] * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


@pytest.mark.parametrize("code", [6, 7, 10, 11])
def test_oracle_gray_pinned(oracle, code):
    cn = 4 if code >= 10 else 3
    rng = np.random.default_rng(code)
    img = rng.integers(0, 256, size=(37, 53, cn), dtype=np.uint8)
    img[0, :8, :3] = [[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [128, 128, 128],
                      [1, 2, 3], [254, 253, 252]]
    g = oracle.cvt_gray(img, code)
    assert (g == _gray_ref(img, code)).all()
    assert g[0, 0] == 0 and g[0, 1] == 255 and g[0, 5] == 128  # the weights sum to 2^14: no saturation
