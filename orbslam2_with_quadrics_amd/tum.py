"""TUM RGB-D sequences in front of the feature path (config 1): the data formats and the per-frame caller.

Mirrors what the reference's example drivers and Tracking do before a Frame reaches the hot path:
  * `load_images_rgbd`  -- Examples/RGB-D/rgbd_tum.cc:142-168 (association file: t rgb t depth per line);
  * `load_images_mono`  -- Examples/Monocular/mono_tum.cc:138-165 (rgb.txt: three header lines, then t path);
  * `read_settings`     -- the cv::FileStorage settings file (Examples/RGB-D/TUM1.yaml), as Tracking reads it
                           (src/Tracking.cc:55-160);
  * `imread_unchanged`  -- cv::imread(path, CV_LOAD_IMAGE_UNCHANGED): colour PNGs as BGR(A), 16-bit depth PNGs
                           as uint16 (decoded with Pillow, which this image ships);
  * `grab_image_rgbd` / `grab_image_monocular` -- Tracking::GrabImageRGBD / GrabImageMonocular up to the Frame
                           (src/Tracking.cc:205-233, 236-260): colour -> gray with cvtColor (on the GPU,
                           orbgpu_extract_color), the depth convertTo(CV_32F, 1/DepthMapFactor) fused into
                           ComputeStereoFromRGBD, then the Frame constructor's UndistortKeyPoints /
                           ComputeImageBounds (src/Frame.cc:107-160).
The SLAM back end behind the Frame (tracking, mapping, loop closing) is out of scope.
"""
from __future__ import annotations

import os

import numpy as np
import yaml

from . import _lib
from .extractor import ORBextractor
from .matcher import ComputeImageBounds, ComputeStereoFromRGBD, Frame, UndistortKeyPoints


def _parse_line(s: str, nfields: int):
    """stringstream >> t >> s ... : whitespace tokens; a missing token leaves "" (t: 0.0, as a failed
    extraction stores 0 since C++11)."""
    tok = s.split()
    out = []
    for k in range(nfields):
        v = tok[k] if k < len(tok) else None
        if k % 2 == 0:
            try:
                out.append(float(v) if v is not None else 0.0)
            except ValueError:
                out.append(0.0)
        else:
            out.append(v if v is not None else "")
    return out


def _lines(path: str):
    # ifstream + getline until eof: every line, the last one included even without a newline
    with open(path, "r") as fp:
        return fp.read().split("\n")


def load_images_rgbd(association_path: str):
    """rgbd_tum.cc LoadImages: (rgb files, depth files, timestamps); empty lines are skipped."""
    rgb, depth, ts = [], [], []
    for s in _lines(association_path):
        if not s:
            continue
        t, srgb, _, sd = _parse_line(s, 4)
        ts.append(t)
        rgb.append(srgb)
        depth.append(sd)
    return rgb, depth, ts


def load_images_mono(rgb_txt_path: str):
    """mono_tum.cc LoadImages: skip three header lines, then (timestamp, file) per non-empty line."""
    files, ts = [], []
    for s in _lines(rgb_txt_path)[3:]:
        if not s:
            continue
        t, f = _parse_line(s, 2)
        ts.append(t)
        files.append(f)
    return files, ts


def read_settings(path: str) -> dict:
    """The settings file Tracking reads with cv::FileStorage (OpenCV YAML: a '%YAML:1.0' first line)."""
    with open(path, "r") as fp:
        text = fp.read()
    if text.startswith("%YAML"):
        text = text.split("\n", 1)[1] if "\n" in text else ""
    return yaml.safe_load(text) or {}


def camera_from_settings(fs: dict):
    """(K4 = fx, fy, cx, cy; distortion k1 k2 p1 p2 [k3]; mbf; DepthMapFactor; bRGB) as Tracking reads them
    (src/Tracking.cc:55-100, 142-146: k3 only when nonzero, mDepthMapFactor = 1/DepthMapFactor unless ~0)."""
    K4 = np.array([fs["Camera.fx"], fs["Camera.fy"], fs["Camera.cx"], fs["Camera.cy"]], np.float32)
    d = [fs["Camera.k1"], fs["Camera.k2"], fs["Camera.p1"], fs["Camera.p2"]]
    k3 = float(fs.get("Camera.k3", 0.0) or 0.0)
    if k3 != 0:
        d.append(k3)
    dist = np.array(d, np.float32)
    mbf = np.float32(fs.get("Camera.bf", 0.0))
    dmf = np.float32(fs.get("DepthMapFactor", 1.0))
    factor = np.float32(1.0) if abs(float(dmf)) < 1e-5 else np.float32(np.float32(1.0) / dmf)
    return K4, dist, mbf, factor, int(fs.get("Camera.RGB", 1)) != 0


def extractor_from_settings(fs: dict, device: int = 0, init: bool = False) -> ORBextractor:
    """The tracking extractor (src/Tracking.cc:108-125); init=True gives the monocular initialiser's
    2 x nFeatures instance."""
    n = int(fs["ORBextractor.nFeatures"])
    return ORBextractor(2 * n if init else n, float(fs["ORBextractor.scaleFactor"]), int(fs["ORBextractor.nLevels"]),
                        int(fs["ORBextractor.iniThFAST"]), int(fs["ORBextractor.minThFAST"]), device=device)


def imread_unchanged(path: str) -> np.ndarray:
    """cv::imread(path, CV_LOAD_IMAGE_UNCHANGED): gray stays gray, colour comes back BGR / BGRA, 16-bit
    stays uint16."""
    from PIL import Image  # Pillow: the only image decoder in this image (no OpenCV)

    with Image.open(path) as im:
        mode = im.mode
        a = np.array(im)
    if mode in ("I;16", "I;16B", "I;16L", "I"):
        return a.astype(np.uint16)
    if a.ndim == 3 and a.shape[2] in (3, 4):
        a = a[..., [2, 1, 0, 3][:a.shape[2]]]  # RGB(A) -> BGR(A), imread's channel order
    return np.ascontiguousarray(a)


def color_code(channels: int, bRGB: bool) -> int | None:
    """The cvtColor code Tracking::GrabImage* applies (src/Tracking.cc:209-225), None for a gray image."""
    if channels == 3:
        return _lib.COLOR_RGB2GRAY if bRGB else _lib.COLOR_BGR2GRAY
    if channels == 4:
        return _lib.COLOR_RGBA2GRAY if bRGB else _lib.COLOR_BGRA2GRAY
    return None


def _extract(ex: ORBextractor, im: np.ndarray, bRGB: bool, K4=None, dist=None):
    if dist is not None and dist.size and float(dist[0]) != 0.0:
        # the context's device-side mvKeysUn (ComputeStereoFromRGBD reads kpU.x from it), set once per camera
        key = (np.asarray(K4, np.float32).tobytes(), np.asarray(dist, np.float32).tobytes())
        if getattr(ex, "_tum_camera", None) != key:
            ex.set_undistortion(K4, dist)
            ex._tum_camera = key
    code = color_code(im.shape[2] if im.ndim == 3 else 1, bRGB)
    return ex(im) if code is None else ex.extract_color(im, code)


def _frame(ex: ORBextractor, k, d, cols: int, rows: int, K4, dist):
    if dist is None or dist.size == 0 or float(dist[0]) == 0.0:
        return Frame(k, d, cols, rows, ex.GetScaleFactors())
    ku = UndistortKeyPoints(ex, K4, dist, k)
    g = ComputeImageBounds(ex, K4, dist, cols, rows)
    return Frame(k, d, cols, rows, ex.GetScaleFactors(), keys_un=ku, grid=g)


def grab_image_rgbd(ex: ORBextractor, imRGB: np.ndarray, imD: np.ndarray, K4, dist, mbf, depth_factor,
                    bRGB: bool = True) -> Frame:
    """Tracking::GrabImageRGBD up to the RGB-D Frame (src/Tracking.cc:205-230, src/Frame.cc:107-160):
    gray conversion + extraction, UndistortKeyPoints, ComputeStereoFromRGBD (mvuRight, mvDepth)."""
    rows, cols = imRGB.shape[:2]
    k, d = _extract(ex, imRGB, bRGB, K4, dist)
    if k is None:
        raise ValueError("grab_image_rgbd: empty image")
    F = _frame(ex, k, d, cols, rows, K4, dist)
    if imD.dtype == np.uint16:  # convertTo(CV_32F, mDepthMapFactor) fused into the lookup
        F.mvuRight, F.mvDepth = ComputeStereoFromRGBD(ex, imD, float(mbf), float(depth_factor))
        return F
    dep = np.asarray(imD, np.float32)
    if abs(float(depth_factor) - 1.0) > 1e-5:  # src/Tracking.cc:227-228 scales a CV_32F map too
        dep = (dep * np.float32(depth_factor)).astype(np.float32)
    F.mvuRight, F.mvDepth = ComputeStereoFromRGBD(ex, dep, float(mbf), 1.0)
    return F


def grab_image_monocular(ex: ORBextractor, im: np.ndarray, K4, dist, bRGB: bool = True) -> Frame:
    """Tracking::GrabImageMonocular up to the monocular Frame (src/Tracking.cc:236-260, src/Frame.cc:161-210)."""
    rows, cols = im.shape[:2]
    k, d = _extract(ex, im, bRGB, K4, dist)
    if k is None:
        raise ValueError("grab_image_monocular: empty image")
    return _frame(ex, k, d, cols, rows, K4, dist)


def sequence_rgbd(sequence_dir: str, association_path: str):
    """Yields (timestamp, imRGB, imD) over a TUM RGB-D sequence, as rgbd_tum.cc's main loop reads them."""
    rgb, depth, ts = load_images_rgbd(association_path)
    if not rgb:
        raise FileNotFoundError("No images found in provided path.")
    for f_rgb, f_d, t in zip(rgb, depth, ts):
        yield t, imread_unchanged(os.path.join(sequence_dir, f_rgb)), imread_unchanged(os.path.join(sequence_dir, f_d))
