"""ctypes binding of the CPU oracle (oracle/build/liborb_oracle.so) -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; the product
(orbslam2_with_quadrics_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborb_oracle.so")
# ORB_ORACLE_FAST=1: the -O3 -march=native build (the reference's flags; bit-identical results) for CPU timing
if os.environ.get("ORB_ORACLE_FAST") == "1":
    LIB_PATH = os.path.join(HERE, "build", "liborb_oracle_fast.so")

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i32, f32, u8p = C.c_void_p, C.c_int, C.c_float, C.c_void_p
        L.oo_create.restype = vp
        L.oo_create.argtypes = [i32, f32, i32, i32, i32]
        L.oo_destroy.argtypes = [vp]
        L.oo_extract.restype = i32
        L.oo_extract.argtypes = [vp, u8p, i32, i32, i32, vp, vp, i32]
        L.oo_scale_tables.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.oo_level_size.argtypes = [vp, i32, C.POINTER(i32), C.POINTER(i32)]
        L.oo_level_image.restype = C.POINTER(C.c_uint8)
        L.oo_level_image.argtypes = [vp, i32]
        L.oo_level_candidates.restype = i32
        L.oo_level_candidates.argtypes = [vp, i32, vp, vp, i32]
        L.oo_distribute_octree.restype = i32
        L.oo_distribute_octree.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp]
        L.oo_resize_linear.argtypes = [vp, i32, i32, vp, i32, i32, i32]
        L.oo_gaussian7.argtypes = [vp, i32, i32, vp, i32]
        L.oo_set_semantics.restype = i32
        L.oo_set_semantics.argtypes = [vp, i32]
        L.oo_fast_score.restype = i32
        L.oo_fast_score.argtypes = [vp, i32, i32, i32]
        L.oo_harris_response.restype = C.c_float
        L.oo_harris_response.argtypes = [vp, i32, i32, i32]
        L.oo_fastatan2.restype = f32
        L.oo_fastatan2.argtypes = [f32, f32]
        L.oo_sincos.argtypes = [f32, C.POINTER(f32), C.POINTER(f32)]
        L.oo_descriptor_distance.restype = i32
        L.oo_descriptor_distance.argtypes = [vp, vp]
        L.oo_grid_params.argtypes = [i32, i32] + [C.POINTER(f32)] * 6
        L.oo_grid_build.argtypes = [vp]
        L.oo_features_in_area.restype = i32
        L.oo_features_in_area.argtypes = [vp, f32, f32, f32, i32, i32, vp]
        L.oo_search_for_initialization.restype = i32
        L.oo_search_for_initialization.argtypes = [vp, vp, f32, i32, vp, vp, i32]
        L.oo_stereo_matches.restype = i32
        L.oo_stereo_matches.argtypes = [vp, vp, vp, vp, i32, vp, vp, i32, f32, f32, vp, vp]
        L.oo_search_by_projection.restype = i32
        L.oo_search_by_projection.argtypes = [vp, vp, f32, f32, vp, vp]
        L.oo_is_in_frustum.restype = i32
        L.oo_is_in_frustum.argtypes = [vp, vp, f32, vp, vp, vp, vp, vp, vp]
        L.oo_kf_predicted_levels.argtypes = [vp, vp, vp]
        L.oo_search_by_projection_kf.restype = i32
        L.oo_search_by_projection_kf.argtypes = [vp, vp, vp, f32, i32, i32, vp]
        L.oo_stereo_from_rgbd.argtypes = [vp, vp, i32, vp, i32, f32, vp, vp]
        L.oo_depth_u16_to_f32.argtypes = [vp, i32, f32, vp]
        L.oo_cvt_gray.argtypes = [vp, i32, i32, i32, i32, i32, vp, i32]
        L.oo_vocab_from_arrays.restype = vp
        L.oo_vocab_from_arrays.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp]
        L.oo_vocab_load_text.restype = vp
        L.oo_vocab_load_text.argtypes = [C.c_char_p]
        L.oo_vocab_free.argtypes = [vp]
        L.oo_vocab_nodes.argtypes = [vp]
        L.oo_vocab_words.argtypes = [vp]
        L.oo_bow_transform.argtypes = [vp, vp, i32, i32, vp, vp, C.POINTER(i32), vp, vp, vp, C.POINTER(i32)]
        L.oo_undistort_points.argtypes = [vp, vp, i32, vp, vp, i32]
        L.oo_undistort_keypoints.argtypes = [vp, vp, i32, vp, vp, i32]
        L.oo_compute_image_bounds.argtypes = [vp, vp, i32, i32, i32] + [C.POINTER(f32)] * 6
        L.oo_search_by_projection_last.restype = i32
        L.oo_search_by_projection_last.argtypes = [vp, vp, vp, vp, f32, i32, i32, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class OracleExtractor:
    """Mirror of ORB_SLAM2::ORBextractor backed by the C oracle."""

    def __init__(self, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, semantics=0):
        self._L = lib()
        self.nfeatures, self.nlevels = nfeatures, nlevels
        self._h = self._L.oo_create(nfeatures, scale_factor, nlevels, ini_th, min_th)
        if not self._h:
            raise ValueError("bad extractor parameters")
        if self._L.oo_set_semantics(self._h, int(semantics)) != 0:
            raise ValueError(f"unknown semantics flags {semantics:#x}")
        self.semantics = int(semantics)

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.oo_destroy(self._h)
            self._h = None

    def tables(self):
        n = self.nlevels
        sf, isf, s2, is2 = (np.zeros(n, np.float32) for _ in range(4))
        fpl = np.zeros(n, np.int32)
        umax = np.zeros(16, np.int32)
        self._L.oo_scale_tables(self._h, _p(sf), _p(isf), _p(s2), _p(is2), _p(fpl), _p(umax))
        return dict(scale=sf, inv_scale=isf, sigma2=s2, inv_sigma2=is2, features_per_level=fpl,
                    umax=umax)

    def __call__(self, img: np.ndarray):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        cap = self.nfeatures + 64 * self.nlevels + 64
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = self._L.oo_extract(self._h, _p(img), img.shape[1], img.shape[0], img.strides[0],
                               _p(kps), _p(desc), cap)
        if n < 0:
            raise RuntimeError("oracle capacity exceeded")
        return kps[:n].copy(), desc[:n].copy()

    def level(self, level: int) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        self._L.oo_level_size(self._h, level, C.byref(w), C.byref(h))
        ptr = self._L.oo_level_image(self._h, level)
        return np.ctypeslib.as_array(ptr, shape=(h.value, w.value)).copy()

    def candidates(self, level: int):
        n = self._L.oo_level_candidates(self._h, level, None, None, 0)
        xy = np.zeros((max(n, 1), 2), np.float32)
        resp = np.zeros(max(n, 1), np.float32)
        self._L.oo_level_candidates(self._h, level, _p(xy), _p(resp), n)
        return xy[:n], resp[:n]


# ------------------------------------------------------------------------------------------------
# Frame / matcher mirrors
# ------------------------------------------------------------------------------------------------
class _OOFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p),
                ("minX", C.c_float), ("minY", C.c_float), ("maxX", C.c_float), ("maxY", C.c_float),
                ("gridInvW", C.c_float), ("gridInvH", C.c_float), ("scale_factors", C.c_void_p),
                ("nlevels", C.c_int), ("cell_start", C.c_void_p), ("cell_items", C.c_void_p)]


class OracleFrame:
    """Snapshot of the Frame fields the matchers read (mvKeysUn, mDescriptors, mvuRight, grid)."""

    def __init__(self, kps, desc, cols, rows, scale_factors, uright=None, bounds=None):
        """bounds: (minX, maxX, minY, maxY, invW, invH) of Frame::ComputeImageBounds; default = image rect."""
        L = lib()
        self.kps = np.ascontiguousarray(kps)
        self.desc = np.ascontiguousarray(desc, dtype=np.uint8)
        self.scale_factors = np.ascontiguousarray(scale_factors, dtype=np.float32)
        self.uright = None if uright is None else np.ascontiguousarray(uright, np.float32)
        self.cell_start = np.zeros(64 * 48 + 1, np.int32)
        self.cell_items = np.zeros(max(len(self.kps), 1), np.int32)
        vals = [C.c_float() for _ in range(6)]
        L.oo_grid_params(cols, rows, *[C.byref(v) for v in vals])
        self.bounds = [v.value for v in vals]  # minX, minY, maxX, maxY, invW, invH
        if bounds is not None:
            mnx, mxx, mny, mxy, iw, ih = bounds
            self.bounds = [mnx, mny, mxx, mxy, iw, ih]
        s = _OOFrame()
        s.n = len(self.kps)
        s.kps = _p(self.kps).value
        s.desc = _p(self.desc).value
        s.uright = None if self.uright is None else _p(self.uright).value
        s.minX, s.minY, s.maxX, s.maxY, s.gridInvW, s.gridInvH = self.bounds
        s.scale_factors = _p(self.scale_factors).value
        s.nlevels = len(self.scale_factors)
        s.cell_start = _p(self.cell_start).value
        s.cell_items = _p(self.cell_items).value
        self._s = s
        L.oo_grid_build(C.byref(s))

    def features_in_area(self, x, y, r, min_level=-1, max_level=-1):
        out = np.zeros(max(len(self.kps), 1), np.int32)
        n = lib().oo_features_in_area(C.byref(self._s), x, y, r, min_level, max_level, _p(out))
        return out[:n].copy()


def search_for_initialization(f1: OracleFrame, f2: OracleFrame, prev_xy, nnratio=0.9,
                              check_ori=True, window=100):
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.zeros(max(len(f1.kps), 1), np.int32)
    n = lib().oo_search_for_initialization(C.byref(f1._s), C.byref(f2._s), nnratio, int(check_ori),
                                           _p(prev), _p(m12), window)
    return n, m12[:len(f1.kps)].copy(), prev


class _OOMapPoints(C.Structure):
    _fields_ = [("m", C.c_int), ("track_in_view", C.c_void_p), ("is_bad", C.c_void_p),
                ("level", C.c_void_p), ("view_cos", C.c_void_p), ("proj_x", C.c_void_p),
                ("proj_y", C.c_void_p), ("proj_xr", C.c_void_p), ("n_obs", C.c_void_p),
                ("desc", C.c_void_p)]


def search_by_projection(f: OracleFrame, mp: dict, nnratio=0.8, th=3.0, owner=None, owner_obs=None):
    n = len(f.kps)
    owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
    owner_obs = (np.zeros(n, np.int32) if owner_obs is None
                 else np.ascontiguousarray(owner_obs, np.int32).copy())
    arrs = dict(track_in_view=np.ascontiguousarray(mp["track_in_view"], np.uint8),
                is_bad=np.ascontiguousarray(mp["is_bad"], np.uint8),
                level=np.ascontiguousarray(mp["level"], np.int32),
                view_cos=np.ascontiguousarray(mp["view_cos"], np.float32),
                proj_x=np.ascontiguousarray(mp["proj_x"], np.float32),
                proj_y=np.ascontiguousarray(mp["proj_y"], np.float32),
                proj_xr=np.ascontiguousarray(mp["proj_xr"], np.float32),
                n_obs=np.ascontiguousarray(mp["n_obs"], np.int32),
                desc=np.ascontiguousarray(mp["desc"], np.uint8))
    s = _OOMapPoints()
    s.m = len(arrs["level"])
    for k, v in arrs.items():
        setattr(s, k, _p(v).value)
    nm = lib().oo_search_by_projection(C.byref(f._s), C.byref(s), nnratio, th, _p(owner), _p(owner_obs))
    return nm, owner, owner_obs


class _OOCamera(C.Structure):
    _fields_ = [("Rcw", C.c_float * 9), ("tcw", C.c_float * 3), ("Ow", C.c_float * 3), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("mbf", C.c_float), ("mb", C.c_float),
                ("scale_factor", C.c_float), ("nlevels", C.c_int), ("minX", C.c_float), ("maxX", C.c_float),
                ("minY", C.c_float), ("maxY", C.c_float)]


def _camera(cam: dict) -> _OOCamera:
    """cam: Rcw (3x3), tcw (3), Ow (3), fx, fy, cx, cy, mbf, mb, scale_factor, nlevels, cols, rows."""
    c = _OOCamera()
    c.Rcw[:] = [float(v) for v in np.asarray(cam["Rcw"], np.float32).reshape(9)]
    c.tcw[:] = [float(v) for v in np.asarray(cam["tcw"], np.float32).reshape(3)]
    c.Ow[:] = [float(v) for v in np.asarray(cam.get("Ow", np.zeros(3)), np.float32).reshape(3)]
    for k in ("fx", "fy", "cx", "cy", "mbf", "mb", "scale_factor"):
        setattr(c, k, float(cam[k]))
    c.nlevels = int(cam["nlevels"])
    vals = [C.c_float() for _ in range(6)]
    lib().oo_grid_params(int(cam["cols"]), int(cam["rows"]), *[C.byref(v) for v in vals])
    c.minX, c.minY, c.maxX, c.maxY = vals[0].value, vals[1].value, vals[2].value, vals[3].value
    return c


class _OOMapPointGeom(C.Structure):
    _fields_ = [("m", C.c_int), ("pos", C.c_void_p), ("normal", C.c_void_p), ("max_dist", C.c_void_p),
                ("min_dist", C.c_void_p)]


def is_in_frustum(cam: dict, pos, normal, max_dist, min_dist, viewing_cos_limit=0.5):
    """Frame::isInFrustum + PredictScale for every point -> dict of the mTrack* SoA fields."""
    pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    normal = np.ascontiguousarray(normal, np.float32).reshape(-1, 3)
    mx = np.ascontiguousarray(max_dist, np.float32)
    mn = np.ascontiguousarray(min_dist, np.float32)
    m = len(pos)
    g = _OOMapPointGeom(m, _p(pos).value, _p(normal).value, _p(mx).value, _p(mn).value)
    out = dict(track_in_view=np.zeros(max(m, 1), np.uint8), proj_x=np.zeros(max(m, 1), np.float32),
               proj_y=np.zeros(max(m, 1), np.float32), proj_xr=np.zeros(max(m, 1), np.float32),
               level=np.zeros(max(m, 1), np.int32), view_cos=np.zeros(max(m, 1), np.float32))
    c = _camera(cam)
    n = lib().oo_is_in_frustum(C.byref(c), C.byref(g), viewing_cos_limit, _p(out["track_in_view"]),
                               _p(out["proj_x"]), _p(out["proj_y"]), _p(out["proj_xr"]), _p(out["level"]),
                               _p(out["view_cos"]))
    return n, {k: v[:m].copy() for k, v in out.items()}


class _OOLastFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("kps", C.c_void_p), ("has_mp", C.c_void_p), ("outlier", C.c_void_p),
                ("pos", C.c_void_p), ("n_obs", C.c_void_p), ("desc", C.c_void_p)]


def search_by_projection_last(f: OracleFrame, cur: dict, last: dict, lf: dict, th=7.0, mono=True, check_ori=True,
                              owner=None, owner_obs=None):
    """SearchByProjection(CurrentFrame, LastFrame, th, bMono).  lf: kps, has_mp, outlier, pos, n_obs, desc."""
    n = len(f.kps)
    owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
    owner_obs = (np.zeros(n, np.int32) if owner_obs is None
                 else np.ascontiguousarray(owner_obs, np.int32).copy())
    arrs = dict(kps=np.ascontiguousarray(lf["kps"]), has_mp=np.ascontiguousarray(lf["has_mp"], np.uint8),
                outlier=np.ascontiguousarray(lf["outlier"], np.uint8),
                pos=np.ascontiguousarray(lf["pos"], np.float32).reshape(-1, 3),
                n_obs=np.ascontiguousarray(lf["n_obs"], np.int32),
                desc=np.ascontiguousarray(lf["desc"], np.uint8))
    s = _OOLastFrame()
    s.n = len(arrs["kps"])
    for k, v in arrs.items():
        setattr(s, k, _p(v).value if v.size else None)
    cc, cl = _camera(cur), _camera(last)
    nm = lib().oo_search_by_projection_last(C.byref(f._s), C.byref(cc), C.byref(cl), C.byref(s), th, int(mono),
                                            int(check_ori), _p(owner) if n else None,
                                            _p(owner_obs) if n else None)
    return nm, owner, owner_obs


class _OOKeyFrame(C.Structure):
    _fields_ = [("n", C.c_int), ("kps", C.c_void_p), ("valid", C.c_void_p), ("pos", C.c_void_p),
                ("max_dist", C.c_void_p), ("min_dist", C.c_void_p), ("desc", C.c_void_p)]


def search_by_projection_kf(f: OracleFrame, cur: dict, kf: dict, th=10.0, orbdist=100, check_ori=True, owner=None):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist).  kf: kps, valid, pos, max_dist,
    min_dist, desc.  Returns (nmatches, owner)."""
    n = len(f.kps)
    owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
    arrs = dict(kps=np.ascontiguousarray(kf["kps"]), valid=np.ascontiguousarray(kf["valid"], np.uint8),
                pos=np.ascontiguousarray(kf["pos"], np.float32).reshape(-1, 3),
                max_dist=np.ascontiguousarray(kf["max_dist"], np.float32),
                min_dist=np.ascontiguousarray(kf["min_dist"], np.float32),
                desc=np.ascontiguousarray(kf["desc"], np.uint8))
    s = _OOKeyFrame()
    s.n = len(arrs["kps"])
    for k, v in arrs.items():
        setattr(s, k, _p(v).value if v.size else None)
    c = _camera(cur)
    nm = lib().oo_search_by_projection_kf(C.byref(f._s), C.byref(c), C.byref(s), th, int(orbdist), int(check_ori),
                                          _p(owner) if n else None)
    return nm, owner


def kf_predicted_levels(cur: dict, kf: dict):
    """Per keyframe point the relocalisation matcher's predicted level, -1 outside the scale range or invalid
    (oo_kf_predicted_levels; what a drop-in binding computes with MapPoint::PredictScale)."""
    arrs = dict(kps=np.ascontiguousarray(kf["kps"]), valid=np.ascontiguousarray(kf["valid"], np.uint8),
                pos=np.ascontiguousarray(kf["pos"], np.float32).reshape(-1, 3),
                max_dist=np.ascontiguousarray(kf["max_dist"], np.float32),
                min_dist=np.ascontiguousarray(kf["min_dist"], np.float32),
                desc=np.ascontiguousarray(kf["desc"], np.uint8))
    s = _OOKeyFrame()
    s.n = len(arrs["kps"])
    for k, v in arrs.items():
        setattr(s, k, _p(v).value if v.size else None)
    out = np.zeros(max(s.n, 1), np.int32)
    lib().oo_kf_predicted_levels(C.byref(_camera(cur)), C.byref(s), _p(out))
    return out[:s.n]


def depth_u16_to_f32(depth_u16, factor):
    src = np.ascontiguousarray(depth_u16, np.uint16)
    out = np.zeros(src.shape, np.float32)
    lib().oo_depth_u16_to_f32(_p(src), src.size, factor, _p(out))
    return out


# cv::cvtColor codes (OpenCV's values) -> (channels, index of blue)
COLOR_CODES = {6: (3, 0), 7: (3, 2), 10: (4, 0), 11: (4, 2)}


def cvt_gray(img, code):
    """cvtColor(img, gray, code) for 8U BGR/RGB/BGRA/RGBA (Tracking::GrabImage*, src/Tracking.cc:169-255)."""
    cn, bidx = COLOR_CODES[code]
    src = np.ascontiguousarray(img, np.uint8)
    assert src.ndim == 3 and src.shape[2] == cn
    rows, cols = src.shape[:2]
    out = np.zeros((rows, cols), np.uint8)
    lib().oo_cvt_gray(_p(src), cols, rows, cols * cn, cn, bidx, _p(out), cols)
    return out


def stereo_from_rgbd(kps, kps_un, depth_f32, mbf):
    """Frame::ComputeStereoFromRGBD -> (uright, depth)."""
    kps = np.ascontiguousarray(kps)
    kps_un = np.ascontiguousarray(kps_un)
    dep = np.ascontiguousarray(depth_f32, np.float32)
    n = len(kps)
    ur = np.zeros(max(n, 1), np.float32)
    de = np.zeros(max(n, 1), np.float32)
    lib().oo_stereo_from_rgbd(_p(kps), _p(kps_un), n, _p(dep), dep.shape[1], mbf, _p(ur), _p(de))
    return ur[:n].copy(), de[:n].copy()


class OracleVocabulary:
    """DBoW2 TemplatedVocabulary<FORB> (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) restated in C."""

    def __init__(self, voc: dict = None, path: str = None):
        L = lib()
        if path is not None:
            self._h = L.oo_vocab_load_text(path.encode())
        else:
            par = np.ascontiguousarray(voc["parent"], np.int32)
            leaf = np.ascontiguousarray(voc["is_leaf"], np.uint8)
            desc = np.ascontiguousarray(voc["desc"], np.uint8)
            w = np.ascontiguousarray(voc["weight"], np.float64)
            self._h = L.oo_vocab_from_arrays(voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(par), _p(par),
                                             _p(leaf), _p(desc), _p(w))
        if not self._h:
            raise ValueError("vocabulary rejected")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oo_vocab_free(self._h)
            self._h = None

    def transform(self, desc, levelsup=4):
        """-> (BowVector {word: value} as (words, values) ascending, FeatureVector as (nodes, offsets, features))."""
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(desc)
        words = np.zeros(max(n, 1), np.int32)
        values = np.zeros(max(n, 1), np.float64)
        nodes = np.zeros(max(n, 1), np.int32)
        off = np.zeros(n + 1, np.int32)
        feats = np.zeros(max(n, 1), np.int32)
        nw, nn = C.c_int(0), C.c_int(0)
        lib().oo_bow_transform(self._h, _p(desc), n, levelsup, _p(words), _p(values), C.byref(nw), _p(nodes), _p(off),
                               _p(feats), C.byref(nn))
        m = int(off[nn.value]) if nn.value else 0
        return ((words[:nw.value].copy(), values[:nw.value].copy()),
                (nodes[:nn.value].copy(), off[:nn.value + 1].copy(), feats[:m].copy()))


def undistort_keypoints(K4, dist, kps):
    """Frame::UndistortKeyPoints -> mvKeysUn (copy of kps with undistorted pt)."""
    K4 = np.ascontiguousarray(K4, np.float32)
    dist = np.ascontiguousarray(dist, np.float32)
    kps = np.ascontiguousarray(kps)
    out = kps.copy()
    lib().oo_undistort_keypoints(_p(K4), _p(dist), len(dist), _p(kps), _p(out), len(kps))
    return out


def compute_image_bounds(K4, dist, cols, rows):
    """Frame::ComputeImageBounds + grid scales -> (minX, maxX, minY, maxY, invW, invH)."""
    K4 = np.ascontiguousarray(K4, np.float32)
    dist = np.ascontiguousarray(dist, np.float32)
    v = [C.c_float() for _ in range(6)]
    lib().oo_compute_image_bounds(_p(K4), _p(dist), len(dist), cols, rows, *[C.byref(x) for x in v])
    return tuple(x.value for x in v)


def distribute_octree(xy, resp, minX, maxX, minY, maxY, N):
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    resp = np.ascontiguousarray(resp, np.float32)
    cap = max(len(resp), N + 3, 64) + 64
    oxy = np.zeros((cap, 2), np.float32)
    orr = np.zeros(cap, np.float32)
    m = lib().oo_distribute_octree(_p(xy), _p(resp), len(resp), minX, maxX, minY, maxY, N, _p(oxy), _p(orr))
    return oxy[:m].copy(), orr[:m].copy()


def stereo_matches(exL: "OracleExtractor", exR: "OracleExtractor", kL, dL, kR, dR, mbf, mb):
    """Frame::ComputeStereoMatches on the two extractors' last pyramids -> (n, uright, depth)."""
    kL = np.ascontiguousarray(kL)
    kR = np.ascontiguousarray(kR)
    dL = np.ascontiguousarray(dL, np.uint8)
    dR = np.ascontiguousarray(dR, np.uint8)
    ur = np.zeros(max(len(kL), 1), np.float32)
    de = np.zeros(max(len(kL), 1), np.float32)
    n = lib().oo_stereo_matches(exL._h, exR._h, _p(kL), _p(dL), len(kL), _p(kR), _p(dR), len(kR), mbf, mb,
                                _p(ur), _p(de))
    return n, ur[:len(kL)].copy(), de[:len(kL)].copy()


def descriptor_distance(a, b) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oo_descriptor_distance(_p(a), _p(b))


def resize_linear(src: np.ndarray, dw: int, dh: int, semantics: int = 0) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().oo_resize_linear(_p(src), src.shape[1], src.shape[0], _p(dst), dw, dh, int(semantics))
    return dst


def gaussian7(src: np.ndarray, semantics: int = 0) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    lib().oo_gaussian7(_p(src), src.shape[1], src.shape[0], _p(dst), int(semantics))
    return dst


def fast_score(img: np.ndarray, x: int, y: int) -> int:
    img = np.ascontiguousarray(img, np.uint8)
    return lib().oo_fast_score(_p(img), img.strides[0], x, y)


def harris_response(img: np.ndarray, x: int, y: int) -> float:
    """OpenCV ORB HARRIS_SCORE response at (x, y) (oracle/orb_oracle.c oo_harris_response; option, parity unpinned)."""
    img = np.ascontiguousarray(img, np.uint8)
    if not (4 <= x < img.shape[1] - 4 and 4 <= y < img.shape[0] - 4):
        raise ValueError("the 9x9 window must lie inside the image")
    return float(lib().oo_harris_response(_p(img), img.strides[0], x, y))


def harris_key(r: float) -> int:
    """The device's order-preserving u32 image of a float response (include/orbgpu.h, orbgpu_debug_octree)."""
    u = int(np.array([r], np.float32).view(np.uint32)[0])
    if u == 0x80000000:
        return 0x80000000
    return (~u & 0xffffffff) if u & 0x80000000 else (u | 0x80000000)


def fastatan2(y: float, x: float) -> float:
    return lib().oo_fastatan2(y, x)


def sincos(a: float):
    s, c = C.c_float(), C.c_float()
    lib().oo_sincos(a, C.byref(s), C.byref(c))
    return s.value, c.value
