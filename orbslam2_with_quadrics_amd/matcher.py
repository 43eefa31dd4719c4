"""Python mirror of ORB_SLAM2::ORBmatcher (include/ORBmatcher.h:37-102) and of the Frame fields the
per-frame matchers read (src/Frame.cc), over the gfx950 C ABI."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .extractor import KP_DTYPE, ORBextractor

FRAME_GRID_COLS, FRAME_GRID_ROWS = 64, 48  # include/Frame.h:39-40


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Frame:
    """The subset of ORB_SLAM2::Frame the hot path produces and the matchers consume: mvKeysUn (no
    distortion -> == mvKeys), mDescriptors, mvuRight, mvScaleFactors and the image bounds/grid scales."""

    def __init__(self, keypoints, descriptors, cols: int, rows: int, scale_factors, uright=None, keys_un=None,
                 grid=None):
        self.mvKeys = np.ascontiguousarray(keypoints, dtype=KP_DTYPE)
        self.mvKeysUn = self.mvKeys if keys_un is None else np.ascontiguousarray(keys_un, dtype=KP_DTYPE)
        self.mDescriptors = np.ascontiguousarray(descriptors, dtype=np.uint8)
        self.mvScaleFactors = np.ascontiguousarray(scale_factors, dtype=np.float32)
        self.N = len(self.mvKeysUn)
        self.mvuRight = None if uright is None else np.ascontiguousarray(uright, np.float32)
        if grid is None:  # no distortion: the image rectangle (Frame::ComputeImageBounds, k1 == 0)
            grid = _lib.GridGeom()
            _lib.check(None, _lib.lib().orbgpu_grid_geom_for_image(cols, rows, C.byref(grid)), "grid_geom")
        self.grid = grid

    @classmethod
    def from_image(cls, extractor: ORBextractor, image: np.ndarray, K4=None, dist=None):
        """Monocular Frame constructor (src/Frame.cc:161-210): extract, UndistortKeyPoints, image bounds."""
        k, d = extractor(image)
        if K4 is None or dist is None:
            return cls(k, d, image.shape[1], image.shape[0], extractor.GetScaleFactors())
        ku = UndistortKeyPoints(extractor, K4, dist, k)
        g = ComputeImageBounds(extractor, K4, dist, image.shape[1], image.shape[0])
        return cls(k, d, image.shape[1], image.shape[0], extractor.GetScaleFactors(), keys_un=ku, grid=g)

    @classmethod
    def from_stereo(cls, ex_left: ORBextractor, ex_right: ORBextractor, im_left: np.ndarray,
                    im_right: np.ndarray, mbf: float, mb: float):
        """Stereo Frame constructor (src/Frame.cc:52-105, no distortion): extract both images, then
        ComputeStereoMatches fills mvuRight / mvDepth."""
        k, d = ex_left(im_left)
        kr, dr = ex_right(im_right)
        f = cls(k, d, im_left.shape[1], im_left.shape[0], ex_left.GetScaleFactors())
        f.mvKeysRight, f.mDescriptorsRight = kr, dr
        f.mbf, f.mb = float(mbf), float(mb)
        f.mvuRight, f.mvDepth, f.nStereo = ComputeStereoMatches(ex_left, ex_right, mbf, mb)
        return f

    def view(self) -> _lib.FrameView:
        v = _lib.FrameView()
        v.n = self.N
        v.kps = _p(self.mvKeysUn).value if self.N else None
        v.desc = _p(self.mDescriptors).value if self.N else None
        v.uright = None if self.mvuRight is None else _p(self.mvuRight).value
        v.grid = self.grid
        v.scale_factors = _p(self.mvScaleFactors).value
        v.nlevels = len(self.mvScaleFactors)
        return v


class ORBmatcher:
    TH_LOW, TH_HIGH, HISTO_LENGTH = 50, 100, 30  # src/ORBmatcher.cc:37-39

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, context: ORBextractor | None = None,
                 device: int = 0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        # HIP stream + scratch come from an extractor context (any will do)
        self._own = context is None
        self._ex = context if context is not None else ORBextractor(1000, 1.2, 8, 20, 7, device=device)

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return _lib.lib().orbgpu_descriptor_distance(_p(a), _p(b))

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray, windowSize: int = 10):
        """Returns (nmatches, vnMatches12); vbPrevMatched (N1 x 2 float32) is updated in place."""
        assert vbPrevMatched.dtype == np.float32 and vbPrevMatched.flags.c_contiguous
        assert vbPrevMatched.shape == (F1.N, 2)
        m12 = np.full(max(F1.N, 1), -1, np.int32)
        nm = C.c_int(0)
        v1, v2 = F1.view(), F2.view()
        ctx = self._ex.ctx
        rc = _lib.lib().orbgpu_search_for_initialization(ctx, C.byref(v1), C.byref(v2), self.mfNNratio,
                                                         int(self.mbCheckOrientation), _p(vbPrevMatched),
                                                         _p(m12), windowSize, C.byref(nm))
        _lib.check(ctx, rc, "orbgpu_search_for_initialization")
        return nm.value, m12[:F1.N].copy()

    def SearchByProjection(self, F: Frame, mappoints: dict, th: float = 3.0, owner=None, owner_obs=None):
        """mappoints: dict of SoA arrays (track_in_view, is_bad, level, view_cos, proj_x, proj_y,
        proj_xr, n_obs, desc).  owner/owner_obs mirror F.mvpMapPoints.  Returns (nmatches, owner,
        owner_obs)."""
        n = F.N
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        owner_obs = (np.zeros(n, np.int32) if owner_obs is None
                     else np.ascontiguousarray(owner_obs, np.int32).copy())
        arrs = dict(track_in_view=np.ascontiguousarray(mappoints["track_in_view"], np.uint8),
                    is_bad=np.ascontiguousarray(mappoints["is_bad"], np.uint8),
                    level=np.ascontiguousarray(mappoints["level"], np.int32),
                    view_cos=np.ascontiguousarray(mappoints["view_cos"], np.float32),
                    proj_x=np.ascontiguousarray(mappoints["proj_x"], np.float32),
                    proj_y=np.ascontiguousarray(mappoints["proj_y"], np.float32),
                    proj_xr=np.ascontiguousarray(mappoints["proj_xr"], np.float32),
                    n_obs=np.ascontiguousarray(mappoints["n_obs"], np.int32),
                    desc=np.ascontiguousarray(mappoints["desc"], np.uint8))
        mv = _lib.MapPointsView()
        mv.m = len(arrs["level"])
        for k, v in arrs.items():
            setattr(mv, k, _p(v).value if v.size else None)
        fv = F.view()
        nm = C.c_int(0)
        ctx = self._ex.ctx
        rc = _lib.lib().orbgpu_search_by_projection(ctx, C.byref(fv), C.byref(mv), self.mfNNratio, th,
                                                    _p(owner) if n else None, _p(owner_obs) if n else None,
                                                    C.byref(nm))
        _lib.check(ctx, rc, "orbgpu_search_by_projection")
        return nm.value, owner, owner_obs

    def IsInFrustum(self, F: Frame, cam: dict, geom: dict, viewingCosLimit: float = 0.5):
        """Frame::isInFrustum (src/Frame.cc:269-325) + PredictScale for every map point of `geom` (pos, normal,
        max_dist, min_dist).  Returns (n_in_view, dict of the mTrack* fields as SearchByProjection inputs)."""
        pos = np.ascontiguousarray(geom["pos"], np.float32).reshape(-1, 3)
        nrm = np.ascontiguousarray(geom["normal"], np.float32).reshape(-1, 3)
        mx = np.ascontiguousarray(geom["max_dist"], np.float32)
        mn = np.ascontiguousarray(geom["min_dist"], np.float32)
        m = len(pos)
        v = _lib.MapPointGeomView(m, _p(pos).value if m else None, _p(nrm).value if m else None,
                                  _p(mx).value if m else None, _p(mn).value if m else None)
        out = dict(track_in_view=np.zeros(max(m, 1), np.uint8), proj_x=np.zeros(max(m, 1), np.float32),
                   proj_y=np.zeros(max(m, 1), np.float32), proj_xr=np.zeros(max(m, 1), np.float32),
                   level=np.zeros(max(m, 1), np.int32), view_cos=np.zeros(max(m, 1), np.float32))
        nin = C.c_int(0)
        c = camera_struct(cam)
        ctx = self._ex.ctx
        rc = _lib.lib().orbgpu_is_in_frustum(ctx, C.byref(c), F.grid, C.byref(v), float(viewingCosLimit),
                                             _p(out["track_in_view"]), _p(out["proj_x"]), _p(out["proj_y"]),
                                             _p(out["proj_xr"]), _p(out["level"]), _p(out["view_cos"]), C.byref(nin))
        _lib.check(ctx, rc, "orbgpu_is_in_frustum")
        return nin.value, {k: a[:m].copy() for k, a in out.items()}


    def SearchByProjectionKeyFrame(self, CurrentFrame: Frame, cur: dict, KF: dict, th: float, ORBdist: int,
                                   owner=None, pred_level=None):
        """ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
        th, ORBdist) (src/ORBmatcher.cc:1472-1599).  KF: dict of kps, valid, pos, max_dist, min_dist, desc.
        pred_level (optional, KF.n ints): the caller's PredictScale per point, -1 outside the scale range
        (orbgpu_search_by_projection_keyframe_levels: max_dist / min_dist are then not read).
        Returns (nmatches, owner) -- owner = keyframe map-point index per keypoint, -1 = NULL."""
        n = CurrentFrame.N
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        arrs = dict(kps=np.ascontiguousarray(KF["kps"], KP_DTYPE), valid=np.ascontiguousarray(KF["valid"], np.uint8),
                    pos=np.ascontiguousarray(KF["pos"], np.float32).reshape(-1, 3),
                    max_dist=np.ascontiguousarray(KF["max_dist"], np.float32),
                    min_dist=np.ascontiguousarray(KF["min_dist"], np.float32),
                    desc=np.ascontiguousarray(KF["desc"], np.uint8))
        kv = _lib.KeyFrameView()
        kv.n = len(arrs["kps"])
        for k, a in arrs.items():
            setattr(kv, k, _p(a).value if a.size else None)
        fv = CurrentFrame.view()
        cc = camera_struct(cur)
        nm = C.c_int(0)
        ctx = self._ex.ctx
        if pred_level is None:
            rc = _lib.lib().orbgpu_search_by_projection_keyframe(ctx, C.byref(fv), C.byref(cc), C.byref(kv),
                                                                 float(th), int(ORBdist), int(self.mbCheckOrientation),
                                                                 _p(owner) if n else None, C.byref(nm))
        else:
            lv = np.ascontiguousarray(pred_level, np.int32)
            rc = _lib.lib().orbgpu_search_by_projection_keyframe_levels(
                ctx, C.byref(fv), C.byref(cc), C.byref(kv), _p(lv) if lv.size else None, float(th), int(ORBdist),
                int(self.mbCheckOrientation), _p(owner) if n else None, C.byref(nm))
        _lib.check(ctx, rc, "orbgpu_search_by_projection_keyframe")
        return nm.value, owner

    def SearchByProjectionLastFrame(self, CurrentFrame: Frame, cur: dict, LastFrame: dict, last: dict, th: float,
                                   bMono: bool, owner=None, owner_obs=None):
        """ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
        (src/ORBmatcher.cc:1328-1470).  LastFrame: dict of kps, has_mp, outlier, pos, n_obs, desc; cur/last: the
        two frames' pose dicts.  Returns (nmatches, owner, owner_obs) -- owner = LastFrame keypoint index."""
        n = CurrentFrame.N
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        owner_obs = (np.zeros(n, np.int32) if owner_obs is None
                     else np.ascontiguousarray(owner_obs, np.int32).copy())
        arrs = dict(kps=np.ascontiguousarray(LastFrame["kps"], KP_DTYPE),
                    has_mp=np.ascontiguousarray(LastFrame["has_mp"], np.uint8),
                    outlier=np.ascontiguousarray(LastFrame["outlier"], np.uint8),
                    pos=np.ascontiguousarray(LastFrame["pos"], np.float32).reshape(-1, 3),
                    n_obs=np.ascontiguousarray(LastFrame["n_obs"], np.int32),
                    desc=np.ascontiguousarray(LastFrame["desc"], np.uint8))
        lv = _lib.LastFrameView()
        lv.n = len(arrs["kps"])
        for k, a in arrs.items():
            setattr(lv, k, _p(a).value if a.size else None)
        fv = CurrentFrame.view()
        cc, cl = camera_struct(cur), camera_struct(last)
        nm = C.c_int(0)
        ctx = self._ex.ctx
        rc = _lib.lib().orbgpu_search_by_projection_last_frame(ctx, C.byref(fv), C.byref(cc), C.byref(cl), C.byref(lv),
                                                               float(th), int(bMono), int(self.mbCheckOrientation),
                                                               _p(owner) if n else None, _p(owner_obs) if n else None,
                                                               C.byref(nm))
        _lib.check(ctx, rc, "orbgpu_search_by_projection_last_frame")
        return nm.value, owner, owner_obs


def ComputeStereoMatches(ex_left: ORBextractor, ex_right: ORBextractor, mbf: float, mb: float):
    """Frame::ComputeStereoMatches (src/Frame.cc:466-640) on the last frame each extractor processed.
    Returns (mvuRight, mvDepth, nmatches): float32 arrays over the left keypoints, -1 where unmatched."""
    L = _lib.lib()
    n, nm = C.c_int(0), C.c_int(0)
    cap = L.orbgpu_max_keypoints(ex_left.ctx)
    ur = np.empty(max(cap, 1), np.float32)
    de = np.empty(max(cap, 1), np.float32)
    rc = L.orbgpu_compute_stereo_matches(ex_left.ctx, ex_right.ctx, float(mbf), float(mb), _p(ur), _p(de), cap,
                                         C.byref(n), C.byref(nm))
    _lib.check(ex_left.ctx, rc, "orbgpu_compute_stereo_matches")
    return ur[:n.value].copy(), de[:n.value].copy(), nm.value


def camera_struct(cam: dict) -> _lib.Camera:
    """orbgpu_camera from a pose/intrinsics dict (synthetic.camera layout: Rcw, tcw, Ow, fx, fy, cx, cy, mbf,
    mb, scale_factor, nlevels)."""
    c = _lib.Camera()
    c.Rcw[:] = [float(v) for v in np.asarray(cam["Rcw"], np.float32).reshape(9)]
    c.tcw[:] = [float(v) for v in np.asarray(cam["tcw"], np.float32).reshape(3)]
    c.Ow[:] = [float(v) for v in np.asarray(cam["Ow"], np.float32).reshape(3)]
    for k in ("fx", "fy", "cx", "cy", "mbf", "mb", "scale_factor"):
        setattr(c, k, float(np.float32(cam[k])))
    c.nlevels = int(cam["nlevels"])
    return c



def UndistortKeyPoints(extractor: ORBextractor, K4, dist, keypoints):
    """Frame::UndistortKeyPoints (src/Frame.cc:404-434) on the GPU -> mvKeysUn."""
    K4 = np.ascontiguousarray(K4, np.float32)
    dist = np.ascontiguousarray(dist, np.float32)
    kin = np.ascontiguousarray(keypoints, KP_DTYPE)
    out = np.empty_like(kin)
    n = len(kin)
    rc = _lib.lib().orbgpu_undistort_keypoints(extractor.ctx, _p(K4), _p(dist) if dist.size else None, int(dist.size),
                                               _p(kin) if n else None, _p(out) if n else None, n)
    _lib.check(extractor.ctx, rc, "orbgpu_undistort_keypoints")
    return out


def ComputeImageBounds(extractor: ORBextractor, K4, dist, cols: int, rows: int) -> _lib.GridGeom:
    """Frame::ComputeImageBounds (src/Frame.cc:436-461) + grid scales, on the GPU."""
    K4 = np.ascontiguousarray(K4, np.float32)
    dist = np.ascontiguousarray(dist, np.float32)
    g = _lib.GridGeom()
    rc = _lib.lib().orbgpu_compute_image_bounds(extractor.ctx, _p(K4), _p(dist) if dist.size else None,
                                                int(dist.size), cols, rows, C.byref(g))
    _lib.check(extractor.ctx, rc, "orbgpu_compute_image_bounds")
    return g


def ComputeStereoFromRGBD(extractor: ORBextractor, depth: np.ndarray, mbf: float, depth_map_factor: float = 1.0):
    """Frame::ComputeStereoFromRGBD (src/Frame.cc:643-664) for the frame `extractor` processed last.
    depth: float32 map (as Frame receives it) or the raw uint16 image, scaled by mDepthMapFactor =
    1/DepthMapFactor as Tracking::GrabImageRGBD does (src/Tracking.cc:227-228).  Returns (mvuRight, mvDepth)."""
    is_u16 = depth.dtype == np.uint16
    dep = np.ascontiguousarray(depth, np.uint16 if is_u16 else np.float32)
    L = _lib.lib()
    cap = L.orbgpu_max_keypoints(extractor.ctx)
    ur = np.empty(max(cap, 1), np.float32)
    de = np.empty(max(cap, 1), np.float32)
    n = C.c_int(0)
    rc = L.orbgpu_compute_stereo_from_rgbd(extractor.ctx, _p(dep), int(is_u16), float(depth_map_factor),
                                           dep.strides[0], float(mbf), _p(ur), _p(de), cap, C.byref(n))
    _lib.check(extractor.ctx, rc, "orbgpu_compute_stereo_from_rgbd")
    return ur[:n.value].copy(), de[:n.value].copy()
