"""Python mirror of ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111) over the gfx950 C ABI.

Same constructor arguments, getters and call semantics as the reference class; the call returns
(keypoints, descriptors) instead of filling OpenCV output arguments.  Keypoints are a numpy structured
array with cv::KeyPoint's 28-byte layout.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class ORBextractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) on HIP device `device`."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 device: int = 0, semantics: int | None = None):
        self._L = _lib.lib()
        self._ctx = self._L.orbgpu_create(device, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        if not self._ctx:
            raise RuntimeError("orbgpu_create failed (no HIP device visible, or invalid parameters)")
        self.nfeatures, self.nlevels = nfeatures, nlevels
        # None: the context's own choice (SEM_DEFAULT)
        self.set_semantics(self._L.orbgpu_get_semantics(self._ctx) if semantics is None else semantics)

    def set_semantics(self, flags: int):
        """OpenCV/compiler behaviours to reproduce (_lib.SEM_*, include/orbgpu.h ORBGPU_SEM_*)."""
        _lib.check(self._ctx, self._L.orbgpu_set_semantics(self._ctx, int(flags)), "orbgpu_set_semantics")
        self.semantics = int(flags)

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.orbgpu_destroy(self._ctx)
            self._ctx = None

    __del__ = close

    @property
    def ctx(self):
        return self._ctx

    # ---- getters, include/ORBextractor.h:63-83
    def GetLevels(self) -> int:
        return self._L.orbgpu_get_levels(self._ctx)

    def GetScaleFactor(self) -> float:
        return self._L.orbgpu_get_scale_factor(self._ctx)

    def _vec(self, fn):
        out = np.zeros(self.nlevels, np.float32)
        _lib.check(self._ctx, fn(self._ctx, _p(out)), fn.__name__)
        return out

    def GetScaleFactors(self):
        return self._vec(self._L.orbgpu_get_scale_factors)

    def GetInverseScaleFactors(self):
        return self._vec(self._L.orbgpu_get_inverse_scale_factors)

    def GetScaleSigmaSquares(self):
        return self._vec(self._L.orbgpu_get_scale_sigma_squares)

    def GetInverseScaleSigmaSquares(self):
        return self._vec(self._L.orbgpu_get_inverse_scale_sigma_squares)

    def features_per_level(self):
        out = np.zeros(self.nlevels, np.int32)
        _lib.check(self._ctx, self._L.orbgpu_get_features_per_level(self._ctx, _p(out)), "features_per_level")
        return out

    # ---- ORBextractor::operator(), src/ORBextractor.cc:1043-1105
    def __call__(self, image: np.ndarray, mask=None):
        """Returns (keypoints, descriptors); (None, None) for an empty image (outputs untouched in the
        reference)."""
        if image is None or image.size == 0:
            return None, None
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise AssertionError("image.type() == CV_8UC1")  # src/ORBextractor.cc:1050
        if img.strides[1] != 1:
            img = np.ascontiguousarray(img)
        cap = self._L.orbgpu_max_keypoints(self._ctx)
        for _ in range(2):
            kps = np.zeros(max(cap, 1), KP_DTYPE)
            desc = np.zeros((max(cap, 1), 32), np.uint8)
            n = C.c_int(0)
            rc = self._L.orbgpu_extract(self._ctx, _p(img), img.shape[1], img.shape[0], img.strides[0],
                                        _p(kps), _p(desc), cap, C.byref(n))
            if rc == _lib.ERR_CAPACITY:
                cap = n.value
                continue
            _lib.check(self._ctx, rc, "orbgpu_extract")
            return kps[:n.value].copy(), desc[:n.value].copy()
        raise RuntimeError("orbgpu_extract: capacity negotiation failed")

    # ---- Tracking::GrabImage* colour conversion + Frame::ExtractORB (src/Tracking.cc:169-255)
    def extract_color(self, image: np.ndarray, code: int):
        """cvtColor(image, gray, code) on the GPU followed by operator() on the gray image (code: one of
        _lib.COLOR_*; image: rows x cols x 3 or 4, uint8).  Returns (keypoints, descriptors) as __call__."""
        if image is None or image.size == 0:
            return None, None
        img = np.asarray(image)
        cn = _lib.COLOR_CHANNELS.get(code)
        if cn is None or img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != cn:
            raise ValueError(f"extract_color: code {code} needs a rows x cols x {cn} uint8 image")
        if img.strides[2] != 1 or img.strides[1] != cn:
            img = np.ascontiguousarray(img)
        cap = self._L.orbgpu_max_keypoints(self._ctx)
        for _ in range(2):
            kps = np.zeros(max(cap, 1), KP_DTYPE)
            desc = np.zeros((max(cap, 1), 32), np.uint8)
            n = C.c_int(0)
            rc = self._L.orbgpu_extract_color(self._ctx, _p(img), img.shape[1], img.shape[0], img.strides[0], code,
                                              _p(kps), _p(desc), cap, C.byref(n))
            if rc == _lib.ERR_CAPACITY:
                cap = n.value
                continue
            _lib.check(self._ctx, rc, "orbgpu_extract_color")
            return kps[:n.value].copy(), desc[:n.value].copy()
        raise RuntimeError("orbgpu_extract_color: capacity negotiation failed")

    def cvt_color_to_gray_batch(self, d_src: int, B: int, cols: int, rows: int, src_pitch: int,
                                src_frame_stride: int, code: int, d_dst: int, dst_pitch: int, dst_frame_stride: int):
        """Device-resident batched cvtColor(..., code) on the context's stream (orbgpu_cvt_color_to_gray_batch)."""
        _lib.check(self._ctx, self._L.orbgpu_cvt_color_to_gray_batch(
            self._ctx, C.c_void_p(d_src), B, cols, rows, src_pitch, src_frame_stride, code, C.c_void_p(d_dst),
            dst_pitch, dst_frame_stride), "orbgpu_cvt_color_to_gray_batch")

    # ---- mvImagePyramid (public member, include/ORBextractor.h:85)
    def level(self, level: int) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        _lib.check(self._ctx, self._L.orbgpu_get_level(self._ctx, level, None, 0, C.byref(w), C.byref(h)),
                   "orbgpu_get_level")
        out = np.zeros((h.value, w.value), np.uint8)
        _lib.check(self._ctx, self._L.orbgpu_get_level(self._ctx, level, _p(out), w.value, C.byref(w),
                                                        C.byref(h)), "orbgpu_get_level")
        return out

    @property
    def mvImagePyramid(self):
        return [self.level(l) for l in range(self.nlevels)]

    # ---- batch / device-resident path
    def extract_batch_device(self, d_imgs: int, B: int, cols: int, rows: int, pitch: int, frame_stride: int):
        _lib.check(self._ctx, self._L.orbgpu_extract_batch_device(self._ctx, C.c_void_p(d_imgs), B, cols, rows,
                                                                   pitch, frame_stride),
                   "orbgpu_extract_batch_device")

    def batch_outputs(self):
        kp, de, cn = C.c_void_p(), C.c_void_p(), C.c_void_p()
        cap = C.c_int()
        _lib.check(self._ctx, self._L.orbgpu_batch_outputs(self._ctx, C.byref(kp), C.byref(de), C.byref(cn),
                                                            C.byref(cap)), "orbgpu_batch_outputs")
        return kp.value, de.value, cn.value, cap.value

    def set_undistortion(self, K4, dist):
        """Device-resident Frame::UndistortKeyPoints for the coming batches (mvKeysUn + undistorted grid)."""
        K4 = np.ascontiguousarray(K4, np.float32)
        dist = np.ascontiguousarray(dist, np.float32)
        _lib.check(self._ctx, self._L.orbgpu_set_undistortion(self._ctx, _p(K4), _p(dist) if dist.size else None,
                                                                int(dist.size)), "orbgpu_set_undistortion")

    def batch_outputs_undistorted(self):
        """(device pointer of mvKeysUn, GridGeom bounds) of the last batch."""
        kp = C.c_void_p()
        g = _lib.GridGeom()
        _lib.check(self._ctx, self._L.orbgpu_batch_outputs_undistorted(self._ctx, C.byref(kp), C.byref(g)),
                   "orbgpu_batch_outputs_undistorted")
        return kp.value, g

    def batch_download(self, b: int):
        cap = self._L.orbgpu_max_keypoints(self._ctx)
        kps = np.zeros(max(cap, 1), KP_DTYPE)
        desc = np.zeros((max(cap, 1), 32), np.uint8)
        n = C.c_int(0)
        _lib.check(self._ctx, self._L.orbgpu_batch_download(self._ctx, b, _p(kps), _p(desc), cap, C.byref(n)),
                   "orbgpu_batch_download")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def synchronize(self):
        _lib.check(self._ctx, self._L.orbgpu_synchronize(self._ctx), "orbgpu_synchronize")

    def stream(self) -> int:
        return self._L.orbgpu_stream(self._ctx)

    def set_stage_timing(self, on: bool):
        self._L.orbgpu_set_stage_timing(self._ctx, int(on))

    def stage_times(self):
        names = (C.c_char_p * 32)()
        ms = (C.c_float * 32)()
        n = self._L.orbgpu_stage_times(self._ctx, names, ms, 32)
        return [(names[i].decode(), ms[i]) for i in range(min(n, 32))]

    def stage_marks(self, ref: "ORBextractor"):
        """[(mark name, ms since ref's first mark)] of the last batch (stage timing on for both)."""
        names = (C.c_char_p * 64)()
        t = (C.c_float * 64)()
        n = self._L.orbgpu_stage_marks(self._ctx, ref.ctx, names, t, 64)
        return [(names[i].decode(), t[i]) for i in range(max(n, 0))]

    # ---- introspection for parity tests
    def debug_candidates(self, b: int, level: int) -> np.ndarray:
        n = self._L.orbgpu_debug_candidates(self._ctx, b, level, None, 0)
        if n < 0:
            _lib.check(self._ctx, n, "orbgpu_debug_candidates")
        out = np.zeros(max(n, 1), np.uint64)
        self._L.orbgpu_debug_candidates(self._ctx, b, level, _p(out), n)
        return out[:n]

    def debug_octree(self, b: int, level: int):
        n = self._L.orbgpu_debug_octree(self._ctx, b, level, None, None, 0)
        if n < 0:
            _lib.check(self._ctx, n, "orbgpu_debug_octree")
        xy = np.zeros(max(n, 1), np.uint32)
        resp = np.zeros(max(n, 1), np.uint32)  # response keys (FAST score, or the Harris key)
        self._L.orbgpu_debug_octree(self._ctx, b, level, _p(xy), _p(resp), n)
        return (xy[:n] & 0xFFFF).astype(np.int32), (xy[:n] >> 16).astype(np.int32), resp[:n]

    # device memory helpers (no torch needed)
    def device_alloc(self, nbytes: int) -> int:
        p = self._L.orbgpu_device_alloc(self._ctx, nbytes)
        if not p:
            raise RuntimeError("orbgpu_device_alloc failed")
        return p

    def device_free(self, p: int):
        self._L.orbgpu_device_free(self._ctx, C.c_void_p(p))

    def h2d(self, dst: int, src: np.ndarray):
        src = np.ascontiguousarray(src)
        _lib.check(self._ctx, self._L.orbgpu_memcpy_h2d(self._ctx, C.c_void_p(dst), _p(src), src.nbytes), "h2d")

    def d2h(self, dst: np.ndarray, src: int):
        _lib.check(self._ctx, self._L.orbgpu_memcpy_d2h(self._ctx, _p(dst), C.c_void_p(src), dst.nbytes), "d2h")
