"""ctypes loader of the in-tree gfx950 library (liborbgpu.so) -- the C ABI of include/orbgpu.h.

The product path has no CPU fallback: if the HIP library is missing or no GPU is visible, calls fail
loudly (RuntimeError).  torch is imported first when available so that torch and this library share
one HIP runtime in the process (both link libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ORBGPU_LIB selects an experiment build of the same library (tools/variant_bench.py, tools/octree_profile.py); default in-tree
LIB_PATH = os.environ.get("ORBGPU_LIB") or os.path.join(HERE, "liborbgpu.so")

# Every symbol include/orbgpu.h declares (checked by tests/test_lib_abi.py).
EXPORTS = [
    "orbgpu_create", "orbgpu_destroy", "orbgpu_get_levels", "orbgpu_get_scale_factor",
    "orbgpu_get_scale_factors", "orbgpu_get_inverse_scale_factors", "orbgpu_get_scale_sigma_squares",
    "orbgpu_get_inverse_scale_sigma_squares", "orbgpu_get_features_per_level", "orbgpu_extract",
    "orbgpu_max_keypoints", "orbgpu_get_level", "orbgpu_extract_batch_device", "orbgpu_batch_outputs",
    "orbgpu_batch_download", "orbgpu_grid_geom_for_image", "orbgpu_descriptor_distance",
    "orbgpu_search_for_initialization", "orbgpu_search_for_initialization_batch",
    "orbgpu_search_by_projection", "orbgpu_search_by_projection_batch", "orbgpu_stream", "orbgpu_synchronize", "orbgpu_set_stage_timing",
    "orbgpu_stage_times", "orbgpu_last_error", "orbgpu_debug_candidates", "orbgpu_debug_octree",
    "orbgpu_device_alloc", "orbgpu_device_free", "orbgpu_memcpy_h2d", "orbgpu_memcpy_d2h",
    "orbgpu_memset_d", "orbgpu_prev_matched_from_frame", "orbgpu_memcpy_d2d_async",
    "orbgpu_batch_candidate_total", "orbgpu_compute_stereo_matches", "orbgpu_compute_stereo_matches_batch",
    "orbgpu_is_in_frustum", "orbgpu_search_by_projection_last_frame", "orbgpu_debug_octree_profile",
    "orbgpu_debug_fast_profile", "orbgpu_debug_set_projection_paths",
    "orbgpu_stage_marks", "orbgpu_undistort_keypoints", "orbgpu_compute_image_bounds", "orbgpu_set_undistortion",
    "orbgpu_batch_outputs_undistorted", "orbgpu_search_by_projection_keyframe",
    "orbgpu_search_by_projection_keyframe_levels",
    "orbgpu_compute_stereo_from_rgbd", "orbgpu_compute_stereo_from_rgbd_batch",
    "orbgpu_vocabulary_load_text", "orbgpu_vocabulary_create", "orbgpu_vocabulary_destroy", "orbgpu_vocabulary_info",
    "orbgpu_compute_bow", "orbgpu_compute_bow_batch", "orbgpu_memcpy_h2d_async", "orbgpu_memcpy_d2h_async",
    "orbgpu_cvt_color_to_gray_batch", "orbgpu_extract_color", "orbgpu_set_semantics", "orbgpu_get_semantics",
    "orbgpu_batch_grid", "orbgpu_debug_math_hash", "orbgpu_is_in_frustum_batch",
    "orbgpu_search_by_projection_batch_shared_map", "orbgpu_frame_record_bytes", "orbgpu_frame_record_pack", "orbgpu_frame_record_unpack",
]

# OpenCV / compiler semantics switch (include/orbgpu.h ORBGPU_SEM_*)
SEM_DEFAULT = 0x00
SEM_RESIZE_FIXEDPT = 0x01
SEM_BLUR_SHIFT = 2
SEM_BLUR_SSE2_257, SEM_BLUR_SCALAR_257, SEM_BLUR_BITEXACT_256, SEM_BLUR_BITEXACT_ED = (v << 2 for v in range(4))
SEM_BRIEF_NOFMA = 0x20
SEM_SCORE_HARRIS = 0x40  # option, not a reference behaviour: rank by the Harris response (parity unpinned)
SEM_ROUND1 = SEM_RESIZE_FIXEDPT | SEM_BLUR_SCALAR_257
# every valid combination: 2 resize forms x 4 blur variants x 2 rotation forms
SEM_ALL_VARIANTS = [r | b | f for r in (0, SEM_RESIZE_FIXEDPT)
                    for b in (SEM_BLUR_SSE2_257, SEM_BLUR_SCALAR_257, SEM_BLUR_BITEXACT_256, SEM_BLUR_BITEXACT_ED)
                    for f in (0, SEM_BRIEF_NOFMA)]


def semantics_name(flags: int) -> str:
    """Human-readable name of a semantics combination (bench lines, test ids)."""
    blur = ["sse2_257", "scalar_257", "bitexact_256", "bitexact_ed"][(flags >> SEM_BLUR_SHIFT) & 7]
    return (f"resize={'fixedpt' if flags & SEM_RESIZE_FIXEDPT else 'opencv8u'},blur={blur},"
            f"brief={'nofma' if flags & SEM_BRIEF_NOFMA else 'fma'}" + (",score=harris" if flags & SEM_SCORE_HARRIS else ""))

# cv::cvtColor codes of the colour entry points (include/orbgpu.h ORBGPU_COLOR_*, OpenCV's values)
COLOR_BGR2GRAY, COLOR_RGB2GRAY, COLOR_BGRA2GRAY, COLOR_RGBA2GRAY = 6, 7, 10, 11
COLOR_CHANNELS = {COLOR_BGR2GRAY: 3, COLOR_RGB2GRAY: 3, COLOR_BGRA2GRAY: 4, COLOR_RGBA2GRAY: 4}

OK, ERR_ARG, ERR_HIP, ERR_CAPACITY, ERR_UNSUPPORTED, ERR_INTERNAL = 0, -1, -2, -3, -4, -5


class KeyPointC(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


class GridGeom(C.Structure):
    _fields_ = [("minX", C.c_float), ("minY", C.c_float), ("maxX", C.c_float), ("maxY", C.c_float),
                ("invW", C.c_float), ("invH", C.c_float)]


class FrameView(C.Structure):
    _fields_ = [("n", C.c_int), ("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p),
                ("grid", GridGeom), ("scale_factors", C.c_void_p), ("nlevels", C.c_int)]


class MapPointsView(C.Structure):
    _fields_ = [("m", C.c_int), ("track_in_view", C.c_void_p), ("is_bad", C.c_void_p),
                ("level", C.c_void_p), ("view_cos", C.c_void_p), ("proj_x", C.c_void_p),
                ("proj_y", C.c_void_p), ("proj_xr", C.c_void_p), ("n_obs", C.c_void_p),
                ("desc", C.c_void_p)]


class Camera(C.Structure):
    _fields_ = [("Rcw", C.c_float * 9), ("tcw", C.c_float * 3), ("Ow", C.c_float * 3), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("mbf", C.c_float), ("mb", C.c_float),
                ("scale_factor", C.c_float), ("nlevels", C.c_int)]


class MapPointGeomView(C.Structure):
    _fields_ = [("m", C.c_int), ("pos", C.c_void_p), ("normal", C.c_void_p), ("max_dist", C.c_void_p),
                ("min_dist", C.c_void_p)]


class LastFrameView(C.Structure):
    _fields_ = [("n", C.c_int), ("kps", C.c_void_p), ("has_mp", C.c_void_p), ("outlier", C.c_void_p),
                ("pos", C.c_void_p), ("n_obs", C.c_void_p), ("desc", C.c_void_p)]


class KeyFrameView(C.Structure):
    _fields_ = [("n", C.c_int), ("kps", C.c_void_p), ("valid", C.c_void_p), ("pos", C.c_void_p),
                ("max_dist", C.c_void_p), ("min_dist", C.c_void_p), ("desc", C.c_void_p)]


_lib = None


def _declare(L):
    vp, i32, f32, sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
    L.orbgpu_create.restype = vp
    L.orbgpu_create.argtypes = [i32, i32, f32, i32, i32, i32]
    L.orbgpu_destroy.argtypes = [vp]
    L.orbgpu_set_semantics.argtypes = [vp, i32]
    L.orbgpu_get_semantics.argtypes = [vp]
    L.orbgpu_batch_grid.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
    L.orbgpu_is_in_frustum_batch.argtypes = [vp, vp, i32, GridGeom, C.POINTER(MapPointGeomView), f32, i32, vp, vp, vp,
                                             vp, vp, vp]
    L.orbgpu_search_by_projection_batch_shared_map.argtypes = [vp, C.POINTER(MapPointsView), i32, f32, f32, vp, vp,
                                                               vp, vp]
    L.orbgpu_debug_math_hash.argtypes = [i32, i32, C.c_ulonglong, C.c_ulonglong, i32, vp, i32]
    L.orbgpu_frame_record_bytes.restype = C.c_longlong
    L.orbgpu_frame_record_bytes.argtypes = [vp]
    L.orbgpu_frame_record_pack.argtypes = [vp, i32, vp]
    L.orbgpu_frame_record_unpack.argtypes = [vp, vp]
    L.orbgpu_get_levels.argtypes = [vp]
    L.orbgpu_get_scale_factor.restype = f32
    L.orbgpu_get_scale_factor.argtypes = [vp]
    for n in ("orbgpu_get_scale_factors", "orbgpu_get_inverse_scale_factors",
              "orbgpu_get_scale_sigma_squares", "orbgpu_get_inverse_scale_sigma_squares",
              "orbgpu_get_features_per_level"):
        getattr(L, n).argtypes = [vp, vp]
    L.orbgpu_extract.argtypes = [vp, vp, i32, i32, sz, vp, vp, i32, C.POINTER(i32)]
    L.orbgpu_extract_color.argtypes = [vp, vp, i32, i32, sz, i32, vp, vp, i32, C.POINTER(i32)]
    L.orbgpu_cvt_color_to_gray_batch.argtypes = [vp, vp, i32, i32, i32, sz, sz, i32, vp, sz, sz]
    L.orbgpu_max_keypoints.argtypes = [vp]
    L.orbgpu_get_level.argtypes = [vp, i32, vp, sz, C.POINTER(i32), C.POINTER(i32)]
    L.orbgpu_extract_batch_device.argtypes = [vp, vp, i32, i32, i32, sz, sz]
    L.orbgpu_batch_outputs.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(i32)]
    L.orbgpu_batch_download.argtypes = [vp, i32, vp, vp, i32, C.POINTER(i32)]
    L.orbgpu_grid_geom_for_image.argtypes = [i32, i32, C.POINTER(GridGeom)]
    L.orbgpu_descriptor_distance.argtypes = [vp, vp]
    L.orbgpu_search_for_initialization.argtypes = [vp, C.POINTER(FrameView), C.POINTER(FrameView), f32,
                                                   i32, vp, vp, i32, C.POINTER(i32)]
    L.orbgpu_search_for_initialization_batch.argtypes = [vp, i32, vp, GridGeom, f32, i32, i32, vp, vp, vp]
    L.orbgpu_search_by_projection.argtypes = [vp, C.POINTER(FrameView), C.POINTER(MapPointsView), f32,
                                              f32, vp, vp, C.POINTER(i32)]
    L.orbgpu_search_by_projection_batch.argtypes = [vp, C.POINTER(MapPointsView), i32, f32, f32, vp, vp, vp, vp]
    L.orbgpu_memcpy_h2d_async.argtypes = [vp, vp, vp, sz]
    L.orbgpu_memcpy_d2h_async.argtypes = [vp, vp, vp, sz]
    L.orbgpu_stream.restype = vp
    L.orbgpu_stream.argtypes = [vp]
    L.orbgpu_synchronize.argtypes = [vp]
    L.orbgpu_set_stage_timing.argtypes = [vp, i32]
    L.orbgpu_stage_times.argtypes = [vp, C.POINTER(C.c_char_p), C.POINTER(f32), i32]
    L.orbgpu_last_error.restype = C.c_char_p
    L.orbgpu_last_error.argtypes = [vp]
    L.orbgpu_debug_candidates.argtypes = [vp, i32, i32, vp, i32]
    L.orbgpu_debug_octree.argtypes = [vp, i32, i32, vp, vp, i32]
    L.orbgpu_device_alloc.restype = vp
    L.orbgpu_device_alloc.argtypes = [vp, sz]
    L.orbgpu_device_free.argtypes = [vp, vp]
    L.orbgpu_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.orbgpu_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.orbgpu_memset_d.argtypes = [vp, vp, i32, sz]
    L.orbgpu_prev_matched_from_frame.argtypes = [vp, i32, vp, vp]
    L.orbgpu_memcpy_d2d_async.argtypes = [vp, vp, vp, sz]
    L.orbgpu_batch_candidate_total.restype = C.c_longlong
    L.orbgpu_debug_octree_profile.argtypes = [vp, vp, i32]
    L.orbgpu_debug_fast_profile.argtypes = [vp, vp, i32]
    L.orbgpu_debug_set_projection_paths.argtypes = [vp, i32]
    L.orbgpu_search_by_projection_keyframe.argtypes = [vp, C.POINTER(FrameView), C.POINTER(Camera),
                                                       C.POINTER(KeyFrameView), f32, i32, i32, vp, C.POINTER(i32)]
    L.orbgpu_search_by_projection_keyframe_levels.argtypes = [vp, C.POINTER(FrameView), C.POINTER(Camera),
                                                              C.POINTER(KeyFrameView), vp, f32, i32, i32, vp,
                                                              C.POINTER(i32)]
    L.orbgpu_compute_stereo_from_rgbd.argtypes = [vp, vp, i32, f32, sz, f32, vp, vp, i32, C.POINTER(i32)]
    L.orbgpu_compute_stereo_from_rgbd_batch.argtypes = [vp, vp, i32, f32, sz, sz, f32, vp, vp]
    L.orbgpu_vocabulary_load_text.restype = vp
    L.orbgpu_vocabulary_load_text.argtypes = [vp, C.c_char_p]
    L.orbgpu_vocabulary_create.restype = vp
    L.orbgpu_vocabulary_create.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp]
    L.orbgpu_vocabulary_destroy.argtypes = [vp]
    L.orbgpu_vocabulary_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    L.orbgpu_compute_bow.argtypes = [vp, vp, vp, i32, i32, vp, vp, C.POINTER(i32), vp, vp, vp, C.POINTER(i32)]
    L.orbgpu_compute_bow_batch.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp]
    L.orbgpu_undistort_keypoints.argtypes = [vp, vp, vp, i32, vp, vp, i32]
    L.orbgpu_compute_image_bounds.argtypes = [vp, vp, vp, i32, i32, i32, C.POINTER(GridGeom)]
    L.orbgpu_set_undistortion.argtypes = [vp, vp, vp, i32]
    L.orbgpu_batch_outputs_undistorted.argtypes = [vp, C.POINTER(vp), C.POINTER(GridGeom)]
    L.orbgpu_stage_marks.argtypes = [vp, vp, C.POINTER(C.c_char_p), C.POINTER(f32), i32]
    L.orbgpu_compute_stereo_matches.argtypes = [vp, vp, f32, f32, vp, vp, i32, C.POINTER(i32), C.POINTER(i32)]
    L.orbgpu_compute_stereo_matches_batch.argtypes = [vp, vp, f32, f32, vp, vp, vp]
    L.orbgpu_batch_candidate_total.argtypes = [vp]
    L.orbgpu_is_in_frustum.argtypes = [vp, C.POINTER(Camera), GridGeom, C.POINTER(MapPointGeomView), f32, vp, vp,
                                       vp, vp, vp, vp, C.POINTER(i32)]
    L.orbgpu_search_by_projection_last_frame.argtypes = [vp, C.POINTER(FrameView), C.POINTER(Camera),
                                                         C.POINTER(Camera), C.POINTER(LastFrameView), f32, i32, i32,
                                                         vp, vp, C.POINTER(i32)]


def lib(load_torch_first: bool = True):
    """Load liborbgpu.so (raises RuntimeError when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP library missing: {LIB_PATH} (run __graft_entry__.build() or "
                               "python -m orbslam2_with_quadrics_amd.build_ext)")
        if load_torch_first:
            try:
                import torch  # noqa: F401  (one HIP runtime per process)
            except Exception:
                pass
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def check(ctx, rc: int, what: str):
    if rc != OK:
        msg = lib().orbgpu_last_error(ctx) if ctx else b""
        raise RuntimeError(f"{what} failed with status {rc}: {msg.decode(errors='replace')}")
