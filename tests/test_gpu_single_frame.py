"""The single-frame path (Frame::ExtractORB's one-frame-at-a-time call, src/Frame.cc:247-253):

* batches of up to 4 frames of at least ORBGPU_FORK_MIN_PIXELS (default 2^20, so the 1080p cases here; the
  640x480 case runs serially in both orders) fork level 0's FAST + octree (and, with the Harris option, level 0's
  Harris pass) onto the context stream and the pyramid + levels >= 1 onto a second stream (orbgpu_capi.cpp
  run_batch); with stage timing on the same batch runs serially.  Both orders must give identical keypoints,
  descriptors and grids;
* orbgpu_extract downloads through one packing kernel into a pinned block (og_pack_host_kernel) and copies a
  contiguous image with its own pitch: it must equal the batch download, for contiguous and strided images, and
  report ORBGPU_ERR_CAPACITY with the needed count when the caller's capacity is short.
"""
import ctypes as C

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import _lib, synthetic
from orbslam2_with_quadrics_amd.extractor import KP_DTYPE

pytestmark = pytest.mark.gpu


def _grid(ex, B):
    cap = ex.batch_outputs()[3]
    cs, ci = C.c_void_p(), C.c_void_p()
    _lib.check(ex.ctx, _lib.lib().orbgpu_batch_grid(ex.ctx, C.byref(cs), C.byref(ci)), "grid")
    CS = np.zeros(B * 3073, np.int32)
    CI = np.zeros(B * cap, np.int32)
    ex.d2h(CS, cs.value)
    ex.d2h(CI, ci.value)
    return CS, CI


@pytest.mark.parametrize("shape,nf,sem", [((480, 640), 1000, 0), ((1080, 1920), 2000, 0), ((1080, 1920), 4000, 0),
                                          ((1080, 1920), 2000, _lib.SEM_SCORE_HARRIS)])
def test_forked_small_batches_equal_serial(gpu, oracle, shape, nf, sem):
    rows, cols = shape
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7, semantics=sem)
    frames = np.stack([synthetic.frame(40 + b, rows, cols) for b in range(5)]).astype(np.uint8)
    d = ex.device_alloc(frames.nbytes)
    try:
        ex.h2d(d, frames)
        for B in (1, 2, 4, 5):
            outs = []
            for timing in (True, False):  # serial (stage marks) / forked (B <= 4, frames >= 2^20 px)
                ex.set_stage_timing(timing)
                ex.extract_batch_device(d, B, cols, rows, cols, rows * cols)
                ex.synchronize()
                outs.append(([ex.batch_download(b) for b in range(B)], _grid(ex, B)))
            ex.set_stage_timing(False)
            (ka, ga), (kb, gb) = outs
            for b in range(B):
                assert ka[b][0].tobytes() == kb[b][0].tobytes() and np.array_equal(ka[b][1], kb[b][1]), (B, b)
            assert np.array_equal(ga[0], gb[0]) and np.array_equal(ga[1], gb[1]), B
        # and the forked single frame against the oracle
        k, dsc = ex(frames[0])
        ko, do = oracle.OracleExtractor(nf, semantics=sem)(frames[0])
        assert k.tobytes() == ko.tobytes() and np.array_equal(dsc, do)
    finally:
        ex.device_free(d)


def test_host_api_download_paths(gpu):
    L = _lib.lib()
    rows, cols = 375, 1242
    img = synthetic.frame(9, rows, cols)
    ex = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    d = ex.device_alloc(img.nbytes)
    ex.h2d(d, img)
    ex.extract_batch_device(d, 1, cols, rows, cols, img.nbytes)
    ex.synchronize()
    kref, dref = ex.batch_download(0)
    ex.device_free(d)
    cap = L.orbgpu_max_keypoints(ex.ctx)
    # contiguous (one linear copy, pitch = cols) and strided (2-D copy into a 64-byte pitch) host images
    wide = np.zeros((rows, cols + 50), np.uint8)
    wide[:, :cols] = img
    for src, step in ((np.ascontiguousarray(img), cols), (wide, cols + 50)):
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int(0)
        rc = L.orbgpu_extract(ex.ctx, src.ctypes.data_as(C.c_void_p), cols, rows, step,
                              kps.ctypes.data_as(C.c_void_p), desc.ctypes.data_as(C.c_void_p), cap, C.byref(n))
        assert rc == 0
        assert kps[:n.value].tobytes() == kref.tobytes() and np.array_equal(desc[:n.value], dref)
    # a short capacity: ERR_CAPACITY and the count needed
    small = len(kref) - 1
    kps = np.zeros(small, KP_DTYPE)
    desc = np.zeros((small, 32), np.uint8)
    n = C.c_int(0)
    rc = L.orbgpu_extract(ex.ctx, img.ctypes.data_as(C.c_void_p), cols, rows, cols,
                          kps.ctypes.data_as(C.c_void_p), desc.ctypes.data_as(C.c_void_p), small, C.byref(n))
    assert rc == _lib.ERR_CAPACITY and n.value == len(kref)
