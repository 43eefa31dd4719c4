"""GPU parity per OpenCV/compiler semantics variant (ORBGPU_SEM_*, include/orbgpu.h).

Every combination (2 resize forms x 4 GaussianBlur variants x FMA / non-FMA rBRIEF rotation) is compared
bit-exactly with the committed oracle goldens at the config-2 (640x480, 1000 features) and config-3 (1920x1080,
2000 features) shapes.  Natural frames rarely separate the blur variants and never the rotation forms, so two
crafted cases make those comparisons meaningful: binarised frames (frequent half-to-even ties in the SSE2
column pass) and the FMA probe image of tools/find_fma_probe.py.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import _lib, synthetic

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def assert_same(k, d, ko, do):
    assert len(k) == len(ko)
    for f in FIELDS:
        bad = np.nonzero(k[f].view(np.int32) != ko[f].view(np.int32))[0]
        assert len(bad) == 0, (f, bad[:5])
    assert np.array_equal(d, do)


_cases = json.load(open(os.path.join(GOLDEN, "extract_golden.json")))["cases"]
_variant_cases = [c for c in _cases if c["frame_id"] in (3, 7)]


@pytest.mark.parametrize("case", _variant_cases,
                         ids=[f"{c['cols']}x{c['rows']}-{c['semantics_name']}" for c in _variant_cases])
def test_extract_each_semantics_vs_golden(gpu, case):
    img = synthetic.frame(case["frame_id"], case["rows"], case["cols"])
    ex = gpu.ORBextractor(case["nfeatures"], 1.2, 8, 20, 7, semantics=case["semantics"])
    k, d = ex(img)
    assert len(k) == case["n"]
    assert hashlib.sha256(k.tobytes()).hexdigest() == case["kps_sha256"]
    assert hashlib.sha256(d.tobytes()).hexdigest() == case["desc_sha256"]


@pytest.mark.parametrize("sem", [0, _lib.SEM_RESIZE_FIXEDPT])
def test_pyramid_each_resize_form(gpu, oracle, sem):
    """All 8 levels of both resize forms (fused and single-level launches) against the oracle, 1080p and an
    odd KITTI-like width."""
    for fid, (h, w) in ((7, (1080, 1920)), (5, (376, 1241))):
        img = synthetic.frame(fid, h, w)
        ex = gpu.ORBextractor(2000, 1.2, 8, 20, 7, semantics=sem)
        ex(img)
        oe = oracle.OracleExtractor(2000, semantics=sem)
        oe(img)
        for lvl in range(8):
            assert np.array_equal(ex.level(lvl), oe.level(lvl)), (sem, fid, lvl)


def test_blur_variants_on_binarised_batch(gpu, oracle):
    """Binarised frames (values 16 / 144) make SSE2 half-to-even ties common: the four blur variants give
    different descriptors, and a batched launch of 16 frames matches the oracle for each of them."""
    B, rows, cols = 16, 480, 640
    frames = np.stack([(synthetic.frame(500 + b, rows, cols) & 0x80) | 0x10 for b in range(B)]).astype(np.uint8)
    outs = {}
    for blur in (_lib.SEM_BLUR_SSE2_257, _lib.SEM_BLUR_SCALAR_257, _lib.SEM_BLUR_BITEXACT_256,
                 _lib.SEM_BLUR_BITEXACT_ED):
        ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7, semantics=blur)
        oe = oracle.OracleExtractor(1000, semantics=blur)
        d_img = ex.device_alloc(frames.nbytes)
        try:
            ex.h2d(d_img, frames)
            ex.extract_batch_device(d_img, B, cols, rows, cols, rows * cols)
            ex.synchronize()
            descs = []
            for b in range(B):
                k, d = ex.batch_download(b)
                ko, do = oe(frames[b])
                assert_same(k, d, ko, do)
                descs.append(do)
            outs[blur] = np.concatenate(descs)
        finally:
            ex.device_free(d_img)
    ref = outs[_lib.SEM_BLUR_SSE2_257]
    assert not np.array_equal(ref, outs[_lib.SEM_BLUR_SCALAR_257])  # the ties changed some descriptor bits
    assert not np.array_equal(ref, outs[_lib.SEM_BLUR_BITEXACT_256])
    assert not np.array_equal(outs[_lib.SEM_BLUR_BITEXACT_256], outs[_lib.SEM_BLUR_BITEXACT_ED])


@pytest.mark.parametrize("sem", [0, _lib.SEM_BRIEF_NOFMA])
def test_rbrief_rotation_probe(gpu, sem):
    """tools/find_fma_probe.py's image: the FMA and the non-FMA rotation give different descriptors there;
    the GPU reproduces the committed oracle hash of each form."""
    sys.path.insert(0, GOLDEN)
    import make_golden

    g = json.load(open(os.path.join(GOLDEN, "semantics_probe.json")))
    img = make_golden.fma_probe_image(g["seed"], g["mods"])
    ex = gpu.ORBextractor(g["nfeatures"], 1.2, 8, 20, 7, semantics=sem)
    k, d = ex(img)
    assert hashlib.sha256(k.tobytes()).hexdigest() == g["kps_sha256"]
    want = g["desc_nofma_sha256"] if sem & _lib.SEM_BRIEF_NOFMA else g["desc_fma_sha256"]
    assert hashlib.sha256(d.tobytes()).hexdigest() == want


def test_semantics_switch_rejects_unknown_flags(gpu):
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    for bad in (0x80, 0x100, 4 << 2, 7 << 2):
        with pytest.raises(RuntimeError, match="semantics"):
            ex.set_semantics(bad)
    assert ex._L.orbgpu_get_semantics(ex.ctx) == 0
    ex.set_semantics(_lib.SEM_ROUND1)
    assert ex._L.orbgpu_get_semantics(ex.ctx) == _lib.SEM_ROUND1
