"""Exhaustive GPU pins of the restated glibc functions (SURVEY.md §7 hard part 3): the device og_sincosf on every
float in [0, 6.5) (all rBRIEF angles: fastAtan2 degrees in [0, 360] times pi/180, src/ORBextractor.cc:113) and the
device og_logf on every positive finite float (MapPoint::PredictScale's log(ratio), src/MapPoint.cc:410), compared
chunk by chunk with hashes of the host libm's values (tests/golden/libm_chunks.json, tools/libm_chunk_hash.c)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("fn", ["sincos", "logf"])
def test_device_libm_restatement_exhaustive(gpu, fn):
    import ctypes as C

    from orbslam2_with_quadrics_amd import _lib

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "libm_chunks.json")))
    spec = g["functions"][fn]
    want = spec["hashes"]
    out = np.zeros(len(want), np.uint64)
    rc = _lib.lib().orbgpu_debug_math_hash(0, 0 if fn == "sincos" else 1, spec["begin"], spec["end"], g["chunk_log2"],
                                           out.ctypes.data_as(C.c_void_p), len(want))
    assert rc == 0
    bad = [i for i, h in enumerate(want) if int(h, 16) != int(out[i])]
    n = spec["end"] - spec["begin"]
    assert not bad, f"{fn}: {len(bad)} of {len(want)} chunks (2^{g['chunk_log2']} inputs each) differ, first {bad[:5]}"
    assert n > 1_000_000_000
