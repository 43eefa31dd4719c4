"""The drop-in binding of INTEGRATION.md is compiled, not prose (CPU test, g++ -fsyntax-only):

* integration/ORBextractor.cc against the reference's UNCHANGED include/ORBextractor.h -- the compiler checks
  every definition against the reference's own declarations (cv::InputArray / OutputArray signatures included);
* integration/ORBmatcher_perframe.cc and integration/Frame_stereo.cc against integration/refdecl, which restates
  the Frame / MapPoint / ORBmatcher declarations the binding uses; each restated line is checked against the
  reference header line it cites (the real headers need Eigen, g2o and DBoW2, absent here).
integration/cvshim declares the cv:: names involved (declarations only, nothing is linked or run).
The reference tree is only read; these tests skip where it is absent (the GPU box)."""
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
INT = os.path.join(ROOT, "integration")
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "include", "ORBextractor.h")),
                                reason="reference tree absent")


def _gxx(src, incs):
    cmd = ["g++", "-std=c++11", "-fsyntax-only", "-Wall", "-Wextra", "-Wno-unused-parameter", src]
    for i in incs:
        cmd += ["-I", i]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_refdecl_lines_match_reference_headers():
    n = 0
    for p in glob.glob(os.path.join(INT, "refdecl", "*.h")):
        for line in open(p):
            m = re.match(r"^(.*?)\s*// ref: (include/\w+\.h):(\d+)\s*$", line.rstrip("\n"))
            if not m:
                continue
            ref = open(os.path.join(REF, m.group(2))).read().split("\n")[int(m.group(3)) - 1]
            assert " ".join(m.group(1).split()) == " ".join(ref.split()), (p, line, ref)
            n += 1
    assert n >= 40


def test_orbextractor_binding_compiles_against_reference_header():
    _gxx(os.path.join(INT, "ORBextractor.cc"),
         [os.path.join(INT, "cvshim"), os.path.join(REF, "include"), os.path.join(ROOT, "include"), INT])


@pytest.mark.parametrize("src", ["ORBmatcher_perframe.cc", "Frame_stereo.cc"])
def test_matcher_and_frame_bindings_compile(src):
    _gxx(os.path.join(INT, src), [os.path.join(INT, "refdecl"), os.path.join(INT, "cvshim"),
                                  os.path.join(REF, "include"), os.path.join(ROOT, "include"), INT])


def test_orbextractor_binding_rejects_a_signature_change(tmp_path):
    """The check has teeth: a definition whose signature differs from the reference declaration fails."""
    src = open(os.path.join(INT, "ORBextractor.cc")).read().replace(
        "std::vector<cv::KeyPoint>& _keypoints,", "std::vector<cv::KeyPoint>* _keypoints,", 1)
    p = tmp_path / "bad.cc"
    p.write_text(src)
    with pytest.raises(AssertionError):
        _gxx(str(p), [os.path.join(INT, "cvshim"), os.path.join(REF, "include"), os.path.join(ROOT, "include"), INT])
