"""The drop-in binding EXECUTED (GPU): integration/ORBextractor.cc, compiled against the reference's unchanged
include/ORBextractor.h (tests/test_integration_compile.py checks the declarations), linked with
tests/binding_run/cvmini.cc (the minimal cv::Mat / InputArray / OutputArray it calls) into
tests/binding_run/run_binding, runs ORB-SLAM2's own call pattern -- one long-lived ORBextractor, one
`(*extractor)(im, cv::Mat(), keys, desc)` per frame (src/Frame.cc:247-253) -- and its keypoints, descriptors, getters
and public mvImagePyramid are compared bit-for-bit with the CPU oracle.

run_binding is built by __graft_entry__.build() / build_ext.build_binding_runner() where the reference headers
are present (this container) and travels to the GPU box with the tree, like liborbgpu.so.
"""
import os
import subprocess

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import KP_DTYPE, synthetic

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(ROOT, "tests", "binding_run", "run_binding")
FIELDS = ("x", "y", "size", "angle", "response", "octave", "class_id")


def _parse(buf, nframes):
    o = 0

    def take(n, dt):
        nonlocal o
        a = np.frombuffer(buf, dt, n, o)
        o += a.nbytes
        return a

    nl = int(take(1, np.int32)[0])
    sf = float(take(1, np.float32)[0])
    tabs = [take(nl, np.float32).copy() for _ in range(4)]
    frames = []
    for _ in range(nframes):
        n = int(take(1, np.int32)[0])
        k = take(n, KP_DTYPE).copy()
        rows, cols = (int(v) for v in take(2, np.int32))
        d = take(rows * cols, np.uint8).reshape(rows, cols).copy()
        frames.append((k, d))
    levels = []
    for _ in range(nl):
        rows, cols = (int(v) for v in take(2, np.int32))
        levels.append(take(rows * cols, np.uint8).reshape(rows, cols).copy())
    assert o == len(buf)
    return nl, sf, tabs, frames, levels


@pytest.mark.parametrize("shape,nfeat,pad", [((1080, 1920), 2000, 0), ((480, 640), 1000, 64), ((376, 1241), 2000, 3)])
def test_binding_runs_reference_call_pattern(gpu, oracle, tmp_path, shape, nfeat, pad):
    if not os.path.exists(RUNNER):
        pytest.fail("tests/binding_run/run_binding was not built (build it where /root/reference exists: "
                    "python -c 'import __graft_entry__ as g; g.build()')")
    H, W = shape
    pitch = W + pad
    imgs = [synthetic.frame(40 + i, H, W) for i in range(3)]
    raw = np.zeros((len(imgs), H, pitch), np.uint8)
    for i, im in enumerate(imgs):
        raw[i, :, :W] = im
    fin, fout = tmp_path / "frames.u8", tmp_path / "out.bin"
    raw.tofile(fin)
    r = subprocess.run([RUNNER, str(fin), str(W), str(H), str(pitch), str(len(imgs)), str(nfeat), "1.2", "8", "20",
                        "7", str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    nl, sf, tabs, frames, levels = _parse(fout.read_bytes(), len(imgs))
    oe = oracle.OracleExtractor(nfeat)
    t = oe.tables()
    assert nl == 8 and sf == np.float32(1.2)
    for got, key in zip(tabs, ("scale", "inv_scale", "sigma2", "inv_sigma2")):
        assert np.array_equal(got.view(np.int32), t[key].view(np.int32)), key
    for im, (k, d) in zip(imgs, frames):
        ko, do = oe(im)
        assert len(k) == len(ko) and d.shape == (len(ko), 32)
        for f in FIELDS:
            assert np.array_equal(k[f].view(np.int32), ko[f].view(np.int32)), f
        assert np.array_equal(d, do)
    for l in range(8):  # the last frame's public mvImagePyramid (read by Frame::ComputeStereoMatches)
        assert np.array_equal(levels[l], oe.level(l)), l
