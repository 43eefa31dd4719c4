"""Config 1: a TUM RGB-D sequence through the feature path, frame by frame (the front half of the
reference's Examples/RGB-D/rgbd_tum.cc, up to the RGB-D Frame: PNG decode, cvtColor + ORB extraction on the
GPU, UndistortKeyPoints, ComputeStereoFromRGBD).  The SLAM back end is out of scope.

    python tools/rgbd_tum.py path_to_settings path_to_sequence path_to_association [--json out.json]
    python tools/rgbd_tum.py --synthetic N [--json out.json]   # a synthetic 640x480 sequence, TUM1 settings

Prints the median / mean per-frame time of the feature path (rgbd_tum.cc's "tracking time" statistics cover
the whole SLAM step; here only the part this framework replaces) and the mean keypoints / valid depths.
"""
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime in the process)

from orbslam2_with_quadrics_amd import synthetic, tum  # noqa: E402

TUM1_SETTINGS = {  # Examples/RGB-D/TUM1.yaml
    "Camera.fx": 517.306408, "Camera.fy": 516.469215, "Camera.cx": 318.643040, "Camera.cy": 255.313989,
    "Camera.k1": 0.262383, "Camera.k2": -0.953104, "Camera.p1": -0.005358, "Camera.p2": 0.002628,
    "Camera.k3": 1.163314, "Camera.width": 640, "Camera.height": 480, "Camera.fps": 30.0, "Camera.bf": 40.0,
    "Camera.RGB": 1, "ThDepth": 40.0, "DepthMapFactor": 5000.0, "ORBextractor.nFeatures": 1000,
    "ORBextractor.scaleFactor": 1.2, "ORBextractor.nLevels": 8, "ORBextractor.iniThFAST": 20,
    "ORBextractor.minThFAST": 7,
}


def run(fs: dict, seq_dir: str, assoc: str) -> dict:
    K4, dist, mbf, factor, bRGB = tum.camera_from_settings(fs)
    ex = tum.extractor_from_settings(fs)
    times, nkp, ndepth, ndecode = [], [], [], []
    for t, imRGB, imD in tum.sequence_rgbd(seq_dir, assoc):
        t1 = time.perf_counter()
        F = tum.grab_image_rgbd(ex, imRGB, imD, K4, dist, mbf, factor, bRGB)
        times.append(time.perf_counter() - t1)
        nkp.append(F.N)
        ndepth.append(int((F.mvDepth > 0).sum()))
    if not times:
        raise SystemExit("No images found in provided path.")
    s = sorted(times)
    return {"frames": len(times), "median_frame_ms": 1e3 * s[len(s) // 2], "mean_frame_ms": 1e3 * statistics.mean(s),
            "frames_per_s": len(times) / sum(times), "mean_keypoints": float(np.mean(nkp)),
            "mean_valid_depths": float(np.mean(ndepth))}


def main():
    argv = sys.argv[1:]
    out = None
    if "--json" in argv:
        out = argv[argv.index("--json") + 1]
        del argv[argv.index("--json"):argv.index("--json") + 2]
    if argv and argv[0] == "--synthetic":
        n = int(argv[1]) if len(argv) > 1 else 30
        d = tempfile.mkdtemp(prefix="tum_synth_")
        assoc = synthetic.write_tum_rgbd_sequence(d, n)
        res = run(dict(TUM1_SETTINGS), d, assoc)
        res["sequence"] = f"synthetic {n} frames 640x480 (TUM1 settings)"
    elif len(argv) == 3:
        res = run(tum.read_settings(argv[0]), argv[1], argv[2])
        res["sequence"] = argv[1]
    else:
        print(__doc__)
        return 1
    print("-------")
    print(f"median feature-path time: {res['median_frame_ms']:.3f} ms")
    print(f"mean feature-path time: {res['mean_frame_ms']:.3f} ms")
    print(json.dumps(res))
    if out:
        with open(out, "w") as fp:
            json.dump(res, fp, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
