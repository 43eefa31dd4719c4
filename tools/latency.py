"""Per-frame latency of the feature path for the real-time SLAM use case (one frame at a time), GPU box.

ORB-SLAM2 extracts one frame per Frame constructor (src/Frame.cc:247-253, ORBextractor::operator()).  Reported,
for 640x480 / 1000 features, 1242x375 (KITTI) / 2000 and 1920x1080 / 2000 (median and p90 of 300 calls):
  host_api      orbgpu_extract through ctypes with preallocated outputs (image H2D, extraction, keypoints +
                descriptors D2H: what integration/ORBextractor.cc calls);
  python_api    the Python mirror ORBextractor.__call__ (adds numpy allocation of the outputs);
  device        a device-resident single-frame batch (orbgpu_extract_batch_device + synchronize);
  h2d           the image upload alone (pageable host memory, as a cv::Mat is);
  stages        per-stage device time of one frame (stage timing on: HIP events between stages).

python tools/latency.py [--json out.json] [--n 300]
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime in the process)

from orbslam2_with_quadrics_amd import ORBextractor, synthetic, _lib  # noqa: E402
from orbslam2_with_quadrics_amd.extractor import KP_DTYPE  # noqa: E402


def stats_ms(fn, n, warm=20):
    for _ in range(warm):
        fn()
    ts = np.empty(n)
    for i in range(n):
        t = time.perf_counter()
        fn()
        ts[i] = (time.perf_counter() - t) * 1e3
    return {"p50": round(float(np.median(ts)), 4), "p90": round(float(np.percentile(ts, 90)), 4),
            "min": round(float(ts.min()), 4)}


def main():
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 300
    L = _lib.lib()
    vp = C.c_void_p
    out = {"note": "milliseconds per frame; one frame at a time (Frame::ExtractORB call pattern)",
           "graph_replay": os.environ.get("ORBGPU_GRAPH", "default")}
    keep = []  # every context lives to the end (as a SLAM process's extractors do)
    for rows, cols, nf in ((480, 640, 1000), (375, 1242, 2000), (1080, 1920, 2000)):
        img = np.ascontiguousarray(synthetic.frame(3, rows, cols))
        ex = ORBextractor(nf, 1.2, 8, 20, 7)
        keep.append(ex)
        cap = L.orbgpu_max_keypoints(ex.ctx)
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        cnt = C.c_int(0)
        ip, kp, dp = img.ctypes.data_as(vp), kps.ctypes.data_as(vp), desc.ctypes.data_as(vp)

        def host():
            rc = L.orbgpu_extract(ex.ctx, ip, cols, rows, cols, kp, dp, cap, C.byref(cnt))
            if rc != 0:
                _lib.check(ex.ctx, rc, "orbgpu_extract")

        r = {"keypoints": None}
        r["host_api"] = stats_ms(host, n)
        r["keypoints"] = cnt.value
        r["python_api"] = stats_ms(lambda: ex(img), n // 3)
        d = ex.device_alloc(img.nbytes)
        r["h2d"] = stats_ms(lambda: ex.h2d(d, img), n // 3)

        def dev():
            ex.extract_batch_device(d, 1, cols, rows, cols, img.nbytes)
            ex.synchronize()

        r["device"] = stats_ms(dev, n)
        ex.set_stage_timing(True)
        acc = {}
        for _ in range(50):
            dev()
            for name, ms in ex.stage_times():
                acc.setdefault(name, []).append(ms)
        ex.set_stage_timing(False)
        r["stages"] = {k: round(float(np.median(v)), 4) for k, v in acc.items()}
        ex.device_free(d)
        out[f"{cols}x{rows}_{nf}"] = r
        print(cols, rows, nf, json.dumps(r), flush=True)
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
