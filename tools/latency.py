"""Per-frame latency of the feature path for the real-time SLAM use case (one frame at a time), GPU box.

Reports the median wall time of (a) ORBextractor::operator() through the host C ABI (image H2D, extraction,
keypoints + descriptors D2H, as Frame::ExtractORB calls it) and (b) a device-resident single-frame batch
(extraction only), for 640x480 / 1000 features and 1920x1080 / 2000 features.

python tools/latency.py [--json out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime in the process)

from orbslam2_with_quadrics_amd import ORBextractor, synthetic  # noqa: E402


def median_ms(fn, n=50, warm=5):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(float(np.median(ts)), 3)


def main():
    out = {}
    for rows, cols, nf in ((480, 640, 1000), (1080, 1920, 2000)):
        img = synthetic.frame(3, rows, cols)
        ex = ORBextractor(nf, 1.2, 8, 20, 7)
        host = median_ms(lambda: ex(img))
        d = ex.device_alloc(img.nbytes)
        ex.h2d(d, img)

        def dev():
            ex.extract_batch_device(d, 1, cols, rows, cols, img.nbytes)
            ex.synchronize()

        devm = median_ms(dev)
        ex.device_free(d)
        out[f"{cols}x{rows}_{nf}"] = {"host_api_ms": host, "device_resident_ms": devm}
        print(cols, rows, nf, "host API", host, "ms; device-resident", devm, "ms", flush=True)
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
