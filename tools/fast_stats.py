"""FAST filter statistics on the synthetic frames (analysis only, CPU, numpy).

For level 0 of a synthetic frame: the fraction of pixels that pass the opposite-pair quick test
(og_fast_quick2) at a threshold, the fraction that are FAST-9 corners (M > t), and the fraction that pass
alternative necessary conditions.  Used to decide where the FAST kernel's stage-2 work goes.

python tools/fast_stats.py [H W]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orbslam2_with_quadrics_amd import synthetic  # noqa: E402

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def stats(img, ts=(7, 20)):
    H, W = img.shape
    v = img[3:H - 3, 3:W - 3].astype(np.int32)
    c = np.stack([img[3 + dy:H - 3 + dy, 3 + dx:W - 3 + dx].astype(np.int32) for dx, dy in CIRCLE])
    n = v.size

    def score_dark(cc, vv):  # v - min over arcs of the arc max
        mx9 = np.stack([np.max(np.stack([cc[(k + j) % 16] for j in range(9)]), 0) for k in range(16)])
        return np.maximum(vv - mx9.min(0), 0)
    Md, Mb = score_dark(c, v), score_dark(255 - c, 255 - v)
    M = np.maximum(Md, Mb)
    md = np.max(np.stack([np.minimum(c[k], c[k + 8]) for k in range(8)]), 0)
    mb = np.min(np.stack([np.maximum(c[k], c[k + 8]) for k in range(8)]), 0)
    # a 9-arc [k, k+8] holds the three points k, k+4, k+8: some k has all three dark (bright)
    qd = np.min(np.stack([np.maximum(np.maximum(c[k], c[(k + 4) % 16]), c[(k + 8) % 16]) for k in range(16)]), 0)
    qb = np.max(np.stack([np.minimum(np.minimum(c[k], c[(k + 4) % 16]), c[(k + 8) % 16]) for k in range(16)]), 0)
    out = {}
    for t in ts:
        quick_d = md < v - t
        quick_b = mb > v + t
        quick = quick_d | quick_b
        q2 = (quick_d & (qd < v - t)) | (quick_b & (qb > v + t))
        corner = M > t
        out[t] = dict(quick=quick.sum() / n, quick_plus_quarter=q2.sum() / n, corner=corner.sum() / n,
                      both_pol=(quick_d & quick_b).sum() / n)
    return out


def main():
    H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1080, 1920)
    img = synthetic.frame(0, H, W)
    for t, d in stats(img).items():
        print(t, {k: round(float(x), 4) for k, x in d.items()})


if __name__ == "__main__":
    main()
