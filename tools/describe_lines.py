"""Line-granular floor of the describe kernel's HBM traffic (CPU only; test infrastructure: runs the oracle).

The describe kernel reads a 43x43 window around every keypoint of its level (src/ORBextractor.cc:1076-1104 blur
window + IC_Angle disk).  SURVEY 8(d)'s algorithmic bytes count the window's bytes, K * (43^2 + 60).  HBM moves
whole 128-byte lines, so no schedule can read less than the DISTINCT lines the frame's windows touch.  This
script counts them for the bench's synthetic 1080p frames with the device layout (level 0 in the caller's
1920-byte rows; levels 1-7 packed in the pyramid block with 64-byte pitches, 256-byte aligned levels), and
prints the floor per 256-frame launch next to the window bytes.

python tools/describe_lines.py [--frames 4] [--json out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_py  # noqa: E402

from orbslam2_with_quadrics_amd import synthetic  # noqa: E402

LINE = 128


def main():
    nfr = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 4
    rows, cols, NF = 1080, 1920, 2000
    oracle_py.build()
    ex = oracle_py.OracleExtractor(NF)
    tot_lines = tot_win = tot_k = 0
    for i in range(nfr):
        img = synthetic.frame(i, rows, cols)
        k, _ = ex(img)
        sf = ex.tables()["scale"]
        # level geometry and the device's pyramid layout (orbgpu_capi.cpp build_plan)
        geo, off = [], 0
        for lvl in range(8):
            lv = ex.level(lvl)
            h, w = lv.shape
            if lvl == 0:
                geo.append((0, cols))  # the caller's frame: its own region, pitch 1920
            else:
                pitch = (w + 63) & ~63
                geo.append((off, pitch))
                off += (pitch * h + 255) & ~255
        lines = set()
        for kp in k:
            lvl = int(kp["octave"])
            x = int(round(float(kp["x"]) / sf[lvl])) if lvl else int(kp["x"])
            y = int(round(float(kp["y"]) / sf[lvl])) if lvl else int(kp["y"])
            base, pitch = geo[lvl]
            tag = 0 if lvl == 0 else 1
            for r in range(y - 21, y + 22):
                a0 = base + r * pitch + (x - 21)
                for ln in range(a0 // LINE, (a0 + 42) // LINE + 1):
                    lines.add((tag, ln))
        tot_lines += len(lines)
        tot_win += len(k) * (43 * 43 + 60)
        tot_k += len(k)
    per = 256 / nfr
    out = {"frames": nfr, "keypoints_per_frame": tot_k / nfr,
           "window_bytes_per_launch": tot_win * per, "line_floor_bytes_per_launch": tot_lines * LINE * per,
           "floor_over_window": tot_lines * LINE / tot_win}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
