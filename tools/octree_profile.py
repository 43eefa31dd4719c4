"""Per-round timeline of the level-0 octree workgroup (test infrastructure).

python tools/octree_profile.py --build [--levels 0,1,..]   # here: variant libraries with OG_OCT_PROFILE=level+1
python tools/octree_profile.py --run [--batch B] [--shape kitti] [--levels 0,1,..]
    # GPU box: one B-frame (default 64) batch of 1080p (or KITTI 1241x376) frames; per-round cycles of the octree
    # workgroup of (frame 0, level l) for each level (one library per level)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LEVELS = [int(v) for v in sys.argv[sys.argv.index("--levels") + 1].split(",")] if "--levels" in sys.argv else [0]


def vlib(level):
    return os.path.join(ROOT, "orbslam2_with_quadrics_amd", "variants", f"liborbgpu_octprof{level}.so")


def build():
    from orbslam2_with_quadrics_amd import build_ext

    for lv in LEVELS:
        os.makedirs(os.path.dirname(vlib(lv)), exist_ok=True)
        print(build_ext.build(force=True, defines=[f"OG_OCT_PROFILE={lv + 1}"], out=vlib(lv)))


def run():
    if len(LEVELS) > 1:  # one process per library (the library is loaded once per process)
        import subprocess
        for lv in LEVELS:
            argv = [a for a in sys.argv[1:]]
            i = argv.index("--levels")
            argv[i + 1] = str(lv)
            subprocess.run([sys.executable, os.path.abspath(__file__), *argv], check=True)
        return
    os.environ["ORBGPU_LIB"] = vlib(LEVELS[0])
    import torch  # noqa: F401

    from orbslam2_with_quadrics_amd import ORBextractor, _lib, synthetic

    rows, cols = (376, 1241) if "kitti" in sys.argv else (1080, 1920)
    print(f"level {LEVELS[0]} of {cols}x{rows}")
    B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 64
    frames = np.stack([synthetic.frame(i % 8, rows, cols) for i in range(B)])
    ex = ORBextractor(2000, 1.2, 8, 20, 7)
    d = ex.device_alloc(frames.nbytes)
    ex.h2d(d, frames)
    for _ in range(3):
        ex.extract_batch_device(d, B, cols, rows, cols, rows * cols)
        ex.synchronize()
    buf = np.zeros(256, np.uint64)
    _lib.check(ex.ctx, _lib.lib().orbgpu_debug_octree_profile(ex.ctx, buf.ctypes.data, 256), "prof")
    t0 = int(buf[0])
    print("candidates", int(buf[1]), "final list", int(buf[5]))
    print("roots+remap  ", int(buf[2]) - t0, "cycles")
    r = 0
    prev = int(buf[2])
    while 8 + 4 * r < 256 and int(buf[8 + 4 * r]) > 0 and int(buf[8 + 4 * r]) >= t0:
        ts, info, tm, sa = (int(v) for v in buf[8 + 4 * r: 12 + 4 * r])
        nxt = int(buf[8 + 4 * (r + 1)]) if int(buf[8 + 4 * (r + 1)]) >= ts else int(buf[3])
        print(f"round {r}: Ln={info & 0xffffffff} mode={info >> 32} S={sa & 0xffffffff} A={sa >> 32} "
              f"plan={tm - ts} keypass={nxt - tm} cycles")
        r += 1
    print("tail (final best pass + output)", int(buf[4]) - int(buf[3]), "cycles; total", int(buf[4]) - t0)
    for r in range(min(r, 4)):  # plan phases of rounds 0-3: split set | S check | children scan | children+kept | barrier
        ts = int(buf[8 + 4 * r])
        marks = [int(buf[200 + 8 * r + j]) for j in range(5)]
        print(f"round {r} plan phases:", [m - p for m, p in zip(marks, [ts] + marks[:-1])])
    ex.device_free(d)


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    if "--run" in sys.argv:
        run()
