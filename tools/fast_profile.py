"""Per-phase timeline of the FAST workgroups under full load (diagnostic, test infrastructure).

python tools/fast_profile.py --build          # here: variant library with OG_FAST_PROFILE=1
python tools/fast_profile.py --run [--batch B] [--name N] # GPU box (--name: variants/liborbgpu_<N>.so)
                                               #: B 1080p frames (default 256); prints the mean cycles of each
                                               # phase over the middle frame's blocks (s_memtime, shader clock)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VNAME = sys.argv[sys.argv.index("--name") + 1] if "--name" in sys.argv else "fastprof"
VLIB = os.path.join(ROOT, "orbslam2_with_quadrics_amd", "variants", f"liborbgpu_{VNAME}.so")
PHASES = ["roi+zero", "stage1 quick", "stage2 score", "stage3 nms+counts", "reservation", "emission"]


def build():
    from orbslam2_with_quadrics_amd import build_ext

    os.makedirs(os.path.dirname(VLIB), exist_ok=True)
    print(build_ext.build(force=True, defines=["OG_FAST_PROFILE=1"], out=VLIB))


def run():
    os.environ["ORBGPU_LIB"] = VLIB
    import torch  # noqa: F401

    from orbslam2_with_quadrics_amd import ORBextractor, _lib, synthetic

    rows, cols = 1080, 1920
    B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 256
    frames = np.stack([synthetic.frame(i % 8, rows, cols) for i in range(B)])
    ex = ORBextractor(2000, 1.2, 8, 20, 7)
    d = ex.device_alloc(frames.nbytes)
    ex.h2d(d, frames)
    for _ in range(3):
        ex.extract_batch_device(d, B, cols, rows, cols, rows * cols)
        ex.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    _lib.check(ex.ctx, _lib.lib().orbgpu_debug_fast_profile(ex.ctx, buf.ctypes.data, buf.size), "prof")
    t = buf.reshape(-1, 8).astype(np.int64)
    t = t[t[:, 0] > 0]
    ns, lev = t[:, 7] & 0xffffffff, t[:, 7] >> 32
    dt = np.diff(t[:, :7], axis=1)
    life = t[:, 6] - t[:, 0]
    print(f"blocks {len(t)}  mean lifetime {life.mean():.0f} cycles (median {np.median(life):.0f})")
    for i, name in enumerate(PHASES):
        print(f"  {name:20s} mean {dt[:, i].mean():8.0f}  median {np.median(dt[:, i]):8.0f}  "
              f"share {dt[:, i].sum() / life.sum():.3f}")
    for l in range(8):
        m = lev == l
        if m.any():
            print(f"  level {l}: blocks {m.sum():5d}  survivors/block {ns[m].mean():6.0f}  lifetime {life[m].mean():7.0f}")
    span = t[:, 6].max() - t[:, 0].min()
    print(f"frame span {span} cycles")
    ex.device_free(d)


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    if "--run" in sys.argv:
        run()
