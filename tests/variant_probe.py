"""Digest of one small run of the feature path with the library ORBGPU_LIB names (test infrastructure for
tests/test_gpu_variants.py; needs a GPU).  Prints one JSON line: sha256 of the keypoints + descriptors of a 1080p and a
KITTI-shaped device batch (every FAST / octree / describe / pyramid path of both shapes), and of the
SearchForInitialization matches of the 1080p batch against its first frame."""
import ctypes as C
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime in the process)

from orbslam2_with_quadrics_amd import ORBextractor, _lib, synthetic  # noqa: E402


def batch_digest(rows, cols, nf, B, seed):
    frames = np.stack([synthetic.frame(seed + i, rows, cols) for i in range(B)])
    ex = ORBextractor(nf, 1.2, 8, 20, 7)
    d = ex.device_alloc(frames.nbytes)
    try:
        ex.h2d(d, frames)
        ex.extract_batch_device(d, B, cols, rows, cols, rows * cols)
        h = hashlib.sha256()
        for b in range(B):
            k, desc = ex.batch_download(b)
            h.update(k.tobytes())
            h.update(desc.tobytes())
        out = {"kd": h.hexdigest()}
        if rows == 1080:
            _, _, _, cap = ex.batch_outputs()
            L = _lib.lib()
            prev = ex.device_alloc(B * cap * 8)
            m12 = ex.device_alloc(B * cap * 4)
            nm = ex.device_alloc(B * 4)
            try:
                _lib.check(ex.ctx, L.orbgpu_prev_matched_from_frame(ex.ctx, 0, ex.ctx, C.c_void_p(prev)), "prev")
                g = _lib.GridGeom()
                _lib.check(ex.ctx, L.orbgpu_grid_geom_for_image(cols, rows, C.byref(g)), "grid")
                _lib.check(ex.ctx, L.orbgpu_search_for_initialization_batch(
                    ex.ctx, 0, ex.ctx, g, 0.9, 1, 100, C.c_void_p(prev), C.c_void_p(m12), C.c_void_p(nm)), "init")
                a = np.zeros(B * cap, np.int32)
                n = np.zeros(B, np.int32)
                ex.d2h(a, m12)
                ex.d2h(n, nm)
                out["init"] = hashlib.sha256(a.tobytes() + n.tobytes()).hexdigest()
                out["nmatches"] = int(n.sum())
            finally:
                for p in (prev, m12, nm):
                    ex.device_free(p)
        return out
    finally:
        ex.device_free(d)


def main():
    res = {"hd": batch_digest(1080, 1920, 2000, 3, 40), "kitti": batch_digest(376, 1241, 2000, 3, 50),
           "vga": batch_digest(480, 640, 1000, 2, 60)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
