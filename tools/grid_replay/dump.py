"""GPU box: dump the keypoint arrays the grid kernel consumes for the batch size at which the round-1 grid kernel
faulted (2 contexts x 256 frames of 1920x1080, 2000 features, bench.py config 3 frames), for the host ASan replay
of that kernel body (tools/grid_replay/replay.cc).  Output: gpurun_out/grid_replay.bin
  int32 B_total, frame_cap; float minX, minY, maxX, maxY, invW, invH; int32 counts[B_total];
  float xy[B_total * frame_cap * 2] (keypoint x, y as mvKeysUn; unused slots 0)."""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

import bench  # noqa: E402
from orbslam2_with_quadrics_amd import ORBextractor, _lib, synthetic  # noqa: E402
from orbslam2_with_quadrics_amd.extractor import KP_DTYPE  # noqa: E402

rows, cols, NF, B = 1080, 1920, 2000, 512
_, frames = bench._frames(synthetic, rows, cols, B, 0)
exs = [ORBextractor(NF, 1.2, 8, 20, 7) for _ in range(2)]
d = exs[0].device_alloc(frames.nbytes)
exs[0].h2d(d, frames)
for s, e in enumerate(exs):
    e.extract_batch_device(d + s * 256 * rows * cols, 256, cols, rows, cols, rows * cols)
for e in exs:
    e.synchronize()
cap = exs[0].batch_outputs()[3]
counts = np.zeros(B, np.int32)
xy = np.zeros((B, cap, 2), np.float32)
for s, e in enumerate(exs):
    kp, de, cn, cap_ = e.batch_outputs()
    c = np.zeros(256, np.int32)
    e.d2h(c, cn)
    k = np.zeros(256 * cap_, KP_DTYPE)
    e.d2h(k.view(np.uint8), kp)
    counts[s * 256:(s + 1) * 256] = c
    xy[s * 256:(s + 1) * 256, :, 0] = k["x"].reshape(256, cap_)
    xy[s * 256:(s + 1) * 256, :, 1] = k["y"].reshape(256, cap_)
g = _lib.GridGeom()
import ctypes as C  # noqa: E402

_lib.lib().orbgpu_grid_geom_for_image(cols, rows, C.byref(g))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "grid_replay.bin"), "wb") as f:
    f.write(struct.pack("<ii6f", B, cap, g.minX, g.minY, g.maxX, g.maxY, g.invW, g.invH))
    f.write(counts.tobytes())
    f.write(xy.tobytes())
print("frames", B, "frame_cap", cap, "max count", int(counts.max()))
