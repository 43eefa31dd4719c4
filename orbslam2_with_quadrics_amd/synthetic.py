"""Deterministic synthetic grey frames for the ORB hot path.

No dataset is available offline, so every test and bench input is generated here from a seed:
smoothed value-noise background + R random axis-aligned rectangles (R = 400 at 1920x1080, scaled by
area) + per-pixel N(0, 6) noise, clamped to u8.  A "scene" is rendered larger than the frame so that
camera motion can be emulated by cropping at an offset (config 3: F2 = F1 shifted by (+7, +3) with
fresh noise; config 4: right image = left shifted by a band-wise disparity).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x0B5EED00


def make_scene(seed: int, height: int, width: int, margin: int = 64) -> np.ndarray:
    """float32 scene of shape (height + 2*margin, width + 2*margin)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    H, W = height + 2 * margin, width + 2 * margin
    cell = 48
    gh, gw = H // cell + 2, W // cell + 2
    grid = rng.uniform(40.0, 200.0, size=(gh, gw)).astype(np.float32)
    ys = np.arange(H, dtype=np.float32) / cell
    xs = np.arange(W, dtype=np.float32) / cell
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    fy = fy * fy * (3 - 2 * fy)
    fx = fx * fx * (3 - 2 * fx)
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    img = (g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy
    nrect = max(8, int(round(400 * (H * W) / (1920.0 * 1080.0))))
    for _ in range(nrect):
        rw = int(rng.integers(6, 140))
        rh = int(rng.integers(6, 140))
        x = int(rng.integers(-rw // 2, W))
        y = int(rng.integers(-rh // 2, H))
        val = float(rng.uniform(0, 255))
        img[max(y, 0):max(y + rh, 0), max(x, 0):max(x + rw, 0)] = val
    return img.astype(np.float32)


def render(scene: np.ndarray, height: int, width: int, dx: int = 0, dy: int = 0,
           noise_seed: int = 0, noise_sigma: float = 6.0, margin: int = 64) -> np.ndarray:
    """Crop the scene at (margin+dy, margin+dx), add N(0, sigma) noise, clamp to u8 (C-contiguous)."""
    rng = np.random.Generator(np.random.PCG64(noise_seed))
    crop = scene[margin + dy: margin + dy + height, margin + dx: margin + dx + width]
    noisy = crop + rng.normal(0.0, noise_sigma, size=crop.shape).astype(np.float32)
    return np.ascontiguousarray(np.clip(np.rint(noisy), 0, 255).astype(np.uint8))


def frame(frame_id: int, height: int, width: int, dx: int = 0, dy: int = 0) -> np.ndarray:
    """Frame `frame_id` of the synthetic stream: scene seed = SEED_BASE + frame_id."""
    scene = make_scene(SEED_BASE + frame_id, height, width)
    return render(scene, height, width, dx, dy, noise_seed=SEED_BASE + 7919 * frame_id + 1)


def frame_pair(pair_id: int, height: int, width: int, shift=(7, 3)):
    """(F1, F2): F2 = F1's scene shifted by `shift` = (+x, +y) pixels with fresh noise (config 3)."""
    scene = make_scene(SEED_BASE + pair_id, height, width)
    f1 = render(scene, height, width, 0, 0, noise_seed=SEED_BASE + 7919 * pair_id + 1)
    f2 = render(scene, height, width, shift[0], shift[1], noise_seed=SEED_BASE + 7919 * pair_id + 2)
    return f1, f2


def flat(height: int, width: int, value: int = 128) -> np.ndarray:
    return np.full((height, width), value, dtype=np.uint8)


def pure_noise(seed: int, height: int, width: int) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(0, 256, size=(height, width), dtype=np.uint8)


def stereo_pair(pair_id: int, height: int, width: int, band: int = 64, dmin: int = 4, dmax: int = 40):
    """(left, right) rectified pair (config 4): the right image sees the scene point of left column x at
    column x - d, with d constant inside horizontal bands of `band` rows and drawn in [dmin, dmax]."""
    scene = make_scene(SEED_BASE + pair_id, height, width)
    left = render(scene, height, width, 0, 0, noise_seed=SEED_BASE + 7919 * pair_id + 1)
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 104729 * pair_id + 3))
    nb = (height + band - 1) // band
    disp = rng.integers(dmin, dmax + 1, size=nb)
    m = 64
    shifted = np.empty((height, width), np.float32)
    for b in range(nb):
        y0, y1 = b * band, min((b + 1) * band, height)
        d = int(disp[b])
        shifted[y0:y1] = scene[m + y0:m + y1, m + d:m + d + width]
    noise = np.random.Generator(np.random.PCG64(SEED_BASE + 7919 * pair_id + 2))
    noisy = shifted + noise.normal(0.0, 6.0, size=shifted.shape).astype(np.float32)
    right = np.ascontiguousarray(np.clip(np.rint(noisy), 0, 255).astype(np.uint8))
    return left, right, disp
