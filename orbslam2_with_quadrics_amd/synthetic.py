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


# ---- 3-D scenarios for the projection matchers -----------------
def rotation(rx: float, ry: float, rz: float) -> np.ndarray:
    """Rz @ Ry @ Rx (radians), float64."""
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def camera(cols: int, rows: int, Rcw=None, tcw=None, fx=None, fy=None, cx=None, cy=None, bf=None,
           scale_factor: float = 1.2, nlevels: int = 8) -> dict:
    """Frame camera snapshot (mRcw, mtcw, mOw = -Rcw^T tcw, K, mbf, mb, scale pyramid, image size) as float32."""
    Rcw = np.eye(3) if Rcw is None else np.asarray(Rcw, np.float64)
    tcw = np.zeros(3) if tcw is None else np.asarray(tcw, np.float64)
    fx = fx if fx is not None else 0.73 * cols
    fy = fy if fy is not None else fx
    cx = cx if cx is not None else cols / 2.0 - 0.37
    cy = cy if cy is not None else rows / 2.0 + 0.21
    bf = bf if bf is not None else 0.54 * fx
    R32 = Rcw.astype(np.float32)
    t32 = tcw.astype(np.float32)
    Ow = (-(R32.astype(np.float64).T @ t32.astype(np.float64))).astype(np.float32)
    return dict(Rcw=R32, tcw=t32, Ow=Ow, fx=np.float32(fx), fy=np.float32(fy), cx=np.float32(cx), cy=np.float32(cy),
                mbf=np.float32(bf), mb=np.float32(np.float32(bf) / np.float32(fx)), scale_factor=np.float32(scale_factor),
                nlevels=int(nlevels), cols=int(cols), rows=int(rows))


def last_frame_points(seed: int, kps, desc, cam_last: dict, depth=(2.0, 9.0), p_no_mp=0.1, p_outlier=0.05,
                      p_flip=0.03, n_obs_zero=0.2) -> dict:
    """LastFrame snapshot for SearchByProjection(Frame&, const Frame&): every keypoint back-projected at a
    random depth through the last camera (world positions), descriptors = keypoint descriptors with bits
    flipped at p_flip; some keypoints without map point, some outliers, some points with 0 observations."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(kps)
    z = rng.uniform(depth[0], depth[1], n)
    fx, fy, cx, cy = (float(cam_last[k]) for k in ("fx", "fy", "cx", "cy"))
    Xc = np.stack([(kps["x"].astype(np.float64) - cx) * z / fx, (kps["y"].astype(np.float64) - cy) * z / fy, z], 1)
    R = cam_last["Rcw"].astype(np.float64)
    t = cam_last["tcw"].astype(np.float64)
    Xw = (Xc - t) @ R  # R^T (Xc - t)
    flips = rng.random((n, 256)) < p_flip
    bits = np.unpackbits(np.asarray(desc, np.uint8).reshape(n, 32), axis=1, bitorder="little") ^ flips
    d = np.packbits(bits.astype(np.uint8), axis=1, bitorder="little")
    return dict(kps=np.ascontiguousarray(kps), has_mp=(rng.random(n) >= p_no_mp).astype(np.uint8),
                outlier=(rng.random(n) < p_outlier).astype(np.uint8), pos=Xw.astype(np.float32),
                n_obs=np.where(rng.random(n) < n_obs_zero, 0, rng.integers(1, 6, n)).astype(np.int32),
                desc=np.ascontiguousarray(d))


def local_map_points(seed: int, m: int, cam: dict, nlevels: int = 8, scale_factor: float = 1.2) -> dict:
    """Map-point geometry for Frame::isInFrustum: points spread over a frustum-shaped volume of `cam`
    (plus points behind it and outside the image), unit normals from a reference camera centre, and the
    distance bounds UpdateNormalAndDepth would set (mfMaxDistance = dist * sf^level, mfMinDistance =
    mfMaxDistance / sf^(nlevels-1))."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = (float(cam[k]) for k in ("fx", "fy", "cx", "cy"))
    W, H = cam["cols"], cam["rows"]
    z = rng.uniform(-1.0, 12.0, m)
    u = rng.uniform(-0.1 * W, 1.1 * W, m)
    v = rng.uniform(-0.1 * H, 1.1 * H, m)
    Xc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    R = cam["Rcw"].astype(np.float64)
    t = cam["tcw"].astype(np.float64)
    Xw = (Xc - t) @ R
    ref_c = -(R.T @ t) + rng.normal(0, 0.6, (m, 3))
    nrm = Xw - ref_c
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm = np.where(rng.random((m, 1)) < 0.1, -nrm, nrm)  # some points seen from the other side
    dref = np.linalg.norm(Xw - ref_c, axis=1) * rng.uniform(0.7, 1.4, m)
    lvl = rng.integers(0, nlevels, m)
    mx = dref * scale_factor ** lvl
    mn = mx / scale_factor ** (nlevels - 1)
    return dict(pos=Xw.astype(np.float32), normal=nrm.astype(np.float32), max_dist=mx.astype(np.float32),
                min_dist=mn.astype(np.float32))


def keyframe_points(seed: int, kps, desc, cam_kf: dict, depth=(2.0, 9.0), p_invalid=0.1, p_flip=0.03,
                    scale_factor: float = 1.2, nlevels: int = 8) -> dict:
    """KeyFrame snapshot for the relocalisation SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist): the
    keyframe's keypoints back-projected at random depths (world positions), descriptors with bits flipped,
    the distance bounds UpdateNormalAndDepth sets (mfMaxDistance = dist * sf^octave), and a validity flag
    (map point present, not bad, not already found)."""
    lf = last_frame_points(seed, kps, desc, cam_kf, depth, p_no_mp=0.0, p_outlier=0.0, p_flip=p_flip)
    rng = np.random.Generator(np.random.PCG64(seed + 77))
    n = len(kps)
    Ow = cam_kf["Ow"].astype(np.float64)
    d = np.linalg.norm(lf["pos"].astype(np.float64) - Ow, axis=1) * rng.uniform(0.85, 1.15, n)
    mx = d * scale_factor ** np.asarray(kps["octave"], np.float64)
    mn = mx / scale_factor ** (nlevels - 1)
    return dict(kps=lf["kps"], valid=(rng.random(n) >= p_invalid).astype(np.uint8), pos=lf["pos"],
                max_dist=mx.astype(np.float32), min_dist=mn.astype(np.float32), desc=lf["desc"])


def depth_u16(seed: int, height: int, width: int, p_hole: float = 0.08) -> np.ndarray:
    """TUM-style raw depth (uint16, DepthMapFactor 5000 => 0.5-8 m as 2500-40000): smooth slanted planes
    plus blocky objects, with missing-depth holes (0)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
    d = 2.0 + 3.0 * yy / height + 0.5 * np.sin(xx / 57.0)
    for _ in range(20):
        w, h = int(rng.integers(20, 200)), int(rng.integers(20, 200))
        x, y = int(rng.integers(0, width)), int(rng.integers(0, height))
        d[y:y + h, x:x + w] = rng.uniform(0.5, 8.0)
    raw = np.clip(np.rint(d * 5000.0), 0, 65535).astype(np.uint16)
    raw[rng.random((height, width)) < p_hole] = 0
    return raw


def vocabulary(seed: int, k: int = 10, L: int = 6, p_short: float = 0.02, p_stop: float = 0.01,
               scoring: int = 0, weighting: int = 0) -> dict:
    """A DBoW2 vocabulary of ORBvoc.txt's shape (k=10, L=6, L1_NORM, TF_IDF by default) with random node
    descriptors, in the node order of DBoW2's depth-first HKmeansStep (children of a node are contiguous,
    created before the recursion into them).  A few nodes stop early (leaves above level L, as clusters with
    <= 1 training feature do) and a few words are stopped (weight 0).  The real vocabulary is a 40 MB
    download absent offline; the transform's semantics do not depend on its contents."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parent, leaf, depth = [], [], []

    def grow(pid, level):  # iterative DFS with the same order as the recursion
        stack = [(pid, level)]
        while stack:
            p, lv = stack.pop()
            first = len(parent) + 1
            for _ in range(k):
                parent.append(p)
                depth.append(lv)
                leaf.append(True)
            ids = list(range(first, first + k))
            kids = []
            if lv < L:
                for nid in ids:
                    if rng.random() >= p_short:
                        leaf[nid - 1] = False
                        kids.append((nid, lv + 1))
            stack.extend(reversed(kids))

    grow(0, 1)
    n = len(parent)
    is_leaf = np.array(leaf, np.uint8)
    weight = np.where(is_leaf == 1, rng.uniform(0.5, 9.0, n), 0.0)
    weight[(is_leaf == 1) & (rng.random(n) < p_stop)] = 0.0
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, parent=np.array(parent, np.int32), is_leaf=is_leaf,
                desc=rng.integers(0, 256, size=(n, 32), dtype=np.uint8), weight=weight)


def write_vocabulary_text(voc: dict, path: str):
    """DBoW2 text format (TemplatedVocabulary::saveToTextFile / ORBvoc.txt): header 'k L scoring weighting',
    then per node 'parent isLeaf d0 .. d31 weight'."""
    with open(path, "w") as fp:
        fp.write(f"{voc['k']} {voc['L']} {voc['scoring']} {voc['weighting']}\n")
        for p, lf, d, w in zip(voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"]):
            fp.write(f"{int(p)} {int(lf)} " + " ".join(str(int(x)) for x in d) + f" {float(w)!r}\n")


def color_frame(frame_id: int, height: int, width: int, alpha: bool = False) -> np.ndarray:
    """A colour (RGB or RGBA, uint8) rendering of frame `frame_id`: the gray frame with seeded per-pixel
    channel offsets, so RGB -> gray and BGR -> gray give different images."""
    g = frame(frame_id, height, width).astype(np.int16)
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + 31 * frame_id + 5))
    off = rng.integers(-24, 25, size=(height, width, 3), dtype=np.int16)
    rgb = np.clip(g[..., None] + off, 0, 255).astype(np.uint8)
    if alpha:
        rgb = np.concatenate([rgb, rng.integers(0, 256, size=(height, width, 1), dtype=np.uint8)], axis=2)
    return np.ascontiguousarray(rgb)


def write_tum_rgbd_sequence(root: str, n: int, height: int = 480, width: int = 640, t0: float = 1305031102.175304):
    """A TUM RGB-D sequence directory (rgb/<t>.png colour, depth/<t>.png 16-bit, associations.txt in the
    format of Examples/RGB-D/associations/*.txt) written with Pillow; returns the association path."""
    import os

    from PIL import Image

    os.makedirs(os.path.join(root, "rgb"), exist_ok=True)
    os.makedirs(os.path.join(root, "depth"), exist_ok=True)
    lines = []
    for i in range(n):
        t = t0 + i / 30.0
        td = t - 0.0149
        name, dname = f"rgb/{t:.6f}.png", f"depth/{td:.6f}.png"
        Image.fromarray(color_frame(i, height, width), "RGB").save(os.path.join(root, name))
        Image.fromarray(depth_u16(SEED_BASE + i, height, width)).save(os.path.join(root, dname))
        lines.append(f"{t:.6f} {name} {td:.6f} {dname}")
    path = os.path.join(root, "associations.txt")
    with open(path, "w") as fp:
        fp.write("\n".join(lines) + "\n")
    return path
