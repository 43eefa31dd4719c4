"""Search a test image on which the rBRIEF rotation's FMA and non-FMA forms give different descriptors
(ORBGPU_SEM_BRIEF_NOFMA vs the default, src/ORBextractor.cc:118-120).  TEST-FIXTURE GENERATOR: uses the oracle.

The two forms round differently only when x*b + y*a lies within ~1 ulp of a .5 boundary: ~1 angle in 20000,
so natural frames almost never separate them.  Recipe: a flat textured image with 24 bright squares whose
top-left corner pixel is the unique FAST maximum; for each such keypoint, find IC-angle moments (m01, m10)
within +-250 of its own whose fastAtan2 angle separates the two forms for some pattern point, then reach
those moments with low-contrast "dust" (|delta| <= 7, below any FAST threshold) on the pixels 6..15 px
above and left of the corner, which move m01 and m10 independently (src/ORBextractor.cc:77-104).
Output: tests/golden/semantics_probe.json (image seed, dust list, oracle hashes of both forms).

    PYTHONPATH=.:oracle python3 tools/find_fma_probe.py
"""
import ctypes as C
import hashlib
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "golden")]
import oracle_py as O  # noqa: E402
from make_golden import fma_probe_base, fma_probe_image  # noqa: E402

F = np.float32
UMAX = [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
_txt = open(os.path.join(ROOT, "oracle", "orb_pattern.inc")).read()
PAT = np.array([int(v) for v in re.findall(r"-?\d+", _txt[_txt.index("{") + 1:_txt.index("};")])]).reshape(256, 4)
K = F(180.0 / 3.14159265358979323846)
P1, P3, P5, P7 = (F(F(c) * K) for c in (0.9997878412794807, -0.3258083974640975, 0.1555786518463281,
                                        -0.04432655554792128))
libm = C.CDLL("libm.so.6")
libm.sincosf.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]


def fast_atan2(y, x):
    """cv::fastAtan2 (oracle/oo_math.h) vectorised in float32; checked against the oracle below."""
    y, x = y.astype(F), x.astype(F)
    ax, ay = np.abs(x), np.abs(y)
    eps = F(2.220446049250313e-16)
    big = ax >= ay
    c = np.where(big, ay / (ax + eps), ax / (ay + eps)).astype(F)
    c2 = (c * c).astype(F)
    a = ((((P7 * c2 + P5) * c2 + P3) * c2 + P1) * c).astype(F)
    a = np.where(big, a, F(90) - a).astype(F)
    a = np.where(x < 0, F(180) - a, a).astype(F)
    return np.where(y < 0, F(360) - a, a).astype(F)


def separating(angles):
    """True where some pattern point rounds differently under fma(x,b,y*a) and x*b + y*a."""
    xs = np.concatenate([PAT[:, 0], PAT[:, 2]]).astype(F)[None, :]
    ys = np.concatenate([PAT[:, 1], PAT[:, 3]]).astype(F)[None, :]
    A, B = np.empty(len(angles), F), np.empty(len(angles), F)
    s, c = C.c_float(), C.c_float()
    fpi = F(3.14159265358979323846 / 180.0)
    for i, ang in enumerate(angles):
        libm.sincosf(F(F(ang) * fpi), C.byref(s), C.byref(c))
        B[i], A[i] = s.value, c.value
    a, b = A[:, None], B[:, None]
    ya, yb = (ys * a).astype(F), (ys * b).astype(F)
    # x*b is exact in double; the double sum then rounds once to float (the candidates are re-checked by the
    # oracle extraction, so a rare double-rounding miss only costs a candidate)
    row_f = (xs.astype(np.float64) * b + ya.astype(np.float64)).astype(F)
    col_f = (xs.astype(np.float64) * a - yb.astype(np.float64)).astype(F)
    row_n = ((xs * b).astype(F) + ya).astype(F)
    col_n = ((xs * a).astype(F) - yb).astype(F)
    return ((np.rint(row_f) != np.rint(row_n)) | (np.rint(col_f) != np.rint(col_n))).any(1)


def moments(img, x, y):
    m01 = m10 = 0
    for v in range(-15, 16):
        for u in range(-UMAX[abs(v)], UMAX[abs(v)] + 1):
            m10 += u * int(img[y + v, x + u])
            m01 += v * int(img[y + v, x + u])
    return m01, m10


def solve(target, coords, lim=7):
    """Deltas |d| <= lim, one per coordinate, with sum(c * d) == target (min sum |d|), or None."""
    states = {0: (0, [])}
    for c in coords:
        ns = {}
        for sm, (cost, ds) in states.items():
            for d in range(-lim, lim + 1):
                t, nc = sm + c * d, cost + abs(d)
                if t not in ns or ns[t][0] > nc:
                    ns[t] = (nc, ds + [d])
        states = ns
    return states[target][1] if target in states else None


def main(seed=0, R=250):
    rng = np.random.default_rng(7)
    ys, xs = rng.integers(-300000, 300000, 2000), rng.integers(-300000, 300000, 2000)
    em = fast_atan2(ys, xs)
    assert all(F(O.fastatan2(float(ys[i]), float(xs[i]))) == em[i] for i in range(2000))
    img, corners = fma_probe_base(seed)
    k, _ = O.OracleExtractor(1000)(img)
    level0 = {(int(p["x"]), int(p["y"])): p for p in k[k["octave"] == 0]}
    dm10, dm01 = (g.ravel() for g in np.meshgrid(np.arange(-R, R + 1), np.arange(-R, R + 1)))
    mods = []
    for (x, y) in corners:
        if (x, y) not in level0:
            continue
        m01, m10 = moments(img, x, y)
        assert F(O.fastatan2(m01, m10)) == level0[(x, y)]["angle"]
        ang = fast_atan2(m01 + dm01, m10 + dm10)
        ua = np.unique(ang)
        hits = np.concatenate([ua[s:s + 4000][separating(ua[s:s + 4000])] for s in range(0, len(ua), 4000)])
        if not len(hits):
            continue
        idx = np.nonzero(ang == hits[0])[0]
        for i in sorted(idx, key=lambda i: abs(dm01[i]) + abs(dm10[i]))[:50]:
            s01 = solve(int(dm01[i]), [-v for v in range(6, 16)])
            s10 = solve(int(dm10[i]), [-u for u in range(6, 16)])
            if s01 is None or s10 is None:
                continue
            mods += [(x, y - (j + 6), d) for j, d in enumerate(s01) if d]
            mods += [(x - (j + 6), y, d) for j, d in enumerate(s10) if d]
            print(f"corner ({x},{y}): target angle {hits[0]} via dm01 {dm01[i]} dm10 {dm10[i]}", flush=True)
            break
    im = fma_probe_image(seed, mods)
    ka, da = O.OracleExtractor(1000)(im)
    kb, db = O.OracleExtractor(1000, semantics=0x20)(im)
    assert ka.tobytes() == kb.tobytes()
    differ = int((da != db).any(1).sum())
    print("descriptors that differ between the FMA and non-FMA rotation:", differ)
    assert differ > 0
    out = dict(generator="tools/find_fma_probe.py (oracle)", seed=seed, mods=[list(map(int, m)) for m in mods],
               nfeatures=1000, n=int(len(ka)), descriptors_differing=differ,
               kps_sha256=hashlib.sha256(ka.tobytes()).hexdigest(),
               desc_fma_sha256=hashlib.sha256(da.tobytes()).hexdigest(),
               desc_nofma_sha256=hashlib.sha256(db.tobytes()).hexdigest())
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "semantics_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
