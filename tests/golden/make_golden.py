"""Regenerate the committed golden fixtures (run from the repo root in the build container).

sincosf.json        : (angle, sinf, cosf) triples from the host libm's sincosf (glibc 2.35, FMA variant)
                      at angles the ORB path produces (fastAtan2 outputs * pi/180) plus edge cases.
extract_golden.json : the oracle's ORB extraction of seeded synthetic frames (hashes + first rows).
                      This pins the oracle against regressions; it is NOT a reference-binary output
                      (the reference cannot be built here -- DESIGN.md §4).
match_golden.json   : oracle SearchForInitialization on a seeded 1080p pair (match vector hash).
"""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_py as O  # noqa: E402
from orbslam2_with_quadrics_amd import synthetic  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def sincos_vectors():
    libm = C.CDLL("libm.so.6")
    libm.sincosf.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    rng = np.random.default_rng(11)
    angles = [0.0, 1e-30, 2.4e-4, 0.7853981, 0.78539819, 1.5707963, 3.1415927, 4.712389, 6.2831855, 6.2831849]
    for _ in range(400):
        m01, m10 = (float(v) for v in rng.integers(-300000, 300000, 2))
        a = O.fastatan2(m01, m10)
        angles.append(float(np.float32(a) * np.float32(np.pi / 180.0)))
    vecs = []
    for a in angles:
        s, c = C.c_float(), C.c_float()
        libm.sincosf(np.float32(a), C.byref(s), C.byref(c))
        vecs.append([float(np.float32(a)), s.value, c.value])
    json.dump({"source": "host libm sincosf (glibc 2.35 x86_64)", "vectors": vecs},
              open(os.path.join(OUT, "sincosf.json"), "w"), indent=0)


def extract_cases():
    cases = []
    for fid, rows, cols, nf in [(3, 480, 640, 1000), (5, 376, 1241, 2000), (7, 1080, 1920, 2000)]:
        img = synthetic.frame(fid, rows, cols)
        k, d = O.OracleExtractor(nf)(img)
        head = np.stack([k["x"], k["y"], k["angle"], k["response"]], 1)[:12].astype(np.float64).tolist()
        cases.append(dict(frame_id=fid, rows=rows, cols=cols, nfeatures=nf, n=int(len(k)),
                          image_sha256=hashlib.sha256(img.tobytes()).hexdigest(),
                          kps_sha256=hashlib.sha256(k.tobytes()).hexdigest(),
                          desc_sha256=hashlib.sha256(d.tobytes()).hexdigest(), head=head))
    json.dump({"generator": "oracle/orb_oracle.c via tests/golden/make_golden.py", "cases": cases},
              open(os.path.join(OUT, "extract_golden.json"), "w"), indent=1)


def match_cases():
    cases = []
    for pid, rows, cols, nf in [(21, 1080, 1920, 2000), (22, 480, 640, 1000)]:
        f1, f2 = synthetic.frame_pair(pid, rows, cols)
        ex = O.OracleExtractor(nf)
        k1, d1 = ex(f1)
        k2, d2 = ex(f2)
        sf = ex.tables()["scale"]
        F1 = O.OracleFrame(k1, d1, cols, rows, sf)
        F2 = O.OracleFrame(k2, d2, cols, rows, sf)
        prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
        n, m12, prev2 = O.search_for_initialization(F1, F2, prev, 0.9, True, 100)
        cases.append(dict(pair_id=pid, rows=rows, cols=cols, nfeatures=nf, nmatches=int(n),
                          matches_sha256=hashlib.sha256(m12.astype(np.int32).tobytes()).hexdigest(),
                          prev_sha256=hashlib.sha256(prev2.tobytes()).hexdigest()))
    json.dump({"generator": "oracle SearchForInitialization via tests/golden/make_golden.py", "cases": cases},
              open(os.path.join(OUT, "match_golden.json"), "w"), indent=1)


if __name__ == "__main__":
    O.build()
    sincos_vectors()
    extract_cases()
    match_cases()
    print("golden fixtures written to", OUT)
