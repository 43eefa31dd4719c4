"""Stage-by-stage GPU-vs-oracle comparison (diagnostic; run on the GPU box).

python tools/gpu_parity_debug.py [H W NFEAT] -- prints the first mismatch of every stage.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
from orbslam2_with_quadrics_amd import ORBextractor, synthetic  # noqa: E402


def main():
    H, W, NF = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (480, 640, 1000)
    img = synthetic.frame(3, H, W)
    t = time.time()
    ex = ORBextractor(NF, 1.2, 8, 20, 7)
    k, d = ex(img)
    print(f"gpu extract {time.time() - t:.3f}s n={len(k)}", flush=True)
    t = time.time()
    k, d = ex(img)
    print(f"gpu extract (warm) {time.time() - t:.4f}s n={len(k)}", flush=True)
    oe = O.OracleExtractor(NF, 1.2, 8, 20, 7)
    t = time.time()
    ko, do = oe(img)
    print(f"oracle extract {time.time() - t:.3f}s n={len(ko)}", flush=True)
    ok = True
    for l in range(8):
        g = ex.level(l)
        o = oe.level(l)
        if g.shape != o.shape or not np.array_equal(g, o):
            diff = np.argwhere(g != o) if g.shape == o.shape else None
            print(f"level {l}: PYRAMID MISMATCH shapes {g.shape} {o.shape} first {diff[:5] if diff is not None else ''}")
            ok = False
            break
    print("pyramid ok" if ok else "pyramid BAD", flush=True)
    for l in range(8):
        c = ex.debug_candidates(0, l)
        gx = (c & 0xFFFF).astype(np.int64)
        gy = ((c >> 16) & 0xFFFF).astype(np.int64)
        gr = ((c >> 32) & 0xFF).astype(np.int64)
        oxy, orr = oe.candidates(l)
        gs = set(zip(gx.tolist(), gy.tolist(), gr.tolist()))
        os_ = set(zip(oxy[:, 0].astype(int).tolist(), oxy[:, 1].astype(int).tolist(), orr.astype(int).tolist()))
        if gs != os_:
            print(f"level {l}: CANDIDATES differ gpu={len(gs)} oracle={len(os_)} "
                  f"gpu-only={sorted(gs - os_)[:5]} oracle-only={sorted(os_ - gs)[:5]}")
            ok = False
        else:
            print(f"level {l}: candidates equal ({len(gs)})")
    # octree outputs: oracle keypoints of level l in order (before scaling) vs GPU octree list
    for l in range(8):
        gx, gy, gr = ex.debug_octree(0, l)
        sel = ko["octave"] == l
        s = 1.0 if l == 0 else float(oe.tables()["scale"][l])
        n_o = int(sel.sum())
        if len(gx) != n_o:
            print(f"level {l}: OCTREE count gpu={len(gx)} oracle={n_o}")
            ok = False
            continue
        gxs = gx.astype(np.float32) * np.float32(s) if l else gx.astype(np.float32)
        gys = gy.astype(np.float32) * np.float32(s) if l else gy.astype(np.float32)
        bad = np.nonzero((gxs != ko["x"][sel]) | (gys != ko["y"][sel]) | (gr != ko["response"][sel]))[0]
        if len(bad):
            i = bad[0]
            print(f"level {l}: OCTREE order/content mismatch at {i}: gpu ({gx[i]},{gy[i]},{gr[i]}) "
                  f"oracle ({ko['x'][sel][i]},{ko['y'][sel][i]},{ko['response'][sel][i]}); {len(bad)} bad")
            ok = False
        else:
            print(f"level {l}: octree equal ({n_o})")
    if len(k) == len(ko):
        for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
            bad = np.nonzero(k[f] != ko[f])[0]
            if len(bad):
                i = bad[0]
                print(f"field {f}: {len(bad)} mismatches, first {i}: gpu {k[i]} oracle {ko[i]}")
                ok = False
        bad = np.nonzero((d != do).any(1))[0]
        if len(bad):
            i = bad[0]
            print(f"descriptors: {len(bad)} rows differ; first {i}: gpu {d[i][:8]} oracle {do[i][:8]}")
            ok = False
    else:
        print(f"keypoint count gpu={len(k)} oracle={len(ko)}")
        ok = False
    print("ALL OK" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
