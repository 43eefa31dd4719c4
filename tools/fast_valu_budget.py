"""Per-phase VALU budget of og_fast_quad_kernel at config 3 (analysis only, CPU): the ISA's static VALU per phase
and per loop body (tools/valu_budget.py, weighted 2 / 4 cycles) times each phase's trip counts, which come from the
kernel's own block plan replayed on a bench frame's pyramid (the oracle's levels):

  phase 0  ROI staging + score-map zeroing      once per wave
  phase 1  stage 1, quick test (4 px per lane)  ceil(units / 8) iterations per wave, units = 2 ceil(dh / 8)
  phase 2  stage 2, exact score per survivor    ceil((ns - 64 w) / 512) iterations of wave w
  phase 3  stage 3, NMS per 64-entry chunk      same chunks
  phase 4  per-cell fallback bookkeeping, reservation   once per wave
  phase 5  emission per 64-entry chunk          same chunks

The block plan is the kernel's (orbgpu_capi.cpp build_plan: 30-px cells, blocks of up to 2 x 2 cells with
detection width <= 64 and height <= 80); ns = pixels passing the quick test at t_q = min(iniThFAST, minThFAST).
The total per wave is compared with the PMC SQ_INSTS_VALU / SQ_WAVES of the same kernel.

    bash tools/isa.sh orb_extract.hip && python tools/fast_valu_budget.py /tmp/isa_orb_extract.s [--pmc file.json] \
        [--weights '%bb.7=0,%bb.17=0.125,%bb.29=0']

--weights scales a basic block's count by the fraction of its executions a wave actually takes (block names from
tools/valu_budget.py's listing of the same .s): e.g. the odd-pitch ROI path (never at 1080p), the ROI's second row
store (only the wave holding ROI rows 64+), the second polarity's score (both polarities pass: 37 of 256k pixels).
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]

import valu_budget as VB  # noqa: E402

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def quick_pass(img, t):
    """cv::FAST's opposite-pair necessary condition at threshold t, for every pixel with a full circle."""
    H, W = img.shape
    v = img[3:H - 3, 3:W - 3].astype(np.int32)
    c = np.stack([img[3 + dy:H - 3 + dy, 3 + dx:W - 3 + dx].astype(np.int32) for dx, dy in CIRCLE])
    dmax = np.max(np.stack([np.minimum(c[k], c[k + 8]) for k in range(8)]), 0)
    bmin = np.min(np.stack([np.maximum(c[k], c[k + 8]) for k in range(8)]), 0)
    out = np.zeros((H, W), bool)
    out[3:H - 3, 3:W - 3] = (dmax < v - t) | (bmin > v + t)
    return out


def blocks_of_level(h, w):
    """(x0, y0, dw, dh) of the level's FAST blocks, as build_plan lays them out (EDGE 19, cells of 30 px)."""
    minB, maxBX, maxBY = 16, w - 16, h - 16
    width, height = float(maxBX - minB), float(maxBY - minB)
    nCols, nRows = int(width / 30), int(height / 30)
    wCell, hCell = math.ceil(width / nCols), math.ceil(height / nRows)
    cells = {}
    for i in range(nRows):
        iniY = minB + i * hCell
        maxY = min(iniY + hCell + 6, maxBY)
        if iniY >= maxBY - 3:
            continue
        for j in range(nCols):
            iniX = minB + j * wCell
            maxX = min(iniX + wCell + 6, maxBX)
            if iniX >= maxBX - 6 or maxX - iniX - 6 <= 0 or maxY - iniY - 6 <= 0:
                continue
            cells[(i, j)] = (iniX, iniY, maxX, maxY)
    nr = max(i for i, _ in cells) + 1
    ncl = max(j for _, j in cells) + 1
    bsj = 2 if 2 * wCell <= 64 else 1
    bsi = 2 if hCell <= 40 else 1
    out = []
    for bi in range(0, nr, bsi):
        for bj in range(0, ncl, bsj):
            ni, nj = min(bsi, nr - bi), min(bsj, ncl - bj)
            x0, y0 = cells[(bi, bj)][:2]
            x1 = cells[(bi, bj + nj - 1)][2]
            y1 = cells[(bi + ni - 1, bj)][3]
            out.append((x0, y0, x1 - x0 - 6, y1 - y0 - 6))
    return out


def main():
    isa = sys.argv[1]
    pmc = sys.argv[sys.argv.index("--pmc") + 1] if "--pmc" in sys.argv else None
    wts = {}
    if "--weights" in sys.argv:
        for kv in sys.argv[sys.argv.index("--weights") + 1].split(","):
            k, v = kv.split("=")
            wts[k] = float(v)
    body = VB.kernel_body(open(isa).read(), "og_fast_quad_kernel")
    ph = VB.summarise(VB.phases(body))
    # per phase: (once-per-wave VALU, cycles), (per-iteration VALU, cycles) from the loop bodies, each basic block
    # scaled by its --weights fraction
    once, it = {}, {}
    for k, n, cyc, blocks in ph:
        on = oc = ln = lc = 0.0
        for bname, loop, bn, bc in blocks:
            f = wts.get(bname, 1.0)
            if loop:
                ln += f * bn
                lc += f * bc
            else:
                on += f * bn
                oc += f * bc
        once[k] = (on, oc)
        it[k] = (ln, lc)
    import oracle_py as O
    import bench
    from orbslam2_with_quadrics_amd import synthetic

    O.build()
    oe = O.OracleExtractor(2000)
    _, frames = bench._frames(synthetic, 1080, 1920, 1, 0)
    oe(frames[0])
    tq = 7
    acc = {k: [0.0, 0.0] for k in range(6)}
    waves = 0
    pix = 0
    for lev in range(8):
        img = oe.level(lev)
        q = quick_pass(img, tq)
        for x0, y0, dw, dh in blocks_of_level(*img.shape):
            ns = int(q[y0 + 3:y0 + 3 + dh, x0 + 3:x0 + 3 + dw].sum())
            units = 2 * math.ceil(dh / 8)
            pix += dw * dh
            for w in range(8):
                waves += 1
                # stage 1: wave w takes the units' first rows R = 8 (w >> 1) + 2 (w & 1), stepping by 32
                trips = {0: 0, 1: len(range(8 * (w >> 1) + 2 * (w & 1), 8 * (units >> 1) + 2 * (w & 1), 32)),
                         2: len(range(64 * w, ns, 512)), 3: len(range(64 * w, ns, 512)), 4: 0,
                         5: len(range(64 * w, ns, 512))}
                for k in range(6):
                    acc[k][0] += once[k][0] + trips[k] * it[k][0]
                    acc[k][1] += once[k][1] + trips[k] * it[k][1]
    names = {0: "ROI staging + score-map zeroing", 1: "stage 1: quick test + survivor list",
             2: "stage 2: exact score", 3: "stage 3: NMS", 4: "stage 4: per-cell fallback + reservation",
             5: "emission"}
    tot_n = sum(v[0] for v in acc.values())
    tot_c = sum(v[1] for v in acc.values())
    print(f"# og_fast_quad_kernel VALU budget, config 3 frame (1920x1080, 8 levels, t_q = {tq}), "
          f"{waves // 8} blocks, {pix} tested pixels")
    print(f"# static counts from {os.path.basename(isa)} (tools/valu_budget.py); trip counts from the block plan; "
          f"block weights {wts or 'none'}")
    print(f"{'phase':48s} {'VALU/wave':>10s} {'cycles/wave':>12s} {'VALU lane-ops/px':>17s} {'share':>6s}")
    for k in range(6):
        n, c = acc[k]
        print(f"{k} {names[k]:46s} {n / waves:10.1f} {c / waves:12.1f} {n * 64 / pix:17.2f} {c / tot_c:6.1%}")
    print(f"{'total':48s} {tot_n / waves:10.1f} {tot_c / waves:12.1f} {tot_n * 64 / pix:17.2f}")
    if pmc:
        k = json.load(open(pmc))["kernels"]["fast"]
        print(f"# PMC check ({pmc}): SQ_INSTS_VALU / SQ_WAVES = {k['SQ_INSTS_VALU'] / k['SQ_WAVES']:.1f} VALU per wave "
              f"(the estimate above counts the 8 waves of every block; padding entries exit at once)")


if __name__ == "__main__":
    main()
