"""Small pure-Python restatements of reference algorithms (test infrastructure).

They are written independently of oracle/orb_oracle.c and follow the reference's control flow and
container semantics literally (std::list push_front/erase, vector push_back order), so they can
cross-check the C oracle on small adversarial inputs (ties, steals, claims).
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


def f32(x):
    return float(np.float32(x))


# ---------------------------------------------------------------------------------------------
# DistributeOctTree, src/ORBextractor.cc:481-537, 539-763
# ---------------------------------------------------------------------------------------------
class _Node:
    _next_id = 0

    def __init__(self):
        self.UL = self.UR = self.BL = self.BR = (0, 0)
        self.keys = []
        self.no_more = False
        _Node._next_id += 1
        self.ptr = _Node._next_id  # bump allocation: address order == creation order


def _divide(p):
    halfX = int(math.ceil(f32(F32(p.UR[0] - p.UL[0]) / F32(2))))
    halfY = int(math.ceil(f32(F32(p.BR[1] - p.UL[1]) / F32(2))))
    n1, n2, n3, n4 = _Node(), _Node(), _Node(), _Node()
    n1.UL = p.UL
    n1.UR = (p.UL[0] + halfX, p.UL[1])
    n1.BL = (p.UL[0], p.UL[1] + halfY)
    n1.BR = (p.UL[0] + halfX, p.UL[1] + halfY)
    n2.UL = n1.UR
    n2.UR = p.UR
    n2.BL = n1.BR
    n2.BR = (p.UR[0], p.UL[1] + halfY)
    n3.UL = n1.BL
    n3.UR = n1.BR
    n3.BL = p.BL
    n3.BR = (n1.BR[0], p.BL[1])
    n4.UL = n3.UR
    n4.UR = n2.BR
    n4.BL = n3.BR
    n4.BR = p.BR
    for kp in p.keys:
        if kp[0] < n1.UR[0]:
            (n1 if kp[1] < n1.BR[1] else n3).keys.append(kp)
        elif kp[1] < n1.BR[1]:
            n2.keys.append(kp)
        else:
            n4.keys.append(kp)
    for n in (n1, n2, n3, n4):
        if len(n.keys) == 1:
            n.no_more = True
    return n1, n2, n3, n4


def distribute_octree(keys, minX, maxX, minY, maxY, N):
    """keys: list of (x, y, response) floats relative to minBorder. Returns list in output order."""
    nIni = int(round(f32(F32(maxX - minX) / F32(maxY - minY))))  # roundf: half away from zero
    hX = f32(F32(maxX - minX) / F32(nIni))
    lst = []  # python list as std::list (index 0 == front)
    ini = []
    for i in range(nIni):
        ni = _Node()
        ni.UL = (int(f32(F32(hX) * F32(i))), 0)
        ni.UR = (int(f32(F32(hX) * F32(i + 1))), 0)
        ni.BL = (ni.UL[0], maxY - minY)
        ni.BR = (ni.UR[0], maxY - minY)
        lst.append(ni)
        ini.append(ni)
    for kp in keys:
        ini[int(f32(F32(kp[0]) / F32(hX)))].keys.append(kp)
    lst2 = []
    for n in lst:
        if len(n.keys) == 1:
            n.no_more = True
            lst2.append(n)
        elif len(n.keys) == 0:
            continue
        else:
            lst2.append(n)
    lst = lst2
    finish = False
    vsp = []
    while not finish:
        prev_size = len(lst)
        n_expand = 0
        vsp = []
        # walk the list; children are pushed to the front (never visited in this pass)
        old = lst
        front = []
        kept = []
        for node in old:
            if node.no_more:
                kept.append(node)
                continue
            for c in _divide(node):
                if c.keys:
                    front.insert(0, c)
                    if len(c.keys) > 1:
                        n_expand += 1
                        vsp.append((len(c.keys), c.ptr, c))
        lst = front + kept
        if len(lst) >= N or len(lst) == prev_size:
            finish = True
        elif len(lst) + n_expand * 3 > N:
            while not finish:
                prev_size = len(lst)
                prev = sorted(vsp, key=lambda t: (t[0], t[1]))
                vsp = []
                for j in range(len(prev) - 1, -1, -1):
                    node = prev[j][2]
                    for c in _divide(node):
                        if c.keys:
                            lst.insert(0, c)
                            if len(c.keys) > 1:
                                vsp.append((len(c.keys), c.ptr, c))
                    lst.remove(node)
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev_size:
                    finish = True
    out = []
    for node in lst:
        best = node.keys[0]
        for k in node.keys[1:]:
            if k[2] > best[2]:
                best = k
        out.append(best)
    return out


# ---------------------------------------------------------------------------------------------
# Frame grid + matchers
# ---------------------------------------------------------------------------------------------
def popcount_dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


class PyFrame:
    def __init__(self, kps, desc, cols, rows, scale_factors, uright=None):
        self.kps = kps
        self.desc = desc
        self.sf = np.asarray(scale_factors, np.float32)
        self.uright = uright
        self.minX, self.minY, self.maxX, self.maxY = 0.0, 0.0, float(cols), float(rows)
        self.invW = f32(F32(64) / F32(cols))
        self.invH = f32(F32(48) / F32(rows))
        self.grid = [[[] for _ in range(48)] for _ in range(64)]
        for i, k in enumerate(kps):
            px = _round_half_away(f32(F32(f32(F32(k["x"]) - F32(self.minX))) * F32(self.invW)))
            py = _round_half_away(f32(F32(f32(F32(k["y"]) - F32(self.minY))) * F32(self.invH)))
            if 0 <= px < 64 and 0 <= py < 48:
                self.grid[px][py].append(i)

    def features_in_area(self, x, y, r, minLevel=-1, maxLevel=-1):
        def fl(v):
            return int(math.floor(v))

        ax = f32(F32(f32(F32(x) - F32(self.minX))) - F32(r))
        bx = f32(F32(f32(F32(x) - F32(self.minX))) + F32(r))
        ay = f32(F32(f32(F32(y) - F32(self.minY))) - F32(r))
        by = f32(F32(f32(F32(y) - F32(self.minY))) + F32(r))
        x0 = max(0, fl(f32(F32(ax) * F32(self.invW))))
        if x0 >= 64:
            return []
        x1 = min(63, int(math.ceil(f32(F32(bx) * F32(self.invW)))))
        if x1 < 0:
            return []
        y0 = max(0, fl(f32(F32(ay) * F32(self.invH))))
        if y0 >= 48:
            return []
        y1 = min(47, int(math.ceil(f32(F32(by) * F32(self.invH)))))
        if y1 < 0:
            return []
        check = minLevel > 0 or maxLevel >= 0
        out = []
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for idx in self.grid[ix][iy]:
                    k = self.kps[idx]
                    if check:
                        if k["octave"] < minLevel:
                            continue
                        if maxLevel >= 0 and k["octave"] > maxLevel:
                            continue
                    dx = f32(F32(k["x"]) - F32(x))
                    dy = f32(F32(k["y"]) - F32(y))
                    if abs(dx) < r and abs(dy) < r:
                        out.append(idx)
        return out


def _round_half_away(v):
    return int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)


def three_maxima(hist_len):
    max1 = max2 = max3 = 0
    ind1 = ind2 = ind3 = -1
    for i, s in enumerate(hist_len):
        if s > max1:
            max3, max2, max1 = max2, max1, s
            ind3, ind2, ind1 = ind2, ind1, i
        elif s > max2:
            max3, max2 = max2, s
            ind3, ind2 = ind2, i
        elif s > max3:
            max3, ind3 = s, i
    if max2 < f32(F32(0.1) * F32(max1)):
        ind2 = ind3 = -1
    elif max3 < f32(F32(0.1) * F32(max1)):
        ind3 = -1
    return ind1, ind2, ind3


def search_for_initialization(F1, F2, prev, nnratio=0.9, check_ori=True, window=100):
    """src/ORBmatcher.cc:405-520; prev is (n1,2) float32 (modified copy returned)."""
    prev = prev.copy()
    n1, n2 = len(F1.kps), len(F2.kps)
    m12 = [-1] * n1
    hist = [[] for _ in range(30)]
    factor = f32(F32(1.0) / F32(30))
    vmd = [2**31 - 1] * n2
    v21 = [-1] * n2
    nm = 0
    for i1 in range(n1):
        if F1.kps[i1]["octave"] > 0:
            continue
        idx2 = F2.features_in_area(float(prev[i1, 0]), float(prev[i1, 1]), float(window), 0, 0)
        if not idx2:
            continue
        best = best2 = 2**31 - 1
        bi = -1
        for i2 in idx2:
            d = popcount_dist(F1.desc[i1], F2.desc[i2])
            if vmd[i2] <= d:
                continue
            if d < best:
                best2, best, bi = best, d, i2
            elif d < best2:
                best2 = d
        if best <= 50 and best < f32(F32(best2) * F32(nnratio)):
            if v21[bi] >= 0:
                m12[v21[bi]] = -1
                nm -= 1
            m12[i1] = bi
            v21[bi] = i1
            vmd[bi] = best
            nm += 1
            if check_ori:
                rot = f32(F32(F1.kps[i1]["angle"]) - F32(F2.kps[bi]["angle"]))
                if rot < 0.0:
                    rot = f32(F32(rot) + F32(360.0))
                b = _round_half_away(f32(F32(rot) * F32(factor)))
                if b == 30:
                    b = 0
                hist[b].append(i1)
    if check_ori:
        i1_, i2_, i3_ = three_maxima([len(h) for h in hist])
        for i in range(30):
            if i in (i1_, i2_, i3_):
                continue
            for idx1 in hist[i]:
                if m12[idx1] >= 0:
                    m12[idx1] = -1
                    nm -= 1
    for i1 in range(n1):
        if m12[i1] >= 0:
            prev[i1, 0] = F2.kps[m12[i1]]["x"]
            prev[i1, 1] = F2.kps[m12[i1]]["y"]
    return nm, np.array(m12, np.int32), prev


def search_by_projection(F, mp, nnratio=0.8, th=3.0, owner=None, owner_obs=None):
    """src/ORBmatcher.cc:45-137."""
    n = len(F.kps)
    owner = list(np.full(n, -1) if owner is None else owner)
    obs = list(np.zeros(n, int) if owner_obs is None else owner_obs)
    nm = 0
    bfac = th != 1.0
    for m in range(len(mp["level"])):
        if not mp["track_in_view"][m] or mp["is_bad"][m]:
            continue
        lvl = int(mp["level"][m])
        r = 2.5 if float(np.float32(mp["view_cos"][m])) > 0.998 else 4.0
        if bfac:
            r = f32(F32(r) * F32(th))
        R = f32(F32(r) * F.sf[lvl])
        idx = F.features_in_area(float(mp["proj_x"][m]), float(mp["proj_y"][m]), R, lvl - 1, lvl)
        if not idx:
            continue
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for i in idx:
            if owner[i] >= 0 and obs[i]:
                continue
            if F.uright is not None and F.uright[i] > 0:
                er = abs(f32(F32(mp["proj_xr"][m]) - F32(F.uright[i])))
                if er > f32(F32(r) * F.sf[lvl]):
                    continue
            d = popcount_dist(mp["desc"][m], F.desc[i])
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, int(F.kps[i]["octave"]), i
            elif d < bd2:
                bl2, bd2 = int(F.kps[i]["octave"]), d
        if bd <= 100:
            if bl == bl2 and bd > f32(F32(nnratio) * F32(bd2)):
                continue
            owner[bi] = m
            obs[bi] = int(mp["n_obs"][m] > 0)
            nm += 1
    return nm, np.array(owner, np.int32), np.array(obs, np.int32)


# ---------------------------------------------------------------------------------------------
# FAST definition (segment test, 9 of 16) and its score
# ---------------------------------------------------------------------------------------------
CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
          (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast_is_corner(patch, t):
    v = int(patch[3, 3])
    ring = [int(patch[3 + dy, 3 + dx]) for dx, dy in CIRCLE]
    for sign in (1, -1):
        ok = [(v - p) * sign > t for p in ring]
        for s in range(16):
            if all(ok[(s + k) % 16] for k in range(9)):
                return True
    return False


def fast_score_definition(patch):
    """Largest threshold t >= 0 for which the centre is still a corner; -1 if none."""
    best = -1
    for t in range(0, 256):
        if fast_is_corner(patch, t):
            best = t
        else:
            break
    return best


# ---------------------------------------------------------------------------------------------
# Frame::ComputeStereoMatches, src/Frame.cc:466-640
# ---------------------------------------------------------------------------------------------
def stereo_matches(kL, dL, kR, dR, pyrL, pyrR, sf, isf, mbf, mb):
    """pyrL/pyrR: lists of u8 level images (level 0 = input).  Returns (uright, depth) float32."""
    N = len(kL)
    rows = pyrL[0].shape[0]
    uright = np.full(N, -1.0, np.float32)
    depth = np.full(N, -1.0, np.float32)
    row_idx = [[] for _ in range(rows)]
    for iR, k in enumerate(kR):
        kpY = F32(k["y"])
        r = F32(2.0) * F32(sf[k["octave"]])
        maxr = math.ceil(f32(kpY + r))
        minr = math.floor(f32(kpY - r))
        for yi in range(minr, maxr + 1):
            if 0 <= yi < rows:  # std::vector::operator[] outside the image is UB in the reference
                row_idx[yi].append(iR)
    minZ = F32(mb)
    minD = F32(0)
    maxD = F32(F32(mbf) / minZ)
    dist_idx = []
    for iL in range(N):
        k = kL[iL]
        levelL = int(k["octave"])
        vL, uL = F32(k["y"]), F32(k["x"])
        cands = row_idx[int(vL)]
        if not cands:
            continue
        minU, maxU = F32(uL - maxD), F32(uL - minD)
        if maxU < 0:
            continue
        bestDist, bestIdxR = 100, 0
        for iR in cands:
            kr = kR[iR]
            if kr["octave"] < levelL - 1 or kr["octave"] > levelL + 1:
                continue
            uR = F32(kr["x"])
            if minU <= uR <= maxU:
                dist = popcount_dist(dL[iL], dR[iR])
                if dist < bestDist:
                    bestDist, bestIdxR = dist, iR
        if bestDist >= (100 + 50) // 2:
            continue
        uR0 = F32(kR[bestIdxR]["x"])
        s = F32(isf[levelL])
        suL = _round_half_away(f32(F32(k["x"]) * s))
        svL = _round_half_away(f32(F32(k["y"]) * s))
        suR0 = _round_half_away(f32(uR0 * s))
        w, L = 5, 5
        IL = pyrL[levelL][svL - w:svL + w + 1, suL - w:suL + w + 1].astype(np.int64)
        IL = IL - IL[w, w]
        iniu, endu = suR0 + L - w, suR0 + L + w + 1
        if iniu < 0 or endu >= pyrR[levelL].shape[1]:
            continue
        best, bestinc = 2 ** 31 - 1, 0
        dists = []
        for inc in range(-L, L + 1):
            IR = pyrR[levelL][svL - w:svL + w + 1, suR0 + inc - w:suR0 + inc + w + 1].astype(np.int64)
            IR = IR - IR[w, w]
            d = int(np.abs(IL - IR).sum())
            if d < best:
                best, bestinc = d, inc
            dists.append(F32(d))
        if bestinc in (-L, L):
            continue
        d1, d2, d3 = dists[L + bestinc - 1], dists[L + bestinc], dists[L + bestinc + 1]
        with np.errstate(divide="ignore", invalid="ignore"):
            deltaR = F32(F32(d1 - d3) / F32(F32(2.0) * F32(F32(d1 + d3) - F32(F32(2.0) * d2))))
        if deltaR < -1 or deltaR > 1:
            continue
        bestuR = F32(F32(sf[levelL]) * F32(F32(F32(suR0) + F32(bestinc)) + deltaR))
        disparity = F32(uL - bestuR)
        if minD <= disparity < maxD:
            if disparity <= 0:
                disparity = F32(0.01)
                bestuR = F32(float(uL) - 0.01)
            depth[iL] = F32(F32(mbf) / disparity)
            uright[iL] = bestuR
            dist_idx.append((best, iL))
    if dist_idx:
        dist_idx.sort()
        median = F32(dist_idx[len(dist_idx) // 2][0])
        thDist = F32(F32(F32(1.5) * F32(1.4)) * median)
        for d, i in reversed(dist_idx):
            if F32(d) < thDist:
                break
            uright[i] = -1
            depth[i] = -1
    return uright, depth


# ---------------------------------------------------------------------------------------------
# Projection matchers: Frame::isInFrustum + MapPoint::PredictScale (src/Frame.cc:269-325,
# src/MapPoint.cc:402-417) and SearchByProjection(Frame&, const Frame&) (src/ORBmatcher.cc:1328-1470)
# ---------------------------------------------------------------------------------------------
def _libm_logf():
    import ctypes

    m = ctypes.CDLL("libm.so.6")
    m.logf.restype = ctypes.c_float
    m.logf.argtypes = [ctypes.c_float]
    return m.logf


def fmaf(a, b, c):
    """Correctly rounded float32 fma (exact rational arithmetic, no double rounding)."""
    from fractions import Fraction

    ex = Fraction(float(F32(a))) * Fraction(float(F32(b))) + Fraction(float(F32(c)))
    d = float(ex)                                  # correctly rounded double
    f = F32(d)
    # double -> float rounding is wrong only when d sits exactly on a float32 midpoint
    lo, hi = (np.nextafter(f, F32(-np.inf)), f) if float(f) > d else (f, np.nextafter(f, F32(np.inf)))
    if float(lo) != float(hi) and Fraction(float(lo)) + Fraction(float(hi)) == 2 * Fraction(d):
        f = hi if ex > Fraction(d) else lo if ex < Fraction(d) else f
    return F32(f)


def _rx_t(R, x, t):
    out = []
    for r in range(3):
        s = F32(F32(R[r][0]) * F32(x[0]))
        s = F32(s + F32(F32(R[r][1]) * F32(x[1])))
        s = F32(s + F32(F32(R[r][2]) * F32(x[2])))
        out.append(F32(s + F32(t[r])))
    return out


def is_in_frustum(cam, pos, normal, max_dist, min_dist, limit=0.5):
    logf = _libm_logf()
    lsf = F32(logf(float(cam["scale_factor"])))
    R = np.asarray(cam["Rcw"], np.float32).reshape(3, 3)
    t = np.asarray(cam["tcw"], np.float32)
    Ow = np.asarray(cam["Ow"], np.float32)
    fx, fy, cx, cy, mbf = (F32(cam[k]) for k in ("fx", "fy", "cx", "cy", "mbf"))
    W, H = F32(cam["cols"]), F32(cam["rows"])
    m = len(pos)
    out = dict(track_in_view=np.zeros(m, np.uint8), proj_x=np.zeros(m, np.float32),
               proj_y=np.zeros(m, np.float32), proj_xr=np.zeros(m, np.float32), level=np.zeros(m, np.int32),
               view_cos=np.zeros(m, np.float32))
    for i in range(m):
        P = np.asarray(pos[i], np.float32)
        Pc = _rx_t(R, P, t)
        if Pc[2] < 0:
            continue
        invz = F32(F32(1.0) / Pc[2])
        u = fmaf(F32(fx * Pc[0]), invz, cx)
        v = fmaf(F32(fy * Pc[1]), invz, cy)
        if u < 0 or u > W or v < 0 or v > H:
            continue
        maxD = F32(F32(1.2) * F32(max_dist[i]))
        minD = F32(F32(0.8) * F32(min_dist[i]))
        PO = [F32(P[k] - Ow[k]) for k in range(3)]
        ss = 0.0
        for k in range(3):
            ss += float(PO[k]) * float(PO[k])
        dist = F32(math.sqrt(ss))
        if dist < minD or dist > maxD:
            continue
        dot = 0.0
        for k in range(3):
            dot += float(PO[k]) * float(F32(normal[i][k]))
        vc = F32(dot / float(dist))
        if vc < F32(limit):
            continue
        ratio = F32(F32(max_dist[i]) / dist)
        ns = int(math.ceil(F32(F32(logf(float(ratio))) / lsf)))
        ns = min(max(ns, 0), int(cam["nlevels"]) - 1)
        out["track_in_view"][i] = 1
        out["proj_x"][i] = u
        out["proj_y"][i] = v
        out["proj_xr"][i] = fmaf(-mbf, invz, u)
        out["level"][i] = ns
        out["view_cos"][i] = vc
    return out


def search_by_projection_last(F, cur, last, lf, th, mono, check_ori, owner=None, owner_obs=None):
    """F: PyFrame (current).  Returns (nmatches, owner, owner_obs)."""
    n = len(F.kps)
    owner = [-1] * n if owner is None else list(owner)
    owner_obs = [0] * n if owner_obs is None else list(owner_obs)
    Rc = np.asarray(cur["Rcw"], np.float32).reshape(3, 3)
    tc = np.asarray(cur["tcw"], np.float32)
    Rl = np.asarray(last["Rcw"], np.float32).reshape(3, 3)
    tl = np.asarray(last["tcw"], np.float32)
    twc = []
    for j in range(3):
        s = F32(Rc[0][j] * tc[0])
        s = F32(s + F32(Rc[1][j] * tc[1]))
        s = F32(s + F32(Rc[2][j] * tc[2]))
        twc.append(F32(-s))
    tlc = _rx_t(Rl, twc, tl)
    mb, mbf = F32(cur["mb"]), F32(cur["mbf"])
    bForward = tlc[2] > mb and not mono
    bBackward = -tlc[2] > mb and not mono
    fx, fy, cx, cy = (F32(cur[k]) for k in ("fx", "fy", "cx", "cy"))
    hist = [[] for _ in range(30)]
    nm = 0
    for i in range(len(lf["kps"])):
        if not lf["has_mp"][i] or lf["outlier"][i]:
            continue
        x3 = _rx_t(Rc, np.asarray(lf["pos"][i], np.float32), tc)
        invzc = F32(1.0 / float(x3[2]))
        if invzc < 0:
            continue
        u = fmaf(F32(fx * x3[0]), invzc, cx)
        v = fmaf(F32(fy * x3[1]), invzc, cy)
        if u < F.minX or u > F.maxX or v < F.minY or v > F.maxY:
            continue
        o = int(lf["kps"][i]["octave"])
        radius = F32(F32(th) * F.sf[o])
        if bForward:
            cands = F.features_in_area(u, v, radius, o, -1)
        elif bBackward:
            cands = F.features_in_area(u, v, radius, 0, o)
        else:
            cands = F.features_in_area(u, v, radius, o - 1, o + 1)
        if not cands:
            continue
        best, bi = 256, -1
        for i2 in cands:
            if owner[i2] >= 0 and owner_obs[i2]:
                continue
            if F.uright is not None and F.uright[i2] > 0:
                ur = fmaf(-mbf, invzc, u)
                if abs(F32(ur - F32(F.uright[i2]))) > radius:
                    continue
            d = popcount_dist(lf["desc"][i], F.desc[i2])
            if d < best:
                best, bi = d, i2
        if best <= 100:
            owner[bi] = i
            owner_obs[bi] = int(lf["n_obs"][i] > 0)
            nm += 1
            if check_ori:
                rot = F32(F32(lf["kps"][i]["angle"]) - F32(F.kps[bi]["angle"]))
                if rot < 0.0:
                    rot = F32(rot + F32(360.0))
                b = _round_half_away(f32(rot * F32(F32(1.0) / F32(30))))
                if b == 30:
                    b = 0
                hist[b].append(bi)
    if check_ori:
        i1, i2_, i3 = three_maxima([len(h) for h in hist])
        for b in range(30):
            if b in (i1, i2_, i3):
                continue
            for k in hist[b]:
                owner[k] = -1
                owner_obs[k] = 0
                nm -= 1
    return nm, owner, owner_obs


# ---------------------------------------------------------------------------------------------
# Frame::UndistortKeyPoints / ComputeImageBounds via cv::undistortPoints (OpenCV 3.4, 5 iterations)
# ---------------------------------------------------------------------------------------------
def undistort_point(K4, dist, px, py):
    k = [float(F32(v)) for v in dist] + [0.0] * (5 - len(dist))
    fx, fy, cx, cy = (float(F32(v)) for v in K4)
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = (float(F32(px)) - cx) * ifx
    y = (float(F32(py)) - cy) * ify
    x0, y0 = x, y
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((0.0 * r2 + 0.0) * r2 + 0.0) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + 0.0 * r2 + 0.0 * r2 * r2
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + 0.0 * r2 + 0.0 * r2 * r2
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    xx = fx * x + 0.0 * y + cx
    yy = 0.0 * x + fy * y + cy
    ww = 1.0 / (0.0 * x + 0.0 * y + 1.0)
    return F32(xx * ww), F32(yy * ww)


def search_by_projection_kf(F, cur, kf, th, orbdist, check_ori, owner=None):
    """SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>&, th, ORBdist) (src/ORBmatcher.cc:1472-1599)."""
    logf = _libm_logf()
    n = len(F.kps)
    owner = [-1] * n if owner is None else list(owner)
    Rc = np.asarray(cur["Rcw"], np.float32).reshape(3, 3)
    tc = np.asarray(cur["tcw"], np.float32)
    Ow = []
    for j in range(3):
        s = F32(Rc[0][j] * tc[0])
        s = F32(s + F32(Rc[1][j] * tc[1]))
        s = F32(s + F32(Rc[2][j] * tc[2]))
        Ow.append(F32(-s))
    lsf = F32(logf(float(cur["scale_factor"])))
    fx, fy, cx, cy = (F32(cur[k]) for k in ("fx", "fy", "cx", "cy"))
    hist = [[] for _ in range(30)]
    nm = 0
    for i in range(len(kf["kps"])):
        if not kf["valid"][i]:
            continue
        X = np.asarray(kf["pos"][i], np.float32)
        x3 = _rx_t(Rc, X, tc)
        invzc = F32(1.0 / float(x3[2]))
        u = fmaf(F32(fx * x3[0]), invzc, cx)
        v = fmaf(F32(fy * x3[1]), invzc, cy)
        if u < F.minX or u > F.maxX or v < F.minY or v > F.maxY:
            continue
        PO = [F32(X[k] - Ow[k]) for k in range(3)]
        ss = 0.0
        for k in range(3):
            ss += float(PO[k]) * float(PO[k])
        d3 = F32(math.sqrt(ss))
        if d3 < F32(F32(0.8) * F32(kf["min_dist"][i])) or d3 > F32(F32(1.2) * F32(kf["max_dist"][i])):
            continue
        lvl = int(math.ceil(F32(F32(logf(float(F32(F32(kf["max_dist"][i]) / d3)))) / lsf)))
        lvl = min(max(lvl, 0), int(cur["nlevels"]) - 1)
        radius = F32(F32(th) * F.sf[lvl])
        cands = F.features_in_area(u, v, radius, lvl - 1, lvl + 1)
        if not cands:
            continue
        best, bi = 256, -1
        for i2 in cands:
            if owner[i2] >= 0:
                continue
            d = popcount_dist(kf["desc"][i], F.desc[i2])
            if d < best:
                best, bi = d, i2
        if best <= orbdist:
            owner[bi] = i
            nm += 1
            if check_ori:
                rot = F32(F32(kf["kps"][i]["angle"]) - F32(F.kps[bi]["angle"]))
                if rot < 0.0:
                    rot = F32(rot + F32(360.0))
                b = _round_half_away(f32(rot * F32(F32(1.0) / F32(30))))
                if b == 30:
                    b = 0
                hist[b].append(bi)
    if check_ori:
        i1, i2_, i3 = three_maxima([len(h) for h in hist])
        for b in range(30):
            if b in (i1, i2_, i3):
                continue
            for k in hist[b]:
                owner[k] = -1
                nm -= 1
    return nm, owner


# ---------------------------------------------------------------------------------------------
# DBoW2 TemplatedVocabulary::transform (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1256)
# ---------------------------------------------------------------------------------------------
def bow_transform(voc, desc, levelsup=4):
    n_nodes = len(voc["parent"]) + 1
    children = [[] for _ in range(n_nodes)]
    word_of = [-1] * n_nodes
    nw = 0
    for i, p in enumerate(voc["parent"]):
        children[int(p)].append(i + 1)
        if voc["is_leaf"][i]:
            word_of[i + 1] = nw
            nw += 1
    bow, fv = {}, {}
    tf = voc["weighting"] in (0, 1)
    for fi, f in enumerate(desc):
        nid_level = voc["L"] - levelsup
        nid, node, level = 0, 0, 0
        while True:
            level += 1
            kids = children[node]
            node = kids[0]
            best = popcount_dist(f, voc["desc"][node - 1])
            for c in kids[1:]:
                d = popcount_dist(f, voc["desc"][c - 1])
                if d < best:
                    best, node = d, c
            if level == nid_level:
                nid = node
            if not children[node]:
                break
        w = float(voc["weight"][node - 1])
        if w > 0:
            wid = word_of[node]
            if wid in bow:
                if tf:
                    bow[wid] += w
            else:
                bow[wid] = w
            fv.setdefault(nid, []).append(fi)
    items = sorted(bow.items())
    must = voc["scoring"] != 5
    if tf and items and not must:
        items = [(k_, v / float(len(items))) for k_, v in items]
    if must:
        if voc["scoring"] == 1:
            norm = math.sqrt(sum(v * v for _, v in items))
        else:
            norm = 0.0
            for _, v in items:
                norm += abs(v)
        if norm > 0.0:
            items = [(k_, v / norm) for k_, v in items]
    return items, sorted(fv.items())
