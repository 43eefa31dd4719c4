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
