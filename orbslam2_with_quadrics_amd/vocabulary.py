"""Python mirror of ORB_SLAM2's ORBVocabulary (DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB>,
include/ORBVocabulary.h) and Frame::ComputeBoW (src/Frame.cc:395-402) over the gfx950 C ABI."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .extractor import ORBextractor


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class ORBVocabulary:
    """Device-resident vocabulary.  Build with loadFromTextFile(path) (TemplatedVocabulary.h:1338-1420) or
    from_arrays(dict(k, L, scoring, weighting, parent, is_leaf, desc, weight))."""

    def __init__(self, context: ORBextractor):
        self._ex = context
        self._h = None

    def loadFromTextFile(self, path: str) -> bool:
        self._free()
        self._h = _lib.lib().orbgpu_vocabulary_load_text(self._ex.ctx, path.encode())
        return bool(self._h)

    @classmethod
    def from_arrays(cls, context: ORBextractor, voc: dict) -> "ORBVocabulary":
        v = cls(context)
        par = np.ascontiguousarray(voc["parent"], np.int32)
        leaf = np.ascontiguousarray(voc["is_leaf"], np.uint8)
        desc = np.ascontiguousarray(voc["desc"], np.uint8)
        w = np.ascontiguousarray(voc["weight"], np.float64)
        v._h = _lib.lib().orbgpu_vocabulary_create(context.ctx, int(voc["k"]), int(voc["L"]), int(voc["scoring"]),
                                                   int(voc["weighting"]), len(par), _p(par), _p(leaf), _p(desc),
                                                   _p(w))
        if not v._h:
            _lib.check(context.ctx, _lib.ERR_ARG, "orbgpu_vocabulary_create")
        return v

    def info(self):
        k, L, n, w = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _lib.check(self._ex.ctx, _lib.lib().orbgpu_vocabulary_info(self._h, C.byref(k), C.byref(L), C.byref(n),
                                                                    C.byref(w)), "orbgpu_vocabulary_info")
        return dict(k=k.value, L=L.value, nodes=n.value, words=w.value)

    def transform(self, descriptors: np.ndarray, levelsup: int = 4):
        """-> (BowVector as (word ids, values) ascending, FeatureVector as (node ids, offsets, feature indices))."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        words = np.zeros(max(n, 1), np.int32)
        values = np.zeros(max(n, 1), np.float64)
        nodes = np.zeros(max(n, 1), np.int32)
        off = np.zeros(n + 1, np.int32)
        feats = np.zeros(max(n, 1), np.int32)
        nw, nn = C.c_int(0), C.c_int(0)
        rc = _lib.lib().orbgpu_compute_bow(self._ex.ctx, self._h, _p(d) if n else None, n, levelsup, _p(words),
                                           _p(values), C.byref(nw), _p(nodes), _p(off), _p(feats), C.byref(nn))
        _lib.check(self._ex.ctx, rc, "orbgpu_compute_bow")
        m = int(off[nn.value]) if nn.value else 0
        return ((words[:nw.value].copy(), values[:nw.value].copy()),
                (nodes[:nn.value].copy(), off[:nn.value + 1].copy(), feats[:m].copy()))

    def _free(self):
        if self._h:
            _lib.lib().orbgpu_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass


def ComputeBoW(voc: ORBVocabulary, descriptors: np.ndarray):
    """Frame::ComputeBoW: mBowVec, mFeatVec = transform(mDescriptors, levelsup = 4)."""
    return voc.transform(descriptors, 4)
