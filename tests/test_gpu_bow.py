"""GPU parity tests of Frame::ComputeBoW (src/Frame.cc:395-402) = DBoW2 TemplatedVocabulary::transform
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1256) through the C ABI vs the CPU oracle: BowVector
word ids and values (doubles compared bit-exactly) and FeatureVector node lists.  The real ORBvoc.txt is
absent offline; vocabularies are synthetic with ORBvoc's shape (k=10, L=6, L1_NORM, TF_IDF) or smaller."""
import ctypes as C

import numpy as np
import pytest

from orbslam2_with_quadrics_amd import synthetic

pytestmark = pytest.mark.gpu


def _same(got, want):
    (gw, gv), (gn, go, gf) = got
    (ww, wv), (wn, wo, wf) = want
    assert np.array_equal(gw, ww) and gv.tobytes() == wv.tobytes()
    assert np.array_equal(gn, wn) and np.array_equal(go, wo) and np.array_equal(gf, wf)


@pytest.mark.parametrize("k,L,scoring,weighting,levelsup", [(10, 6, 0, 0, 4), (10, 3, 0, 0, 1), (6, 4, 1, 1, 2),
                                                            (9, 3, 5, 0, 1), (8, 3, 0, 3, 1), (20, 2, 2, 2, 0)])
def test_compute_bow_vs_oracle(gpu, oracle, k, L, scoring, weighting, levelsup):
    voc = synthetic.vocabulary(k * 37 + L, k, L, scoring=scoring, weighting=weighting, p_short=0.05, p_stop=0.02)
    ex = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    _, desc = ex(synthetic.frame(3, 480, 640))
    gv = gpu.ORBVocabulary.from_arrays(ex, voc)
    ov = oracle.OracleVocabulary(voc)
    _same(gv.transform(desc, levelsup), ov.transform(desc, levelsup))
    assert gv.info()["words"] == int(voc["is_leaf"].sum())


def test_vocabulary_text_loader(gpu, oracle, tmp_path):
    voc = synthetic.vocabulary(5, 10, 3, p_short=0.1, p_stop=0.05)
    path = str(tmp_path / "voc.txt")
    synthetic.write_vocabulary_text(voc, path)
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    _, desc = ex(synthetic.frame(4, 480, 640))
    gv = gpu.ORBVocabulary(ex)
    assert gv.loadFromTextFile(path)
    _same(gv.transform(desc, 1), oracle.OracleVocabulary(path=path).transform(desc, 1))
    assert not gpu.ORBVocabulary(ex).loadFromTextFile(str(tmp_path / "missing.txt"))


def test_compute_bow_empty_and_tiny(gpu, oracle):
    voc = synthetic.vocabulary(9, 10, 3)
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7)
    gv, ov = gpu.ORBVocabulary.from_arrays(ex, voc), oracle.OracleVocabulary(voc)
    for n in (0, 1, 2, 3):
        d = np.random.default_rng(n).integers(0, 256, size=(n, 32), dtype=np.uint8)
        _same(gv.transform(d, 1), ov.transform(d, 1))


def test_compute_bow_batch_vs_oracle(gpu, oracle):
    from orbslam2_with_quadrics_amd import _lib

    B, rows, cols = 4, 480, 640
    voc = synthetic.vocabulary(77, 10, 6)
    imgs = np.stack([synthetic.frame(60 + b, rows, cols) for b in range(B)])
    ex = gpu.ORBextractor(2000, 1.2, 8, 20, 7)
    gv = gpu.ORBVocabulary.from_arrays(ex, voc)
    ov = oracle.OracleVocabulary(voc)
    di = ex.device_alloc(imgs.nbytes)
    try:
        ex.h2d(di, imgs)
        ex.extract_batch_device(di, B, cols, rows, cols, rows * cols)
        _, _, _, cap = ex.batch_outputs()
        sz = B * cap * (4 + 8 + 4 + 4) + B * (cap + 1) * 4 + B * 8
        dout = ex.device_alloc(sz)
        p = dout
        dw, p = p, p + B * cap * 4
        dv, p = p, p + B * cap * 8
        dnd, p = p, p + B * cap * 4
        dof, p = p, p + B * (cap + 1) * 4
        dft, p = p, p + B * cap * 4
        dnw, dnn = p, p + B * 4
        _lib.check(ex.ctx, _lib.lib().orbgpu_compute_bow_batch(ex.ctx, gv._h, 4, *[C.c_void_p(x) for x in
                                                                                   (dw, dv, dnw, dnd, dof, dft, dnn)]),
                   "bow_batch")
        ex.synchronize()
        hw = np.zeros((B, cap), np.int32)
        hv = np.zeros((B, cap), np.float64)
        hnd = np.zeros((B, cap), np.int32)
        hof = np.zeros((B, cap + 1), np.int32)
        hft = np.zeros((B, cap), np.int32)
        hnw = np.zeros(B, np.int32)
        hnn = np.zeros(B, np.int32)
        for a, d in ((hw, dw), (hv, dv), (hnd, dnd), (hof, dof), (hft, dft), (hnw, dnw), (hnn, dnn)):
            ex.d2h(a, d)
        for b in range(B):
            _, desc = ex.batch_download(b)
            want = ov.transform(desc, 4)
            nw, nn = hnw[b], hnn[b]
            got = ((hw[b, :nw], hv[b, :nw]), (hnd[b, :nn], hof[b, :nn + 1], hft[b, :hof[b, nn]]))
            _same(got, want)
            assert nw > 100
        ex.device_free(dout)
    finally:
        ex.device_free(di)
