"""Host-side integer identities the kernels rely on (CPU only).

* describe's frame index: og_launch_describe passes dmagic = floor(2^32 / blocks) + 1 and the kernel takes
  lin / blocks as mulhi(lin, dmagic) whenever blocks^2 * B < 2^32 (orb_extract.hip, og_launch_describe).
* FAST's stage-1 unit walk: units u = w, w + 8, ... of a wave start at rows R = 8 (u >> 1) + 2 (u & 1), walked as
  R += 32 up to 8 (nunits >> 1) + 2 (w & 1) (og_fast_quad_kernel).
* FAST's column counts: OgFastBlk::colw byte k = clamp(dw - 16 k, 0, 16), mask (0x10001 << n) - 0x10001 per 16-lane
  group.
* describe's cvRound of the rotated rBRIEF coordinates (og_cvround_plus, orb_math_dev.h): the bits of the float sum
  v + 1.5 * 2^23 are 0x4B400000 + rint(v) (round half to even) for |v| < 2^22; the sample coordinates are |v| <= 18.5.
* the FAST frame-interleaved dispatch (og_fast_quad_kernel): workgroup lin of a (nb, B) grid is block lin / B of frame
  lin % B, a bijection onto (block, frame), and every block of frame f runs on XCD f % 8 when B % 8 == 0.
* FAST's stage-1 pass test as a sign (og_fast_quick2v and its caller): on the f16-biased pixels (1024 + p), the halves
  of dmax - (v - t) and (v + t) - bmin are negative exactly when the pixel passes the dark / bright quick test, their
  packed minimum is negative exactly when it passes either, and the survivor entry's bits 14 / 15 are those signs.
"""
import random


def mulhi32(a, b):
    return (a * b) >> 32


def test_describe_frame_magic_exact():
    rng = random.Random(7)
    cases = [(d, b) for d in (2, 3, 7, 250, 500, 512, 1000, 1001, 1023, 2047, 4095) for b in (1, 2, 64, 256, 512, 1024)]
    cases += [(rng.randrange(2, 5000), rng.randrange(1, 2049)) for _ in range(60)]
    checked = 0
    for d, b in cases:
        if d * d * b >= 1 << 32:
            continue
        m = (1 << 32) // d + 1
        assert m < 1 << 32
        n = d * b
        pts = set(range(0, min(n, 4096))) | set(range(max(0, n - 4096), n)) | {rng.randrange(n) for _ in range(2000)}
        # every multiple of d and its predecessor: where a wrong quotient would first show
        pts |= {q * d for q in range(b)} | {q * d - 1 for q in range(1, b + 1)}
        for x in pts:
            assert mulhi32(x, m) == x // d, (d, b, x)
        checked += 1
    assert checked > 40


def test_fast_unit_rows_walk():
    for dh in range(1, 81):
        nunits = ((dh + 7) >> 3) * 2
        for w in range(8):
            want = [8 * (u >> 1) + 2 * (u & 1) for u in range(w, nunits, 8)]
            got = list(range(8 * (w >> 1) + 2 * (w & 1), 8 * (nunits >> 1) + 2 * (w & 1), 32))
            assert got == want, (dh, w)


def test_fast_column_masks():
    for dw in range(1, 65):
        colw = 0
        for k in range(4):
            colw |= min(max(dw - 16 * k, 0), 16) << (8 * k)
        for k in range(4):
            n = (colw >> (8 * k)) & 31
            m32 = ((0x10001 << n) - 0x10001) & 0xFFFFFFFF
            lanes = [lane for lane in range(32) if (m32 >> lane) & 1]
            assert lanes == [lane for lane in range(32) if (lane & 15) + 16 * k < dw], (dw, k)


def test_cvround_plus_magic_rounding():
    import numpy as np

    rng = np.random.default_rng(7)
    v = np.concatenate([rng.uniform(-20, 20, 200000).astype(np.float32),
                        (np.arange(-40, 41, dtype=np.float32) / 2),            # every half-integer tie in range
                        np.nextafter(np.arange(-40, 41, dtype=np.float32) / 2, np.float32(np.inf)),
                        np.nextafter(np.arange(-40, 41, dtype=np.float32) / 2, np.float32(-np.inf))])
    t = (v + np.float32(12582912.0)).astype(np.float32)                      # one f32 add, round to nearest even
    got = (t.view(np.uint32).astype(np.int64) - 0x4B400000)
    want = np.rint(v).astype(np.int64)                                         # numpy rint: half to even
    assert np.array_equal(got, want)
    # with the + 18 the kernel folds into the subtraction: window coordinates 0 .. 36 for |v| <= 18.5
    k = 18
    got18 = (t.view(np.uint32).astype(np.int64) - (0x4B400000 - k)) & 0xFFFFFFFF
    assert np.array_equal(got18[np.abs(v) <= 18.5], (want + k)[np.abs(v) <= 18.5])


def test_fast_frame_interleave_mapping():
    for nb, B in ((13, 8), (7, 3), (530, 256), (1, 1), (5, 16)):
        seen = set()
        for lin in range(nb * B):
            f, p = lin % B, lin // B
            assert 0 <= p < nb
            seen.add((p, f))
            if B % 8 == 0:
                assert lin % 8 == f % 8
        assert len(seen) == nb * B



def test_fast_quick_test_sign_form():
    import numpy as np

    rng = np.random.default_rng(11)
    n = 200000
    # circle samples and centres: random bytes, plus near-flat patches where the ties (x - x) decide
    c = rng.integers(0, 256, (n, 16))
    v = rng.integers(0, 256, n)
    flat = rng.random(n) < 0.5
    c[flat] = np.clip(v[flat, None] + rng.integers(-12, 13, (int(flat.sum()), 16)), 0, 255)
    t = rng.integers(0, 256, n)
    t[: n // 2] = rng.integers(0, 25, n // 2)
    # the integer quick test (cv::FAST, pairs {k, k + 8})
    lo, hi = np.minimum(c[:, :8], c[:, 8:]), np.maximum(c[:, :8], c[:, 8:])
    dark = (lo < (v - t)[:, None]).all(axis=1)
    bright = (hi > (v + t)[:, None]).all(axis=1)
    # the kernel's f16 form: every operand and result is an integer below 2048, exact in f16
    h = (c + 1024).astype(np.float16)
    hv, ht = (v + 1024).astype(np.float16), t.astype(np.float16)
    dmax = np.minimum(h[:, :8], h[:, 8:]).max(axis=1)
    bmin = np.maximum(h[:, :8], h[:, 8:]).min(axis=1)
    ed = (dmax - (hv - ht)).astype(np.float16)
    eb = ((hv + ht) - bmin).astype(np.float16)
    e = np.minimum(ed, eb)

    def neg(x):  # the sign bit of the f16 (v_cmp_gt_i16 0, x / bit 15 or 31 of the packed dword)
        return (x.view(np.uint16) & 0x8000) != 0

    assert np.array_equal(neg(ed), dark)
    assert np.array_equal(neg(eb), bright)
    assert np.array_equal(neg(e), dark | bright)
    assert not (ed.view(np.uint16) == 0x8000).any() and not (eb.view(np.uint16) == 0x8000).any()  # no -0
    # survivor entries: ((ed >> 1) & 0x4000) | (eb & 0x8000) on each 16-bit half
    ent = ((ed.view(np.uint16).astype(np.uint32) >> 1) & 0x4000) | (eb.view(np.uint16).astype(np.uint32) & 0x8000)
    assert np.array_equal((ent & 0x4000) != 0, dark) and np.array_equal((ent & 0x8000) != 0, bright)
    assert dark.any() and bright.any()
