/*
 * oracle/oo_math.h -- TEST INFRASTRUCTURE ONLY (CPU oracle; never linked into the product).
 *
 * Scalar float/double primitives the reference's ORB hot path reaches through OpenCV and glibc,
 * restated with every rounding step explicit.  This translation unit is compiled with
 * -ffp-contract=off; every fused multiply-add that the reference build performs is written out as
 * fmaf()/fma().
 *
 *  - oo_cvround: cvRound(float) = SSE cvtss2si = round-half-even (used at src/ORBextractor.cc:81,115,
 *    119-120,442,1112).
 *  - oo_fast_atan2: OpenCV 3.x cv::fastAtan2 (called at src/ORBextractor.cc:103), float, no FMA.
 *  - oo_sincosf: glibc 2.35 x86_64 FMA-ifunc sincosf.  The reference line
 *    `float a = (float)cos(angle), b = (float)sin(angle);` (src/ORBextractor.cc:113) is merged into one
 *    sincosf call by GCC -O3 -march=native (probe: tools/probe_contraction.sh).  The arithmetic below
 *    follows the machine code of libm.so.6's FMA variant (constants read from its table) and is
 *    pinned by an exhaustive comparison against the container's libm over every float in [0, 8)
 *    (tools/verify_sincosf.c, tests/test_oracle_pins.py).
 *  - oo_logf: glibc 2.35 logf (16-entry table, degree-3 polynomial in double).  The reference calls
 *    std::log(float) -- `using namespace std` is global via Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:36
 *    -- in MapPoint::PredictScale (src/MapPoint.cc:410) and Frame (src/Frame.cc:71).  Pinned by an
 *    exhaustive comparison against the container's libm over every positive normal float
 *    (tools/verify_logf.c).
 */
#ifndef OO_MATH_H
#define OO_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline int oo_cvround(float v) { return (int)lrintf(v); }      /* RNE in default mode */
static inline int oo_cvround_d(double v) { return (int)lrint(v); }
static inline int oo_cvfloor(float v) { return (int)floorf(v); }
static inline int oo_cvceil(float v) { return (int)ceilf(v); }

/* cv::fastAtan2 (OpenCV 3.x core, scalar build, no contraction). */
static inline float oo_fast_atan2(float y, float x)
{
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k;
    const float p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k;
    const float p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;  /* (float)DBL_EPSILON */
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* glibc sincosf table (libm.so.6, FMA variant), in the order the table is laid out in memory:
 * sign[4], 2/pi*2^24, pi/2, c0, c1, s1, c2, s2, c3, s3, c4. Second row = quadrants with n&2. */
static const double oo_sincosf_tab[2][14] = {
    {1.0, -1.0, -1.0, 1.0, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     0x1.0p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {1.0, -1.0, -1.0, 1.0, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     -0x1.0p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16},
};

static inline uint32_t oo_abstop12(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    return (u >> 20) & 0x7ff;
}

/* Valid for |y| < 120 (the ORB path only feeds angles in [0, 2*pi]). Returns 0 if out of range. */
static inline int oo_sincosf(float y, float* sinp, float* cosp)
{
    const uint32_t t = oo_abstop12(y);
    const double* T;
    double xs, x2;
    int n = 0;
    if (t < 0x3f4) {                    /* |y| < pi/4 */
        if (t < 0x398) { *sinp = y; *cosp = 1.0f; return 1; }
        T = oo_sincosf_tab[0];
        xs = (double)y;
        x2 = xs * xs;
    } else if (t < 0x42f) {             /* |y| < 120 */
        const double x = (double)y;
        const double* T0 = oo_sincosf_tab[0];
        n = (((int32_t)(x * T0[4])) + 0x800000) >> 24;
        const double r = fma(-(double)n, T0[5], x);
        T = oo_sincosf_tab[(n & 2) ? 1 : 0];
        xs = r * T0[n & 3];
        x2 = r * r;
    } else {
        return 0;
    }
    const double x3 = x2 * xs, x4 = x2 * x2;
    const double x5 = x2 * x3, x6 = x2 * x4;
    const double s1v = fma(x2, T[12], T[10]);
    const double c2v = fma(x2, T[13], T[11]);
    const double c1v = fma(x2, T[7], T[6]);
    const double s = fma(x3, T[8], xs);
    const double c = fma(x4, T[9], c1v);
    const float so = (float)fma(s1v, x5, s);
    const float co = (float)fma(c2v, x6, c);
    if (n & 1) { *sinp = co; *cosp = so; }
    else       { *sinp = so; *cosp = co; }
    return 1;
}

/* glibc logf data: (invc, logc) per 16 subintervals of [0x1.66p-1, 0x1.66p0), ln2, polynomial */
static const double oo_logf_tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};
static const double oo_logf_ln2 = 0x1.62e42fefa39efp-1;
static const double oo_logf_poly[3] = {-0x1.00ea348b88334p-2, 0x1.5575b0be00b6ap-2, -0x1.ffffef20a4123p-2};

/* logf for positive normal x (the only inputs PredictScale produces); other inputs follow IEEE limits */
static inline float oo_logf(float x)
{
    uint32_t ix;
    memcpy(&ix, &x, 4);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;
        /* subnormal: normalise */
        const float xs = x * 0x1p23f;
        memcpy(&ix, &xs, 4);
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    float zf;
    memcpy(&zf, &iz, 4);
    const double z = zf, invc = oo_logf_tab[i][0], logc = oo_logf_tab[i][1];
    const double r = fma(z, invc, -1.0);
    const double y0 = logc + (double)k * oo_logf_ln2;
    const double r2 = r * r;
    double y = fma(oo_logf_poly[1], r, oo_logf_poly[2]);
    y = fma(oo_logf_poly[0], r2, y);
    y = fma(y, r2, y0 + r);
    return (float)y;
}

#endif
