// orb_math_dev.h -- bit-exact device restatements of the scalar float/double steps of the reference
// path.  The library is compiled with -ffp-contract=off: every fused multiply-add below is written
// out (fmaf / fma) exactly where the reference build performs one, and nowhere else.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// cvRound(float): cvtss2si under the default MXCSR = round-half-even (v_rndne_f32).
__device__ __forceinline__ int og_cvround(float v) { return (int)__builtin_rintf(v); }

// cvRound(v) + k for |v| < 2^22, as the low bits of v + 1.5 * 2^23: the add rounds v half-to-even to an integer (the
// float's ulp there is 1) and the bits of 1.5 * 2^23 + n are 0x4B400000 + n.  Two 2-cycle instructions (v_add_f32,
// v_sub_u32) where v_rndne_f32 + v_cvt_i32_f32 are two 4-cycle ones (profiles/r05_valu_issue_rates.txt).
// (asm: the compiler would pack two such adds into one v_pk_add_f32 plus a v_mov, and fold the subtraction into
// every address that uses the result; the empty asm keeps it one v_sub_u32)
__device__ __forceinline__ unsigned og_cvround_plus(float v, int k)
{
    float t;
    __asm__("v_add_f32 %0, %1, %2" : "=v"(t) : "s"(12582912.0f), "v"(v));
    unsigned u = __builtin_bit_cast(unsigned, t) - (0x4B400000u - (unsigned)k);
    __asm__("" : "+v"(u));
    return u;
}

// cv::fastAtan2 (OpenCV 3.x scalar, no FMA), called at src/ORBextractor.cc:103.
__device__ __forceinline__ float og_fast_atan2(float y, float x)
{
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k;
    const float p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k;
    const float p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;
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

// glibc 2.35 x86_64 sincosf (FMA ifunc variant) for |y| < 120; the reference's
// `(float)cos(angle), (float)sin(angle)` (src/ORBextractor.cc:113) is one sincosf call under
// GCC -O3 -march=native.  Same double-precision operation sequence as the host libm machine code.
// The constants of the two coefficient tables of that code; the second table negates entries 6, 7, 9, 11 and
// 13 (and the quadrant sign is +1, -1, -1, +1 for n & 3).  Selected, not indexed, so the function makes no
// memory access (a describe wave keeps the next keypoint's window loads in flight across it).
__device__ __forceinline__ void og_sincosf(float y, float* sinp, float* cosp)
{
    const double C4 = 0x1.45f306dc9c883p+23, C5 = 0x1.921fb54442d18p+0;
    const double C7 = -0x1.ffffffd0c621cp-2, C8 = -0x1.555545995a603p-3, C9 = 0x1.55553e1068f19p-5;
    const double C10 = 0x1.1107605230bc4p-7, C11 = -0x1.6c087e89a359dp-10, C12 = -0x1.994eb3774cf24p-13;
    const double C13 = 0x1.99343027bf8c3p-16;
    const uint32_t t = (__float_as_uint(y) >> 20) & 0x7ff;
    bool flip = false;  // second table
    double xs, x2;
    int n = 0;
    if (t < 0x3f4) {
        if (t < 0x398) { *sinp = y; *cosp = 1.0f; return; }
        xs = (double)y;
        x2 = __dmul_rn(xs, xs);
    } else {
        const double x = (double)y;
        n = (((int32_t)__dmul_rn(x, C4)) + 0x800000) >> 24;
        const double r = __fma_rn(-(double)n, C5, x);
        flip = (n & 2) != 0;
        const double sg = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
        xs = __dmul_rn(r, sg);
        x2 = __dmul_rn(r, r);
    }
    const double T6 = flip ? -1.0 : 1.0, T7 = flip ? -C7 : C7, T9 = flip ? -C9 : C9;
    const double T11 = flip ? -C11 : C11, T13 = flip ? -C13 : C13;
    const double x3 = __dmul_rn(x2, xs), x4 = __dmul_rn(x2, x2);
    const double x5 = __dmul_rn(x2, x3), x6 = __dmul_rn(x2, x4);
    const double s1v = __fma_rn(x2, C12, C10);
    const double c2v = __fma_rn(x2, T13, T11);
    const double c1v = __fma_rn(x2, T7, T6);
    const double s = __fma_rn(x3, C8, xs);
    const double c = __fma_rn(x4, T9, c1v);
    const float so = (float)__fma_rn(s1v, x5, s);
    const float co = (float)__fma_rn(c2v, x6, c);
    if (n & 1) { *sinp = co; *cosp = so; }
    else       { *sinp = so; *cosp = co; }
}

// ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1647-1663): popcount of the XOR of 8 u32 words.
__device__ __forceinline__ int og_hamming(const uint4 a0, const uint4 a1, const uint4 b0, const uint4 b1)
{
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// glibc 2.35 logf (the reference's std::log(float) in MapPoint::PredictScale, src/MapPoint.cc:410, and
// Frame's mfLogScaleFactor, src/Frame.cc:71): 16-entry (1/c, log c) table + degree-3 polynomial in
// double, the libm operation sequence (pinned exhaustively against the host libm).
__constant__ const double og_logf_tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};

__device__ __forceinline__ float og_logf(float x)
{
    uint32_t ix = __float_as_uint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -__builtin_inff();
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
        ix = __float_as_uint(x * 0x1p23f) - (23u << 23);  // subnormal
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15);
    const int k = (int32_t)tmp >> 23;
    const double z = (double)__uint_as_float(ix - (tmp & 0xff800000u));
    const double r = __fma_rn(z, og_logf_tab[i][0], -1.0);
    const double y0 = __dadd_rn(og_logf_tab[i][1], __dmul_rn((double)k, 0x1.62e42fefa39efp-1));
    const double r2 = __dmul_rn(r, r);
    double y = __fma_rn(0x1.5575b0be00b6ap-2, r, -0x1.ffffef20a4123p-2);
    y = __fma_rn(-0x1.00ea348b88334p-2, r2, y);
    y = __fma_rn(y, r2, __dadd_rn(y0, r));
    return (float)y;
}
