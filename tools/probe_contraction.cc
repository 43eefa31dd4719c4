// Compiler probe (test infrastructure): with the reference's flags (-O3 -march=native, GNU C++),
// does GCC fuse the rBRIEF sample rotation `x*b + y*a` / `x*a - y*b` (same expression shape as
// src/ORBextractor.cc:118-120) as fma(x, b, y*a) / fma(x, a, -(y*b))?  Compares the compiler's
// contracted result with the explicit forms over many inputs and prints the mismatch counts.
#include <cmath>
#include <cstdio>
#include <cstdlib>

struct P { int x, y; };

__attribute__((noinline)) void rot(const P* pt, int n, float a, float b, float* r, float* c)
{
    for (int i = 0; i < n; i++) {
        r[i] = pt[i].x * b + pt[i].y * a;
        c[i] = pt[i].x * a - pt[i].y * b;
    }
}

int main()
{
    const int n = 4096;
    P* pt = new P[n];
    float *r = new float[n], *c = new float[n];
    unsigned s = 12345;
    long long bad_first = 0, bad_second = 0, total = 0;
    for (int it = 0; it < 2000; it++) {
        for (int i = 0; i < n; i++) {
            s = s * 1103515245u + 12345u;
            pt[i].x = (int)((s >> 8) % 27) - 13;
            s = s * 1103515245u + 12345u;
            pt[i].y = (int)((s >> 8) % 27) - 13;
        }
        s = s * 1103515245u + 12345u;
        const float ang = (float)((s >> 8) % 36000) * 0.01f * 0.017453292f;
        const float a = std::cos(ang), b = std::sin(ang);
        rot(pt, n, a, b, r, c);
        for (int i = 0; i < n; i++) {
            const float x = (float)pt[i].x, y = (float)pt[i].y;
            const float er = std::fma(x, b, y * a), ec = std::fma(x, a, -(y * b));
            const float sr = std::fma(y, a, x * b), sc = std::fma(-y, b, x * a);
            total++;
            if (r[i] != er || c[i] != ec) bad_first++;
            if (r[i] != sr || c[i] != sc) bad_second++;
        }
    }
    std::printf("total %lld fused-first-product mismatches %lld fused-second-product mismatches %lld\n", total,
                bad_first, bad_second);
    return 0;
}
