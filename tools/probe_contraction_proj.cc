// Compiler probe (test infrastructure): with the reference's flags (-O3 -march=native, GNU C++), how
// does GCC contract the projection expressions of Frame::isInFrustum (src/Frame.cc:287-288,316) and
// ORBmatcher::SearchByProjection(Frame&, const Frame&) (src/ORBmatcher.cc:1370-1371,1404)?
//   u  = fx*X*invz + cx      -> fma(fx*X, invz, cx) ?
//   ur = u - mbf*invz        -> fma(-mbf, invz, u) ?
//   lev = c + k*d (float)    -> fma(k, d, c) ?
// Prints mismatch counts of each explicit form against the compiler's code.
#include <cmath>
#include <cstdio>

__attribute__((noinline)) void proj(const float* X, const float* Z, int n, float fx, float cx, float mbf, float* u,
                                    float* ur)
{
    for (int i = 0; i < n; i++) {
        const float invz = 1.0f / Z[i];
        const float uu = fx * X[i] * invz + cx;
        u[i] = uu;
        ur[i] = uu - mbf * invz;
    }
}

int main()
{
    const int n = 1 << 16;
    float *X = new float[n], *Z = new float[n], *u = new float[n], *ur = new float[n];
    unsigned s = 777;
    long long bad_u = 0, bad_ur = 0, bad_u_plain = 0, total = 0;
    for (int it = 0; it < 64; it++) {
        for (int i = 0; i < n; i++) {
            s = s * 1103515245u + 12345u;
            X[i] = ((int)(s >> 8) % 200000 - 100000) * 1.37e-4f;
            s = s * 1103515245u + 12345u;
            Z[i] = 0.1f + (float)((s >> 8) % 100000) * 3.1e-4f;
        }
        const float fx = 718.856f, cx = 607.1928f, mbf = 386.1448f;
        proj(X, Z, n, fx, cx, mbf, u, ur);
        for (int i = 0; i < n; i++) {
            const float invz = 1.0f / Z[i];
            const float eu = std::fma(fx * X[i], invz, cx);
            volatile float t1 = fx * X[i];
            volatile float t2 = t1 * invz;
            const float pu = t2 + cx;  // unfused (volatile temporaries block contraction)
            const float eur = std::fma(-mbf, invz, eu);
            total++;
            if (u[i] != eu) bad_u++;
            if (u[i] != pu) bad_u_plain++;
            if (ur[i] != eur) bad_ur++;
        }
    }
    std::printf("total %lld u!=fma(fx*X,invz,cx) %lld u!=unfused %lld ur!=fma(-mbf,invz,u) %lld\n", total, bad_u,
                bad_u_plain, bad_ur);
    return 0;
}
