/*
 * Exhaustive pin of oracle/oo_math.h::oo_sincosf against the host libm sincosf (test infrastructure).
 * Usage: verify_sincosf [stride]   -- checks every stride-th float bit pattern in [0, 8.0f).
 * Prints "checked N mismatches M" and exits 1 on any mismatch.
 * Build: gcc -O2 -ffp-contract=off -fopenmp tools/verify_sincosf.c -lm
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../oracle/oo_math.h"

int main(int argc, char** argv)
{
    const uint32_t stride = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : 1u;
    const float hi = 8.0f;
    uint32_t uhi;
    memcpy(&uhi, &hi, 4);
    long long mism = 0, checked = 0;
#pragma omp parallel for reduction(+ : mism, checked) schedule(static, 65536)
    for (long long i = 0; i < (long long)uhi; i += stride) {
        uint32_t u = (uint32_t)i;
        float x;
        memcpy(&x, &u, 4);
        float s0, c0, s1, c1;
        sincosf(x, &s0, &c0);
        oo_sincosf(x, &s1, &c1);
        checked++;
        if (memcmp(&s0, &s1, 4) || memcmp(&c0, &c1, 4)) {
            if (mism < 10)
                fprintf(stderr, "mismatch x=%a libm=(%a,%a) oracle=(%a,%a)\n", x, s0, c0, s1, c1);
            mism++;
        }
        /* separate sinf/cosf calls must agree with sincosf too (reference may call either) */
        float s2 = sinf(x), c2 = cosf(x);
        if (memcmp(&s0, &s2, 4) || memcmp(&c0, &c2, 4)) mism++;
    }
    printf("checked %lld mismatches %lld\n", checked, mism);
    return mism ? 1 : 0;
}
