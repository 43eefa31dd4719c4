/*
 * Exhaustive pin of oracle/oo_math.h::oo_logf against the host libm logf (test infrastructure).
 * Usage: verify_logf [stride]   -- checks every stride-th positive float bit pattern (normals,
 * subnormals, 0, inf).  Prints "checked N mismatches M" and exits 1 on any mismatch.
 * Build: gcc -O2 -ffp-contract=off -fopenmp tools/verify_logf.c -lm
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
    long long mism = 0, checked = 0;
#pragma omp parallel for reduction(+ : mism, checked) schedule(static, 65536)
    for (long long i = 0; i <= 0x7f800000LL; i += stride) {
        uint32_t u = (uint32_t)i;
        float x, a, b;
        memcpy(&x, &u, 4);
        a = logf(x);
        b = oo_logf(x);
        checked++;
        if (memcmp(&a, &b, 4)) {
            if (mism < 10) fprintf(stderr, "mismatch x=%a libm=%a oracle=%a\n", x, a, b);
            mism++;
        }
    }
    printf("checked %lld mismatches %lld\n", checked, mism);
    return mism != 0;
}
