/*
 * Chunked hashes of the host libm over whole float ranges (TEST-FIXTURE GENERATOR, test infrastructure):
 * the values tests/test_gpu_pins.py compares the device restatements og_sincosf / og_logf
 * (orbslam2_with_quadrics_amd/csrc/orb_math_dev.h) against, on every input of the range.
 *
 *   libm_chunk_hash sincos|logf BEGIN END CHUNK_LOG2
 * For every float bit pattern u in [BEGIN, END): v = (sinbits << 32 | cosbits) for sincosf, logbits for logf;
 * chunk (u >> CHUNK_LOG2) accumulates og_hash_mix(v + u * 0x9E3779B97F4A7C15) mod 2^64 (an order-free sum, so the
 * GPU can add in any order).  Prints one line per chunk: "<chunk> <hash hex>".
 * Build: gcc -O2 -fopenmp tools/libm_chunk_hash.c -o libm_chunk_hash -lm   (glibc 2.35, the image's libm)
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv)
{
    if (argc != 5) return 2;
    const int fn = strcmp(argv[1], "sincos") == 0 ? 0 : 1;
    const uint64_t b = strtoull(argv[2], 0, 0), e = strtoull(argv[3], 0, 0);
    const int cl = atoi(argv[4]);
    const uint64_t c0 = b >> cl, c1 = (e - 1) >> cl;
    const int64_t nc = (int64_t)(c1 - c0 + 1);
    uint64_t* h = calloc((size_t)nc, 8);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t c = 0; c < nc; c++) {
        const uint64_t lo = ((c0 + c) << cl) > b ? ((c0 + c) << cl) : b;
        const uint64_t hi = ((c0 + c + 1) << cl) < e ? ((c0 + c + 1) << cl) : e;
        uint64_t acc = 0;
        for (uint64_t u = lo; u < hi; u++) {
            const uint32_t ub = (uint32_t)u;
            float x;
            memcpy(&x, &ub, 4);
            uint64_t v;
            if (fn == 0) {
                float s, co;
                sincosf(x, &s, &co);
                uint32_t sb, cb;
                memcpy(&sb, &s, 4);
                memcpy(&cb, &co, 4);
                v = ((uint64_t)sb << 32) | cb;
            } else {
                const float y = logf(x);
                uint32_t yb;
                memcpy(&yb, &y, 4);
                v = yb;
            }
            acc += mix(v + u * 0x9E3779B97F4A7C15ull);
        }
        h[c] = acc;
    }
    for (int64_t c = 0; c < nc; c++) printf("%lld %016llx\n", (long long)(c0 + c), (unsigned long long)h[c]);
    free(h);
    return 0;
}
