/*
 * tests/c/oracle_sanitize.c -- TEST INFRASTRUCTURE: drives the C oracle (oracle/orb_oracle.c, oo_bow.c) through
 * every entry point the GPU tests compare against, for a build with -fsanitize=address,undefined
 * (tests/test_sanitize.py).  Synthetic inputs are generated here (an LCG value-noise image with
 * rectangles), so the driver needs nothing but the oracle.  Exit status 0 and no sanitizer report = pass.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/orb_oracle.h"

static unsigned lcg(unsigned* s)
{
    *s = *s * 1664525u + 1013904223u;
    return *s >> 8;
}

/* smooth value noise + rectangles + per-pixel noise, shifted by (dx, dy) */
static void make_image(uint8_t* img, int w, int h, int dx, int dy, unsigned seed)
{
    unsigned s = seed;
    const int G = 24;
    const int gw = (w + 64) / G + 3, gh = (h + 64) / G + 3;
    float* grid = (float*)malloc(sizeof(float) * gw * gh);
    for (int i = 0; i < gw * gh; i++) grid[i] = 40.f + (float)(lcg(&s) % 160);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const int X = x + dx + 32, Y = y + dy + 32;
            const int gx = X / G, gy = Y / G;
            const float fx = (float)(X % G) / G, fy = (float)(Y % G) / G;
            const float a = grid[gy * gw + gx], b = grid[gy * gw + gx + 1], c = grid[(gy + 1) * gw + gx],
                        d = grid[(gy + 1) * gw + gx + 1];
            img[y * w + x] = (uint8_t)(a + (b - a) * fx + (c - a) * fy + (a - b - c + d) * fx * fy);
        }
    for (int r = 0; r < 60; r++) {
        const int x0 = (int)(lcg(&s) % (unsigned)w) - dx, y0 = (int)(lcg(&s) % (unsigned)h) - dy;
        const int rw = 5 + (int)(lcg(&s) % 40), rh = 5 + (int)(lcg(&s) % 40);
        const uint8_t v = (uint8_t)(lcg(&s) & 255);
        for (int y = y0; y < y0 + rh; y++)
            for (int x = x0; x < x0 + rw; x++)
                if (x >= 0 && x < w && y >= 0 && y < h) img[y * w + x] = v;
    }
    unsigned n = seed * 7919u + 1u;
    for (int i = 0; i < w * h; i++) {
        const int v = img[i] + (int)(lcg(&n) % 13) - 6;
        img[i] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    free(grid);
}

static oo_frame frame_of(const oo_keypoint* k, const uint8_t* d, int n, int w, int h, const float* sf, int nl)
{
    oo_frame f;
    memset(&f, 0, sizeof(f));
    f.n = n;
    f.kps = k;
    f.desc = d;
    f.scale_factors = sf;
    f.nlevels = nl;
    oo_grid_params(w, h, &f.minX, &f.minY, &f.maxX, &f.maxY, &f.gridInvW, &f.gridInvH);
    f.cell_start = (int*)malloc(sizeof(int) * (64 * 48 + 1));
    f.cell_items = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    oo_grid_build(&f);
    return f;
}

int main(void)
{
    const int W = 640, H = 480, NF = 1000, CAP = NF + 64 * 8 + 64;
    uint8_t* a = (uint8_t*)malloc(W * H);
    uint8_t* b = (uint8_t*)malloc(W * H);
    make_image(a, W, H, 0, 0, 11);
    make_image(b, W, H, 7, 3, 11);
    int checks = 0;
    for (int sem = 0; sem < 0x40; sem++) {  /* every valid semantics combination, and rejection of the rest */
        oo_extractor* e = oo_create(NF, 1.2f, 8, 20, 7);
        if (oo_set_semantics(e, sem) != 0) {
            oo_destroy(e);
            continue;
        }
        oo_keypoint* k1 = (oo_keypoint*)malloc(sizeof(oo_keypoint) * CAP);
        oo_keypoint* k2 = (oo_keypoint*)malloc(sizeof(oo_keypoint) * CAP);
        uint8_t* d1 = (uint8_t*)malloc(32 * CAP);
        uint8_t* d2 = (uint8_t*)malloc(32 * CAP);
        const int n1 = oo_extract(e, a, W, H, W, k1, d1, CAP);
        const int n2 = oo_extract(e, b, W, H, W, k2, d2, CAP);
        if (n1 <= 0 || n2 <= 0) return 2;
        float sf[8];
        oo_scale_tables(e, sf, NULL, NULL, NULL, NULL, NULL);
        oo_frame F1 = frame_of(k1, d1, n1, W, H, sf, 8), F2 = frame_of(k2, d2, n2, W, H, sf, 8);
        float* prev = (float*)malloc(sizeof(float) * 2 * n1);
        int* m12 = (int*)malloc(sizeof(int) * n1);
        for (int i = 0; i < n1; i++) {
            prev[2 * i] = k1[i].x;
            prev[2 * i + 1] = k1[i].y;
        }
        const int nm = oo_search_for_initialization(&F1, &F2, 0.9f, 1, prev, m12, 100);
        /* SearchByProjection against map points made from F1's own keypoints */
        const int M = 1500;
        uint8_t* tiv = (uint8_t*)malloc(M);
        uint8_t* bad = (uint8_t*)calloc(M, 1);
        int* lvl = (int*)malloc(sizeof(int) * M);
        int* nob = (int*)malloc(sizeof(int) * M);
        float *vc = (float*)malloc(4 * M), *px = (float*)malloc(4 * M), *py = (float*)malloc(4 * M),
              *pxr = (float*)malloc(4 * M);
        uint8_t* md = (uint8_t*)malloc(32 * M);
        unsigned s = 5;
        for (int m = 0; m < M; m++) {
            const int i = (int)(lcg(&s) % (unsigned)n2);
            tiv[m] = 1;
            lvl[m] = k2[i].octave;
            nob[m] = 2;
            vc[m] = 0.95f;
            px[m] = k2[i].x + 0.5f;
            py[m] = k2[i].y - 0.5f;
            pxr[m] = -1.f;
            memcpy(md + 32 * m, d2 + 32 * i, 32);
            md[32 * m + (m & 31)] ^= 0x11;
        }
        oo_mappoints mp = {M, tiv, bad, lvl, vc, px, py, pxr, nob, md};
        int* own = (int*)malloc(sizeof(int) * n2);
        int* obs = (int*)malloc(sizeof(int) * n2);
        for (int i = 0; i < n2; i++) own[i] = obs[i] = -1;
        const int np = oo_search_by_projection(&F2, &mp, 0.8f, 1.0f, own, obs);
        int* area = (int*)malloc(sizeof(int) * n2);
        const int na = oo_features_in_area(&F2, 320.f, 240.f, 50.f, -1, -1, area);
        if (sem == 0) printf("n1 %d n2 %d init matches %d projection matches %d area %d\n", n1, n2, nm, np, na);
        free(area); free(own); free(obs); free(tiv); free(bad); free(lvl); free(nob); free(vc); free(px); free(py);
        free(pxr); free(md); free(prev); free(m12); free(F1.cell_start); free(F1.cell_items); free(F2.cell_start);
        free(F2.cell_items); free(k1); free(k2); free(d1); free(d2);
        oo_destroy(e);
        checks++;
    }
    /* stereo on a horizontally shifted pair */
    {
        oo_extractor *L = oo_create(1000, 1.2f, 8, 20, 7), *R = oo_create(1000, 1.2f, 8, 20, 7);
        make_image(a, W, H, 0, 0, 21);
        make_image(b, W, H, 12, 0, 21);
        oo_keypoint* kl = (oo_keypoint*)malloc(sizeof(oo_keypoint) * CAP);
        oo_keypoint* kr = (oo_keypoint*)malloc(sizeof(oo_keypoint) * CAP);
        uint8_t* dl = (uint8_t*)malloc(32 * CAP);
        uint8_t* dr = (uint8_t*)malloc(32 * CAP);
        const int nl = oo_extract(L, a, W, H, W, kl, dl, CAP), nr = oo_extract(R, b, W, H, W, kr, dr, CAP);
        float* ur = (float*)malloc(4 * nl);
        float* de = (float*)malloc(4 * nl);
        const int ns = oo_stereo_matches(L, R, kl, dl, nl, kr, dr, nr, 386.1448f, 0.537f, ur, de);
        printf("stereo %d of %d\n", ns, nl);
        free(ur); free(de); free(kl); free(kr); free(dl); free(dr);
        oo_destroy(L);
        oo_destroy(R);
    }
    /* an empty image and a flat one */
    {
        oo_extractor* e = oo_create(500, 1.2f, 8, 20, 7);
        oo_keypoint k[600];
        uint8_t d[600 * 32];
        memset(a, 128, W * H);
        if (oo_extract(e, NULL, 0, 0, 0, k, d, 600) != 0) return 3;
        if (oo_extract(e, a, W, H, W, k, d, 600) != 0) return 4;
        oo_destroy(e);
    }
    free(a);
    free(b);
    printf("semantics variants exercised: %d\n", checks);
    return checks == 16 ? 0 : 5;
}
