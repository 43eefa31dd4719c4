/*
 * oracle/orb_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h for the parity status).
 *
 * Plain-C restatement of the reference's per-frame ORB hot path.  Every function cites the reference
 * file:line it follows.  Build: see oracle/Makefile (gcc -O2 -ffp-contract=off; FMAs explicit).
 */
#include "orb_oracle.h"
#include "oo_math.h"

#include <assert.h>
#include <limits.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#define OO_PATCH_SIZE 31
#define OO_HALF_PATCH 15
#define OO_EDGE 19
#define OO_MAXLEVELS 32
#define OO_GRID_COLS 64
#define OO_GRID_ROWS 48

#include "orb_pattern.inc" /* static const signed char oo_orb_pattern[256*4] (x0,y0,x1,y1 per pair) */

/* ------------------------------------------------------------------------------------------------ */
/* small growable arrays                                                                              */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { float x, y, resp; } oo_cand;  /* the fields of cv::KeyPoint the octree reads */
typedef struct { oo_cand* v; int n, cap; } oo_candvec;

static void cv_push(oo_candvec* a, oo_cand c)
{
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 16;
        a->v = (oo_cand*)realloc(a->v, sizeof(oo_cand) * (size_t)a->cap);
    }
    a->v[a->n++] = c;
}

struct oo_extractor {
    int nfeatures, nlevels, iniTh, minTh;
    int sem;                                  /* OO_SEM_* (orb_oracle.h), default 0 */
    double scaleFactor;                       /* double member, src/ORBextractor.h:98 */
    float sf[OO_MAXLEVELS], isf[OO_MAXLEVELS], sig2[OO_MAXLEVELS], isig2[OO_MAXLEVELS];
    int nfeat[OO_MAXLEVELS];
    int umax[OO_HALF_PATCH + 1];
    /* last call */
    int lw[OO_MAXLEVELS], lh[OO_MAXLEVELS];
    uint8_t* lev[OO_MAXLEVELS];
    oo_candvec cand[OO_MAXLEVELS];
};

/* ORBextractor::ORBextractor, src/ORBextractor.cc:410-470 */
oo_extractor* oo_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
{
    if (nlevels < 1 || nlevels > OO_MAXLEVELS) return NULL;
    oo_extractor* e = (oo_extractor*)calloc(1, sizeof(oo_extractor));
    e->nfeatures = nfeatures;
    e->scaleFactor = (double)scaleFactor;
    e->nlevels = nlevels;
    e->iniTh = iniThFAST;
    e->minTh = minThFAST;
    e->sf[0] = 1.0f;
    e->sig2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        e->sf[i] = (float)((double)e->sf[i - 1] * e->scaleFactor); /* float*double -> double -> float */
        e->sig2[i] = e->sf[i] * e->sf[i];
    }
    for (int i = 0; i < nlevels; i++) {
        e->isf[i] = 1.0f / e->sf[i];
        e->isig2[i] = 1.0f / e->sig2[i];
    }
    const float factor = (float)(1.0f / e->scaleFactor);
    float nd = (float)nfeatures * (1.0f - factor) /
               (1.0f - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        e->nfeat[l] = oo_cvround(nd);
        sum += e->nfeat[l];
        nd *= factor;
    }
    e->nfeat[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;

    /* umax, src/ORBextractor.cc:454-469 */
    int v, v0;
    const int vmax = oo_cvfloor(OO_HALF_PATCH * sqrtf(2.f) / 2 + 1);
    const int vmin = oo_cvceil(OO_HALF_PATCH * sqrtf(2.f) / 2);
    const double hp2 = OO_HALF_PATCH * OO_HALF_PATCH;
    for (v = 0; v <= vmax; ++v) e->umax[v] = oo_cvround_d(sqrt(hp2 - v * v));
    for (v = OO_HALF_PATCH, v0 = 0; v >= vmin; --v) {
        while (e->umax[v0] == e->umax[v0 + 1]) ++v0;
        e->umax[v] = v0;
        ++v0;
    }
    return e;
}

void oo_destroy(oo_extractor* e)
{
    if (!e) return;
    for (int l = 0; l < OO_MAXLEVELS; l++) {
        free(e->lev[l]);
        free(e->cand[l].v);
    }
    free(e);
}

int oo_nlevels(const oo_extractor* e) { return e->nlevels; }

int oo_set_semantics(oo_extractor* e, int sem)
{
    if (sem & ~OO_SEM_ALL || ((sem >> OO_SEM_BLUR_SHIFT) & 7) > 3) return -1;
    e->sem = sem;
    return 0;
}

void oo_scale_tables(const oo_extractor* e, float* scale, float* inv_scale, float* sigma2,
                     float* inv_sigma2, int* fpl, int* umax16)
{
    for (int l = 0; l < e->nlevels; l++) {
        if (scale) scale[l] = e->sf[l];
        if (inv_scale) inv_scale[l] = e->isf[l];
        if (sigma2) sigma2[l] = e->sig2[l];
        if (inv_sigma2) inv_sigma2[l] = e->isig2[l];
        if (fpl) fpl[l] = e->nfeat[l];
    }
    if (umax16) memcpy(umax16, e->umax, sizeof(int) * 16);
}

/* ------------------------------------------------------------------------------------------------ */
/* cv::resize INTER_LINEAR, CV_8UC1 (external; call site src/ORBextractor.cc:1120).  Generic           */
/* fixed-point path (resizeGeneric_ + HResizeLinear + VResizeLinear).  The vertical pass has two forms   */
/* (sem & OO_SEM_RESIZE_FIXEDPT):                                                         */
/*   0: OpenCV's VResizeLinear<uchar, int, short, FixedPtCast<int,uchar,22>, VResizeLinearVec_32s8u>      */
/*      specialisation: ((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2 -- the SSE2 mulhi body and the  */
/*      scalar tail compute the same form, so no SIMD/tail split exists;                                 */
/*   1: the generic template's FixedPtCast (b0*D0 + b1*D1 + 2^21) >> 22 (round-1 semantics).             */
/* ------------------------------------------------------------------------------------------------ */
void oo_resize_linear(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh, int sem)
{
    const int fixedpt = (sem & OO_SEM_RESIZE_FIXEDPT) != 0;
    const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    int* xofs = (int*)malloc(sizeof(int) * (size_t)dw);
    short* alpha = (short*)malloc(sizeof(short) * 2 * (size_t)dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = oo_cvfloor(fx);
        fx -= (float)sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) { fx = 0.f; sx = sw - 1; }
        }
        xofs[dx] = sx;
        alpha[2 * dx] = (short)oo_cvround((1.f - fx) * 2048);
        alpha[2 * dx + 1] = (short)oo_cvround(fx * 2048);
    }
    int* rows = (int*)malloc(sizeof(int) * 2 * (size_t)dw);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = oo_cvfloor(fy);
        fy -= (float)sy;
        const int b0 = (short)oo_cvround((1.f - fy) * 2048), b1 = (short)oo_cvround(fy * 2048);
        for (int k = 0; k < 2; k++) {
            int y = sy + k;
            y = y >= 0 ? (y < sh ? y : sh - 1) : 0;
            const uint8_t* S = src + (size_t)y * sw;
            int* D = rows + (size_t)k * dw;
            for (int dx = 0; dx < dw; dx++) {
                const int x = xofs[dx];
                D[dx] = dx < xmax ? S[x] * alpha[2 * dx] + S[x + 1] * alpha[2 * dx + 1] : S[x] * 2048;
            }
        }
        uint8_t* o = dst + (size_t)dy * dw;
        for (int dx = 0; dx < dw; dx++) {
            int val;
            if (fixedpt)
                val = (b0 * rows[dx] + b1 * rows[dw + dx] + (1 << 21)) >> 22;
            else
                val = (((b0 * (rows[dx] >> 4)) >> 16) + ((b1 * (rows[dw + dx] >> 4)) >> 16) + 2) >> 2;
            o[dx] = (uint8_t)(val < 0 ? 0 : val > 255 ? 255 : val);
        }
    }
    free(rows);
    free(xofs);
    free(alpha);
}

/* ------------------------------------------------------------------------------------------------ */
/* cv::GaussianBlur 7x7 sigma 2 BORDER_REFLECT_101 on CV_8U (src/ORBextractor.cc:1086).  Separable      */
/* integer kernel k (8 fractional bits), row sums exact; the column result by variant                  */
/* ((sem >> OO_SEM_BLUR_SHIFT) & 7):                                                    */
/*   0 SSE2_257: OpenCV 3.0-3.4.1 on x86-64 without IPP: FilterEngine with k = cvRound(256 g) =          */
/*     [18,34,49,55,...] (sum 257); SymmColumnVec_32s8u converts the column sums to float (exact below   */
/*     2^24) and rounds half-to-even (cvtps2dq) for x < 4*floor(w/4); the scalar tail x >= 4*floor(w/4)  */
/*     uses FixedPtCastEx (S + 2^15) >> 16;                                                             */
/*   1 SCALAR_257: the same kernel, FixedPtCastEx everywhere (a build without SSE2 vector ops);          */
/*   2 BITEXACT_256: the fixed-point GaussianBlur, centre = 256 - 2*sum(sides): [18,34,49,54,...];       */
/*   3 BITEXACT_ED: the fixed-point GaussianBlur with the error-diffused kernel [18,34,48,56,...].       */
/* All: out = sat_u8(round(S / 2^16)), S = sum_y k_y sum_x k_x I.                                       */
/* ------------------------------------------------------------------------------------------------ */
static const int oo_gk_tab[4][4] = {{18, 34, 49, 55}, {18, 34, 49, 55}, {18, 34, 49, 54}, {18, 34, 48, 56}};

static inline int oo_reflect101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

void oo_gaussian7(const uint8_t* src, int w, int h, uint8_t* dst, int sem)
{
    const int var = (sem >> OO_SEM_BLUR_SHIFT) & 7;
    const int* c = oo_gk_tab[var < 4 ? var : 0];
    const int gk[7] = {c[0], c[1], c[2], c[3], c[2], c[1], c[0]};
    const int xsimd = var == 0 ? (w & ~3) : 0;  /* columns whose result is rounded half-to-even */
    int* tmp = (int*)malloc(sizeof(int) * (size_t)w * (size_t)h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int k = -3; k <= 3; k++) s += gk[k + 3] * src[(size_t)y * w + oo_reflect101(x + k, w)];
            tmp[(size_t)y * w + x] = s;
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int k = -3; k <= 3; k++) s += gk[k + 3] * tmp[(size_t)oo_reflect101(y + k, h) * w + x];
            int v = (s + (1 << 15)) >> 16;
            if (x < xsimd && (s & 0x1ffff) == 0x8000) v--; /* tie with an even quotient: half-to-even */
            dst[(size_t)y * w + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    free(tmp);
}

/* ------------------------------------------------------------------------------------------------ */
/* cv::FAST(img, kps, threshold, nonmax=true), TYPE_9_16 (external; src/ORBextractor.cc:809,814)      */
/* ------------------------------------------------------------------------------------------------ */
static const int oo_circle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                     {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                     {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

static void oo_make_offsets(int* pixel, int stride)
{
    int k;
    for (k = 0; k < 16; k++) pixel[k] = oo_circle[k][0] + oo_circle[k][1] * stride;
    for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

static inline int oo_imin(int a, int b) { return a < b ? a : b; }
static inline int oo_imax(int a, int b) { return a > b ? a : b; }

/* cornerScore<16> */
static int oo_corner_score(const uint8_t* ptr, const int* pixel, int threshold)
{
    int d[25], k, v = ptr[0];
    for (k = 0; k < 25; k++) d[k] = v - ptr[pixel[k]];
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = oo_imin(d[k + 1], d[k + 2]);
        a = oo_imin(a, d[k + 3]);
        if (a <= a0) continue;
        a = oo_imin(a, d[k + 4]);
        a = oo_imin(a, d[k + 5]);
        a = oo_imin(a, d[k + 6]);
        a = oo_imin(a, d[k + 7]);
        a = oo_imin(a, d[k + 8]);
        a0 = oo_imax(a0, oo_imin(a, d[k]));
        a0 = oo_imax(a0, oo_imin(a, d[k + 9]));
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = oo_imax(d[k + 1], d[k + 2]);
        b = oo_imax(b, d[k + 3]);
        b = oo_imax(b, d[k + 4]);
        b = oo_imax(b, d[k + 5]);
        if (b >= b0) continue;
        b = oo_imax(b, d[k + 6]);
        b = oo_imax(b, d[k + 7]);
        b = oo_imax(b, d[k + 8]);
        b0 = oo_imin(b0, oo_imax(b, d[k]));
        b0 = oo_imin(b0, oo_imax(b, d[k + 9]));
    }
    return -b0 - 1;
}

/* the 9-of-16 contiguous segment test */
static int oo_is_corner(const uint8_t* ptr, const int* pixel, int t)
{
    const int v = ptr[0];
    int count = 0;
    for (int k = 0; k < 25; k++) {
        if (ptr[pixel[k]] < v - t) { if (++count > 8) return 1; }
        else count = 0;
    }
    count = 0;
    for (int k = 0; k < 25; k++) {
        if (ptr[pixel[k]] > v + t) { if (++count > 8) return 1; }
        else count = 0;
    }
    return 0;
}

int oo_fast_score(const uint8_t* img, int stride, int x, int y)
{
    int pixel[25];
    oo_make_offsets(pixel, stride);
    const uint8_t* p = img + (size_t)y * stride + x;
    if (!oo_is_corner(p, pixel, 0)) return -1;
    return oo_corner_score(p, pixel, 0);
}

/* FAST on the ROI [x0,x1) x [y0,y1) of an image with the given stride; appends keypoints in ROI
 * coordinates, raster order, exactly as FAST_t<16> with nonmax_suppression emits them. */
static void oo_fast_roi(const uint8_t* img, int stride, int x0, int y0, int x1, int y1, int threshold,
                        oo_candvec* out)
{
    const int cols = x1 - x0, rows = y1 - y0;
    if (threshold < 0) threshold = 0;
    if (threshold > 255) threshold = 255;
    if (rows < 7 || cols < 7) return;  /* no interior (the reference's loops are then empty) */
    int pixel[25];
    oo_make_offsets(pixel, stride);
    uint8_t* buf = (uint8_t*)calloc((size_t)rows * cols, 1); /* score map, 0 = not a corner */
    for (int i = 3; i < rows - 3; i++)
        for (int j = 3; j < cols - 3; j++) {
            const uint8_t* p = img + (size_t)(y0 + i) * stride + (x0 + j);
            if (oo_is_corner(p, pixel, threshold))
                buf[(size_t)i * cols + j] = (uint8_t)oo_corner_score(p, pixel, threshold);
        }
    for (int i = 3; i < rows - 3; i++)
        for (int j = 3; j < cols - 3; j++) {
            const int s = buf[(size_t)i * cols + j];
            if (!s) continue; /* not a corner (a score-0 corner can never pass the strict test) */
            const uint8_t* pr = buf + (size_t)(i - 1) * cols;
            const uint8_t* cr = buf + (size_t)i * cols;
            const uint8_t* nr = buf + (size_t)(i + 1) * cols;
            if (s > pr[j - 1] && s > pr[j] && s > pr[j + 1] && s > cr[j - 1] && s > cr[j + 1] &&
                s > nr[j - 1] && s > nr[j] && s > nr[j + 1]) {
                oo_cand c = {(float)j, (float)i, (float)s};
                cv_push(out, c);
            }
        }
    free(buf);
}

/* ------------------------------------------------------------------------------------------------ */
/* Harris response (option OO_SEM_SCORE_HARRIS, not part of ORB-SLAM2, which ranks by the FAST score,    */
/* src/ORBextractor.cc:795-806).  OpenCV's ORB HARRIS_SCORE (modules/features2d/src/orb.cpp               */
/* HarrisResponses, OpenCV 3.x; OpenCV is an external dependency absent from /root/reference): over the  */
/* blockSize x blockSize block centred on the pixel, the 3x3 Sobel-form gradients                        */
/*   Ix = 2 (p[0,1] - p[0,-1]) + (p[-1,1] - p[-1,-1]) + (p[1,1] - p[1,-1]),  Iy likewise over rows,       */
/* the integer sums a = sum Ix^2, b = sum Iy^2, c = sum Ix Iy, and the float response                     */
/*   ((a*b - c*c) - k (a+b) (a+b)) * scale^4,  scale = 1 / (4 * blockSize * 255), k = 0.04, blockSize 7.   */
/* Parity unpinned: no reference fixture holds a Harris response.                       */
/* ------------------------------------------------------------------------------------------------ */
float oo_harris_response(const uint8_t* img, int stride, int x, int y)
{
    const int bs = 7, r = bs / 2;
    const float scale = 1.f / ((1 << 2) * bs * 255.f);
    const float s4 = scale * scale * scale * scale;
    int a = 0, b = 0, c = 0;
    for (int i = -r; i <= r; i++)
        for (int j = -r; j <= r; j++) {
            const uint8_t* p = img + (ptrdiff_t)(y + i) * stride + (x + j);
            const int ix = (p[1] - p[-1]) * 2 + (p[-stride + 1] - p[-stride - 1]) + (p[stride + 1] - p[stride - 1]);
            const int iy = (p[stride] - p[-stride]) * 2 + (p[stride - 1] - p[-stride - 1]) +
                           (p[stride + 1] - p[-stride + 1]);
            a += ix * ix;
            b += iy * iy;
            c += ix * iy;
        }
    const float fa = (float)a, fb = (float)b, fc = (float)c;
    return (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * s4;
}

/* ------------------------------------------------------------------------------------------------ */
/* Octree: ExtractorNode::DivideNode + ORBextractor::DistributeOctTree,                               */
/* src/ORBextractor.cc:481-537, 539-763.  std::list replaced by an index-linked list over a bump pool  */
/* so that the (size, pointer) sort of :684 orders ties by creation order.            */
/* ------------------------------------------------------------------------------------------------ */
typedef struct {
    int ulx, uly, urx, ury, blx, bly, brx, bry;
    oo_candvec keys;
    int noMore;
    int prev, next; /* list links, -1 = none */
} oo_node;

typedef struct {
    oo_node* v;
    int n, cap;
    int head, tail, size;
} oo_nodelist;

static int nl_new(oo_nodelist* L)
{
    if (L->n == L->cap) {
        L->cap = L->cap ? L->cap * 2 : 64;
        L->v = (oo_node*)realloc(L->v, sizeof(oo_node) * (size_t)L->cap);
    }
    memset(&L->v[L->n], 0, sizeof(oo_node));
    L->v[L->n].prev = L->v[L->n].next = -1;
    return L->n++;
}
static void nl_push_front(oo_nodelist* L, int id)
{
    L->v[id].prev = -1;
    L->v[id].next = L->head;
    if (L->head >= 0) L->v[L->head].prev = id; else L->tail = id;
    L->head = id;
    L->size++;
}
static void nl_push_back(oo_nodelist* L, int id)
{
    L->v[id].next = -1;
    L->v[id].prev = L->tail;
    if (L->tail >= 0) L->v[L->tail].next = id; else L->head = id;
    L->tail = id;
    L->size++;
}
static int nl_erase(oo_nodelist* L, int id) /* returns next */
{
    oo_node* n = &L->v[id];
    const int nx = n->next;
    if (n->prev >= 0) L->v[n->prev].next = n->next; else L->head = n->next;
    if (n->next >= 0) L->v[n->next].prev = n->prev; else L->tail = n->prev;
    L->size--;
    free(n->keys.v);
    n->keys.v = NULL;
    return nx;
}

/* children are created (pool ids) in n1..n4 order, as the four locals of the reference */
static void oo_divide(oo_nodelist* L, int pid, int ch[4])
{
    for (int k = 0; k < 4; k++) ch[k] = nl_new(L);
    oo_node* p = &L->v[pid];
    oo_node *n1 = &L->v[ch[0]], *n2 = &L->v[ch[1]], *n3 = &L->v[ch[2]], *n4 = &L->v[ch[3]];
    const int halfX = (int)ceilf((float)(p->urx - p->ulx) / 2);
    const int halfY = (int)ceilf((float)(p->bry - p->uly) / 2);
    n1->ulx = p->ulx; n1->uly = p->uly;
    n1->urx = p->ulx + halfX; n1->ury = p->uly;
    n1->blx = p->ulx; n1->bly = p->uly + halfY;
    n1->brx = p->ulx + halfX; n1->bry = p->uly + halfY;
    n2->ulx = n1->urx; n2->uly = n1->ury;
    n2->urx = p->urx; n2->ury = p->ury;
    n2->blx = n1->brx; n2->bly = n1->bry;
    n2->brx = p->urx; n2->bry = p->uly + halfY;
    n3->ulx = n1->blx; n3->uly = n1->bly;
    n3->urx = n1->brx; n3->ury = n1->bry;
    n3->blx = p->blx; n3->bly = p->bly;
    n3->brx = n1->brx; n3->bry = p->bly;
    n4->ulx = n3->urx; n4->uly = n3->ury;
    n4->urx = n2->brx; n4->ury = n2->bry;
    n4->blx = n3->brx; n4->bly = n3->bry;
    n4->brx = p->brx; n4->bry = p->bry;
    for (int i = 0; i < p->keys.n; i++) {
        const oo_cand kp = p->keys.v[i];
        oo_node* dst;
        if (kp.x < n1->urx) dst = kp.y < n1->bry ? n1 : n3;
        else dst = kp.y < n1->bry ? n2 : n4;
        cv_push(&dst->keys, kp);
    }
    for (int k = 0; k < 4; k++)
        if (L->v[ch[k]].keys.n == 1) L->v[ch[k]].noMore = 1;
}

typedef struct { int size, id; } oo_sizeptr;
static int oo_sizeptr_cmp(const void* a, const void* b)
{
    const oo_sizeptr *x = (const oo_sizeptr*)a, *y = (const oo_sizeptr*)b;
    if (x->size != y->size) return x->size < y->size ? -1 : 1;
    return x->id < y->id ? -1 : (x->id > y->id);
}

static int oo_distribute(const oo_candvec* in, int minX, int maxX, int minY, int maxY, int N,
                         oo_cand* out)
{
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    oo_nodelist L;
    memset(&L, 0, sizeof(L));
    L.head = L.tail = -1;
    int* ini = (int*)malloc(sizeof(int) * (size_t)(nIni > 0 ? nIni : 1));
    for (int i = 0; i < nIni; i++) {
        const int id = nl_new(&L);
        oo_node* ni = &L.v[id];
        ni->ulx = (int)(hX * (float)i); ni->uly = 0;
        ni->urx = (int)(hX * (float)(i + 1)); ni->ury = 0;
        ni->blx = ni->ulx; ni->bly = maxY - minY;
        ni->brx = ni->urx; ni->bry = maxY - minY;
        nl_push_back(&L, id);
        ini[i] = id;
    }
    for (int i = 0; i < in->n; i++) {
        const size_t r = (size_t)(in->v[i].x / hX);
        cv_push(&L.v[ini[r]].keys, in->v[i]);
    }
    for (int it = L.head; it >= 0;) {
        if (L.v[it].keys.n == 1) { L.v[it].noMore = 1; it = L.v[it].next; }
        else if (L.v[it].keys.n == 0) it = nl_erase(&L, it);
        else it = L.v[it].next;
    }
    free(ini);

    int bFinish = 0;
    oo_sizeptr* vsp = NULL;
    int nsp = 0, capsp = 0;
#define PUSH_SP(sz, idv)                                                                  \
    do {                                                                                  \
        if (nsp == capsp) { capsp = capsp ? 2 * capsp : 64;                               \
            vsp = (oo_sizeptr*)realloc(vsp, sizeof(oo_sizeptr) * (size_t)capsp); }        \
        vsp[nsp].size = (sz); vsp[nsp].id = (idv); nsp++;                                 \
    } while (0)

    while (!bFinish) {
        int prevSize = L.size;
        int nToExpand = 0;
        nsp = 0;
        for (int it = L.head; it >= 0;) {
            if (L.v[it].noMore) { it = L.v[it].next; continue; }
            int ch[4];
            oo_divide(&L, it, ch);
            for (int k = 0; k < 4; k++) {
                const int c = ch[k];
                if (L.v[c].keys.n > 0) {
                    nl_push_front(&L, c);
                    if (L.v[c].keys.n > 1) { nToExpand++; PUSH_SP(L.v[c].keys.n, c); }
                }
            }
            it = nl_erase(&L, it);
        }
        if (L.size >= N || L.size == prevSize) {
            bFinish = 1;
        } else if (L.size + nToExpand * 3 > N) {
            while (!bFinish) {
                prevSize = L.size;
                oo_sizeptr* prev = (oo_sizeptr*)malloc(sizeof(oo_sizeptr) * (size_t)(nsp ? nsp : 1));
                const int nprev = nsp;
                memcpy(prev, vsp, sizeof(oo_sizeptr) * (size_t)nsp);
                nsp = 0;
                qsort(prev, (size_t)nprev, sizeof(oo_sizeptr), oo_sizeptr_cmp);
                for (int j = nprev - 1; j >= 0; j--) {
                    int ch[4];
                    oo_divide(&L, prev[j].id, ch);
                    for (int k = 0; k < 4; k++) {
                        const int c = ch[k];
                        if (L.v[c].keys.n > 0) {
                            nl_push_front(&L, c);
                            if (L.v[c].keys.n > 1) PUSH_SP(L.v[c].keys.n, c);
                        }
                    }
                    nl_erase(&L, prev[j].id);
                    if (L.size >= N) break;
                }
                free(prev);
                if (L.size >= N || L.size == prevSize) bFinish = 1;
            }
        }
    }
#undef PUSH_SP
    free(vsp);

    int nout = 0;
    for (int it = L.head; it >= 0; it = L.v[it].next) {
        const oo_candvec* k = &L.v[it].keys;
        int best = 0;
        float maxr = k->v[0].resp;
        for (int i = 1; i < k->n; i++)
            if (k->v[i].resp > maxr) { best = i; maxr = k->v[i].resp; }
        out[nout++] = k->v[best];
    }
    for (int i = 0; i < L.n; i++) free(L.v[i].keys.v);
    free(L.v);
    return nout;
}

/* ------------------------------------------------------------------------------------------------ */
/* IC_Angle (src/ORBextractor.cc:77-104) and computeOrbDescriptor (:108-147)                         */
/* ------------------------------------------------------------------------------------------------ */
static float oo_ic_angle(const uint8_t* img, int stride, float px, float py, const int* umax)
{
    int m01 = 0, m10 = 0;
    const uint8_t* center = img + (size_t)oo_cvround(py) * stride + oo_cvround(px);
    for (int u = -OO_HALF_PATCH; u <= OO_HALF_PATCH; ++u) m10 += u * center[u];
    for (int v = 1; v <= OO_HALF_PATCH; ++v) {
        int v_sum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int vp = center[u + v * stride], vm = center[u - v * stride];
            v_sum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * v_sum;
    }
    return oo_fast_atan2((float)m01, (float)m10);
}

static void oo_orb_descriptor(float kx, float ky, float angle_deg, const uint8_t* img, int stride,
                              uint8_t* desc, int nofma)
{
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float angle = angle_deg * factorPI;
    float a = 0.f, b = 0.f; /* angle in [0, 2pi]: oo_sincosf always writes both (its |y| >= 120 branch is unreachable) */
    oo_sincosf(angle, &b, &a);
    const uint8_t* center = img + (size_t)oo_cvround(ky) * stride + oo_cvround(kx);
    const signed char* pat = oo_orb_pattern;
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int k = 0; k < 8; k++, pat += 4) {
            int t[2];
            for (int q = 0; q < 2; q++) {
                const float x = (float)pat[2 * q], y = (float)pat[2 * q + 1];
                /* GCC -O3 -march=native contraction of the GET_VALUE expressions, or the
                 * separately rounded products of a build without FMA contraction (OO_SEM_BRIEF_NOFMA) */
                int row, col;
                if (nofma) {
                    row = oo_cvround(x * b + y * a);
                    col = oo_cvround(x * a - y * b);
                } else {
                    row = oo_cvround(fmaf(x, b, y * a));
                    col = oo_cvround(fmaf(x, a, -(y * b)));
                }
                t[q] = center[row * stride + col];
            }
            val |= (t[0] < t[1]) << k;
        }
        desc[i] = (uint8_t)val;
    }
}

float oo_fastatan2(float y, float x) { return oo_fast_atan2(y, x); }
void oo_sincos(float ang, float* s, float* c) { oo_sincosf(ang, s, c); }

/* ------------------------------------------------------------------------------------------------ */
/* ORBextractor::operator() (src/ORBextractor.cc:1043-1105) with ComputePyramid (:1107-1132) and      */
/* ComputeKeyPointsOctTree (:765-853).                                                                */
/* ------------------------------------------------------------------------------------------------ */
int oo_extract(oo_extractor* e, const uint8_t* img, int cols, int rows, int step, oo_keypoint* kps,
               uint8_t* desc, int cap)
{
    if (!img || cols <= 0 || rows <= 0) return 0; /* _image.empty(): outputs untouched */
    const int nl = e->nlevels;
    /* ComputePyramid */
    for (int l = 0; l < nl; l++) {
        const int w = oo_cvround((float)cols * e->isf[l]);
        const int h = oo_cvround((float)rows * e->isf[l]);
        free(e->lev[l]);
        e->lev[l] = (uint8_t*)malloc((size_t)w * (size_t)h);
        e->lw[l] = w;
        e->lh[l] = h;
        if (l == 0) {
            for (int y = 0; y < h; y++) memcpy(e->lev[0] + (size_t)y * w, img + (size_t)y * step, (size_t)w);
        } else {
            oo_resize_linear(e->lev[l - 1], e->lw[l - 1], e->lh[l - 1], e->lev[l], w, h, e->sem);
        }
    }
    /* ComputeKeyPointsOctTree */
    oo_keypoint* all[OO_MAXLEVELS];
    int nall[OO_MAXLEVELS];
    const float W = 30;
    for (int l = 0; l < nl; l++) {
        const uint8_t* im = e->lev[l];
        const int lw = e->lw[l], lh = e->lh[l];
        const int minBX = OO_EDGE - 3, minBY = minBX;
        const int maxBX = lw - OO_EDGE + 3, maxBY = lh - OO_EDGE + 3;
        oo_candvec* cand = &e->cand[l];
        cand->n = 0;
        const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
        oo_candvec cell = {0, 0, 0};
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBY - 3) continue;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBX - 6) continue;
                if (maxX > maxBX) maxX = (float)maxBX;
                cell.n = 0;
                oo_fast_roi(im, lw, (int)iniX, (int)iniY, (int)maxX, (int)maxY, e->iniTh, &cell);
                if (cell.n == 0) oo_fast_roi(im, lw, (int)iniX, (int)iniY, (int)maxX, (int)maxY, e->minTh, &cell);
                for (int k = 0; k < cell.n; k++) {
                    oo_cand c = cell.v[k];
                    c.x += (float)(j * wCell);
                    c.y += (float)(i * hCell);
                    cv_push(cand, c);
                }
            }
        }
        free(cell.v);
        if (e->sem & OO_SEM_SCORE_HARRIS) /* option: rank by the Harris response at the level pixel */
            for (int k = 0; k < cand->n; k++)
                cand->v[k].resp = oo_harris_response(im, lw, (int)cand->v[k].x + minBX, (int)cand->v[k].y + minBY);
        oo_cand* dist = (oo_cand*)malloc(sizeof(oo_cand) * (size_t)(cand->n + 1));
        const int nd = oo_distribute(cand, minBX, maxBX, minBY, maxBY, e->nfeat[l], dist);
        const int scaledPatchSize = (int)(OO_PATCH_SIZE * e->sf[l]);
        all[l] = (oo_keypoint*)malloc(sizeof(oo_keypoint) * (size_t)(nd + 1));
        nall[l] = nd;
        for (int i = 0; i < nd; i++) {
            oo_keypoint* k = &all[l][i];
            k->x = dist[i].x + (float)minBX;
            k->y = dist[i].y + (float)minBY;
            k->size = (float)scaledPatchSize;
            k->angle = -1.f;
            k->response = dist[i].resp;
            k->octave = l;
            k->class_id = -1;
        }
        free(dist);
    }
    for (int l = 0; l < nl; l++)
        for (int i = 0; i < nall[l]; i++)
            all[l][i].angle = oo_ic_angle(e->lev[l], e->lw[l], all[l][i].x, all[l][i].y, e->umax);

    int total = 0;
    for (int l = 0; l < nl; l++) total += nall[l];
    if (total > cap) {
        for (int l = 0; l < nl; l++) free(all[l]);
        return -1;
    }
    int off = 0;
    for (int l = 0; l < nl; l++) {
        if (nall[l] == 0) { free(all[l]); continue; }
        uint8_t* blurred = (uint8_t*)malloc((size_t)e->lw[l] * (size_t)e->lh[l]);
        oo_gaussian7(e->lev[l], e->lw[l], e->lh[l], blurred, e->sem);
        for (int i = 0; i < nall[l]; i++)
            oo_orb_descriptor(all[l][i].x, all[l][i].y, all[l][i].angle, blurred, e->lw[l],
                              desc + (size_t)(off + i) * 32, (e->sem & OO_SEM_BRIEF_NOFMA) != 0);
        free(blurred);
        if (l != 0) {
            const float s = e->sf[l];
            for (int i = 0; i < nall[l]; i++) { all[l][i].x *= s; all[l][i].y *= s; }
        }
        memcpy(kps + off, all[l], sizeof(oo_keypoint) * (size_t)nall[l]);
        off += nall[l];
        free(all[l]);
    }
    return total;
}

int oo_distribute_octree(const float* xy, const float* resp, int n, int minX, int maxX, int minY, int maxY,
                         int N, float* out_xy, float* out_resp)
{
    oo_candvec in = {0, 0, 0};
    for (int i = 0; i < n; i++) {
        oo_cand c = {xy[2 * i], xy[2 * i + 1], resp[i]};
        cv_push(&in, c);
    }
    oo_cand* out = (oo_cand*)malloc(sizeof(oo_cand) * (size_t)(n + 1));
    const int m = oo_distribute(&in, minX, maxX, minY, maxY, N, out);
    for (int i = 0; i < m; i++) {
        out_xy[2 * i] = out[i].x;
        out_xy[2 * i + 1] = out[i].y;
        out_resp[i] = out[i].resp;
    }
    free(out);
    free(in.v);
    return m;
}

int oo_level_size(const oo_extractor* e, int level, int* cols, int* rows)
{
    if (level < 0 || level >= e->nlevels) return -1;
    *cols = e->lw[level];
    *rows = e->lh[level];
    return 0;
}
const uint8_t* oo_level_image(const oo_extractor* e, int level) { return e->lev[level]; }
int oo_level_candidates(const oo_extractor* e, int level, float* xy, float* resp, int cap)
{
    const oo_candvec* c = &e->cand[level];
    for (int i = 0; i < c->n && i < cap; i++) {
        xy[2 * i] = c->v[i].x;
        xy[2 * i + 1] = c->v[i].y;
        resp[i] = c->v[i].resp;
    }
    return c->n;
}

/* ------------------------------------------------------------------------------------------------ */
/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1647-1663)                                      */
/* ------------------------------------------------------------------------------------------------ */
int oo_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24);
    }
    return dist;
}

/* ------------------------------------------------------------------------------------------------ */
/* Frame grid: ComputeImageBounds (no distortion, src/Frame.cc:457-463), grid scales (:212-213),     */
/* AssignFeaturesToGrid (:230-245), PosInGrid (:382-392), GetFeaturesInArea (:327-380)               */
/* ------------------------------------------------------------------------------------------------ */
void oo_grid_params(int cols, int rows, float* minX, float* minY, float* maxX, float* maxY,
                    float* invW, float* invH)
{
    *minX = 0.0f;
    *maxX = (float)cols;
    *minY = 0.0f;
    *maxY = (float)rows;
    *invW = (float)OO_GRID_COLS / (*maxX - *minX);
    *invH = (float)OO_GRID_ROWS / (*maxY - *minY);
}

static int oo_pos_in_grid(const oo_frame* f, const oo_keypoint* kp, int* px, int* py)
{
    *px = (int)roundf((kp->x - f->minX) * f->gridInvW);
    *py = (int)roundf((kp->y - f->minY) * f->gridInvH);
    if (*px < 0 || *px >= OO_GRID_COLS || *py < 0 || *py >= OO_GRID_ROWS) return 0;
    return 1;
}

void oo_grid_build(oo_frame* f)
{
    const int nc = OO_GRID_COLS * OO_GRID_ROWS;
    int* cnt = (int*)calloc((size_t)nc + 1, sizeof(int));
    for (int i = 0; i < f->n; i++) {
        int px, py;
        if (oo_pos_in_grid(f, &f->kps[i], &px, &py)) cnt[px * OO_GRID_ROWS + py]++;
    }
    f->cell_start[0] = 0;
    for (int c = 0; c < nc; c++) f->cell_start[c + 1] = f->cell_start[c] + cnt[c];
    memset(cnt, 0, sizeof(int) * (size_t)nc);
    for (int i = 0; i < f->n; i++) {
        int px, py;
        if (oo_pos_in_grid(f, &f->kps[i], &px, &py)) {
            const int c = px * OO_GRID_ROWS + py;
            f->cell_items[f->cell_start[c] + cnt[c]++] = i;
        }
    }
    free(cnt);
}

int oo_features_in_area(const oo_frame* f, float x, float y, float r, int minLevel, int maxLevel,
                        int* out)
{
    int n = 0;
    const int nMinCellX = oo_imax(0, (int)floorf((x - f->minX - r) * f->gridInvW));
    if (nMinCellX >= OO_GRID_COLS) return 0;
    const int nMaxCellX = oo_imin(OO_GRID_COLS - 1, (int)ceilf((x - f->minX + r) * f->gridInvW));
    if (nMaxCellX < 0) return 0;
    const int nMinCellY = oo_imax(0, (int)floorf((y - f->minY - r) * f->gridInvH));
    if (nMinCellY >= OO_GRID_ROWS) return 0;
    const int nMaxCellY = oo_imin(OO_GRID_ROWS - 1, (int)ceilf((y - f->minY + r) * f->gridInvH));
    if (nMaxCellY < 0) return 0;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * OO_GRID_ROWS + iy;
            for (int j = f->cell_start[c]; j < f->cell_start[c + 1]; j++) {
                const int idx = f->cell_items[j];
                const oo_keypoint* kp = &f->kps[idx];
                if (bCheckLevels) {
                    if (kp->octave < minLevel) continue;
                    if (maxLevel >= 0 && kp->octave > maxLevel) continue;
                }
                const float distx = kp->x - x, disty = kp->y - y;
                if (fabsf(distx) < r && fabsf(disty) < r) out[n++] = idx;
            }
        }
    return n;
}

/* ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1601-1642) */
static void oo_three_maxima(const int* histo_len, int L, int* ind1, int* ind2, int* ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = histo_len[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            *ind3 = *ind2; *ind2 = i;
        } else if (s > max3) {
            max3 = s;
            *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) { *ind2 = -1; *ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { *ind3 = -1; }
}

#define OO_TH_HIGH 100
#define OO_TH_LOW 50
#define OO_HISTO 30

/* ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:405-520) */
int oo_search_for_initialization(const oo_frame* F1, const oo_frame* F2, float nnratio, int checkOri,
                                 float* prev_xy, int* matches12, int windowSize)
{
    int nmatches = 0;
    for (int i = 0; i < F1->n; i++) matches12[i] = -1;
    int* hist = (int*)malloc(sizeof(int) * OO_HISTO * (size_t)(F1->n + 1));
    int hlen[OO_HISTO] = {0};
    const float factor = 1.0f / OO_HISTO;
    int* vMatchedDistance = (int*)malloc(sizeof(int) * (size_t)(F2->n + 1));
    int* vnMatches21 = (int*)malloc(sizeof(int) * (size_t)(F2->n + 1));
    int* idx = (int*)malloc(sizeof(int) * (size_t)(F2->n + 1));
    for (int i = 0; i < F2->n; i++) { vMatchedDistance[i] = INT_MAX; vnMatches21[i] = -1; }

    for (int i1 = 0; i1 < F1->n; i1++) {
        const oo_keypoint kp1 = F1->kps[i1];
        const int level1 = kp1.octave;
        if (level1 > 0) continue;
        const int nc = oo_features_in_area(F2, prev_xy[2 * i1], prev_xy[2 * i1 + 1], (float)windowSize,
                                           level1, level1, idx);
        if (nc == 0) continue;
        const uint8_t* d1 = F1->desc + (size_t)i1 * 32;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = idx[c];
            const int dist = oo_descriptor_distance(d1, F2->desc + (size_t)i2 * 32);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx2 = i2; }
            else if (dist < bestDist2) bestDist2 = dist;
        }
        if (bestDist <= OO_TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    matches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                matches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) {
                    float rot = F1->kps[i1].angle - F2->kps[bestIdx2].angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == OO_HISTO) bin = 0;
                    assert(bin >= 0 && bin < OO_HISTO);
                    hist[bin * (F1->n + 1) + hlen[bin]++] = i1;
                }
            }
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        oo_three_maxima(hlen, OO_HISTO, &ind1, &ind2, &ind3);
        for (int i = 0; i < OO_HISTO; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j = 0; j < hlen[i]; j++) {
                const int idx1 = hist[i * (F1->n + 1) + j];
                if (matches12[idx1] >= 0) { matches12[idx1] = -1; nmatches--; }
            }
        }
    }
    for (int i1 = 0; i1 < F1->n; i1++)
        if (matches12[i1] >= 0) {
            prev_xy[2 * i1] = F2->kps[matches12[i1]].x;
            prev_xy[2 * i1 + 1] = F2->kps[matches12[i1]].y;
        }
    free(hist);
    free(vMatchedDistance);
    free(vnMatches21);
    free(idx);
    return nmatches;
}

/* ORBmatcher::RadiusByViewingCos (src/ORBmatcher.cc:131-137) */
static float oo_radius_by_viewing_cos(float viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:45-129) */
int oo_search_by_projection(const oo_frame* F, const oo_mappoints* mp, float nnratio, float th,
                            int* owner, int* owner_obs)
{
    int nmatches = 0;
    const int bFactor = th != 1.0;
    int* idx = (int*)malloc(sizeof(int) * (size_t)(F->n + 1));
    for (int m = 0; m < mp->m; m++) {
        if (!mp->track_in_view[m]) continue;
        if (mp->is_bad[m]) continue;
        const int nPredictedLevel = mp->level[m];
        float r = oo_radius_by_viewing_cos(mp->view_cos[m]);
        if (bFactor) r *= th;
        const int nc = oo_features_in_area(F, mp->proj_x[m], mp->proj_y[m],
                                           r * F->scale_factors[nPredictedLevel], nPredictedLevel - 1,
                                           nPredictedLevel, idx);
        if (nc == 0) continue;
        const uint8_t* MPdescriptor = mp->desc + (size_t)m * 32;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int i = idx[c];
            if (owner[i] >= 0 && owner_obs[i]) continue;
            if (F->uright && F->uright[i] > 0) {
                const float er = fabsf(mp->proj_xr[m] - F->uright[i]);
                if (er > r * F->scale_factors[nPredictedLevel]) continue;
            }
            const int dist = oo_descriptor_distance(MPdescriptor, F->desc + (size_t)i * 32);
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist;
                bestLevel2 = bestLevel; bestLevel = F->kps[i].octave;
                bestIdx = i;
            } else if (dist < bestDist2) {
                bestLevel2 = F->kps[i].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= OO_TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            owner[bestIdx] = m;
            owner_obs[bestIdx] = mp->n_obs[m] > 0;
            nmatches++;
        }
    }
    free(idx);
    return nmatches;
}

/* ------------------------------------------------------------------------------------------------ */
/* Frame::ComputeStereoMatches (src/Frame.cc:466-640): left keypoints/descriptors (mvKeys), right      */
/* keypoints/descriptors (mvKeysRight), both extractors' pyramids (mvImagePyramid).                    */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { int first, second; } oo_pair;
static int oo_pair_cmp(const void* a, const void* b)
{
    const oo_pair *x = (const oo_pair*)a, *y = (const oo_pair*)b;
    if (x->first != y->first) return x->first < y->first ? -1 : 1;
    return x->second < y->second ? -1 : (x->second > y->second);
}

int oo_stereo_matches(const oo_extractor* EL, const oo_extractor* ER, const oo_keypoint* kL, const uint8_t* dL,
                      int N, const oo_keypoint* kR, const uint8_t* dR, int Nr, float mbf, float mb,
                      float* uright, float* depth)
{
    for (int i = 0; i < N; i++) { uright[i] = -1.0f; depth[i] = -1.0f; }
    const int thOrbDist = (OO_TH_HIGH + OO_TH_LOW) / 2;
    const int nRows = EL->lh[0];
    int* rowCnt = (int*)calloc((size_t)nRows + 1, sizeof(int));
    /* row -> right keypoint indices, in iR order (vRowIndices, :476-493) */
    for (int pass = 0; pass < 2; pass++) {
        for (int iR = 0; iR < Nr; iR++) {
            const float kpY = kR[iR].y;
            const float r = 2.0f * EL->sf[kR[iR].octave];
            const int maxr = (int)ceilf(kpY + r);
            const int minr = (int)floorf(kpY - r);
            for (int yi = minr; yi <= maxr; yi++) {
                if (yi < 0 || yi >= nRows) continue; /* out of range is UB in the reference */
                rowCnt[yi]++;
            }
        }
        if (pass == 0) break;
    }
    int* rowStart = (int*)malloc(sizeof(int) * ((size_t)nRows + 1));
    rowStart[0] = 0;
    for (int y = 0; y < nRows; y++) rowStart[y + 1] = rowStart[y] + rowCnt[y];
    int* rowItems = (int*)malloc(sizeof(int) * ((size_t)rowStart[nRows] + 1));
    memset(rowCnt, 0, sizeof(int) * (size_t)nRows);
    for (int iR = 0; iR < Nr; iR++) {
        const float kpY = kR[iR].y;
        const float r = 2.0f * EL->sf[kR[iR].octave];
        const int maxr = (int)ceilf(kpY + r);
        const int minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++) {
            if (yi < 0 || yi >= nRows) continue;
            rowItems[rowStart[yi] + rowCnt[yi]++] = iR;
        }
    }
    const float minZ = mb;
    const float minD = 0;
    const float maxD = mbf / minZ;
    oo_pair* vDistIdx = (oo_pair*)malloc(sizeof(oo_pair) * ((size_t)N + 1));
    int nDist = 0;
    for (int iL = 0; iL < N; iL++) {
        const oo_keypoint* kpL = &kL[iL];
        const int levelL = kpL->octave;
        const float vL = kpL->y, uL = kpL->x;
        const int row = (int)vL;
        if (row < 0 || row >= nRows) continue;
        const int cb = rowStart[row], ce = rowStart[row + 1];
        if (cb == ce) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = OO_TH_HIGH;
        int bestIdxR = 0;
        const uint8_t* dl = dL + (size_t)iL * 32;
        for (int c = cb; c < ce; c++) {
            const int iR = rowItems[c];
            const oo_keypoint* kpR = &kR[iR];
            if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
            const float uR = kpR->x;
            if (uR >= minU && uR <= maxU) {
                const int dist = oo_descriptor_distance(dl, dR + (size_t)iR * 32);
                if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
            }
        }
        if (bestDist < thOrbDist) {
            const float uR0 = kR[bestIdxR].x;
            const float scaleFactor = EL->isf[kpL->octave];
            const float scaleduL = roundf(kpL->x * scaleFactor);
            const float scaledvL = roundf(kpL->y * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            const int w = 5;
            const int lw = EL->lw[levelL];
            const uint8_t* IL = EL->lev[levelL];
            const uint8_t* IRim = ER->lev[levelL];
            const int rw = ER->lw[levelL];
            const int ivL = (int)scaledvL, iuL = (int)scaleduL, iuR0 = (int)scaleduR0;
            const float cL = (float)IL[(size_t)ivL * lw + iuL];
            int bestD = INT_MAX;
            int bestincR = 0;
            const int L = 5;
            float vDists[11];
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= rw) continue;
            for (int incR = -L; incR <= +L; incR++) {
                const float cR = (float)IRim[(size_t)ivL * rw + iuR0 + incR];
                double acc = 0; /* cv::norm(IL, IR, NORM_L1) on CV_32F: exact (integer-valued) */
                for (int yy = -w; yy <= w; yy++)
                    for (int xx = -w; xx <= w; xx++) {
                        const float a = (float)IL[(size_t)(ivL + yy) * lw + iuL + xx] - cL;
                        const float b = (float)IRim[(size_t)(ivL + yy) * rw + iuR0 + incR + xx] - cR;
                        acc += fabs((double)a - (double)b);
                    }
                const float dist = (float)acc;
                if (dist < bestD) { bestD = (int)dist; bestincR = incR; }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[L + bestincR - 1];
            const float dist2 = vDists[L + bestincR];
            const float dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = EL->sf[kpL->octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01f;
                    bestuR = (float)((double)uL - 0.01);
                }
                depth[iL] = mbf / disparity;
                uright[iL] = bestuR;
                vDistIdx[nDist].first = bestD;
                vDistIdx[nDist].second = iL;
                nDist++;
            }
        }
    }
    int nvalid = nDist;
    if (nDist > 0) {
        qsort(vDistIdx, (size_t)nDist, sizeof(oo_pair), oo_pair_cmp);
        const float median = (float)vDistIdx[nDist / 2].first;
        const float thDist = 1.5f * 1.4f * median;
        for (int i = nDist - 1; i >= 0; i--) {
            if (vDistIdx[i].first < thDist) break;
            uright[vDistIdx[i].second] = -1;
            depth[vDistIdx[i].second] = -1;
            nvalid--;
        }
    }
    free(rowCnt);
    free(rowStart);
    free(rowItems);
    free(vDistIdx);
    return nvalid;
}

/* ------------------------------------------------------------------------------------------------ */
/* Projection helpers.  cv::Mat float algebra of the reference, pinned (OpenCV internals are not     */
/* available here): R*x + t as ((r0*x0 + r1*x1) + r2*x2) + t in float (OpenCV's     */
/* small-matrix gemm path; OpenCV is not built with FMA); the reference's own expressions contract   */
/* into fma under GCC -O3 -march=native (tools/probe_contraction_proj.cc).                            */
/* ------------------------------------------------------------------------------------------------ */
static void oo_rx_plus_t(const float* R, const float* x, const float* t, float* out)
{
    for (int r = 0; r < 3; r++) {
        float s = R[3 * r] * x[0];
        s = s + R[3 * r + 1] * x[1];
        s = s + R[3 * r + 2] * x[2];
        out[r] = s + t[r];
    }
}

/* Frame::isInFrustum (src/Frame.cc:269-325) + MapPoint::PredictScale (src/MapPoint.cc:402-417) */
int oo_is_in_frustum(const oo_camera* cam, const oo_mappoint_geom* mp, float viewingCosLimit, uint8_t* in_view,
                     float* proj_x, float* proj_y, float* proj_xr, int* level, float* view_cos)
{
    const float logsf = oo_logf(cam->scale_factor);  /* mfLogScaleFactor = log(mfScaleFactor), :71 */
    int nin = 0;
    for (int m = 0; m < mp->m; m++) {
        in_view[m] = 0;
        const float* P = mp->pos + 3 * (size_t)m;
        float Pc[3];
        oo_rx_plus_t(cam->Rcw, P, cam->tcw, Pc);
        if (Pc[2] < 0.0f) continue;
        const float invz = 1.0f / Pc[2];
        const float u = fmaf(cam->fx * Pc[0], invz, cam->cx);
        const float v = fmaf(cam->fy * Pc[1], invz, cam->cy);
        if (u < cam->minX || u > cam->maxX) continue;
        if (v < cam->minY || v > cam->maxY) continue;
        const float maxDistance = 1.2f * mp->max_dist[m];  /* GetMaxDistanceInvariance, src/MapPoint.cc:379 */
        const float minDistance = 0.8f * mp->min_dist[m];  /* GetMinDistanceInvariance, :373 */
        const float PO[3] = {P[0] - cam->Ow[0], P[1] - cam->Ow[1], P[2] - cam->Ow[2]};
        /* cv::norm(PO): NORM_L2 of 32F accumulates squares in double, sqrt in double */
        double ss = 0.0;
        for (int k = 0; k < 3; k++) ss += (double)PO[k] * (double)PO[k];
        const float dist = (float)sqrt(ss);
        if (dist < minDistance || dist > maxDistance) continue;
        /* PO.dot(Pn): double accumulation of float products; /dist in double */
        const float* Pn = mp->normal + 3 * (size_t)m;
        double dot = 0.0;
        for (int k = 0; k < 3; k++) dot += (double)PO[k] * (double)Pn[k];
        const float viewCos = (float)(dot / (double)dist);
        if (viewCos < viewingCosLimit) continue;
        /* PredictScale: ratio = mfMaxDistance/currentDist; ceil(log(ratio)/mfLogScaleFactor), clamp */
        const float ratio = mp->max_dist[m] / dist;
        int nScale = (int)ceilf(oo_logf(ratio) / logsf);
        if (nScale < 0) nScale = 0;
        else if (nScale >= cam->nlevels) nScale = cam->nlevels - 1;
        in_view[m] = 1;
        proj_x[m] = u;
        proj_xr[m] = fmaf(-cam->mbf, invz, u);
        proj_y[m] = v;
        level[m] = nScale;
        view_cos[m] = viewCos;
        nin++;
    }
    return nin;
}

/* ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (src/ORBmatcher.cc:1328-1470) */
int oo_search_by_projection_last(const oo_frame* F, const oo_camera* cur, const oo_camera* last,
                                 const oo_last_frame* LF, float th, int bMono, int checkOri, int* owner,
                                 int* owner_obs)
{
    int nmatches = 0;
    const float factor = 1.0f / OO_HISTO;
    int hlen[OO_HISTO] = {0};
    int* hist = (int*)malloc(sizeof(int) * OO_HISTO * (size_t)(LF->n + 1));
    int* idx = (int*)malloc(sizeof(int) * (size_t)(F->n + 1));
    /* twc = -Rcw^T tcw ; tlc = Rlw*twc + tlw  (:1338-1346) */
    float twc[3], tlc[3];
    for (int j = 0; j < 3; j++) {
        float s = cur->Rcw[j] * cur->tcw[0];
        s = s + cur->Rcw[3 + j] * cur->tcw[1];
        s = s + cur->Rcw[6 + j] * cur->tcw[2];
        twc[j] = -s;
    }
    oo_rx_plus_t(last->Rcw, twc, last->tcw, tlc);
    const int bForward = tlc[2] > cur->mb && !bMono;
    const int bBackward = -tlc[2] > cur->mb && !bMono;
    for (int i = 0; i < LF->n; i++) {
        if (!LF->has_mp[i] || LF->outlier[i]) continue;
        float x3Dc[3];
        oo_rx_plus_t(cur->Rcw, LF->pos + 3 * (size_t)i, cur->tcw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0) continue;
        const float u = fmaf(cur->fx * xc, invzc, cur->cx);
        const float v = fmaf(cur->fy * yc, invzc, cur->cy);
        if (u < F->minX || u > F->maxX) continue;
        if (v < F->minY || v > F->maxY) continue;
        if (u != u || v != v) continue;  /* zc == 0 with xc == 0: undefined in the reference */
        const int nLastOctave = LF->kps[i].octave;
        const float radius = th * F->scale_factors[nLastOctave];
        int nc;
        if (bForward) nc = oo_features_in_area(F, u, v, radius, nLastOctave, -1, idx);
        else if (bBackward) nc = oo_features_in_area(F, u, v, radius, 0, nLastOctave, idx);
        else nc = oo_features_in_area(F, u, v, radius, nLastOctave - 1, nLastOctave + 1, idx);
        if (nc == 0) continue;
        const uint8_t* dMP = LF->desc + 32 * (size_t)i;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = idx[c];
            if (owner[i2] >= 0 && owner_obs[i2]) continue;
            if (F->uright && F->uright[i2] > 0) {
                const float ur = fmaf(-cur->mbf, invzc, u);
                const float er = fabsf(ur - F->uright[i2]);
                if (er > radius) continue;
            }
            const int dist = oo_descriptor_distance(dMP, F->desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= OO_TH_HIGH) {
            owner[bestIdx2] = i;
            owner_obs[bestIdx2] = LF->n_obs[i] > 0;
            nmatches++;
            if (checkOri) {
                float rot = LF->kps[i].angle - F->kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == OO_HISTO) bin = 0;
                assert(bin >= 0 && bin < OO_HISTO);
                hist[bin * (LF->n + 1) + hlen[bin]++] = bestIdx2;
            }
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        oo_three_maxima(hlen, OO_HISTO, &ind1, &ind2, &ind3);
        for (int b = 0; b < OO_HISTO; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int j = 0; j < hlen[b]; j++) {
                const int i2 = hist[b * (LF->n + 1) + j];
                owner[i2] = -1;
                owner_obs[i2] = 0;
                nmatches--;
            }
        }
    }
    free(hist);
    free(idx);
    return nmatches;
}

/* ------------------------------------------------------------------------------------------------ */
/* cv::undistortPoints(src, dst, K, D, noArray(), K) as Frame::UndistortKeyPoints (src/Frame.cc:404-434)  */
/* and Frame::ComputeImageBounds (:436-461) call it.  OpenCV 3.4 cvUndistortPointsInternal with the     */
/* default TermCriteria(COUNT, 5, 0.01): 5 fixed-point iterations in double; R = I, P = K; the tilt and */
/* thin-prism terms are identity / +0.0 for <= 5 coefficients.  OpenCV's baseline build has no FMA.     */
/* ------------------------------------------------------------------------------------------------ */
void oo_undistort_points(const float* K4, const float* dist, int ndist, const float* xy, float* out, int n)
{
    double k[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < ndist && i < 5; i++) k[i] = (double)dist[i];
    const double fx = K4[0], fy = K4[1], cx = K4[2], cy = K4[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    for (int i = 0; i < n; i++) {
        double x = xy[2 * i], y = xy[2 * i + 1];
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            const double r2 = x * x + y * y;
            const double icdist = 1. / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        /* P = K, R = I: xx = fx*x + 0*y + cx, yy = 0*x + fy*y + cy, ww = 1/(0*x + 0*y + 1) */
        out[2 * i] = (float)(fx * x + cx);
        out[2 * i + 1] = (float)(fy * y + cy);
    }
}

void oo_undistort_keypoints(const float* K4, const float* dist, int ndist, const oo_keypoint* in, oo_keypoint* out,
                            int n)
{
    for (int i = 0; i < n; i++) out[i] = in[i];
    if (ndist < 1 || dist[0] == 0.0f) return;  /* mDistCoef.at<float>(0)==0.0: mvKeysUn = mvKeys */
    for (int i = 0; i < n; i++) {
        float p[2] = {in[i].x, in[i].y}, q[2];
        oo_undistort_points(K4, dist, ndist, p, q, 1);
        out[i].x = q[0];
        out[i].y = q[1];
    }
}

/* Frame::ComputeImageBounds (src/Frame.cc:436-461) + the grid scales (src/Frame.cc:103-104) */
void oo_compute_image_bounds(const float* K4, const float* dist, int ndist, int cols, int rows, float* minX,
                             float* maxX, float* minY, float* maxY, float* invW, float* invH)
{
    if (ndist >= 1 && dist[0] != 0.0f) {
        const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
        float u[8];
        oo_undistort_points(K4, dist, ndist, c, u, 4);
        *minX = fminf(u[0], u[4]);
        *maxX = fmaxf(u[2], u[6]);
        *minY = fminf(u[1], u[3]);
        *maxY = fmaxf(u[5], u[7]);
    } else {
        *minX = 0.0f;
        *maxX = (float)cols;
        *minY = 0.0f;
        *maxY = (float)rows;
    }
    *invW = (float)OO_GRID_COLS / (*maxX - *minX);
    *invH = (float)OO_GRID_ROWS / (*maxY - *minY);
}

/* The scale gate of the relocalisation matcher per keyframe point, as the drop-in binding computes it with the
 * reference's own MapPoint methods (src/ORBmatcher.cc:1513-1523; PredictScale src/MapPoint.cc:402-417):
 * level[i] = PredictScale(dist3D) when 0.8 * mfMinDistance <= dist3D <= 1.2 * mfMaxDistance, else -1 (and -1 for
 * invalid points).  dist3D = ||X - Ow||, Ow = -Rcw^T tcw as below. */
void oo_kf_predicted_levels(const oo_camera* cur, const oo_keyframe* KF, int* level)
{
    const float logsf = oo_logf(cur->scale_factor);
    float Ow[3];
    for (int j = 0; j < 3; j++) {
        float s = cur->Rcw[j] * cur->tcw[0];
        s = s + cur->Rcw[3 + j] * cur->tcw[1];
        s = s + cur->Rcw[6 + j] * cur->tcw[2];
        Ow[j] = -s;
    }
    for (int i = 0; i < KF->n; i++) {
        level[i] = -1;
        if (!KF->valid[i]) continue;
        const float* X = KF->pos + 3 * (size_t)i;
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        double ss = 0.0;
        for (int k = 0; k < 3; k++) ss += (double)PO[k] * (double)PO[k];
        const float dist3D = (float)sqrt(ss);
        if (dist3D < 0.8f * KF->min_dist[i] || dist3D > 1.2f * KF->max_dist[i]) continue;
        int l = (int)ceilf(oo_logf(KF->max_dist[i] / dist3D) / logsf);
        level[i] = l < 0 ? 0 : (l >= cur->nlevels ? cur->nlevels - 1 : l);
    }
}

/* ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)
 * (src/ORBmatcher.cc:1472-1599): relocalisation / loop matcher of the map points of one keyframe */
int oo_search_by_projection_kf(const oo_frame* F, const oo_camera* cur, const oo_keyframe* KF, float th, int ORBdist,
                               int checkOri, int* owner)
{
    int nmatches = 0;
    const float factor = 1.0f / OO_HISTO;
    int hlen[OO_HISTO] = {0};
    int* hist = (int*)malloc(sizeof(int) * OO_HISTO * (size_t)(KF->n + 1));
    int* idx = (int*)malloc(sizeof(int) * (size_t)(F->n + 1));
    const float logsf = oo_logf(cur->scale_factor);
    float Ow[3];  /* Ow = -Rcw^T tcw (:1478), pinned like twc in oo_search_by_projection_last */
    for (int j = 0; j < 3; j++) {
        float s = cur->Rcw[j] * cur->tcw[0];
        s = s + cur->Rcw[3 + j] * cur->tcw[1];
        s = s + cur->Rcw[6 + j] * cur->tcw[2];
        Ow[j] = -s;
    }
    for (int i = 0; i < KF->n; i++) {
        if (!KF->valid[i]) continue;
        const float* X = KF->pos + 3 * (size_t)i;
        float x3Dc[3];
        oo_rx_plus_t(cur->Rcw, X, cur->tcw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        const float u = fmaf(cur->fx * xc, invzc, cur->cx);
        const float v = fmaf(cur->fy * yc, invzc, cur->cy);
        if (u < F->minX || u > F->maxX) continue;
        if (v < F->minY || v > F->maxY) continue;
        if (u != u || v != v) continue;  /* zc == 0 with xc == 0: undefined in the reference */
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        double ss = 0.0;
        for (int k = 0; k < 3; k++) ss += (double)PO[k] * (double)PO[k];
        const float dist3D = (float)sqrt(ss);
        const float maxDistance = 1.2f * KF->max_dist[i];
        const float minDistance = 0.8f * KF->min_dist[i];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        int nPredictedLevel = (int)ceilf(oo_logf(KF->max_dist[i] / dist3D) / logsf);
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= cur->nlevels) nPredictedLevel = cur->nlevels - 1;
        const float radius = th * F->scale_factors[nPredictedLevel];
        const int nc = oo_features_in_area(F, u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1, idx);
        if (nc == 0) continue;
        const uint8_t* dMP = KF->desc + 32 * (size_t)i;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = idx[c];
            if (owner[i2] >= 0) continue;
            const int dist = oo_descriptor_distance(dMP, F->desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= ORBdist) {
            owner[bestIdx2] = i;
            nmatches++;
            if (checkOri) {
                float rot = KF->kps[i].angle - F->kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == OO_HISTO) bin = 0;
                assert(bin >= 0 && bin < OO_HISTO);
                hist[bin * (KF->n + 1) + hlen[bin]++] = bestIdx2;
            }
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        oo_three_maxima(hlen, OO_HISTO, &ind1, &ind2, &ind3);
        for (int b = 0; b < OO_HISTO; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int j = 0; j < hlen[b]; j++) {
                owner[hist[b * (KF->n + 1) + j]] = -1;
                nmatches--;
            }
        }
    }
    free(hist);
    free(idx);
    return nmatches;
}

/* Frame::ComputeStereoFromRGBD (src/Frame.cc:643-664) on a float depth map (imDepth after
 * Tracking::GrabImageRGBD's convertTo(CV_32F, mDepthMapFactor), src/Tracking.cc:227-228).  step in floats. */
void oo_stereo_from_rgbd(const oo_keypoint* kps, const oo_keypoint* kps_un, int n, const float* depth, int step,
                         float mbf, float* uright, float* depth_out)
{
    for (int i = 0; i < n; i++) {
        uright[i] = -1;
        depth_out[i] = -1;
        const int v = (int)kps[i].y, u = (int)kps[i].x;  /* imDepth.at<float>(v,u): float -> int */
        const float d = depth[(size_t)v * step + u];
        if (d > 0) {
            depth_out[i] = d;
            uright[i] = kps_un[i].x - mbf / d;
        }
    }
}

/* imDepth.convertTo(imDepth, CV_32F, mDepthMapFactor) for a CV_16U depth image (shift 0: one product) */
void oo_depth_u16_to_f32(const uint16_t* src, int n, float factor, float* dst)
{
    for (int i = 0; i < n; i++) dst[i] = (float)src[i] * factor;
}

/* cv::cvtColor(img, gray, CV_{BGR,RGB,BGRA,RGBA}2GRAY) on 8U, as Tracking::GrabImage{Stereo,RGBD,Monocular}
 * apply it before the Frame is built (src/Tracking.cc:169-198, 209-225, 240-255).  OpenCV 3.x RGB2Gray<uchar>
 * (third-party, not vendored; restated): yuv_shift = 14, B2Y = 1868, G2Y = 9617, R2Y = 4899,
 * Y = (B*B2Y + G*G2Y + R*R2Y + (1 << 13)) >> 14.  bidx = index of the blue channel (0 for BGR/BGRA, 2 for
 * RGB/RGBA), cn = 3 or 4 (alpha ignored). */
void oo_cvt_gray(const uint8_t* src, int cols, int rows, int step, int cn, int bidx, uint8_t* dst, int dstep)
{
    const int cb = bidx == 0 ? 1868 : 4899, cr = bidx == 0 ? 4899 : 1868;
    for (int y = 0; y < rows; y++) {
        const uint8_t* s = src + (size_t)y * step;
        for (int x = 0; x < cols; x++, s += cn)
            dst[(size_t)y * dstep + x] = (uint8_t)((s[0] * cb + s[1] * 9617 + s[2] * cr + (1 << 13)) >> 14);
    }
}
