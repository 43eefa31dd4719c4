// orbgpu_capi.cpp -- host runtime of the gfx950 ORB path: plan construction (the reference's scalar
// setup math, reproduced exactly), device buffer management, the per-batch launch sequence and the
// extern "C" boundary declared in include/orbgpu.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/orbgpu.h"
#include "orbgpu_internal.h"
#include "orbgpu_launch.h"

static_assert(sizeof(orbgpu_keypoint) == 28, "cv::KeyPoint layout");
static_assert(sizeof(orbgpu_kp_dev) == 28, "cv::KeyPoint layout");

namespace {

inline int cv_round(float v) { return (int)std::lrintf(v); }
inline int cv_round_d(double v) { return (int)std::lrint(v); }

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;  // elements
};

struct StageTimer {
    bool on = false;
    std::vector<hipEvent_t> ev;
    std::vector<const char*> names;
    int used = 0;
    std::vector<float> last_ms;
    std::vector<const char*> last_names;
};

}  // namespace

struct orbgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    // small batches: level 0 on `stream`, pyramid + levels >= 1 on stream2 (run_batch), forked and joined by events
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    uint32_t rec_hdr[3] = {0, 0, 0};  // frame-record header staged for orbgpu_frame_record_pack's async copy
    // ORBextractor parameters and scale tables (src/ORBextractor.cc:410-470)
    int nfeatures = 0, nlevels = 0, iniTh = 0, minTh = 0;
    int sem = ORBGPU_SEM_DEFAULT;  // OpenCV/compiler semantics (orbgpu_set_semantics)
    double scaleFactor = 0;  // `double scaleFactor` member, include/ORBextractor.h:98
    std::vector<float> sf, isf, sig2, isig2;
    std::vector<int> nfeat;
    int umax[16] = {0};
    // plan for the current geometry
    int W = 0, H = 0;
    bool planned = false;
    int dbg_proj = 0;  // orbgpu_debug_set_projection_paths (tests only)
    OgPlan plan{};
    std::vector<OgCell> cells_h;
    std::vector<int4> xtab_h, ytab_h;
    DevBuf<OgFastBlk> cells;  // the FAST kernel's block table
    DevBuf<int4> tabs;
    // batch buffers
    int Bcap = 0;
    DevBuf<uint8_t> pyr;
    DevBuf<unsigned long long> cand;
    DevBuf<int> cand_count;
    DevBuf<uint16_t> node_of;
    DevBuf<unsigned> oct_best;
    DevBuf<uint32_t> oct_xy;
    DevBuf<uint32_t> oct_resp;  // response keys (FAST score, or the Harris key under ORBGPU_SEM_SCORE_HARRIS)
    DevBuf<int> oct_count;
    DevBuf<orbgpu_kp_dev> kps;
    DevBuf<uint8_t> desc;
    DevBuf<int> counts;
    DevBuf<int> cell_start, cell_items;
    DevBuf<int> status;
    // last batch
    const uint8_t* last_img = nullptr;
    long long last_pitch = 0, last_fstride = 0;
    int last_B = 0;
    OgGridGeom grid_geom{};
    // single-frame host path
    DevBuf<uint8_t> in_img;
    DevBuf<uint8_t> in_color;  // colour frame staged by orbgpu_extract_color
    uint8_t* hpin = nullptr;   // pinned download block of the single-frame path (og_launch_pack_host)
    void* hpin_dev = nullptr;  // ... its device-side address
    size_t hpin_size = 0;
    // matcher scratch
    DevBuf<uint8_t> mscratch;
    DevBuf<uint32_t> mlists;  // SearchForInitialization candidate lists {dist:16|i2:16}
    DevBuf<int> mlist_n;
    DevBuf<uint8_t> mcands;   // projection-matcher candidate lists (grown on demand, kept)
    DevBuf<int> pj_int;       // projection matcher: kept counts, decisions
    DevBuf<float> sf_dev;     // mvScaleFactors on the device
    // Frame::UndistortKeyPoints on the device (set by orbgpu_set_undistortion): batches then also hold
    // mvKeysUn, and the grid and the matchers use it with the undistorted image bounds
    bool undist = false;
    OgUndistort und{};
    DevBuf<orbgpu_kp_dev> kps_un;
    DevBuf<float> und_pts;
    // ComputeBoW scratch: per-descriptor word / weight / node
    DevBuf<int> bow_word, bow_nid;
    DevBuf<double> bow_wt;
    // stereo scratch (Frame::ComputeStereoMatches)
    DevBuf<int> st_row_start, st_row_items, st_sad, st_nm;
    DevBuf<float> st_out;
    StageTimer timer;
    std::string err;
};

static thread_local std::string g_create_err;

#define HIP_TRY(ctx, expr)                                                                          \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            if (ctx) (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);                \
            return ORBGPU_ERR_HIP;                                                                  \
        }                                                                                           \
    } while (0)

template <class T>
static hipError_t ensure(DevBuf<T>& b, size_t n)
{
    if (b.n >= n && b.p) return hipSuccess;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    hipError_t e = hipMalloc((void**)&b.p, std::max<size_t>(n, 1) * sizeof(T));
    if (e == hipSuccess) b.n = n;
    return e;
}

template <class T>
static void release(DevBuf<T>& b)
{
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
}

// Frame::ComputeImageBounds (src/Frame.cc:436-461) + mfGridElementWidthInv/HeightInv (:103-104): the
// undistorted corners (on the device, same kernel as the keypoints) or the plain image rectangle
static int image_bounds(orbgpu_ctx* c, bool undist, const OgUndistort& U, int cols, int rows, OgGridGeom* G)
{
    if (!undist) {
        orbgpu_grid_geom g;
        orbgpu_grid_geom_for_image(cols, rows, &g);
        *G = OgGridGeom{g.minX, g.minY, g.maxX, g.maxY, g.invW, g.invH};
        return ORBGPU_OK;
    }
    const float corners[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
    float u[8];
    HIP_TRY(c, ensure(c->und_pts, 16));
    HIP_TRY(c, hipMemcpyAsync(c->und_pts.p, corners, sizeof(corners), hipMemcpyHostToDevice, c->stream));
    og_launch_undistort_points(c->stream, c->und_pts.p, c->und_pts.p + 8, 4, U);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(u, c->und_pts.p + 8, sizeof(u), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    G->minX = std::min(u[0], u[4]);
    G->maxX = std::max(u[2], u[6]);
    G->minY = std::min(u[1], u[3]);
    G->maxY = std::max(u[5], u[7]);
    G->invW = (float)OG_GRID_COLS / (G->maxX - G->minX);
    G->invH = (float)OG_GRID_ROWS / (G->maxY - G->minY);
    return ORBGPU_OK;
}

// ------------------------------------------------------------------------------------------------
// plan: geometry of one image size (all quantities the reference derives per call)
// ------------------------------------------------------------------------------------------------
static int build_plan(orbgpu_ctx* c, int W, int H)
{
    if (c->planned && c->W == W && c->H == H) return ORBGPU_OK;
    if (W >= 32768 || H >= 32768) {  // candidate keys and the octree's remap records pack coordinates in 15 bits
        c->err = "image larger than 32767 pixels in a dimension";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    OgPlan P{};
    P.nlevels = c->nlevels;
    P.sem = c->sem;
    P.iniTh = c->iniTh;
    P.minTh = c->minTh;
    std::memcpy(P.umax, c->umax, sizeof(P.umax));
    std::vector<OgCell> cells;
    std::vector<int4> tabs;
    long long pyr_off = 0, cand_off = 0;
    int koff = 0;
    int pw = W, ph = H;
    for (int l = 0; l < c->nlevels; l++) {
        OgLevel& L = P.lv[l];
        // ComputePyramid level size (src/ORBextractor.cc:1111-1112)
        L.w = cv_round((float)W * c->isf[l]);
        L.h = cv_round((float)H * c->isf[l]);
        L.pitch = (L.w + 63) & ~63;
        if (l >= 1) {
            L.pyr_off = pyr_off;
            pyr_off += ((long long)L.pitch * L.h + 255) & ~255LL;
        }
        // FAST cell grid (src/ORBextractor.cc:773-787)
        L.minB = OG_EDGE - 3;
        L.maxBX = L.w - OG_EDGE + 3;
        L.maxBY = L.h - OG_EDGE + 3;
        const float width = (float)(L.maxBX - L.minB), height = (float)(L.maxBY - L.minB);
        const float Wc = 30;
        L.nCols = (int)(width / Wc);
        L.nRows = (int)(height / Wc);
        if (L.nCols < 1 || L.nRows < 1 || L.w < 2 * OG_EDGE + 8 || L.h < 2 * OG_EDGE + 8) {
            c->err = "pyramid level " + std::to_string(l) + " (" + std::to_string(L.w) + "x" + std::to_string(L.h) +
                     ") is smaller than one FAST cell: the reference divides by zero here";
            return ORBGPU_ERR_UNSUPPORTED;
        }
        L.wCell = (int)std::ceil(width / L.nCols);
        L.hCell = (int)std::ceil(height / L.nRows);
        if (L.wCell > OG_MAX_CELL_W || L.hCell > OG_MAX_CELL_W) {
            c->err = "cell larger than the LDS tile";
            return ORBGPU_ERR_UNSUPPORTED;
        }
        L.cell_base = (int)cells.size();
        long long cap = 0;
        for (int i = 0; i < L.nRows; i++) {
            const float iniY = (float)(L.minB + i * L.hCell);
            float maxY = iniY + L.hCell + 6;
            if (iniY >= L.maxBY - 3) continue;
            if (maxY > L.maxBY) maxY = (float)L.maxBY;
            for (int j = 0; j < L.nCols; j++) {
                const float iniX = (float)(L.minB + j * L.wCell);
                float maxX = iniX + L.wCell + 6;
                if (iniX >= L.maxBX - 6) continue;
                if (maxX > L.maxBX) maxX = (float)L.maxBX;
                OgCell cd;
                cd.level = (short)l;
                cd.i = (short)i;
                cd.j = (short)j;
                cd.pad = 0;
                cd.x0 = (short)(int)iniX;
                cd.y0 = (short)(int)iniY;
                cd.x1 = (short)(int)maxX;
                cd.y1 = (short)(int)maxY;
                const int dw = cd.x1 - cd.x0 - 6, dh = cd.y1 - cd.y0 - 6;
                if (dw <= 0 || dh <= 0) continue;
                cells.push_back(cd);
                cap += (long long)((dw + 1) / 2) * ((dh + 1) / 2);  // NMS keeps an independent set
            }
        }
        // FAST blocks of up to 2x2 valid cells (og_fast_quad_kernel); the valid cells form a rectangle
        // (the skip tests depend on the row or the column only)
        {
            std::vector<OgCell> lc(cells.begin() + L.cell_base, cells.end());
            cells.resize(L.cell_base);
            int nr = 0, ncl = 0;
            for (const OgCell& cc : lc) {
                nr = std::max(nr, (int)cc.i + 1);
                ncl = std::max(ncl, (int)cc.j + 1);
            }
            if ((int)lc.size() != nr * ncl) {
                c->err = "FAST cells do not form a rectangle";
                return ORBGPU_ERR_INTERNAL;
            }
            // the kernel's quad layout holds detection widths <= 4 * 16 and heights <= 80 (FQ_S, FB_MW)
            const int bsj = (2 * L.wCell <= 64) ? 2 : 1, bsi = (L.hCell <= 40) ? 2 : 1;
            for (int bi = 0; bi < nr; bi += bsi)
                for (int bj = 0; bj < ncl; bj += bsj) {
                    const int ni = std::min(bsi, nr - bi), nj = std::min(bsj, ncl - bj);
                    const OgCell& a = lc[bi * ncl + bj];
                    const OgCell& right = lc[bi * ncl + bj + nj - 1];
                    const OgCell& below = lc[(bi + ni - 1) * ncl + bj];
                    OgCell blk = a;
                    blk.pad = (short)((ni << 8) | nj);
                    blk.x1 = right.x1;
                    blk.y1 = below.y1;
                    if (blk.x1 - blk.x0 - 6 > 64 || blk.y1 - blk.y0 - 6 > 80) {
                        c->err = "FAST block larger than the kernel's LDS tile";
                        return ORBGPU_ERR_INTERNAL;
                    }
                    cells.push_back(blk);
                }
        }
        L.ncells = (int)cells.size() - L.cell_base;
        L.cand_off = cand_off;
        L.cand_cap = (int)std::max<long long>(cap, 1);
        cand_off += (L.cand_cap + 31) & ~31;
        // octree (src/ORBextractor.cc:543-545)
        L.N = c->nfeat[l];
        L.nIni = (int)std::round((float)(L.maxBX - L.minB) / (L.maxBY - L.minB));
        if (L.nIni < 1) {
            c->err = "image aspect ratio gives zero initial octree nodes (the reference divides by zero)";
            return ORBGPU_ERR_UNSUPPORTED;
        }
        L.hX = (float)(L.maxBX - L.minB) / L.nIni;
        L.kcap = std::max(L.N + 3, 4 * L.nIni);
        if (L.kcap > OG_OCT_MAXL_BIG - 8) {
            c->err = "features per level exceed the LDS octree capacity (" + std::to_string(OG_OCT_MAXL_BIG - 8) +
                     " list nodes)";
            return ORBGPU_ERR_UNSUPPORTED;
        }
        if (L.kcap > OG_OCT_MAXL - 8) {
            if (P.oct_big != l) {  // levels shrink with l: the big-list levels are a prefix
                c->err = "octree: a large level after a small one";
                return ORBGPU_ERR_INTERNAL;
            }
            P.oct_big = l + 1;
        }
        L.koff = koff;
        koff += L.kcap;
        L.scale = c->sf[l];
        L.patch_size = (int)(OG_PATCH * c->sf[l]);
        // resize tables: cv::resize INTER_LINEAR fixed point (generic path, scalar vertical form)
        if (l >= 1) {
            const int sw = pw, sh = ph, dw = L.w, dh = L.h;
            const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
            const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
            L.xtab_off = (int)tabs.size();
            L.xmax = dw;
            for (int dx = 0; dx < dw; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = (int)std::floor(fx);
                fx -= (float)sx;
                if (sx < 0) {
                    fx = 0.f;
                    sx = 0;
                }
                if (sx + 1 >= sw) {
                    if (dx < L.xmax) L.xmax = dx;
                    if (sx >= sw - 1) {
                        fx = 0.f;
                        sx = sw - 1;
                    }
                }
                tabs.push_back(make_int4(sx, (short)cv_round((1.f - fx) * 2048), (short)cv_round(fx * 2048), 0));
            }
            L.ytab_off = (int)tabs.size();
            for (int dy = 0; dy < dh; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = (int)std::floor(fy);
                fy -= (float)sy;
                auto clip = [sh](int y) { return y >= 0 ? (y < sh ? y : sh - 1) : 0; };
                tabs.push_back(make_int4(clip(sy), clip(sy + 1), (short)cv_round((1.f - fy) * 2048),
                                         (short)cv_round(fy * 2048)));
            }
        }
        pw = L.w;
        ph = L.h;
    }
    // fused resize launches (levels l, l+1 for odd l): the largest S / A regions over the tiles of l+1, replaying
    // og_resize2_kernel's region arithmetic on the host tables
    for (int l = 1; l + 1 < P.nlevels; l += 2) {
        OgLevel& A = P.lv[l];
        const OgLevel& Bv = P.lv[l + 1];
        const OgLevel& S = P.lv[l - 1];
        const int4* xA = tabs.data() + A.xtab_off;
        const int4* yA = tabs.data() + A.ytab_off;
        const int4* xB = tabs.data() + Bv.xtab_off;
        const int4* yB = tabs.data() + Bv.ytab_off;
        int SR = 0, SC = 0, AR = 0, AC = 0;
        std::vector<int4> tt;  // per tile of B: the region bounds og_resize2_kernel reads (3 int4, row-major tiles)
        for (int by0 = 0; by0 < Bv.h; by0 += RZ2_TH)
            for (int bx0 = 0; bx0 < Bv.w; bx0 += 256) {
                const int nyB = std::min(RZ2_TH, Bv.h - by0), nxB = std::min(256, Bv.w - bx0);
                const int ar0 = yB[by0].x;
                const int own_r1 = by0 + nyB == Bv.h ? A.h : yB[by0 + nyB].x;
                const int ar1 = std::max(yB[by0 + nyB - 1].y, own_r1 - 1);
                // the region starts at a 4-column boundary, so the owned A quads are dword-aligned stores; the up
                // to 3 extra columns are owned by the tile to the left, which stores the same values
                const int ac0 = xB[bx0].x & ~3;
                const int own_c1 = bx0 + nxB == Bv.w ? A.w : xB[bx0 + nxB].x;
                const int ac1 = std::max(std::min(xB[bx0 + nxB - 1].x + 1, A.w - 1), own_c1 - 1);
                const int sr0 = yA[ar0].x, sr1 = yA[ar1].y;
                const int sc0 = xA[ac0].x, sc1 = std::min(xA[ac1].x + 1, S.w - 1);
                SR = std::max(SR, sr1 - sr0 + 1);
                SC = std::max(SC, ((sc1 - sc0 + 1 + 15 + 15) >> 4) * 16 + 16);
                AR = std::max(AR, ar1 - ar0 + 1);
                AC = std::max(AC, ((ac1 - ac0 + 1 + 3) & ~3) + 16);
                tt.push_back(make_int4(ar0, ar1, own_r1, ac0));
                tt.push_back(make_int4(ac1, own_c1, sr0, sr1));
                tt.push_back(make_int4(sc0, sc1, 0, 0));
            }
        A.fz_tile_off = (int)tabs.size();  // xA.. are not used past this point: the append may reallocate
        tabs.insert(tabs.end(), tt.begin(), tt.end());
        A.fz_SR = SR;
        A.fz_SC = SC;
        A.fz_AR = AR;
        A.fz_AC = AC;
        // SR <= 127 and SC <= 2048: og_resize2_kernel's row index (7 bits) and exact float chunk quotient
        if (og_rz2_lds_bytes(SR, SC, AR, AC) > 64 * 1024 || SR > 127 || SC > 2048) {
            c->err = "fused resize region exceeds the LDS budget";
            return ORBGPU_ERR_UNSUPPORTED;
        }
    }
    if (koff > OG_GRID_LDS_ITEMS) {
        c->err = "more than " + std::to_string(OG_GRID_LDS_ITEMS) + " keypoints per frame (grid capacity)";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    P.total_cells = (int)cells.size();
    // the FAST kernel's block table (OgFastBlk): level-major, each level's blocks in plan order (row-major), no
    // padding.  The kernel's grid is (64 frames, blocks, frame chunks), so a frame's blocks all run on XCD f % 8
    // whatever the table holds; the table order only sets the order of a frame's blocks in time.  Runs of 4 or 8
    // row-adjacent blocks (round 3's XCD runs under frame-major dispatch) were 0.4 % slower under the chunked
    // dispatch (profiles/sweeps/r06_ab_fast_table_padding_order.txt) and are gone.
    std::vector<OgFastBlk> fblk;
    {
        std::vector<int> order;  // table entry -> cell index
        for (int l = 0; l < P.nlevels; l++) {
            OgLevel& L = P.lv[l];
            L.fb_off = (int)order.size();
            for (int b = 0; b < L.ncells; b++) order.push_back(L.cell_base + b);
        }
        const int n = (int)order.size();
        fblk.resize(n);
        for (int p = 0; p < n; p++) {
            OgFastBlk& r = fblk[p];
            std::memset(&r, 0, sizeof(r));
            const OgCell& cd = cells[order[p]];
            const OgLevel& L = P.lv[cd.level];
            const int rw = cd.x1 - cd.x0, rh = cd.y1 - cd.y0;
            if (rw - 6 > 64 || rh - 6 > 80 || rw < 7 || rh < 7 || L.wCell > 255 || L.hCell > 255) {
                c->err = "FAST block outside the kernel's LDS tile";
                return ORBGPU_ERR_INTERNAL;
            }
            r.lev = cd.level;
            r.y0 = cd.y0;
            r.pitch = cd.level == 0 ? 0 : L.pitch;
            r.src_off = cd.level == 0 ? cd.x0 : (int)(L.pyr_off + (long long)cd.y0 * L.pitch + cd.x0);
            r.rw = (unsigned char)rw;
            r.rh = (unsigned char)rh;
            r.wC = (unsigned char)L.wCell;
            r.hC = (unsigned char)L.hCell;
            r.cand_off = (int)L.cand_off;
            r.cand_cap = L.cand_cap;
            r.ox = (short)(cd.x0 - L.minB + 3);
            r.oy = (short)(cd.y0 - L.minB + 3);
            for (int k = 0; k < 4; k++) r.colw |= (unsigned)std::min(std::max(rw - 6 - 16 * k, 0), 16) << (8 * k);
        }
        P.fast_blocks = n;
        if (cand_off >= (1LL << 31) || std::max<long long>(pyr_off, 256) >= (1LL << 31)) {
            c->err = "per-frame candidate or pyramid block of 2^31 or more";
            return ORBGPU_ERR_UNSUPPORTED;
        }
    }
    P.kcap_total = koff;
    P.frame_cap = koff;
    P.cand_per_frame = cand_off;
    P.pyr_per_frame = std::max<long long>(pyr_off, 256);
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, ensure(c->cells, fblk.size()));
    HIP_TRY(c, ensure(c->tabs, tabs.size()));
    HIP_TRY(c, hipMemcpyAsync(c->cells.p, fblk.data(), fblk.size() * sizeof(OgFastBlk), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->tabs.p, tabs.data(), tabs.size() * sizeof(int4), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->plan = P;
    c->cells_h.swap(cells);
    c->W = W;
    c->H = H;
    c->planned = true;
    c->Bcap = 0;  // batch buffers must be re-sized for the new plan
    return image_bounds(c, c->undist, c->und, W, H, &c->grid_geom);
}

// the device status word collects capacity-guard flags (atomicOr) from every launch until a status check reads
// and clears it (check_status): zeroed once at allocation, never by a launch sequence, so a flag raised by one
// chunk survives the next chunk's extraction
static int ensure_status(orbgpu_ctx* c)
{
    if (c->status.p) return ORBGPU_OK;
    HIP_TRY(c, ensure(c->status, 4));
    HIP_TRY(c, hipMemsetAsync(c->status.p, 0, sizeof(int) * 4, c->stream));
    return ORBGPU_OK;
}

// Frame::AssignFeaturesToGrid of host-supplied frames (single-frame matcher entry points): the grid kernel sorts a
// frame's items in LDS, OG_GRID_LDS_ITEMS of them at most
static int launch_host_grid(orbgpu_ctx* c, hipStream_t s, const orbgpu_kp_dev* k, const int* cnt, int cap, int n,
                            const OgGridGeom& G, int* cs, int* ci)
{
    if (n > OG_GRID_LDS_ITEMS) {
        c->err = "more than " + std::to_string(OG_GRID_LDS_ITEMS) + " keypoints in one frame (grid capacity)";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    if (int r = ensure_status(c)) return r;
    og_launch_grid(s, k, cnt, cap, G, cs, ci, c->status.p, 1);
    return ORBGPU_OK;
}

static int ensure_batch(orbgpu_ctx* c, int B)
{
    if (c->Bcap >= B) return ORBGPU_OK;
    const OgPlan& P = c->plan;
    const size_t Bn = (size_t)B;
    // the describe kernel indexes keypoint slots of a batch with 32-bit offsets (frame x frame_cap + slot)
    if ((long long)B * (long long)P.frame_cap >= (1LL << 31)) {
        c->err = "batch x keypoint capacity of 2^31 or more";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, ensure(c->pyr, Bn * (size_t)P.pyr_per_frame));
    HIP_TRY(c, ensure(c->cand, Bn * (size_t)P.cand_per_frame));
    HIP_TRY(c, ensure(c->cand_count, Bn * (size_t)P.nlevels));
    HIP_TRY(c, ensure(c->node_of, Bn * (size_t)P.cand_per_frame));
    HIP_TRY(c, ensure(c->oct_best, Bn * (size_t)P.nlevels * OG_OCT_BEST_CELLS));
    HIP_TRY(c, ensure(c->oct_xy, Bn * (size_t)P.kcap_total));
    HIP_TRY(c, ensure(c->oct_resp, Bn * (size_t)P.kcap_total));
    HIP_TRY(c, ensure(c->oct_count, Bn * (size_t)P.nlevels));
    HIP_TRY(c, ensure(c->kps, Bn * (size_t)P.frame_cap));
    HIP_TRY(c, ensure(c->kps_un, Bn * (size_t)P.frame_cap));
    HIP_TRY(c, ensure(c->desc, Bn * (size_t)P.frame_cap * 32));
    HIP_TRY(c, ensure(c->counts, Bn));
    HIP_TRY(c, ensure(c->cell_start, Bn * (OG_GRID_CELLS + 1)));
    HIP_TRY(c, ensure(c->cell_items, Bn * (size_t)P.frame_cap));
    if (int r = ensure_status(c)) return r;
    c->Bcap = B;
    return ORBGPU_OK;
}

// ---- stage timing ---------------------------------------------------------------------------------
static void timer_begin(orbgpu_ctx* c)
{
    c->timer.used = 0;
    c->timer.names.clear();
}
// ORBGPU_DEBUG_SYNC=1 (diagnostics only): synchronise after every stage and report the first stage whose
// kernels failed, so a device fault names its kernel instead of surfacing at the next unrelated sync
// (ORBGPU_DEBUG_SYNC=2 also prints every stage as it completes: a hang names the stage that never does)
static int debug_sync_level()
{
    static const int lv = [] {
        const char* e = std::getenv("ORBGPU_DEBUG_SYNC");
        return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
    }();
    return lv;
}
static bool debug_sync() { return debug_sync_level() != 0; }

static void timer_mark(orbgpu_ctx* c, const char* name)
{
    if (debug_sync()) {
        if (debug_sync_level() == 2) {
            std::fprintf(stderr, "orbgpu: stage '%s' enqueued, synchronising\n", name);
            std::fflush(stderr);
        }
        const hipError_t e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            std::fprintf(stderr, "orbgpu: stage '%s' failed: %s\n", name, hipGetErrorString(e));
            std::fflush(stderr);
        } else if (debug_sync_level() == 2) {
            std::fprintf(stderr, "orbgpu: stage '%s' done\n", name);
            std::fflush(stderr);
        }
    }
    StageTimer& t = c->timer;
    if (!t.on) return;
    if ((int)t.ev.size() <= t.used) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        t.ev.push_back(e);
    }
    (void)hipEventRecord(t.ev[t.used++], c->stream);
    t.names.push_back(name);
}

// the keypoints the Frame-level code reads (mvKeysUn): undistorted when the context has a distortion model
static const orbgpu_kp_dev* kps_match(const orbgpu_ctx* c) { return c->undist ? c->kps_un.p : c->kps.p; }

// k1: chained pyramid, src/ORBextractor.cc:1107-1132
// levels (1,2), (3,4), (5,6) in one launch each (og_resize2_kernel), a last odd level alone
static void launch_pyramid(orbgpu_ctx* c, hipStream_t s, const uint8_t* d_imgs, int B, long long pitch, long long fstride)
{
    const OgPlan& P = c->plan;
    for (int l = 1; l < P.nlevels;) {
        const OgLevel& L = P.lv[l];
        const OgLevel& Lp = P.lv[l - 1];
        const uint8_t* src = l == 1 ? d_imgs : c->pyr.p + Lp.pyr_off;
        const long long sp = l == 1 ? pitch : Lp.pitch;
        const long long sfs = l == 1 ? fstride : P.pyr_per_frame;
        if (l + 1 < P.nlevels) {
            const OgLevel& Ln = P.lv[l + 1];
            OgRz2Geom g{Lp.w, Lp.h, L.w, L.h, Ln.w, Ln.h, c->tabs.p + L.xtab_off, c->tabs.p + L.ytab_off, L.xmax,
                        c->tabs.p + Ln.xtab_off, c->tabs.p + Ln.ytab_off, Ln.xmax, L.fz_SR, L.fz_SC, L.fz_AR, L.fz_AC,
                        c->tabs.p + L.fz_tile_off};
            og_launch_resize2(s, src, sp, sfs, c->pyr.p + L.pyr_off, L.pitch, c->pyr.p + Ln.pyr_off, Ln.pitch,
                              P.pyr_per_frame, g, c->status.p, B, P.sem);
            l += 2;
        } else {
            og_launch_resize(s, src, sp, sfs, c->pyr.p + L.pyr_off, L.pitch, P.pyr_per_frame, Lp.w, Lp.h, L.w, L.h,
                             c->tabs.p + L.xtab_off, c->tabs.p + L.ytab_off, L.xmax, c->status.p, B, P.sem);
            l += 1;
        }
    }
}

// FAST (+ the Harris option) and the octree of levels [lb, le) on stream s; the FAST block table is level-major,
// so the levels' blocks are one contiguous range
static void launch_levels(orbgpu_ctx* c, hipStream_t s, int lb, int le, const uint8_t* d_imgs, int B, long long pitch,
                          long long fstride, bool marks)
{
    const OgPlan& P = c->plan;
    og_launch_fast(s, P, lb, le, c->cells.p, d_imgs, pitch, fstride, c->pyr.p, c->cand.p, c->cand_count.p,
                   c->status.p, B);
    if (marks) timer_mark(c, "fast");
    if (P.sem & ORBGPU_SEM_SCORE_HARRIS) {  // option: rank by the Harris response (include/orbgpu.h)
        og_launch_harris(s, P, lb, le, d_imgs, pitch, fstride, c->pyr.p, c->cand.p, c->cand_count.p, B);
        if (marks) timer_mark(c, "harris");
    }
    og_launch_octree(s, P, lb, le, c->cand.p, c->cand_count.p, c->node_of.p, c->oct_best.p, c->oct_xy.p, c->oct_resp.p,
                     c->oct_count.p, c->status.p, B);
}

// batches of up to this many frames run level 0's FAST + octree (the single-frame critical path, ~60 % of a
// 1080p frame's device time) on the context stream while a second stream builds the pyramid and runs levels >= 1.
// The fork and join cost more than they hide below ~1 MP (tools/latency.py: 1242x375 0.177 -> 0.211 ms forked,
// 1920x1080 0.294 -> 0.238 ms), so only frames of at least ORBGPU_FORK_MIN_PIXELS (default 2^20) fork.
#define OG_FORK_MAX_B 4
// ORBGPU_FORK_MAX_B (measurement): fork batches up to this size instead (level 0's octree beside levels 1-7's FAST)
static int fork_max_b()
{
    static const int v = [] {
        const char* e = std::getenv("ORBGPU_FORK_MAX_B");
        return e && *e ? std::atoi(e) : OG_FORK_MAX_B;
    }();
    return v;
}
static long long fork_min_pixels()
{
    static const long long v = [] {
        const char* e = std::getenv("ORBGPU_FORK_MIN_PIXELS");
        return e && *e ? std::atoll(e) : (1LL << 20);
    }();
    return v;
}

static int run_batch(orbgpu_ctx* c, const uint8_t* d_imgs, int B, long long pitch, long long fstride)
{
    const OgPlan& P = c->plan;
    hipStream_t s = c->stream;
    timer_begin(c);
    timer_mark(c, "start");
    og_launch_zero(s, c->cand_count.p, B * P.nlevels);
    // stage timing and the debug sync keep the serial order (their marks are stage boundaries on one stream)
    const bool fork = B <= fork_max_b() && P.nlevels > 1 && !c->timer.on && !debug_sync() && c->stream2 &&
                      (long long)c->W * c->H >= fork_min_pixels();
    if (fork) {
        HIP_TRY(c, hipEventRecord(c->ev_fork, s));
        HIP_TRY(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
        launch_levels(c, s, 0, 1, d_imgs, B, pitch, fstride, false);
        launch_pyramid(c, c->stream2, d_imgs, B, pitch, fstride);
        launch_levels(c, c->stream2, 1, P.nlevels, d_imgs, B, pitch, fstride, false);
        HIP_TRY(c, hipEventRecord(c->ev_join, c->stream2));
        HIP_TRY(c, hipStreamWaitEvent(s, c->ev_join, 0));
    } else {
        launch_pyramid(c, s, d_imgs, B, pitch, fstride);
        timer_mark(c, "pyramid");
        launch_levels(c, s, 0, P.nlevels, d_imgs, B, pitch, fstride, true);
    }
    timer_mark(c, "octree");
    og_launch_describe(s, P, d_imgs, pitch, fstride, c->pyr.p, c->oct_xy.p, c->oct_resp.p, c->oct_count.p, c->kps.p,
                       c->desc.p, c->counts.p, B);
    timer_mark(c, "describe");
    if (c->undist) og_launch_undistort(s, c->kps.p, c->kps_un.p, c->counts.p, 0, P.frame_cap, c->und, B);
    og_launch_grid(s, kps_match(c), c->counts.p, P.frame_cap, c->grid_geom, c->cell_start.p, c->cell_items.p,
                   c->status.p, B, c->status.p + 1);
    timer_mark(c, "grid");
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(c->done, s));
    c->last_img = d_imgs;
    c->last_pitch = pitch;
    c->last_fstride = fstride;
    c->last_B = B;
    return ORBGPU_OK;
}

static int collect_timer(orbgpu_ctx* c)
{
    StageTimer& t = c->timer;
    if (!t.on || t.used < 2) return 0;
    if (hipEventSynchronize(t.ev[t.used - 1]) != hipSuccess) return 0;
    t.last_ms.clear();
    t.last_names.clear();
    for (int i = 1; i < t.used; i++) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, t.ev[i - 1], t.ev[i]);
        t.last_ms.push_back(ms);
        t.last_names.push_back(t.names[i]);
    }
    return (int)t.last_ms.size();
}

static int check_status(orbgpu_ctx* c)
{
    if (!c->status.p) return ORBGPU_OK;  // nothing launched yet
    int st[4] = {0};
    HIP_TRY(c, hipMemcpyAsync(st, c->status.p, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (st[0]) {  // read and clear: the flags of every launch since the last check (word 0 only: word 1 is frame 0's
                  // refused-record state, owned by unpack / extraction, og_record_check_kernel)
        HIP_TRY(c, hipMemsetAsync(c->status.p, 0, sizeof(int), c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if (st[0] == 128) {  // og_record_unpack_kernel: a refused frame record (a caller error, not a device guard)
            c->err = "frame record does not match this context's plan (frame_cap / undistortion) or has a bad count";
            return ORBGPU_ERR_ARG;
        }
        if ((st[0] & ~128) == 256) {  // og_init_resolve_kernel: F1 is another context's frame 0 and that is a refused record
            c->err = "the reference frame (frame 0 of the reference context) holds a refused frame record";
            return ORBGPU_ERR_ARG;
        }
        c->err = "device capacity guard tripped (status " + std::to_string(st[0]) + ")";
        return ORBGPU_ERR_INTERNAL;
    }
    return ORBGPU_OK;
}

// ------------------------------------------------------------------------------------------------
// extern "C"
// ------------------------------------------------------------------------------------------------
extern "C" {

orbgpu_ctx* orbgpu_create(int device, int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
{
    // scaleFactor <= 1.6 keeps one 8x1024 resize tile's source inside the LDS staging buffer
    if (nlevels < 1 || nlevels > OG_MAXLEVELS || nfeatures < 0 || !(scaleFactor > 1.0f) || scaleFactor > 1.6f)
        return nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    orbgpu_ctx* c = new orbgpu_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess || og_upload_pattern(device) != hipSuccess ||
        og_prepare_device() != hipSuccess) {
        delete c;
        return nullptr;
    }
    c->nfeatures = nfeatures;
    c->nlevels = nlevels;
    c->iniTh = iniThFAST;
    c->minTh = minThFAST;
    c->scaleFactor = (double)scaleFactor;
    // src/ORBextractor.cc:415-446
    c->sf.assign(nlevels, 0.f);
    c->sig2.assign(nlevels, 0.f);
    c->isf.assign(nlevels, 0.f);
    c->isig2.assign(nlevels, 0.f);
    c->nfeat.assign(nlevels, 0);
    c->sf[0] = 1.0f;
    c->sig2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        c->sf[i] = (float)((double)c->sf[i - 1] * c->scaleFactor);
        c->sig2[i] = c->sf[i] * c->sf[i];
    }
    for (int i = 0; i < nlevels; i++) {
        c->isf[i] = 1.0f / c->sf[i];
        c->isig2[i] = 1.0f / c->sig2[i];
    }
    const float factor = (float)(1.0f / c->scaleFactor);
    float nd = (float)nfeatures * (1.0f - factor) / (1.0f - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        c->nfeat[l] = cv_round(nd);
        sum += c->nfeat[l];
        nd *= factor;
    }
    c->nfeat[nlevels - 1] = std::max(nfeatures - sum, 0);
    // umax, src/ORBextractor.cc:454-469
    int v, v0;
    const int vmax = (int)std::floor(OG_HALF_PATCH * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(OG_HALF_PATCH * std::sqrt(2.f) / 2);
    const double hp2 = OG_HALF_PATCH * OG_HALF_PATCH;
    for (v = 0; v <= vmax; ++v) c->umax[v] = cv_round_d(std::sqrt(hp2 - v * v));
    for (v = OG_HALF_PATCH, v0 = 0; v >= vmin; --v) {
        while (c->umax[v0] == c->umax[v0 + 1]) ++v0;
        c->umax[v] = v0;
        ++v0;
    }
    static const int kUmax[16] = {OG_UMAX};
    if (std::memcmp(c->umax, kUmax, sizeof(kUmax)) != 0) {  // cannot happen: umax depends on constants only
        orbgpu_destroy(c);
        return nullptr;
    }
    return c;
}

int orbgpu_set_semantics(orbgpu_ctx* c, int flags)
{
    if (!c) return ORBGPU_ERR_ARG;
    if ((flags & ~ORBGPU_SEM_ALL) || (flags & ORBGPU_SEM_BLUR_MASK) > ORBGPU_SEM_BLUR_BITEXACT_ED) {
        c->err = "unknown semantics flags";
        return ORBGPU_ERR_ARG;
    }
    c->sem = flags;
    c->plan.sem = flags;  // the plan is passed by value to each launch: takes effect at the next extraction
    return ORBGPU_OK;
}

int orbgpu_get_semantics(const orbgpu_ctx* c) { return c ? c->sem : ORBGPU_ERR_ARG; }

void orbgpu_destroy(orbgpu_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    release(c->cells);
    release(c->tabs);
    release(c->pyr);
    release(c->cand);
    release(c->cand_count);
    release(c->node_of);
    release(c->oct_best);
    release(c->oct_xy);
    release(c->oct_resp);
    release(c->oct_count);
    release(c->kps);
    release(c->desc);
    release(c->counts);
    release(c->cell_start);
    release(c->cell_items);
    release(c->status);
    release(c->in_img);
    release(c->in_color);
    if (c->hpin) (void)hipHostFree(c->hpin);
    c->hpin = nullptr;
    release(c->mscratch);
    release(c->mlists);
    release(c->mlist_n);
    release(c->mcands);
    release(c->pj_int);
    release(c->sf_dev);
    release(c->kps_un);
    release(c->bow_word);
    release(c->bow_nid);
    release(c->bow_wt);
    release(c->und_pts);
    release(c->st_row_start);
    release(c->st_row_items);
    release(c->st_sad);
    release(c->st_nm);
    release(c->st_out);
    for (hipEvent_t e : c->timer.ev) (void)hipEventDestroy(e);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int orbgpu_get_levels(const orbgpu_ctx* c) { return c ? c->nlevels : ORBGPU_ERR_ARG; }
float orbgpu_get_scale_factor(const orbgpu_ctx* c) { return c ? (float)c->scaleFactor : 0.f; }

static int copy_vec(const orbgpu_ctx* c, const std::vector<float>& v, float* out)
{
    if (!c || !out) return ORBGPU_ERR_ARG;
    std::memcpy(out, v.data(), v.size() * sizeof(float));
    return ORBGPU_OK;
}
int orbgpu_get_scale_factors(const orbgpu_ctx* c, float* out) { return c ? copy_vec(c, c->sf, out) : ORBGPU_ERR_ARG; }
int orbgpu_get_inverse_scale_factors(const orbgpu_ctx* c, float* out) { return c ? copy_vec(c, c->isf, out) : ORBGPU_ERR_ARG; }
int orbgpu_get_scale_sigma_squares(const orbgpu_ctx* c, float* out) { return c ? copy_vec(c, c->sig2, out) : ORBGPU_ERR_ARG; }
int orbgpu_get_inverse_scale_sigma_squares(const orbgpu_ctx* c, float* out)
{
    return c ? copy_vec(c, c->isig2, out) : ORBGPU_ERR_ARG;
}
int orbgpu_get_features_per_level(const orbgpu_ctx* c, int* out)
{
    if (!c || !out) return ORBGPU_ERR_ARG;
    std::memcpy(out, c->nfeat.data(), c->nfeat.size() * sizeof(int));
    return ORBGPU_OK;
}

int orbgpu_max_keypoints(const orbgpu_ctx* c)
{
    if (!c) return ORBGPU_ERR_ARG;
    if (c->planned) return c->plan.frame_cap;
    int s = 0;  // before the first frame: kcap = max(N+3, 4*nIni) with nIni <= 16 assumed
    for (int l = 0; l < c->nlevels; l++) s += std::max(c->nfeat[l] + 3, 64);
    return s;
}

int orbgpu_extract_batch_device(orbgpu_ctx* c, const uint8_t* d_imgs, int B, int cols, int rows, size_t pitch,
                                size_t frame_stride)
{
    if (!c || !d_imgs || B < 1 || cols <= 0 || rows <= 0 || pitch < (size_t)cols) return ORBGPU_ERR_ARG;
    if (pitch >= OG_MAX_PITCH) {  // the kernels' per-lane row offsets are 24-bit products
        c->err = "row pitch of 16 MiB or more";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    int r = build_plan(c, cols, rows);
    if (r) return r;
    r = ensure_batch(c, B);
    if (r) return r;
    return run_batch(c, d_imgs, B, (long long)pitch, (long long)frame_stride);
}

int orbgpu_batch_outputs(orbgpu_ctx* c, orbgpu_keypoint** d_kps, uint8_t** d_desc, int** d_counts, int* frame_cap)
{
    if (!c || !c->planned || !c->last_B) return ORBGPU_ERR_ARG;
    if (d_kps) *d_kps = (orbgpu_keypoint*)c->kps.p;
    if (d_desc) *d_desc = c->desc.p;
    if (d_counts) *d_counts = c->counts.p;
    if (frame_cap) *frame_cap = c->plan.frame_cap;
    return ORBGPU_OK;
}

// ---- one frame as a flat device record (the unit a multi-GPU run broadcasts: SURVEY §8(e), config 3's initial
// frame).  Layout: int32 count, 12 pad bytes, frame_cap keypoints (28 B), frame_cap descriptors (32 B), and with an
// undistortion model frame_cap mvKeysUn keypoints.
static size_t ref_record_bytes(const orbgpu_ctx* c)
{
    return 16 + (size_t)c->plan.frame_cap * (28 + 32 + (c->undist ? 28 : 0));
}

int orbgpu_debug_math_hash(int device, int fn, unsigned long long begin, unsigned long long end, int chunk_log2,
                           unsigned long long* out, int nchunks)
{
    if (fn < 0 || fn > 1 || begin >= end || end > (1ull << 32) || chunk_log2 < 12 || chunk_log2 > 32 || !out)
        return ORBGPU_ERR_ARG;
    if ((long long)(((end - 1) >> chunk_log2) - (begin >> chunk_log2) + 1) != nchunks) return ORBGPU_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return ORBGPU_ERR_HIP;
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d, (size_t)nchunks * 8) != hipSuccess) return ORBGPU_ERR_HIP;
    hipError_t e = hipMemset(d, 0, (size_t)nchunks * 8);
    if (e == hipSuccess) e = og_math_hash(fn, begin, end, chunk_log2, d, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d, (size_t)nchunks * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? ORBGPU_OK : ORBGPU_ERR_HIP;
}

int orbgpu_batch_grid(orbgpu_ctx* c, int** d_cell_start, int** d_cell_items)
{
    if (!c || !c->planned || !c->last_B) return ORBGPU_ERR_ARG;
    if (d_cell_start) *d_cell_start = c->cell_start.p;
    if (d_cell_items) *d_cell_items = c->cell_items.p;
    return ORBGPU_OK;
}

long long orbgpu_frame_record_bytes(const orbgpu_ctx* c)
{
    if (!c || !c->planned) return ORBGPU_ERR_ARG;
    return (long long)ref_record_bytes(c);
}

int orbgpu_frame_record_pack(orbgpu_ctx* c, int b, void* d_dst)
{
    if (!c || !c->planned || !d_dst || b < 0 || b >= c->last_B) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t cap = (size_t)c->plan.frame_cap, o = (size_t)b * cap;
    uint8_t* d = (uint8_t*)d_dst;
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemcpyAsync(d, c->counts.p + b, 4, hipMemcpyDeviceToDevice, s));
    // header words 1-3: magic, frame_cap, undistortion flag -- unpack checks them against the receiving context
    c->rec_hdr[0] = 0x5246474fu;  // "OGFR"
    c->rec_hdr[1] = (uint32_t)c->plan.frame_cap;
    c->rec_hdr[2] = c->undist ? 1u : 0u;
    HIP_TRY(c, hipMemcpyAsync(d + 4, c->rec_hdr, 12, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d + 16, c->kps.p + o, cap * 28, hipMemcpyDeviceToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(d + 16 + cap * 28, c->desc.p + o * 32, cap * 32, hipMemcpyDeviceToDevice, s));
    if (c->undist)
        HIP_TRY(c, hipMemcpyAsync(d + 16 + cap * 60, c->kps_un.p + o, cap * 28, hipMemcpyDeviceToDevice, s));
    return ORBGPU_OK;
}

int orbgpu_frame_record_unpack(orbgpu_ctx* c, const void* d_src)
{
    // frame 0 of a batch of one; the context must be planned for the record's geometry (same frame_cap)
    if (!c || !c->planned || !d_src) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    if (int r = ensure_batch(c, 1)) return r;
    // the header must describe this context's plan (frame_cap, undistortion) and a count within it; a record from
    // a differently planned context would otherwise be misread, and a larger count would send the matchers past
    // the frame.  Checked on the device, so the call stays stream-ordered (no host synchronisation): a mismatch
    // leaves count 0 and is reported as ORBGPU_ERR_ARG by the next status check.  So does a record whose keypoints
    // are not in extraction order (levels nondecreasing): the batched SearchForInitialization relies on it.
    hipStream_t s = c->stream;
    og_launch_record_unpack(s, d_src, c->plan.frame_cap, c->undist ? 1 : 0, c->plan.lv[0].kcap, c->counts.p, c->kps.p, c->desc.p,
                            c->undist ? c->kps_un.p : nullptr, c->status.p);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipEventRecord(c->done, s));  // matchers on other contexts wait for this record
    c->last_B = std::max(c->last_B, 1);
    return ORBGPU_OK;
}

int orbgpu_batch_download(orbgpu_ctx* c, int b, orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n)
{
    if (!c || !n || b < 0 || b >= c->last_B) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    int r = check_status(c);
    collect_timer(c);
    if (r) return r;
    int cnt = 0;
    HIP_TRY(c, hipMemcpy(&cnt, c->counts.p + b, sizeof(int), hipMemcpyDeviceToHost));
    *n = cnt;
    if (cnt > cap) return ORBGPU_ERR_CAPACITY;
    const size_t o = (size_t)b * c->plan.frame_cap;
    if (cnt > 0) {
        if (kps) HIP_TRY(c, hipMemcpy(kps, c->kps.p + o, (size_t)cnt * sizeof(orbgpu_kp_dev), hipMemcpyDeviceToHost));
        if (desc) HIP_TRY(c, hipMemcpy(desc, c->desc.p + o * 32, (size_t)cnt * 32, hipMemcpyDeviceToHost));
    }
    return ORBGPU_OK;
}

// the single-frame download (orbgpu_extract*): one packing kernel into the pinned block, one wait
static int download_single(orbgpu_ctx* c, orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n)
{
    const size_t fc = (size_t)c->plan.frame_cap;
    const size_t need = 16 + fc * 60;
    if (c->hpin_size < need) {
        if (c->hpin) HIP_TRY(c, hipHostFree(c->hpin));
        c->hpin = nullptr;
        c->hpin_size = 0;
        HIP_TRY(c, hipHostMalloc((void**)&c->hpin, need, hipHostMallocDefault));
        HIP_TRY(c, hipHostGetDevicePointer(&c->hpin_dev, c->hpin, 0));
        c->hpin_size = need;
    }
    og_launch_pack_host(c->stream, c->status.p, c->counts.p, c->kps.p, c->desc.p, (int)fc, c->hpin_dev);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    collect_timer(c);
    int hdr[2];
    std::memcpy(hdr, c->hpin, sizeof(hdr));
    if (hdr[0]) {  // capacity guard: read and clear word 0, as check_status
        HIP_TRY(c, hipMemsetAsync(c->status.p, 0, sizeof(int), c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->err = "device capacity guard tripped (status " + std::to_string(hdr[0]) + ")";
        return ORBGPU_ERR_INTERNAL;
    }
    if (hdr[1] < 0 || hdr[1] > (int)fc) {  // og_pack_host_kernel copies at most frame_cap entries
        c->err = "keypoint count " + std::to_string(hdr[1]) + " outside [0, frame_cap]";
        return ORBGPU_ERR_INTERNAL;
    }
    *n = hdr[1];
    if (hdr[1] > cap) return ORBGPU_ERR_CAPACITY;
    if (hdr[1] > 0) {
        if (kps) std::memcpy(kps, c->hpin + 16, (size_t)hdr[1] * sizeof(orbgpu_kp_dev));
        if (desc) std::memcpy(desc, c->hpin + 16 + fc * sizeof(orbgpu_kp_dev), (size_t)hdr[1] * 32);
    }
    return ORBGPU_OK;
}

int orbgpu_extract(orbgpu_ctx* c, const uint8_t* img, int cols, int rows, size_t step, orbgpu_keypoint* kps,
                   uint8_t* desc, int cap, int* n)
{
    if (!c || !n) return ORBGPU_ERR_ARG;
    if (!img || cols <= 0 || rows <= 0) {  // _image.empty(): return without touching the outputs
        *n = -1;
        return ORBGPU_OK;
    }
    if (step < (size_t)cols) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    // a contiguous image (cv::Mat::isContinuous, the usual case) keeps its own pitch: one linear copy instead of
    // a row-by-row 2-D copy (the kernels take any pitch)
    const size_t pitch = step == (size_t)cols ? step : (((size_t)cols + 63) & ~(size_t)63);
    HIP_TRY(c, ensure(c->in_img, pitch * (size_t)rows));
    if (pitch == step)
        HIP_TRY(c, hipMemcpyAsync(c->in_img.p, img, step * (size_t)rows, hipMemcpyHostToDevice, c->stream));
    else
        HIP_TRY(c, hipMemcpy2DAsync(c->in_img.p, pitch, img, step, (size_t)cols, (size_t)rows, hipMemcpyHostToDevice,
                                    c->stream));
    int r = orbgpu_extract_batch_device(c, c->in_img.p, 1, cols, rows, pitch, pitch * (size_t)rows);
    if (r) return r;
    return download_single(c, kps, desc, cap, n);
}

static int og_color_code(int code, int* cn, int* bidx)
{
    switch (code) {
    case ORBGPU_COLOR_BGR2GRAY: *cn = 3; *bidx = 0; return 1;
    case ORBGPU_COLOR_RGB2GRAY: *cn = 3; *bidx = 2; return 1;
    case ORBGPU_COLOR_BGRA2GRAY: *cn = 4; *bidx = 0; return 1;
    case ORBGPU_COLOR_RGBA2GRAY: *cn = 4; *bidx = 2; return 1;
    default: return 0;
    }
}

int orbgpu_cvt_color_to_gray_batch(orbgpu_ctx* c, const uint8_t* d_src, int B, int cols, int rows, size_t src_pitch,
                                   size_t src_frame_stride, int code, uint8_t* d_dst, size_t dst_pitch,
                                   size_t dst_frame_stride)
{
    int cn = 0, bidx = 0;
    if (!c || !d_src || !d_dst || B < 1 || cols <= 0 || rows <= 0 || !og_color_code(code, &cn, &bidx))
        return ORBGPU_ERR_ARG;
    if (src_pitch < (size_t)cols * cn || dst_pitch < (size_t)cols ||
        (B > 1 && (src_frame_stride < src_pitch * rows || dst_frame_stride < dst_pitch * rows)))
        return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    og_launch_gray(c->stream, d_src, cols, rows, cn, bidx, (long long)src_pitch, (long long)src_frame_stride, d_dst,
                   (long long)dst_pitch, (long long)dst_frame_stride, B);
    HIP_TRY(c, hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_extract_color(orbgpu_ctx* c, const uint8_t* img, int cols, int rows, size_t step, int code,
                         orbgpu_keypoint* kps, uint8_t* desc, int cap, int* n)
{
    int cn = 0, bidx = 0;
    if (!c || !n || !og_color_code(code, &cn, &bidx)) return ORBGPU_ERR_ARG;
    if (!img || cols <= 0 || rows <= 0) {  // _image.empty(): return without touching the outputs
        *n = -1;
        return ORBGPU_OK;
    }
    if (step < (size_t)cols * cn) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t cpitch = ((size_t)cols * cn + 63) & ~(size_t)63;
    const size_t pitch = ((size_t)cols + 63) & ~(size_t)63;
    HIP_TRY(c, ensure(c->in_color, cpitch * (size_t)rows));
    HIP_TRY(c, ensure(c->in_img, pitch * (size_t)rows));
    HIP_TRY(c, hipMemcpy2DAsync(c->in_color.p, cpitch, img, step, (size_t)cols * cn, (size_t)rows,
                                hipMemcpyHostToDevice, c->stream));
    int r = orbgpu_cvt_color_to_gray_batch(c, c->in_color.p, 1, cols, rows, cpitch, cpitch * (size_t)rows, code,
                                           c->in_img.p, pitch, pitch * (size_t)rows);
    if (r) return r;
    r = orbgpu_extract_batch_device(c, c->in_img.p, 1, cols, rows, pitch, pitch * (size_t)rows);
    if (r) return r;
    return download_single(c, kps, desc, cap, n);
}

int orbgpu_get_level(orbgpu_ctx* c, int level, uint8_t* dst, size_t dst_step, int* cols, int* rows)
{
    if (!c || level < 0 || level >= c->nlevels || !c->planned || !c->last_B) return ORBGPU_ERR_ARG;
    const OgLevel& L = c->plan.lv[level];
    if (cols) *cols = L.w;
    if (rows) *rows = L.h;
    if (!dst) return ORBGPU_OK;
    if (dst_step < (size_t)L.w) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const uint8_t* src = level == 0 ? c->last_img : c->pyr.p + L.pyr_off;
    const size_t sp = level == 0 ? (size_t)c->last_pitch : (size_t)L.pitch;
    HIP_TRY(c, hipMemcpy2DAsync(dst, dst_step, src, sp, (size_t)L.w, (size_t)L.h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return ORBGPU_OK;
}

int orbgpu_grid_geom_for_image(int cols, int rows, orbgpu_grid_geom* g)
{
    if (!g || cols <= 0 || rows <= 0) return ORBGPU_ERR_ARG;
    g->minX = 0.0f;
    g->maxX = (float)cols;
    g->minY = 0.0f;
    g->maxY = (float)rows;
    g->invW = (float)OG_GRID_COLS / (g->maxX - g->minX);
    g->invH = (float)OG_GRID_ROWS / (g->maxY - g->minY);
    return ORBGPU_OK;
}

int orbgpu_descriptor_distance(const uint8_t* a, const uint8_t* b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        dist += __builtin_popcount(x ^ y);
    }
    return dist;
}

// ---- matchers -----------------------------------------------------------------------------------
// every scratch_carve rounds its region up to 256 B: kCarvePad covers the rounding of up to 64 carves
static constexpr size_t kCarvePad = 64 * 256;

static uint8_t* scratch_carve(uint8_t*& cur, size_t bytes)
{
    uint8_t* p = cur;
    cur += (bytes + 255) & ~(size_t)255;
    return p;
}

int orbgpu_search_for_initialization(orbgpu_ctx* c, const orbgpu_frame_view* F1, const orbgpu_frame_view* F2,
                                     float nnratio, int checkOri, float* prev_xy, int* matches12, int windowSize,
                                     int* nmatches)
{
    if (!c || !F1 || !F2 || !prev_xy || !matches12 || !nmatches || F1->n < 0 || F2->n < 0) return ORBGPU_ERR_ARG;
    if ((F1->n && (!F1->kps || !F1->desc)) || (F2->n && (!F2->kps || !F2->desc))) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const int cap1 = std::max(F1->n, 1), cap2 = std::max(F2->n, 1);
    const size_t need = kCarvePad + (size_t)cap1 * (28 + 32 + 8 + 4) + (size_t)cap2 * (28 + 32 + 4) +
                        (OG_GRID_CELLS + 1) * 4 + 16;
    HIP_TRY(c, ensure(c->mscratch, need));
    uint8_t* cur = c->mscratch.p;
    orbgpu_kp_dev* k1 = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)cap1 * 28);
    uint8_t* d1 = scratch_carve(cur, (size_t)cap1 * 32);
    orbgpu_kp_dev* k2 = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)cap2 * 28);
    uint8_t* d2 = scratch_carve(cur, (size_t)cap2 * 32);
    int* cnts = (int*)scratch_carve(cur, 16);
    int* cs = (int*)scratch_carve(cur, (OG_GRID_CELLS + 1) * 4);
    int* ci = (int*)scratch_carve(cur, (size_t)cap2 * 4);
    float* pv = (float*)scratch_carve(cur, (size_t)cap1 * 8);
    int* m12 = (int*)scratch_carve(cur, (size_t)cap1 * 4);
    int* nm = (int*)scratch_carve(cur, 16);
    hipStream_t s = c->stream;
    int hc[2] = {F1->n, F2->n};
    if (F1->n) {
        HIP_TRY(c, hipMemcpyAsync(k1, F1->kps, (size_t)F1->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(d1, F1->desc, (size_t)F1->n * 32, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(pv, prev_xy, (size_t)F1->n * 8, hipMemcpyHostToDevice, s));
    }
    if (F2->n) {
        HIP_TRY(c, hipMemcpyAsync(k2, F2->kps, (size_t)F2->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(d2, F2->desc, (size_t)F2->n * 32, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(c, hipMemcpyAsync(cnts, hc, sizeof(hc), hipMemcpyHostToDevice, s));
    const OgGridGeom G{F2->grid.minX, F2->grid.minY, F2->grid.maxX, F2->grid.maxY, F2->grid.invW, F2->grid.invH};
    if (int r = launch_host_grid(c, s, k2, cnts + 1, cap2, F2->n, G, cs, ci)) return r;
    OgFrameDev f1{k1, d1, cnts, nullptr, nullptr, nullptr, cap1};
    OgFrameDev f2{k2, d2, cnts + 1, cs, ci, nullptr, cap2};
    int n2oct0 = 0;  // only octave-0 keypoints of F2 can be candidates (level1 == 0)
    for (int i = 0; i < F2->n; i++) n2oct0 += F2->kps[i].octave == 0;
    const int list_cap = std::max(n2oct0, 1);
    if (og_init_resolve_lds(cap1, cap2, list_cap) > OG_INIT_LDS_MAX) {
        c->err = "SearchForInitialization: frames too large for the LDS-resident ordered pass";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, ensure(c->mlists, (size_t)cap1 * list_cap));
    HIP_TRY(c, ensure(c->mlist_n, (size_t)cap1));
    if (int r = ensure_status(c)) return r;
    og_launch_search_init(s, f1, 0, f2, G, nnratio, checkOri, windowSize, pv, 2 * cap1, m12, cap1, nm, c->mlists.p,
                          list_cap, c->mlist_n.p, c->status.p, 1);
    HIP_TRY(c, hipGetLastError());
    int hnm = 0;
    HIP_TRY(c, hipMemcpyAsync(&hnm, nm, sizeof(int), hipMemcpyDeviceToHost, s));
    if (F1->n) {
        HIP_TRY(c, hipMemcpyAsync(matches12, m12, (size_t)F1->n * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(prev_xy, pv, (size_t)F1->n * 8, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(c, hipStreamSynchronize(s));
    int r = check_status(c);
    if (r) return r;
    *nmatches = hnm;
    return ORBGPU_OK;
}

int orbgpu_search_for_initialization_batch(orbgpu_ctx* cref, int ref, orbgpu_ctx* c, orbgpu_grid_geom grid,
                                           float nnratio, int checkOri, int windowSize, float* d_prev_xy,
                                           int* d_matches12, int* d_nmatches)
{
    if (!cref || !c || !cref->last_B || !c->last_B || ref < 0 || ref >= cref->last_B) return ORBGPU_ERR_ARG;
    if (!d_prev_xy || !d_matches12 || !d_nmatches) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (cref != c) HIP_TRY(c, hipStreamWaitEvent(s, cref->done, 0));
    const OgGridGeom G{grid.minX, grid.minY, grid.maxX, grid.maxY, grid.invW, grid.invH};
    if (std::memcmp(&G, &c->grid_geom, sizeof(G)) != 0) {
        c->grid_geom = G;
        og_launch_grid(s, kps_match(c), c->counts.p, c->plan.frame_cap, G, c->cell_start.p, c->cell_items.p, c->status.p,
                       c->last_B);
    }
    OgFrameDev f1{kps_match(cref), cref->desc.p, cref->counts.p, nullptr, nullptr, nullptr, cref->plan.frame_cap};
    OgFrameDev f2{kps_match(c), c->desc.p, c->counts.p, c->cell_start.p, c->cell_items.p, nullptr, c->plan.frame_cap};
    const int list_cap = c->plan.lv[0].kcap;  // F2 has at most kcap_0 octave-0 keypoints
    const size_t cap1 = (size_t)cref->plan.frame_cap;
    if (og_init_resolve_lds((int)cap1, c->plan.frame_cap, list_cap) > OG_INIT_LDS_MAX) {
        c->err = "SearchForInitialization: frames too large for the LDS-resident ordered pass";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, ensure(c->mlists, (size_t)c->last_B * cap1 * list_cap));
    HIP_TRY(c, ensure(c->mlist_n, (size_t)c->last_B * cap1));
    timer_mark(c, "match_init");
    og_launch_search_init(s, f1, ref, f2, G, nnratio, checkOri, windowSize, d_prev_xy, 2 * cref->plan.frame_cap,
                          d_matches12, cref->plan.frame_cap, d_nmatches, c->mlists.p, list_cap, c->mlist_n.p,
                          c->status.p, c->last_B, cref != c ? cref->status.p : nullptr, cref->plan.lv[0].kcap);
    timer_mark(c, "search_init");
    HIP_TRY(c, hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_prev_matched_from_frame(orbgpu_ctx* cref, int ref, orbgpu_ctx* c, float* d_prev_xy)
{
    if (!cref || !c || !cref->last_B || !c->last_B || ref < 0 || ref >= cref->last_B || !d_prev_xy) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    if (cref != c) HIP_TRY(c, hipStreamWaitEvent(c->stream, cref->done, 0));
    OgFrameDev f1{kps_match(cref), cref->desc.p, cref->counts.p, nullptr, nullptr, nullptr, cref->plan.frame_cap};
    og_launch_prev_from_frame(c->stream, f1, ref, d_prev_xy, 2 * cref->plan.frame_cap, c->last_B);
    HIP_TRY(c, hipGetLastError());
    return ORBGPU_OK;
}

// ---- Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:404-461) ------------------------------
static int parse_undistort(const float* K4, const float* dist, int ndist, OgUndistort* U, bool* active)
{
    if (!K4 || ndist < 0 || ndist > 5 || (ndist > 0 && !dist)) return ORBGPU_ERR_ARG;
    *U = OgUndistort{};
    for (int i = 0; i < 4; i++) U->K[i] = K4[i];
    for (int i = 0; i < ndist; i++) U->d[i] = dist[i];
    *active = ndist >= 1 && dist[0] != 0.0f;  // mDistCoef.at<float>(0)==0.0 -> mvKeysUn = mvKeys
    return ORBGPU_OK;
}

int orbgpu_set_undistortion(orbgpu_ctx* c, const float* K4, const float* dist, int ndist)
{
    if (!c) return ORBGPU_ERR_ARG;
    OgUndistort U;
    bool active = false;
    int r = parse_undistort(K4, dist, ndist, &U, &active);
    if (r) return r;
    HIP_TRY(c, hipSetDevice(c->device));
    c->undist = active;
    c->und = U;
    if (c->planned) return image_bounds(c, c->undist, c->und, c->W, c->H, &c->grid_geom);
    return ORBGPU_OK;
}

int orbgpu_undistort_keypoints(orbgpu_ctx* c, const float* K4, const float* dist, int ndist,
                               const orbgpu_keypoint* in, orbgpu_keypoint* out, int n)
{
    if (!c || n < 0 || (n && (!in || !out))) return ORBGPU_ERR_ARG;
    OgUndistort U;
    bool active = false;
    int r = parse_undistort(K4, dist, ndist, &U, &active);
    if (r) return r;
    if (n == 0) return ORBGPU_OK;
    if (!active) {
        if (out != in) std::memcpy(out, in, (size_t)n * sizeof(orbgpu_keypoint));
        return ORBGPU_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, ensure(c->mscratch, kCarvePad + (size_t)n * 56));
    uint8_t* cur = c->mscratch.p;
    orbgpu_kp_dev* din = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)n * 28);
    orbgpu_kp_dev* dout = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)n * 28);
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemcpyAsync(din, in, (size_t)n * 28, hipMemcpyHostToDevice, s));
    og_launch_undistort(s, din, dout, nullptr, n, n, U, 1);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipMemcpyAsync(out, dout, (size_t)n * 28, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    return ORBGPU_OK;
}

int orbgpu_compute_image_bounds(orbgpu_ctx* c, const float* K4, const float* dist, int ndist, int cols, int rows,
                                orbgpu_grid_geom* g)
{
    if (!c || !g || cols <= 0 || rows <= 0) return ORBGPU_ERR_ARG;
    OgUndistort U;
    bool active = false;
    int r = parse_undistort(K4, dist, ndist, &U, &active);
    if (r) return r;
    HIP_TRY(c, hipSetDevice(c->device));
    OgGridGeom G;
    r = image_bounds(c, active, U, cols, rows, &G);
    if (r) return r;
    *g = orbgpu_grid_geom{G.minX, G.minY, G.maxX, G.maxY, G.invW, G.invH};
    return ORBGPU_OK;
}

int orbgpu_batch_outputs_undistorted(orbgpu_ctx* c, orbgpu_keypoint** d_kps_un, orbgpu_grid_geom* bounds)
{
    if (!c || !c->planned || !c->last_B) return ORBGPU_ERR_ARG;
    if (d_kps_un) *d_kps_un = (orbgpu_keypoint*)kps_match(c);
    if (bounds) {
        const OgGridGeom& G = c->grid_geom;
        *bounds = orbgpu_grid_geom{G.minX, G.minY, G.maxX, G.maxY, G.invW, G.invH};
    }
    return ORBGPU_OK;
}

// ---- Frame::ComputeStereoFromRGBD (src/Frame.cc:643-664) ---------------------------------------------------
int orbgpu_compute_stereo_from_rgbd_batch(orbgpu_ctx* c, const void* d_depth, int is_u16, float factor,
                                          size_t pitch_bytes, size_t frame_stride_bytes, float mbf, float* d_uright,
                                          float* d_depth_out)
{
    if (!c || !c->last_B || !d_depth || !d_uright || !d_depth_out) return ORBGPU_ERR_ARG;
    const size_t px = is_u16 ? 2 : 4;
    if (pitch_bytes < (size_t)c->W * px || pitch_bytes % px) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    timer_mark(c, "rgbd_in");
    og_launch_rgbd(c->stream, c->kps.p, kps_match(c), c->counts.p, 0, c->plan.frame_cap, (const uint8_t*)d_depth,
                   is_u16 ? 1 : 0, factor, (long long)pitch_bytes, (long long)frame_stride_bytes, mbf, d_uright,
                   d_depth_out, c->last_B);
    timer_mark(c, "rgbd");
    HIP_TRY(c, hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_compute_stereo_from_rgbd(orbgpu_ctx* c, const void* depth, int is_u16, float factor, size_t step_bytes,
                                    float mbf, float* uright, float* depth_out, int cap, int* n)
{
    if (!c || !depth || !n) return ORBGPU_ERR_ARG;
    if (c->last_B != 1) {
        c->err = "ComputeStereoFromRGBD: host form needs one extracted frame";
        return ORBGPU_ERR_ARG;
    }
    const size_t px = is_u16 ? 2 : 4;
    if (step_bytes < (size_t)c->W * px) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t pitch = ((size_t)c->W * px + 255) & ~(size_t)255;
    const int fc = c->plan.frame_cap;
    HIP_TRY(c, ensure(c->mscratch, kCarvePad + pitch * (size_t)c->H + (size_t)fc * 8));
    uint8_t* cur = c->mscratch.p;
    uint8_t* dd = scratch_carve(cur, pitch * (size_t)c->H);
    float* ur = (float*)scratch_carve(cur, (size_t)fc * 4);
    float* de = (float*)scratch_carve(cur, (size_t)fc * 4);
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemcpy2DAsync(dd, pitch, depth, step_bytes, (size_t)c->W * px, (size_t)c->H, hipMemcpyHostToDevice, s));
    int r = orbgpu_compute_stereo_from_rgbd_batch(c, dd, is_u16, factor, pitch, pitch * (size_t)c->H, mbf, ur, de);
    if (r) return r;
    int cnt = 0;
    HIP_TRY(c, hipMemcpyAsync(&cnt, c->counts.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    *n = cnt;
    if (cnt > cap) return ORBGPU_ERR_CAPACITY;
    if (cnt > 0) {
        if (uright) HIP_TRY(c, hipMemcpy(uright, ur, (size_t)cnt * 4, hipMemcpyDeviceToHost));
        if (depth_out) HIP_TRY(c, hipMemcpy(depth_out, de, (size_t)cnt * 4, hipMemcpyDeviceToHost));
    }
    return ORBGPU_OK;
}

// ---- Frame::ComputeBoW: DBoW2 vocabulary + transform (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) ------
struct orbgpu_vocabulary {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, n = 0, nwords = 0;
    DevBuf<uint8_t> desc;
    DevBuf<int> child_start, child_cnt, children, word_id;
    DevBuf<double> weight;
};

static OgVocDev voc_dev(const orbgpu_vocabulary* v)
{
    return OgVocDev{v->n, v->L, v->scoring, v->weighting, v->desc.p, v->child_start.p, v->child_cnt.p,
                    v->children.p, v->word_id.p, v->weight.p};
}

static void voc_release(orbgpu_vocabulary* v)
{
    release(v->desc);
    release(v->child_start);
    release(v->child_cnt);
    release(v->children);
    release(v->word_id);
    release(v->weight);
}

// nn entries describe nodes 1..nn (node 0 = root) in file order: m_nodes[pid].children.push_back(nid) and
// leaves numbered as words in file order (TemplatedVocabulary::loadFromTextFile, :1368-1418)
static orbgpu_vocabulary* voc_build(orbgpu_ctx* c, int k, int L, int scoring, int weighting, int nn,
                                    const int* parent, const uint8_t* is_leaf, const uint8_t* desc,
                                    const double* weight)
{
    if (!c || nn < 0 || (nn && (!parent || !is_leaf || !desc || !weight))) return nullptr;
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3) {
        c->err = "vocabulary: header out of range (loadFromTextFile limits)";
        return nullptr;
    }
    const int n = nn + 1;
    std::vector<int> cs(n + 1, 0), cc(n, 0), ch(n, 0), wid(n, -1), fill(n, 0);
    std::vector<double> w(n, 0.0);
    std::vector<uint8_t> d(32 * (size_t)n, 0);
    int nwords = 0;
    for (int i = 0; i < nn; i++) {
        const int p = parent[i];
        if (p < 0 || p > i) {  // a parent must precede its child (file order)
            c->err = "vocabulary: node " + std::to_string(i + 1) + " has an invalid parent";
            return nullptr;
        }
        cc[p]++;
        std::memcpy(&d[32 * (size_t)(i + 1)], desc + 32 * (size_t)i, 32);
        w[i + 1] = weight[i];
        wid[i + 1] = is_leaf[i] ? nwords++ : -1;
    }
    for (int i = 0; i < n; i++) {
        if (cc[i] > 64) {
            c->err = "vocabulary: more than 64 children per node";
            return nullptr;
        }
        cs[i + 1] = cs[i] + cc[i];
    }
    for (int i = 0; i < nn; i++) ch[cs[parent[i]] + fill[parent[i]]++] = i + 1;
    orbgpu_vocabulary* v = new orbgpu_vocabulary();
    v->device = c->device;
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->n = n;
    v->nwords = nwords;
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = ensure(v->desc, d.size());
    if (e == hipSuccess) e = ensure(v->child_start, (size_t)n);
    if (e == hipSuccess) e = ensure(v->child_cnt, (size_t)n);
    if (e == hipSuccess) e = ensure(v->children, (size_t)n);
    if (e == hipSuccess) e = ensure(v->word_id, (size_t)n);
    if (e == hipSuccess) e = ensure(v->weight, (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(v->desc.p, d.data(), d.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->child_start.p, cs.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->child_cnt.p, cc.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->children.p, ch.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->word_id.p, wid.data(), sizeof(int) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(v->weight.p, w.data(), sizeof(double) * n, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        c->err = std::string("vocabulary upload: ") + hipGetErrorString(e);
        voc_release(v);
        delete v;
        return nullptr;
    }
    return v;
}

orbgpu_vocabulary* orbgpu_vocabulary_create(orbgpu_ctx* c, int k, int L, int scoring, int weighting, int nn,
                                            const int* parent, const uint8_t* is_leaf, const uint8_t* desc,
                                            const double* weight)
{
    return voc_build(c, k, L, scoring, weighting, nn, parent, is_leaf, desc, weight);
}

orbgpu_vocabulary* orbgpu_vocabulary_load_text(orbgpu_ctx* c, const char* path)
{
    if (!c || !path) return nullptr;
    std::ifstream f(path);
    if (!f) {
        c->err = std::string("vocabulary: cannot open ") + path;
        return nullptr;
    }
    std::string line;
    std::getline(f, line);
    std::stringstream hs(line);
    int k = -1, L = -1, sc = -1, wt = -1;
    hs >> k >> L >> sc >> wt;
    std::vector<int> par;
    std::vector<uint8_t> leaf, desc;
    std::vector<double> w;
    while (std::getline(f, line)) {
        std::stringstream ss(line);
        int pid, il;
        if (!(ss >> pid >> il)) continue;  // blank line (the reference would parse it as a node)
        uint8_t d[32];
        for (int i = 0; i < 32; i++) {
            int x = 0;
            ss >> x;
            d[i] = (uint8_t)x;
        }
        double ww = 0;
        ss >> ww;
        par.push_back(pid);
        leaf.push_back(il > 0);
        desc.insert(desc.end(), d, d + 32);
        w.push_back(ww);
    }
    return voc_build(c, k, L, sc, wt, (int)par.size(), par.data(), leaf.data(), desc.data(), w.data());
}

void orbgpu_vocabulary_destroy(orbgpu_vocabulary* v)
{
    if (!v) return;
    (void)hipSetDevice(v->device);
    voc_release(v);
    delete v;
}

int orbgpu_vocabulary_info(const orbgpu_vocabulary* v, int* k, int* L, int* nodes, int* words)
{
    if (!v) return ORBGPU_ERR_ARG;
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (nodes) *nodes = v->n;
    if (words) *words = v->nwords;
    return ORBGPU_OK;
}

int orbgpu_compute_bow_batch(orbgpu_ctx* c, const orbgpu_vocabulary* v, int levelsup, int32_t* d_words,
                             double* d_values, int32_t* d_nwords, int32_t* d_nodes, int32_t* d_node_off,
                             int32_t* d_feats, int32_t* d_nnodes)
{
    if (!c || !v || !c->last_B || !d_words || !d_values || !d_nwords || !d_nodes || !d_node_off || !d_feats ||
        !d_nnodes)
        return ORBGPU_ERR_ARG;
    if (v->device != c->device) return ORBGPU_ERR_ARG;
    const int fc = c->plan.frame_cap, B = c->last_B;
    if (fc > OG_BOW_MAXN) {
        c->err = "ComputeBoW: more keypoints per frame than the LDS sort holds";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, ensure(c->bow_word, (size_t)B * fc));
    HIP_TRY(c, ensure(c->bow_nid, (size_t)B * fc));
    HIP_TRY(c, ensure(c->bow_wt, (size_t)B * fc));
    timer_mark(c, "bow_in");
    og_launch_bow(c->stream, voc_dev(v), c->desc.p, c->counts.p, 0, fc, levelsup, c->bow_word.p, c->bow_wt.p,
                  c->bow_nid.p, d_words, d_values, d_nwords, d_nodes, d_node_off, d_feats, d_nnodes, B);
    timer_mark(c, "bow");
    HIP_TRY(c, hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_compute_bow(orbgpu_ctx* c, const orbgpu_vocabulary* v, const uint8_t* desc, int n, int levelsup,
                       int32_t* words, double* values, int* nwords, int32_t* nodes, int32_t* node_off,
                       int32_t* feats, int* nnodes)
{
    if (!c || !v || n < 0 || (n && !desc) || !words || !values || !nwords || !nodes || !node_off || !feats ||
        !nnodes)
        return ORBGPU_ERR_ARG;
    if (v->device != c->device) return ORBGPU_ERR_ARG;
    if (n > OG_BOW_MAXN) {
        c->err = "ComputeBoW: more descriptors than the LDS sort holds";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    *nwords = 0;
    *nnodes = 0;
    node_off[0] = 0;
    if (n == 0 || v->n <= 1) return ORBGPU_OK;  // empty(): v.clear(), fv.clear()
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t nn = (size_t)n;
    HIP_TRY(c, ensure(c->mscratch, kCarvePad + nn * (32 + 4 + 8 + 4 + 4 + 8 + 4 + 4 + 4) + 64));
    uint8_t* cur = c->mscratch.p;
    uint8_t* dd = scratch_carve(cur, nn * 32);
    int* wrd = (int*)scratch_carve(cur, nn * 4);
    double* wt = (double*)scratch_carve(cur, nn * 8);
    int* nid = (int*)scratch_carve(cur, nn * 4);
    int* ow = (int*)scratch_carve(cur, nn * 4);
    double* ov = (double*)scratch_carve(cur, nn * 8);
    int* ond = (int*)scratch_carve(cur, nn * 4);
    int* onoff = (int*)scratch_carve(cur, (nn + 1) * 4);
    int* oft = (int*)scratch_carve(cur, nn * 4);
    int* cnt = (int*)scratch_carve(cur, 16);
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemcpyAsync(dd, desc, nn * 32, hipMemcpyHostToDevice, s));
    og_launch_bow(s, voc_dev(v), dd, nullptr, n, n, levelsup, wrd, wt, nid, ow, ov, cnt, ond, onoff, oft, cnt + 1, 1);
    HIP_TRY(c, hipGetLastError());
    int hc[2] = {0, 0};
    HIP_TRY(c, hipMemcpyAsync(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    *nwords = hc[0];
    *nnodes = hc[1];
    HIP_TRY(c, hipMemcpy(words, ow, (size_t)hc[0] * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(values, ov, (size_t)hc[0] * 8, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(nodes, ond, (size_t)hc[1] * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(node_off, onoff, ((size_t)hc[1] + 1) * 4, hipMemcpyDeviceToHost));
    int m = 0;
    HIP_TRY(c, hipMemcpy(&m, onoff + hc[1], 4, hipMemcpyDeviceToHost));
    if (m > 0) HIP_TRY(c, hipMemcpy(feats, oft, (size_t)m * 4, hipMemcpyDeviceToHost));
    return ORBGPU_OK;
}

// ---- stereo: Frame::ComputeStereoMatches (src/Frame.cc:466-640) -------------------------------------
static int stereo_launch(orbgpu_ctx* L, orbgpu_ctx* R, float mbf, float mb, float* d_ur, float* d_depth, int* d_nm)
{
    if (!L || !R || !L->last_B || !R->last_B || L->last_B != R->last_B) return ORBGPU_ERR_ARG;
    if (L->W != R->W || L->H != R->H || L->nlevels != R->nlevels || L->sf != R->sf ||
        L->plan.pyr_per_frame != R->plan.pyr_per_frame) {
        L->err = "stereo: left and right extractors must share image size and scale pyramid";
        return ORBGPU_ERR_ARG;
    }
    if (!(mb > 0.0f)) {
        L->err = "stereo: baseline must be positive";
        return ORBGPU_ERR_ARG;
    }
    if (R->plan.frame_cap > 8192) {  // og_stereo_rows_kernel keeps the right keypoints' bands in LDS
        L->err = "stereo: more than 8192 right keypoints per frame";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    const int B = L->last_B;
    const OgPlan& P = L->plan;
    HIP_TRY(L, hipSetDevice(L->device));
    hipStream_t s = L->stream;
    if (R != L) HIP_TRY(L, hipStreamWaitEvent(s, R->done, 0));
    OgStereoDev S{};
    S.L = OgFrameDev{L->kps.p, L->desc.p, L->counts.p, nullptr, nullptr, nullptr, P.frame_cap};
    S.R = OgFrameDev{R->kps.p, R->desc.p, R->counts.p, nullptr, nullptr, nullptr, R->plan.frame_cap};
    S.L0 = L->last_img;
    S.R0 = R->last_img;
    S.L0_pitch = L->last_pitch;
    S.L0_fstride = L->last_fstride;
    S.R0_pitch = R->last_pitch;
    S.R0_fstride = R->last_fstride;
    S.Lpyr = L->pyr.p;
    S.Rpyr = R->pyr.p;
    S.pyr_fstride = P.pyr_per_frame;
    for (int l = 0; l < P.nlevels; l++) {
        S.lvl_off[l] = P.lv[l].pyr_off;
        S.lvl_pitch[l] = P.lv[l].pitch;
        S.lvl_w[l] = P.lv[l].w;
        S.sf[l] = L->sf[l];
        S.isf[l] = L->isf[l];
    }
    S.mbf = mbf;
    S.mb = mb;
    S.nRows = L->H;
    if (S.nRows > 8192) {
        L->err = "stereo: more than 8192 image rows";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    // every right keypoint spans at most 2*ceil(2*sf)+2 rows of vRowIndices
    const int span = 2 * (int)std::ceil(2.0f * L->sf[P.nlevels - 1]) + 2;
    S.row_cap = R->plan.frame_cap * span;
    HIP_TRY(L, ensure(L->st_row_start, (size_t)B * (S.nRows + 1)));
    HIP_TRY(L, ensure(L->st_row_items, (size_t)B * S.row_cap));
    HIP_TRY(L, ensure(L->st_sad, (size_t)B * P.frame_cap));
    S.row_start = L->st_row_start.p;
    S.row_items = L->st_row_items.p;
    S.sad = L->st_sad.p;
    S.uright = d_ur;
    S.depth = d_depth;
    S.nmatches = d_nm;
    timer_mark(L, "stereo_in");
    og_launch_stereo(s, S, B);
    timer_mark(L, "stereo");
    HIP_TRY(L, hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_compute_stereo_matches_batch(orbgpu_ctx* left, orbgpu_ctx* right, float mbf, float mb, float* d_uright,
                                        float* d_depth, int* d_nmatches)
{
    if (!d_uright || !d_depth || !d_nmatches) return ORBGPU_ERR_ARG;
    return stereo_launch(left, right, mbf, mb, d_uright, d_depth, d_nmatches);
}

int orbgpu_compute_stereo_matches(orbgpu_ctx* left, orbgpu_ctx* right, float mbf, float mb, float* uright,
                                  float* depth, int cap, int* n, int* nmatches)
{
    if (!left || !right || !n) return ORBGPU_ERR_ARG;
    if (left->last_B != 1 || right->last_B != 1) {
        left->err = "stereo: host form needs one extracted frame on each side";
        return ORBGPU_ERR_ARG;
    }
    HIP_TRY(left, hipSetDevice(left->device));
    const int fc = left->plan.frame_cap;
    HIP_TRY(left, ensure(left->st_out, 2 * (size_t)fc));
    HIP_TRY(left, ensure(left->st_nm, 4));
    int r = stereo_launch(left, right, mbf, mb, left->st_out.p, left->st_out.p + fc, left->st_nm.p);
    if (r) return r;
    int hc[2] = {0, 0};
    HIP_TRY(left, hipMemcpyAsync(&hc[0], left->counts.p, sizeof(int), hipMemcpyDeviceToHost, left->stream));
    HIP_TRY(left, hipMemcpyAsync(&hc[1], left->st_nm.p, sizeof(int), hipMemcpyDeviceToHost, left->stream));
    HIP_TRY(left, hipStreamSynchronize(left->stream));
    *n = hc[0];
    if (nmatches) *nmatches = hc[1];
    if (hc[0] > cap) return ORBGPU_ERR_CAPACITY;
    if (hc[0] > 0) {
        if (uright)
            HIP_TRY(left, hipMemcpy(uright, left->st_out.p, (size_t)hc[0] * 4, hipMemcpyDeviceToHost));
        if (depth)
            HIP_TRY(left, hipMemcpy(depth, left->st_out.p + fc, (size_t)hc[0] * 4, hipMemcpyDeviceToHost));
    }
    return ORBGPU_OK;
}

// The batched projection matcher: one enumeration pass into fixed per-point slots, then the fixed-point resolve
// (og_launch_projb, orb_match.hip); stream-ordered, no host synchronisation.
static int run_projection(orbgpu_ctx* c, hipStream_t s, const OgFrameDev& fd, const OgGridGeom& G, const float* sfd,
                          const OgMapPointsDev& mpd, int stride, int B, float nnratio, float th, int* own, int* obs,
                          int* nm)
{
    const size_t pts = (size_t)B * (size_t)std::max(stride, 1);
    HIP_TRY(c, ensure(c->pj_int, 2 * pts));
    HIP_TRY(c, ensure(c->mcands, pts * OG_PJ_K * sizeof(uint32_t)));
    int* kept = c->pj_int.p;
    int* res = kept + pts;
    og_launch_projb(s, fd, G, sfd, mpd, stride, nnratio, th, B, (uint32_t*)c->mcands.p, kept, res, own, obs, nm,
                    c->status.p, c->dbg_proj);
    HIP_TRY(c, hipGetLastError());
    return ORBGPU_OK;
}

int orbgpu_search_by_projection(orbgpu_ctx* c, const orbgpu_frame_view* F, const orbgpu_mappoints_view* mp,
                                float nnratio, float th, int32_t* owner, int32_t* owner_obs, int* nmatches)
{
    if (!c || !F || !mp || !nmatches || F->n < 0 || mp->m < 0) return ORBGPU_ERR_ARG;
    if (F->n && (!owner || !owner_obs)) return ORBGPU_ERR_ARG;
    if (!F->scale_factors || F->nlevels < 1) return ORBGPU_ERR_ARG;
    if ((size_t)2 * sizeof(int) * (size_t)std::max(F->n, 1) > OG_INIT_LDS_MAX) {
        c->err = "SearchByProjection: more keypoints than the LDS-resident claim table holds";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    const int n = std::max(F->n, 1), m = std::max(mp->m, 1);
    const size_t fixed = kCarvePad + (size_t)n * (28 + 32 + 4 + 4 + 4 + 4) + (OG_GRID_CELLS + 1) * 4 +
                         (size_t)m * (1 + 1 + 4 + 4 + 4 + 4 + 4 + 4 + 32) + 64 + F->nlevels * 4;
    HIP_TRY(c, ensure(c->mscratch, fixed));
    uint8_t* cur = c->mscratch.p;
    orbgpu_kp_dev* k = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)n * 28);
    uint8_t* d = scratch_carve(cur, (size_t)n * 32);
    float* ur = (float*)scratch_carve(cur, (size_t)n * 4);
    int* own = (int*)scratch_carve(cur, (size_t)n * 4);
    int* obs = (int*)scratch_carve(cur, (size_t)n * 4);
    int* cnts = (int*)scratch_carve(cur, 16);
    int* cs = (int*)scratch_carve(cur, (OG_GRID_CELLS + 1) * 4);
    int* ci = (int*)scratch_carve(cur, (size_t)n * 4);
    float* sfd = (float*)scratch_carve(cur, (size_t)F->nlevels * 4);
    uint8_t* tiv = scratch_carve(cur, (size_t)m);
    uint8_t* bad = scratch_carve(cur, (size_t)m);
    int* lvl = (int*)scratch_carve(cur, (size_t)m * 4);
    float* vc = (float*)scratch_carve(cur, (size_t)m * 4);
    float* px = (float*)scratch_carve(cur, (size_t)m * 4);
    float* py = (float*)scratch_carve(cur, (size_t)m * 4);
    float* pxr = (float*)scratch_carve(cur, (size_t)m * 4);
    int* nobs = (int*)scratch_carve(cur, (size_t)m * 4);
    uint8_t* md = scratch_carve(cur, (size_t)m * 32);
    int* nm = (int*)scratch_carve(cur, 16);
    hipStream_t s = c->stream;
    if (F->n) {
        HIP_TRY(c, hipMemcpyAsync(k, F->kps, (size_t)F->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(d, F->desc, (size_t)F->n * 32, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(own, owner, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(obs, owner_obs, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
        if (F->uright) HIP_TRY(c, hipMemcpyAsync(ur, F->uright, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(c, hipMemcpyAsync(sfd, F->scale_factors, (size_t)F->nlevels * 4, hipMemcpyHostToDevice, s));
    if (mp->m) {
        HIP_TRY(c, hipMemcpyAsync(tiv, mp->track_in_view, (size_t)mp->m, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(bad, mp->is_bad, (size_t)mp->m, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(lvl, mp->level, (size_t)mp->m * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(vc, mp->view_cos, (size_t)mp->m * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(px, mp->proj_x, (size_t)mp->m * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(py, mp->proj_y, (size_t)mp->m * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(pxr, mp->proj_xr, (size_t)mp->m * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(nobs, mp->n_obs, (size_t)mp->m * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(md, mp->desc, (size_t)mp->m * 32, hipMemcpyHostToDevice, s));
    }
    int hc = F->n;
    HIP_TRY(c, hipMemcpyAsync(cnts, &hc, sizeof(int), hipMemcpyHostToDevice, s));
    const OgGridGeom G{F->grid.minX, F->grid.minY, F->grid.maxX, F->grid.maxY, F->grid.invW, F->grid.invH};
    if (int r = launch_host_grid(c, s, k, cnts, n, F->n, G, cs, ci)) return r;
    OgFrameDev fd{k, d, cnts, cs, ci, F->uright ? ur : nullptr, n};
    OgMapPointsDev mpd{mp->m, tiv, bad, lvl, vc, px, py, pxr, nobs, md};
    int r = run_projection(c, s, fd, G, sfd, mpd, m, 1, nnratio, th, own, obs, nm);
    if (r) return r;
    int hnm = 0;
    HIP_TRY(c, hipMemcpyAsync(&hnm, nm, sizeof(int), hipMemcpyDeviceToHost, s));
    if (F->n) {
        HIP_TRY(c, hipMemcpyAsync(owner, own, (size_t)F->n * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(owner_obs, obs, (size_t)F->n * 4, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(c, hipStreamSynchronize(s));
    r = check_status(c);
    if (r) return r;
    *nmatches = hnm;
    return ORBGPU_OK;
}

int orbgpu_search_by_projection_batch(orbgpu_ctx* c, const orbgpu_mappoints_view* d_mp, int mp_stride, float nnratio,
                                      float th, const float* d_uright, int32_t* d_owner, int32_t* d_owner_obs,
                                      int* d_nmatches)
{
    if (!c || !c->last_B || !d_mp || d_mp->m < 0 || mp_stride < d_mp->m || !d_owner || !d_owner_obs || !d_nmatches)
        return ORBGPU_ERR_ARG;
    if (d_mp->m && (!d_mp->track_in_view || !d_mp->is_bad || !d_mp->level || !d_mp->view_cos || !d_mp->proj_x ||
                    !d_mp->proj_y || !d_mp->proj_xr || !d_mp->n_obs || !d_mp->desc))
        return ORBGPU_ERR_ARG;
    if ((size_t)2 * sizeof(int) * (size_t)c->plan.frame_cap > OG_INIT_LDS_MAX) {
        c->err = "SearchByProjection: frame capacity exceeds the LDS-resident claim table";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (c->sf_dev.n < (size_t)c->nlevels) {
        HIP_TRY(c, ensure(c->sf_dev, (size_t)c->nlevels));
        HIP_TRY(c, hipMemcpyAsync(c->sf_dev.p, c->sf.data(), sizeof(float) * c->nlevels, hipMemcpyHostToDevice, s));
    }
    timer_mark(c, "match_proj");
    OgFrameDev fd{kps_match(c), c->desc.p, c->counts.p, c->cell_start.p, c->cell_items.p, d_uright, c->plan.frame_cap};
    OgMapPointsDev mpd{d_mp->m,      d_mp->track_in_view, d_mp->is_bad, d_mp->level, d_mp->view_cos, d_mp->proj_x,
                       d_mp->proj_y, d_mp->proj_xr,       d_mp->n_obs,  d_mp->desc};
    int r = run_projection(c, s, fd, c->grid_geom, c->sf_dev.p, mpd, mp_stride, c->last_B, nnratio, th, d_owner,
                           d_owner_obs, d_nmatches);
    timer_mark(c, "search_proj");
    return r;
}

int orbgpu_search_by_projection_batch_shared_map(orbgpu_ctx* c, const orbgpu_mappoints_view* d_mp, int mp_stride,
                                                 float nnratio, float th, const float* d_uright, int32_t* d_owner,
                                                 int32_t* d_owner_obs, int* d_nmatches)
{
    if (!c || !c->last_B || !d_mp || d_mp->m < 0 || mp_stride < d_mp->m || !d_owner || !d_owner_obs || !d_nmatches)
        return ORBGPU_ERR_ARG;
    if (d_mp->m && (!d_mp->track_in_view || !d_mp->is_bad || !d_mp->level || !d_mp->view_cos || !d_mp->proj_x ||
                    !d_mp->proj_y || !d_mp->proj_xr || !d_mp->n_obs || !d_mp->desc))
        return ORBGPU_ERR_ARG;
    if ((size_t)2 * sizeof(int) * (size_t)c->plan.frame_cap > OG_INIT_LDS_MAX) {
        c->err = "SearchByProjection: frame capacity exceeds the LDS-resident claim table";
        return ORBGPU_ERR_UNSUPPORTED;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (c->sf_dev.n < (size_t)c->nlevels) {
        HIP_TRY(c, ensure(c->sf_dev, (size_t)c->nlevels));
        HIP_TRY(c, hipMemcpyAsync(c->sf_dev.p, c->sf.data(), sizeof(float) * c->nlevels, hipMemcpyHostToDevice, s));
    }
    timer_mark(c, "match_proj");
    OgFrameDev fd{kps_match(c), c->desc.p, c->counts.p, c->cell_start.p, c->cell_items.p, d_uright, c->plan.frame_cap};
    OgMapPointsDev mpd{d_mp->m,      d_mp->track_in_view, d_mp->is_bad, d_mp->level, d_mp->view_cos, d_mp->proj_x,
                       d_mp->proj_y, d_mp->proj_xr,       d_mp->n_obs,  d_mp->desc, 1};
    int r = run_projection(c, s, fd, c->grid_geom, c->sf_dev.p, mpd, mp_stride, c->last_B, nnratio, th, d_owner,
                           d_owner_obs, d_nmatches);
    timer_mark(c, "search_proj");
    return r;
}

int orbgpu_is_in_frustum_batch(orbgpu_ctx* c, const orbgpu_camera* d_cams, int B, orbgpu_grid_geom bounds,
                               const orbgpu_mappoint_geom_view* d_mp, float viewingCosLimit, int m_stride,
                               uint8_t* d_in_view, float* d_px, float* d_py, float* d_pxr, int32_t* d_level,
                               float* d_vc)
{
    static_assert(sizeof(orbgpu_camera) == 23 * 4, "orbgpu_camera: 22 floats + int");
    if (!c || !d_cams || B < 0 || !d_mp || d_mp->m < 0 || m_stride < d_mp->m) return ORBGPU_ERR_ARG;
    if (d_mp->m && (!d_mp->pos || !d_mp->normal || !d_mp->max_dist || !d_mp->min_dist || !d_in_view || !d_px ||
                    !d_py || !d_pxr || !d_level || !d_vc))
        return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    timer_mark(c, "frustum0");
    og_launch_frustum_batch(c->stream, d_cams, B, bounds.minX, bounds.maxX, bounds.minY, bounds.maxY,
                            OgMapGeomDev{d_mp->m, d_mp->pos, d_mp->normal, d_mp->max_dist, d_mp->min_dist},
                            viewingCosLimit, OgFrustumOut{d_in_view, d_px, d_py, d_pxr, d_level, d_vc, nullptr},
                            m_stride);
    HIP_TRY(c, hipGetLastError());
    timer_mark(c, "frustum");
    return ORBGPU_OK;
}

static OgCameraDev camera_dev(const orbgpu_camera* cam, float minX, float maxX, float minY, float maxY)
{
    OgCameraDev d{};
    std::memcpy(d.R, cam->Rcw, sizeof(d.R));
    std::memcpy(d.t, cam->tcw, sizeof(d.t));
    std::memcpy(d.Ow, cam->Ow, sizeof(d.Ow));
    d.fx = cam->fx;
    d.fy = cam->fy;
    d.cx = cam->cx;
    d.cy = cam->cy;
    d.mbf = cam->mbf;
    d.mb = cam->mb;
    d.scale_factor = cam->scale_factor;
    d.nlevels = cam->nlevels;
    d.minX = minX;
    d.maxX = maxX;
    d.minY = minY;
    d.maxY = maxY;
    return d;
}

int orbgpu_is_in_frustum(orbgpu_ctx* c, const orbgpu_camera* cam, orbgpu_grid_geom bounds,
                         const orbgpu_mappoint_geom_view* mp, float viewingCosLimit, uint8_t* track_in_view,
                         float* proj_x, float* proj_y, float* proj_xr, int32_t* level, float* view_cos,
                         int* n_in_view)
{
    if (!c || !cam || !mp || mp->m < 0 || cam->nlevels < 1 || !(cam->scale_factor > 0)) return ORBGPU_ERR_ARG;
    if (mp->m && (!mp->pos || !mp->normal || !mp->max_dist || !mp->min_dist || !track_in_view || !proj_x ||
                  !proj_y || !proj_xr || !level || !view_cos))
        return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t m = (size_t)std::max(mp->m, 1);
    HIP_TRY(c, ensure(c->mscratch, kCarvePad + m * (12 + 12 + 4 + 4 + 1 + 4 * 5) + 64));
    uint8_t* cur = c->mscratch.p;
    float* pos = (float*)scratch_carve(cur, m * 12);
    float* nrm = (float*)scratch_carve(cur, m * 12);
    float* mxd = (float*)scratch_carve(cur, m * 4);
    float* mnd = (float*)scratch_carve(cur, m * 4);
    uint8_t* iv = scratch_carve(cur, m);
    float* px = (float*)scratch_carve(cur, m * 4);
    float* py = (float*)scratch_carve(cur, m * 4);
    float* pxr = (float*)scratch_carve(cur, m * 4);
    int* lv = (int*)scratch_carve(cur, m * 4);
    float* vc = (float*)scratch_carve(cur, m * 4);
    int* nin = (int*)scratch_carve(cur, 16);
    hipStream_t s = c->stream;
    const size_t M = (size_t)mp->m;
    if (M) {
        HIP_TRY(c, hipMemcpyAsync(pos, mp->pos, M * 12, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(nrm, mp->normal, M * 12, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(mxd, mp->max_dist, M * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(mnd, mp->min_dist, M * 4, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(c, hipMemsetAsync(nin, 0, 4, s));
    og_launch_frustum(s, camera_dev(cam, bounds.minX, bounds.maxX, bounds.minY, bounds.maxY),
                      OgMapGeomDev{mp->m, pos, nrm, mxd, mnd}, viewingCosLimit,
                      OgFrustumOut{iv, px, py, pxr, lv, vc, nin});
    HIP_TRY(c, hipGetLastError());
    int hn = 0;
    HIP_TRY(c, hipMemcpyAsync(&hn, nin, 4, hipMemcpyDeviceToHost, s));
    if (M) {
        HIP_TRY(c, hipMemcpyAsync(track_in_view, iv, M, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(proj_x, px, M * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(proj_y, py, M * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(proj_xr, pxr, M * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(level, lv, M * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(view_cos, vc, M * 4, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(c, hipStreamSynchronize(s));
    if (n_in_view) *n_in_view = hn;
    return ORBGPU_OK;
}

// bForward / bBackward of SearchByProjection(Frame&, const Frame&) (src/ORBmatcher.cc:1338-1349):
// twc = -Rcw^T tcw, tlc = Rlw*twc + tlw, float, left to right (pinned as in the oracle)
static int last_frame_mode(const orbgpu_camera* cur, const orbgpu_camera* last, int bMono)
{
    float twc[3], tlc[3];
    for (int j = 0; j < 3; j++) {
        float s = cur->Rcw[j] * cur->tcw[0];
        s = s + cur->Rcw[3 + j] * cur->tcw[1];
        s = s + cur->Rcw[6 + j] * cur->tcw[2];
        twc[j] = -s;
    }
    for (int r = 0; r < 3; r++) {
        float s = last->Rcw[3 * r] * twc[0];
        s = s + last->Rcw[3 * r + 1] * twc[1];
        s = s + last->Rcw[3 * r + 2] * twc[2];
        tlc[r] = s + last->tcw[r];
    }
    if (tlc[2] > cur->mb && !bMono) return 1;
    if (-tlc[2] > cur->mb && !bMono) return 2;
    return 0;
}

int orbgpu_search_by_projection_last_frame(orbgpu_ctx* c, const orbgpu_frame_view* F, const orbgpu_camera* curc,
                                           const orbgpu_camera* lastc, const orbgpu_last_frame_view* LF, float th,
                                           int bMono, int checkOri, int32_t* owner, int32_t* owner_obs,
                                           int* nmatches)
{
    if (!c || !F || !curc || !lastc || !LF || !nmatches || F->n < 0 || LF->n < 0) return ORBGPU_ERR_ARG;
    if (F->n && (!owner || !owner_obs)) return ORBGPU_ERR_ARG;
    if (!F->scale_factors || F->nlevels < 1) return ORBGPU_ERR_ARG;
    if (LF->n && (!LF->kps || !LF->has_mp || !LF->outlier || !LF->pos || !LF->n_obs || !LF->desc))
        return ORBGPU_ERR_ARG;
    if (LF->n >= (1 << 24) || F->n >= (1 << 24)) return ORBGPU_ERR_UNSUPPORTED;
    HIP_TRY(c, hipSetDevice(c->device));
    const int n = std::max(F->n, 1), L = std::max(LF->n, 1);
    const size_t fixed = kCarvePad + (size_t)n * (28 + 32 + 4 + 4 + 4 + 4) + (OG_GRID_CELLS + 1) * 4 +
                         (size_t)L * (28 + 1 + 1 + 12 + 4 + 32 + 4 + 4 + 4) + 64 + F->nlevels * 4;
    HIP_TRY(c, ensure(c->mscratch, fixed));
    uint8_t* cur = c->mscratch.p;
    orbgpu_kp_dev* k = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)n * 28);
    uint8_t* d = scratch_carve(cur, (size_t)n * 32);
    float* ur = (float*)scratch_carve(cur, (size_t)n * 4);
    int* own = (int*)scratch_carve(cur, (size_t)n * 4);
    int* obs = (int*)scratch_carve(cur, (size_t)n * 4);
    int* cnts = (int*)scratch_carve(cur, 16);
    int* cs = (int*)scratch_carve(cur, (OG_GRID_CELLS + 1) * 4);
    int* ci = (int*)scratch_carve(cur, (size_t)n * 4);
    float* sfd = (float*)scratch_carve(cur, (size_t)F->nlevels * 4);
    orbgpu_kp_dev* lk = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)L * 28);
    uint8_t* hm = scratch_carve(cur, (size_t)L);
    uint8_t* ol = scratch_carve(cur, (size_t)L);
    float* lp = (float*)scratch_carve(cur, (size_t)L * 12);
    int* lo = (int*)scratch_carve(cur, (size_t)L * 4);
    uint8_t* ld = scratch_carve(cur, (size_t)L * 32);
    int* cnt = (int*)scratch_carve(cur, (size_t)L * 4);
    int* off = (int*)scratch_carve(cur, (size_t)(L + 1) * 4);
    int* ent = (int*)scratch_carve(cur, (size_t)L * 4);
    int* nm = (int*)scratch_carve(cur, 16);
    hipStream_t s = c->stream;
    if (F->n) {
        HIP_TRY(c, hipMemcpyAsync(k, F->kps, (size_t)F->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(d, F->desc, (size_t)F->n * 32, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(own, owner, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(obs, owner_obs, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
        if (F->uright) HIP_TRY(c, hipMemcpyAsync(ur, F->uright, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(c, hipMemcpyAsync(sfd, F->scale_factors, (size_t)F->nlevels * 4, hipMemcpyHostToDevice, s));
    if (LF->n) {
        HIP_TRY(c, hipMemcpyAsync(lk, LF->kps, (size_t)LF->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(hm, LF->has_mp, (size_t)LF->n, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(ol, LF->outlier, (size_t)LF->n, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(lp, LF->pos, (size_t)LF->n * 12, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(lo, LF->n_obs, (size_t)LF->n * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(ld, LF->desc, (size_t)LF->n * 32, hipMemcpyHostToDevice, s));
    }
    int hc = F->n;
    HIP_TRY(c, hipMemcpyAsync(cnts, &hc, sizeof(int), hipMemcpyHostToDevice, s));
    const OgGridGeom G{F->grid.minX, F->grid.minY, F->grid.maxX, F->grid.maxY, F->grid.invW, F->grid.invH};
    if (int r = launch_host_grid(c, s, k, cnts, n, F->n, G, cs, ci)) return r;
    OgFrameDev fd{k, d, cnts, cs, ci, F->uright ? ur : nullptr, n};
    OgLastFrameDev lfd{LF->n, lk, hm, ol, lp, lo, ld};
    const OgCameraDev cam = camera_dev(curc, G.minX, G.maxX, G.minY, G.maxY);
    const int mode = last_frame_mode(curc, lastc, bMono);
    og_launch_last_count(s, fd, G, sfd, cam, lfd, th, mode, cnt, off);
    int total = 0;
    HIP_TRY(c, hipMemcpyAsync(&total, off + LF->n, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    HIP_TRY(c, ensure(c->mcands, (size_t)std::max(total, 1) * sizeof(OgLastCand)));
    og_launch_last_resolve(s, fd, G, sfd, cam, lfd, th, mode, checkOri, off, (OgLastCand*)c->mcands.p, ent, own, obs,
                           nm);
    HIP_TRY(c, hipGetLastError());
    int hnm = 0;
    HIP_TRY(c, hipMemcpyAsync(&hnm, nm, sizeof(int), hipMemcpyDeviceToHost, s));
    if (F->n) {
        HIP_TRY(c, hipMemcpyAsync(owner, own, (size_t)F->n * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipMemcpyAsync(owner_obs, obs, (size_t)F->n * 4, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(c, hipStreamSynchronize(s));
    *nmatches = hnm;
    return ORBGPU_OK;
}

static int search_by_projection_keyframe(orbgpu_ctx* c, const orbgpu_frame_view* F, const orbgpu_camera* curc,
                                         const orbgpu_keyframe_view* KF, const int32_t* pred_level, float th,
                                         int ORBdist, int checkOri, int32_t* owner, int* nmatches)
{
    if (!c || !F || !curc || !KF || !nmatches || F->n < 0 || KF->n < 0) return ORBGPU_ERR_ARG;
    if (F->n && !owner) return ORBGPU_ERR_ARG;
    if (!F->scale_factors || F->nlevels < 1) return ORBGPU_ERR_ARG;
    if (KF->n && (!KF->kps || !KF->valid || !KF->pos || !KF->desc)) return ORBGPU_ERR_ARG;
    if (KF->n && !pred_level && (!KF->max_dist || !KF->min_dist)) return ORBGPU_ERR_ARG;
    if (KF->n >= (1 << 24) || F->n >= (1 << 24)) return ORBGPU_ERR_UNSUPPORTED;
    HIP_TRY(c, hipSetDevice(c->device));
    const int n = std::max(F->n, 1), L = std::max(KF->n, 1);
    const size_t fixed = kCarvePad + (size_t)n * (28 + 32 + 4 + 4) + (OG_GRID_CELLS + 1) * 4 +
                         (size_t)L * (28 + 1 + 12 + 4 + 4 + 32 + 4 + 4 + 4) + 64 + F->nlevels * 4;
    HIP_TRY(c, ensure(c->mscratch, fixed));
    uint8_t* cur = c->mscratch.p;
    orbgpu_kp_dev* k = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)n * 28);
    uint8_t* d = scratch_carve(cur, (size_t)n * 32);
    int* own = (int*)scratch_carve(cur, (size_t)n * 4);
    int* cnts = (int*)scratch_carve(cur, 16);
    int* cs = (int*)scratch_carve(cur, (OG_GRID_CELLS + 1) * 4);
    int* ci = (int*)scratch_carve(cur, (size_t)n * 4);
    float* sfd = (float*)scratch_carve(cur, (size_t)F->nlevels * 4);
    orbgpu_kp_dev* kk = (orbgpu_kp_dev*)scratch_carve(cur, (size_t)L * 28);
    uint8_t* kv = scratch_carve(cur, (size_t)L);
    float* kp3 = (float*)scratch_carve(cur, (size_t)L * 12);
    float* kmx = (float*)scratch_carve(cur, (size_t)L * 4);  // (pred_level: the levels)
    float* kmn = (float*)scratch_carve(cur, (size_t)L * 4);
    uint8_t* kd = scratch_carve(cur, (size_t)L * 32);
    int* cnt = (int*)scratch_carve(cur, (size_t)L * 4);
    int* off = (int*)scratch_carve(cur, (size_t)(L + 1) * 4);
    int* ent = (int*)scratch_carve(cur, (size_t)L * 4);
    int* nm = (int*)scratch_carve(cur, 16);
    hipStream_t s = c->stream;
    if (F->n) {
        HIP_TRY(c, hipMemcpyAsync(k, F->kps, (size_t)F->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(d, F->desc, (size_t)F->n * 32, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(own, owner, (size_t)F->n * 4, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(c, hipMemcpyAsync(sfd, F->scale_factors, (size_t)F->nlevels * 4, hipMemcpyHostToDevice, s));
    if (KF->n) {
        HIP_TRY(c, hipMemcpyAsync(kk, KF->kps, (size_t)KF->n * 28, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(kv, KF->valid, (size_t)KF->n, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(kp3, KF->pos, (size_t)KF->n * 12, hipMemcpyHostToDevice, s));
        if (pred_level) {
            HIP_TRY(c, hipMemcpyAsync(kmx, pred_level, (size_t)KF->n * 4, hipMemcpyHostToDevice, s));
        } else {
            HIP_TRY(c, hipMemcpyAsync(kmx, KF->max_dist, (size_t)KF->n * 4, hipMemcpyHostToDevice, s));
            HIP_TRY(c, hipMemcpyAsync(kmn, KF->min_dist, (size_t)KF->n * 4, hipMemcpyHostToDevice, s));
        }
        HIP_TRY(c, hipMemcpyAsync(kd, KF->desc, (size_t)KF->n * 32, hipMemcpyHostToDevice, s));
    }
    int hc = F->n;
    HIP_TRY(c, hipMemcpyAsync(cnts, &hc, sizeof(int), hipMemcpyHostToDevice, s));
    const OgGridGeom G{F->grid.minX, F->grid.minY, F->grid.maxX, F->grid.maxY, F->grid.invW, F->grid.invH};
    if (int r = launch_host_grid(c, s, k, cnts, n, F->n, G, cs, ci)) return r;
    OgFrameDev fd{k, d, cnts, cs, ci, nullptr, n};
    OgLastFrameDev kfd{KF->n, kk, kv, nullptr, kp3, nullptr, kd};
    OgCameraDev cam = camera_dev(curc, G.minX, G.maxX, G.minY, G.maxY);
    for (int j = 0; j < 3; j++) {  // Ow = -Rcw^T tcw as the matcher computes it (src/ORBmatcher.cc:1478)
        float t = curc->Rcw[j] * curc->tcw[0];
        t = t + curc->Rcw[3 + j] * curc->tcw[1];
        t = t + curc->Rcw[6 + j] * curc->tcw[2];
        cam.Ow[j] = -t;
    }
    const int* lv = pred_level ? (const int*)kmx : nullptr;
    og_launch_kf_count(s, fd, G, sfd, cam, kfd, kmx, kmn, lv, th, cnt, off);
    int total = 0;
    HIP_TRY(c, hipMemcpyAsync(&total, off + KF->n, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    HIP_TRY(c, ensure(c->mcands, (size_t)std::max(total, 1) * sizeof(OgLastCand)));
    og_launch_kf_resolve(s, fd, G, sfd, cam, kfd, kmx, kmn, lv, th, ORBdist, checkOri, off, (OgLastCand*)c->mcands.p,
                         ent, own, nm);
    HIP_TRY(c, hipGetLastError());
    int hnm = 0;
    HIP_TRY(c, hipMemcpyAsync(&hnm, nm, sizeof(int), hipMemcpyDeviceToHost, s));
    if (F->n) HIP_TRY(c, hipMemcpyAsync(owner, own, (size_t)F->n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    *nmatches = hnm;
    return ORBGPU_OK;
}

int orbgpu_search_by_projection_keyframe(orbgpu_ctx* c, const orbgpu_frame_view* F, const orbgpu_camera* curc,
                                         const orbgpu_keyframe_view* KF, float th, int ORBdist, int checkOri,
                                         int32_t* owner, int* nmatches)
{
    return search_by_projection_keyframe(c, F, curc, KF, nullptr, th, ORBdist, checkOri, owner, nmatches);
}

int orbgpu_search_by_projection_keyframe_levels(orbgpu_ctx* c, const orbgpu_frame_view* F, const orbgpu_camera* curc,
                                                const orbgpu_keyframe_view* KF, const int32_t* pred_level, float th,
                                                int ORBdist, int checkOri, int32_t* owner, int* nmatches)
{
    if (KF && KF->n && !pred_level) return ORBGPU_ERR_ARG;
    return search_by_projection_keyframe(c, F, curc, KF, pred_level, th, ORBdist, checkOri, owner, nmatches);
}

int orbgpu_debug_candidates(orbgpu_ctx* c, int b, int level, uint64_t* out, int cap)
{
    if (!c || !c->last_B || b < 0 || b >= c->last_B || level < 0 || level >= c->nlevels) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const OgLevel& L = c->plan.lv[level];
    int n = 0;
    HIP_TRY(c, hipMemcpy(&n, c->cand_count.p + (size_t)b * c->nlevels + level, sizeof(int), hipMemcpyDeviceToHost));
    n = std::min(n, L.cand_cap);
    if (out && cap > 0)
        HIP_TRY(c, hipMemcpy(out, c->cand.p + (size_t)b * c->plan.cand_per_frame + L.cand_off,
                             (size_t)std::min(n, cap) * 8, hipMemcpyDeviceToHost));
    return n;
}

int orbgpu_debug_octree(orbgpu_ctx* c, int b, int level, uint32_t* xy, uint32_t* resp, int cap)
{
    if (!c || !c->last_B || b < 0 || b >= c->last_B || level < 0 || level >= c->nlevels) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const OgLevel& L = c->plan.lv[level];
    int n = 0;
    HIP_TRY(c, hipMemcpy(&n, c->oct_count.p + (size_t)b * c->nlevels + level, sizeof(int), hipMemcpyDeviceToHost));
    const size_t o = (size_t)b * c->plan.kcap_total + L.koff;
    const int m = std::min(n, cap);
    if (xy && m > 0) HIP_TRY(c, hipMemcpy(xy, c->oct_xy.p + o, (size_t)m * 4, hipMemcpyDeviceToHost));
    if (resp && m > 0) HIP_TRY(c, hipMemcpy(resp, c->oct_resp.p + o, (size_t)m * 4, hipMemcpyDeviceToHost));
    return n;
}

int orbgpu_debug_octree_profile(orbgpu_ctx* c, unsigned long long* out, int n)
{
    if (!c || !out || n <= 0) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const hipError_t e = og_read_oct_prof(out, n);
    if (e == hipErrorNotSupported) return ORBGPU_ERR_UNSUPPORTED;
    HIP_TRY(c, e);
    return ORBGPU_OK;
}

int orbgpu_debug_set_projection_paths(orbgpu_ctx* c, int flags)
{
    if (!c || (flags & ~(ORBGPU_DEBUG_PROJ_FILL_HBM | ORBGPU_DEBUG_PROJ_RESOLVE_HBM))) return ORBGPU_ERR_ARG;
    c->dbg_proj = flags;
    return ORBGPU_OK;
}

int orbgpu_debug_fast_profile(orbgpu_ctx* c, unsigned long long* out, int n)
{
    if (!c || !out || n <= 0) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const hipError_t e = og_read_fast_prof(out, n);
    if (e == hipErrorNotSupported) return ORBGPU_ERR_UNSUPPORTED;
    HIP_TRY(c, e);
    return ORBGPU_OK;
}

void* orbgpu_stream(orbgpu_ctx* c) { return c ? (void*)c->stream : nullptr; }

int orbgpu_synchronize(orbgpu_ctx* c)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return check_status(c);
}

int orbgpu_set_stage_timing(orbgpu_ctx* c, int on)
{
    if (!c) return ORBGPU_ERR_ARG;
    c->timer.on = on != 0;
    return ORBGPU_OK;
}

int orbgpu_stage_times(orbgpu_ctx* c, const char** names, float* ms, int cap)
{
    if (!c) return ORBGPU_ERR_ARG;
    const int n = collect_timer(c) ? (int)c->timer.last_ms.size() : (int)c->timer.last_ms.size();
    for (int i = 0; i < n && i < cap; i++) {
        if (names) names[i] = c->timer.last_names[i];
        if (ms) ms[i] = c->timer.last_ms[i];
    }
    return n;
}

int orbgpu_stage_marks(orbgpu_ctx* c, orbgpu_ctx* ref, const char** names, float* t_ms, int cap)
{
    if (!c || !ref || !names || !t_ms || cap < 0) return ORBGPU_ERR_ARG;
    StageTimer& t = c->timer;
    StageTimer& r = ref->timer;
    if (!t.on || !r.on || t.used < 1 || r.used < 1) return 0;
    HIP_TRY(c, hipEventSynchronize(t.ev[t.used - 1]));
    HIP_TRY(c, hipEventSynchronize(r.ev[0]));
    const int n = std::min(cap, t.used);
    for (int i = 0; i < n; i++) {
        float ms = 0;
        HIP_TRY(c, hipEventElapsedTime(&ms, r.ev[0], t.ev[i]));
        t_ms[i] = ms;
        names[i] = t.names[i];
    }
    return n;
}

const char* orbgpu_last_error(const orbgpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* orbgpu_device_alloc(orbgpu_ctx* c, size_t bytes)
{
    if (!c) return nullptr;
    void* p = nullptr;
    if (hipSetDevice(c->device) != hipSuccess || hipMalloc(&p, std::max<size_t>(bytes, 1)) != hipSuccess) return nullptr;
    return p;
}
int orbgpu_device_free(orbgpu_ctx* c, void* p)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipFree(p));
    return ORBGPU_OK;
}
int orbgpu_memcpy_h2d(orbgpu_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return ORBGPU_OK;
}
int orbgpu_memcpy_d2h(orbgpu_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return ORBGPU_OK;
}
int orbgpu_memcpy_h2d_async(orbgpu_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    return ORBGPU_OK;
}
int orbgpu_memcpy_d2h_async(orbgpu_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    return ORBGPU_OK;
}
int orbgpu_memcpy_d2d_async(orbgpu_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    return ORBGPU_OK;
}

long long orbgpu_batch_candidate_total(orbgpu_ctx* c)
{
    if (!c || !c->last_B) return ORBGPU_ERR_ARG;
    if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) return ORBGPU_ERR_HIP;
    std::vector<int> cc((size_t)c->last_B * c->nlevels);
    if (hipMemcpy(cc.data(), c->cand_count.p, cc.size() * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return ORBGPU_ERR_HIP;
    long long t = 0;
    for (int v : cc) t += v;
    return t;
}

int orbgpu_memset_d(orbgpu_ctx* c, void* dst, int value, size_t bytes)
{
    if (!c) return ORBGPU_ERR_ARG;
    HIP_TRY(c, hipMemsetAsync(dst, value, bytes, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return ORBGPU_OK;
}

}  // extern "C"
