// orbgpu_internal.h -- shared host/device definitions of the gfx950 ORB pipeline.
//
// Layout in HBM (per context, B frames per batch):
//   pyramid   : levels 1..L-1 of every frame, each row padded to a 64-byte pitch (level 0 is read
//               in place from the caller's frame buffer -- the reference pads it by 19 px, a region
//               the hot path never reads, src/ORBextractor.cc:1113-1128).
//   cand      : per (frame, level) FAST candidate slots, one u64 {x_rel:16, y_rel:16, response:8};
//               slot capacity = the exact NMS bound of that level (no overflow possible).
//   node_of   : per candidate u16 node index (octree scratch).
//   oct_best  : per (frame, level) OG_OCT_BEST_CELLS u32: the octree's depth-D cell-best table (scratch).
//   octree out: per (frame, level) up to kcap u32 {x:16, y:16} + u8 response, list order.
//   kps/desc  : per frame `frame_cap` orbgpu_keypoint (28 B AoS, cv::KeyPoint layout) + 32-B rows.
#pragma once
#include <stdint.h>

#include "../../include/orbgpu.h"  // ORBGPU_SEM_* (semantics switch)

// umax of src/ORBextractor.cc:454-469 for HALF_PATCH_SIZE = 15 (the reference's constant); the describe
// kernel's flattened IC_Angle disk is built from it at compile time
#define OG_UMAX 15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3
#define OG_MAXLEVELS 16
#define OG_EDGE 19
#define OG_PATCH 31
#define OG_HALF_PATCH 15
#define OG_GRID_COLS 64
#define OG_GRID_ROWS 48
#define OG_GRID_CELLS (OG_GRID_COLS * OG_GRID_ROWS)
#define OG_OCT_MAXL 1024   // max octree list length handled in LDS (N_l + 3 + slack), one node per thread
#define OG_OCT_BEST_CELLS (4 * OG_OCT_MAXL)  // octree cell-best table entries per (frame, level): >= depth-D cells
#define OG_OCT_MAXL_BIG 2048  // the same with two list nodes per thread (~143 KB of LDS): levels of up to ~2040 features
#define OG_MAX_CELL_W 64   // wCell <= 59 for any width (nCols = floor(w/30))
#define OG_MAX_PITCH (1u << 24)  // row pitches (bytes) below this: 24-bit row-offset products in the kernels
#define OG_GRID_LDS_ITEMS 8192  // per-frame keypoint capacity (frame_cap) the grid kernel sorts in LDS

struct OgLevel {
    int w, h;              // level size
    int pitch;             // bytes per row in the pyramid buffer (levels >= 1)
    long long pyr_off;     // byte offset of the level inside one frame's pyramid block (levels >= 1)
    // FAST cell grid, src/ORBextractor.cc:773-787
    int minB, maxBX, maxBY;
    int nCols, nRows, wCell, hCell;
    int cell_base, ncells; // into the flat cell table
    int fb_off;            // first entry of the level in the FAST block table (OgFastBlk, padded per level)
    // octree, src/ORBextractor.cc:539-563
    int N;                 // mnFeaturesPerLevel
    int nIni;
    float hX;
    int kcap;              // octree output capacity of the level
    int koff;              // offset of the level's octree slots inside a frame
    long long cand_off;    // offset (entries) of the level's candidate slots inside a frame
    int cand_cap;
    // resize tables (levels >= 1), src/ORBextractor.cc:1120 -> cv::resize INTER_LINEAR
    int xtab_off, ytab_off, xmax;
    // level l fused with level l+1 in one launch (og_resize2_kernel): LDS capacities over all tiles of l+1
    int fz_SR, fz_SC, fz_AR, fz_AC;
    int fz_tile_off;       // per-tile region bounds of that launch (3 int4 per tile of l+1, in the resize tables)
    float scale;           // mvScaleFactor[l]
    int patch_size;        // (int)(PATCH_SIZE * mvScaleFactor[l])
};

struct OgCell {            // one FAST block of up to 2x2 cells (ROI union), src/ORBextractor.cc:789-829
    short level, i, j, pad;   // first cell (row i, column j); pad = (cell rows << 8) | cell columns
    short x0, y0, x1, y1;  // ROI [x0,x1) x [y0,y1) in level pixels
};

// One FAST block as the kernel reads it (og_fast_quad_kernel): everything it needs from the block, its level and
// the plan, precomputed on the host and read with one 32-byte scalar load (no per-wave level-table lookups).
struct OgFastBlk {
    int src_off;           // levels >= 1: byte offset of ROI pixel (0, 0) inside the frame's pyramid block;
                           // level 0: the ROI's first column (the row term y0 * pitch0 is added at run time)
    int pitch;             // row pitch of the level (levels >= 1); 0 for level 0 (the caller's pitch)
    short y0, lev;         // ROI first row (level 0's row term), pyramid level
    unsigned char rw, rh;  // ROI size (detection area + 6): rw - 6 <= 64, rh - 6 <= 80
    unsigned char wC, hC;  // FAST cell size of the level
    int cand_off;          // the level's candidate slots inside a frame (entries)
    int cand_cap;          // ... and their number (the exact NMS bound)
    short ox, oy;          // candidate coordinates of detection pixel (0, 0): x0 - minB + 3, y0 - minB + 3
    unsigned colw;         // byte k: detection columns of the block in 16-column segment k, clamp(dw - 16 k, 0, 16)
};

struct OgPlan {
    int nlevels;
    int sem;               // ORBGPU_SEM_* of the context (include/orbgpu.h)
    int oct_big;           // levels 0 .. oct_big-1 run the OG_OCT_MAXL_BIG octree kernel (their lists may exceed OG_OCT_MAXL)
    int iniTh, minTh;
    int total_cells;
    int fast_blocks;       // entries of the OgFastBlk table per frame
    int kcap_total;        // sum of kcap (octree slots per frame)
    int frame_cap;         // final keypoints per frame (== kcap_total)
    long long cand_per_frame;
    long long pyr_per_frame;   // bytes
    int umax[16];
    OgLevel lv[OG_MAXLEVELS];
};

// packed FAST candidate
__host__ __device__ inline unsigned long long og_pack_cand(int x, int y, int resp)
{
    return (unsigned long long)(unsigned)(x & 0xffff) | ((unsigned long long)(unsigned)(y & 0xffff) << 16) |
           ((unsigned long long)(unsigned)(resp & 0xff) << 32);
}
