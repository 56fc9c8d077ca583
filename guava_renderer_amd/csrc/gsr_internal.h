// gsr_internal.h -- kernel parameter blocks, scratch-arena layout and launchers.
//
// HBM layout (DESIGN.md "Data layout"): every per-Gaussian quantity is a structure-of-arrays
// slab over B*P entries (frame-major), every per-pixel quantity a slab over B*H*W, every
// per-tile quantity a slab over B*T, every per-instance (Gaussian x tile) quantity a slab over
// the batch's R.  Slabs start on 256-byte boundaries.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gsr_math.h"

namespace gsr {

constexpr int kScanBlock = 256;       // Gaussians per preprocess / binning workgroup
constexpr int kSortSmallCap = 2048;   // instances per tile sorted by the 256-thread LDS sort
constexpr int kSortLargeCap = 8192;   // instances per tile sorted by the 1024-thread LDS sort
constexpr int kLdsTileHist = 8192;    // tiles per frame counted in LDS (more -> global atomics)
constexpr int kRenderBatch = 64;      // Gaussians staged in LDS per render_bwd round
constexpr int kStrips = 4;            // 16x4 pixel strips per 16x16 tile (one render wave each)
constexpr int kMaxGaussians = 1 << 28; // Gaussian index field of the binning key (bits 4..31)

// control words (uint32) at the head of the geometry arena
enum Ctrl : int {
    kCtrlRLo = 0,        // total instances of the batch
    kCtrlOverflow = 1,   // R > binning capacity
    kCtrlError = 2,      // bit0: prefiltered point culled
    kCtrlNumLarge = 3,   // tiles whose list exceeds kSortSmallCap
    kCtrlRenderHead = 4, // render worklist dequeue counter
    kCtrlBwdHead = 5,    // render-backward worklist dequeue counter
    kCtrlNonEmpty = 6,   // tiles of the batch with a non-empty list
    kCtrlXcdQueue = 1024,  // 8 per-XCD render dequeue counters, 4 KiB apart
    kCtrlXcdStride = 1024,
    kCtrlWords = 9216
};

struct GeomArena {
    uint32_t* ctrl;
    float* depth;
    float* invdepth;
    int* radii;
    float2* means2D;
    float* cov3D;
    float4* conic;
    uint2* rect;          // (xmin | ymin<<16, xmax | ymax<<16)
    float4* rrec;         // render record, 2 x float4 per Gaussian: (x, y, opacity, 1/depth),
                          // (-a/2, -b, -c/2, 0) of the conic (see render_fwd.hip)
    uint32_t* tiles;
    uint32_t* offsets;    // inclusive scan of tiles over the batch
    uint32_t* blocksums;  // per scan block; scanned in place to exclusive block offsets
};

struct ImageArena {
    float* final_T;
    uint32_t* n_contrib;
    uint2* ranges;        // per tile [start, end) into the batch's point_list
    uint32_t* tile_count;
    uint32_t* large_list; // worklist of tiles with > kSortSmallCap instances
    uint32_t* work_list;  // every tile of the batch, longest list first (render scheduling)
};

struct BinArena {
    uint32_t* point_list;  // per tile, depth-sorted Gaussian index (within its frame)
    uint64_t* keys;        // unsorted (depth bits << 32 | index), grouped per tile
    uint32_t* inst_slot;   // per (Gaussian, tile) instance: rank inside its tile's list
    uint8_t* smask;        // per sorted instance: bit s set <=> the Gaussian can reach alpha >= 1/255
                           // somewhere in the tile's 16x4 pixel strip s (render_fwd's wave unit)
};

struct Dims {
    int B, P, W, H, gx, gy, T, nblk;  // nblk: scan blocks per frame
};

inline Dims make_dims(int B, int P, int W, int H) {
    Dims d;
    d.B = B; d.P = P; d.W = W; d.H = H;
    d.gx = (W + GSR_BX - 1) / GSR_BX;
    d.gy = (H + GSR_BY - 1) / GSR_BY;
    d.T = d.gx * d.gy;
    d.nblk = (P + kScanBlock - 1) / kScanBlock;
    return d;
}

// Arena carving (base == nullptr -> size query).
size_t carve_geom(char* base, const Dims& d, GeomArena* g);
size_t carve_image(char* base, const Dims& d, ImageArena* im);
size_t carve_bin(char* base, int64_t R, BinArena* b);

struct Inputs {
    const float* means3D; int64_t s_means;     // element stride between frames (0 = shared)
    const float* scales; int64_t s_scales;
    const float* rot; int64_t s_rot;
    const float* opac; int64_t s_opac;
    const float* cov3D_pre; int64_t s_cov;
    const float* colors; int64_t s_colors;
    const float* view;                          // 16 floats per frame
    const float* proj;                          // 16 floats per frame
    const float* tan_dev;                       // 2 floats per frame, or null -> tanx/tany
    float tanx, tany;
    const float* bg; int64_t s_bg;
    float scale_mod;
    int prefiltered, antialiasing;
};

struct Outputs {
    float* out_color;     // [B][C][H][W]
    float* out_invdepth;  // [B][H][W] or null
    int* radii;           // [B][P] or null
    uint64_t* stats;      // gsr_render_counters words, or null (production kernel)
};

struct Grads {
    const float* dL_dpix;        // [B][C][H][W]
    const float* dL_dinvdepth;   // [B][H][W] or null
    float* dL_dmean2D;           // [B][P][3]  (accumulated)
    float* dL_dconic;            // [B][P][4]  (accumulated)
    float* dL_dopacity;          // [B][P]     (accumulated, then AA-scaled)
    float* dL_dcolors;           // [B][P][C]  (accumulated)
    float* dL_dinvdepth_g;       // [B][P] or null (accumulated)
    float* dL_dmeans3D;          // [B][P][3]
    float* dL_dcov3D;            // [B][P][6]
    float* dL_dscale;            // [B][P][3] or null
    float* dL_drot;              // [B][P][4] or null
};

// Workgroups for a persistent (work-queue) launch: CUs of the current device x per_cu.
int persistent_grid(int per_cu);

// ---- launchers (all asynchronous on `stream`) ----
void launch_preprocess(const Dims& d, const Inputs& in, const GeomArena& g, const Outputs& o,
                       hipStream_t s);
void launch_scan_blocksums(const Dims& d, const GeomArena& g, int64_t R_cap, hipStream_t s);
void launch_bin_count(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                      hipStream_t s);
void launch_tile_scan(const Dims& d, const GeomArena& g, const ImageArena& im, hipStream_t s);
void launch_bin_scatter(const Dims& d, const GeomArena& g, const ImageArena& im,
                        const BinArena& b, hipStream_t s);
void launch_tile_sort(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                      hipStream_t s);
void launch_render_fwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Outputs& o, bool exact, hipStream_t s);
void launch_render_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Grads& gr, bool exact, hipStream_t s);
void launch_preprocess_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const Grads& gr,
                           hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t s);

}  // namespace gsr
