// gsr_internal.h -- kernel parameter blocks, scratch-arena layout and launchers.
//
// HBM layout (DESIGN.md "Data layout"): every per-Gaussian quantity is a structure-of-arrays
// slab over B*P entries (frame-major), every per-pixel quantity a slab over B*H*W, every
// per-tile quantity a slab over B*T, every per-instance (Gaussian x tile) quantity a slab over
// the batch's R.  Slabs start on 256-byte boundaries.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gsr_math.h"

namespace gsr {

// Tuning and timing-ablation switches (GSR_RENDER_*, GSR_SCATTER_*, GSR_BWD_*, ...).  The product
// library always takes the default: only the A/B builds of tools/build_ab.py (-DGSR_TUNING) read
// them from the environment, and only those builds contain the ablation kernels (which produce
// wrong images by construction).  A stray variable in a deployment therefore changes nothing
// (tests/test_boundary.py::test_product_library_has_no_tuning_switches).
#ifdef GSR_TUNING
inline int tune_env(const char* name, int def) {
    const char* e = getenv(name);
    return e ? atoi(e) : def;
}
#else
inline int tune_env(const char*, int def) { return def; }
#endif

constexpr int kScanBlock = 256;       // Gaussians per preprocess / binning workgroup
constexpr int kSortSmallCap = 2048;   // keys per segment sorted by the 256-thread LDS sort
constexpr int kSortLargeCap = 8192;   // keys per segment sorted by the 1024-thread LDS sort
constexpr int kTinyBucket = 64;       // depth buckets up to this size are ranked in place
constexpr int kSlots = 256;           // k_ordered_scatter: Gaussians per pass (one per thread)
constexpr int kRenderBatch = 64;      // Gaussians staged in LDS per render_bwd round
constexpr int kStrips = 4;            // 64-pixel strips per 16x16 tile (one render wave each)
#ifndef GSR_STRIP_W
#define GSR_STRIP_W 8
#endif
constexpr int kStripW = GSR_STRIP_W;        // strip width: 8 (8x8 strips, 2x2 per tile) or 16 (16x4)
constexpr int kStripH = 64 / kStripW;
constexpr int kStripsX = GSR_BX / kStripW;  // strips per tile row
static_assert(kStripsX * (GSR_BY / kStripH) == kStrips, "4 strips of 64 pixels per tile");
// pixel origin of strip s of tile (tx, ty); lane l of its wave owns pixel (x0 + l % kStripW, y0 + l / kStripW)
__host__ __device__ __forceinline__ void strip_origin(int tx, int ty, int s, int& x0, int& y0) {
    x0 = tx * GSR_BX + (s % kStripsX) * kStripW;
    y0 = ty * GSR_BY + (s / kStripsX) * kStripH;
}

// control words (uint32) at the head of the geometry arena
enum Ctrl : int {
    kCtrlRLo = 0,        // total instances of the batch
    kCtrlOverflow = 1,   // R > binning capacity
    kCtrlError = 2,      // bit0: prefiltered point culled
    kCtrlNumBig = 3,     // depth buckets longer than kTinyBucket (segment-sort worklist)
    kCtrlRenderHead = 4, // render worklist dequeue counter
    kCtrlBwdHead = 5,    // render-backward worklist dequeue counter
    kCtrlNonEmpty = 6,   // tiles of the batch with a non-empty list
    kCtrlFwdOnly = 7,    // set by a GSR_FORWARD_ONLY forward: the backward-only rows were not written
    kCtrlQStart = 16,    // queue map 2: first strip_list tile of each XCD queue (8 words), then
                         // the queue's tile count (8 words)
    kCtrlXcdQueue = 1024,  // 8 per-XCD render dequeue counters, 4 KiB apart
    kCtrlXcdStride = 1024,
    kCtrlWords = 9216
};
// per-frame words following the control words (zeroed with them)
enum FrameStat : int {
    kFsNotKeyMax = 0,  // max of ~depth_bits over the frame's visible Gaussians (= ~min key)
    kFsKeyMax = 1,     // max of depth_bits
    kFsVisible = 2,    // visible Gaussians (bucket-scan total)
    kFsR = 3,          // instances of the frame
    kFsRBase = 4,      // instances of the frames before it (batch-wide list offset)
    kFsNonEmpty = 5,   // non-empty tiles of the frame
    kFsWords = 8
};
constexpr int kMaxFrames = 256;   // frames per batch (per-frame tables live in LDS)
constexpr int kLptBuckets = 34;   // render work list: clz(list length), 33 = empty tile
constexpr int kStripBuckets = 129;  // strip work list: 4 buckets per octave of survivors, 128 = none

struct GeomArena {
    uint32_t* ctrl;       // kCtrlWords control words, then kFsWords per frame
    uint32_t* fstat;      // = ctrl + kCtrlWords
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
    uint32_t* blocksums;  // per scan block; scanned in place to exclusive block offsets
    uint32_t* blockkey;   // per scan block: max depth key, max ~depth key of its visible Gaussians
    // per-frame depth sort of the visible Gaussians (bucket sort on the depth float bits)
    uint32_t* bslot;      // per Gaussian: arrival slot inside its depth bucket
    uint32_t* bstart;     // per frame NB+1 bucket counts, scanned in place to bucket starts
    uint64_t* skey;       // per frame, (depth bits << 32 | index) grouped by bucket
    uint32_t* big;        // worklist of buckets longer than kTinyBucket: frame * NB + bucket
    uint32_t* order;      // per frame, visible Gaussians in (depth, index) order
    uint32_t* table;      // [B][nchunk][T] instance counts per (depth chunk, tile), scanned per tile
    uint32_t* fsplit;     // [P][32] features pre-split for the split-bf16 blend: bf16 (hi | lo << 16)
    float* gterm;         // [B*P][8] render_bwd's per-Gaussian screen-space gradient sums (kGt* order),
                          // consumed by preprocess_bwd
    // batch path only (else null): status words that survive the per-call ctrl reset --
    // [kStickyOverflow] set by any overflowing forward, [kStickyRMax] largest batch R seen; cleared
    // by the host (gsr_batch_status_offset)
    uint32_t* sticky = nullptr;
};
// gterm row: dL/dmean2D x, y, dL/dconic x, y, w, dL/dopacity, dL/dinvdepth, (unused)
enum GTerm : int { kGtM2x = 0, kGtM2y = 1, kGtCx = 2, kGtCy = 3, kGtCw = 4, kGtOp = 5, kGtInv = 6, kGtWords = 8 };
enum Sticky : int { kStickyOverflow = 0, kStickyRMax = 1, kStickyWords = 4 };

struct ImageArena {
    float* final_T;
    uint32_t* n_contrib;
    uint2* ranges;        // per tile [start, end) into the batch's point_list
    uint32_t* tile_count;
    uint32_t* work_list;  // every tile of the batch, longest list first (render scheduling)
    uint32_t* lpt_hist;   // per frame: tiles per work-list bucket
    uint32_t* strip_cnt;  // per tile x 4 strips: list entries whose strip bit is set
    uint32_t* strip_list; // the strips of the non-empty tiles, most survivors first: tile << 2 | strip
    uint32_t* strip_hist; // per frame: strips per kStripBuckets bucket (map 2: per XCD queue x bucket,
                          // then rewritten in place as list offsets)
    uint32_t* strip_list_bwd;  // the backward's list: one longest-first list, tile-major (map 1)
};

struct BinArena {
    uint32_t* point_list;  // per tile, depth-sorted: Gaussian index (within its frame, bits 0..27) |
                           // strip mask << 28, bit s set <=> the Gaussian can reach alpha >= 1/255
                           // somewhere in the tile's pixel strip s (strip_origin; render_fwd's wave unit)
    uint32_t* qmask;       // single-frame arenas only (else null): per point_list entry, bit 4 s + q set
                           // <=> it can reach alpha >= 1/255 in quad q (4x4) of strip s (the quad waves)
};

struct Dims {
    int B, P, W, H, gx, gy, T, nblk;  // nblk: scan blocks per frame
    int NB;                           // depth buckets per frame (power of two)
    int chunk;                        // depth-ordered Gaussians per instance-count table row
    int nchunk;                       // rows of the count table per frame
};

inline Dims make_dims(int B, int P, int W, int H) {
    Dims d;
    d.B = B; d.P = P; d.W = W; d.H = H;
    d.gx = (W + GSR_BX - 1) / GSR_BX;
    d.gy = (H + GSR_BY - 1) / GSR_BY;
    d.T = d.gx * d.gy;
    d.nblk = (P + kScanBlock - 1) / kScanBlock;
    int nb = 64;
    // up to 512k Gaussians: <= 16384 buckets, so the frame's bucket table fits the LDS of
    // k_bucket_count_lds (64 KB; <= 32 keys per bucket on average); beyond, ~8 keys per bucket
    // (global-atomic counting) so that the buckets stay small enough for in-place ranking
    const int nb_cap = P <= (1 << 19) ? (1 << 14) : (1 << 20);
    static const int kdiv = [] {  // GSR_BUCKET_DIV: keys per bucket target (tuning)
        const int v = tune_env("GSR_BUCKET_DIV", 16);
        return v >= 2 && v <= 256 ? v : 16;
    }();
    while (nb < P / kdiv && nb < nb_cap) nb <<= 1;
    d.NB = nb;
    // count-table rows: kSlots Gaussians (one scatter pass) up to 1024 tiles; beyond, the dense
    // (row x tile) table and each row's base[] load outweigh the extra passes (1024-Gaussian rows)
    static const int passes_env = [] {  // GSR_CHUNK_PASSES: scatter passes per table row (tuning)
        const int v = tune_env("GSR_CHUNK_PASSES", 0);
        return v >= 1 && v <= 64 ? v : 0;
    }();
    d.chunk = (passes_env ? passes_env : (d.T > 1024 ? 4 : 1)) * kSlots;
    d.nchunk = (P + d.chunk - 1) / d.chunk;
    return d;
}

// Arena carving (base == nullptr -> size query).
size_t carve_geom(char* base, const Dims& d, GeomArena* g);
size_t carve_image(char* base, const Dims& d, ImageArena* im);
size_t carve_bin(char* base, int64_t R, BinArena* b, bool qmask = false);

// Upper bound on P: the render kernels address a frame's feature rows (128 B per Gaussian) through
// a buffer resource with 32-bit byte offsets, so P * 128 must stay below 2^31.
constexpr int kMaxGaussians = 1 << 24;
constexpr uint32_t kIndexMask = (1u << 28) - 1u;  // point_list entry -> Gaussian index
// Upper bound on tiles per frame (the ordered scatter keeps a per-tile counter array in LDS).
constexpr int kMaxTiles = 16384;

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
    int fwd_only;         // GSR_FORWARD_ONLY: preprocess writes only what binning and compositing read
    int zero_ctrl;        // the forward's first kernel zeroes the control words (no memset launch)
    uint32_t xcd_map;     // render work-queue mapping (queue_item): 1 = tile-affine (strip order tile-major)
    int fuse_totals;      // B = 1, no host read-back of R: the frame totals are reduced inside the
    int64_t totals_cap;   // depth sort's bucket count (launch_depth_sort), against this R capacity
};

struct Outputs {
    float* out_color;     // [B][C][H][W]
    float* out_invdepth;  // [B][H][W] or null
    int* radii;           // [B][P] or null
    uint64_t* stats;      // gsr_render_counters words, or null (production kernel)
    uint32_t* timeline;   // gsr_render_timeline records (instrumented kernel only), or null
    uint32_t timeline_cap;
    // refiner-head epilogue (gsr_forward_batch_refine) over gsr_refine_prepare'd features:
    // out_refine [B][n_out][H][W] = leaky_relu(channels [keep, keep+n_out) + b); null = off.
    // keep: channels of out_color written.
    const float* rb = nullptr;  // [n_out] or null
    float* out_refine = nullptr;
    int n_out = 0;
    int keep = GSR_C;
    float slope = 0.2f;
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
    int invd;                    // dL_dinvdepth is given (its term enters dL/dt_z)
    int reduce;                  // frame-reduced outputs: colors [P][C] (accumulated), opacity [P],
                                 // means3D [P][3], scale [P][3], rot [P][4] summed over frames;
                                 // the per-frame mean2D / conic / cov3D / invdepth outputs unused
};

// Records `msg` for gsr_last_error() and returns -status (capi.hip).
int api_fail(int status, const char* msg);

// Workgroups for a persistent (work-queue) launch: CUs of the current device x per_cu.
int persistent_grid(int per_cu);
// whether a forward of these dims / numerics / outputs composites on the single-frame quad kernel
// (the only reader of the binning arena's quad masks): otherwise no mask is carved or computed
bool render_uses_quad(const Dims& d, bool split, const Outputs& o);
// persistent grid of a launch on stream s: the CUs that stream may use (a CU-masked stream made by
// gsr_stream_create_cu_mask) times per_cu
int persistent_grid_on(hipStream_t s, int per_cu);
// GSR_STRIP_ORDER: "strip" orders the render work by each strip's survivors; "tile" (default) by
// tile (its longest strip), the 4 strips consecutive and dealt to one XCD queue (L2 reuse).
int strip_order_tile_major();
// GSR_XCD_MAP: the render work-queue map (queue_item) -- 1 tile-affine, 2 block-affine (default)
int xcd_queue_map();
// map 2: the XCD queue of tile t -- 4x4-tile blocks (64x64 pixels) dealt over the eight queues,
// shifted by 3 per block row, so every queue holds a spread of blocks (balanced) and neighbouring
// tiles, which share Gaussians, read them through one L2
#ifndef GSR_XCD_BLOCK_SHIFT
#define GSR_XCD_BLOCK_SHIFT 2  // log2 of the block side in tiles
#endif
__host__ __device__ __forceinline__ uint32_t tile_queue(int t, int gx) {
    const int tx = t % gx, ty = t / gx;
    return (uint32_t)((tx >> GSR_XCD_BLOCK_SHIFT) + 3 * (ty >> GSR_XCD_BLOCK_SHIFT)) & 7u;
}

// Render work items (render_fwd / render_bwd): the 4 strips of each of the ne non-empty tiles in
// strip_list order (items [0, 4 ne)), then nempty whole empty tiles (items [4 ne, 4 ne + nempty)).
// Eight per-XCD queues; the k-th dequeue of queue q returns:
//  * map 0: item q + 8k;
//  * map 1 (tile-affine): queue q owns list tiles q, q+8, q+16, ... with their 4 strips consecutive,
//    then the empty tiles e = q (mod 8): a tile's strips read the same Gaussians from one L2;
//  * map 2 (block-affine): queue q owns its segment of the strip list (the tiles of its blocks,
//    tile_queue, most survivors first; bounds in ctrl[kCtrlQStart..]), 4 strips per tile
//    consecutive, then the empty tiles e = q (mod 8).
// 0xFFFFFFFF when queue q is drained.
__device__ __forceinline__ uint32_t queue_item(uint32_t q, uint32_t k, uint32_t ne, uint32_t nempty,
                                               uint32_t map, const uint32_t* ctrl) {
    if (map == 0) {
        const uint32_t item = q + 8u * k;
        return item < 4u * ne + nempty ? item : 0xFFFFFFFFu;
    }
    if (map == 2) {
        const uint32_t nq = ctrl[kCtrlQStart + 8 + q];
        if (k < 4u * nq) return 4u * (ctrl[kCtrlQStart + q] + (k >> 2)) + (k & 3u);
        const uint32_t e = q + 8u * (k - 4u * nq);
        return e < nempty ? 4u * ne + e : 0xFFFFFFFFu;
    }
    const uint32_t ntq = ne > q ? (ne - q + 7u) >> 3 : 0u;  // tiles owned by queue q
    if (k < 4u * ntq) return 4u * (q + 8u * (k >> 2)) + (k & 3u);
    const uint32_t e = q + 8u * (k - 4u * ntq);
    return e < nempty ? 4u * ne + e : 0xFFFFFFFFu;
}

// The same mapping with every strip split into S work items (S = 2: half-strip render waves, 4: quad
// waves): 4 S items per non-empty tile, then the empty tiles.
template <uint32_t S>
__device__ __forceinline__ uint32_t queue_item_n(uint32_t q, uint32_t k, uint32_t ne, uint32_t nempty,
                                                 uint32_t map, const uint32_t* ctrl) {
    constexpr uint32_t per = 4u * S;  // items per tile
    if (map == 0) {
        const uint32_t item = q + 8u * k;
        return item < per * ne + nempty ? item : 0xFFFFFFFFu;
    }
    if (map == 2) {
        const uint32_t nq = ctrl[kCtrlQStart + 8 + q];
        if (k < per * nq) return per * (ctrl[kCtrlQStart + q] + k / per) + k % per;
        const uint32_t e = q + 8u * (k - per * nq);
        return e < nempty ? per * ne + e : 0xFFFFFFFFu;
    }
    const uint32_t ntq = ne > q ? (ne - q + 7u) >> 3 : 0u;
    if (k < per * ntq) return per * (q + 8u * (k / per)) + k % per;
    const uint32_t e = q + 8u * (k - per * ntq);
    return e < nempty ? per * ne + e : 0xFFFFFFFFu;
}

// ---- launchers (all asynchronous on `stream`) ----
void launch_preprocess(const Dims& d, const Inputs& in, const GeomArena& g, const Outputs& o,
                       hipStream_t s);
void launch_scan_blocksums(const Dims& d, const GeomArena& g, int64_t R_cap, hipStream_t s);
// per-frame depth sort of the visible Gaussians -> g.order
void launch_depth_sort(const Dims& d, const GeomArena& g, hipStream_t s, int64_t fused_totals_cap = -1);
// instance counts per (depth chunk, tile), scanned per tile -> g.table, im.tile_count
void launch_chunk_count(const Dims& d, const GeomArena& g, const ImageArena& im, hipStream_t s);
void launch_tile_scan(const Dims& d, const GeomArena& g, const ImageArena& im, hipStream_t s);
// depth-ordered instance emission -> point_list (index | strip mask << 28)
// survivors per strip -> strip_cnt; strips of the non-empty tiles, most survivors first -> strip_list
void launch_strip_order(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                        hipStream_t s);
// the strip list of queue map 1 (one longest-first list, tile-major) into `out` (render_bwd)
void launch_strip_list_tile(const Dims& d, const ImageArena& im, uint32_t* out, hipStream_t s);
void launch_ordered_scatter(const Dims& d, const GeomArena& g, const ImageArena& im,
                            const BinArena& b, hipStream_t s);
void launch_render_fwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Outputs& o, bool exact, bool split, hipStream_t s);
void launch_render_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Grads& gr, bool exact, bool split, hipStream_t s);
// the split-bf16 (hi | lo << 16) words of a [P][32] feature table -> out (g.fsplit)
void launch_split_features(int P, const float* colors, uint32_t* out, hipStream_t s);
void launch_preprocess_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const Grads& gr,
                           hipStream_t s);
void launch_refine_prepare(int n, const float* in, const float* w, int n_out, int keep, float* out,
                           hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t s);

}  // namespace gsr
