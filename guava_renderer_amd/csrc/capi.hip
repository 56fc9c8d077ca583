// capi.hip -- host driver behind include/gsr.h: carves the scratch arenas, sequences the kernels
// on the caller's HIP stream and reports errors.  The single-frame entry points keep the
// reference's one host synchronisation (num_rendered sizes the binning buffer,
// rasterizer_impl.cu:284-288); the batch entry points have none.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_deform.h"

#include "gsr_internal.h"

using namespace gsr;

namespace {

thread_local std::string g_err;
uint64_t* g_render_counters = nullptr;  // gsr_render_counters
uint32_t* g_timeline = nullptr;         // gsr_render_timeline
uint32_t g_timeline_cap = 0;

int fail(gsr_status st, const std::string& msg) {
    g_err = msg;
    return -(int)st;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(GSR_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

#define STAGE(debug, stream, name)                                                           \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ == hipSuccess && (debug)) e_ = hipStreamSynchronize(stream);                  \
        if (e_ != hipSuccess)                                                                \
            return fail(GSR_ERR_HIP, std::string(name) + ": " + hipGetErrorString(e_));      \
    } while (0)

// ---- stage profiling (HIP events on the launch stream) ----
constexpr int kStages = GSR_NUM_STAGES;
uint32_t g_prof_mask = 0;
struct EvPair { hipEvent_t a, b; int stage; };
std::vector<EvPair> g_ev_pool;
size_t g_ev_used = 0;
double g_prof_ms[kStages] = {0};
int g_prof_cnt[kStages] = {0};

struct StageTimer {
    EvPair* p = nullptr;
    hipStream_t s;
    StageTimer(int stage, hipStream_t st) : s(st) {
        if (!(g_prof_mask & (1u << stage))) return;
        if (g_ev_used == g_ev_pool.size()) {
            EvPair e;
            if (hipEventCreate(&e.a) != hipSuccess || hipEventCreate(&e.b) != hipSuccess) return;
            g_ev_pool.push_back(e);
        }
        p = &g_ev_pool[g_ev_used++];
        p->stage = stage;
        hipEventRecord(p->a, s);
    }
    ~StageTimer() {
        if (p) hipEventRecord(p->b, s);
    }
};

// per-call numerics flags (include/gsr.h GSR_NUMERICS_*)
inline bool exact_exp(uint32_t numerics) { return (numerics & GSR_NUMERICS_FAST_EXP) == 0; }
inline bool split_bf16(uint32_t numerics) { return (numerics & GSR_NUMERICS_SPLIT_BF16) != 0; }
constexpr uint32_t kNumericsKnown = GSR_NUMERICS_FAST_EXP | GSR_NUMERICS_SPLIT_BF16;
constexpr uint32_t kForwardBatchKnown = kNumericsKnown | GSR_FORWARD_ONLY;

inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }
inline size_t ctrl_words(const Dims& d) { return (size_t)kCtrlWords + (size_t)kFsWords * d.B; }

template <typename T>
inline T* take(char* base, size_t& off, size_t count) {
    off = align_up(off);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += sizeof(T) * count;
    return p;
}

}  // namespace

namespace gsr {

static void env_tuning(Inputs& in) {
    in.xcd_map = strip_order_tile_major() ? (uint32_t)xcd_queue_map() : 0u;
}

int xcd_queue_map() {
    static const int v = tune_env("GSR_XCD_MAP", 2) == 1 ? 1 : 2;
    return v;
}

int strip_order_tile_major() {
    static const int v = tune_env("GSR_STRIP_ORDER_TILE", 1) != 0 ? 1 : 0;  // 0: strips ordered alone (A/B)
    return v;
}

int persistent_grid(int per_cu) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus * per_cu;
}

// CU counts of the CU-masked streams made by gsr_stream_create_cu_mask
static std::mutex g_cu_mu;
static std::unordered_map<hipStream_t, int> g_stream_cus;

int persistent_grid_on(hipStream_t s, int per_cu) {
    {
        std::lock_guard<std::mutex> lk(g_cu_mu);
        const auto it = g_stream_cus.find(s);
        if (it != g_stream_cus.end()) return it->second * per_cu;
    }
    return persistent_grid(per_cu);
}

size_t carve_geom(char* base, const Dims& d, GeomArena* g) {
    const size_t n = (size_t)d.B * d.P;
    size_t off = 0;
    GeomArena a;
    a.ctrl = take<uint32_t>(base, off, ctrl_words(d));
    a.fstat = a.ctrl ? a.ctrl + kCtrlWords : nullptr;
    a.depth = take<float>(base, off, n);
    a.invdepth = take<float>(base, off, n);
    a.radii = take<int>(base, off, n);
    a.means2D = take<float2>(base, off, n);
    a.cov3D = take<float>(base, off, 6 * n);
    a.conic = take<float4>(base, off, n);
    a.rect = take<uint2>(base, off, n);
    a.rrec = take<float4>(base, off, 2 * n);
    a.tiles = take<uint32_t>(base, off, n);
    a.blocksums = take<uint32_t>(base, off, (size_t)d.B * d.nblk + 1);
    a.blockkey = take<uint32_t>(base, off, (size_t)d.B * d.nblk * 2);
    a.bslot = take<uint32_t>(base, off, n);
    a.bstart = take<uint32_t>(base, off, (size_t)d.B * (d.NB + 1));
    a.skey = take<uint64_t>(base, off, n);
    a.big = take<uint32_t>(base, off, (size_t)d.B * d.NB);
    a.order = take<uint32_t>(base, off, n);
    a.table = take<uint32_t>(base, off, (size_t)d.B * d.nchunk * d.T);
    a.fsplit = take<uint32_t>(base, off, (size_t)d.P * GSR_C);
    a.gterm = take<float>(base, off, n * kGtWords);
    if (g) *g = a;
    return align_up(off) + 256;
}

size_t carve_image(char* base, const Dims& d, ImageArena* im) {
    const size_t npx = (size_t)d.B * d.W * d.H;
    const size_t nt = (size_t)d.B * d.T;
    size_t off = 0;
    ImageArena a;
    a.final_T = take<float>(base, off, npx);
    a.n_contrib = take<uint32_t>(base, off, npx);
    a.ranges = take<uint2>(base, off, nt);
    a.tile_count = take<uint32_t>(base, off, nt);
    a.work_list = take<uint32_t>(base, off, nt);
    a.lpt_hist = take<uint32_t>(base, off, (size_t)d.B * kLptBuckets);
    a.strip_cnt = take<uint32_t>(base, off, (size_t)kStrips * nt);
    a.strip_list = take<uint32_t>(base, off, (size_t)kStrips * nt);
    a.strip_hist = take<uint32_t>(base, off, (size_t)d.B * 8 * kStripBuckets);
    a.strip_list_bwd = take<uint32_t>(base, off, (size_t)kStrips * nt);
    if (im) *im = a;
    return align_up(off) + 256;
}

// qmask: the single-frame quad masks after the list (forward entry points of one frame, and batch
// workspaces of B = 1)
size_t carve_bin(char* base, int64_t R, BinArena* b, bool qmask) {
    const size_t n = (size_t)(R > 0 ? R : 1);
    size_t off = 0;
    BinArena a;
    a.point_list = take<uint32_t>(base, off, n);
    a.qmask = qmask ? take<uint32_t>(base, off, n) : nullptr;
    if (b) *b = a;
    return align_up(off) + 256;
}

// the fused assembly + projection of the avatar pipeline (deform.hip)
void launch_deform_preprocess(const Dims& d, const Inputs& in, const GeomArena& g, const Outputs& o,
                              const GsrDeformInputs& dg, hipStream_t s);

}  // namespace gsr

namespace {

// Render placement (gsr_set_render_stream): forwards enqueued on a registered stream run their
// compositing kernel on its render stream, ordered by two events (the render waits for the binning,
// the stream's later work waits for the render).
struct RenderRoute {
    hipStream_t render;
    hipEvent_t ready, done;
};
std::mutex g_route_mu;
std::unordered_map<hipStream_t, RenderRoute> g_routes;

bool render_route(hipStream_t s, RenderRoute* r) {
    std::lock_guard<std::mutex> lk(g_route_mu);
    const auto it = g_routes.find(s);
    if (it == g_routes.end()) return false;
    *r = it->second;
    return true;
}

// Shared forward sequence once R is known and the binning arena exists.
int run_binning_and_render(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                           const BinArena& bn, const Outputs& o, uint32_t numerics, int debug, hipStream_t s) {
    { StageTimer st_(2, s); launch_depth_sort(d, g, s, in.fuse_totals ? in.totals_cap : -1); }
    STAGE(debug, s, "depth_sort");
    { StageTimer st_(3, s); launch_chunk_count(d, g, im, s); }
    STAGE(debug, s, "chunk_count");
    { StageTimer st_(4, s); launch_tile_scan(d, g, im, s); }
    STAGE(debug, s, "tile_scan");
    {
        StageTimer st_(5, s);
        launch_ordered_scatter(d, g, im, bn, s);
        launch_strip_order(d, g, im, bn, s);
    }
    STAGE(debug, s, "ordered_scatter");
    RenderRoute rt;
    const bool routed = render_route(s, &rt);
    hipStream_t rs = s;
    if (routed) {
        HIP_TRY(hipEventRecord(rt.ready, s));
        HIP_TRY(hipStreamWaitEvent(rt.render, rt.ready, 0));
        rs = rt.render;
    }
    { StageTimer st_(6, rs); launch_render_fwd(d, in, g, im, bn, o, exact_exp(numerics), split_bf16(numerics), rs); }
    if (routed) {
        HIP_TRY(hipEventRecord(rt.done, rs));
        HIP_TRY(hipStreamWaitEvent(s, rt.done, 0));
    }
    STAGE(debug, s, "render_fwd");
    return 0;
}

}  // namespace

// error reporting for the other C-ABI translation units (deform.hip)
int gsr::api_fail(int status, const char* msg) { return fail((gsr_status)status, msg); }

extern "C" {

#ifndef GSR_SRC_HASH
#define GSR_SRC_HASH "unstamped"
#endif
// "gsr-gfx950 <version> <source hash>": the hash of the sources the library was built from
// (guava_renderer_amd/build.py source_hash), checked against the tree by the Python loader
const char* gsr_version(void) { return "gsr-gfx950 0.2 " GSR_SRC_HASH; }
const char* gsr_last_error(void) { return g_err.c_str(); }

size_t gsr_geometry_bytes(int P, int width, int height) {
    return carve_geom(nullptr, make_dims(1, P, width, height), nullptr);
}
size_t gsr_image_bytes(int width, int height) {
    return carve_image(nullptr, make_dims(1, 1, width, height), nullptr);
}
size_t gsr_binning_bytes(int64_t R) { return carve_bin(nullptr, R, nullptr, true); }

// Instances one frame can produce at most: every Gaussian in every tile (getRect clamps to the
// grid), capped at the int range of num_rendered.
static int64_t async_bound(const Dims& d) {
    const int64_t b = (int64_t)d.P * d.T;
    return b < 0x7FFFFFFFll ? b : 0x7FFFFFFFll;
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream) {
    if (P < 0) return fail(GSR_ERR_ARG, "P < 0");
    launch_mark_visible(P, means3D, viewmatrix, projmatrix, present, (hipStream_t)stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GSR_ERR_HIP, std::string("mark_visible: ") + hipGetErrorString(e));
    return 0;
}

// gsr_forward_async without a status block (prefiltered 0): the async path, nothing copied back
static uint32_t* const kNoStatus = reinterpret_cast<uint32_t*>(uintptr_t(1));

// status_host == nullptr: the reference's synchronous contract (R read back after the scan, the
// binning buffer sized to R, num_rendered returned).  Otherwise the binning buffer is sized to
// the upper bound P x tiles (R cannot exceed it), nothing waits on the device, and the control
// words {R, overflow, error flags, 0} are copied to status_host (pinned) at the end of the stream.
static int forward_single(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                          void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                          const float* means3D, const float* shs, const float* colors_precomp,
                          const float* opacities, const float* scales, float scale_modifier,
                          const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                          const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                          int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                          int debug, uint32_t* status_host, uint32_t numerics, hipStream_t s) {
    (void)D; (void)M; (void)shs; (void)cam_pos;
    if (P < 0 || width <= 0 || height <= 0) return fail(GSR_ERR_ARG, "bad P/width/height");
    if (numerics & ~kNumericsKnown) return fail(GSR_ERR_ARG, "unknown numerics flags");
    if (P >= kMaxGaussians) return fail(GSR_ERR_ARG, "P must be < 2^24");
    if ((int64_t)((width + 15) / 16) * ((height + 15) / 16) > kMaxTiles) return fail(GSR_ERR_ARG, "image too large");
    const Dims d = make_dims(1, P, width, height);
    GeomArena g;
    ImageArena im;
    char* gb = geometryBuffer(alloc_ctx, carve_geom(nullptr, d, nullptr));
    if (!gb) return fail(GSR_ERR_ALLOC, "geometryBuffer allocation failed");
    carve_geom(gb, d, &g);
    char* ib = imageBuffer(alloc_ctx, carve_image(nullptr, d, nullptr));
    if (!ib) return fail(GSR_ERR_ALLOC, "imageBuffer allocation failed");
    carve_image(ib, d, &im);
    if (colors_precomp == nullptr)
        return fail(GSR_ERR_NO_COLORS, "For non-RGB, provide precomputed Gaussian colors!");
    if (((uintptr_t)colors_precomp & 15) != 0) return fail(GSR_ERR_ARG, "colors_precomp must be 16-byte aligned");
    if (cov3D_precomp == nullptr && (scales == nullptr || rotations == nullptr))
        return fail(GSR_ERR_ARG, "scales/rotations or cov3D_precomp required");

    Inputs in{};
    env_tuning(in);
    in.means3D = means3D; in.s_means = 0;
    in.scales = scales; in.s_scales = 0;
    in.rot = rotations; in.s_rot = 0;
    in.opac = opacities; in.s_opac = 0;
    in.cov3D_pre = cov3D_precomp; in.s_cov = 0;
    in.colors = colors_precomp; in.s_colors = 0;
    in.view = viewmatrix; in.proj = projmatrix;
    in.tan_dev = nullptr; in.tanx = tan_fovx; in.tany = tan_fovy;
    in.bg = background; in.s_bg = 0;
    in.scale_mod = scale_modifier;
    in.prefiltered = prefiltered; in.antialiasing = antialiasing;
    Outputs o{out_color, depth, radii, g_render_counters, g_timeline, g_timeline_cap};

    // the control words are zeroed by the first kernel (zero_ctrl_words), except for a prefiltered
    // forward (its culling-error word is set during that kernel) or an empty one (no kernel)
    in.zero_ctrl = !in.prefiltered && d.P > 0 && d.B > 0;
    if (!in.zero_ctrl) HIP_TRY(hipMemsetAsync(g.ctrl, 0, ctrl_words(d) * 4, s));
    // quad masks (4 B per instance and a pass) only for a forward that composites on the quad kernel
    const bool quad = render_uses_quad(d, split_bf16(numerics), o);
    { StageTimer st_(0, s); launch_preprocess(d, in, g, o, s); }
    STAGE(debug, s, "preprocess");
    if (status_host) {
        const int64_t cap = async_bound(d);
        // nothing reads R on the host before the binning: the frame totals go into the depth sort's
        // first kernel (launch_depth_sort)
        in.fuse_totals = 1;
        in.totals_cap = cap;
        STAGE(debug, s, "scan");
        char* bb = binningBuffer(alloc_ctx, carve_bin(nullptr, cap, nullptr, quad));
        if (!bb) return fail(GSR_ERR_ALLOC, "binningBuffer allocation failed");
        BinArena bn;
        carve_bin(bb, cap, &bn, quad);
        int rc = run_binning_and_render(d, in, g, im, bn, o, numerics, debug, s);
        if (rc < 0) return rc;
        if (status_host != kNoStatus)
            HIP_TRY(hipMemcpyAsync(status_host, g.ctrl, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        return 0;
    }
    { StageTimer st_(1, s); launch_scan_blocksums(d, g, (int64_t)0xFFFFFFF0u, s); }
    STAGE(debug, s, "scan");
    uint32_t ctrl_h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(ctrl_h, g.ctrl, sizeof(ctrl_h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ctrl_h[kCtrlError] & 1u)
        return fail(GSR_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (ctrl_h[kCtrlOverflow] || ctrl_h[kCtrlRLo] > 0x7FFFFFFFu)
        return fail(GSR_ERR_CAPACITY, "instance count exceeds 2^31 - 1 (num_rendered is an int)");
    const int64_t R = ctrl_h[kCtrlRLo];
    char* bb = binningBuffer(alloc_ctx, carve_bin(nullptr, R, nullptr, quad));
    if (!bb) return fail(GSR_ERR_ALLOC, "binningBuffer allocation failed");
    BinArena bn;
    carve_bin(bb, R, &bn, quad);
    int rc = run_binning_and_render(d, in, g, im, bn, o, numerics, debug, s);
    if (rc < 0) return rc;
    return (int)R;
}

int gsr_forward(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                const float* means3D, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier,
                const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                int debug, void* stream) {
    return forward_single(geometryBuffer, binningBuffer, imageBuffer, alloc_ctx, P, D, M, background, width,
                          height, means3D, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                          cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                          out_color, depth, antialiasing, radii, debug, nullptr, GSR_NUMERICS_EXACT,
                          (hipStream_t)stream);
}

int gsr_forward_ex(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                   void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                   const float* means3D, const float* shs, const float* colors_precomp,
                   const float* opacities, const float* scales, float scale_modifier,
                   const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                   const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                   int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                   int debug, uint32_t numerics, void* stream) {
    return forward_single(geometryBuffer, binningBuffer, imageBuffer, alloc_ctx, P, D, M, background, width,
                          height, means3D, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                          cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                          out_color, depth, antialiasing, radii, debug, nullptr, numerics, (hipStream_t)stream);
}

int64_t gsr_forward_async_bound(int P, int width, int height) {
    if (P <= 0 || width <= 0 || height <= 0) return 0;
    return async_bound(make_dims(1, P, width, height));
}

int gsr_forward_async(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                      void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                      const float* means3D, const float* shs, const float* colors_precomp,
                      const float* opacities, const float* scales, float scale_modifier,
                      const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                      const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                      int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                      int debug, uint32_t* status_host, uint32_t numerics, void* stream) {
    if (!status_host && prefiltered) return fail(GSR_ERR_ARG, "gsr_forward_async: null status_host with prefiltered");
    if (debug) return fail(GSR_ERR_ARG, "gsr_forward_async: debug mode synchronises; use gsr_forward");
    return forward_single(geometryBuffer, binningBuffer, imageBuffer, alloc_ctx, P, D, M, background, width,
                          height, means3D, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                          cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                          out_color, depth, antialiasing, radii, debug, status_host ? status_host : kNoStatus,
                          numerics, (hipStream_t)stream);
}

char* gsr_scratch_geometry(void* scratch, size_t bytes) {
    const gsr_scratch* sc = static_cast<const gsr_scratch*>(scratch);
    return sc && bytes <= sc->geometry_cap ? sc->geometry : nullptr;
}
char* gsr_scratch_binning(void* scratch, size_t bytes) {
    const gsr_scratch* sc = static_cast<const gsr_scratch*>(scratch);
    return sc && bytes <= sc->binning_cap ? sc->binning : nullptr;
}
char* gsr_scratch_image(void* scratch, size_t bytes) {
    const gsr_scratch* sc = static_cast<const gsr_scratch*>(scratch);
    return sc && bytes <= sc->image_cap ? sc->image : nullptr;
}

int gsr_backward_ex(int P, int D, int M, int R, const float* background, int width, int height,
                    const float* means3D, const float* shs, const float* colors_precomp,
                    const float* opacities, const float* scales, float scale_modifier,
                    const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                    const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                    const int* radii, char* geom_buffer, char* binning_buffer, char* image_buffer,
                    const float* dL_dpix, const float* dL_invdepths, float* dL_dmean2D,
                    float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth,
                    float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                    float* dL_drot, int antialiasing, int debug, uint32_t numerics, void* stream) {
    (void)D; (void)M; (void)shs; (void)campos; (void)radii; (void)dL_dsh;
    hipStream_t s = (hipStream_t)stream;
    if (numerics & ~kNumericsKnown) return fail(GSR_ERR_ARG, "unknown numerics flags");
    if (P <= 0) return 0;
    if (colors_precomp == nullptr)
        return fail(GSR_ERR_NO_COLORS, "For non-RGB, provide precomputed Gaussian colors!");
    const Dims d = make_dims(1, P, width, height);
    GeomArena g;
    ImageArena im;
    BinArena bn;
    carve_geom(geom_buffer, d, &g);
    carve_image(image_buffer, d, &im);
    carve_bin(binning_buffer, R, &bn, true);
    Inputs in{};
    env_tuning(in);
    in.means3D = means3D;
    in.scales = scales;
    in.rot = rotations;
    in.opac = opacities;
    in.cov3D_pre = cov3D_precomp;
    in.colors = colors_precomp;
    in.view = viewmatrix; in.proj = projmatrix;
    in.tan_dev = nullptr; in.tanx = tan_fovx; in.tany = tan_fovy;
    in.bg = background;
    in.scale_mod = scale_modifier;
    in.antialiasing = antialiasing;
    Grads gr{};
    gr.dL_dpix = dL_dpix;
    gr.dL_dinvdepth = dL_invdepths;
    gr.dL_dmean2D = dL_dmean2D;
    gr.dL_dconic = dL_dconic;
    gr.dL_dopacity = dL_dopacity;
    gr.dL_dcolors = dL_dcolor;
    gr.dL_dinvdepth_g = dL_invdepths ? dL_dinvdepth : nullptr;
    gr.invd = gr.dL_dinvdepth != nullptr && gr.dL_dinvdepth_g != nullptr;
    gr.dL_dmeans3D = dL_dmean3D;
    gr.dL_dcov3D = dL_dcov3D;
    gr.dL_dscale = (cov3D_precomp == nullptr) ? dL_dscale : nullptr;
    gr.dL_drot = (cov3D_precomp == nullptr) ? dL_drot : nullptr;
    { StageTimer st_(7, s); launch_render_bwd(d, in, g, im, bn, gr, exact_exp(numerics), split_bf16(numerics), s); }
    STAGE(debug, s, "render_bwd");
    { StageTimer st_(8, s); launch_preprocess_bwd(d, in, g, gr, s); }
    STAGE(debug, s, "preprocess_bwd");
    return 0;
}

int gsr_backward(int P, int D, int M, int R, const float* background, int width, int height,
                 const float* means3D, const float* shs, const float* colors_precomp,
                 const float* opacities, const float* scales, float scale_modifier,
                 const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                 const int* radii, char* geom_buffer, char* binning_buffer, char* image_buffer,
                 const float* dL_dpix, const float* dL_invdepths, float* dL_dmean2D,
                 float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth,
                 float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                 float* dL_drot, int antialiasing, int debug, void* stream) {
    return gsr_backward_ex(P, D, M, R, background, width, height, means3D, shs, colors_precomp, opacities,
                           scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, campos,
                           tan_fovx, tan_fovy, radii, geom_buffer, binning_buffer, image_buffer, dL_dpix,
                           dL_invdepths, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolor, dL_dinvdepth,
                           dL_dmean3D, dL_dcov3D, dL_dsh, dL_dscale, dL_drot, antialiasing, debug,
                           GSR_NUMERICS_EXACT, stream);
}

// Batch workspace: geometry | image | binning arenas, then 256 bytes of sticky status words
// (kStickyWords, never reset by a call; the host zeroes them when it creates the workspace).
size_t gsr_batch_status_offset(int B, int P, int width, int height, int64_t R_capacity) {
    const Dims d = make_dims(B, P, width, height);
    return carve_geom(nullptr, d, nullptr) + carve_image(nullptr, d, nullptr) +
           carve_bin(nullptr, R_capacity, nullptr, B == 1);
}

size_t gsr_batch_workspace_bytes(int B, int P, int width, int height, int64_t R_capacity) {
    return gsr_batch_status_offset(B, P, width, height, R_capacity) + 256;
}

static void carve_workspace(char* ws, const Dims& d, int64_t R_cap, GeomArena* g, ImageArena* im,
                            BinArena* bn) {
    const size_t gsz = carve_geom(nullptr, d, nullptr);
    const size_t isz = carve_image(nullptr, d, nullptr);
    const size_t bsz = carve_bin(nullptr, R_cap, nullptr, d.B == 1);
    carve_geom(ws, d, g);
    carve_image(ws + gsz, d, im);
    carve_bin(ws + gsz + isz, R_cap, bn, d.B == 1);
    g->sticky = reinterpret_cast<uint32_t*>(ws + gsz + isz + bsz);
}

int gsr_forward_batch(int B, int P, int width, int height, const float* means3D,
                      int64_t means_stride, const float* colors, int64_t colors_stride,
                      const float* opacities, int64_t opac_stride, const float* scales,
                      int64_t scales_stride, const float* rotations, int64_t rot_stride,
                      float scale_modifier, const float* viewmatrices, const float* projmatrices,
                      const float* tanfov, const float* backgrounds, int64_t bg_stride,
                      char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                      int* radii, int antialiasing, uint32_t numerics, void* stream) {
    return gsr_forward_batch_refine(B, P, width, height, means3D, means_stride, colors, colors_stride,
                                    opacities, opac_stride, scales, scales_stride, rotations, rot_stride,
                                    scale_modifier, viewmatrices, projmatrices, tanfov, backgrounds,
                                    bg_stride, workspace, R_capacity, out_color, out_invdepth, radii,
                                    antialiasing, nullptr, numerics, stream);
}

// Host-side record of which batch workspaces the last forward left forward-only (GSR_FORWARD_ONLY
// or the fused deform path): a gsr_backward_batch* on such a workspace fails with GSR_ERR_ARG
// instead of returning the caller's zeroed gradients (the device word kCtrlFwdOnly still keeps
// the kernels from computing on it, e.g. for a workspace forwarded by another process).
static std::mutex g_ws_mu;
static std::unordered_map<const void*, bool> g_ws_fwd_only;
static void note_workspace(const void* ws, bool fwd_only) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    g_ws_fwd_only[ws] = fwd_only;
}
static bool workspace_fwd_only(const void* ws) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    const auto it = g_ws_fwd_only.find(ws);
    return it != g_ws_fwd_only.end() && it->second;
}

static int forward_batch_impl(int B, int P, int width, int height, const float* means3D,
                              int64_t means_stride, const float* colors, int64_t colors_stride,
                              const float* opacities, int64_t opac_stride, const float* scales,
                              int64_t scales_stride, const float* rotations, int64_t rot_stride,
                              float scale_modifier, const float* viewmatrices, const float* projmatrices,
                              const float* tanfov, const float* backgrounds, int64_t bg_stride,
                              char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                              int* radii, int antialiasing, const gsr_refine_epilogue* refine,
                              uint32_t numerics, const GsrDeformInputs* dg, hipStream_t s) {
    if (numerics & ~kForwardBatchKnown) return fail(GSR_ERR_ARG, "unknown numerics flags");
    if (refine) {
        if (!refine->out_refine || refine->n_out < 1 || refine->keep_channels < 0 ||
            refine->keep_channels + refine->n_out > GSR_C)
            return fail(GSR_ERR_ARG, "refine epilogue: out_refine required, n_out >= 1, keep + n_out <= 32");
    }
    if (B <= 0 || P <= 0 || width <= 0 || height <= 0 || !workspace || !tanfov)
        return fail(GSR_ERR_ARG, "bad batch arguments");
    if ((int64_t)((width + 15) / 16) * ((height + 15) / 16) > kMaxTiles) return fail(GSR_ERR_ARG, "image too large");
    if (B > kMaxFrames) return fail(GSR_ERR_ARG, "too many frames per batch");
    if (P >= kMaxGaussians) return fail(GSR_ERR_ARG, "P must be < 2^24");
    if (!colors) return fail(GSR_ERR_NO_COLORS, "For non-RGB, provide precomputed Gaussian colors!");
    if (((uintptr_t)colors & 15) != 0 || ((colors_stride * 4) & 15) != 0)
        return fail(GSR_ERR_ARG, "colors must be 16-byte aligned per frame");
    const Dims d = make_dims(B, P, width, height);
    GeomArena g;
    ImageArena im;
    BinArena bn;
    carve_workspace(workspace, d, R_capacity, &g, &im, &bn);
    Inputs in{};
    env_tuning(in);
    in.means3D = means3D; in.s_means = means_stride;
    in.scales = scales; in.s_scales = scales_stride;
    in.rot = rotations; in.s_rot = rot_stride;
    in.opac = opacities; in.s_opac = opac_stride;
    in.cov3D_pre = nullptr; in.s_cov = 0;
    in.colors = colors; in.s_colors = colors_stride;
    in.view = viewmatrices; in.proj = projmatrices;
    in.tan_dev = tanfov;
    in.bg = backgrounds; in.s_bg = bg_stride;
    in.scale_mod = scale_modifier;
    in.prefiltered = 0; in.antialiasing = antialiasing;
    in.fwd_only = (numerics & GSR_FORWARD_ONLY) != 0 || dg != nullptr;
    // recorded before any launch or early return: a workspace whose address the allocator reuses, or
    // whose forward failed partway, carries this forward's flag, not an older one
    note_workspace(workspace, in.fwd_only != 0);
    Outputs o{out_color, out_invdepth, radii, g_render_counters, g_timeline, g_timeline_cap};
    if (refine) {
        o.rb = refine->bias;
        o.out_refine = refine->out_refine;
        o.n_out = refine->n_out;
        o.keep = refine->keep_channels;
        o.slope = refine->negative_slope;
    }
    // a B = 1 workspace carries the quad-mask slab; the masks are computed only when the quad kernel
    // will read them
    if (!render_uses_quad(d, split_bf16(numerics), o)) bn.qmask = nullptr;
    // the control words are zeroed by the first kernel (zero_ctrl_words), except for a prefiltered
    // forward (its culling-error word is set during that kernel) or an empty one (no kernel)
    in.zero_ctrl = !in.prefiltered && d.P > 0 && d.B > 0;
    if (!in.zero_ctrl) HIP_TRY(hipMemsetAsync(g.ctrl, 0, ctrl_words(d) * 4, s));
    if (dg) {  // (forward-only: the deformed attributes are not kept, no backward can use the workspace)
        StageTimer st_(0, s);
        launch_deform_preprocess(d, in, g, o, *dg, s);
    } else {
        StageTimer st_(0, s);
        launch_preprocess(d, in, g, o, s);
    }
    if (d.B == 1) {  // (the frame totals in the depth sort's first kernel: launch_depth_sort)
        in.fuse_totals = 1;
        in.totals_cap = R_capacity;
    } else {
        StageTimer st_(1, s);
        launch_scan_blocksums(d, g, R_capacity, s);
    }
    int rc = run_binning_and_render(d, in, g, im, bn, o, numerics, 0, s);
    if (rc < 0) return rc;
    return 0;
}

int gsr_forward_batch_refine(int B, int P, int width, int height, const float* means3D,
                             int64_t means_stride, const float* colors, int64_t colors_stride,
                             const float* opacities, int64_t opac_stride, const float* scales,
                             int64_t scales_stride, const float* rotations, int64_t rot_stride,
                             float scale_modifier, const float* viewmatrices, const float* projmatrices,
                             const float* tanfov, const float* backgrounds, int64_t bg_stride,
                             char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                             int* radii, int antialiasing, const gsr_refine_epilogue* refine,
                             uint32_t numerics, void* stream) {
    return forward_batch_impl(B, P, width, height, means3D, means_stride, colors, colors_stride, opacities,
                              opac_stride, scales, scales_stride, rotations, rot_stride, scale_modifier,
                              viewmatrices, projmatrices, tanfov, backgrounds, bg_stride, workspace, R_capacity,
                              out_color, out_invdepth, radii, antialiasing, refine, numerics, nullptr,
                              (hipStream_t)stream);
}

int gsr_forward_batch_deformed(int B, int width, int height, const GsrDeformInputs* dg, const float* colors,
                               int64_t colors_stride, const float* opacities, int64_t opac_stride,
                               float scale_modifier, const float* viewmatrices, const float* projmatrices,
                               const float* tanfov, const float* backgrounds, int64_t bg_stride,
                               char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                               int* radii, int antialiasing, uint32_t numerics, void* stream) {
    if (!dg || dg->V < 0 || dg->N < 0 || dg->F < 0 || dg->V + dg->N == 0 || !dg->verts)
        return fail(GSR_ERR_ARG, "gsr_forward_batch_deformed: bad deform inputs");
    if (dg->V > 0 && (!dg->vert_transforms || !dg->vtx_rotations || !dg->vtx_scales))
        return fail(GSR_ERR_ARG, "gsr_forward_batch_deformed: vertex Gaussians need transforms, rotations, scales");
    if (dg->N > 0 && (!dg->faces || !dg->binding_face || !dg->face_bary || !dg->local_xyz || !dg->uv_rotations ||
                      !dg->uv_scales || dg->F == 0))
        return fail(GSR_ERR_ARG, "gsr_forward_batch_deformed: UV Gaussians need faces and binding data");
    auto bad_stride = [](int64_t st, int64_t full) { return st != 0 && st != full; };
    if (bad_stride(dg->vtx_rot_stride, 4LL * dg->V) || bad_stride(dg->vtx_scale_stride, 3LL * dg->V) ||
        bad_stride(dg->local_stride, 3LL * dg->N) || bad_stride(dg->uv_rot_stride, 4LL * dg->N) ||
        bad_stride(dg->uv_scale_stride, 3LL * dg->N))
        return fail(GSR_ERR_ARG, "gsr_forward_batch_deformed: strides must be 0 or a whole frame");
    return forward_batch_impl(B, dg->V + dg->N, width, height, nullptr, 0, colors, colors_stride, opacities,
                              opac_stride, nullptr, 0, nullptr, 0, scale_modifier, viewmatrices, projmatrices,
                              tanfov, backgrounds, bg_stride, workspace, R_capacity, out_color, out_invdepth, radii,
                              antialiasing, nullptr, numerics | GSR_FORWARD_ONLY, dg, (hipStream_t)stream);
}

int gsr_refine_prepare(int n, const float* rows, const float* weight, int n_out, int keep_channels,
                       float* prepared, void* stream) {
    if (n < 0 || !weight || n_out < 1 || keep_channels < 0 || keep_channels + n_out > GSR_C)
        return fail(GSR_ERR_ARG, "gsr_refine_prepare: need weight, n_out >= 1, keep + n_out <= 32");
    if (n == 0) return 0;
    if (!rows || !prepared || ((uintptr_t)rows & 15) != 0)
        return fail(GSR_ERR_ARG, "gsr_refine_prepare: rows must be 16-byte aligned, prepared non-null");
    launch_refine_prepare(n, rows, weight, n_out, keep_channels, prepared, (hipStream_t)stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GSR_ERR_HIP, std::string("refine_prepare: ") + hipGetErrorString(e));
    return 0;
}

static int backward_batch(int B, int P, int width, int height, const float* means3D, int64_t means_stride,
                          const float* colors, int64_t colors_stride, const float* opacities, int64_t opac_stride,
                          const float* scales, int64_t scales_stride, const float* rotations, int64_t rot_stride,
                          float scale_modifier, const float* viewmatrices, const float* projmatrices,
                          const float* tanfov, const float* backgrounds, int64_t bg_stride, char* workspace,
                          int64_t R_capacity, const Grads& grads, int antialiasing, uint32_t numerics,
                          hipStream_t s) {
    if (B <= 0 || P <= 0 || !workspace || !tanfov) return fail(GSR_ERR_ARG, "bad batch arguments");
    if (numerics & ~kNumericsKnown) return fail(GSR_ERR_ARG, "unknown numerics flags");
    if (P >= kMaxGaussians) return fail(GSR_ERR_ARG, "P must be < 2^24");
    if (workspace_fwd_only(workspace))
        return fail(GSR_ERR_ARG, "backward_batch: the workspace's last forward was GSR_FORWARD_ONLY (no backward rows)");
    const Dims d = make_dims(B, P, width, height);
    GeomArena g;
    ImageArena im;
    BinArena bn;
    carve_workspace(workspace, d, R_capacity, &g, &im, &bn);
    Inputs in{};
    env_tuning(in);
    in.means3D = means3D; in.s_means = means_stride;
    in.scales = scales; in.s_scales = scales_stride;
    in.rot = rotations; in.s_rot = rot_stride;
    in.opac = opacities; in.s_opac = opac_stride;
    in.colors = colors; in.s_colors = colors_stride;
    in.view = viewmatrices; in.proj = projmatrices;
    in.tan_dev = tanfov;
    in.bg = backgrounds; in.s_bg = bg_stride;
    in.scale_mod = scale_modifier;
    in.antialiasing = antialiasing;
    { StageTimer st_(7, s); launch_render_bwd(d, in, g, im, bn, grads, exact_exp(numerics), split_bf16(numerics), s); }
    { StageTimer st_(8, s); launch_preprocess_bwd(d, in, g, grads, s); }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GSR_ERR_HIP, std::string("backward_batch: ") + hipGetErrorString(e));
    return 0;
}

int gsr_backward_batch(int B, int P, int width, int height, const float* means3D,
                       int64_t means_stride, const float* colors, int64_t colors_stride,
                       const float* opacities, int64_t opac_stride, const float* scales,
                       int64_t scales_stride, const float* rotations, int64_t rot_stride,
                       float scale_modifier, const float* viewmatrices, const float* projmatrices,
                       const float* tanfov, const float* backgrounds, int64_t bg_stride,
                       char* workspace, int64_t R_capacity, const float* dL_dpix,
                       const float* dL_dinvdepth, float* dL_dmean2D, float* dL_dconic,
                       float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth_g,
                       float* dL_dmean3D, float* dL_dcov3D, float* dL_dscale, float* dL_drot,
                       int antialiasing, uint32_t numerics, void* stream) {
    if (!dL_dpix || !dL_dmean2D || !dL_dconic || !dL_dopacity || !dL_dcolor || !dL_dmean3D || !dL_dcov3D)
        return fail(GSR_ERR_ARG, "backward_batch: null gradient buffer");
    Grads gr{};
    gr.dL_dpix = dL_dpix;
    gr.dL_dinvdepth = dL_dinvdepth;
    gr.dL_dmean2D = dL_dmean2D;
    gr.dL_dconic = dL_dconic;
    gr.dL_dopacity = dL_dopacity;
    gr.dL_dcolors = dL_dcolor;
    gr.dL_dinvdepth_g = dL_dinvdepth ? dL_dinvdepth_g : nullptr;
    gr.invd = dL_dinvdepth != nullptr && dL_dinvdepth_g != nullptr;
    gr.dL_dmeans3D = dL_dmean3D;
    gr.dL_dcov3D = dL_dcov3D;
    gr.dL_dscale = dL_dscale;
    gr.dL_drot = dL_drot;
    return backward_batch(B, P, width, height, means3D, means_stride, colors, colors_stride, opacities,
                          opac_stride, scales, scales_stride, rotations, rot_stride, scale_modifier,
                          viewmatrices, projmatrices, tanfov, backgrounds, bg_stride, workspace, R_capacity, gr,
                          antialiasing, numerics, (hipStream_t)stream);
}

int gsr_backward_batch_shared(int B, int P, int width, int height, const float* means3D,
                              int64_t means_stride, const float* colors, int64_t colors_stride,
                              const float* opacities, int64_t opac_stride, const float* scales,
                              int64_t scales_stride, const float* rotations, int64_t rot_stride,
                              float scale_modifier, const float* viewmatrices, const float* projmatrices,
                              const float* tanfov, const float* backgrounds, int64_t bg_stride,
                              char* workspace, int64_t R_capacity, const float* dL_dpix,
                              const float* dL_dinvdepth, float* dL_dopacity, float* dL_dcolor,
                              float* dL_dmean3D, float* dL_dscale, float* dL_drot, int antialiasing,
                              uint32_t numerics, void* stream) {
    if (!dL_dpix || !dL_dopacity || !dL_dcolor || !dL_dmean3D || !dL_dscale || !dL_drot)
        return fail(GSR_ERR_ARG, "backward_batch_shared: null gradient buffer");
    if (!scales || !rotations) return fail(GSR_ERR_ARG, "backward_batch_shared: needs scales and rotations");
    Grads gr{};
    gr.dL_dpix = dL_dpix;
    gr.dL_dinvdepth = dL_dinvdepth;
    gr.invd = dL_dinvdepth != nullptr;
    gr.reduce = 1;
    gr.dL_dopacity = dL_dopacity;
    gr.dL_dcolors = dL_dcolor;
    gr.dL_dmeans3D = dL_dmean3D;
    gr.dL_dscale = dL_dscale;
    gr.dL_drot = dL_drot;
    return backward_batch(B, P, width, height, means3D, means_stride, colors, colors_stride, opacities,
                          opac_stride, scales, scales_stride, rotations, rot_stride, scale_modifier,
                          viewmatrices, projmatrices, tanfov, backgrounds, bg_stride, workspace, R_capacity, gr,
                          antialiasing, numerics, (hipStream_t)stream);
}

int gsr_render_counters(uint64_t* device_counters) {
    g_render_counters = device_counters;
    return 0;
}

int gsr_render_timeline(uint32_t* device_records, uint32_t capacity) {
    g_timeline = device_records;
    g_timeline_cap = device_records ? capacity : 0u;
    return 0;
}

int gsr_profile_enable(uint32_t stage_mask) {
    g_prof_mask = stage_mask;
    return 0;
}

int gsr_profile_read(double* ms, int* counts, int n) {
    for (size_t i = 0; i < g_ev_used; i++) {
        EvPair& e = g_ev_pool[i];
        HIP_TRY(hipEventSynchronize(e.b));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, e.a, e.b));
        g_prof_ms[e.stage] += t;
        g_prof_cnt[e.stage] += 1;
    }
    g_ev_used = 0;
    for (int i = 0; i < n && i < kStages; i++) {
        if (ms) ms[i] = g_prof_ms[i];
        if (counts) counts[i] = g_prof_cnt[i];
    }
    for (int i = 0; i < kStages; i++) { g_prof_ms[i] = 0; g_prof_cnt[i] = 0; }
    return 0;
}

int gsr_batch_status(const char* workspace, int B, int P, int64_t* R_total, int* overflow,
                     void* stream) {
    hipStream_t s = (hipStream_t)stream;
    uint32_t ctrl_h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(ctrl_h, workspace, sizeof(ctrl_h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    (void)B; (void)P;
    if (R_total) *R_total = ctrl_h[kCtrlRLo];
    if (overflow) *overflow = ctrl_h[kCtrlOverflow] ? 1 : 0;
    return 0;
}

int gsr_stream_create_cu_mask(uint32_t n_words, const uint32_t* cu_mask, void** stream_out) {
    if (!stream_out || !cu_mask || n_words == 0) return fail(GSR_ERR_ARG, "gsr_stream_create_cu_mask: bad arguments");
    int cus = 0;
    for (uint32_t i = 0; i < n_words; i++) cus += __builtin_popcount(cu_mask[i]);
    if (cus == 0) return fail(GSR_ERR_ARG, "gsr_stream_create_cu_mask: empty CU mask");
    hipStream_t st = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&st, n_words, cu_mask));
    {
        std::lock_guard<std::mutex> lk(g_cu_mu);
        g_stream_cus[st] = cus;
    }
    *stream_out = (void*)st;
    return 0;
}

int gsr_stream_destroy(void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!st) return 0;
    {
        std::lock_guard<std::mutex> lk(g_route_mu);
        for (auto it = g_routes.begin(); it != g_routes.end();) {
            if (it->first == st || it->second.render == st) {
                hipEventDestroy(it->second.ready);
                hipEventDestroy(it->second.done);
                it = g_routes.erase(it);
            } else {
                ++it;
            }
        }
    }
    {
        std::lock_guard<std::mutex> lk(g_cu_mu);
        g_stream_cus.erase(st);
    }
    HIP_TRY(hipStreamDestroy(st));
    return 0;
}

int gsr_set_render_stream(void* stream, void* render_stream) {
    hipStream_t st = (hipStream_t)stream, rs = (hipStream_t)render_stream;
    std::lock_guard<std::mutex> lk(g_route_mu);
    const auto it = g_routes.find(st);
    if (it != g_routes.end()) {
        hipEventDestroy(it->second.ready);
        hipEventDestroy(it->second.done);
        g_routes.erase(it);
    }
    if (!rs || rs == st) return 0;
    RenderRoute r{rs, nullptr, nullptr};
    HIP_TRY(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
    g_routes[st] = r;
    return 0;
}

}  // extern "C"
