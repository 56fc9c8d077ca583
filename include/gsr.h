/*
 * gsr.h -- C ABI of the MI355X (gfx950) 32-channel Gaussian-splat rasterizer.
 *
 * Drop-in boundary for GUAVA's diff-gaussian-rasterization-32.  Each entry point replaces one
 * function of the reference's native layer
 * (/root/reference/submodules/diff-gaussian-rasterization-32/):
 *
 *   gsr_forward      <- CudaRasterizer::Rasterizer::forward     cuda_rasterizer/rasterizer.h:31-61
 *                       (driver: cuda_rasterizer/rasterizer_impl.cu:198-341)
 *   gsr_backward     <- CudaRasterizer::Rasterizer::backward    cuda_rasterizer/rasterizer.h:63-91
 *                       (driver: cuda_rasterizer/rasterizer_impl.cu:345-450)
 *   gsr_mark_visible <- CudaRasterizer::Rasterizer::markVisible cuda_rasterizer/rasterizer.h:24-29
 *                       (kernel: rasterizer_impl.cu:54-66)
 *   gsr_forward_batch / gsr_backward_batch: B frames in one launch set with a preallocated
 *                       workspace and no host synchronisation (replaces the per-frame Python loop
 *                       of models/UbodyAvatar/gaussian_render.py:37-67).
 *
 * Conventions: every pointer is a device pointer (HBM) unless stated; float32 everywhere; the
 * layouts are the reference's (means3D [P,3], rotations [P,4] wxyz, colors [P,32], viewmatrix /
 * projmatrix 4x4 column-major as produced by utils/graphics_utils.py:44-50, out_color [32,H,W]).
 * `stream` is a hipStream_t (NULL = default stream).  Return codes: >= 0 success (forward:
 * num_rendered), < 0 = -gsr_status; gsr_last_error() returns a message for the last failure.
 */
#ifndef GSR_H
#define GSR_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_NUM_CHANNELS 32
#define GSR_BLOCK_X 16
#define GSR_BLOCK_Y 16

typedef enum {
    GSR_OK = 0,
    GSR_ERR_ARG = 1,          /* invalid argument / shape */
    GSR_ERR_HIP = 2,          /* HIP runtime error (message in gsr_last_error) */
    GSR_ERR_PREFILTERED = 3,  /* prefiltered=true and a point was culled (reference: __trap) */
    GSR_ERR_NO_COLORS = 4,    /* colors_precomp missing with 32 channels (rasterizer_impl.cu:244-247) */
    GSR_ERR_CAPACITY = 5,     /* batch: instances exceed the workspace's R capacity */
    GSR_ERR_ALLOC = 6         /* allocator callback returned NULL */
} gsr_status;

/* Mirrors the reference's std::function<char*(size_t)> buffer resizers (rasterize_points.cu:27-33):
 * must return a device buffer of at least `bytes` bytes that stays alive until backward. */
typedef char* (*gsr_alloc_fn)(void* ctx, size_t bytes);

const char* gsr_version(void);
const char* gsr_last_error(void);

/* Numerics of ONE call (bit flags, the `numerics` argument of the *_ex / async / batch entry points;
 * there is no process-wide mode).  GSR_NUMERICS_EXACT (0) is what the reference-signature entry
 * points gsr_forward / gsr_backward use: bit-identical to the CPU oracle.
 *   GSR_NUMERICS_FAST_EXP: the blend exponent on the hardware v_exp_f32 instead of the
 *     deterministic polynomial (alpha thresholds can flip on rare pixels).
 *   GSR_NUMERICS_SPLIT_BF16: colour accumulation of the forward blend as split-bf16 MFMAs
 *     (f = f_hi + f_lo, four exact bf16 products per feature x weight, f32 accumulation):
 *     <= 3e-5 relative per product, colour L-inf within the north_star's 1e-4; final_T,
 *     n_contrib and inverse depth stay bit-exact.  In the backward the same flag puts the two
 *     contractions (g = f . dL/dpixel, dL/dcolor = sum_px w dL/dpixel) on split-bf16 MFMAs;
 *     gradients stay within 1e-4 of their scale.  No reference counterpart (forward.cu:371-372
 *     accumulates in f32).
 * Unknown bits are rejected (GSR_ERR_ARG). */
#define GSR_NUMERICS_EXACT 0u
#define GSR_NUMERICS_FAST_EXP 1u
#define GSR_NUMERICS_SPLIT_BF16 2u
/* Not numerics, in the same flag word of gsr_forward_batch / gsr_forward_batch_refine:
 * GSR_FORWARD_ONLY -- no backward will read this call's workspace (inference: main/test.py,
 * render_motion.py).  Preprocess then writes only what binning and compositing read (depth, render
 * record, tile rect and count; plus the caller's radii) and skips the rows kept for the backward
 * (cov3D, means2D, conic, inverse depth, radii in the workspace): 56 of 108 bytes per visible
 * Gaussian.  Images are unchanged.  A gsr_backward_batch* on a workspace whose last forward was
 * forward-only fails with GSR_ERR_ARG (the library records it per workspace pointer on the host;
 * the kernels also skip such a workspace, so nothing is computed either way). */
#define GSR_FORWARD_ONLY 0x100u

/* Scratch sizes used by gsr_forward (the three resizer requests).  Unlike the reference's
 * GeometryState, the geometry arena also holds the per-frame depth sort and the (depth chunk x tile)
 * instance-count table, so it depends on the image size too.  Images are limited to 16384 tiles
 * (2048 x 2048 pixels). */
size_t gsr_geometry_bytes(int P, int width, int height);
size_t gsr_image_bytes(int width, int height);
size_t gsr_binning_bytes(int64_t R);

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/* Rasterizer::forward.  D, M, shs, cam_pos are accepted for signature parity (32 channels need
 * colors_precomp, as in the reference).  out_color [32,H,W], depth = inverse-depth image [H,W]
 * (may be NULL), radii [P] (may be NULL).  Returns num_rendered or -status. */
int gsr_forward(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                const float* means3D, const float* shs, const float* colors_precomp,
                const float* opacities, const float* scales, float scale_modifier,
                const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                int debug, void* stream);
/* gsr_forward with explicit per-call numerics (GSR_NUMERICS_*). */
int gsr_forward_ex(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                   void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                   const float* means3D, const float* shs, const float* colors_precomp,
                   const float* opacities, const float* scales, float scale_modifier,
                   const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                   const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                   int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                   int debug, uint32_t numerics, void* stream);

/* gsr_forward without the host synchronisation after the scan (the reference reads num_rendered
 * back before sizing the binning buffer, rasterizer_impl.cu:279-291 of the reference driver):
 * the binning buffer is requested at the upper bound gsr_forward_async_bound(P, W, H) = P x tiles
 * instances (4 B each; every Gaussian in every tile), so every later launch is queued at once.
 * status_host (4 uint32, host-visible, e.g. pinned) receives {num_rendered, overflow, error bits,
 * 0} at the end of the stream's work: read it after synchronising (error bit 0 = a culled point
 * with prefiltered set, the reference's trap; overflow only if the bound hit 2^31 - 1).  Returns
 * 0 or -status.  debug must be 0.  status_host may be NULL when prefiltered is 0 (no error is then
 * possible and num_rendered is not wanted, e.g. inference): nothing is copied back. */
int64_t gsr_forward_async_bound(int P, int width, int height);
int gsr_forward_async(gsr_alloc_fn geometryBuffer, gsr_alloc_fn binningBuffer, gsr_alloc_fn imageBuffer,
                      void* alloc_ctx, int P, int D, int M, const float* background, int width, int height,
                      const float* means3D, const float* shs, const float* colors_precomp,
                      const float* opacities, const float* scales, float scale_modifier,
                      const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                      const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                      int prefiltered, float* out_color, float* depth, int antialiasing, int* radii,
                      int debug, uint32_t* status_host, uint32_t numerics, void* stream);

/* Preallocated scratch for the three gsr_alloc_fn resizers: pass gsr_scratch_geometry /
 * gsr_scratch_binning / gsr_scratch_image as the callbacks and a gsr_scratch* as alloc_ctx; each
 * returns its buffer when `bytes` fits its capacity and NULL otherwise (the call then fails with
 * GSR_ERR_ALLOC).  No host callback runs during the forward (a caller keeps one scratch per stream). */
typedef struct {
    char* geometry; size_t geometry_cap;
    char* binning; size_t binning_cap;
    char* image; size_t image_cap;
} gsr_scratch;
char* gsr_scratch_geometry(void* scratch, size_t bytes);
char* gsr_scratch_binning(void* scratch, size_t bytes);
char* gsr_scratch_image(void* scratch, size_t bytes);

/* Rasterizer::backward.  Gradient buffers are accumulated into and must be zeroed by the caller
 * (the reference's torch::zeros, rasterize_points.cu:163-179): dL_dmean2D [P,3], dL_dconic [P,4],
 * dL_dopacity [P], dL_dcolor [P,32], dL_dinvdepth [P] (NULL when dL_invdepths is NULL),
 * dL_dmean3D [P,3], dL_dcov3D [P,6], dL_dscale [P,3], dL_drot [P,4]; dL_dsh is unused (no SH
 * path with 32 channels). */
int gsr_backward(int P, int D, int M, int R, const float* background, int width, int height,
                 const float* means3D, const float* shs, const float* colors_precomp,
                 const float* opacities, const float* scales, float scale_modifier,
                 const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                 const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                 const int* radii, char* geom_buffer, char* binning_buffer, char* image_buffer,
                 const float* dL_dpix, const float* dL_invdepths, float* dL_dmean2D,
                 float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth,
                 float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                 float* dL_drot, int antialiasing, int debug, void* stream);
/* gsr_backward with explicit per-call numerics (GSR_NUMERICS_*). */
int gsr_backward_ex(int P, int D, int M, int R, const float* background, int width, int height,
                    const float* means3D, const float* shs, const float* colors_precomp,
                    const float* opacities, const float* scales, float scale_modifier,
                    const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                    const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                    const int* radii, char* geom_buffer, char* binning_buffer, char* image_buffer,
                    const float* dL_dpix, const float* dL_invdepths, float* dL_dmean2D,
                    float* dL_dconic, float* dL_dopacity, float* dL_dcolor, float* dL_dinvdepth,
                    float* dL_dmean3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscale,
                    float* dL_drot, int antialiasing, int debug, uint32_t numerics, void* stream);

/* ---- batched multi-frame path (B frames, one launch per stage, capture-safe) ----
 * Per-frame inputs use an element stride between frames (0 = shared by every frame).
 * viewmatrices/projmatrices: [B,16]; tanfov: [B,2] (x,y); backgrounds: [B,32] with bg_stride.
 * workspace: gsr_batch_workspace_bytes(B,P,W,H,R_capacity) bytes of device memory, reused by
 * gsr_backward_batch.  Outputs: out_color [B,32,H,W], out_invdepth [B,H,W] (or NULL),
 * radii [B,P] (or NULL).  P < 2^24.  No host synchronisation: call gsr_batch_status() to learn R
 * and whether the capacity overflowed (then every output pixel of the call is NaN and the
 * workspace's sticky overflow word is set, gsr_batch_status_offset). */
size_t gsr_batch_workspace_bytes(int B, int P, int width, int height, int64_t R_capacity);
int gsr_forward_batch(int B, int P, int width, int height, const float* means3D,
                      int64_t means_stride, const float* colors, int64_t colors_stride,
                      const float* opacities, int64_t opac_stride, const float* scales,
                      int64_t scales_stride, const float* rotations, int64_t rot_stride,
                      float scale_modifier, const float* viewmatrices, const float* projmatrices,
                      const float* tanfov, const float* backgrounds, int64_t bg_stride,
                      char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                      int* radii, int antialiasing, uint32_t numerics, void* stream);
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
                       int antialiasing, uint32_t numerics, void* stream);

/* gsr_backward_batch for Gaussian attributes SHARED by the B frames (one avatar seen from B
 * cameras, the training batch of main/trainer.py:82-102): the attribute gradients come back summed
 * over the frames, [P,k], with no per-frame [B,P,k] buffers (the reference's autograd sums the
 * per-frame gradients of the shared leaves).  dL_dcolor [P,32] is ACCUMULATED into (zero it);
 * dL_dopacity [P], dL_dmean3D [P,3], dL_dscale [P,3], dL_drot [P,4] are written.  Each Gaussian's
 * frames are summed in frame order.  Not bitwise reproducible run to run: dL_dcolor and each
 * frame's screen-space gradient row (dL/dmean2D, conic, opacity, inverse depth, from which the
 * mean3D / opacity / scale / rotation gradients follow) are accumulated with float atomics across
 * strips and tiles, as the reference's backward accumulates them with atomicAdd. */
int gsr_backward_batch_shared(int B, int P, int width, int height, const float* means3D,
                              int64_t means_stride, const float* colors, int64_t colors_stride,
                              const float* opacities, int64_t opac_stride, const float* scales,
                              int64_t scales_stride, const float* rotations, int64_t rot_stride,
                              float scale_modifier, const float* viewmatrices, const float* projmatrices,
                              const float* tanfov, const float* backgrounds, int64_t bg_stride,
                              char* workspace, int64_t R_capacity, const float* dL_dpix,
                              const float* dL_dinvdepth, float* dL_dopacity, float* dL_dcolor,
                              float* dL_dmean3D, float* dL_dscale, float* dL_drot, int antialiasing,
                              uint32_t numerics, void* stream);
/* Refiner-head epilogue: GaussianRenderer feeds the 32-channel render to the
 * StyleUNet refiner (gaussian_render.py:73), whose first layer is a 1x1 conv 32 -> 16 + leaky ReLU
 * (styleunet.py:110,178).  The conv is linear in the features, so it commutes with compositing:
 *   W.(sum_g f_g alpha_g T_g + T bg) = sum_g (W.f_g) alpha_g T_g + T (W.bg).
 * gsr_refine_prepare turns each 32-float row (a Gaussian's features, or a frame's background) into
 *   [f_0 .. f_{keep-1}, W.f (n_out values), 0 ...]
 * and gsr_forward_batch_refine, given prepared colors AND prepared backgrounds, composites those rows
 * with the unchanged blend kernel and finishes in the epilogue:
 *   out_color[b][c]   = channel c           for c < keep_channels (raw renders; GaussianRenderer
 *                                            keeps 0-2 as raw_renders, 3 as extra_renders,
 *                                            gaussian_render.py:71,83); other channels unwritten
 *   out_refine[b][o]  = leaky_relu(channel keep+o + bias[o], negative_slope),  o < n_out
 * so the 33-channel feature image is never written nor re-read.  Forward-only (inference:
 * main/test.py, render_motion.py); keep_channels + n_out <= 32. */
typedef struct {
    const float* weight;   /* [n_out][32] (Conv2d weight [n_out,32,1,1]); used by gsr_refine_prepare */
    const float* bias;     /* [n_out] or NULL */
    int n_out;             /* >= 1 */
    float negative_slope;  /* 0.2 in StyleUNet */
    float* out_refine;     /* [B][n_out][H][W] */
    int keep_channels;     /* raw channels of out_color still written */
} gsr_refine_epilogue;
/* rows [n,32] (16-byte aligned) -> prepared [n,32]. */
int gsr_refine_prepare(int n, const float* rows, const float* weight, int n_out, int keep_channels,
                       float* prepared, void* stream);
int gsr_forward_batch_refine(int B, int P, int width, int height, const float* means3D,
                             int64_t means_stride, const float* colors, int64_t colors_stride,
                             const float* opacities, int64_t opac_stride, const float* scales,
                             int64_t scales_stride, const float* rotations, int64_t rot_stride,
                             float scale_modifier, const float* viewmatrices, const float* projmatrices,
                             const float* tanfov, const float* backgrounds, int64_t bg_stride,
                             char* workspace, int64_t R_capacity, float* out_color, float* out_invdepth,
                             int* radii, int antialiasing, const gsr_refine_epilogue* refine,
                             uint32_t numerics, void* stream);
/* Stage timing with HIP events recorded on the launch stream around each stage whose bit is set in
 * `stage_mask` (bit i = stage i: 0 preprocess, 1 block scan, 2 depth sort, 3 chunk count,
 * 4 tile scan, 5 ordered scatter, 6 render fwd, 7 render bwd, 8 preprocess bwd); 0 disables.
 * gsr_profile_read synchronises the recorded events, writes the summed milliseconds and launch
 * counts of the first `n` stages and resets the accumulators. */
#define GSR_NUM_STAGES 9
int gsr_profile_enable(uint32_t stage_mask);
int gsr_profile_read(double* ms, int* counts, int n);
/* Work counters for the roofline report.  When `device_counters` is non-NULL, later forward calls run
 * an instrumented render kernel (same results, slower) that atomically adds into 8 uint64 device
 * words: [0] (pixel, Gaussian) pairs evaluated by the reference's per-pixel loop (sum over pixels
 * of the list positions visited before the pixel finished: n_contrib, or the terminating
 * position, or the whole list), [1] pairs that contributed (alpha >= 1/255, before termination),
 * [2] (wave strip, Gaussian) pairs blended after the per-wave cull, [3] MFMA k-steps issued per
 * wave, [4] Gaussians staged (list entries loaded into LDS), [5] list entries of all tiles,
 * [6] tiles rendered, [7] k-steps in which no pixel of the wave took either Gaussian.  NULL
 * restores the production kernel. */
int gsr_render_counters(uint64_t* device_counters);
/* Work-item timeline of the render kernel (a lightly instrumented variant runs while set):
 * record i (4 uint32: start, end in 100 MHz ticks, MFMA k-steps, XCD) for the first `capacity`
 * work items in longest-first order (strip items first, 4 per non-empty tile).  Single-frame quad
 * waves: (start, end, steps | refills << 16, list entries walked); with capacity | 0x80000000 they
 * also write, after the `capacity` records, 4 uint32 of core-clock sums per item (operand issue,
 * next-step alpha, blend + MFMA), so the buffer must then hold 8 x capacity words. */
int gsr_render_timeline(uint32_t* device_records, uint32_t capacity);

/* Byte offset, inside a batch workspace, of its 4 sticky status words (uint32): [0] = 1 once any
 * gsr_forward_batch* on it overflowed the R capacity (that call's frames are NaN), [1] = the largest
 * batch instance count R seen.  Calls never reset them (the per-call control words are reset);
 * the owner zeroes them when it allocates the workspace and after it has read an overflow, and may
 * copy them to host memory asynchronously after each call to notice an overflow without a
 * synchronisation.  No reference counterpart (the reference sizes the binning buffer after a
 * host synchronisation, rasterizer_impl.cu:284-288). */
size_t gsr_batch_status_offset(int B, int P, int width, int height, int64_t R_capacity);
/* Synchronises `stream`; writes the batch's instance count and overflow flag. */
int gsr_batch_status(const char* workspace, int B, int P, int64_t* R_total, int* overflow,
                     void* stream);

/* Consumer-side frame encoding for the multi-GPU frame exchange: the first
 * `channels` planes of B frames [.., H, W] (frame i at src + i * frame_stride floats) ->
 * dst [B][channels][H][W] uint8 = (uint8)(255 * clip(x, 0, 1)), GUAVA's to8b
 * (utils/general_utils.py:316-317, applied to every rendered frame at main/test.py:85); NaN -> 0. */
int gsr_frames_to8b(int B, int channels, int height, int width, const float* src, int64_t frame_stride,
                    uint8_t* dst, void* stream);

/* Placement of the compositing kernel (no reference counterpart; the reference runs every stage on
 * one stream).  gsr_stream_create_cu_mask makes a HIP stream whose kernels run only on the CUs set
 * in cu_mask (n_words 32-bit words, bit i = CU i; hipExtStreamCreateWithCUMask); persistent render
 * grids launched on it are sized to those CUs.  gsr_set_render_stream(stream, render_stream): batched
 * and single-frame forwards enqueued on `stream` launch their compositing kernel on render_stream,
 * after the binning on `stream` (event) and before `stream`'s later work (event), so the call stays
 * stream-ordered for its caller; render_stream NULL (or == stream) removes the routing.
 * gsr_stream_destroy removes the stream's routes and destroys it. */
int gsr_stream_create_cu_mask(uint32_t n_words, const uint32_t* cu_mask, void** stream_out);
int gsr_stream_destroy(void* stream);
int gsr_set_render_stream(void* stream, void* render_stream);

#ifdef __cplusplus
}
#endif
#endif
