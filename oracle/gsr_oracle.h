/*
 * gsr_oracle.h -- CPU restatement of the 32-channel Gaussian-splat rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker.  The product path (guava_renderer_amd / libgsr.so) never calls it.
 *
 * Follows, line by line, the reference in
 *   /root/reference/submodules/diff-gaussian-rasterization-32/cuda_rasterizer/
 *     forward.cu:74-148 (computeCov2D, computeCov3D), :151-269 (preprocessCUDA),
 *     :274-397 (renderCUDA fwd), backward.cu:147-326 (computeCov2DCUDA),
 *     :330-393 (computeCov3D bwd), :398-449 (preprocessCUDA bwd),
 *     :452-638 (renderCUDA bwd), rasterizer_impl.cu:35-50 (getHigherMsb),
 *     :54-66 (checkFrustum), :70-111 (duplicateWithKeys), :116-138
 *     (identifyTileRanges), :198-341 (forward driver), :345-450 (backward),
 *     auxiliary.h:40-176 (ndc2Pix, getRect, transforms, in_frustum).
 *
 * Evaluation order.  The reference is compiled by nvcc with FMA contraction
 * on, so its last-ulp rounding is not knowable without running it.  This
 * restatement fixes one IEEE evaluation order (documented in DESIGN.md
 * "Numerics contract"), which the HIP kernels implement identically:
 *   - preprocess (fwd): every expression left-to-right as written in the
 *     reference, glm mat3 products in glm's summation order, ndc2Pix in
 *     double, no contraction (built with -ffp-contract=off);
 *   - blend: power = fma(dy, fma(Cc,dy, Bb*dx), (A*dx)*dx) with A=-cx/2,
 *     Bb=-cy, Cc=-cz/2; accumulate C = fma(f, alpha*T, C);
 *   - exp: gsr_expf (Cody-Waite + degree-6 polynomial, pure fma/mul/add,
 *     bit-reproducible on CPU and GPU) in "exact" mode.
 * Parity status: the reference ships no tests or golden vectors for this
 * path and its CUDA build cannot run here, so the rasterizer
 * restatement is "parity unpinned" against reference outputs; it is pinned
 * by analytic known-answer cases and an independent float64 torch dense
 * restatement (tests/test_oracle.py).
 */
#ifndef GSR_ORACLE_H
#define GSR_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#define GSRO_C 32
#define GSRO_BX 16
#define GSRO_BY 16

#ifdef __cplusplus
extern "C" {
#endif

/* Deterministic exp used by both the oracle and the HIP kernels ("exact" mode). */
float gsro_expf(float x);
/* the blend's alpha = min(0.99, o exp(x)) and exp(x) (gsr_oracle.c: blend_parts) */
float gsro_blend_alpha(float o, float x, int exact);
float gsro_blend_G(float x, int exact);

/* markVisible: rasterizer_impl.cu:54-66 / auxiliary.h:151-176 (prefiltered=false). */
void gsro_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present);

/* preprocessCUDA (forward.cu:151-269).  Returns 0, or -1 if prefiltered and a point was culled
 * (the reference __trap()s there).  cov3D_precomp may be NULL (then scales/rot used). */
int gsro_preprocess(int P, const float* means3D, const float* scales, float scale_mod,
                    const float* rot, const float* opac, const float* cov3D_precomp,
                    const float* view, const float* proj, int W, int H,
                    float tanx, float tany, int prefiltered, int antialiasing,
                    int* radii, float* means2D, float* depths, float* cov3D,
                    float* conic_opacity, uint32_t* tiles_touched);

/* InclusiveSum + duplicateWithKeys + stable radix sort + identifyTileRanges
 * (rasterizer_impl.cu:280-320).  point_offsets[P]; point_list[R]; ranges[2*T]
 * (T = ceil(W/16)*ceil(H/16)).  Returns R. */
int64_t gsro_bin(int P, int W, int H, const int* radii, const float* means2D, const float* depths,
                 const uint32_t* tiles_touched, uint32_t* point_offsets,
                 uint32_t* point_list, uint64_t* point_keys, uint32_t* ranges, int64_t R_cap);

/* renderCUDA fwd (forward.cu:274-397).  exact_exp selects the blend arithmetic: 1 the bit-reproducible
 * restatement (gsro_blend_alpha), 0 the same with libm expf, 2 the reference's expressions as written
 * with libm expf (gsr_oracle.c, "Blend arithmetic modes").
 * out_color[C*H*W], out_invdepth[H*W] (may be NULL), final_T[H*W], n_contrib[H*W]. */
void gsro_render(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                 const float* means2D, const float* colors, const float* conic_opacity,
                 const float* depths, const float* bg, int exact_exp,
                 float* out_color, float* out_invdepth, float* final_T, uint32_t* n_contrib);

/* renderCUDA bwd (backward.cu:452-638).  Gradient buffers must be zeroed by the caller.
 * dL_dinvdepth_pix / dL_dinvdepth_g may be NULL (the "no invdepth grad" path).
 * dL_dmean2D[3P], dL_dconic[4P], dL_dopacity[P], dL_dcolors[C*P], dL_dinvdepth_g[P]. */
void gsro_render_counts(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                        const float* means2D, const float* conic_opacity, int exact_exp,
                        uint64_t* out);
/* Pixels whose take/stop decisions differ between two blend modes (test only): exact_exp = 1 and
 * libm expf, or any two of the modes 0 / 1 / 2 (gsr_oracle.c: GSRO_RESTATED, _LIBM_EXP, _LITERAL). */
uint64_t gsro_render_decision_flips_modes(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                                          const float* means2D, const float* conic_opacity, int mode_a,
                                          int mode_b, uint8_t* flags);
uint64_t gsro_render_decision_flips(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                                    const float* means2D, const float* conic_opacity, uint8_t* flags);
/* Accumulation order of gsro_render_backward (test only): 0 forward, 1 tiles and pixels reversed. */
void gsro_set_backward_order(int reverse);
void gsro_render_backward(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                          const float* bg, const float* means2D, const float* conic_opacity,
                          const float* colors, const float* depths, const float* final_T,
                          const uint32_t* n_contrib, const float* dL_dpix,
                          const float* dL_dinvdepth_pix, int exact_exp,
                          float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                          float* dL_dcolors, float* dL_dinvdepth_g);

/* computeCov2DCUDA + preprocessCUDA bwd (backward.cu:147-326, 330-393, 398-449).
 * dL_dopacity is read-modify-written (AA branch).  dL_dinvdepth_g may be NULL.
 * scales/rot may be NULL when cov3D_precomp was used (then no scale/rot grads).
 * dL_dmeans3D[3P], dL_dcov3D[6P], dL_dscale[3P], dL_drot[4P] zeroed by caller. */
void gsro_preprocess_backward(int P, int W, int H, const float* means3D, const int* radii,
                              const float* scales, float scale_mod, const float* rot,
                              const float* opac, const float* cov3D, const float* view,
                              const float* proj, float tanx, float tany,
                              const float* dL_dmean2D, const float* dL_dconic,
                              const float* dL_dinvdepth_g, int antialiasing,
                              float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                              float* dL_dscale, float* dL_drot);

/* Thread count used by the parallel loops (OpenMP); <=0 means OMP default. */
void gsro_set_threads(int n);
int gsro_get_threads(void);

#ifdef __cplusplus
}
#endif
#endif
