/*
 * gsr_ssim.h -- C ABI of the MI355X (gfx950) fused SSIM (BASELINE config 4).
 *
 * Replaces the reference's fused-ssim CUDA extension (/root/reference/submodules/fused-ssim/):
 *   gsr_fused_ssim          <- fusedssim()          ssim.cu:368-404 (kernel fusedssimCUDA :187-286)
 *   gsr_fused_ssim_backward <- fusedssim_backward() ssim.cu:406-444 (kernel :288-366)
 *   gsr_image_loss          <- the L1 terms of the training loss and their gradient (utils/loss_utils.py)
 * Python front-end with the reference's API (FusedSSIMMap, fused_ssim): guava_renderer_amd/fused_ssim.
 *
 * Images are [B, CH, H, W] float32 device arrays (contiguous).  The 11x11 Gaussian window
 * (sigma 1.5) uses "same" zero padding; "valid" is a crop done by the caller as in the reference
 * (fused_ssim/__init__.py:14-15, :29-31).  C1 = 0.01^2, C2 = 0.03^2 in the reference.
 * Return codes: 0 = success, < 0 = -gsr_status (gsr_last_error()).
 */
#ifndef GSR_SSIM_H
#define GSR_SSIM_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ssim_map [B,CH,H,W]; dm_dmu1 / dm_dsigma1_sq / dm_dsigma12 [B,CH,H,W] all non-NULL (train) or
 * all NULL (inference). */
int gsr_fused_ssim(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                   float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, void* stream);

/* dL_dimg1 [B,CH,H,W] (written, not accumulated) from dL_dmap and the forward's partial maps. */
int gsr_fused_ssim_backward(int B, int CH, int H, int W, float C1, float C2, const float* img1,
                            const float* img2, const float* dL_dmap, const float* dm_dmu1,
                            const float* dm_dsigma1_sq, const float* dm_dsigma12, float* dL_dimg1,
                            void* stream);

/* The training step's image loss apart from SSIM, one pass over the rendered features
 * (SplatTrainer, guava_renderer_amd/train.py; the reference's Optimization_Loss terms
 * utils/loss_utils.py:92,116-119 on `renders` and `raw_renders`):
 *   loss = l1_weight * mean|feat[:, :3] - target| + refine_weight * mean|W . feat - target|
 * with W [3,32] the refined image's 1x1 head (NULL: no refine term) and both means over B*3*H*W.
 * Writes dL_dfeat [B,32,H,W] = d loss / d feat + (channels 0-2) extra_grad [B,3,H,W] (e.g. the SSIM
 * term's gradient; may be NULL), and per-workgroup loss partial sums into loss_partials
 * [gsr_image_loss_partials(B,H,W)] (sum them for the loss; fixed order, deterministic).
 * feat, target, extra_grad contiguous float32. */
int gsr_image_loss_partials(int B, int H, int W);
int gsr_image_loss(int B, int H, int W, const float* feat, const float* target, const float* refine_w,
                   float l1_weight, float refine_weight, const float* extra_grad, float* dL_dfeat,
                   float* loss_partials, void* stream);

#ifdef __cplusplus
}
#endif
#endif
