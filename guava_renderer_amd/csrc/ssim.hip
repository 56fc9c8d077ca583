// ssim.hip -- fused SSIM forward / backward for gfx950 (include/gsr_ssim.h).
//
// Reference: submodules/fused-ssim/ssim.cu:187-286 (fusedssimCUDA), :288-366 (backward),
// fused_ssim/__init__.py:8-41.  Same math: 11-tap separable Gaussian (sigma 1.5, the reference's
// G_00..G_10 constants), zero padding of 5, per pixel and channel
//   mu1, mu2, sigma1^2 = G*(x1^2) - mu1^2, sigma2^2, sigma12 = G*(x1 x2) - mu1 mu2
//   map = (2 mu1 mu2 + C1)(2 sigma12 + C2) / ((mu1^2 + mu2^2 + C1)(sigma1^2 + sigma2^2 + C2))
// plus, in training, the three partials dmap/dmu1, dmap/dsigma1^2, dmap/dsigma12 that the backward
// turns into dL/dimg1 = G*(dL dm_dmu1) + 2 x1 G*(dL dm_dsigma1^2) + x2 G*(dL dm_dsigma12).
//
// Structure (unlike the reference's five separate convolution passes with ~20 block barriers per
// channel): one 32x32 output tile per 256-thread workgroup; per channel the two 42x42 input tiles are
// staged in LDS once, ONE horizontal pass produces all five (forward) or three (backward) filtered
// quantities into LDS, and ONE vertical pass finishes them, each thread owning a 4-pixel column
// segment (a 14-row sliding window per quantity).  Three barriers per channel.  Loads and stores are
// row-contiguous (coalesced); the kernel is HBM/LDS-bound: per pixel and channel the forward reads
// 8 bytes and writes 16 (4 with train = false), the backward reads 24 and writes 4.
#include "../../include/gsr.h"
#include "../../include/gsr_ssim.h"
#include "gsr_internal.h"

namespace gsr {

constexpr int kSX = 32, kSY = 32;          // output tile
constexpr int kHX = kSX + 10, kHY = kSY + 10;  // with the 5-pixel halo
constexpr int kLdsPitch = kHX + 1;         // odd pitch: column walks hit distinct banks
constexpr int kRowsPerThread = 4;          // vertical pass: 256 threads = 32 columns x 8 segments

__constant__ float kG[11] = {0.001028380123898387f, 0.0075987582094967365f, 0.036000773310661316f,
                             0.10936068743467331f,  0.21300552785396576f,   0.26601171493530273f,
                             0.21300552785396576f,  0.10936068743467331f,   0.036000773310661316f,
                             0.0075987582094967365f, 0.001028380123898387f};

// stage a (kHY x kHX) halo tile of channel plane `src` (zero outside the image) into LDS
__device__ __forceinline__ void stage(float (*dst)[kLdsPitch], const float* __restrict__ src, int H, int W,
                                      int y0, int x0) {
    for (int i = threadIdx.x; i < kHY * kHX; i += blockDim.x) {
        const int ly = i / kHX, lx = i - ly * kHX;
        const int y = y0 - 5 + ly, x = x0 - 5 + lx;
        dst[ly][lx] = (y >= 0 && y < H && x >= 0 && x < W) ? src[(int64_t)y * W + x] : 0.0f;
    }
}

template <int NQ>
__device__ __forceinline__ void vertical(const float (*hx)[kHY][kSX + 1], int cx, int ry, float out[NQ][kRowsPerThread]) {
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        float win[kRowsPerThread + 10];
#pragma unroll
        for (int k = 0; k < kRowsPerThread + 10; k++) win[k] = hx[q][ry + k][cx];
#pragma unroll
        for (int r = 0; r < kRowsPerThread; r++) {
            float v = 0.0f;
#pragma unroll
            for (int k = 0; k < 11; k++) v = fmaf(kG[k], win[r + k], v);
            out[q][r] = v;
        }
    }
}

__global__ __launch_bounds__(256) void k_ssim_fwd(int CH, int H, int W, float C1, float C2,
                                                  const float* __restrict__ img1,
                                                  const float* __restrict__ img2,
                                                  float* __restrict__ map, float* __restrict__ dmu1,
                                                  float* __restrict__ ds1, float* __restrict__ ds12) {
    __shared__ float t1[kHY][kLdsPitch];
    __shared__ float t2[kHY][kLdsPitch];
    __shared__ float hx[5][kHY][kSX + 1];
    const int x0 = blockIdx.x * kSX, y0 = blockIdx.y * kSY, b = blockIdx.z;
    const int cx = threadIdx.x & 31, ry = (threadIdx.x >> 5) * kRowsPerThread;
    const int64_t plane = (int64_t)H * W;
    for (int c = 0; c < CH; c++) {
        const int64_t base = ((int64_t)b * CH + c) * plane;
        stage(t1, img1 + base, H, W, y0, x0);
        stage(t2, img2 + base, H, W, y0, x0);
        __syncthreads();
        // horizontal pass: x1, x1^2, x2, x2^2, x1 x2 over all kHY rows of the tile's 32 columns
        for (int i = threadIdx.x; i < kHY * kSX; i += blockDim.x) {
            const int ly = i >> 5, lx = i & 31;
            float a = 0.f, a2 = 0.f, bb = 0.f, b2 = 0.f, ab = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) {
                const float p = t1[ly][lx + k], q = t2[ly][lx + k];
                a = fmaf(kG[k], p, a);
                a2 = fmaf(kG[k], p * p, a2);
                bb = fmaf(kG[k], q, bb);
                b2 = fmaf(kG[k], q * q, b2);
                ab = fmaf(kG[k], p * q, ab);
            }
            hx[0][ly][lx] = a; hx[1][ly][lx] = a2; hx[2][ly][lx] = bb; hx[3][ly][lx] = b2; hx[4][ly][lx] = ab;
        }
        __syncthreads();
        float v[5][kRowsPerThread];
        vertical<5>(hx, cx, ry, v);
        const int x = x0 + cx;
#pragma unroll
        for (int r = 0; r < kRowsPerThread; r++) {
            const int y = y0 + ry + r;
            const float mu1 = v[0][r], mu2 = v[2][r];
            const float s1 = v[1][r] - mu1 * mu1;
            const float s2 = v[3][r] - mu2 * mu2;
            const float s12 = v[4][r] - mu1 * mu2;
            const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
            const float Cn = 2.0f * mu1_mu2 + C1;
            const float D = 2.0f * s12 + C2;
            const float A = (mu1_sq + mu2_sq) + C1;
            const float Bd = (s1 + s2) + C2;
            if (x < W && y < H) {
                const int64_t gi = base + (int64_t)y * W + x;
                map[gi] = (Cn * D) / (A * Bd);
                if (dmu1) {
                    dmu1[gi] = (mu2 * 2.0f * D) / (A * Bd) - (mu2 * 2.0f * Cn) / (A * Bd) -
                               (mu1 * 2.0f * Cn * D) / (A * A * Bd) + (mu1 * 2.0f * Cn * D) / (A * Bd * Bd);
                    ds1[gi] = (-Cn * D) / (A * Bd * Bd);
                    ds12[gi] = (2.0f * Cn) / (A * Bd);
                }
            }
        }
        __syncthreads();  // the next channel restages t1/t2/hx
    }
}

__global__ __launch_bounds__(256) void k_ssim_bwd(int CH, int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2,
                                                  const float* __restrict__ dL, const float* __restrict__ dmu1,
                                                  const float* __restrict__ ds1, const float* __restrict__ ds12,
                                                  float* __restrict__ dimg1) {
    __shared__ float tm[3][kHY][kLdsPitch];
    __shared__ float hx[3][kHY][kSX + 1];
    const int x0 = blockIdx.x * kSX, y0 = blockIdx.y * kSY, b = blockIdx.z;
    const int cx = threadIdx.x & 31, ry = (threadIdx.x >> 5) * kRowsPerThread;
    const int64_t plane = (int64_t)H * W;
    for (int c = 0; c < CH; c++) {
        const int64_t base = ((int64_t)b * CH + c) * plane;
        // staged products dL * dm/d(.), as the reference's multiply_shared_mem (ssim.cu:316-352)
        for (int i = threadIdx.x; i < kHY * kHX; i += blockDim.x) {
            const int ly = i / kHX, lx = i - ly * kHX;
            const int y = y0 - 5 + ly, x = x0 - 5 + lx;
            float g = 0.f, m0 = 0.f, m1 = 0.f, m2 = 0.f;
            if (y >= 0 && y < H && x >= 0 && x < W) {
                const int64_t gi = base + (int64_t)y * W + x;
                g = dL[gi];
                m0 = dmu1[gi] * g;
                m1 = ds1[gi] * g;
                m2 = ds12[gi] * g;
            }
            tm[0][ly][lx] = m0; tm[1][ly][lx] = m1; tm[2][ly][lx] = m2;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < kHY * kSX; i += blockDim.x) {
            const int ly = i >> 5, lx = i & 31;
            float a = 0.f, s = 0.f, t = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) {
                a = fmaf(kG[k], tm[0][ly][lx + k], a);
                s = fmaf(kG[k], tm[1][ly][lx + k], s);
                t = fmaf(kG[k], tm[2][ly][lx + k], t);
            }
            hx[0][ly][lx] = a; hx[1][ly][lx] = s; hx[2][ly][lx] = t;
        }
        __syncthreads();
        float v[3][kRowsPerThread];
        vertical<3>(hx, cx, ry, v);
        const int x = x0 + cx;
#pragma unroll
        for (int r = 0; r < kRowsPerThread; r++) {
            const int y = y0 + ry + r;
            if (x < W && y < H) {
                const int64_t gi = base + (int64_t)y * W + x;
                const float p1 = img1[gi], p2 = img2[gi];
                float d = v[0][r];
                d = d + p1 * 2.0f * v[1][r];
                d = d + p2 * v[2][r];
                dimg1[gi] = d;
            }
        }
        __syncthreads();
    }
}


// ---- the training step's L1 terms (gsr_image_loss): one thread per pixel, 32 channel reads and 32
// gradient writes (coalesced across the workgroup's pixels), the refine head's 3 x 32 weights as
// wave-uniform operands; the loss partial of each workgroup by a fixed-shape LDS tree.
__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ __launch_bounds__(256) void k_image_loss(int HW, const float* __restrict__ feat,
                                                    const float* __restrict__ target,
                                                    const float* __restrict__ rw, float l1w, float rfw,
                                                    float inv_n, const float* __restrict__ extra,
                                                    float* __restrict__ dL, float* __restrict__ partials) {
    __shared__ float red[256];
    const int b = blockIdx.y;
    const int p = blockIdx.x * 256 + threadIdx.x;
    float part = 0.f;
    if (p < HW) {
        const float* f = feat + (int64_t)b * 32 * HW + p;
        const float* t = target + (int64_t)b * 3 * HW + p;
        float fc[32];
#pragma unroll
        for (int c = 0; c < 32; c++) fc[c] = f[(int64_t)c * HW];
        float tt[3], s[3] = {0.f, 0.f, 0.f}, e[3];
#pragma unroll
        for (int o = 0; o < 3; o++) {
            tt[o] = t[(int64_t)o * HW];
            e[o] = fc[o] - tt[o];
            part += l1w * fabsf(e[o]);
        }
        if (rw) {
#pragma unroll
            for (int o = 0; o < 3; o++) {
                float r = 0.f;
#pragma unroll
                for (int c = 0; c < 32; c++) r = fmaf(rw[32 * o + c], fc[c], r);
                const float d = r - tt[o];
                part += rfw * fabsf(d);
                s[o] = rfw * inv_n * sgnf(d);
            }
        }
        float* g = dL + (int64_t)b * 32 * HW + p;
#pragma unroll
        for (int c = 0; c < 32; c++) {
            float v = rw ? fmaf(rw[c], s[0], fmaf(rw[32 + c], s[1], rw[64 + c] * s[2])) : 0.f;
            if (c < 3) {
                v += l1w * inv_n * sgnf(e[c]);
                if (extra) v += extra[(int64_t)b * 3 * HW + (int64_t)c * HW + p];
            }
            g[(int64_t)c * HW] = v;
        }
    }
    red[threadIdx.x] = part;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[(int64_t)b * gridDim.x + blockIdx.x] = red[0] * inv_n;
}

}  // namespace gsr

using namespace gsr;

extern "C" {

int gsr_fused_ssim(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                   float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, void* stream) {
    if (B < 0 || CH < 0 || H < 0 || W < 0) return api_fail(GSR_ERR_ARG, "gsr_fused_ssim: negative size");
    if ((int64_t)B * CH * H * W == 0) return 0;
    if (!img1 || !img2 || !ssim_map) return api_fail(GSR_ERR_ARG, "gsr_fused_ssim: null image");
    if ((dm_dmu1 || dm_dsigma1_sq || dm_dsigma12) && !(dm_dmu1 && dm_dsigma1_sq && dm_dsigma12))
        return api_fail(GSR_ERR_ARG, "gsr_fused_ssim: give all three partial maps or none");
    if (B > 65535) return api_fail(GSR_ERR_ARG, "gsr_fused_ssim: B > 65535");
    const dim3 grid((W + kSX - 1) / kSX, (H + kSY - 1) / kSY, B);
    hipLaunchKernelGGL(k_ssim_fwd, grid, dim3(256), 0, (hipStream_t)stream, CH, H, W, C1, C2, img1, img2,
                       ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : api_fail(GSR_ERR_HIP, hipGetErrorString(e));
}

int gsr_fused_ssim_backward(int B, int CH, int H, int W, float C1, float C2, const float* img1,
                            const float* img2, const float* dL_dmap, const float* dm_dmu1,
                            const float* dm_dsigma1_sq, const float* dm_dsigma12, float* dL_dimg1,
                            void* stream) {
    (void)C1;
    (void)C2;
    if (B < 0 || CH < 0 || H < 0 || W < 0) return api_fail(GSR_ERR_ARG, "gsr_fused_ssim_backward: negative size");
    if ((int64_t)B * CH * H * W == 0) return 0;
    if (!img1 || !img2 || !dL_dmap || !dm_dmu1 || !dm_dsigma1_sq || !dm_dsigma12 || !dL_dimg1)
        return api_fail(GSR_ERR_ARG, "gsr_fused_ssim_backward: null pointer (forward must run with train)");
    if (B > 65535) return api_fail(GSR_ERR_ARG, "gsr_fused_ssim_backward: B > 65535");
    const dim3 grid((W + kSX - 1) / kSX, (H + kSY - 1) / kSY, B);
    hipLaunchKernelGGL(k_ssim_bwd, grid, dim3(256), 0, (hipStream_t)stream, CH, H, W, img1, img2, dL_dmap,
                       dm_dmu1, dm_dsigma1_sq, dm_dsigma12, dL_dimg1);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : api_fail(GSR_ERR_HIP, hipGetErrorString(e));
}

int gsr_image_loss_partials(int B, int H, int W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return B * ((H * W + 255) / 256);
}

int gsr_image_loss(int B, int H, int W, const float* feat, const float* target, const float* refine_w,
                   float l1_weight, float refine_weight, const float* extra_grad, float* dL_dfeat,
                   float* loss_partials, void* stream) {
    if (B <= 0 || H <= 0 || W <= 0) return gsr::api_fail(GSR_ERR_ARG, "gsr_image_loss: bad sizes");
    if (!feat || !target || !dL_dfeat || !loss_partials)
        return gsr::api_fail(GSR_ERR_ARG, "gsr_image_loss: null required pointer");
    const int HW = H * W;
    const double n = 3.0 * (double)B * (double)HW;
    hipLaunchKernelGGL(gsr::k_image_loss, dim3((HW + 255) / 256, B), dim3(256), 0, (hipStream_t)stream, HW,
                       feat, target, refine_w, l1_weight, refine_weight, (float)(1.0 / n), extra_grad, dL_dfeat,
                       loss_partials);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gsr::api_fail(GSR_ERR_HIP, hipGetErrorString(e));
    return 0;
}

}  // extern "C"
