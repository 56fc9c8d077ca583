// render_fwd.hip -- front-to-back alpha compositing of 32-channel features (forward.cu:274-397 of
// the reference), one 256-thread workgroup per 16x16 tile per frame.
//
// Structure (gfx950):
//  * Each wave owns a 16x4 pixel strip of the tile (lane = pixel).  The workgroup stages the
//    tile's depth-sorted list in rounds of 64 Gaussians into LDS (position, opacity, 1/depth,
//    pre-scaled conic, cull box, 128-byte feature row).
//  * Per round every wave culls the 64 Gaussians against its strip with the conservative
//    alpha >= 1/255 box computed in preprocess (one lane per Gaussian, one ballot): culled pairs
//    cannot change any blend decision, so the result is identical to visiting every pair.
//  * Survivors are processed in chunks of 8.  Each lane walks the chunk front to back for its own
//    pixel (alpha, the T<1e-4 stop, n_contrib) producing blend weights w = alpha*T; the 32-channel
//    accumulation C += f*w is then done on the matrix cores as D[ch][px] += F^T[ch][k] W[k][px]
//    with v_mfma_f32_32x32x2_f32 (2 strips of 32 pixels, 4 k-steps per chunk).  The f32 MFMA is an
//    exact k-ordered fma chain, i.e. bit-identical to accumulating fmaf(f, w, C) Gaussian by
//    Gaussian -- the oracle's contract -- while the VALU computes the next chunk's weights.
//  * A pixel that does not take a Gaussian gets w = 0, which leaves its accumulator unchanged.
//
// Roofline: per frame the kernel must read 156 B per visible Gaussian (features + 2D attributes)
// and write 140 B per pixel (32 channels, inverse depth, final_T, n_contrib); the blend itself is
// VALU-latency bound (~25 VALU per (pixel, Gaussian) pair) and the MFMA work is 64 cycles per
// (wave, Gaussian).  bench.py reports both the HBM fraction and the pair count.
#include "gsr_internal.h"

namespace gsr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kFeatStride = GSR_C;  // floats per staged feature row

template <bool EXACT>
__global__ __launch_bounds__(GSR_TILE_PIX) void k_render_fwd(Dims d, Inputs in, GeomArena g,
                                                             ImageArena im, BinArena bn, Outputs o) {
    __shared__ float4 s_a[kRenderBatch];   // gx, gy, opacity, 1/depth
    __shared__ float4 s_c[kRenderBatch];   // A=-cx/2, Bb=-cy, Cq=-cz/2, unused
    __shared__ float4 s_box[kRenderBatch]; // gx-hx, gx+hx, gy-hy, gy+hy (empty box: never)
    __shared__ __attribute__((aligned(16))) float s_f[kRenderBatch * kFeatStride];
    __shared__ int s_done[GSR_TILE_PIX / 64];
    if (g.ctrl[kCtrlOverflow]) return;

    const int tile_g = blockIdx.x;
    const int b = tile_g / d.T;
    const int t = tile_g - b * d.T;
    const int tx = t % d.gx, ty = t / d.gx;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    // lane <-> pixel of the wave's 16x4 strip
    const int px = tx * GSR_BX + (lane & 15);
    const int py = ty * GSR_BY + wv * 4 + (lane >> 4);
    const bool inside = px < d.W && py < d.H;
    const float pfx = (float)px, pfy = (float)py;
    // strip box for culling
    const float sx0 = (float)(tx * GSR_BX), sx1 = (float)(tx * GSR_BX + 15);
    const float sy0 = (float)(ty * GSR_BY + wv * 4), sy1 = sy0 + 3.0f;

    const uint2 range = im.ranges[tile_g];
    const int n = (int)(range.y - range.x);
    const int64_t gbase = (int64_t)b * d.P;
    const float* __restrict__ colors = in.colors + in.s_colors * b;

    floatx16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; r++) { acc0[r] = 0.f; acc1[r] = 0.f; }
    float T = 1.0f, invd = 0.f;
    uint32_t last = 0;
    bool done = !inside;

    const int lj = threadIdx.x >> 2, lq = threadIdx.x & 3;
    for (int base = 0; base < n; base += kRenderBatch) {
        // ---- stage the round ----
        if (base + lj < n) {
            const uint32_t idx = bn.point_list[range.x + base + lj];
            const float4* fs = reinterpret_cast<const float4*>(colors + (int64_t)idx * GSR_C) + lq * 2;
            float4* fd = reinterpret_cast<float4*>(s_f + lj * kFeatStride) + lq * 2;
            fd[0] = fs[0];
            fd[1] = fs[1];
            if (lq == 0) {
                const float2 m = g.means2D[gbase + idx];
                const float4 co = g.conic[gbase + idx];
                const float2 e = g.ext[gbase + idx];
                s_a[lj] = make_float4(m.x, m.y, co.w, g.invdepth[gbase + idx]);
                s_c[lj] = make_float4(-0.5f * co.x, -co.y, -0.5f * co.z, 0.f);
                s_box[lj] = make_float4(m.x - e.x, m.x + e.x, m.y - e.y, m.y + e.y);
            }
        }
        __syncthreads();
        const int cnt = min(kRenderBatch, n - base);
        const bool wave_active = __any(!done);
        if (wave_active) {
            // ---- cull the round against this wave's strip: lane j tests Gaussian j ----
            bool keep = false;
            if (lane < cnt) {
                const float4 bx = s_box[lane];
                keep = bx.y >= sx0 && bx.x <= sx1 && bx.w >= sy0 && bx.z <= sy1;
            }
            uint64_t mask = __ballot(keep);
            while (mask) {
                // ---- next chunk of up to 8 surviving Gaussians (uniform indices) ----
                int ids[8];
                int nk = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    ids[k] = mask ? (int)__builtin_ctzll(mask) : -1;
                    if (mask) { mask &= mask - 1; nk++; }
                }
                float w[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    w[k] = 0.f;
                    if (ids[k] >= 0) {
                        const float4 a = s_a[ids[k]];
                        const float4 c = s_c[ids[k]];
                        if (!done) {
                            const float dx = a.x - pfx, dy = a.y - pfy;
                            const float power = blend_power(c.x, c.y, c.z, dx, dy);
                            if (!(power > 0.0f)) {
                                const float alpha = fminf(0.99f, a.z * blend_exp<EXACT>(power));
                                if (!(alpha < 1.0f / 255.0f)) {
                                    const float test_T = T * (1.0f - alpha);
                                    if (test_T < 0.0001f) {
                                        done = true;
                                    } else {
                                        const float wk = alpha * T;
                                        w[k] = wk;
                                        invd = fmaf(a.w, wk, invd);
                                        T = test_T;
                                        last = (uint32_t)(base + ids[k] + 1);
                                    }
                                }
                            }
                        }
                    }
                }
                // ---- C[ch][px] += F[ch][k] * W[k][px] on the matrix cores ----
                if (__any(w[0] != 0.f || w[1] != 0.f || w[2] != 0.f || w[3] != 0.f || w[4] != 0.f ||
                          w[5] != 0.f || w[6] != 0.f || w[7] != 0.f)) {
                    const int hi = lane >> 5;
                    const int ch = lane & 31;
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        const int ga = ids[2 * s] >= 0 ? ids[2 * s] : ids[0];
                        const int gb = ids[2 * s + 1] >= 0 ? ids[2 * s + 1] : ids[0];
                        const float fa = s_f[(hi ? gb : ga) * kFeatStride + ch];
                        const auto sw = __builtin_amdgcn_permlane32_swap(
                            __float_as_uint(w[2 * s]), __float_as_uint(w[2 * s + 1]), false, false);
                        const float b0 = __uint_as_float(sw[0]);
                        const float b1 = __uint_as_float(sw[1]);
                        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, b0, acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, b1, acc1, 0, 0, 0);
                    }
                }
                if (!__any(!done)) break;
            }
        }
        // ---- round end: stop when every pixel of the tile is saturated ----
        const bool wave_busy = __any(!done);  // ballot with the full wave, outside the lane-0 branch
        if (lane == 0) s_done[wv] = wave_busy ? 0 : 1;
        __syncthreads();
        bool all = true;
#pragma unroll
        for (int w2 = 0; w2 < GSR_TILE_PIX / 64; w2++) all = all && s_done[w2];
        if (all) break;
    }

    // ---- epilogue ----
    const int64_t HW = (int64_t)d.H * d.W;
    if (inside) {
        const int64_t pix = (int64_t)py * d.W + px;
        im.final_T[b * HW + pix] = T;
        im.n_contrib[b * HW + pix] = last;
        if (o.out_invdepth) o.out_invdepth[b * HW + pix] = invd;
    }
    // accumulator layout: acc_n[r] at lane l = channel (r&3)+8*(r>>2)+4*(l>>5) of strip pixel
    // 32n + (l&31); that pixel's transmittance lives in lane 32n + (l&31).
    const float T0 = __shfl(T, lane & 31);
    const float T1 = __shfl(T, 32 + (lane & 31));
    const float* bg = in.bg + in.s_bg * b;
    float* out = o.out_color + (int64_t)b * GSR_C * HW;
    const int j = lane & 31;
    const int qx = tx * GSR_BX + (j & 15);
    const int qy0 = ty * GSR_BY + wv * 4 + (j >> 4);
    const int qy1 = qy0 + 2;
    const bool in0 = qx < d.W && qy0 < d.H;
    const bool in1 = qx < d.W && qy1 < d.H;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int ch = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float bgc = bg[ch];
        if (in0) out[ch * HW + (int64_t)qy0 * d.W + qx] = fmaf(T0, bgc, acc0[r]);
        if (in1) out[ch * HW + (int64_t)qy1 * d.W + qx] = fmaf(T1, bgc, acc1[r]);
    }
}

void launch_render_fwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Outputs& o, bool exact, hipStream_t s) {
    const int ntiles = d.B * d.T;
    if (ntiles == 0) return;
    if (exact)
        hipLaunchKernelGGL(k_render_fwd<true>, dim3(ntiles), dim3(GSR_TILE_PIX), 0, s, d, in, g, im, b, o);
    else
        hipLaunchKernelGGL(k_render_fwd<false>, dim3(ntiles), dim3(GSR_TILE_PIX), 0, s, d, in, g, im, b, o);
}

}  // namespace gsr
