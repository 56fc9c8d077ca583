// render_bwd.hip -- back-to-front gradient replay (backward.cu:452-638 of the reference), one
// 256-thread workgroup per 16x16 tile per frame.
//
// Differences in structure (same math):
//  * the replay starts at the workgroup's largest n_contrib instead of the end of the tile list;
//  * the 32-channel "accumulated colour behind" recurrence is carried as its dot product with
//    dL/dpixel (linear, so sum_ch (c - accum_rec_ch) dL_ch == g - accum_dot with g = f . dL);
//  * per (wave, Gaussian) the 39 per-Gaussian gradient terms are reduced across the 64 pixels of
//    the wave with a transpose-reduction (40 -> 5 values per lane in 3 halving rounds + a 3-round
//    all-reduce) and issued as ONE 40-lane atomic instruction, instead of 39 atomics per pixel.
#include "gsr_internal.h"

namespace gsr {

// Reduce v[40] across the 64 lanes; lane l ends holding the sum of component
// ((l>>5)&1)*20 + ((l>>4)&1)*10 + ((l>>3)&1)*5 + k in out[k], k < 5.
__device__ __forceinline__ void wave_transpose_reduce40(float (&v)[40], float (&out)[5]) {
    const int lane = threadIdx.x & 63;
    float a[20];
    {
        const bool hi = lane & 32;
#pragma unroll
        for (int k = 0; k < 20; k++) {
            const float keep = hi ? v[k + 20] : v[k];
            const float send = hi ? v[k] : v[k + 20];
            a[k] = keep + __shfl_xor(send, 32);
        }
    }
    float bb[10];
    {
        const bool hi = lane & 16;
#pragma unroll
        for (int k = 0; k < 10; k++) {
            const float keep = hi ? a[k + 10] : a[k];
            const float send = hi ? a[k] : a[k + 10];
            bb[k] = keep + __shfl_xor(send, 16);
        }
    }
    {
        const bool hi = lane & 8;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const float keep = hi ? bb[k + 5] : bb[k];
            const float send = hi ? bb[k] : bb[k + 5];
            out[k] = keep + __shfl_xor(send, 8);
        }
    }
#pragma unroll
    for (int off = 4; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < 5; k++) out[k] += __shfl_xor(out[k], off);
}

template <bool EXACT, bool INVD>
__global__ __launch_bounds__(GSR_TILE_PIX) void k_render_bwd(Dims d, Inputs in, GeomArena g,
                                                             ImageArena im, BinArena bn, Grads gr) {
    __shared__ float4 s_a[kRenderBatch];      // gx, gy, opacity, 1/depth
    __shared__ float4 s_c[kRenderBatch];      // cx, cy, cz (conic), unused
    __shared__ float4 s_f[kRenderBatch * 8];  // features
    __shared__ uint32_t s_idx[kRenderBatch];
    __shared__ uint32_t s_red[GSR_TILE_PIX / 64];
    const int tile_g = blockIdx.x;
    const int b = tile_g / d.T;
    const int t = tile_g - b * d.T;
    const int tx = t % d.gx, ty = t / d.gx;
    const int px = tx * GSR_BX + (threadIdx.x & 15);
    const int py = ty * GSR_BY + (threadIdx.x >> 4);
    const bool inside = px < d.W && py < d.H;
    const uint2 range = im.ranges[tile_g];
    const int64_t HW = (int64_t)d.H * d.W;
    const int64_t pix = (int64_t)py * d.W + px;
    const int64_t gbase = (int64_t)b * d.P;
    const float* __restrict__ colors = in.colors + in.s_colors * b;
    const float pfx = (float)px, pfy = (float)py;
    const int lane = threadIdx.x & 63;

    const float T_final = inside ? im.final_T[b * HW + pix] : 0.f;
    const uint32_t last_contributor = inside ? im.n_contrib[b * HW + pix] : 0u;
    float dL[GSR_C];
    const float* bg = in.bg + in.s_bg * b;
    float bg_dot = 0.f;
#pragma unroll
    for (int ch = 0; ch < GSR_C; ch++) {
        dL[ch] = inside ? gr.dL_dpix[(b * GSR_C + ch) * HW + pix] : 0.f;
        bg_dot += bg[ch] * dL[ch];
    }
    const float dL_inv = (INVD && inside) ? gr.dL_dinvdepth[b * HW + pix] : 0.f;
    const float ddelx_dx = 0.5f * (float)d.W;
    const float ddely_dy = 0.5f * (float)d.H;

    // replay length: the largest n_contrib of the tile
    uint32_t mx = last_contributor;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, off));
    if (lane == 0) s_red[threadIdx.x >> 6] = mx;
    __syncthreads();
    uint32_t n = 0;
#pragma unroll
    for (int w = 0; w < GSR_TILE_PIX / 64; w++) n = max(n, s_red[w]);

    float T = T_final;
    float accum_dot = 0.f, last_gdot = 0.f, last_alpha = 0.f;
    float accum_inv = 0.f, last_inv = 0.f;
    uint32_t contributor = n;
    const int lj = threadIdx.x >> 2, lq = threadIdx.x & 3;
    for (int done_cnt = 0; done_cnt < (int)n; done_cnt += kRenderBatch) {
        const int cnt = min(kRenderBatch, (int)n - done_cnt);
        __syncthreads();
        if (lj < cnt) {
            const uint32_t idx = bn.point_list[range.x + n - 1 - done_cnt - lj] & kIndexMask;
            const float4* fs = reinterpret_cast<const float4*>(colors + (int64_t)idx * GSR_C) + lq * 2;
            s_f[lj * 8 + lq * 2] = fs[0];
            s_f[lj * 8 + lq * 2 + 1] = fs[1];
            if (lq == 0) {
                const float2 m = g.means2D[gbase + idx];
                const float4 co = g.conic[gbase + idx];
                s_a[lj] = make_float4(m.x, m.y, co.w, g.invdepth[gbase + idx]);
                s_c[lj] = make_float4(co.x, co.y, co.z, 0.f);
                s_idx[lj] = idx;
            }
        }
        __syncthreads();
        for (int j = 0; j < cnt; j++) {
            contributor--;
            const float4 a = s_a[j];
            const float4 c = s_c[j];
            const float dx = a.x - pfx, dy = a.y - pfy;
            const float power = blend_power(-0.5f * c.x, -c.y, -0.5f * c.z, dx, dy);
            bool act = inside && contributor < last_contributor && !(power > 0.0f);
            float G = 0.f, alpha = 0.f;
            if (act) {
                G = blend_exp<EXACT>(power);
                alpha = fminf(0.99f, a.z * G);
                act = !(alpha < 1.0f / 255.0f);
            }
            if (!__any(act)) continue;
            float v[40];
#pragma unroll
            for (int k = 0; k < 40; k++) v[k] = 0.f;
            if (act) {
                T = T / (1.f - alpha);
                const float wgt = alpha * T;
                float gdot = 0.f;
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const float4 f = s_f[j * 8 + q];
                    gdot = fmaf(f.x, dL[4 * q + 0], gdot);
                    gdot = fmaf(f.y, dL[4 * q + 1], gdot);
                    gdot = fmaf(f.z, dL[4 * q + 2], gdot);
                    gdot = fmaf(f.w, dL[4 * q + 3], gdot);
                }
#pragma unroll
                for (int ch = 0; ch < GSR_C; ch++) v[ch] = wgt * dL[ch];
                accum_dot = last_alpha * last_gdot + (1.f - last_alpha) * accum_dot;
                last_gdot = gdot;
                float dL_dalpha = gdot - accum_dot;
                if (INVD) {
                    const float invdg = a.w;
                    accum_inv = last_alpha * last_inv + (1.f - last_alpha) * accum_inv;
                    last_inv = invdg;
                    dL_dalpha += (invdg - accum_inv) * dL_inv;
                    v[38] = wgt * dL_inv;
                }
                dL_dalpha *= T;
                last_alpha = alpha;
                dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                const float dL_dG = a.z * dL_dalpha;
                const float gdx = G * dx;
                const float gdy = G * dy;
                const float dG_ddelx = -gdx * c.x - gdy * c.y;
                const float dG_ddely = -gdy * c.z - gdx * c.y;
                v[32] = dL_dG * dG_ddelx * ddelx_dx;
                v[33] = dL_dG * dG_ddely * ddely_dy;
                v[34] = -0.5f * gdx * dx * dL_dG;
                v[35] = -0.5f * gdx * dy * dL_dG;
                v[36] = -0.5f * gdy * dy * dL_dG;
                v[37] = G * dL_dalpha;
            }
            float r[5];
            wave_transpose_reduce40(v, r);
            const int sub = lane & 7;
            if (sub < 5) {
                const int comp = ((lane >> 5) & 1) * 20 + ((lane >> 4) & 1) * 10 + ((lane >> 3) & 1) * 5 + sub;
                float val = r[0];
                val = sub == 1 ? r[1] : val;
                val = sub == 2 ? r[2] : val;
                val = sub == 3 ? r[3] : val;
                val = sub == 4 ? r[4] : val;
                const int64_t gg = gbase + s_idx[j];
                float* dst = nullptr;
                if (comp < 32) dst = gr.dL_dcolors + gg * GSR_C + comp;
                else if (comp == 32) dst = gr.dL_dmean2D + gg * 3;
                else if (comp == 33) dst = gr.dL_dmean2D + gg * 3 + 1;
                else if (comp == 34) dst = gr.dL_dconic + gg * 4;
                else if (comp == 35) dst = gr.dL_dconic + gg * 4 + 1;
                else if (comp == 36) dst = gr.dL_dconic + gg * 4 + 3;
                else if (comp == 37) dst = gr.dL_dopacity + gg;
                else if (comp == 38 && INVD) dst = gr.dL_dinvdepth_g + gg;
                if (dst && val != 0.f) atomicAdd(dst, val);
            }
        }
    }
}

void launch_render_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Grads& gr, bool exact, hipStream_t s) {
    const int ntiles = d.B * d.T;
    if (ntiles == 0) return;
    const bool invd = gr.dL_dinvdepth != nullptr && gr.dL_dinvdepth_g != nullptr;
    dim3 grid(ntiles), blk(GSR_TILE_PIX);
    if (exact) {
        if (invd) hipLaunchKernelGGL((k_render_bwd<true, true>), grid, blk, 0, s, d, in, g, im, b, gr);
        else hipLaunchKernelGGL((k_render_bwd<true, false>), grid, blk, 0, s, d, in, g, im, b, gr);
    } else {
        if (invd) hipLaunchKernelGGL((k_render_bwd<false, true>), grid, blk, 0, s, d, in, g, im, b, gr);
        else hipLaunchKernelGGL((k_render_bwd<false, false>), grid, blk, 0, s, d, in, g, im, b, gr);
    }
}

}  // namespace gsr
