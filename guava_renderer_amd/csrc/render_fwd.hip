// render_fwd.hip -- front-to-back alpha compositing of 32-channel features (forward.cu:274-397 of
// the reference).
//
// Structure (gfx950):
//  * Persistent 256-thread workgroups dequeue 16x16 tiles from k_tile_scan's work list (longest
//    list first), so every XCD gets work and the long tiles start early.
//  * Each wave owns a 16x4 pixel strip of the tile (lane = pixel).  The tile's depth-sorted list
//    is staged in rounds of 64 Gaussians by LDS-DMA (global_load_lds_dwordx4, double-buffered):
//    a 64-byte render record per Gaussian (position, opacity, 1/depth, pre-scaled conic, cull box;
//    written by preprocess) and its 128-byte feature row.  Round r+1 is in flight while round r is
//    blended, and no staging data lives in VGPRs.
//  * Per round every wave culls the 64 Gaussians against its strip with the conservative
//    alpha >= 1/255 box (one lane per Gaussian, one ballot): a culled pair cannot change any blend
//    decision, so the result is identical to visiting every pair.
//  * Survivors are taken two at a time in list order (one MFMA k-step): each lane runs the
//    branch-free blend step for its pixel (alpha, the T<1e-4 stop, n_contrib) giving the weight
//    w = alpha*T (0 where the pixel does not take the Gaussian), and the 32-channel accumulation
//    C += f*w runs on the matrix cores as D[ch][px] += F^T[ch][k] W[k][px] with
//    v_mfma_f32_32x32x2_f32 over the strip's two 32-pixel halves.  The f32 MFMA is an exact
//    k-ordered fma chain, i.e. bit-identical to fmaf(f, w, C) Gaussian by Gaussian (the oracle's
//    contract); a zero weight leaves the accumulator unchanged.  An odd tail uses a null Gaussian.
//
// Roofline: per frame the kernel must read 156 B per visible Gaussian (features + 2D attributes)
// and write 140 B per pixel (32 channels, inverse depth, final_T, n_contrib).
#include "gsr_internal.h"

namespace gsr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kRB = kRenderBatch;      // Gaussians per round (64)
constexpr int kNull = kRB;             // slot of the null Gaussian in each buffer
constexpr int kRecF4 = 4;              // float4 per render record
constexpr int kSlots = kRB + 1;

// One (pixel, Gaussian) step of the front-to-back blend (forward.cu:349-381), branch-free.
// Returns the blend weight alpha*T (0 when the pixel does not take this Gaussian) and updates the
// pixel's transmittance, inverse depth, last contributor (1-based list position) and done flag.
template <bool EXACT>
__device__ __forceinline__ float blend_one(const float4 ga, const float4 gc, float pfx, float pfy,
                                           int pos, float& T, float& invd, uint32_t& last, bool& done) {
    const float dx = ga.x - pfx, dy = ga.y - pfy;
    const float power = blend_power(gc.x, gc.y, gc.z, dx, dy);
    const float alpha = fminf(0.99f, ga.z * blend_exp<EXACT>(power));
    const bool take = !done && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
    const float test_T = T * (1.0f - alpha);
    const bool term = take && (test_T < 0.0001f);
    const bool contrib = take && !term;
    const float w = contrib ? alpha * T : 0.0f;
    invd = fmaf(ga.w, w, invd);
    T = contrib ? test_T : T;
    last = contrib ? (uint32_t)pos : last;
    done = done || term;
    return w;
}

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                     (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <bool EXACT, bool STATS>
__global__ __launch_bounds__(GSR_TILE_PIX) void k_render_fwd(Dims d, Inputs in, GeomArena g,
                                                             ImageArena im, BinArena bn, Outputs o) {
    __shared__ __attribute__((aligned(16))) float4 s_rec[2][kSlots * kRecF4];
    __shared__ __attribute__((aligned(16))) float s_f[2][kSlots * GSR_C];
    __shared__ int s_done[GSR_TILE_PIX / 64];
    __shared__ int s_item;
    if (g.ctrl[kCtrlOverflow]) return;
    const int ntiles = d.B * d.T;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    // null Gaussian in both buffers: power 0, opacity 0 -> alpha 0, never taken, zero features
    if (threadIdx.x < 2 * kRecF4)
        s_rec[threadIdx.x >> 2][kNull * kRecF4 + (threadIdx.x & 3)] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (threadIdx.x < 2 * GSR_C) s_f[threadIdx.x >> 5][kNull * GSR_C + (threadIdx.x & 31)] = 0.f;
    // DMA lane roles: records of Gaussians 16*wv + lane/4 (part lane%4), features of Gaussians
    // 16*wv + lane/8 and 16*wv + 8 + lane/8 (part lane%8)
    const int rg = 16 * wv + (lane >> 2), rp = lane & 3;
    const int fg0 = 16 * wv + (lane >> 3), fg1 = fg0 + 8, fp = lane & 7;

    for (;;) {
        if (threadIdx.x == 0) s_item = (int)atomicAdd(&g.ctrl[kCtrlRenderHead], 1u);
        __syncthreads();
        const int item = s_item;
        if (item >= ntiles) break;
        const int tile_g = (int)im.work_list[item];
        const int b = tile_g / d.T;
        const int t = tile_g - b * d.T;
        const int tx = t % d.gx, ty = t / d.gx;
        const int px = tx * GSR_BX + (lane & 15);
        const int py = ty * GSR_BY + wv * 4 + (lane >> 4);
        const bool inside = px < d.W && py < d.H;
        const float pfx = (float)px, pfy = (float)py;
        const float sx0 = (float)(tx * GSR_BX), sx1 = sx0 + 15.0f;
        const float sy0 = (float)(ty * GSR_BY + wv * 4), sy1 = sy0 + 3.0f;
        const uint2 range = im.ranges[tile_g];
        const int n = (int)(range.y - range.x);
        const uint32_t* __restrict__ plist = bn.point_list + range.x;
        const float4* __restrict__ rrec = g.rrec + (int64_t)b * d.P * kRecF4;
        const float* __restrict__ colors = in.colors + in.s_colors * b;

        floatx16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; r++) { acc0[r] = 0.f; acc1[r] = 0.f; }
        float T = 1.0f, invd = 0.f;
        uint32_t last = 0;
        bool done = !inside;
        uint64_t n_surv = 0, n_steps = 0, n_contrib_pairs = 0, n_staged = 0;
        uint32_t stop = 0;

        // stage round `base` into buffer `buf` (lanes beyond the list stay idle)
#define GSR_ISSUE(base_, buf_)                                                                      \
        {                                                                                           \
            if ((base_) + rg < n)                                                                   \
                glds16(rrec + (int64_t)ir * kRecF4 + rp, &s_rec[(buf_)][(16 * wv) * kRecF4]);       \
            if ((base_) + fg0 < n)                                                                  \
                glds16(colors + (int64_t)if0 * GSR_C + fp * 4, &s_f[(buf_)][(16 * wv) * GSR_C]);    \
            if ((base_) + fg1 < n)                                                                  \
                glds16(colors + (int64_t)if1 * GSR_C + fp * 4, &s_f[(buf_)][(16 * wv + 8) * GSR_C]);\
        }
#define GSR_PREFETCH_IDX(nb_)                                                                       \
        {                                                                                           \
            ir = ((nb_) + rg < n) ? (int)plist[(nb_) + rg] : 0;                                     \
            if0 = ((nb_) + fg0 < n) ? (int)plist[(nb_) + fg0] : 0;                                  \
            if1 = ((nb_) + fg1 < n) ? (int)plist[(nb_) + fg1] : 0;                                  \
        }
        int ir, if0, if1;
        GSR_PREFETCH_IDX(0)
        if (n > 0) GSR_ISSUE(0, 0)
        GSR_PREFETCH_IDX(kRB)
        __syncthreads();  // round 0 landed (the barrier drains the DMA); s_item consumed

        int buf = 0;
        for (int base = 0; base < n; base += kRB) {
            if (base + kRB < n) {
                GSR_ISSUE(base + kRB, buf ^ 1)
                GSR_PREFETCH_IDX(base + 2 * kRB)
            }
            const int cnt = min(kRB, n - base);
            if (STATS) n_staged += cnt;
            const float4* __restrict__ rec = s_rec[buf];
            const float* __restrict__ fb = s_f[buf];
            if (__any(!done)) {
                bool keep = false;
                if (lane < cnt) {
                    const float4 bx = rec[lane * kRecF4 + 2];
                    keep = bx.y >= sx0 && bx.x <= sx1 && bx.w >= sy0 && bx.z <= sy1;
                }
                uint64_t mask = __ballot(keep);
                if (STATS) n_surv += __popcll(mask);
                const int hi = lane >> 5;
                const int ch = lane & 31;
                while (mask) {
                    const int ia = (int)__builtin_ctzll(mask);
                    mask &= mask - 1;
                    const int ib = mask ? (int)__builtin_ctzll(mask) : kNull;
                    mask &= mask - 1;
                    const float fa = fb[(hi ? ib : ia) * GSR_C + ch];
                    const bool was_done = done;
                    const float wa = blend_one<EXACT>(rec[ia * kRecF4], rec[ia * kRecF4 + 1], pfx, pfy,
                                                      base + ia + 1, T, invd, last, done);
                    const bool done_a = done;
                    const float wb = blend_one<EXACT>(rec[ib * kRecF4], rec[ib * kRecF4 + 1], pfx, pfy,
                                                      base + ib + 1, T, invd, last, done);
                    if (STATS) {
                        // list position at which a pixel terminated inside this step
                        if (!was_done && done_a) stop = (uint32_t)(base + ia + 1);
                        else if (!done_a && done) stop = (uint32_t)(base + ib + 1);
                        n_contrib_pairs += __popcll(__ballot(wa > 0.f)) + __popcll(__ballot(wb > 0.f));
                        n_steps++;
                    }
                    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(wa), __float_as_uint(wb),
                                                                     false, false);
                    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, __uint_as_float(sw[0]), acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, __uint_as_float(sw[1]), acc1, 0, 0, 0);
                }
            }
            const bool wave_busy = __any(!done);
            if (lane == 0) s_done[wv] = wave_busy ? 0 : 1;
            __syncthreads();  // also retires the next round's DMA for every wave
            const bool all = s_done[0] && s_done[1] && s_done[2] && s_done[3];
            buf ^= 1;
            if (all) break;
        }
#undef GSR_ISSUE
#undef GSR_PREFETCH_IDX

        // ---- epilogue ----
        const int64_t HW = (int64_t)d.H * d.W;
        if (STATS) {
            unsigned long long* cnt = (unsigned long long*)o.stats;
            uint64_t ev = inside ? (done ? stop : (uint32_t)n) : 0;
            for (int off = 32; off > 0; off >>= 1) ev += __shfl_xor(ev, off);
            if (lane == 0) {
                atomicAdd(&cnt[0], (unsigned long long)ev);
                atomicAdd(&cnt[1], (unsigned long long)n_contrib_pairs);
                atomicAdd(&cnt[2], (unsigned long long)n_surv);
                atomicAdd(&cnt[3], (unsigned long long)n_steps);
                if (wv == 0) {
                    atomicAdd(&cnt[4], (unsigned long long)n_staged);
                    atomicAdd(&cnt[5], (unsigned long long)n);
                    atomicAdd(&cnt[6], 1ull);
                }
            }
        }
        if (inside) {
            const int64_t pix = (int64_t)py * d.W + px;
            im.final_T[b * HW + pix] = T;
            im.n_contrib[b * HW + pix] = last;
            if (o.out_invdepth) o.out_invdepth[b * HW + pix] = invd;
        }
        // acc_n[r] at lane l = channel (r&3)+8*(r>>2)+4*(l>>5) of strip pixel 32n + (l&31), whose
        // transmittance lives in lane 32n + (l&31).
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
        __syncthreads();  // LDS buffers and s_item are reused by the next tile
    }
}

void launch_render_fwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Outputs& o, bool exact, hipStream_t s) {
    const int ntiles = d.B * d.T;
    if (ntiles == 0) return;
    const int grid = min(ntiles, persistent_grid(4));
    const dim3 gr(grid), bl(GSR_TILE_PIX);
    if (o.stats) {
        if (exact) hipLaunchKernelGGL((k_render_fwd<true, true>), gr, bl, 0, s, d, in, g, im, b, o);
        else hipLaunchKernelGGL((k_render_fwd<false, true>), gr, bl, 0, s, d, in, g, im, b, o);
    } else {
        if (exact) hipLaunchKernelGGL((k_render_fwd<true, false>), gr, bl, 0, s, d, in, g, im, b, o);
        else hipLaunchKernelGGL((k_render_fwd<false, false>), gr, bl, 0, s, d, in, g, im, b, o);
    }
}

}  // namespace gsr
