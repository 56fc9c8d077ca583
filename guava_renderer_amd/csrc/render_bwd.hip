// render_bwd.hip -- back-to-front gradient replay (backward.cu:452-638 of the reference).
//
// Differences in structure (same math):
//  * one wave per 8x8 strip from persistent per-XCD queues, replaying only the Gaussians binning
//    marked as reaching the strip, from the strip's largest n_contrib instead of the tile list end;
//  * the 32-channel "accumulated colour behind" recurrence is carried as its dot product with
//    dL/dpixel (linear, so sum_ch (c - accum_rec_ch) dL_ch == g - accum_dot with g = f . dL);
//  * dL/dcolor of a Gaussian is sum_px w_px dL_px (w = alpha T): a contraction over the strip's 64
//    pixels, done on the matrix cores for batches of 32 active Gaussians -- each lane parks its
//    pixel's weight in wave-private LDS, and at the end of a batch 32 v_mfma_f32_32x32x2_f32 (two
//    pixels per k-step) give the [32 channels x 32 Gaussians] block, issued as 16 atomic
//    instructions, instead of 32 multiplies and a 32-channel cross-lane reduction per Gaussian;
//  * the other 7 per-Gaussian terms (mean2D, conic, opacity, inverse depth) are reduced across the
//    64 pixels with an 8-wide transpose-reduction, parked in LDS and issued with the batch, so no
//    atomic sits in vmcnt ahead of the next survivor's loads;
//  * one survivor of look-ahead: the next render record is loaded (vector loads, in-order vmcnt)
//    while the current survivor runs.
#include "gsr_internal.h"

namespace gsr {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kBwdBatch = 32;      // active Gaussians per colour-gradient MFMA batch
constexpr int kBwdPitch = 65;      // LDS row pitch (floats) of the [32][64] weight / dL tiles
constexpr int kBwdComps = 8;      // per-Gaussian non-colour gradient terms parked per batch slot
constexpr int kBwdLdsWave = kBwdBatch * kBwdPitch + kBwdBatch * kBwdComps;  // floats per wave

// Orders this wave's LDS accesses (rocPRIM's wave_barrier): the LDS executes a wave's DS
// instructions in order, so a lane then reads what another lane of its wave wrote before.
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Reduce v[8] across the 64 lanes; lane l ends holding the sum of component
// ((l>>5)&1)*4 + ((l>>4)&1)*2 + ((l>>3)&1) (complete in every lane of its group of 8).  VALU only:
// v_permlane32_swap / v_permlane16_swap halve across the wave halves and rows, DPP row_ror:8 across
// the half-rows, then quad_perm and row_half_mirror finish inside each group of 8 -- no LDS
// round trip (ds_bpermute) in the per-Gaussian chain.
__device__ __forceinline__ float wave_transpose_reduce8(const float (&v)[8]) {
    const int lane = threadIdx.x & 63;
    float a[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // lanes 0-31 keep component k, lanes 32-63 component k+4
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[k]), __float_as_uint(v[k + 4]),
                                                         false, false);
        a[k] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    float bb[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {  // even rows keep a[k], odd rows a[k+2]
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[k]), __float_as_uint(a[k + 2]),
                                                         false, false);
        bb[k] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    const float c0 = bb[0] + dpp<0x128>(bb[0]);  // row_ror:8 = the other half-row
    const float c1 = bb[1] + dpp<0x128>(bb[1]);
    float c = (lane & 8) ? c1 : c0;
    c += dpp<0xB1>(c);   // quad_perm [1,0,3,2]
    c += dpp<0x4E>(c);   // quad_perm [2,3,0,1]
    c += dpp<0x141>(c);  // row_half_mirror: the other quad of the group of 8
    return c;
}

// Work: the 8x8 strips of the non-empty tiles, in strip_list order (most survivors first), dealt to
// per-XCD queues exactly like render_fwd (separate counters).  One wave owns a strip (lane = pixel)
// and replays its tile's depth-sorted list back to front from the strip's largest n_contrib,
// taking only the Gaussians whose strip bit is set in point_list (binning's exact test that the
// Gaussian reaches alpha >= 1/255 somewhere in the strip; the others cannot be active on any of its
// pixels).  No workgroup barriers: render records and feature rows arrive by scalar loads (the
// Gaussian index is wave-uniform); the LDS is wave-private.
constexpr int kBwdQueueOffset = 32;  // words after each forward XCD counter (own cache line)

template <bool EXACT, bool INVD>
__global__ __launch_bounds__(GSR_TILE_PIX) __attribute__((amdgpu_waves_per_eu(3))) void k_render_bwd(Dims d, Inputs in, GeomArena g,
                                                             ImageArena im, BinArena bn, Grads gr) {
    __shared__ float lds_all[(GSR_TILE_PIX / 64) * kBwdLdsWave];
    if (g.ctrl[kCtrlOverflow]) return;
    const uint32_t ne = g.ctrl[kCtrlNonEmpty];
    const int lane = threadIdx.x & 63;
    float* wl = lds_all + (threadIdx.x >> 6) * kBwdLdsWave;  // this wave's [32][65] tile
    float* cl = wl + kBwdBatch * kBwdPitch;                    // and its [32][8] term slots
    uint32_t vzero;  // a VGPR zero: indexes the uniform record loads so they stay vector loads
    asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
    const int hi = lane >> 5, l32 = lane & 31;
    uint32_t q = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;  // HW_REG_XCC_ID
    uint32_t q_left = 8;
    const int64_t HW = (int64_t)d.H * d.W;
    const float ddelx_dx = 0.5f * (float)d.W;
    const float ddely_dy = 0.5f * (float)d.H;

    for (;;) {
        uint32_t item = 0xFFFFFFFFu;
        while (q_left) {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g.ctrl[kCtrlXcdQueue + kCtrlXcdStride * q + kBwdQueueOffset], 1u);
            k = __builtin_amdgcn_readfirstlane(k);
            item = queue_item(q, k, ne, 0u, in.xcd_map);
            if (item != 0xFFFFFFFFu) break;
            q = (q + 1) & 7u;
            q_left--;
        }
        if (!q_left) break;
        const uint32_t code = im.strip_list[item];
        const int tile_g = (int)(code >> 2);
        const int strip = (int)(code & 3u);
        const int b = tile_g / d.T;
        const int t = tile_g - b * d.T;
        const int tx = t % d.gx, ty = t / d.gx;
        int sx0, sy0;
        strip_origin(tx, ty, strip, sx0, sy0);
        const int px = sx0 + lane % kStripW;
        const int py = sy0 + lane / kStripW;
        const bool inside = px < d.W && py < d.H;
        const int64_t pix = b * HW + (int64_t)py * d.W + px;
        const float pfx = (float)px, pfy = (float)py;
        const uint32_t smask_bit = 1u << (28 + strip);
        const uint2 range = im.ranges[tile_g];
        const uint32_t* __restrict__ plist = bn.point_list + range.x;
        const float4* __restrict__ rrec = g.rrec + (int64_t)b * d.P * 2;
        const float* __restrict__ colors = in.colors + in.s_colors * b;
        const int64_t gbase = (int64_t)b * d.P;

        const float T_final = inside ? im.final_T[pix] : 0.f;
        const uint32_t last_contributor = inside ? im.n_contrib[pix] : 0u;
        // the strip's replay length
        uint32_t ns = last_contributor;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) ns = max(ns, (uint32_t)__shfl_xor(ns, off));
        ns = __builtin_amdgcn_readfirstlane(ns);
        if (ns == 0) continue;
        float dL[GSR_C];
        const float* bg = in.bg + in.s_bg * b;
        float bg_dot = 0.f;
#pragma unroll
        for (int ch = 0; ch < GSR_C; ch++) {
            dL[ch] = inside ? gr.dL_dpix[(b * GSR_C + ch) * HW + (pix - b * HW)] : 0.f;
            bg_dot += bg[ch] * dL[ch];
        }
        const float dL_inv = (INVD && inside) ? gr.dL_dinvdepth[pix] : 0.f;

        // MFMA A operands of the colour-gradient contraction: step j covers strip pixels 2j, 2j+1;
        // lane l holds dL[pixel 2j + (l>>5)][channel l&31].  Transposed through the LDS tile.
        float adl[kBwdBatch];
        wave_lds_order();
#pragma unroll
        for (int ch = 0; ch < GSR_C; ch++) wl[ch * kBwdPitch + lane] = dL[ch];
        wave_lds_order();
#pragma unroll
        for (int j = 0; j < kBwdBatch; j++) adl[j] = wl[l32 * kBwdPitch + 2 * j + hi];
        wave_lds_order();

        // the current batch: slot s holds Gaussian gbat[lane s], its weights at wl[s][pixel]
        int slot = 0;
        int gbat = 0;
        auto flush = [&]() {
            wave_lds_order();
            floatx16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
            for (int j = 0; j < kBwdBatch; j++) {
                const float w = l32 < slot ? wl[l32 * kBwdPitch + 2 * j + hi] : 0.f;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(adl[j], w, acc, 0, 0, 0);
            }
            wave_lds_order();
            // acc[r] at lane l: channel (r&3) + 8(r>>2) + 4(l>>5) of the batch's Gaussian l&31
            const uint32_t gsel = (uint32_t)__shfl(gbat, l32);
            if (l32 < slot) {
                const int64_t gg = gbase + gsel;
                float* dst = gr.dL_dcolors + gg * GSR_C + 4 * hi;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const float val = acc[r];
                    if (val != 0.f) atomicAdd(dst + (r & 3) + 8 * (r >> 2), val);
                }
                // the parked terms: lane l takes terms 4(l>>5) .. +3 of slot l&31
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int comp = 4 * hi + u;
                    const float val = cl[l32 * kBwdComps + comp];
                    float* dc = nullptr;
                    if (comp == 0) dc = gr.dL_dmean2D + gg * 3;
                    else if (comp == 1) dc = gr.dL_dmean2D + gg * 3 + 1;
                    else if (comp == 2) dc = gr.dL_dconic + gg * 4;
                    else if (comp == 3) dc = gr.dL_dconic + gg * 4 + 1;
                    else if (comp == 4) dc = gr.dL_dconic + gg * 4 + 3;
                    else if (comp == 5) dc = gr.dL_dopacity + gg;
                    else if (comp == 6 && INVD) dc = gr.dL_dinvdepth_g + gg;
                    if (dc && val != 0.f) atomicAdd(dc, val);
                }
            }
            wave_lds_order();
            slot = 0;
        };

        float T = T_final;
        float accum_dot = 0.f, last_gdot = 0.f, last_alpha = 0.f;
        float accum_inv = 0.f, last_inv = 0.f;
        // survivor stream, back to front: chunks of 64 list positions, last chunk first (the next
        // lower chunk prefetched), the strip's survivors of a chunk from its highest bit down
        int base = (int)((ns - 1) & ~63u) + 64;
        uint32_t cidx = 0;
        uint32_t nidx = base - 64 + lane < (int)ns ? plist[base - 64 + lane] : 0u;
        uint64_t mask = 0;
        auto next_survivor = [&](uint32_t& gi_o, uint32_t& contrib_o) -> bool {
            while (mask == 0) {
                base -= 64;
                if (base < 0) return false;
                cidx = nidx;
                if (base >= 64) nidx = plist[base - 64 + lane];
                mask = __ballot(base + lane < (int)ns && (cidx & smask_bit) != 0u);
            }
            const int i = 63 - (int)__builtin_clzll(mask);
            mask &= ~(1ull << i);
            gi_o = __builtin_amdgcn_readlane(cidx, i) & kIndexMask;
            contrib_o = (uint32_t)(base + i);  // 0-based list position
            return true;
        };
        // one survivor of look-ahead: its render record is in flight while the current one runs
        uint32_t gi = 0, contributor = 0;
        bool have = next_survivor(gi, contributor);
        float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rc = ra;
        if (have) { ra = rrec[2 * gi + vzero]; rc = rrec[2 * gi + 1 + vzero]; }
        while (have) {
            uint32_t gi_n = 0, contributor_n = 0;
            const bool have_n = next_survivor(gi_n, contributor_n);
            float4 ra_n = ra, rc_n = rc;
            if (have_n) { ra_n = rrec[2 * gi_n + vzero]; rc_n = rrec[2 * gi_n + 1 + vzero]; }
            {
                // ra: x, y, opacity, 1/depth; rc: -a/2, -b, -c/2
                const float dx = ra.x - pfx, dy = ra.y - pfy;
                const float power = blend_power(rc.x, rc.y, rc.z, dx, dy);
                bool act = inside && contributor < last_contributor && !(power > 0.0f);
                float G = 0.f, alpha = 0.f;
                if (act) {
                    G = blend_exp<EXACT>(power);
                    alpha = fminf(0.99f, ra.z * G);
                    act = !(alpha < 1.0f / 255.0f);
                }
                if (__any(act)) {
                    float v[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) v[k] = 0.f;
                    float wgt = 0.f;
                    if (act) {
                        const float ca = -2.0f * rc.x, cb = -rc.y, cc = -2.0f * rc.z;  // exact
                        T = T / (1.f - alpha);
                        wgt = alpha * T;
                        const float* f = colors + (int64_t)gi * GSR_C;
                        float gdot = 0.f;
#pragma unroll
                        for (int ch = 0; ch < GSR_C; ch++) gdot = fmaf(f[ch], dL[ch], gdot);
                        accum_dot = last_alpha * last_gdot + (1.f - last_alpha) * accum_dot;
                        last_gdot = gdot;
                        float dL_dalpha = gdot - accum_dot;
                        if (INVD) {
                            const float invdg = ra.w;
                            accum_inv = last_alpha * last_inv + (1.f - last_alpha) * accum_inv;
                            last_inv = invdg;
                            dL_dalpha += (invdg - accum_inv) * dL_inv;
                            v[6] = wgt * dL_inv;
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = ra.z * dL_dalpha;
                        const float gdx = G * dx;
                        const float gdy = G * dy;
                        const float dG_ddelx = -gdx * ca - gdy * cb;
                        const float dG_ddely = -gdy * cc - gdx * cb;
                        v[0] = dL_dG * dG_ddelx * ddelx_dx;
                        v[1] = dL_dG * dG_ddely * ddely_dy;
                        v[2] = -0.5f * gdx * dx * dL_dG;
                        v[3] = -0.5f * gdx * dy * dL_dG;
                        v[4] = -0.5f * gdy * dy * dL_dG;
                        v[5] = G * dL_dalpha;
                    }
                    // this Gaussian joins the batch: its weights and its 7 reduced terms are parked
                    // in LDS, all of its atomics go out with the batch (none between two flushes)
                    wl[slot * kBwdPitch + lane] = wgt;
                    gbat = lane == slot ? (int)gi : gbat;
                    const float r = wave_transpose_reduce8(v);
                    if ((lane & 7) == 0)
                        cl[slot * kBwdComps + ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1)] = r;
                    slot++;
                    if (slot == kBwdBatch) flush();
                }
            }
            gi = gi_n; contributor = contributor_n; ra = ra_n; rc = rc_n; have = have_n;
        }
        if (slot) flush();
    }
}

__global__ void k_zero_bwd_queues(uint32_t* ctrl) {
    if (threadIdx.x < 8) ctrl[kCtrlXcdQueue + kCtrlXcdStride * threadIdx.x + kBwdQueueOffset] = 0u;
}

void launch_render_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Grads& gr, bool exact, hipStream_t s) {
    const int nwaves = d.B * d.T * kStrips;  // upper bound of the work items
    if (nwaves == 0) return;
    hipLaunchKernelGGL(k_zero_bwd_queues, dim3(1), dim3(64), 0, s, g.ctrl);
    const bool invd = gr.dL_dinvdepth != nullptr && gr.dL_dinvdepth_g != nullptr;
    const dim3 grid(min((nwaves + 3) / 4, persistent_grid(8))), blk(GSR_TILE_PIX);
    if (exact) {
        if (invd) hipLaunchKernelGGL((k_render_bwd<true, true>), grid, blk, 0, s, d, in, g, im, b, gr);
        else hipLaunchKernelGGL((k_render_bwd<true, false>), grid, blk, 0, s, d, in, g, im, b, gr);
    } else {
        if (invd) hipLaunchKernelGGL((k_render_bwd<false, true>), grid, blk, 0, s, d, in, g, im, b, gr);
        else hipLaunchKernelGGL((k_render_bwd<false, false>), grid, blk, 0, s, d, in, g, im, b, gr);
    }
}

}  // namespace gsr
