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
// pixels).  No workgroup barriers: the LDS is wave-private.
//
// Survivors are processed in batches of 32 (back to front):
//  * the list is scanned 64 entries at a time and the strip's survivors are appended to a
//    wave-private LDS ring (slot = rank of the entry among the chunk's survivors), so batches are
//    full whatever the survivor density;
//  * a batch's render records and feature rows are loaded lane-distributed (lane s: survivor s)
//    while the PREVIOUS batch is replayed, so their latency hides behind a whole batch;
//  * g = f . dL (the colour term of dL/dalpha) for the batch's 32 Gaussians x 64 pixels is one
//    f32 MFMA contraction over the 32 channels (16 v_mfma_f32_32x32x2_f32 per pixel half, exact
//    f32 products), one v_permlane32_swap per register puts each pixel's 32 values in its lane;
//  * the serial replay then needs per survivor only its record fields (v_readlane from the
//    lane-distributed batch) and the pixel's g from a register.
constexpr int kBwdQueueOffset = 32;  // words after each forward XCD counter (own cache line)
constexpr int kBwdRing = 128;        // survivor ring entries per wave (LDS)

template <bool EXACT, bool INVD>
__global__ __launch_bounds__(GSR_TILE_PIX) __attribute__((amdgpu_waves_per_eu(2))) void k_render_bwd(
    Dims d, Inputs in, GeomArena g, ImageArena im, BinArena bn, Grads gr) {
    __shared__ float lds_all[(GSR_TILE_PIX / 64) * (kBwdLdsWave + 2 * kBwdRing)];
    if (g.ctrl[kCtrlOverflow]) return;
    const uint32_t ne = g.ctrl[kCtrlNonEmpty];
    const int lane = threadIdx.x & 63;
    float* wl = lds_all + (threadIdx.x >> 6) * (kBwdLdsWave + 2 * kBwdRing);  // this wave's [32][65] tile
    float* cl = wl + kBwdBatch * kBwdPitch;                    // its [32][8] term slots
    uint32_t* ring_g = reinterpret_cast<uint32_t*>(cl + kBwdBatch * kBwdComps);  // survivor ring
    uint32_t* ring_p = ring_g + kBwdRing;
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

        // colour-gradient MFMA A operands: step j covers strip pixels 2j, 2j+1; lane l holds
        // dL[pixel 2j + (l>>5)][channel l&31].  Transposed through the LDS tile.
        float adl[kBwdBatch];
        wave_lds_order();
#pragma unroll
        for (int ch = 0; ch < GSR_C; ch++) wl[ch * kBwdPitch + lane] = dL[ch];
        wave_lds_order();
#pragma unroll
        for (int j = 0; j < kBwdBatch; j++) adl[j] = wl[l32 * kBwdPitch + 2 * j + hi];
        wave_lds_order();
        // g = f . dL MFMA B operands: k-step k of pixel half h, lane l: dL[channel 16(l>>5) + k]
        // [pixel 32h + (l&31)] -- one swap per k turns (dL[k], dL[16+k]) into the two halves' operands
        float bh0[16], bh1[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dL[k]), __float_as_uint(dL[16 + k]),
                                                             false, false);
            bh0[k] = __uint_as_float(sw[0]);
            bh1[k] = __uint_as_float(sw[1]);
        }

        // ---- survivor stream: chunks of 64 list positions, last chunk first (the next lower chunk
        // prefetched); survivors appended to the ring in back-to-front order
        int base = (int)((ns - 1) & ~63u) + 64;
        uint32_t nidx = base - 64 + lane < (int)ns ? plist[base - 64 + lane] : 0u;
        uint32_t head = 0, tail = 0;  // wave-uniform ring counters
        bool list_done = false;
        auto fill = [&](uint32_t want) {
            while (!list_done && tail - head < want) {
                base -= 64;
                if (base < 0) { list_done = true; break; }
                const uint32_t cidx = nidx;
                if (base >= 64) nidx = plist[base - 64 + lane];
                const bool sv = base + lane < (int)ns && (cidx & smask_bit) != 0u;
                const uint64_t m = __ballot(sv);
                if (sv) {
                    // rank among the chunk's survivors counted from the back (higher positions first)
                    const uint32_t above = lane == 63 ? 0u : (uint32_t)__popcll(m >> (lane + 1));
                    const uint32_t slot = (tail + above) & (kBwdRing - 1);
                    ring_g[slot] = cidx & kIndexMask;
                    ring_p[slot] = (uint32_t)(base + lane);
                }
                tail += (uint32_t)__popcll(m);
            }
            wave_lds_order();
        };
        // a batch, lane-distributed: lane l holds survivor l&31's index / position, its render
        // record (both halves) and 16 channels 16(l>>5).. of its feature row
        uint32_t nb = 0, bg_ = 0, bp_ = 0;
        float4 ra_ = make_float4(0.f, 0.f, 0.f, 0.f), rc_ = ra_;
        float fr[16];
        auto pop = [&](uint32_t& nb_o, uint32_t& g_o, uint32_t& p_o, float4& ra_o, float4& rc_o, float (&f_o)[16]) {
            nb_o = min(tail - head, (uint32_t)kBwdBatch);
            const uint32_t slot = (head + (uint32_t)l32) & (kBwdRing - 1);
            const bool valid = (uint32_t)l32 < nb_o;
            g_o = valid ? ring_g[slot] : 0u;
            p_o = valid ? ring_p[slot] : 0xFFFFFFFFu;
            head += nb_o;
            if (valid) {
                ra_o = rrec[2 * g_o];
                rc_o = rrec[2 * g_o + 1];
                const float4* fsrc = reinterpret_cast<const float4*>(colors + (int64_t)g_o * GSR_C + 16 * hi);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float4 v = fsrc[u];
                    f_o[4 * u] = v.x; f_o[4 * u + 1] = v.y; f_o[4 * u + 2] = v.z; f_o[4 * u + 3] = v.w;
                }
            } else {
                ra_o = make_float4(0.f, 0.f, 0.f, 0.f);
                rc_o = ra_o;
#pragma unroll
                for (int u = 0; u < 16; u++) f_o[u] = 0.f;
            }
        };
        fill(kBwdBatch);
        pop(nb, bg_, bp_, ra_, rc_, fr);

        float T = T_final;
        float accum_dot = 0.f, last_gdot = 0.f, last_alpha = 0.f;
        float accum_inv = 0.f, last_inv = 0.f;
        while (nb) {
            // next batch: survivors into the ring, then its loads in flight during this batch
            uint32_t nb_n, bg_n, bp_n;
            float4 ra_n, rc_n;
            float fr_n[16];
            fill(kBwdBatch);
            pop(nb_n, bg_n, bp_n, ra_n, rc_n, fr_n);

            // g[s][px] = sum_ch f_s[ch] dL[ch][px] for the batch (rows s, columns px of each half)
            floatx16 gd0, gd1;
#pragma unroll
            for (int r = 0; r < 16; r++) { gd0[r] = 0.f; gd1[r] = 0.f; }
#pragma unroll
            for (int k = 0; k < 16; k++) {
                gd0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[k], bh0[k], gd0, 0, 0, 0);
                gd1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[k], bh1[k], gd1, 0, 0, 0);
            }
            // to pixel lanes: gd0[r] = g of slot (r&3) + 8(r>>2), gd1[r] = of slot (r&3) + 8(r>>2) + 4
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(gd0[r]), __float_as_uint(gd1[r]),
                                                                 false, false);
                gd0[r] = __uint_as_float(sw[0]);
                gd1[r] = __uint_as_float(sw[1]);
            }

            // serial replay of the batch, slot by slot (static slots: g lives in registers)
#pragma unroll
            for (int s = 0; s < kBwdBatch; s++) {
                if ((uint32_t)s >= nb) continue;  // (not break: the loop must unroll -- static slots)
                const float gdot = (s & 4) ? gd1[(s & 3) + 4 * (s >> 3)] : gd0[(s & 3) + 4 * (s >> 3)];
                const uint32_t contributor = __builtin_amdgcn_readlane(bp_, s);
                // record: x, y, opacity, 1/depth | -a/2, -b, -c/2
                const float rx = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ra_.x), s));
                const float ry = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ra_.y), s));
                const float ro = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ra_.z), s));
                const float rinv = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ra_.w), s));
                const float qa = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rc_.x), s));
                const float qb = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rc_.y), s));
                const float qc = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rc_.z), s));
                const float dx = rx - pfx, dy = ry - pfy;
                // branch-free: every lane evaluates, `act` selects (the divergent form costs exec
                // juggling around every step and saves nothing -- both sides run anyway)
                const float power = blend_power(qa, qb, qc, dx, dy);
                const float G = blend_exp<EXACT>(power);
                const float alpha = fminf(0.99f, ro * G);
                const bool act = inside && contributor < last_contributor && !(power > 0.0f) &&
                                 !(alpha < 1.0f / 255.0f);
                const float one_m = 1.f - alpha;
                const float rinv1m = __builtin_amdgcn_rcpf(one_m);
                // T / (1 - alpha): reciprocal + one Newton step on the quotient (<= 1 ulp)
                float Tq = T * rinv1m;
                Tq = fmaf(fmaf(-Tq, one_m, T), rinv1m, Tq);
                T = act ? Tq : T;
                const float wgt = act ? alpha * T : 0.f;
                const float acc_n = last_alpha * last_gdot + (1.f - last_alpha) * accum_dot;
                accum_dot = act ? acc_n : accum_dot;
                last_gdot = act ? gdot : last_gdot;
                float dL_dalpha = gdot - accum_dot;
                float v[8];
                v[7] = 0.f;
                v[6] = 0.f;
                if (INVD) {
                    const float ai_n = last_alpha * last_inv + (1.f - last_alpha) * accum_inv;
                    accum_inv = act ? ai_n : accum_inv;
                    last_inv = act ? rinv : last_inv;
                    dL_dalpha += (rinv - accum_inv) * dL_inv;
                    v[6] = wgt * dL_inv;
                }
                dL_dalpha *= T;
                last_alpha = act ? alpha : last_alpha;
                dL_dalpha += (-T_final * rinv1m) * bg_dot;
                dL_dalpha = act ? dL_dalpha : 0.f;
                {
                    const float Ga = act ? G : 0.f;  // inactive lanes: every term exactly 0 (G may be inf)
                    const float ca = -2.0f * qa, cb = -qb, cc = -2.0f * qc;  // exact
                    const float dL_dG = ro * dL_dalpha;
                    const float gdx = Ga * dx;
                    const float gdy = Ga * dy;
                    const float dG_ddelx = -gdx * ca - gdy * cb;
                    const float dG_ddely = -gdy * cc - gdx * cb;
                    v[0] = dL_dG * dG_ddelx * ddelx_dx;
                    v[1] = dL_dG * dG_ddely * ddely_dy;
                    v[2] = -0.5f * gdx * dx * dL_dG;
                    v[3] = -0.5f * gdx * dy * dL_dG;
                    v[4] = -0.5f * gdy * dy * dL_dG;
                    v[5] = Ga * dL_dalpha;
                }
                // weights and the 7 reduced terms parked in LDS; the atomics go out with the batch
                wl[s * kBwdPitch + lane] = wgt;
                float r = 0.f;
                if (__any(act)) r = wave_transpose_reduce8(v);
                if ((lane & 7) == 0)
                    cl[s * kBwdComps + ((lane >> 5) & 1) * 4 + ((lane >> 4) & 1) * 2 + ((lane >> 3) & 1)] = r;
            }

            // ---- flush: dL/dcolor = sum_px w dL on the matrix cores, then the batch's atomics
            wave_lds_order();
            floatx16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
            for (int j = 0; j < kBwdBatch; j++) {
                const float w = (uint32_t)l32 < nb ? wl[l32 * kBwdPitch + 2 * j + hi] : 0.f;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(adl[j], w, acc, 0, 0, 0);
            }
            wave_lds_order();
            // acc[r] at lane l: channel (r&3) + 8(r>>2) + 4(l>>5) of the batch's Gaussian l&31
            if ((uint32_t)l32 < nb) {
                const int64_t gg = gbase + bg_;
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

            nb = nb_n; bg_ = bg_n; bp_ = bp_n; ra_ = ra_n; rc_ = rc_n;
#pragma unroll
            for (int u = 0; u < 16; u++) fr[u] = fr_n[u];
        }
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
    const dim3 grid(min((nwaves + 3) / 4, persistent_grid(2))), blk(GSR_TILE_PIX);
    if (exact) {
        if (invd) hipLaunchKernelGGL((k_render_bwd<true, true>), grid, blk, 0, s, d, in, g, im, b, gr);
        else hipLaunchKernelGGL((k_render_bwd<true, false>), grid, blk, 0, s, d, in, g, im, b, gr);
    } else {
        if (invd) hipLaunchKernelGGL((k_render_bwd<false, true>), grid, blk, 0, s, d, in, g, im, b, gr);
        else hipLaunchKernelGGL((k_render_bwd<false, false>), grid, blk, 0, s, d, in, g, im, b, gr);
    }
}

}  // namespace gsr
