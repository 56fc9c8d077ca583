// render_bwd.hip -- back-to-front gradient replay (backward.cu:452-638 of the reference).
//
// Same math as the reference, reorganised for the matrix cores and a short per-Gaussian chain:
//  * one wave per 8x8 strip from persistent per-XCD queues (lane = pixel), replaying only the
//    Gaussians binning marked as reaching the strip, from the strip's largest n_contrib instead of
//    the tile list end;
//  * survivors go in batches of 32: the list is scanned 64 entries at a time and the strip's
//    survivors are appended to a wave-private LDS ring, so batches are full whatever the survivor
//    density; a batch's render records and feature rows are loaded while the previous batch is
//    replayed;
//  * the 32-channel "accumulated colour behind" recurrence is carried as its dot product with
//    dL/dpixel (linear: sum_ch (c - accum_rec_ch) dL_ch == g - accum_dot with g = f . dL); g for a
//    batch's 32 Gaussians x 64 pixels is ONE contraction over the channels on the matrix cores;
//  * per (pixel, Gaussian) the serial replay keeps only what depends on the pixel's transmittance:
//    alpha, T, the weight w = alpha T and u = G dL/dalpha, parked in two LDS tiles;
//  * per batch, dL/dcolor = sum_px w dL is a second matrix-core contraction, and the six other
//    per-Gaussian terms come from pixel moments of u (dL/dmean2D, dL/dconic and dL/dopacity are
//    a, b, c, o combinations of sum u, sum u dx, sum u dy, sum u dx^2, sum u dx dy, sum u dy^2 --
//    see the flush), with dL/dinvdepth = sum w dL/dinvdepth_px; the batch's atomics go out together.
//
// Both contractions run on v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation).  With the
// split-bf16 switch (gsr_set_split_bf16, SPLIT > 0) the g contraction runs on
// v_mfma_f32_32x32x8_bf16 instead: f = f_hi + f_lo and dL = d_hi + d_lo, all four products of a
// channel exact in f32 and summed in f32 (<= 3e-5 relative per product).  The features come
// pre-split (SPLIT 2: the batch-shared table of k_split_features) or are split here (SPLIT 1:
// per-frame features).
#include <cstdlib>

#include "gsr_internal.h"

namespace gsr {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uint4x __attribute__((ext_vector_type(4)));
typedef unsigned uint2x __attribute__((ext_vector_type(2)));
typedef short shortx4 __attribute__((ext_vector_type(4)));

#ifndef GSR_BWD_SLOT_GROUP
#define GSR_BWD_SLOT_GROUP 2  // measured: 1 -> 0.614, 2 -> 0.582, 4 -> 0.589 ms per 6 frames
#endif
constexpr int kBwdBatch = 32;   // survivors per batch
constexpr int kBwdPitch = 65;   // LDS row pitch (floats) of the [32][64] w / u tiles
constexpr int kBwdRing = 128;   // survivor ring entries per wave
// per wave: w tile, u tile, batch records [32][8], ring (index, position), dL/dinvdepth row [64]
constexpr int kBwdLdsWave = 2 * kBwdBatch * kBwdPitch + kBwdBatch * 8 + 2 * kBwdRing + 64;
constexpr int kBwdQueueOffset = 32;  // words after each forward XCD counter (own cache line)

// Orders this wave's LDS accesses (rocPRIM's wave_barrier): the LDS executes a wave's DS
// instructions in order, so a lane then reads what another lane of its wave wrote before.
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bf16x8 bf8(unsigned a, unsigned b, unsigned c, unsigned d) {
    return __builtin_bit_cast(bf16x8, (uint4x){a, b, c, d});
}

// 16 bytes at byte offset off of a buffer resource (zeros outside its range)
__device__ __forceinline__ float4 bwd_load16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
}

// lane l's value summed with lane l^32's
__device__ __forceinline__ float add_halves(float x) {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
}

// ABL (timing ablations only, wrong gradients): 1 = no atomics, 2 = no serial replay, 3 = no
// flush (colour MFMA, moments, atomics), 4 = no list walk beyond the ring fill (batches empty),
// 5 / 6 = VALU stand-ins for the g / the colour contraction's MFMAs
template <bool EXACT, bool INVD, int SPLIT = 0, int ABL = 0>
__global__ __launch_bounds__(GSR_TILE_PIX) __attribute__((amdgpu_waves_per_eu(2))) void k_render_bwd(
    Dims d, Inputs in, GeomArena g, ImageArena im, BinArena bn, Grads gr) {
    __shared__ float lds_all[(GSR_TILE_PIX / 64) * kBwdLdsWave];
    if (g.ctrl[kCtrlOverflow] || g.ctrl[kCtrlFwdOnly]) return;
    const uint32_t ne = g.ctrl[kCtrlNonEmpty];
    const int lane = threadIdx.x & 63;
    float* wl = lds_all + (threadIdx.x >> 6) * kBwdLdsWave;  // w tile [slot][pixel]
    float* ul = wl + kBwdBatch * kBwdPitch;                  // u tile [slot][pixel]
    float4* rl = reinterpret_cast<float4*>(ul + kBwdBatch * kBwdPitch);  // records [slot][2]
    uint32_t* ring_g = reinterpret_cast<uint32_t*>(rl + 2 * kBwdBatch);
    uint32_t* ring_p = ring_g + kBwdRing;
    float* dli_row = reinterpret_cast<float*>(ring_p + kBwdRing);  // dL/dinvdepth per strip pixel
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
            item = queue_item(q, k, ne, 0u, in.xcd_map, g.ctrl);
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
        const uint32_t* __restrict__ plist = bn.point_list + __builtin_amdgcn_readfirstlane(range.x);
        // render records and feature rows through buffer resources (32-bit offsets, range-checked)
        const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(g.rrec + (int64_t)b * d.P * 2), 0, (int)min((int64_t)d.P * 32, (int64_t)0x7FFFFFFF), 0x00020000);
        const __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc(
            SPLIT == 2 ? (void*)g.fsplit : (void*)(in.colors + in.s_colors * b), 0,
            (int)min((int64_t)d.P * GSR_C * 4, (int64_t)0x7FFFFFFF), 0x00020000);
        constexpr uint32_t kOOB = 0x80000000u;
        const int64_t gbase = (int64_t)b * d.P;
        const int64_t cbase = gr.reduce ? 0 : gbase;  // frame-reduced colour gradients: one [P][C] block
        // the flush's gradient atomics through buffer resources of this frame's rows (P < 2^24, so
        // P x 128 B fits the 32-bit range): a lane that adds nothing gets an out-of-range offset, so
        // every atomic is issued unconditionally -- no branch around it, and the compiler's memory-
        // counter waits for the next batch's loads count exactly past them instead of waiting for
        // the atomics themselves (a branch-skipped atomic makes the count unknown: vmcnt(0)-like waits)
        const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(gr.dL_dcolors + cbase * GSR_C), 0, (int)min((int64_t)d.P * GSR_C * 4, (int64_t)0x7FFFFFFF),
            0x00020000);
        const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(g.gterm + gbase * kGtWords), 0, (int)min((int64_t)d.P * kGtWords * 4, (int64_t)0x7FFFFFFF),
            0x00020000);

        const float T_final = inside ? im.final_T[pix] : 0.f;
        const uint32_t last_contributor = inside ? im.n_contrib[pix] : 0u;
        // the strip's replay length
        uint32_t ns = last_contributor;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) ns = max(ns, (uint32_t)__shfl_xor(ns, off));
        ns = __builtin_amdgcn_readfirstlane(ns);
        if (ns == 0) continue;

        // ---- per-strip operands
        float bg_dot = 0.f;
        float dL[GSR_C];
        {
            const float* bg = in.bg + in.s_bg * b;
#pragma unroll
            for (int ch = 0; ch < GSR_C; ch++) {
                dL[ch] = inside ? gr.dL_dpix[(b * GSR_C + ch) * HW + (pix - b * HW)] : 0.f;
                bg_dot += bg[ch] * dL[ch];
            }
        }
        const float dL_inv = (INVD && inside) ? gr.dL_dinvdepth[pix] : 0.f;
        // colour contraction A operands: step j covers strip pixels 2j, 2j+1; lane l holds
        // dL[pixel 2j + (l>>5)][channel l&31].  Transposed through the w tile (free until the first
        // batch).
        float adl[kBwdBatch];
        wave_lds_order();
#pragma unroll
        for (int ch = 0; ch < GSR_C; ch++) wl[ch * kBwdPitch + lane] = dL[ch];
        if (INVD) dli_row[lane] = dL_inv;
        wave_lds_order();
#pragma unroll
        for (int j = 0; j < kBwdBatch; j++) adl[j] = wl[l32 * kBwdPitch + 2 * j + hi];
        wave_lds_order();
        // g = f . dL contraction B operands: k-step k of pixel half h, lane l: dL[channel 16(l>>5) + k]
        // [pixel 32h + (l&31)] -- one swap per k turns (dL[k], dL[16+k]) into both halves' operands
        float bh0[16], bh1[16];
        // SPLIT: the g contraction's dL operands as packed bf16 (hi | lo)
        unsigned bp0[16], bp1[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dL[k]), __float_as_uint(dL[16 + k]),
                                                             false, false);
            bh0[k] = __uint_as_float(sw[0]);
            bh1[k] = __uint_as_float(sw[1]);
            if (SPLIT) {
                bp0[k] = split_hl(bh0[k]);
                bp1[k] = split_hl(bh1[k]);
            }
        }

        // ---- survivor stream: chunks of 64 list positions, last chunk first (the next lower chunk
        // prefetched); survivors appended to the ring in back-to-front order
        int base = (int)((ns - 1) & ~63u) + 64;
        // list entries through a buffer resource: the prefetch below is one unconditional load (an
        // out-of-range offset reads 0), so it lands in nidx's own register -- a conditional load
        // merged into it by a register copy would wait for the load right after issuing it
        const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)plist, 0, (int)(ns * 4u), 0x00020000);
        auto list_load = [&](int pos) {
            return __builtin_amdgcn_raw_buffer_load_b32(lrs, pos >= 0 ? (int)((uint32_t)pos * 4u) : (int)kOOB, 0, 0);
        };
        // the next two lower chunks are kept in flight (nidx, nidx2): a fill takes one or two chunks
        // (about 27 of a chunk's 64 entries reach a strip), and a chunk loaded inside the fill is
        // waited for at once -- behind the previous batch's gradient atomics, which stay counted in
        // the memory counter for thousands of cycles
        uint32_t nidx = list_load(base - 64 + lane);
        uint32_t nidx2 = list_load(base - 128 + lane);
        uint32_t head = 0, tail = 0;  // wave-uniform ring counters
        bool list_done = false;
        auto take_chunk = [&](uint32_t cidx) {
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
        };
        auto fill = [&](uint32_t want) {
            if (!list_done && tail - head < want) {
                base -= 64;
                if (base < 0) list_done = true;
                else take_chunk(nidx);
            }
            if (!list_done && tail - head < want) {
                base -= 64;
                if (base < 0) list_done = true;
                else take_chunk(nidx2);
            }
            while (!list_done && tail - head < want) {  // (rare: a third chunk, loaded here)
                base -= 64;
                if (base < 0) { list_done = true; break; }
                take_chunk(list_load(base + lane));
            }
            // the next two lower chunks, unconditional loads at the end (the same chunks again when
            // none was used), in flight until the next fill: a load merged into a register on some
            // paths only would reach it through a register copy that waits for the load at once
            __builtin_amdgcn_sched_barrier(0);
            nidx = list_load(base - 64 + lane);  // (0 below the list's start)
            nidx2 = list_load(base - 128 + lane);
            wave_lds_order();
        };
        // a batch, lane-distributed: lane l holds survivor l&31's index and list position, its
        // render record and its feature channels 16h .. 16h + 15 (h = lane half)
        auto pop = [&](uint32_t& nb_o, uint32_t& g_o, uint32_t& p_o, float4& ra_o, float4& rc_o,
                       float (&f_o)[16]) {
            nb_o = min(tail - head, (uint32_t)kBwdBatch);
            const uint32_t slot = (head + (uint32_t)l32) & (kBwdRing - 1);
            const bool valid = (uint32_t)l32 < nb_o;
            g_o = valid ? ring_g[slot] : 0u;
            p_o = valid ? ring_p[slot] : 0xFFFFFFFFu;
            head += nb_o;
            // branch-free loads (every path issues the same six, so the compiler can count them
            // in its waits): an invalid lane's offsets fall outside the resources and read zeros
            const uint32_t ro = valid ? g_o * 32u : kOOB;
            ra_o = bwd_load16(rrs, ro);
            rc_o = bwd_load16(rrs, ro + 16u);
            const uint32_t fo = valid ? g_o * (uint32_t)(GSR_C * 4) + 64u * (uint32_t)hi : kOOB;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const float4 v = bwd_load16(frs, fo + 16u * (uint32_t)u);
                f_o[4 * u] = v.x; f_o[4 * u + 1] = v.y; f_o[4 * u + 2] = v.z; f_o[4 * u + 3] = v.w;
            }
        };
        // a batch's operands; two of them, used in turn (the batch loop below is unrolled by two so
        // that each is one fixed set of registers: a rotated copy would wait for the next batch's
        // loads right after issuing them)
        struct Batch {
            uint32_t nb, g, p;
            float4 ra, rc;
            float fr[16];
        };
        Batch bA, bB;
        fill(kBwdBatch);
        pop(bA.nb, bA.g, bA.p, bA.ra, bA.rc, bA.fr);
        // as many (empty: out-of-range) atomics as a batch's flush issues, so that every path into
        // the batch loop has the same memory-counter history: the first batch's waits for its
        // loads then count past a flush's atomics as on every later entry, instead of the loop
        // head taking this path's smaller count and waiting for the previous flush's atomics
        if (ABL != 1) {
#pragma unroll
            for (int r = 0; r < 16 + 4; r++) __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(0.f, crs, (int)kOOB, 0, 0);
        }

        // strip-centred pixel offsets (exact in f32): the moments use lx = x - cx, ly = y - cy
        const float cx = (float)sx0 + 3.5f, cy = (float)sy0 + 3.5f;
        const float bg_term = -T_final * bg_dot;  // per pixel, so the background term is one fma per slot
        float T = T_final;
        float accum_dot = 0.f, last_gdot = 0.f, last_alpha = 0.f;
        float accum_inv = 0.f, last_inv = 0.f;
        auto run_batch = [&](Batch& cur, Batch& nxt) {
            // this batch's records to LDS (read back as wave-uniform values per slot), the list
            // position in the record's spare word
            if (lane < kBwdBatch) {
                rl[2 * lane] = cur.ra;
                rl[2 * lane + 1] = make_float4(cur.rc.x, cur.rc.y, cur.rc.z, __uint_as_float(cur.p));
            }
            // next batch: survivors into the ring, then its loads in flight during this batch
            fill(kBwdBatch);
            pop(nxt.nb, nxt.g, nxt.p, nxt.ra, nxt.rc, nxt.fr);

            // g[s][px] = sum_ch f_s[ch] dL[ch][px]: f32 MFMA, A = f (row s), B = dL (column px)
            floatx16 gd0, gd1;
#pragma unroll
            for (int r = 0; r < 16; r++) { gd0[r] = 0.f; gd1[r] = 0.f; }
            if (SPLIT) {
                // k-pairs (k, k+1): lane half h's four k-slots hold (d_hi, d_lo) of channels 16h + k and
                // 16h + k + 1 (B, compact: one register per channel); A repeats f_hi (then f_lo) of
                // the same channels, so two MFMAs give all four products of both channels
#pragma unroll
                for (int k = 0; k < 16; k += 2) {
                    unsigned fh0, fl0, fh1, fl1;
                    if (SPLIT == 2) {  // (hi | lo) table words -> (hi | hi), (lo | lo)
                        const unsigned t0 = __float_as_uint(cur.fr[k]), t1 = __float_as_uint(cur.fr[k + 1]);
                        fh0 = __builtin_amdgcn_perm(t0, t0, 0x01000100u);
                        fl0 = __builtin_amdgcn_perm(t0, t0, 0x03020302u);
                        fh1 = __builtin_amdgcn_perm(t1, t1, 0x01000100u);
                        fl1 = __builtin_amdgcn_perm(t1, t1, 0x03020302u);
                    } else {
                        split_hh_ll(cur.fr[k], fh0, fl0);
                        split_hh_ll(cur.fr[k + 1], fh1, fl1);
                    }
                    const shortx4 ah = __builtin_bit_cast(shortx4, (uint2x){fh0, fh1});
                    const shortx4 al = __builtin_bit_cast(shortx4, (uint2x){fl0, fl1});
                    const shortx4 b0 = __builtin_bit_cast(shortx4, (uint2x){bp0[k], bp0[k + 1]});
                    const shortx4 b1 = __builtin_bit_cast(shortx4, (uint2x){bp1[k], bp1[k + 1]});
                    gd0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(ah, b0, gd0, 0, 0, 0);
                    gd1 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(ah, b1, gd1, 0, 0, 0);
                    gd0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(al, b0, gd0, 0, 0, 0);
                    gd1 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(al, b1, gd1, 0, 0, 0);
                }
            } else
#pragma unroll
            for (int k = 0; k < 16; k++) {
                if (ABL == 5) {  /* timing ablation: VALU stand-in for the g contraction */
                    gd0[k] = fmaf(cur.fr[k], bh0[k], gd0[k]);
                    gd1[k] = fmaf(cur.fr[k], bh1[k], gd1[k]);
                } else {
                    gd0 = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.fr[k], bh0[k], gd0, 0, 0, 0);
                    gd1 = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.fr[k], bh1[k], gd1, 0, 0, 0);
                }
            }
            // to pixel lanes: gd0[r] = g of slot (r&3) + 8(r>>2), gd1[r] = of slot (r&3) + 8(r>>2) + 4
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(gd0[r]), __float_as_uint(gd1[r]),
                                                                 false, false);
                gd0[r] = __uint_as_float(sw[0]);
                gd1[r] = __uint_as_float(sw[1]);
            }
            wave_lds_order();

            // ---- serial replay of the batch, slot by slot (static slots: g lives in registers)
#pragma unroll
            for (int s = 0; s < kBwdBatch; s++) {
                // slots past the batch: skipped a group of GSR_BWD_SLOT_GROUP at a time (branches only at
                // group starts, so the scheduler sees whole groups); inside a group `act` drops them
                if (ABL == 2) continue;
                if (GSR_BWD_SLOT_GROUP == 1) {
                    if ((uint32_t)s >= cur.nb) continue;  // (not break: this loop must unroll -- static slots)
                } else if ((s % GSR_BWD_SLOT_GROUP) == 0 && (uint32_t)s >= cur.nb) {
                    break;
                }
                const float gdot = (s & 4) ? gd1[(s & 3) + 4 * (s >> 3)] : gd0[(s & 3) + 4 * (s >> 3)];
                const float4 ra = rl[2 * s], rc = rl[2 * s + 1];  // x, y, opacity, 1/depth | -a/2, -b, -c/2, pos
                const uint32_t contributor = __float_as_uint(rc.w);
                const float dx = ra.x - pfx, dy = ra.y - pfy;
                // branch-free: every lane evaluates, `act` selects
                const float power = blend_power(rc.x, rc.y, rc.z, dx, dy);
                // alpha exactly as the forward's alpha_of (render_fwd.hip); power < -87 never blends
                float G, alpha;
                if constexpr (EXACT) {
                    float q;
                    int k;
                    blend_parts(power, q, k);
                    G = blend_G(q, k);
                    alpha = fminf(0.99f, blend_oexp(ra.z, q, k));
                } else {
                    G = expf_fast(power);
                    alpha = fminf(0.99f, ra.z * G);
                }
                const bool act = (GSR_BWD_SLOT_GROUP == 1 || (uint32_t)s < cur.nb) &&
                                 contributor < last_contributor && !(power > 0.0f) &&  // (outside: last 0)
                                 !(power < -87.0f) && !(alpha < 1.0f / 255.0f);
                const float one_m = 1.f - alpha;
                const float rinv1m = __builtin_amdgcn_rcpf(one_m);
                // T / (1 - alpha): reciprocal + one Newton step on the quotient (<= 1 ulp)
                float Tq = T * rinv1m;
                Tq = fmaf(fmaf(-Tq, one_m, T), rinv1m, Tq);
                T = act ? Tq : T;
                const float wgt = act ? alpha * T : 0.f;
                // the reference's recurrence a' = la * lg + (1 - la) a (backward.cu:532-537), as a + la (lg - a)
                const float acc_n = fmaf(last_alpha, last_gdot - accum_dot, accum_dot);
                accum_dot = act ? acc_n : accum_dot;
                last_gdot = act ? gdot : last_gdot;
                float dL_dalpha = gdot - accum_dot;
                if (INVD) {
                    const float ai_n = fmaf(last_alpha, last_inv - accum_inv, accum_inv);
                    accum_inv = act ? ai_n : accum_inv;
                    last_inv = act ? ra.w : last_inv;
                    dL_dalpha = fmaf(ra.w - accum_inv, dL_inv, dL_dalpha);
                }
                dL_dalpha *= T;
                last_alpha = act ? alpha : last_alpha;
                dL_dalpha = fmaf(bg_term, rinv1m, dL_dalpha);  // + (-T_final / (1 - alpha)) bg . dL
                // u = G dL/dalpha (0 where the pixel does not take the Gaussian; G may be inf there)
                const float u = act ? G * dL_dalpha : 0.f;
                wl[s * kBwdPitch + lane] = wgt;
                ul[s * kBwdPitch + lane] = u;
                // GSR_BWD_SLOT_GROUP slots per scheduling region: the next slot's transmittance-free
                // part (power, exp, alpha) may overlap this slot's serial tail
                if ((s % GSR_BWD_SLOT_GROUP) == GSR_BWD_SLOT_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
            }
            wave_lds_order();

            // ---- flush: dL/dcolor[s][ch] = sum_px w[s][px] dL[px][ch] on the matrix cores (slot rows,
            // channel columns: each register's atomics cover two whole 128-byte feature rows)
            if (ABL == 3) {
#pragma unroll
                for (int u = 0; u < 16; u++) nxt.fr[u] += gd0[u] + gd1[u];
                return; }
            floatx16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
            for (int j = 0; j < kBwdBatch; j++) {
                const float w = wl[l32 * kBwdPitch + 2 * j + hi];
                if (ABL == 6) acc[j & 15] = fmaf(w, adl[j], acc[j & 15]);  /* timing ablation */
                else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w, adl[j], acc, 0, 0, 0);
            }
            // pixel moments of u for slot l&31 over this lane half's 32 pixels (strip rows 4h..4h+3):
            // lx = (i % 8) - 3.5, ly = (i / 8) - 3.5 + 4h
            float S0 = 0.f, Sx = 0.f, Sy = 0.f, Sxx = 0.f, Sxy = 0.f, Syy = 0.f, Si = 0.f;
#pragma unroll 1
            for (int row = 0; row < 4; row++) {  // one strip row (8 pixels) at a time
                const float ly = (float)row - 3.5f;
                const float* urow = ul + l32 * kBwdPitch + 32 * hi + 8 * row;
                const float* wrow = wl + l32 * kBwdPitch + 32 * hi + 8 * row;
                float r0 = 0.f, rx = 0.f, rxx = 0.f, ri = 0.f;
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    const float lx = (float)c - 3.5f;
                    const float uu = urow[c];
                    r0 += uu;
                    rx = fmaf(uu, lx, rx);
                    rxx = fmaf(uu, lx * lx, rxx);
                    if (INVD) ri = fmaf(wrow[c], dli_row[32 * hi + 8 * row + c], ri);
                }
                S0 += r0;
                Sx += rx;
                Sxx += rxx;
                Sy = fmaf(r0, ly, Sy);
                Sxy = fmaf(rx, ly, Sxy);
                Syy = fmaf(r0, ly * ly, Syy);
                Si += ri;
            }
            if (hi) {  // rows 4..7: ly = ly_i + 4
                Syy = fmaf(8.f, Sy, fmaf(16.f, S0, Syy));
                Sxy = fmaf(4.f, Sx, Sxy);
                Sy = fmaf(4.f, S0, Sy);
            }
            S0 = add_halves(S0); Sx = add_halves(Sx); Sy = add_halves(Sy);
            Sxx = add_halves(Sxx); Sxy = add_halves(Sxy); Syy = add_halves(Syy);
            if (INVD) Si = add_halves(Si);
            wave_lds_order();
            // acc[r] at lane l: channel l&31 of the batch's slot (r&3) + 8(r>>2) + 4(l>>5)
            if (ABL != 1) {
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const uint32_t sl = (uint32_t)((r & 3) + 8 * (r >> 2) + 4 * hi);
                    const uint32_t gsl = __builtin_amdgcn_readlane(cur.g, (r & 3) + 8 * (r >> 2)) ;
                    const uint32_t gsh = __builtin_amdgcn_readlane(cur.g, (r & 3) + 8 * (r >> 2) + 4);
                    const uint32_t gs = hi ? gsh : gsl;
                    // slots past the batch hold stale tiles; a zero sum (no pixel took the Gaussian,
                    // or no gradient) adds nothing: those lanes' offsets fall outside the resource
                    const uint32_t off = (sl < cur.nb && acc[r] != 0.f) ? (gs * GSR_C + (uint32_t)l32) * 4u : kOOB;
                    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(acc[r], crs, (int)off, 0, 0);
                }
            }
            // the other terms of slot l&31, from the pixel moments of u about the Gaussian's centre
            // (dx = X - lx, dy = Y - ly); lanes 0-31 write the slot's kGtWords row to LDS (the record
            // tile is free now), then 8 lanes per slot add it to the slot's gterm row
            {
                const float X = cur.ra.x - cx, Y = cur.ra.y - cy;
                const float Sdx = X * S0 - Sx;
                const float Sdy = Y * S0 - Sy;
                const float Sdxx = (X * X) * S0 - 2.f * X * Sx + Sxx;
                const float Sdxy = (X * Y) * S0 - X * Sy - Y * Sx + Sxy;
                const float Sdyy = (Y * Y) * S0 - 2.f * Y * Sy + Syy;
                const float o = cur.ra.z;
                const float ca = -2.0f * cur.rc.x, cb = -cur.rc.y, cc = -2.0f * cur.rc.z;  // conic a, b, c (exact)
                float* row = reinterpret_cast<float*>(rl) + 8 * l32;
                if (!hi) {
                    // dL/dmean2D = sum dL/dG dG/ddelx ddelx/dx, dG/ddelx = -G (a dx + b dy)
                    // (backward.cu:597-627); dL/dconic = -1/2 o sum u (dx^2, dx dy, dy^2)
                    row[kGtM2x] = -o * ddelx_dx * (ca * Sdx + cb * Sdy);
                    row[kGtM2y] = -o * ddely_dy * (cc * Sdy + cb * Sdx);
                    row[kGtCx] = -0.5f * o * Sdxx;
                    row[kGtCy] = -0.5f * o * Sdxy;
                } else {
                    row[kGtCw] = -0.5f * o * Sdyy;
                    row[kGtOp] = S0;  // dL/dopacity = sum G dL/dalpha
                    row[kGtInv] = Si;
                    row[7] = 0.f;
                }
            }
            wave_lds_order();
            if (ABL != 1) {
                const float* rows = reinterpret_cast<const float*>(rl);
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    const uint32_t sl = (uint32_t)(8 * qq + (lane >> 3));
                    const uint32_t gs = (uint32_t)__shfl((int)cur.g, (int)sl);
                    const float val = rows[8 * sl + (lane & 7)];
                    const bool add = sl < cur.nb && val != 0.f && (lane & 7) != 7 && (INVD || (lane & 7) != kGtInv);
                    const uint32_t off = add ? (gs * (uint32_t)kGtWords + (uint32_t)(lane & 7)) * 4u : kOOB;
                    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(val, grs, (int)off, 0, 0);
                }
            }
            wave_lds_order();

        };
        for (;;) {
            if (!bA.nb) break;
            run_batch(bA, bB);
            if (!bB.nb) break;
            run_batch(bB, bA);
        }
    }
}

__global__ void k_zero_bwd_queues(uint32_t* ctrl) {
    if (threadIdx.x < 8) ctrl[kCtrlXcdQueue + kCtrlXcdStride * threadIdx.x + kBwdQueueOffset] = 0u;
}

void launch_render_bwd(const Dims& d, const Inputs& in_, const GeomArena& g, const ImageArena& im_,
                       const BinArena& b, const Grads& gr, bool exact, bool split, hipStream_t s) {
    Inputs in = in_;  // one frame: strip_list is one longest-first list (launch_strip_order)
    if (d.B == 1 && in.xcd_map == 2u) in.xcd_map = 1u;
    // The forward's block-affine segments cost the backward 8%: it walks a tile-affine list of its
    // own (one longest-first list, built here from the forward's strip counts, ~10 us);
    // GSR_BWD_TILE_LIST=0 walks the forward's segments
    static const bool own_list = tune_env("GSR_BWD_TILE_LIST", 1) != 0;
    ImageArena im = im_;
    if (in.xcd_map == 2u && own_list) {
        launch_strip_list_tile(d, im_, im_.strip_list_bwd, s);
        im.strip_list = im_.strip_list_bwd;
        in.xcd_map = 1u;
    }
    const int nwaves = d.B * d.T * kStrips;  // upper bound of the work items
    if (nwaves == 0) return;
    hipLaunchKernelGGL(k_zero_bwd_queues, dim3(1), dim3(64), 0, s, g.ctrl);
    hipMemsetAsync(g.gterm, 0, (size_t)d.B * d.P * kGtWords * sizeof(float), s);
    const bool invd = gr.invd != 0;
    // GSR_BWD_WG_PER_CU (A/B): 1 halves the residency (one wave per SIMD), what an LDS row cache
    // for a tile-merged write-back would cost at this register and LDS budget
    static const int wg_per_cu = tune_env("GSR_BWD_WG_PER_CU", 2);
    const dim3 grid(min((nwaves + 3) / 4, persistent_grid(wg_per_cu))), blk(GSR_TILE_PIX);
#ifdef GSR_TUNING
    // timing ablations (wrong gradients by construction): tools/build_ab.py builds only
    static const int ablate = tune_env("GSR_BWD_ABLATE", 0);
    if (ablate >= 1 && ablate <= 6 && exact && invd) {
        if (ablate == 1) hipLaunchKernelGGL((k_render_bwd<true, true, 0, 1>), grid, blk, 0, s, d, in, g, im, b, gr);
        if (ablate == 2) hipLaunchKernelGGL((k_render_bwd<true, true, 0, 2>), grid, blk, 0, s, d, in, g, im, b, gr);
        if (ablate == 3) hipLaunchKernelGGL((k_render_bwd<true, true, 0, 3>), grid, blk, 0, s, d, in, g, im, b, gr);
        if (ablate == 5) hipLaunchKernelGGL((k_render_bwd<true, true, 0, 5>), grid, blk, 0, s, d, in, g, im, b, gr);
        if (ablate == 6) hipLaunchKernelGGL((k_render_bwd<true, true, 0, 6>), grid, blk, 0, s, d, in, g, im, b, gr);
        return;
    }
#endif
    // split-bf16 contractions; one feature table for the batch is split once (into the forward's
    // fsplit rows, which this launch owns until it ends)
    // GSR_BWD_SPLIT=0: f32 contractions even with the split switch on (A/B)
    static const bool bwd_split = tune_env("GSR_BWD_SPLIT", 1) != 0;
    int sp = 0;
    if (split && bwd_split) {
        sp = 1;
        if (in.s_colors == 0) {
            launch_split_features(d.P, in.colors, g.fsplit, s);
            sp = 2;
        }
    }
#define GSR_BWD(E, I, S) hipLaunchKernelGGL((k_render_bwd<E, I, S>), grid, blk, 0, s, d, in, g, im, b, gr)
#define GSR_BWD_S(E, I) { if (sp == 2) GSR_BWD(E, I, 2); else if (sp == 1) GSR_BWD(E, I, 1); else GSR_BWD(E, I, 0); }
    if (exact) {
        if (invd) GSR_BWD_S(true, true) else GSR_BWD_S(true, false)
    } else {
        if (invd) GSR_BWD_S(false, true) else GSR_BWD_S(false, false)
    }
#undef GSR_BWD_S
#undef GSR_BWD
}

}  // namespace gsr
