// render_fwd.hip -- front-to-back alpha compositing of 32-channel features (forward.cu:274-397 of
// the reference).
//
// Structure (gfx950):
//  * The unit of work is one 64-pixel strip (8x8, strip_origin) of a 16x16 tile, owned by ONE wave
//    (lane = pixel).  Waves dequeue strips independently from eight per-XCD queues (queue_item), so
//    there is no workgroup barrier anywhere: a wave whose pixels all finished moves on at once.
//  * The wave walks the tile's depth-sorted list 64 entries at a time (one coalesced load of indices
//    and strip masks).  The binning pass already decided, with an exact conservative
//    ellipse/rectangle test, whether each Gaussian can reach alpha >= 1/255 anywhere in each strip;
//    one ballot over the strip bit gives the chunk's survivors.  A culled pair cannot change any
//    blend decision, so the result is identical to visiting every pair.
//  * Survivors are taken two at a time in list order (one MFMA k-step) through a three-slot
//    software pipeline: the records and feature words of step s+2 load while step s+1's alphas
//    (the exp-heavy, transmittance-independent part) are computed and step s's serial blend runs.
//    Each lane runs the branch-free blend step for its pixel (the 1/255 skip, the T < 1e-4 stop,
//    n_contrib), giving the weight w = alpha T (0 where the pixel does not take the Gaussian).  The
//    32-channel accumulation C += f w runs on the matrix cores as D[ch][px] += F[ch][k] W[k][px]
//    with v_mfma_f32_32x32x2_f32 over the strip's two 32-pixel halves (lanes 0-31 carry one
//    Gaussian's 128-byte feature row, lanes 32-63 the other's).  The f32 MFMA is an exact k-ordered
//    fma chain, i.e. bit-identical to fmaf(f, w, C) Gaussian by Gaussian (the oracle's contract); a
//    zero weight leaves the accumulator unchanged.
//  * One frame (the per-frame drop-in path): every strip is two work items, one wave per 32-pixel
//    half, each lane computing ONE alpha per k-step (HALF below): the longest strip's chain is what
//    sets a single frame's time.
//
// Roofline: per frame the kernel must read 156 B per visible Gaussian (features + 2D attributes)
// and write 140 B per pixel (32 channels, inverse depth, final_T, n_contrib).
#include "gsr_cull.h"
#include "gsr_internal.h"

namespace gsr {

// A k-step's two render records reach the wave through a per-wave LDS slot: lanes 0..7 load dword
// `lane` of record a and of record b (4-B vector loads, the record offsets in SGPRs), write them with
// one ds_write2 and every lane reads them back as uniform-address ds_read_b128.  (Wave-uniform 16-B
// vector loads, scalar loads and a v_readlane broadcast were measured and dropped: DESIGN.md §5.1, §7.)
#ifndef GSR_LDS_EARLY
#define GSR_LDS_EARLY 1  // record LDS reads of the next slot issued before this slot's blend
#endif
#ifndef GSR_PAD_SALU
#define GSR_PAD_SALU 0  // instrumentation: extra SALU per k-step (A/B builds)
#endif
#ifndef GSR_PAD_VALU
#define GSR_PAD_VALU 0  // instrumentation: extra VALU per k-step (A/B builds)
#endif
#ifndef GSR_BATCH_NSLOT
#define GSR_BATCH_NSLOT 3  // pipeline slots of the batched (throughput) kernels
#endif

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned uint4x __attribute__((ext_vector_type(4)));
typedef unsigned uint2x __attribute__((ext_vector_type(2)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// The blend step of forward.cu:349-381 split in two (both halves are branch-free):
//  * alpha_of: the pixel-local alpha of one Gaussian, independent of the pixel's transmittance, with
//    the `power > 0` skip folded in as alpha = 0 (0 < 1/255 is never taken; a NaN power still gives
//    alpha = min(0.99, NaN) = 0.99 as in the reference) -- computed one step ahead;
//  * take_step: the serial part on the pixel's state (the 1/255 skip, the T < 1e-4 stop, the
//    weight alpha*T, inverse depth, last contributor = 1-based list position, done flag).
template <bool EXACT>
__device__ __forceinline__ float alpha_of(const float4 ga, const float4 gc, float pfx, float pfy) {
    const float dx = ga.x - pfx, dy = ga.y - pfy;
    const float power = blend_power(gc.x, gc.y, gc.z, dx, dy);
    float alpha;
    if constexpr (EXACT) {
        float q;
        int k;
        blend_parts(power, q, k);
        alpha = fminf(0.99f, blend_oexp(ga.z, q, k));
    } else {
        alpha = fminf(0.99f, ga.z * expf_fast(power));
    }
    // power < -87: exp < 2e-38, alpha < 1/255 -- never taken, as in the reference
    return (power > 0.0f || power < -87.0f) ? 0.0f : alpha;
}

// With eff = alpha where the pixel takes the Gaussian (alpha >= 1/255, not done) and 0 elsewhere,
// test_T = T (1 - eff) equals T where nothing is taken, and a live pixel always has T >= 1e-4 (T
// only drops to a test_T that passed the stop test), so `test_T < 1e-4` alone is the stop test:
// the same decisions and the same products as forward.cu:352-381 with fewer lane-mask operations.
__device__ __forceinline__ float take_step(float alpha, float inv_depth, uint32_t pos, float& T, float& invd,
                                           uint32_t& last, bool& done) {
    const bool take = !done && !(alpha < 1.0f / 255.0f);
    const float eff = take ? alpha : 0.0f;
    const float test_T = T * (1.0f - eff);
    const bool term = test_T < 0.0001f;
    const bool contrib = take && !term;
    const float w = contrib ? eff * T : 0.0f;
    invd = fmaf(inv_depth, w, invd);
    T = contrib ? test_T : T;
    last = contrib ? pos : last;
    done = done || term;
    return w;
}

// Split-bf16 accumulation (gsr_set_split_bf16): f = f_hi + f_lo with f_hi = bf16_rne(f),
// f_lo = bf16_rne(f - f_hi); the four bf16 products f_hi.w_hi + f_lo.w_hi + f_hi.w_lo + f_lo.w_lo
// are exact in f32, so the only loss is the split residual (|f - f_hi - f_lo| <= 2^-17 |f|, the same
// for w): <= 3e-5 relative per product, summed under sum(w) <= 1.  One v_mfma_f32_32x32x16_bf16
// (8 passes) replaces the 16-pass f32 MFMA per pixel half.
// The split of a batch-shared feature table, once per launch (P x 32 words; render_fwd then loads
// the packed word in place of the f32 feature).
__global__ __launch_bounds__(256) void k_split_features(int n4, const float4* __restrict__ f,
                                                        uint4* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;  // 4 features per thread (rows are 32 floats)
    if (i < n4) {
        const float4 v = f[i];
        out[i] = make_uint4(split_hl(v.x), split_hl(v.y), split_hl(v.z), split_hl(v.w));
    }
}

// one 16-byte half of a render record at a wave-uniform byte offset (voffset, so that the range
// check turns the null index P into zeros)
// A wave-uniform 64-bit mask with bit i cleared: one s_bitset0_b64 (mask &= mask - 1 is three SALU:
// a 64-bit subtract and an and).
__device__ __forceinline__ uint64_t clear_bit(uint64_t m, int i) {
    asm("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(i));
    return m;
}

__device__ __forceinline__ float4 rec_load(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
}

// Epilogue of one strip: final_T, n_contrib, inverse depth (lane = pixel) and the 32
// channel-major colour rows C + T*bg from the MFMA accumulators.  acc_n[r] at lane l holds channel
// (r&3)+8*(r>>2)+4*(l>>5) of strip pixel 32n + (l&31), whose transmittance lives in lane 32n + (l&31).
// REFINE (gsr_forward_batch_refine): the features were pre-contracted by gsr_refine_prepare, so
// channels [keep, keep + n_out) already hold the refiner head's 1x1 conv W.(C + T bg); they get the
// bias and the leaky ReLU here and go to out_refine, channels [0, keep) to out_color, the rest
// nowhere.  No extra registers: the blend loop is the same kernel.
template <bool EMPTY, bool REFINE>
__device__ __forceinline__ void store_strip(const Dims& d, const ImageArena& im, const Outputs& o,
                                            const float* bg, int b, int sx0, int sy0, int lane,
                                            const floatx16& acc0, const floatx16& acc1, float T,
                                            float invd, uint32_t last) {
    const int64_t HW = (int64_t)d.H * d.W;
    const int px = sx0 + lane % kStripW;
    const int py = sy0 + lane / kStripW;
    if (px < d.W && py < d.H) {
        const int64_t pix = b * HW + (int64_t)py * d.W + px;
        im.final_T[pix] = T;
        im.n_contrib[pix] = last;
        if (o.out_invdepth) o.out_invdepth[pix] = invd;
    }
    const float T0 = __shfl(T, lane & 31);
    const float T1 = __shfl(T, 32 + (lane & 31));
    // the background: one load of bg[lane % 32], then each register's channel (which differs
    // between the half-waves) by ds_bpermute -- a per-lane `hi ? bg[c + 4] : bg[c]` compiled to 16
    // dependent global loads, each waited for before its stores
    const float bgl = bg[lane & 31];
    // channel rows through a buffer resource: one VGPR byte offset per half-strip row, the channel
    // offset in an SGPR; pixels outside the image get an offset past the buffer and are dropped
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        o.out_color + (int64_t)b * GSR_C * HW, 0, (int)((int64_t)GSR_C * HW * 4), 0x00020000);
    const int j = lane & 31;
    const int qx = sx0 + j % kStripW;
    const int qy0 = sy0 + j / kStripW;
    const int qy1 = qy0 + 32 / kStripW;  // the upper 32 pixels of the strip
    const int hi = lane >> 5;
    const int hoff = hi * 4 * (int)HW;  // channels +4 for the upper half-wave
    const int v0 = (qx < d.W && qy0 < d.H) ? (hoff + qy0 * d.W + qx) * 4 : 0x7FFFFFF0;
    const int v1 = (qx < d.W && qy1 < d.H) ? (hoff + qy1 * d.W + qx) * 4 : 0x7FFFFFF0;
    __amdgpu_buffer_rsrc_t rr = rs;
    if (REFINE)
        rr = __builtin_amdgcn_make_buffer_rsrc(o.out_refine + (int64_t)b * o.n_out * HW, 0,
                                               (int)((int64_t)o.n_out * HW * 4), 0x00020000);
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int c = (r & 3) + 8 * (r >> 2);  // + 4 in the upper half-wave (in hoff)
        const float bgc = __shfl(bgl, c + 4 * hi);
        const int so = c * (int)HW * 4;
        float x0 = EMPTY ? bgc : fmaf(T0, bgc, acc0[r]);
        float x1 = EMPTY ? bgc : fmaf(T1, bgc, acc1[r]);
        if (!REFINE) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x0), rs, v0, so, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x1), rs, v1, so, 0);
        } else {
            // branch-free: every channel is offered to both outputs; the one it does not belong to
            // gets an offset past its buffer (dropped by the buffer range check)
            const int ch_lo = c, ch_hi = c + 4;  // this register's channel in either half-wave
            const int oc_lo = ch_lo - o.keep, oc_hi = ch_hi - o.keep;  // wave-uniform
            const bool col_lo = ch_lo < o.keep, col_hi = ch_hi < o.keep;
            const bool ref_lo = oc_lo >= 0 && oc_lo < o.n_out, ref_hi = oc_hi >= 0 && oc_hi < o.n_out;
            const float b_lo = (ref_lo && o.rb) ? o.rb[oc_lo] : 0.0f;  // scalar loads
            const float b_hi = (ref_hi && o.rb) ? o.rb[oc_hi] : 0.0f;
            const bool col = hi ? col_hi : col_lo, ref = hi ? ref_hi : ref_lo;
            const int oc = hi ? oc_hi : oc_lo;
            const float bias = hi ? b_hi : b_lo;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x0), rs, col ? v0 : 0x7FFFFFF0, so, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x1), rs, col ? v1 : 0x7FFFFFF0, so, 0);
            float y0 = x0 + bias, y1 = x1 + bias;
            y0 = y0 >= 0.0f ? y0 : y0 * o.slope;  // F.leaky_relu_(x, 0.2)
            y1 = y1 >= 0.0f ? y1 : y1 * o.slope;
            // out_refine rows: the same pixel offsets without the +4-channel half-wave shift
            const int w0 = (ref && v0 != 0x7FFFFFF0) ? v0 - hoff * 4 + oc * (int)HW * 4 : 0x7FFFFFF0;
            const int w1 = (ref && v1 != 0x7FFFFFF0) ? v1 - hoff * 4 + oc * (int)HW * 4 : 0x7FFFFFF0;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y0), rr, w0, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y1), rr, w1, 0, 0);
            __builtin_amdgcn_sched_barrier(0);  // one channel at a time: no register build-up
        }
    }
}

// Epilogue of one half-strip wave (HALF): its 32 pixels start at (hx0, hy0) (kStripW wide); acc[r]
// at lane l holds channel (r&3)+8*(r>>2)+4*(l>>5) of pixel l&31, whose state (T, ...) lane l holds.
__device__ __forceinline__ void store_half(const Dims& d, const ImageArena& im, const Outputs& o, const float* bg,
                                           int b, int hx0, int hy0, int lane, const floatx16& acc, float T,
                                           float invd, uint32_t last) {
    const int64_t HW = (int64_t)d.H * d.W;
    const int j = lane & 31;
    const int qx = hx0 + j % kStripW, qy = hy0 + j / kStripW;
    const bool in_img = qx < d.W && qy < d.H;
    if (in_img && lane < 32) {
        const int64_t pix = b * HW + (int64_t)qy * d.W + qx;
        im.final_T[pix] = T;
        im.n_contrib[pix] = last;
        if (o.out_invdepth) o.out_invdepth[pix] = invd;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        o.out_color + (int64_t)b * GSR_C * HW, 0, (int)((int64_t)GSR_C * HW * 4), 0x00020000);
    const int hi = lane >> 5;
    const int v = in_img ? (hi * 4 * (int)HW + qy * d.W + qx) * 4 : 0x7FFFFFF0;
    const float bgl = bg[lane & 31];  // (as store_strip)
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int c = (r & 3) + 8 * (r >> 2);  // + 4 in the upper half-wave (in v)
        const float bgc = __shfl(bgl, c + 4 * hi);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaf(T, bgc, acc[r])), rs, v, c * (int)HW * 4, 0);
    }
}

// An empty tile inside the image (W a multiple of 4): background colour, T = 1, n_contrib = 0,
// inverse depth 0, as 16-byte stores -- lane l owns pixels 4 (l % 4) .. +3 of tile row l / 4, so each
// store instruction writes one channel of the whole tile (a quarter of store_strip's instruction
// count for the same bytes).
__device__ __forceinline__ void fill_tile(const Dims& d, const ImageArena& im, const Outputs& o, const float* bg,
                                          int b, int tx, int ty, int lane) {
    const int64_t HW = (int64_t)d.H * d.W;
    const int off = (ty * GSR_BY + lane / 4) * d.W + tx * GSR_BX + 4 * (lane % 4);  // first pixel, in floats
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        o.out_color + (int64_t)b * GSR_C * HW, 0, (int)((int64_t)GSR_C * HW * 4), 0x00020000);
#pragma unroll 8
    for (int c = 0; c < GSR_C; c++) {
        const unsigned v = __float_as_uint(bg[c]);
        __builtin_amdgcn_raw_buffer_store_b128((uint4x){v, v, v, v}, rs, off * 4, c * (int)HW * 4, 0);
    }
    const unsigned one = __float_as_uint(1.0f);
    *reinterpret_cast<uint4x*>(im.final_T + b * HW + off) = (uint4x){one, one, one, one};
    *reinterpret_cast<uint4x*>(im.n_contrib + b * HW + off) = (uint4x){0u, 0u, 0u, 0u};
    if (o.out_invdepth) *reinterpret_cast<uint4x*>(o.out_invdepth + b * HW + off) = (uint4x){0u, 0u, 0u, 0u};
}

// gsr_refine_prepare: rows [f_0..f_{keep-1}, W.f (n_out values), 0...] of 32 floats.
__global__ __launch_bounds__(256) void k_refine_prepare(int n, const float* __restrict__ in,
                                                        const float* __restrict__ w, int n_out,
                                                        int keep, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float f[GSR_C];
    const float4* src = reinterpret_cast<const float4*>(in + (int64_t)i * GSR_C);
#pragma unroll
    for (int q = 0; q < GSR_C / 4; q++) {
        const float4 v = src[q];
        f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
    }
    float* dst = out + (int64_t)i * GSR_C;
    for (int c = 0; c < GSR_C; c++) {
        float v = 0.0f;
        if (c < keep) {
            v = f[c];
        } else if (c < keep + n_out) {
            const float* wr = w + (c - keep) * GSR_C;
#pragma unroll
            for (int k = 0; k < GSR_C; k++) v = fmaf(wr[k], f[k], v);
        }
        dst[c] = v;
    }
}

void launch_split_features(int P, const float* colors, uint32_t* out, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_split_features, dim3((P * GSR_C / 4 + 255) / 256), dim3(256), 0, s, P * GSR_C / 4,
                       reinterpret_cast<const float4*>(colors), reinterpret_cast<uint4*>(out));
}

void launch_refine_prepare(int n, const float* in, const float* w, int n_out, int keep, float* out,
                           hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_refine_prepare, dim3((n + 255) / 256), dim3(256), 0, s, n, in, w, n_out, keep, out);
}

// Capacity overflow (batch path): nothing was binned, so the call's images are filled with NaN --
// a consumer cannot mistake a stale or partial frame for a render.  Grid-stride over the whole
// grid, taken only on overflow.
__device__ __forceinline__ void overflow_fill(const Dims& d, const Outputs& o) {
    const float qnan = __builtin_nanf("");
    const int64_t HW = (int64_t)d.H * d.W;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < (int64_t)d.B * GSR_C * HW; i += stride) o.out_color[i] = qnan;
    if (o.out_invdepth)
        for (int64_t i = i0; i < (int64_t)d.B * HW; i += stride) o.out_invdepth[i] = qnan;
    if (o.out_refine)
        for (int64_t i = i0; i < (int64_t)d.B * o.n_out * HW; i += stride) o.out_refine[i] = qnan;
}

// Work items: the 4 strips of each non-empty tile in strip_list order, most survivors first (items
// [0, 4*NE)), then each empty tile whole (items [4*NE, 3*NE + B*T)).  Eight queues, one per
// XCD (queue_item); a wave dequeues from its own XCD's queue and, once that is drained, from the
// others, so no counter sees more than a fraction of the traffic.
//
// The survivor stream runs as a software pipeline over k-steps (two Gaussians each) held in NSLOT
// rotating register slots: the records and feature operand of step s+NSLOT-1 are loaded while step
// s+1's alphas are computed and step s's serial blend and MFMA accumulation run.
//
// SPLIT: 0 = f32 MFMA (exact), 1 = split-bf16 products of per-frame features, 2 = of the batch's
// pre-split feature table (k_split_features).  HALF: one frame, a wave per half strip.  STATS / TL:
// the instrumented variants (gsr_render_counters / gsr_render_timeline).  ABL: timing ablations
// (GSR_TUNING builds only).
template <bool EXACT, bool STATS, bool TL, bool REFINE, int ABL = 0, int SPLIT = 0, int NSLOT = 3,
          bool HALF = false>
__device__ __forceinline__ void render_fwd_body(const Dims& d, const Inputs& in, const GeomArena& g,
                                                const ImageArena& im, const BinArena& bn,
                                                const Outputs& o) {
    if (g.ctrl[kCtrlOverflow]) {  // the lists were not built: every output pixel of the call is NaN
        overflow_fill(d, o);
        return;
    }
    static_assert(!HALF || (!STATS && !TL && !REFINE && ABL == 0), "half-strip waves: production kernel only");
    static_assert(NSLOT == 3 || NSLOT == 5, "three or five pipeline slots");
    const uint32_t ne = g.ctrl[kCtrlNonEmpty];
    // HALF: every strip is two work items (one wave per 32-pixel half, the strip's rows 0-3 / 4-7)
    const uint32_t nstrip = (HALF ? 2u : 1u) * (uint32_t)kStrips * ne;
    const uint32_t nitems = nstrip + (uint32_t)(d.B * d.T) - ne;
    const int lane = threadIdx.x & 63;
    const int hi = lane >> 5;
    const int ch = lane & 31;
    uint32_t q = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;  // HW_REG_XCC_ID
    uint32_t q_left = 8;

    for (;;) {
        uint32_t item = 0xFFFFFFFFu;
        while (q_left) {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g.ctrl[kCtrlXcdQueue + kCtrlXcdStride * q], 1u);
            k = __builtin_amdgcn_readfirstlane(k);
            item = HALF ? queue_item_n<2>(q, k, ne, nitems - nstrip, in.xcd_map, g.ctrl)
                        : queue_item(q, k, ne, nitems - nstrip, in.xcd_map, g.ctrl);
            if (item != 0xFFFFFFFFu) break;
            q = (q + 1) & 7u;
            q_left--;
        }
        if (!q_left) break;
        if (item >= nstrip) {  // empty tile: background everywhere, T = 1
            const uint64_t te_start = TL ? __builtin_amdgcn_s_memrealtime() : 0;
            const int tile_g = (int)im.work_list[ne + (item - nstrip)];
            const int b = tile_g / d.T;
            const int t = tile_g - b * d.T;
            const floatx16 unused = {};
            if (ABL == 8) {  /* timing ablation: no empty-tile stores */
            } else if (!REFINE && (d.W & 3) == 0 &&
                       ((reinterpret_cast<uintptr_t>(o.out_color) | reinterpret_cast<uintptr_t>(o.out_invdepth)) &
                        15u) == 0 &&
                       (t % d.gx + 1) * GSR_BX <= d.W && (t / d.gx + 1) * GSR_BY <= d.H) {
                fill_tile(d, im, o, in.bg + in.s_bg * b, b, t % d.gx, t / d.gx, lane);
            } else {
                for (int sp = 0; sp < kStrips; sp++) {
                    int ex0, ey0;
                    strip_origin(t % d.gx, t / d.gx, sp, ex0, ey0);
                    store_strip<true, REFINE>(d, im, o, in.bg + in.s_bg * b, b, ex0, ey0, lane, unused, unused,
                                              1.0f, 0.f, 0u);
                }
            }
            if (TL && lane == 0 && item < (o.timeline_cap & 0x7FFFFFFFu)) {  // empty tiles: k-steps 0xFFFFFFFF
                uint32_t* rec = o.timeline + 4 * (size_t)item;
                rec[0] = (uint32_t)te_start;
                rec[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
                rec[2] = 0xFFFFFFFFu;
                rec[3] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;
            }
            continue;
        }
        const uint64_t t_start = TL ? __builtin_amdgcn_s_memrealtime() : 0;
        const uint32_t code = im.strip_list[HALF ? item >> 1 : item];
        const int half = HALF ? (int)(item & 1u) : 0;
        const int tile_g = (int)(code >> 2);
        const int strip = (int)(code & 3u);
        const int b = tile_g / d.T;
        const int t = tile_g - b * d.T;
        const int tx = t % d.gx, ty = t / d.gx;
        int sx0, sy0;
        strip_origin(tx, ty, strip, sx0, sy0);
        // this lane's pixel of the strip: HALF: pixel 32 half + (lane & 31), in both lane halves
        // (lanes l and l + 32 carry the same pixel's state; their alphas are Gaussians a and b)
        const int lpix = HALF ? 32 * half + (lane & 31) : lane;
        const int px = sx0 + lpix % kStripW;
        const int py = sy0 + lpix / kStripW;
        const float pfx = (float)px, pfy = (float)py;
        bool done = !(px < d.W && py < d.H);
        float T = 1.0f, invd = 0.f;
        uint32_t last = 0, stop = 0;
        const uint32_t smask_bit = 1u << (28 + strip);
        if (!STATS && !TL && im.strip_cnt[(int64_t)tile_g * kStrips + strip] == 0u) {
            // no list entry reaches the strip (k_strip_count): nothing is taken anywhere in it, so
            // its outputs are the background, T = 1, n_contrib = 0, inverse depth 0 -- the values
            // the list walk would give -- without walking the tile's list
            const floatx16 zero = {};
            if constexpr (HALF) store_half(d, im, o, in.bg + in.s_bg * b, b, sx0, sy0 + half * (32 / kStripW), lane,
                                           zero, 1.0f, 0.f, 0u);
            else store_strip<false, REFINE>(d, im, o, in.bg + in.s_bg * b, b, sx0, sy0, lane, zero, zero, 1.0f,
                                            0.f, 0u);
            continue;
        }
        const uint2 range = im.ranges[tile_g];
        const int n = (int)(range.y - range.x);
        const uint32_t* __restrict__ plist = bn.point_list + range.x;
        // render records through a buffer resource: the byte offset of a (wave-uniform) record is
        // one SGPR, no 64-bit address arithmetic per survivor
        const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(g.rrec + (int64_t)b * d.P * 2), 0, (int)min((int64_t)d.P * 32, (int64_t)0x7FFFFFFF), 0x00020000);
        // this wave's record staging slot (words 0..15; lanes 8..63 write their out-of-range zeros to
        // the spare words 24..87)
        __shared__ unsigned rec_lds_all[GSR_TILE_PIX / 64][88];
        unsigned* rec_lds = rec_lds_all[threadIdx.x >> 6];
        const int rec_widx = lane < 8 ? lane : 16 + lane;
        // per-lane byte offsets, the survivor's row in the SGPR offset: lanes whose offset is kOOB
        // fall outside the resource (num_records < 2^31, row offsets < 2^31) and read zeros
        constexpr uint32_t kOOB = 0x80000000u;
        const int rec_voff = (int)(lane < 8 ? (uint32_t)lane * 4 : kOOB);
        const int feat_voff_a = (int)(hi ? kOOB : (uint32_t)ch * 4);
        const int feat_voff_b = (int)(hi ? (uint32_t)ch * 4 : kOOB);
        // feature rows through a buffer resource: 32-bit byte offsets, the base in SGPRs
        // (SPLIT == 2: the pre-split (hi, lo) words of k_split_features, shared by every frame)
        const __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc(
            SPLIT == 2 ? (void*)g.fsplit : (void*)(in.colors + in.s_colors * b), 0,
            (int)min((int64_t)d.P * GSR_C * 4, (int64_t)0x7FFFFFFF), 0x00020000);

        floatx16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; r++) { acc0[r] = 0.f; acc1[r] = 0.f; }
        uint64_t n_surv = 0, n_steps = 0, n_contrib_pairs = 0, n_staged = 0, n_dead = 0;

        // Survivor stream: wave-uniform state walking the list 64 entries at a time.
        int base = -64;
        uint64_t mask = 0;
        uint32_t cidx = 0;

        // next survivor -> (g, pos); false at the end of the list
#define GSR_NEXT(g_, pos_)                                                                          \
        ({                                                                                          \
            bool ok_ = true;                                                                        \
            while (mask == 0) {                                                                     \
                base += 64;                                                                         \
                if (base >= n) { ok_ = false; break; }                                              \
                cidx = lane < n - base ? plist[base + lane] : 0u;                                   \
                mask = __ballot(lane < n - base && (cidx & smask_bit) != 0u);                       \
                if (STATS) n_staged += min(64, n - base);                                           \
            }                                                                                       \
            if (ok_) {                                                                              \
                const int i_ = (int)__builtin_ctzll(mask);                                          \
                mask = clear_bit(mask, i_);                                                         \
                g_ = __builtin_amdgcn_readlane(cidx, i_) & kIndexMask;                              \
                pos_ = base + i_ + 1;                                                               \
            }                                                                                       \
            ok_;                                                                                    \
        })
        // stage 1: fetch the next k-step (two survivors) into slot S: render records and this
        // lane's feature word (in-order completion)
#define GSR_FETCH(S)                                                                                \
        {                                                                                           \
            uint32_t ga_ = 0, gb_ = 0;                                                              \
            int pa_ = 0, pb_ = 0;                                                                   \
            if (__builtin_expect(__builtin_popcountll(mask) >= 2, 1)) {                             \
                /* common case: both survivors from the chunk in hand, no loop, no refill test */   \
                const int i0_ = (int)__builtin_ctzll(mask);                                         \
                mask = clear_bit(mask, i0_);                                                        \
                const int i1_ = (int)__builtin_ctzll(mask);                                         \
                mask = clear_bit(mask, i1_);                                                        \
                ga_ = __builtin_amdgcn_readlane(cidx, i0_) & kIndexMask;                            \
                gb_ = __builtin_amdgcn_readlane(cidx, i1_) & kIndexMask;                            \
                pa_ = base + i0_ + 1;                                                               \
                pb_ = base + i1_ + 1;                                                               \
                S##v = true;                                                                        \
                S##hb = true;                                                                       \
            } else {                                                                                \
                S##v = GSR_NEXT(ga_, pa_);                                                          \
                S##hb = S##v && GSR_NEXT(gb_, pb_);                                                 \
                /* a missing survivor reads index P: past both buffer resources' ranges, so its */  \
                /* record and feature load as zeros, opacity 0 gives alpha 0 and nothing is taken */ \
                if (!S##v) ga_ = (uint32_t)d.P;                                                     \
                if (!S##hb) { gb_ = (uint32_t)d.P; pb_ = pa_; }                                     \
            }                                                                                       \
            S##pa = pa_; S##pb = pb_;                                                               \
            if (HALF) {  /* lane half h: survivor h's whole record, two 16-B loads */               \
                const uint32_t gl_ = hi ? gb_ : ga_;                                                \
                S##a0 = rec_load(rrs, gl_ * 32);                                                    \
                S##a1 = rec_load(rrs, gl_ * 32 + 16);                                               \
            } else {  /* lanes 0..7: dword `lane` of both records, SGPR offsets */                  \
                S##r = __builtin_amdgcn_raw_buffer_load_b32(rrs, rec_voff, (int)(ga_ * 32), 0);     \
                S##r2 = __builtin_amdgcn_raw_buffer_load_b32(rrs, rec_voff, (int)(gb_ * 32), 0);    \
            }                                                                                       \
            /* this lane's feature word: channel ch of survivor a (lanes 0..31) or b (32..63), */  \
            /* the survivor's row offset in the SGPR offset (range-checked like voffset: the */     \
            /* other half's lanes are out of range and read 0) */                                   \
            S##fa = ABL == 2 ? 0u : __builtin_amdgcn_raw_buffer_load_b32(frs, feat_voff_a,          \
                                                                        (int)(ga_ * (GSR_C * 4)), 0); \
            S##fb = ABL == 2 ? 0u : __builtin_amdgcn_raw_buffer_load_b32(frs, feat_voff_b,          \
                                                                        (int)(gb_ * (GSR_C * 4)), 0); \
        }
        // stage 2: the pixel-local alphas of slot S (a missing survivor has alpha 0): the records
        // through the wave's LDS slot (GSR_ALPHA_LDS), then the alpha arithmetic (GSR_ALPHA_MATH)
#define GSR_ALPHA_LDS(S)                                                                            \
        if (!HALF) {  /* uniform-address b128 reads (lanes 8..63 wrote spare words) */       \
            rec_lds[rec_widx] = S##r; rec_lds[rec_widx + 8] = S##r2;                                \
            __builtin_amdgcn_wave_barrier();                                                        \
            S##a0 = __builtin_bit_cast(float4, *(const uint4x*)&rec_lds[0]);                        \
            S##a1 = __builtin_bit_cast(float4, *(const uint4x*)&rec_lds[4]);                        \
            S##b0 = __builtin_bit_cast(float4, *(const uint4x*)&rec_lds[8]);                        \
            S##b1 = __builtin_bit_cast(float4, *(const uint4x*)&rec_lds[12]);                       \
            __builtin_amdgcn_wave_barrier();                                                        \
        }
#define GSR_ALPHA_MATH(S)                                                                           \
        {                                                                                           \
            S##al = alpha_of<EXACT>(S##a0, S##a1, pfx, pfy);                                        \
            S##ai = S##a0.w;                                                                        \
            if (!HALF) {                                                                            \
                S##bl = alpha_of<EXACT>(S##b0, S##b1, pfx, pfy);                                    \
                S##bi = S##b0.w;                                                                    \
            }                                                                                       \
            S##f = __uint_as_float(S##fa | S##fb);                                                  \
            if (SPLIT) S##fp = SPLIT == 2 ? __float_as_uint(S##f) : split_hl(S##f);                 \
        }
#define GSR_ALPHA(S) GSR_ALPHA_LDS(S) GSR_ALPHA_MATH(S)
        // GSR_LDS_EARLY: slot S+1's record reads are issued before slot S's serial blend, so the LDS
        // latency runs under the blend (the alpha arithmetic of S+1 still follows it)
#if GSR_LDS_EARLY
#define GSR_STEP(N, S) GSR_ALPHA_LDS(N) __builtin_amdgcn_sched_barrier(0); GSR_TAKE(S) GSR_ALPHA_MATH(N) GSR_PAD()
#else
#define GSR_STEP(N, S) GSR_ALPHA(N) GSR_TAKE(S) GSR_PAD()
#endif
#if GSR_PAD_SALU || GSR_PAD_VALU
        // issue-sensitivity instrumentation (A/B builds only): extra SALU / VALU per k-step
        uint32_t pad_s = __builtin_amdgcn_readfirstlane((uint32_t)n);
        float pad_v = pfx;
#define GSR_PAD()                                                                                   \
        {                                                                                           \
            _Pragma("unroll") for (int i_ = 0; i_ < GSR_PAD_SALU; i_++)                             \
                asm volatile("s_add_u32 %0, %0, 1" : "+s"(pad_s) :: "scc");                         \
            _Pragma("unroll") for (int i_ = 0; i_ < GSR_PAD_VALU; i_++)                             \
                asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(pad_v));                                \
        }
#else
#define GSR_PAD()
#endif
        // stage 3: the serial blend of slot S and its accumulation on the matrix cores
#define GSR_TAKE(S)                                                                                 \
        if (HALF) {  /* both alphas to every lane (one swap each), the pixel's blend duplicated */ \
            const auto sal_ = __builtin_amdgcn_permlane32_swap(__float_as_uint(S##al),              \
                                                               __float_as_uint(S##al), false, false); \
            const auto sai_ = __builtin_amdgcn_permlane32_swap(__float_as_uint(S##ai),              \
                                                               __float_as_uint(S##ai), false, false); \
            const float wa_ = take_step(__uint_as_float(sal_[0]), __uint_as_float(sai_[0]),         \
                                        (uint32_t)S##pa, T, invd, last, done);                      \
            const float wb_ = take_step(__uint_as_float(sal_[1]), __uint_as_float(sai_[1]),         \
                                        (uint32_t)S##pb, T, invd, last, done);                      \
            const float w_ = hi ? wb_ : wa_;  /* k 0..3: Gaussian a (lanes 0-31), 4..7: b */        \
            if (SPLIT) {                                                                            \
                unsigned h_, l_;                                                                    \
                split_hh_ll(w_, h_, l_);                                                            \
                const uint2x a2_ = {S##fp, S##fp}, b2_ = {h_, l_};                                  \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(__builtin_bit_cast(shortx4, a2_),   \
                                                               __builtin_bit_cast(shortx4, b2_), acc0, 0, 0, 0); \
            } else {                                                                                \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(S##f, w_, acc0, 0, 0, 0);               \
            }                                                                                       \
        } else {                                                                                    \
            const float f_ = S##f;                                                                  \
            const bool was_done_ = done;                                                            \
            const float wa_ = take_step(S##al, S##ai, (uint32_t)S##pa, T, invd, last, done);        \
            const bool done_a_ = done;                                                              \
            const float wb_ = take_step(S##bl, S##bi, (uint32_t)S##pb, T, invd, last, done);        \
            if (STATS) {                                                                            \
                if (!was_done_ && done_a_) stop = (uint32_t)S##pa;                                  \
                else if (!done_a_ && done) stop = (uint32_t)S##pb;                                  \
                n_contrib_pairs += __popcll(__ballot(wa_ > 0.f)) + __popcll(__ballot(wb_ > 0.f));   \
                n_dead += (S##v && __ballot(wa_ > 0.f || wb_ > 0.f) == 0ull) ? 1 : 0;               \
                n_surv += S##v ? (S##hb ? 2 : 1) : 0;                                               \
            }                                                                                       \
            if (STATS || TL) n_steps += S##v ? 1 : 0;                                               \
            if (ABL == 1) {  /* timing ablation: VALU stand-in for the MFMAs */                     \
                const auto sw_ = __builtin_amdgcn_permlane32_swap(__float_as_uint(wa_),             \
                                                                  __float_as_uint(wb_), false, false); \
                acc0[0] = fmaf(f_, __uint_as_float(sw_[0]), acc0[0]);                               \
                acc1[0] = fmaf(f_, __uint_as_float(sw_[1]), acc1[0]);                               \
            } else if (SPLIT) {  /* k 0..3 of each half: f_hi.w_hi + f_lo.w_hi + f_hi.w_lo + f_lo.w_lo */ \
                /* split both weights, then swap the (hi, hi) and (lo, lo) words: the swaps */      \
                /* consume the split words, the weights stay for the inverse depth */               \
                const unsigned fp_ = S##fp;                                                         \
                unsigned ha_, la_, hb_, lb_;                                                        \
                split_hh_ll(wa_, ha_, la_);                                                         \
                split_hh_ll(wb_, hb_, lb_);                                                         \
                const auto sh_ = __builtin_amdgcn_permlane32_swap(ha_, hb_, false, false);          \
                const auto sl_ = __builtin_amdgcn_permlane32_swap(la_, lb_, false, false);          \
                const uint2x a2_ = {fp_, fp_}, b0_ = {sh_[0], sl_[0]}, b1_ = {sh_[1], sl_[1]};      \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(__builtin_bit_cast(shortx4, a2_),   \
                                                               __builtin_bit_cast(shortx4, b0_), acc0, 0, 0, 0); \
                acc1 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(__builtin_bit_cast(shortx4, a2_),   \
                                                               __builtin_bit_cast(shortx4, b1_), acc1, 0, 0, 0); \
            } else {                                                                                \
                const auto sw_ = __builtin_amdgcn_permlane32_swap(__float_as_uint(wa_),             \
                                                                  __float_as_uint(wb_), false, false); \
                const float fa_ = ABL == 2 ? 1.0f : f_;  /* timing ablation: no feature operand */  \
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa_, __uint_as_float(sw_[0]), acc0, 0, 0, 0); \
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa_, __uint_as_float(sw_[1]), acc1, 0, 0, 0); \
            }                                                                                       \
        }
#define GSR_SLOT(S) bool S##v, S##hb; int S##pa, S##pb; float4 S##a0, S##a1, S##b0, S##b1; unsigned S##r, S##r2, S##fa, S##fb; \
        float S##f, S##al, S##bl, S##ai, S##bi; unsigned S##fp = 0;
        GSR_SLOT(A)
        GSR_SLOT(B)
        GSR_SLOT(C)
        // An invalid slot takes nothing (alpha 0, feature 0); the loop leaves only at its head and
        // its foot, which keeps the MFMA accumulators in one register chain.
        if constexpr (NSLOT == 3) {
            GSR_FETCH(A)
            GSR_FETCH(B)
            GSR_FETCH(C)
            GSR_ALPHA(A)
            while (Av) {
                GSR_STEP(B, A)
                GSR_FETCH(A)
                GSR_STEP(C, B)
                GSR_FETCH(B)
                GSR_STEP(A, C)
                GSR_FETCH(C)
                if (!__any(!done)) break;  // every pixel of the strip finished
            }
        } else {
            // latency mode (single-frame launches, where one wave's strip sets the kernel time): five
            // slots, each slot's records requested four k-steps before its alphas
            GSR_SLOT(D)
            GSR_SLOT(E)
            GSR_FETCH(A)
            GSR_FETCH(B)
            GSR_FETCH(C)
            GSR_FETCH(D)
            GSR_FETCH(E)
            GSR_ALPHA(A)
            while (Av) {
                GSR_STEP(B, A)
                GSR_FETCH(A)
                GSR_STEP(C, B)
                GSR_FETCH(B)
                GSR_STEP(D, C)
                GSR_FETCH(C)
                GSR_STEP(E, D)
                GSR_FETCH(D)
                GSR_STEP(A, E)
                GSR_FETCH(E)
                if (!__any(!done)) break;
            }
        }
#undef GSR_NEXT
#undef GSR_FETCH
#undef GSR_ALPHA
#undef GSR_ALPHA_LDS
#undef GSR_ALPHA_MATH
#undef GSR_STEP
#undef GSR_TAKE
#undef GSR_SLOT
#undef GSR_PAD

        // ---- epilogue ----
        if (STATS) {
            unsigned long long* cn = (unsigned long long*)o.stats;
            uint64_t ev = (px < d.W && py < d.H) ? (done ? stop : (uint32_t)n) : 0;
            for (int off = 32; off > 0; off >>= 1) ev += __shfl_xor(ev, off);
            if (lane == 0) {
                atomicAdd(&cn[0], (unsigned long long)ev);
                atomicAdd(&cn[1], (unsigned long long)n_contrib_pairs);
                atomicAdd(&cn[2], (unsigned long long)n_surv);
                atomicAdd(&cn[3], (unsigned long long)n_steps);
                atomicAdd(&cn[4], (unsigned long long)n_staged);
                atomicAdd(&cn[7], (unsigned long long)n_dead);
                if (strip == 0) {
                    atomicAdd(&cn[5], (unsigned long long)n);
                    atomicAdd(&cn[6], 1ull);
                }
            }
        }
        if (TL && lane == 0 && item < (o.timeline_cap & 0x7FFFFFFFu)) {  // (start, end) in 100 MHz ticks, k-steps, XCC
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            uint32_t* rec = o.timeline + 4 * (size_t)item;
            rec[0] = (uint32_t)t_start;
            rec[1] = (uint32_t)t_end;
            rec[2] = (uint32_t)n_steps;
            rec[3] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;
        }
        if constexpr (HALF) store_half(d, im, o, in.bg + in.s_bg * b, b, sx0, sy0 + half * (32 / kStripW), lane,
                                       acc0, T, invd, last);
        else if (ABL == 9) {  /* timing ablation: only final_T of the strip is stored */
            if (px < d.W && py < d.H) im.final_T[b * (int64_t)d.H * d.W + (int64_t)py * d.W + px] = T + acc0[0] + acc1[0];
        }
        else store_strip<false, REFINE>(d, im, o, in.bg + in.s_bg * b, b, sx0, sy0, lane, acc0, acc1, T,
                                        invd, last);
    }
}

// Register budget: 5 waves per SIMD (96 registers; the few values spilled live outside the blend
// loop) for the 3-slot kernel, launched 5 workgroups per CU at 16+ frames: the blend loop is
// VALU-issue-bound with latency that 4 waves did not cover.  The half-strip (one frame) kernel
// keeps a 3-wave budget (launched 3 per CU).
#ifndef GSR_RENDER_WPE
#define GSR_RENDER_WPE 5
#endif
#ifndef GSR_HALF_WPE
#define GSR_HALF_WPE 3
#endif
template <bool EXACT, bool STATS, bool TL, int SPLIT = 0, int NSLOT = GSR_BATCH_NSLOT, bool HALF = false>
__global__ __launch_bounds__(GSR_TILE_PIX)
__attribute__((amdgpu_waves_per_eu(HALF ? GSR_HALF_WPE : GSR_RENDER_WPE))) void k_render_fwd(
    Dims d, Inputs in, GeomArena g, ImageArena im, BinArena bn, Outputs o) {
    render_fwd_body<EXACT, STATS, TL, false, 0, SPLIT, NSLOT, HALF>(d, in, g, im, bn, o);
}

#ifdef GSR_TUNING
// Timing ablations of the production kernel (GSR_RENDER_ABLATE=1: VALU stand-in for the MFMAs,
// 2: no feature loads, 8: no empty-tile stores, 9: no strip colour stores).  Wrong images by
// construction; for attributing render_fwd time only, and only in tools/build_ab.py builds.
template <int ABL>
__global__ __launch_bounds__(GSR_TILE_PIX) __attribute__((amdgpu_waves_per_eu(GSR_RENDER_WPE)))
void k_render_fwd_ablate(Dims d, Inputs in, GeomArena g, ImageArena im, BinArena bn, Outputs o) {
    render_fwd_body<true, false, false, false, ABL>(d, in, g, im, bn, o);
}
#endif

// The refiner-head variant: the epilogue's extra stores would raise the register count past the
// 4-waves-per-SIMD budget of the blend loop; pin the budget (the few extra live values of the
// epilogue spill instead).
template <bool EXACT>
__global__ __launch_bounds__(GSR_TILE_PIX) __attribute__((amdgpu_waves_per_eu(4))) void k_render_fwd_refine(
    Dims d, Inputs in, GeomArena g, ImageArena im, BinArena bn, Outputs o) {
    render_fwd_body<EXACT, false, false, true>(d, in, g, im, bn, o);
}

// ---------------------------------------------------------------- one frame: quad waves
// The per-frame drop-in path renders ONE frame per launch; its 4,096 strips leave most of the chip
// idle and the longest strips' serial chains set the time.  Here every strip is four work items,
// one wave per 4x4 quad, and each quad wave walks only the Gaussians that can reach alpha >= 1/255
// in ITS 16 pixels: per 64-entry list chunk, each lane loads the render record of one strip
// survivor and tests it against the quad's pixel-centre box (box_reach, binning's strip test on a
// 4x4 rectangle), and the quad survivors' records (word 7 := Gaussian index) and list positions
// are appended to a per-wave LDS ring.  Offline, one C2 frame's longest quad chain is 0.63 of the
// longest half-strip chain and 0.31 of it in 4-Gaussian steps (tools/analysis/quad_tail.py).
//
// A step takes the next FOUR ring entries: lane = pixel j (0..15) + 16 q, and each lane computes
// Gaussian q's alpha at pixel j (one alpha per lane).  The four alphas and inverse depths reach
// every lane by one permlane16 and two permlane32 swaps; each lane runs its pixel's serial blend
// over the four in list order (the same decisions and products as forward.cu:349-381) and keeps
// Gaussian q's weight, which is exactly the B operand of v_mfma_f32_16x16x4_f32 (B[k = q][n = j]),
// with A[m][k = q] = channel m of Gaussian q: two MFMAs (channels 0-15, 16-31) accumulate the
// quad's 32 x 16 colour tile as an exact k-ordered fma chain, bit-identical to fmaf(f, w, C)
// Gaussian by Gaussian (the oracle).  Ring entries past the list's end are the null Gaussian
// (zero record: opacity 0, nothing taken).  The next step's records (LDS) and feature words
// (global) load while this step blends; the chunk after next's list entries and the next chunk's
// records are loaded one refill ahead.
#ifndef GSR_QUAD_WPE
#define GSR_QUAD_WPE 2  // waves per SIMD: 2 leave the registers (220) for 6 operand slots
#endif
#ifndef GSR_QUAD_SLOTS
// operand slots: a step's record / feature loads are issued GSR_QUAD_SLOTS - 1 steps before their
// use.  Per C2 frame: 4 slots at 3 waves per SIMD (168 registers) 122.4 us, 4 at 2 waves 123.5,
// 5 at 2 waves 119.1, 6 / 7 / 8 at 2 waves 117.6-118.6 (220 / 241 / 256 registers)
#define GSR_QUAD_SLOTS 6
#endif
template <int K>
struct QSlot {
    static constexpr int k = K;
};
#ifndef GSR_QUAD_RCH
#define GSR_QUAD_RCH 3  // 64-entry list chunks per refill (per C2 frame at 6 slots: 2 -> 116.5 us, 3 -> 115.9, 4 -> 118.2, 8 -> 119.4)
#endif
constexpr int kQRch = GSR_QUAD_RCH;
constexpr int kQRing = kQRch <= 4 ? 512 : 1024;  // ring entries per wave
// live entries: a refill (ensure) runs while fewer than 8 GSR_QUAD_SLOTS are queued and adds at most
// 64 kQRch; behind the head, up to 4 GSR_QUAD_SLOTS entries of the steps whose operands are in flight;
// past the tail, 4 GSR_QUAD_SLOTS null entries once the list is exhausted
static_assert(kQRing >= 64 * kQRch + 16 * GSR_QUAD_SLOTS, "quad ring too small for a refill beside the slots in flight");
constexpr uint32_t kQNull = 0x07FFFFFFu;  // the null Gaussian: record / feature offsets out of range

// TL (gsr_render_timeline): per quad item, (start, end) in 100 MHz ticks, steps | refills << 16, list
// entries walked
template <bool EXACT, bool TL = false>
__global__ __launch_bounds__(GSR_TILE_PIX) __attribute__((amdgpu_waves_per_eu(GSR_QUAD_WPE))) void k_render_quad(
    Dims d, Inputs in, GeomArena g, ImageArena im, BinArena bn, Outputs o, int prio_n) {
    if (g.ctrl[kCtrlOverflow]) {
        overflow_fill(d, o);
        return;
    }
    __shared__ uint32_t qg_all[GSR_TILE_PIX / 64][kQRing];    // ring Gaussian indices
    __shared__ uint32_t qpos_all[GSR_TILE_PIX / 64][kQRing];  // ring list positions (1-based)
    uint32_t* qg = qg_all[threadIdx.x >> 6];
    uint32_t* qpos = qpos_all[threadIdx.x >> 6];
    const uint32_t ne = g.ctrl[kCtrlNonEmpty];
    const uint32_t nquad = 16u * ne;  // 4 strips x 4 quads per non-empty tile
    const uint32_t nempty = (uint32_t)(d.B * d.T) - ne;
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, qq = lane >> 4;
    const uint32_t sel1 = (qq & 1) ? 0xFFFFFFFFu : 0u, sel2 = (qq & 2) ? 0xFFFFFFFFu : 0u;
    const int64_t HW = (int64_t)d.H * d.W;
    uint32_t q = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;  // HW_REG_XCC_ID
    uint32_t q_left = 8;
    for (;;) {
        uint32_t item = 0xFFFFFFFFu;
        uint32_t k_item = 0;
        while (q_left) {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g.ctrl[kCtrlXcdQueue + kCtrlXcdStride * q], 1u);
            k = __builtin_amdgcn_readfirstlane(k);
            k_item = k;
            item = queue_item_n<4>(q, k, ne, nempty, in.xcd_map, g.ctrl);
            if (item != 0xFFFFFFFFu) break;
            q = (q + 1) & 7u;
            q_left--;
        }
        if (!q_left) break;
        // the first items of each queue are the longest quads (longest-first strip order): their
        // waves take issue priority over the co-resident shorter ones, whose slack covers them
        if (prio_n > 0) {
            if (k_item < (uint32_t)prio_n) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (item >= nquad) {  // empty tile: background everywhere, T = 1
            const int tile_g = (int)im.work_list[ne + (item - nquad)];
            const int b = tile_g / d.T;
            const int t = tile_g - b * d.T;
            if ((d.W & 3) == 0 &&
                ((reinterpret_cast<uintptr_t>(o.out_color) | reinterpret_cast<uintptr_t>(o.out_invdepth)) & 15u) ==
                    0 &&
                (t % d.gx + 1) * GSR_BX <= d.W && (t / d.gx + 1) * GSR_BY <= d.H) {
                fill_tile(d, im, o, in.bg + in.s_bg * b, b, t % d.gx, t / d.gx, lane);
            } else {
                const floatx16 unused = {};
                for (int sp = 0; sp < kStrips; sp++) {
                    int ex0, ey0;
                    strip_origin(t % d.gx, t / d.gx, sp, ex0, ey0);
                    store_strip<true, false>(d, im, o, in.bg + in.s_bg * b, b, ex0, ey0, lane, unused, unused, 1.0f,
                                             0.f, 0u);
                }
            }
            continue;
        }
        const uint64_t t_start = TL ? __builtin_amdgcn_s_memrealtime() : 0;
        uint32_t n_steps = 0, n_refills = 0, n_walk = 0;
        uint64_t ph_issue = 0, ph_alpha = 0, ph_blend = 0;
        const uint32_t code = im.strip_list[item >> 2];
        const int quad = (int)(item & 3u);
        const int tile_g = (int)(code >> 2);
        const int strip = (int)(code & 3u);
        const int b = tile_g / d.T;
        const int t = tile_g - b * d.T;
        int sx0, sy0;
        strip_origin(t % d.gx, t / d.gx, strip, sx0, sy0);
        const int qx0 = sx0 + 4 * (quad & 1), qy0 = sy0 + 4 * (quad >> 1);
        const int px = qx0 + (j & 3), py = qy0 + (j >> 2);
        const bool inside = px < d.W && py < d.H;
        const float pfx = (float)px, pfy = (float)py;
        bool done = !inside;
        float T = 1.0f, invd = 0.f;
        uint32_t last = 0;
        floatx4 qa0 = {0.f, 0.f, 0.f, 0.f}, qa1 = {0.f, 0.f, 0.f, 0.f};
        if (im.strip_cnt[(int64_t)tile_g * kStrips + strip] != 0u) {
            const uint2 range = im.ranges[tile_g];
            const int n = (int)(range.y - range.x);
            const uint32_t* __restrict__ plist = bn.point_list + range.x;
            const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(g.rrec + (int64_t)b * d.P * 2), 0, (int)min((int64_t)d.P * 32, (int64_t)0x7FFFFFFF),
                0x00020000);
            const __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(in.colors + in.s_colors * b), 0, (int)min((int64_t)d.P * GSR_C * 4, (int64_t)0x7FFFFFFF),
                0x00020000);
            // list walk, 64 GSR_QUAD_RCH entries per refill (GSR_QUAD_RCH per lane): the entries and their quad masks
            // (binning's box test of this quad, BinArena.qmask) are contiguous loads with no
            // dependent ones, double-buffered one refill ahead; the survivors' Gaussian indices and
            // list positions go to the ring
            const uint32_t qbit = 4u * (uint32_t)strip + (uint32_t)quad;
            const uint32_t* __restrict__ qm = bn.qmask + range.x;
            int base = 0;                  // first list position of the next refill
            uint32_t head = 0, tail = 0;   // ring counters (head advances by 4: entries never wrap in a step)
            uint32_t ec[kQRch], mc[kQRch];
            // list entries and quad masks through buffer resources over the tile's list: a position past
            // its end reads 0 (nothing kept) without a branch -- a conditional load merged into its
            // register compiled to a copy that waited for the load at once, i.e. for every operand load
            // in flight, at every refill
            const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc((void*)plist, 0, n * 4, 0x00020000);
            const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc((void*)qm, 0, n * 4, 0x00020000);
            auto load_chunks = [&](int b0, uint32_t (&e)[kQRch], uint32_t (&m)[kQRch]) {
#pragma unroll
                for (int u = 0; u < kQRch; u++) {
                    const int off = (b0 + 64 * u + lane) * 4;
                    e[u] = __builtin_amdgcn_raw_buffer_load_b32(lrs, off, 0, 0);
                    m[u] = __builtin_amdgcn_raw_buffer_load_b32(mrs, off, 0, 0);
                }
            };
            load_chunks(0, ec, mc);
            auto refill = [&]() {
#pragma unroll
                for (int u = 0; u < kQRch; u++) {
                    const bool keep = ((mc[u] >> qbit) & 1u) != 0u;
                    const uint64_t km = __ballot(keep);
                    if (keep) {
                        const uint32_t slot = (tail + __builtin_amdgcn_mbcnt_hi((uint32_t)(km >> 32),
                                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)km, 0u))) &
                                              (kQRing - 1);
                        qg[slot] = ec[u] & kIndexMask;
                        qpos[slot] = (uint32_t)(base + 64 * u + lane + 1);
                    }
                    tail += (uint32_t)__builtin_popcountll(km);
                }
                base += 64 * kQRch;
                if (TL) n_refills++;
                // the next refill's chunk into the same registers (one set, loaded one refill ahead: a
                // second set rotated into this one compiled to copies that waited for the loads just issued)
                load_chunks(base, ec, mc);
                __builtin_amdgcn_wave_barrier();
            };
            // fill so that entries [head, head + 4 GSR_QUAD_SLOTS) exist; once the list is
            // exhausted, the ring slots past its last entry hold the null Gaussian (an index whose record and feature
            // offsets are out of range: zeros, opacity 0, nothing taken), so the step operands are read
            // without a validity branch
            // ensure() runs once per group of GSR_QUAD_SLOTS steps (the unrolled step loop), so between a
            // refill's chunk loads and the next refill's use of them a group's operand loads (4 per step)
            // are issued, and the memory-counter wait there counts past the operand loads in flight
            // instead of draining them (only a back-to-back refill, whose ring ran short, waits for its
            // chunk).  It keeps two groups' entries queued (one group runs, the other is read
            // GSR_QUAD_SLOTS - 1 steps ahead).
            bool nulled = false;
            auto ensure = [&]() {
                if (tail - head < 8u * GSR_QUAD_SLOTS && base < n) {
                    refill();
                    // a back-to-back refill waits for the chunk just loaded (the newest loads: vmcnt(0)),
                    // explicitly, so that this loop stays apart from the first refill, whose wait then
                    // counts from the group's operand loads alone
                    while (tail - head < 8u * GSR_QUAD_SLOTS && base < n) {
                        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
                        refill();
                    }
                }
                if (base >= n && !nulled) {
                    nulled = true;
                    if (lane < 4 * GSR_QUAD_SLOTS) {
                        const uint32_t slot = (tail + (uint32_t)lane) & (kQRing - 1);
                        qg[slot] = kQNull;
                        qpos[slot] = 0u;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            };
            // one step's render records (lane group qq: ring entry h + qq) and feature words (A operands:
            // channels j and 16 + j), from global memory GSR_QUAD_SLOTS - 1 steps ahead of their use
            auto records = [&](uint32_t h, float4& r0, float4& r1, float& f0, float& f1) {
                const uint32_t gi = qg[(h + (uint32_t)qq) & (kQRing - 1)];
#ifdef GSR_QUAD_ABL_NOLOAD  /* timing ablation (A/B builds only, wrong images): no operand loads */
                r0 = make_float4(pfx + 0.5f * (float)(gi & 7u), pfy + 0.5f, 0.5f, 1.0f);
                r1 = make_float4(-0.05f, 0.01f, -0.05f, __uint_as_float(gi));
                f0 = (float)(gi & 3u);
                f1 = f0;
#else
                r0 = rec_load(rrs, gi * 32u);
                r1 = rec_load(rrs, gi * 32u + 16u);
#ifdef GSR_QUAD_ABL_NOFEAT  /* timing ablation (A/B builds only, wrong images): no feature loads */
                f0 = (float)(gi & 3u);
                f1 = f0;
#else
                const uint32_t fo = gi * (uint32_t)(GSR_C * 4) + (uint32_t)j * 4u;
                f0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(frs, (int)fo, 0, 0));
                f1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(frs, (int)(fo + 64u), 0, 0));
#endif
#endif
            };
            auto positions = [&](uint32_t h) { return *reinterpret_cast<const uint4*>(&qpos[h & (kQRing - 1)]); };
            ensure();
            __builtin_amdgcn_wave_barrier();
            // operand pipeline of GSR_QUAD_SLOTS slots: step i's records and feature words sit in slot
            // i % NS, loaded NS - 1 steps ahead (step i issues step i + NS - 1's loads into the slot step
            // i - 1 freed).  The step loop is unrolled by NS so that every slot is one fixed set of
            // registers: a rotated array compiles to register copies, and a copy of a register whose
            // load is still in flight waits for it (s_waitcnt vmcnt(0) every step: no prefetch at all).
            constexpr int NS = GSR_QUAD_SLOTS;
            float4 pr0[NS], pr1[NS];
            float pf0[NS], pf1[NS];
#pragma unroll
            for (int k = 0; k + 1 < NS; k++) records(head + 4u * k, pr0[k], pr1[k], pf0[k], pf1[k]);
            uint4 p4 = positions(head);
            float al = alpha_of<EXACT>(pr0[0], pr1[0], pfx, pfy);
            auto step = [&](auto slot) {
                constexpr int c = decltype(slot)::k;
                constexpr int nx = (c + 1) % NS, ld = (c + NS - 1) % NS;
                // (TL: core-clock sums of the step's phases -- operand issue incl. refills, the next
                // alpha (its records' wait), this step's blend + MFMAs)
                uint64_t c0 = 0, c1 = 0, c2 = 0;
                if (TL) { __builtin_amdgcn_sched_barrier(0); c0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); }
                // the operands of step i + NS - 1 first (their loads run under this step and the next ones;
                // the ring holds them: ensure() at the top of the step group)
                records(head + 4u * (NS - 1), pr0[ld], pr1[ld], pf0[ld], pf1[ld]);
                const uint4 np4 = positions(head + 4u);
                if (TL) { __builtin_amdgcn_sched_barrier(0); c1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); }
                // the next step's alpha (independent of this step's transmittance chain, so the two
                // interleave: a lone tail wave is latency-bound, one dependent instruction after another)
                const float nal = alpha_of<EXACT>(pr0[nx], pr1[nx], pfx, pfy);
                if (TL) {
                    __builtin_amdgcn_sched_barrier(0);
                    c2 = __builtin_amdgcn_s_memtime() + (uint64_t)(__float_as_uint(nal) & 0u);
                    __builtin_amdgcn_sched_barrier(0);
                }
                const float rw = pr0[c].w;
                const float f0 = pf0[c], f1 = pf1[c];
                // this step
                const auto a16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(al), __float_as_uint(al), false, false);
                const auto a02 = __builtin_amdgcn_permlane32_swap(a16[0], a16[0], false, false);
                const auto a13 = __builtin_amdgcn_permlane32_swap(a16[1], a16[1], false, false);
                const auto i16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(rw), __float_as_uint(rw), false,
                                                                  false);
                const auto i02 = __builtin_amdgcn_permlane32_swap(i16[0], i16[0], false, false);
                const auto i13 = __builtin_amdgcn_permlane32_swap(i16[1], i16[1], false, false);
                const float w0 = take_step(__uint_as_float(a02[0]), __uint_as_float(i02[0]), p4.x, T, invd, last, done);
                const float w1 = take_step(__uint_as_float(a13[0]), __uint_as_float(i13[0]), p4.y, T, invd, last, done);
                const float w2 = take_step(__uint_as_float(a02[1]), __uint_as_float(i02[1]), p4.z, T, invd, last, done);
                const float w3 = take_step(__uint_as_float(a13[1]), __uint_as_float(i13[1]), p4.w, T, invd, last, done);
                // Gaussian qq's weight, by two bit selects on loop-invariant lane masks (v_bfi_b32; a
                // ternary chain on qq compiled to divergent branches)
                const uint32_t w01 = (__float_as_uint(w1) & sel1) | (__float_as_uint(w0) & ~sel1);
                const uint32_t w23 = (__float_as_uint(w3) & sel1) | (__float_as_uint(w2) & ~sel1);
                const float wq = __uint_as_float((w23 & sel2) | (w01 & ~sel2));
                qa0 = __builtin_amdgcn_mfma_f32_16x16x4f32(f0, wq, qa0, 0, 0, 0);
                qa1 = __builtin_amdgcn_mfma_f32_16x16x4f32(f1, wq, qa1, 0, 0, 0);
                head += 4u;
                if (TL) {
                    __builtin_amdgcn_sched_barrier(0);
                    const uint64_t c3 = __builtin_amdgcn_s_memtime() + (uint64_t)(__float_as_uint(qa0[0] + qa1[0]) & 0u);
                    __builtin_amdgcn_sched_barrier(0);
                    n_steps++;
                    ph_issue += c1 - c0;
                    ph_alpha += c2 - c1;
                    ph_blend += c3 - c2;
                }
                p4 = np4;
                al = nal;
                return head < tail && __any(!done);  // (false: the list is done or every pixel of the quad finished)
            };
            static_assert(NS >= 3 && NS <= 8, "GSR_QUAD_SLOTS");
            while (head < tail) {
                ensure();
                __builtin_amdgcn_wave_barrier();
                if (!step(QSlot<0>{})) break;
                if (!step(QSlot<1>{})) break;
                if (!step(QSlot<2>{})) break;
                if constexpr (NS >= 4) {
                    if (!step(QSlot<3 % NS>{})) break;
                }
                if constexpr (NS >= 5) {
                    if (!step(QSlot<4 % NS>{})) break;
                }
                if constexpr (NS >= 6) {
                    if (!step(QSlot<5 % NS>{})) break;
                }
                if constexpr (NS >= 7) {
                    if (!step(QSlot<6 % NS>{})) break;
                }
                if constexpr (NS >= 8) {
                    if (!step(QSlot<7 % NS>{})) break;
                }
            }
            // the slot registers are read after the loop (an empty asm use: one wait per item), so every
            // path out of a step uses its operand loads and the compiler keeps them in the step that
            // issues them -- otherwise it sank them past the break tests to the loop's back edge, where
            // a whole group's loads were issued at once and waited for within the next group
#pragma unroll
            for (int k = 0; k < NS; k++)
                asm volatile("" ::"v"(pr0[k].x), "v"(pr1[k].x), "v"(pf0[k]), "v"(pf1[k]));
            if (TL) n_walk = (uint32_t)min(base, n);
        }
        if (TL && lane == 0 && item < (o.timeline_cap & 0x7FFFFFFFu)) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            uint32_t* rec = o.timeline + 4 * (size_t)item;
            rec[0] = (uint32_t)t_start;
            rec[1] = (uint32_t)t_end;
            rec[2] = min(n_steps, 0xFFFFu) | (min(n_refills, 0xFFFFu) << 16);
            rec[3] = n_walk;
            if (o.timeline_cap & 0x80000000u) {  // phase sums requested: a second block of records
                uint32_t* ph = o.timeline + 4 * (size_t)(o.timeline_cap & 0x7FFFFFFFu) + 4 * (size_t)item;
                ph[0] = (uint32_t)ph_issue;
                ph[1] = (uint32_t)ph_alpha;
                ph[2] = (uint32_t)ph_blend;
                ph[3] = 0u;
            }
        }
        // epilogue: group 0 stores final_T / n_contrib / inverse depth, every lane its channels
        // 4 qq + r and 16 + 4 qq + r of pixel j
        const float* bgp = in.bg + in.s_bg * b;
        const int64_t pix = (int64_t)py * d.W + px;
        if (inside && qq == 0) {
            im.final_T[b * HW + pix] = T;
            im.n_contrib[b * HW + pix] = last;
            if (o.out_invdepth) o.out_invdepth[b * HW + pix] = invd;
        }
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            o.out_color + (int64_t)b * GSR_C * HW, 0, (int)((int64_t)GSR_C * HW * 4), 0x00020000);
        const int vo = inside ? (int)(pix * 4) : 0x7FFFFFF0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c0_ = 4 * qq + r, c1_ = 16 + 4 * qq + r;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaf(T, bgp[c0_], qa0[r])), rs, vo,
                                                  c0_ * (int)HW * 4, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaf(T, bgp[c1_], qa1[r])), rs, vo,
                                                  c1_ * (int)HW * 4, 0);
        }
    }
}

// GSR_RENDER_QUAD=0: single-frame launches on the half-strip kernel (A/B)
static bool quad_mode_on() {
    static const bool v = tune_env("GSR_RENDER_QUAD", 1) != 0;
    return v;
}

bool render_uses_quad(const Dims& d, bool split, const Outputs& o) {
    return d.B == 1 && quad_mode_on() && !split && !o.stats && !o.out_refine;
}

void launch_render_fwd(const Dims& d, const Inputs& in_, const GeomArena& g, const ImageArena& im,
                       const BinArena& b, const Outputs& o, bool exact, bool split, hipStream_t s) {
    Inputs in = in_;  // one frame: strip_list is one longest-first list (launch_strip_order)
    if (d.B == 1 && in.xcd_map == 2u) in.xcd_map = 1u;
    const int nwaves = d.B * d.T * kStrips;  // upper bound of the work items
    if (nwaves == 0) return;
    // workgroups per CU: at most the resident capacity (GSR_RENDER_WPE waves/SIMD at the kernel's
    // register budget), so no render workgroup waits in the dispatcher ahead of another stream's
    // kernels.  Large batches take all 5 (-3% at 32 frames); small ones 4 (5 was +4% at the
    // 6-frame training batch, where fewer strips per wave leave a longer tail).
    static const int wg_env = tune_env("GSR_RENDER_WG_PER_CU", 0);
    const int wg_per_cu = wg_env > 0 ? wg_env : (d.B >= 16 ? GSR_RENDER_WPE : 4);
    // GSR_RENDER_HALF=0: single-frame launches on the throughput kernel (A/B); GSR_RENDER_HALF_WG: WGs per CU
    static const bool half_mode = tune_env("GSR_RENDER_HALF", 1) != 0;
    // (GSR_RENDER_QUAD_WG: quad-kernel workgroups per CU)
    const bool quad_mode = quad_mode_on();
    static const int quad_wg = tune_env("GSR_RENDER_QUAD_WG", GSR_QUAD_WPE);
    static const int half_wg = tune_env("GSR_RENDER_HALF_WG", GSR_HALF_WPE);
    const int grid = min((nwaves + 3) / 4, persistent_grid_on(s, wg_per_cu));
    const dim3 gr(grid), bl(GSR_TILE_PIX);
#ifdef GSR_TUNING
    static const int ablate = tune_env("GSR_RENDER_ABLATE", 0);
    if (!o.stats && !o.timeline && !o.out_refine && ablate) {
        if (ablate == 1) hipLaunchKernelGGL((k_render_fwd_ablate<1>), gr, bl, 0, s, d, in, g, im, b, o);
        else if (ablate == 2) hipLaunchKernelGGL((k_render_fwd_ablate<2>), gr, bl, 0, s, d, in, g, im, b, o);
        else if (ablate == 8) hipLaunchKernelGGL((k_render_fwd_ablate<8>), gr, bl, 0, s, d, in, g, im, b, o);
        else if (ablate == 9) hipLaunchKernelGGL((k_render_fwd_ablate<9>), gr, bl, 0, s, d, in, g, im, b, o);
        return;
    }
#endif
#define GSR_LAUNCH(SPL, ...)                                                                            \
    {                                                                                                   \
        if (exact) hipLaunchKernelGGL((k_render_fwd<true, __VA_ARGS__>), gr, bl, 0, s, d, in, g, im, b, o);   \
        else hipLaunchKernelGGL((k_render_fwd<false, __VA_ARGS__>), gr, bl, 0, s, d, in, g, im, b, o);        \
    }
    if (o.stats) {
        GSR_LAUNCH(0, true, false)
    } else if (o.timeline && d.B == 1 && quad_mode && !split && b.qmask) {  // the quad kernel's own timeline
        const dim3 gq(min((4 * nwaves + 3) / 4, persistent_grid(quad_wg)));
        if (exact) hipLaunchKernelGGL((k_render_quad<true, true>), gq, bl, 0, s, d, in, g, im, b, o, 0);
        else hipLaunchKernelGGL((k_render_quad<false, true>), gq, bl, 0, s, d, in, g, im, b, o, 0);
    } else if (o.timeline) {
        GSR_LAUNCH(0, false, true)
    } else if (o.out_refine) {  // (4-wave register budget: 4 workgroups per CU)
        const dim3 grf(min((nwaves + 3) / 4, persistent_grid(4)));
        if (exact) hipLaunchKernelGGL((k_render_fwd_refine<true>), grf, bl, 0, s, d, in, g, im, b, o);
        else hipLaunchKernelGGL((k_render_fwd_refine<false>), grf, bl, 0, s, d, in, g, im, b, o);
    } else if (d.B == 1 && quad_mode && !split && b.qmask) {
        // one frame, quad waves walking their quad masks: the longest quads' chains are what count here
        const dim3 gq(min((4 * nwaves + 3) / 4, persistent_grid(quad_wg)));
        // GSR_QUAD_PRIO: queue items per XCD that run at issue priority 1 (A/B)
        static const int prio_n = tune_env("GSR_QUAD_PRIO", 0);
        if (exact) hipLaunchKernelGGL((k_render_quad<true>), gq, bl, 0, s, d, in, g, im, b, o, prio_n);
        else hipLaunchKernelGGL((k_render_quad<false>), gq, bl, 0, s, d, in, g, im, b, o, prio_n);
    } else if (d.B == 1 && half_mode) {
        // one frame, half-strip waves: a strip's two halves run in parallel, each lane one
        // (pixel, Gaussian) alpha per k-step -- the longest strip's time is what counts here
        const dim3 gl(min((2 * nwaves + 3) / 4, persistent_grid(half_wg)));
        if (split) {
            if (exact) hipLaunchKernelGGL((k_render_fwd<true, false, false, 1, 5, true>), gl, bl, 0, s, d, in, g, im, b, o);
            else hipLaunchKernelGGL((k_render_fwd<false, false, false, 1, 5, true>), gl, bl, 0, s, d, in, g, im, b, o);
        } else {
            if (exact) hipLaunchKernelGGL((k_render_fwd<true, false, false, 0, 5, true>), gl, bl, 0, s, d, in, g, im, b, o);
            else hipLaunchKernelGGL((k_render_fwd<false, false, false, 0, 5, true>), gl, bl, 0, s, d, in, g, im, b, o);
        }
    } else if (split && in.s_colors == 0) {  // one feature set for the batch: split it once
        hipLaunchKernelGGL(k_split_features, dim3((d.P * GSR_C / 4 + 255) / 256), dim3(256), 0, s,
                           d.P * GSR_C / 4, reinterpret_cast<const float4*>(in.colors),
                           reinterpret_cast<uint4*>(g.fsplit));
        GSR_LAUNCH(0, false, false, 2)
    } else if (split) {
        GSR_LAUNCH(0, false, false, 1)
    } else {
        GSR_LAUNCH(0, false, false)
    }
#undef GSR_LAUNCH
}

}  // namespace gsr
