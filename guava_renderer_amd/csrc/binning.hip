// binning.hip -- tile binning and per-tile depth sort (replaces rasterizer_impl.cu:280-320 of the
// reference: cub InclusiveSum, duplicateWithKeys, cub DeviceRadixSort over 32+msb(T) key bits,
// identifyTileRanges).
//
// Result contract (bit-exact with the reference): tile t's list is every visible Gaussian whose
// tile rect covers t, ordered by (depth float bits, Gaussian index) -- exactly the order a stable
// LSD sort of (tile<<32 | depth bits) over Gaussian-major emission produces.
//
// MI355X structure (no global radix sort):
//   1. k_scan_blocksums   exclusive scan of the per-256-Gaussian tile counts (1 workgroup)
//   2. k_bin_count        per 256 Gaussians: instance offsets + LDS tile histogram; one global
//                         atomic per (workgroup, tile) hands out each workgroup's slot range
//   3. k_tile_scan        exclusive scan of per-tile counts -> ranges; worklist of long tiles
//   4. k_bin_scatter      each instance writes its 64-bit (depth bits, index, strip mask) key into
//                         its tile's segment (order inside a segment arbitrary)
//   5. k_tile_sort_*      one workgroup per tile sorts its segment in LDS: linear bucket pass on
//                         the depth bits + in-bucket ranking on the full key (O(n) for smooth depth
//                         distributions); bitonic in LDS for degenerate buckets; bitonic in global
//                         memory for tiles longer than kSortLargeCap.
// All passes are HBM/L2-bound integer work: 4+4+8+8+5 B per instance.
#include "gsr_internal.h"

namespace gsr {

// ---------------------------------------------------------------- block scan helpers
template <typename TV, int NT>
__device__ __forceinline__ TV block_excl_scan(TV v, TV* total, TV* sh /* NT/64 + 1 */) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    TV x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        TV y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        TV acc = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) {
            TV t = sh[w];
            sh[w] = acc;
            acc += t;
        }
        sh[NT / 64] = acc;
    }
    __syncthreads();
    TV res = sh[wid] + x - v;
    *total = sh[NT / 64];
    __syncthreads();
    return res;
}

// ---------------------------------------------------------------- 1. block-sum scan
__global__ __launch_bounds__(1024) void k_scan_blocksums(uint32_t* __restrict__ bs, int n,
                                                         uint32_t* ctrl, int64_t R_cap) {
    __shared__ uint64_t sh[1024 / 64 + 1];
    const int per = (n + 1023) / 1024;
    const int beg = threadIdx.x * per;
    const int end = min(n, beg + per);
    uint64_t s = 0;
    for (int i = beg; i < end; i++) s += bs[i];
    uint64_t total;
    uint64_t ex = block_excl_scan<uint64_t, 1024>(s, &total, sh);
    for (int i = beg; i < end; i++) {
        const uint32_t v = bs[i];
        bs[i] = (uint32_t)ex;
        ex += v;
    }
    if (threadIdx.x == 0) {
        ctrl[kCtrlRLo] = (uint32_t)min(total, (uint64_t)0xFFFFFFFFu);
        ctrl[kCtrlOverflow] = (total > (uint64_t)R_cap || total >= 0xFFFFFFF0ull) ? 1u : 0u;
    }
}

void launch_scan_blocksums(const Dims& d, const GeomArena& g, int64_t R_cap, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_blocksums, dim3(1), dim3(1024), 0, s, g.blocksums, d.B * d.nblk, g.ctrl,
                       R_cap);
}

// ---------------------------------------------------------------- 2. offsets + tile counts
__global__ __launch_bounds__(kScanBlock) void k_bin_count(Dims d, GeomArena g, ImageArena im,
                                                          BinArena bn) {
    extern __shared__ uint32_t hist[];  // d.T entries when d.T <= kLdsTileHist
    __shared__ uint32_t sh[kScanBlock / 64 + 1];
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.y;
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    const int64_t gid = (int64_t)b * d.P + i;
    const bool valid = i < d.P;
    const uint32_t tiles = valid ? g.tiles[gid] : 0u;
    uint32_t total;
    const uint32_t excl = block_excl_scan<uint32_t, kScanBlock>(tiles, &total, sh) +
                          g.blocksums[(int64_t)b * d.nblk + blockIdx.x];
    if (valid) g.offsets[gid] = excl + tiles;
    const bool use_lds = d.T <= kLdsTileHist;
    if (use_lds) {
        for (int t = threadIdx.x; t < d.T; t += kScanBlock) hist[t] = 0;
        __syncthreads();
    }
    uint32_t* gcount = im.tile_count + (int64_t)b * d.T;
    uint2 rect = make_uint2(0, 0);
    if (tiles) {
        rect = g.rect[gid];
        const uint32_t x0 = rect.x & 0xFFFF, y0 = rect.x >> 16, x1 = rect.y & 0xFFFF, y1 = rect.y >> 16;
        uint32_t k = excl;
        for (uint32_t y = y0; y < y1; y++)
            for (uint32_t x = x0; x < x1; x++) {
                const uint32_t t = y * (uint32_t)d.gx + x;
                bn.inst_slot[k++] = use_lds ? atomicAdd(&hist[t], 1u) : atomicAdd(&gcount[t], 1u);
            }
    }
    if (!use_lds) return;
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += kScanBlock) {
        const uint32_t c = hist[t];
        if (c) hist[t] = atomicAdd(&gcount[t], c);
    }
    __syncthreads();
    if (tiles) {
        const uint32_t x0 = rect.x & 0xFFFF, y0 = rect.x >> 16, x1 = rect.y & 0xFFFF, y1 = rect.y >> 16;
        uint32_t k = excl;
        for (uint32_t y = y0; y < y1; y++)
            for (uint32_t x = x0; x < x1; x++) {
                const uint32_t t = y * (uint32_t)d.gx + x;
                bn.inst_slot[k] += hist[t];
                k++;
            }
    }
}

void launch_bin_count(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                      hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    const size_t lds = d.T <= kLdsTileHist ? (size_t)d.T * 4 : 0;
    hipLaunchKernelGGL(k_bin_count, dim3(d.nblk, d.B), dim3(kScanBlock), lds, s, d, g, im, b);
}

// ---------------------------------------------------------------- 3. tile ranges
// Also emits the render worklist: every tile of the batch ordered by descending log2 list length
// (counting sort over 34 buckets; empty tiles last), so persistent render workgroups take the
// longest tiles first (LPT scheduling) and no XCD is left with only empty tiles.
__global__ __launch_bounds__(1024) void k_tile_scan(int n, const uint32_t* __restrict__ cnt,
                                                    uint2* __restrict__ ranges, uint32_t* ctrl,
                                                    uint32_t* large_list, uint32_t* work_list) {
    constexpr int kBuckets = 34;  // bucket 0: longest (2^32..), bucket 33: empty
    __shared__ uint32_t sh[1024 / 64 + 1];
    __shared__ uint32_t bcount[kBuckets];
    const bool ovf = ctrl[kCtrlOverflow] != 0;
    if (threadIdx.x < kBuckets) bcount[threadIdx.x] = 0;
    const int per = (n + 1023) / 1024;
    const int beg = threadIdx.x * per;
    const int end = min(n, beg + per);
    uint32_t s = 0;
    if (!ovf)
        for (int i = beg; i < end; i++) s += cnt[i];
    uint32_t total;
    uint32_t ex = block_excl_scan<uint32_t, 1024>(s, &total, sh);  // (barriers order bcount init)
    for (int i = beg; i < end; i++) {
        const uint32_t c = ovf ? 0u : cnt[i];
        // empty tiles keep the reference's memset value (0,0) (rasterizer_impl.cu:313)
        ranges[i] = c ? make_uint2(ex, ex + c) : make_uint2(0u, 0u);
        if (c > (uint32_t)kSortSmallCap) large_list[atomicAdd(&ctrl[kCtrlNumLarge], 1u)] = (uint32_t)i;
        const int bk = c ? __clz(c) : kBuckets - 1;
        atomicAdd(&bcount[bk], 1u);
        ex += c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < kBuckets; k++) {
            if (k == kBuckets - 1) ctrl[kCtrlNonEmpty] = acc;
            const uint32_t v = bcount[k];
            bcount[k] = acc;
            acc += v;
        }
    }
    __syncthreads();
    for (int i = beg; i < end; i++) {
        const uint32_t c = ovf ? 0u : cnt[i];
        const int bk = c ? __clz(c) : kBuckets - 1;
        work_list[atomicAdd(&bcount[bk], 1u)] = (uint32_t)i;
    }
}

void launch_tile_scan(const Dims& d, const GeomArena& g, const ImageArena& im, hipStream_t s) {
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, d.B * d.T, im.tile_count, im.ranges,
                       g.ctrl, im.large_list, im.work_list);
}

// ---------------------------------------------------------------- 4. scatter keys
// Minimum over the pixel-centre rectangle dx in [dxl, dxh], dy in [dyl, dyh] (dx = mean - pixel)
// of the conic's quadratic form Q = a dx^2 + 2b dx dy + c dy^2 (power = -Q/2 in the blend).  Q is
// convex (a, c > 0, ac > b^2), so the minimum is 0 if the mean lies inside, else it lies on an edge:
// each edge is a 1-D quadratic minimised by clamping its vertex.
__device__ __forceinline__ float rect_qmin(float a, float b, float c, float dxl, float dxh, float dyl,
                                           float dyh) {
    if (dxl <= 0.f && dxh >= 0.f && dyl <= 0.f && dyh >= 0.f) return 0.f;
    float q = 3.0e38f;
    const float ia = 1.0f / a, ic = 1.0f / c;
    const float xs[2] = {dxl, dxh}, ys[2] = {dyl, dyh};
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const float X = xs[k];
        const float y = fminf(fmaxf(-b * X * ic, dyl), dyh);
        q = fminf(q, a * X * X + 2.f * b * X * y + c * y * y);
        const float Y = ys[k];
        const float x = fminf(fmaxf(-b * Y * ia, dxl), dxh);
        q = fminf(q, a * x * x + 2.f * b * x * Y + c * Y * Y);
    }
    return q;
}

// Strip mask of one (Gaussian, tile) instance: bit s is set unless no pixel centre of the tile's
// s-th 16x4 strip can give alpha = min(0.99, o*exp(-Q/2)) >= 1/255, i.e. unless Q > 2 ln(255 o)
// on the whole strip.  A cleared bit only ever removes pairs the blend skips anyway (alpha < 1/255,
// forward.cu:362-363), so culling with it is decision-preserving; the slack (1e-4 of the form's
// term magnitudes + 1e-3 relative) covers float rounding of both this test and the blend's power.
// Non-finite or non-positive-definite conics keep every strip.
__device__ __forceinline__ uint32_t strip_mask(float4 co, float2 m, int tx, int ty) {
    const float a = co.x, b = co.y, c = co.z, o = co.w;
    if (o < 1.0f / 255.0f) return 0u;  // alpha <= o < 1/255 at every pixel
    if (!(a > 0.f) || !(c > 0.f) || !(a * c - b * b > 0.f) || !(o <= 3.0e38f)) return (1u << kStrips) - 1u;
    const float K = 2.0f * logf(255.0f * o);
    const float dxl = m.x - (float)(tx * GSR_BX + GSR_BX - 1), dxh = m.x - (float)(tx * GSR_BX);
    const float mx = fmaxf(fabsf(dxl), fabsf(dxh));
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < kStrips; s++) {
        const float y0 = (float)(ty * GSR_BY + s * (GSR_BY / kStrips));
        const float dyl = m.y - (y0 + (float)(GSR_BY / kStrips - 1)), dyh = m.y - y0;
        const float my = fmaxf(fabsf(dyl), fabsf(dyh));
        const float slack = 1e-4f * (a * mx * mx + 2.f * fabsf(b) * mx * my + c * my * my) + 1e-3f * K + 1e-3f;
        const float q = rect_qmin(a, b, c, dxl, dxh, dyl, dyh);
        if (!(q > K + slack)) bits |= 1u << s;
    }
    return bits;
}

// Key of an instance: depth bits << 32 | Gaussian index << 4 | strip mask.  Sorting the full key
// orders a tile by (depth, index) as the reference's stable sort does (the index is unique in a
// tile, so the mask bits never decide).
__global__ __launch_bounds__(kScanBlock) void k_bin_scatter(Dims d, GeomArena g, ImageArena im,
                                                            BinArena bn) {
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.y;
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    if (i >= d.P) return;
    const int64_t gid = (int64_t)b * d.P + i;
    const uint32_t tiles = g.tiles[gid];
    if (!tiles) return;
    const uint2 rect = g.rect[gid];
    const float4 co = g.conic[gid];
    const float2 m = g.means2D[gid];
    const uint64_t key_hi = (uint64_t)__float_as_uint(g.depth[gid]) << 32;
    const uint2* rg = im.ranges + (int64_t)b * d.T;
    const uint32_t x0 = rect.x & 0xFFFF, y0 = rect.x >> 16, x1 = rect.y & 0xFFFF, y1 = rect.y >> 16;
    uint32_t k = g.offsets[gid] - tiles;
    for (uint32_t y = y0; y < y1; y++)
        for (uint32_t x = x0; x < x1; x++) {
            const uint32_t t = y * (uint32_t)d.gx + x;
            const uint32_t sm = strip_mask(co, m, (int)x, (int)y);
            bn.keys[rg[t].x + bn.inst_slot[k]] = key_hi | ((uint32_t)i << 4) | sm;
            k++;
        }
}

void launch_bin_scatter(const Dims& d, const GeomArena& g, const ImageArena& im,
                        const BinArena& b, hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    hipLaunchKernelGGL(k_bin_scatter, dim3(d.nblk, d.B), dim3(kScanBlock), 0, s, d, g, im, b);
}

// ---------------------------------------------------------------- 5. per-tile sort
template <typename TV, int NT>
__device__ __forceinline__ TV block_reduce_max(TV v, TV* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { TV y = __shfl_xor(v, off); v = v > y ? v : y; }
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    TV r = sh[0];
#pragma unroll
    for (int w = 1; w < NT / 64; w++) r = r > sh[w] ? r : sh[w];
    __syncthreads();
    return r;
}
template <typename TV, int NT>
__device__ __forceinline__ TV block_reduce_min(TV v, TV* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) { TV y = __shfl_xor(v, off); v = v < y ? v : y; }
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    TV r = sh[0];
#pragma unroll
    for (int w = 1; w < NT / 64; w++) r = r < sh[w] ? r : sh[w];
    __syncthreads();
    return r;
}

// All-ascending bitonic network over n keys (virtual +inf padding to a power of two).
template <int NT>
__device__ void bitonic_sort(uint64_t* key, int n) {
    int N = 1;
    while (N < n) N <<= 1;
    for (int k = 2; k <= N; k <<= 1) {
        const int hk = k >> 1;
        for (int i = threadIdx.x; i < N / 2; i += NT) {
            const int lo = (i / hk) * k + (i % hk);
            const int hi = lo ^ (k - 1);
            if (hi < n) {
                const uint64_t a = key[lo], c = key[hi];
                if (a > c) { key[lo] = c; key[hi] = a; }
            }
        }
        __syncthreads();
        for (int j = k >> 2; j >= 1; j >>= 1) {
            for (int i = threadIdx.x; i < N / 2; i += NT) {
                const int lo = (i / j) * (2 * j) + (i % j);
                const int hi = lo + j;
                if (hi < n) {
                    const uint64_t a = key[lo], c = key[hi];
                    if (a > c) { key[lo] = c; key[hi] = a; }
                }
            }
            __syncthreads();
        }
    }
}

// Sort one tile segment of n <= CAP keys in LDS; writes the Gaussian indices to out[0..n).
// Sorted key -> point_list entry (Gaussian index) and strip mask.
__device__ __forceinline__ void emit(uint64_t key, uint32_t* out, uint8_t* msk, int i) {
    out[i] = ((uint32_t)key) >> 4;
    msk[i] = (uint8_t)(key & 0xF);
}

template <int NT, int CAP>
__device__ void sort_segment_lds(const uint64_t* __restrict__ gkeys, uint32_t* __restrict__ out,
                                 uint8_t* __restrict__ msk, int n, char* smem) {
    constexpr int ITEMS = CAP / NT;
    constexpr uint32_t kDegenerate = 48;
    uint64_t* key = (uint64_t*)smem;                        // CAP
    uint32_t* cnt = (uint32_t*)(smem + 8 * CAP);            // CAP (bucket ends; later output)
    uint16_t* mem = (uint16_t*)(smem + 12 * CAP);           // CAP
    uint32_t* red = (uint32_t*)(smem + 14 * CAP);           // NT/64 + 1
    uint32_t hmin = 0xFFFFFFFFu, hmax = 0u;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        const int i = k * NT + threadIdx.x;
        if (i < n) {
            const uint64_t v = gkeys[i];
            key[i] = v;
            const uint32_t h = (uint32_t)(v >> 32);
            hmin = min(hmin, h);
            hmax = max(hmax, h);
        }
    }
    for (int i = threadIdx.x; i < n; i += NT) cnt[i] = 0;
    hmin = block_reduce_min<uint32_t, NT>(hmin, red);
    hmax = block_reduce_max<uint32_t, NT>(hmax, red);  // includes the barrier after the zeroing
    const float scale = (float)n / ((float)(hmax - hmin) + 1.0f);
    uint32_t bk[ITEMS];
    uint32_t mycnt_max = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        const int i = k * NT + threadIdx.x;
        bk[k] = 0;
        if (i < n) {
            const uint32_t h = (uint32_t)(key[i] >> 32);
            uint32_t bb = (uint32_t)((float)(h - hmin) * scale);
            bb = min(bb, (uint32_t)(n - 1));
            bk[k] = bb;
            const uint32_t c = atomicAdd(&cnt[bb], 1u) + 1u;
            mycnt_max = max(mycnt_max, c);
        }
    }
    const uint32_t maxb = block_reduce_max<uint32_t, NT>(mycnt_max, red);
    if (maxb > kDegenerate) {
        bitonic_sort<NT>(key, n);
        for (int i = threadIdx.x; i < n; i += NT) emit(key[i], out, msk, i);
        return;
    }
    // exclusive scan of bucket counts (chunked per thread), kept as bucket START
    {
        const int per = (n + NT - 1) / NT;
        const int beg = threadIdx.x * per;
        const int end = min(n, beg + per);
        uint32_t s = 0;
        for (int i = beg; i < end; i++) s += cnt[i];
        uint32_t tot;
        uint32_t ex = block_excl_scan<uint32_t, NT>(s, &tot, red);
        for (int i = beg; i < end; i++) {
            const uint32_t c = cnt[i];
            cnt[i] = ex;
            ex += c;
        }
    }
    __syncthreads();
    // scatter member positions; afterwards cnt[b] == end of bucket b == start of bucket b+1
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        const int i = k * NT + threadIdx.x;
        if (i < n) mem[atomicAdd(&cnt[bk[k]], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    uint32_t rank[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        const int i = k * NT + threadIdx.x;
        rank[k] = 0;
        if (i < n) {
            const uint32_t bb = bk[k];
            const uint32_t s = bb ? cnt[bb - 1] : 0u, e = cnt[bb];
            const uint64_t mine = key[i];
            uint32_t r = s;
            for (uint32_t m = s; m < e; m++) r += key[mem[m]] < mine ? 1u : 0u;
            rank[k] = r;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < ITEMS; k++) {
        const int i = k * NT + threadIdx.x;
        if (i < n) cnt[rank[k]] = (uint32_t)key[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += NT) {
        const uint32_t v = cnt[i];
        out[i] = v >> 4;
        msk[i] = (uint8_t)(v & 0xF);
    }
}

constexpr size_t sort_lds_bytes(int NT, int CAP) { return (size_t)14 * CAP + 4 * (NT / 64 + 1) + 16; }

__global__ __launch_bounds__(256) void k_tile_sort_small(ImageArena im, BinArena bn, const uint32_t* ctrl) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (ctrl[kCtrlOverflow]) return;
    const uint2 r = im.ranges[blockIdx.x];
    const int n = (int)(r.y - r.x);
    if (n == 0 || n > kSortSmallCap) return;
    if (n == 1) {
        if (threadIdx.x == 0) emit(bn.keys[r.x], bn.point_list + r.x, bn.smask + r.x, 0);
        return;
    }
    sort_segment_lds<256, kSortSmallCap>(bn.keys + r.x, bn.point_list + r.x, bn.smask + r.x, n, smem);
}

__global__ __launch_bounds__(1024) void k_tile_sort_large(ImageArena im, BinArena bn, const uint32_t* ctrl) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (ctrl[kCtrlOverflow]) return;
    const uint32_t nl = ctrl[kCtrlNumLarge];
    for (uint32_t w = blockIdx.x; w < nl; w += gridDim.x) {
        const uint2 r = im.ranges[im.large_list[w]];
        const int n = (int)(r.y - r.x);
        if (n <= kSortLargeCap) {
            sort_segment_lds<1024, kSortLargeCap>(bn.keys + r.x, bn.point_list + r.x, bn.smask + r.x, n, smem);
        } else {
            // pathological tile: bitonic network directly on the global segment
            bitonic_sort<1024>(bn.keys + r.x, n);
            for (int i = threadIdx.x; i < n; i += 1024) emit(bn.keys[r.x + i], bn.point_list + r.x, bn.smask + r.x, i);
        }
        __syncthreads();
    }
}

void launch_tile_sort(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                      hipStream_t s) {
    const int ntiles = d.B * d.T;
    if (ntiles == 0) return;
    hipLaunchKernelGGL(k_tile_sort_small, dim3(ntiles), dim3(256), sort_lds_bytes(256, kSortSmallCap), s,
                       im, b, (const uint32_t*)g.ctrl);
    static bool attr = false;
    if (!attr) {
        attr = true;
        hipFuncSetAttribute((const void*)k_tile_sort_large, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sort_lds_bytes(1024, kSortLargeCap));
    }
    const int grid = ntiles < 256 ? ntiles : 256;
    hipLaunchKernelGGL(k_tile_sort_large, dim3(grid), dim3(1024), sort_lds_bytes(1024, kSortLargeCap), s,
                       im, b, (const uint32_t*)g.ctrl);
}

}  // namespace gsr
