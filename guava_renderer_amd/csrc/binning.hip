// binning.hip -- tile binning with depth-ordered lists (replaces rasterizer_impl.cu:280-320 of the
// reference: cub InclusiveSum, duplicateWithKeys, cub DeviceRadixSort over 32+msb(T) key bits,
// identifyTileRanges).
//
// Result contract (bit-exact with the reference): tile t's list is every visible Gaussian whose
// tile rect covers t, ordered by (depth float bits, Gaussian index) -- exactly the order a stable
// LSD sort of (tile<<32 | depth bits) over Gaussian-major emission produces.
//
// MI355X structure: the instances (Gaussian x tile, ~6 per Gaussian) are never sorted.  The
// Gaussians are sorted once per frame by (depth bits, index); emitting instances in that order
// with stable per-tile ranks yields every tile's list already ordered.
//   1. k_frame_totals      per-frame instance counts and depth-key ranges, batch R (1 workgroup)
//   2. depth sort          per frame: bucket count on the depth bits (range from preprocess),
//                          bucket scan, scatter of (depth bits, index) keys, in-place ranking of
//                          small buckets, LDS segment sort of the few large ones -> order[]
//   3. k_chunk_count       per 256 depth-ordered Gaussians: tile histogram in LDS from 4 corner
//                          updates per rect (2-D difference array) -> count table row;
//      k_column_scan_wide  per tile: exclusive scan down the table -> chunk bases, tile counts
//   4. k_tile_scan/place   per frame: tile counts -> ranges; longest-first render work list
//   5. k_ordered_scatter   per chunk: load-balanced expansion of the instances over the workgroup,
//                          stable rank = tile base + chunk base + earlier slots covering the tile
//                          (popcount of row/column ballots), plus the exact 4-bit strip mask
// Traffic per instance: 4 B point_list + 1 B strip mask written once; per Gaussian a few words.
#include "gsr_cull.h"
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

// ---------------------------------------------------------------- 1. frame totals
// One workgroup, one wave per frame at a time: the frame's instance count (sum of preprocess's
// block sums) and depth-key range for the bucket sort; then the batch-wide list offsets and the
// batch total against the capacity.
__global__ __launch_bounds__(1024) void k_frame_totals(const uint32_t* __restrict__ bs,
                                                       const uint32_t* __restrict__ bkey, int B, int nblk,
                                                       uint32_t* ctrl, uint32_t* fstat, int64_t R_cap,
                                                       uint32_t* sticky) {
    extern __shared__ uint32_t rf[];  // [B] instances per frame
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int f = wv; f < B; f += 1024 / 64) {
        const uint32_t* fb = bs + (int64_t)f * nblk;
        const uint32_t* fk = bkey + 2 * (int64_t)f * nblk;
        uint32_t r = 0, km = 0, nkm = 0;
        for (int i = lane; i < nblk; i += 64) {
            r += fb[i];
            km = max(km, fk[2 * i]);
            nkm = max(nkm, fk[2 * i + 1]);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            r += __shfl_xor(r, off);
            km = max(km, (uint32_t)__shfl_xor(km, off));
            nkm = max(nkm, (uint32_t)__shfl_xor(nkm, off));
        }
        if (lane == 0) {
            rf[f] = r;
            fstat[kFsWords * f + kFsR] = r;
            fstat[kFsWords * f + kFsKeyMax] = km;
            fstat[kFsWords * f + kFsNotKeyMax] = nkm;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t base = 0;
        for (int f = 0; f < B; f++) {
            fstat[kFsWords * f + kFsRBase] = (uint32_t)min(base, (uint64_t)0xFFFFFFFFu);
            base += rf[f];
        }
        ctrl[kCtrlRLo] = (uint32_t)min(base, (uint64_t)0xFFFFFFFFu);
        const uint32_t ovf = (base > (uint64_t)R_cap || base >= 0xFFFFFFF0ull) ? 1u : 0u;
        ctrl[kCtrlOverflow] = ovf;
        if (sticky) {
            if (ovf) sticky[kStickyOverflow] = 1u;
            sticky[kStickyRMax] = max(sticky[kStickyRMax], (uint32_t)min(base, (uint64_t)0xFFFFFFFFu));
        }
    }
}

void launch_scan_blocksums(const Dims& d, const GeomArena& g, int64_t R_cap, hipStream_t s) {
    hipLaunchKernelGGL(k_frame_totals, dim3(1), dim3(1024), (size_t)d.B * 4, s, g.blocksums, g.blockkey, d.B,
                       d.nblk, g.ctrl, g.fstat, R_cap, g.sticky);
}

// ---------------------------------------------------------------- segment sort (LDS)
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
template <int NT, int CAP>
__device__ void sort_segment_lds(const uint64_t* __restrict__ gkeys, uint32_t* __restrict__ out, int n,
                                 char* smem) {
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
        for (int i = threadIdx.x; i < n; i += NT) out[i] = (uint32_t)key[i];
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
    for (int i = threadIdx.x; i < n; i += NT) out[i] = cnt[i];
}

// ---------------------------------------------------------------- 2. per-frame depth sort
// Bucket of a depth key: linear in the key bits over the frame's [kmin, kmax]; monotone
// non-decreasing in the key, so bucket order is key order and equal keys share a bucket.
__device__ __forceinline__ uint32_t bucket_of(uint32_t key, uint32_t kmin, float scale, int NB) {
    const uint32_t bk = (uint32_t)((float)(key - kmin) * scale);
    return min(bk, (uint32_t)(NB - 1));
}
__device__ __forceinline__ float bucket_scale(uint32_t kmin, uint32_t kmax, int NB) {
    return (float)NB / ((float)(kmax - kmin) + 1.0f);
}

__global__ __launch_bounds__(kScanBlock) void k_bucket_count(Dims d, GeomArena g) {
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.y;
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    if (i >= d.P) return;
    const int64_t gid = (int64_t)b * d.P + i;
    if (!g.tiles[gid]) return;
    const uint32_t kmin = ~g.fstat[kFsWords * b + kFsNotKeyMax], kmax = g.fstat[kFsWords * b + kFsKeyMax];
    const uint32_t bk = bucket_of(__float_as_uint(g.depth[gid]), kmin, bucket_scale(kmin, kmax, d.NB), d.NB);
    g.bslot[gid] = atomicAdd(&g.bstart[(int64_t)b * (d.NB + 1) + bk], 1u);
}

// The same arrival slots with the counting done in LDS: a workgroup takes kCountPer x 1024
// consecutive Gaussians of one frame (neighbours on the avatar, so few distinct depth buckets),
// counts them in an LDS copy of the frame's bucket table (the local slot from the LDS atomic), then
// claims each non-empty bucket's range with ONE returning global atomic.  Slots stay unique and
// dense per bucket; k_bucket_rank orders them.  Scattered returning global atomics run at the
// memory side (MI355X_MICROARCH.md, global atomics), so this cuts them by the Gaussians per
// (workgroup, bucket).
constexpr int kCountThreads = 1024, kCountPer = 8;
// the LDS bucket table of k_bucket_count_lds: at most kLdsBuckets buckets (64 KB), each claimed by
// the register array cl[kLdsBuckets / kCountThreads] below; launch_depth_sort takes the global-atomic
// kernel above that size, and make_dims' nb_cap keeps NB there for every P it serves
constexpr int kLdsBuckets = 16384;
static_assert(kLdsBuckets % kCountThreads == 0, "bucket claims: whole rows of the workgroup");
// PER Gaussians per thread: kCountPer, or fewer for the single-frame launch (more workgroups for a
// latency-bound grid)
// TOT (one frame, no host read-back of R): k_frame_totals folded in -- every workgroup reduces the
// frame's block summaries itself (a few hundred words) for the key range and the overflow test, and
// workgroup 0 writes what k_frame_totals writes; one launch fewer per single-frame forward
template <int PER, bool TOT = false>
__global__ __launch_bounds__(kCountThreads) void k_bucket_count_lds(Dims d, GeomArena g, int64_t R_cap) {
    extern __shared__ uint32_t hist[];  // NB
    const int b = blockIdx.y;
    uint32_t kmin, kmax;
    if constexpr (TOT) {
        __shared__ uint32_t red[3][kCountThreads / 64];
        uint32_t r = 0, km = 0, nkm = 0;
        for (int i = threadIdx.x; i < d.nblk; i += kCountThreads) {
            r += g.blocksums[i];
            km = max(km, g.blockkey[2 * i]);
            nkm = max(nkm, g.blockkey[2 * i + 1]);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            r += __shfl_xor(r, off);
            km = max(km, (uint32_t)__shfl_xor(km, off));
            nkm = max(nkm, (uint32_t)__shfl_xor(nkm, off));
        }
        if ((threadIdx.x & 63) == 0) {
            red[0][threadIdx.x >> 6] = r;
            red[1][threadIdx.x >> 6] = km;
            red[2][threadIdx.x >> 6] = nkm;
        }
        __syncthreads();
        r = 0; km = 0; nkm = 0;
#pragma unroll
        for (int w = 0; w < kCountThreads / 64; w++) {
            r += red[0][w];
            km = max(km, red[1][w]);
            nkm = max(nkm, red[2][w]);
        }
        const uint32_t ovf = ((uint64_t)r > (uint64_t)R_cap || r >= 0xFFFFFFF0u) ? 1u : 0u;
        if (blockIdx.x == 0 && threadIdx.x == 0) {  // (k_frame_totals' words, B = 1)
            g.fstat[kFsR] = r;
            g.fstat[kFsKeyMax] = km;
            g.fstat[kFsNotKeyMax] = nkm;
            g.fstat[kFsRBase] = 0u;
            g.ctrl[kCtrlRLo] = r;
            g.ctrl[kCtrlOverflow] = ovf;
            if (g.sticky) {
                if (ovf) g.sticky[kStickyOverflow] = 1u;
                g.sticky[kStickyRMax] = max(g.sticky[kStickyRMax], r);
            }
        }
        if (ovf) return;
        kmin = ~nkm;
        kmax = km;
    } else {
        if (g.ctrl[kCtrlOverflow]) return;
        kmin = ~g.fstat[kFsWords * b + kFsNotKeyMax];
        kmax = g.fstat[kFsWords * b + kFsKeyMax];
    }
    const int i0 = blockIdx.x * kCountThreads * PER;
    for (int k = threadIdx.x; k < d.NB; k += kCountThreads) hist[k] = 0u;
    __syncthreads();
    const float scale = bucket_scale(kmin, kmax, d.NB);
    uint32_t bk[PER], ls[PER];
#pragma unroll
    for (int p = 0; p < PER; p++) {
        const int i = i0 + p * kCountThreads + threadIdx.x;
        bk[p] = 0xFFFFFFFFu;
        ls[p] = 0u;
        if (i < d.P) {
            const int64_t gid = (int64_t)b * d.P + i;
            if (g.tiles[gid]) {
                bk[p] = bucket_of(__float_as_uint(g.depth[gid]), kmin, scale, d.NB);
                ls[p] = atomicAdd(&hist[bk[p]], 1u);
            }
        }
    }
    __syncthreads();
    uint32_t* bs = g.bstart + (int64_t)b * (d.NB + 1);
    // the workgroup's claims, all of a thread's returning atomics in flight together (NB <= 16384
    // = 16 per thread here; a loop that waits for each claim before the next costs a frame's
    // latency-bound single launch ~16 memory round trips)
    constexpr int kClaims = kLdsBuckets / kCountThreads;
    uint32_t cl[kClaims];
#pragma unroll
    for (int j = 0; j < kClaims; j++) {
        const int k = threadIdx.x + j * kCountThreads;
        cl[j] = k < d.NB ? hist[k] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kClaims; j++)
        if (cl[j]) cl[j] = atomicAdd(&bs[threadIdx.x + j * kCountThreads], cl[j]);
#pragma unroll
    for (int j = 0; j < kClaims; j++) {
        const int k = threadIdx.x + j * kCountThreads;
        if (k < d.NB && hist[k]) hist[k] = cl[j];
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < PER; p++) {
        const int i = i0 + p * kCountThreads + threadIdx.x;
        if (bk[p] != 0xFFFFFFFFu) g.bslot[(int64_t)b * d.P + i] = hist[bk[p]] + ls[p];
    }
}

// One workgroup per frame: bucket counts -> bucket starts (entry NB = visible count); buckets
// longer than kTinyBucket go to the segment-sort worklist.  The table (NB + 1 <= 16385 words) is
// staged through LDS with coalesced loads and stores; each thread scans a contiguous run of it
// there (odd run length: conflict-free), so no thread walks global memory at a stride.
constexpr int kBucketScanLds = (1 << 14) + 1;
__global__ __launch_bounds__(1024) void k_bucket_scan(Dims d, GeomArena g) {
    __shared__ uint32_t sh[1024 / 64 + 1];
    __shared__ uint32_t tab[kBucketScanLds];
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.x;
    uint32_t* bs = g.bstart + (int64_t)b * (d.NB + 1);
    const int n = d.NB + 1;
    const bool staged = n <= kBucketScanLds;  // uniform (NB <= 16384 up to 512k Gaussians)
    uint32_t* t = staged ? tab : bs;
    if (staged) {
        for (int k = threadIdx.x; k < n; k += 1024) tab[k] = bs[k];
        __syncthreads();
    }
    const int per = (n + 1023) / 1024;
    const int beg = threadIdx.x * per;
    const int end = min(n, beg + per);
    uint32_t s = 0;
    for (int k = beg; k < end; k++) s += t[k];
    uint32_t total;
    uint32_t ex = block_excl_scan<uint32_t, 1024>(s, &total, sh);  // (barriers inside)
    for (int k = beg; k < end; k++) {
        const uint32_t c = t[k];
        t[k] = ex;
        if (c > (uint32_t)kTinyBucket) g.big[atomicAdd(&g.ctrl[kCtrlNumBig], 1u)] = (uint32_t)(b * d.NB + k);
        ex += c;
    }
    if (staged) {
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += 1024) bs[k] = tab[k];
    }
    if (threadIdx.x == 0) g.fstat[kFsWords * b + kFsVisible] = total;
}

// SCAN (one frame, NB + 1 words fitting the LDS): k_bucket_scan folded in -- every workgroup scans
// the frame's bucket counts itself in LDS (the same runs and block scan as k_bucket_scan, so the same
// starts), and workgroup 0 writes the starts back, lists the large buckets and the visible count:
// one launch fewer per single-frame forward.
template <bool SCAN = false>
__global__ __launch_bounds__(kScanBlock) void k_bucket_scatter(Dims d, GeomArena g) {
    extern __shared__ uint32_t btab[];  // SCAN: the frame's NB + 1 bucket starts
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.y;
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    uint32_t* bs = g.bstart + (int64_t)b * (d.NB + 1);
    if constexpr (SCAN) {
        __shared__ uint32_t sh[kScanBlock / 64 + 1];
        const int n = d.NB + 1;
        for (int k = threadIdx.x; k < n; k += kScanBlock) btab[k] = bs[k];
        __syncthreads();
        const int per = (n + kScanBlock - 1) / kScanBlock;
        const int beg = threadIdx.x * per, end = min(n, beg + per);
        uint32_t sum = 0;
        for (int k = beg; k < end; k++) sum += btab[k];
        uint32_t total;
        uint32_t ex = block_excl_scan<uint32_t, kScanBlock>(sum, &total, sh);  // (barriers inside)
        for (int k = beg; k < end; k++) {
            const uint32_t c = btab[k];
            btab[k] = ex;
            if (blockIdx.x == 0 && c > (uint32_t)kTinyBucket)
                g.big[atomicAdd(&g.ctrl[kCtrlNumBig], 1u)] = (uint32_t)(b * d.NB + k);
            ex += c;
        }
        __syncthreads();
        if (blockIdx.x == 0) {
            for (int k = threadIdx.x; k < n; k += kScanBlock) bs[k] = btab[k];
            if (threadIdx.x == 0) g.fstat[kFsWords * b + kFsVisible] = total;
        }
    }
    if (i >= d.P) return;
    const int64_t gid = (int64_t)b * d.P + i;
    if (!g.tiles[gid]) return;
    const uint32_t kmin = ~g.fstat[kFsWords * b + kFsNotKeyMax], kmax = g.fstat[kFsWords * b + kFsKeyMax];
    const uint32_t key = __float_as_uint(g.depth[gid]);
    const uint32_t bk = bucket_of(key, kmin, bucket_scale(kmin, kmax, d.NB), d.NB);
    const uint32_t pos = (SCAN ? btab[bk] : bs[bk]) + g.bslot[gid];
    g.skey[(int64_t)b * d.P + pos] = ((uint64_t)key << 32) | (uint32_t)i;
}

// Small buckets: each key's final position is its bucket start plus the number of smaller keys in
// the bucket (keys are unique: the index is in the low word).  A small bucket holding one of the
// workgroup's keys lies within kTinyBucket of the workgroup's range, so the keys it compares are
// staged in LDS with that halo (one coalesced load each instead of a global load per comparison).
__global__ __launch_bounds__(kScanBlock) void k_bucket_rank(Dims d, GeomArena g) {
    __shared__ uint64_t win[kScanBlock + 2 * kTinyBucket];
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.y;
    const int V = (int)g.fstat[kFsWords * b + kFsVisible];
    const int j0 = blockIdx.x * kScanBlock;
    if (j0 >= V) return;  // (uniform)
    const uint64_t* sk = g.skey + (int64_t)b * d.P;
    for (int t = threadIdx.x; t < kScanBlock + 2 * kTinyBucket; t += kScanBlock) {
        const int m = j0 - kTinyBucket + t;
        win[t] = (m >= 0 && m < V) ? sk[m] : 0ull;
    }
    __syncthreads();
    const int j = j0 + threadIdx.x;
    if (j >= V) return;
    const uint32_t kmin = ~g.fstat[kFsWords * b + kFsNotKeyMax], kmax = g.fstat[kFsWords * b + kFsKeyMax];
    const uint64_t key = win[threadIdx.x + kTinyBucket];
    const uint32_t bk = bucket_of((uint32_t)(key >> 32), kmin, bucket_scale(kmin, kmax, d.NB), d.NB);
    const uint32_t* bs = g.bstart + (int64_t)b * (d.NB + 1);
    const uint32_t s0 = bs[bk], e0 = bs[bk + 1];
    if (e0 - s0 > (uint32_t)kTinyBucket) return;
    uint32_t r = s0;
    // (win[m - j0 + kTinyBucket] = sk[m] for m in [j0 - kTinyBucket, j0 + kScanBlock + kTinyBucket))
    for (int m = (int)s0 - j0 + kTinyBucket; m < (int)e0 - j0 + kTinyBucket; m++) r += win[m] < key ? 1u : 0u;
    g.order[(int64_t)b * d.P + r] = (uint32_t)key;
}

constexpr size_t sort_lds_bytes(int NT, int CAP) { return (size_t)14 * CAP + 4 * (NT / 64 + 1) + 16; }

// Large buckets (worklist from k_bucket_scan): LDS sort, 256 threads up to kSortSmallCap keys,
// 1024 threads up to kSortLargeCap, a bitonic network in global memory beyond.
// ALL: one launch takes every listed bucket (the single-frame path, whose few long buckets do not
// pay for a second launch)
template <int NT, int CAP, bool ALL = false>
__global__ __launch_bounds__(NT) void k_bucket_sort(Dims d, GeomArena g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if (g.ctrl[kCtrlOverflow]) return;
    const uint32_t nbig = g.ctrl[kCtrlNumBig];
    for (uint32_t w = blockIdx.x; w < nbig; w += gridDim.x) {
        const uint32_t fb = g.big[w];
        const int b = (int)(fb / (uint32_t)d.NB), bk = (int)(fb % (uint32_t)d.NB);
        const uint32_t* bs = g.bstart + (int64_t)b * (d.NB + 1);
        const uint32_t s0 = bs[bk];
        const int n = (int)(bs[bk + 1] - s0);
        const bool mine = ALL || ((CAP == kSortSmallCap) ? n <= kSortSmallCap : n > kSortSmallCap);
        if (!mine) continue;
        uint64_t* keys = g.skey + (int64_t)b * d.P + s0;
        uint32_t* out = g.order + (int64_t)b * d.P + s0;
        if (n <= CAP) {
            sort_segment_lds<NT, CAP>(keys, out, n, smem);
        } else {
            bitonic_sort<NT>(keys, n);
            for (int i = threadIdx.x; i < n; i += NT) out[i] = (uint32_t)keys[i];
        }
        __syncthreads();
    }
}

void launch_depth_sort(const Dims& d, const GeomArena& g, hipStream_t s, int64_t fused_totals_cap) {
    if (d.P == 0 || d.B == 0) return;
    // fused_totals_cap >= 0: launch_scan_blocksums deferred the frame totals to the bucket count
    const bool fuse = fused_totals_cap >= 0 && d.B == 1 && d.NB <= kLdsBuckets;
    if (fused_totals_cap >= 0 && !fuse) launch_scan_blocksums(d, g, fused_totals_cap, s);
    if (d.NB <= kLdsBuckets) {  // every bucket has a claim slot (kClaims per thread)
        // GSR_B1_COUNT_PER: Gaussians per thread of the single-frame count, 2 (49 workgroups at 100k
        // Gaussians: -5 us per frame against 8) or kCountPer (A/B)
        static const int b1_per = tune_env("GSR_B1_COUNT_PER", 2);
        if (d.B == 1 && b1_per == 2) {
            const int per_wg = kCountThreads * 2;
            const dim3 gr((d.P + per_wg - 1) / per_wg, d.B);
            if (fuse)
                hipLaunchKernelGGL((k_bucket_count_lds<2, true>), gr, dim3(kCountThreads), (size_t)d.NB * 4, s, d, g,
                                   fused_totals_cap);
            else
                hipLaunchKernelGGL((k_bucket_count_lds<2>), gr, dim3(kCountThreads), (size_t)d.NB * 4, s, d, g,
                                   (int64_t)0);
        } else {
            const int per_wg = kCountThreads * kCountPer;
            const dim3 gr((d.P + per_wg - 1) / per_wg, d.B);
            if (fuse)
                hipLaunchKernelGGL((k_bucket_count_lds<kCountPer, true>), gr, dim3(kCountThreads), (size_t)d.NB * 4,
                                   s, d, g, fused_totals_cap);
            else
                hipLaunchKernelGGL((k_bucket_count_lds<kCountPer>), gr, dim3(kCountThreads), (size_t)d.NB * 4, s, d,
                                   g, (int64_t)0);
        }
    } else {
        hipLaunchKernelGGL(k_bucket_count, dim3(d.nblk, d.B), dim3(kScanBlock), 0, s, d, g);
    }
    // GSR_B1_SCAN_FUSED=0: the single-frame bucket scan in its own launch (A/B)
    static const bool scan_fused_on = tune_env("GSR_B1_SCAN_FUSED", 1) != 0;
    if (d.B == 1 && scan_fused_on && (size_t)(d.NB + 1) * 4 <= 65536) {
        hipLaunchKernelGGL(k_bucket_scatter<true>, dim3(d.nblk, d.B), dim3(kScanBlock), (size_t)(d.NB + 1) * 4, s, d,
                           g);
    } else {
        hipLaunchKernelGGL(k_bucket_scan, dim3(d.B), dim3(1024), 0, s, d, g);
        hipLaunchKernelGGL(k_bucket_scatter<false>, dim3(d.nblk, d.B), dim3(kScanBlock), 0, s, d, g);
    }
    hipLaunchKernelGGL(k_bucket_rank, dim3(d.nblk, d.B), dim3(kScanBlock), 0, s, d, g);
    static bool attr = false;
    if (!attr) {
        attr = true;
        hipFuncSetAttribute((const void*)k_bucket_sort<1024, kSortLargeCap>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sort_lds_bytes(1024, kSortLargeCap));
        hipFuncSetAttribute((const void*)k_bucket_sort<1024, kSortLargeCap, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)sort_lds_bytes(1024, kSortLargeCap));
    }
    // GSR_SORT1=0: the two launches at B = 1 too (A/B)
    static const bool one_launch = tune_env("GSR_SORT1", 1) != 0;
    if (d.B == 1 && one_launch) {
        hipLaunchKernelGGL((k_bucket_sort<1024, kSortLargeCap, true>), dim3(persistent_grid(1) / 4), dim3(1024),
                           sort_lds_bytes(1024, kSortLargeCap), s, d, g);
        return;
    }
    hipLaunchKernelGGL((k_bucket_sort<256, kSortSmallCap>), dim3(persistent_grid(2)), dim3(256),
                       sort_lds_bytes(256, kSortSmallCap), s, d, g);
    hipLaunchKernelGGL((k_bucket_sort<1024, kSortLargeCap>), dim3(persistent_grid(1) / 4), dim3(1024),
                       sort_lds_bytes(1024, kSortLargeCap), s, d, g);
}

// ---------------------------------------------------------------- 3. instance count table
// Inclusive scan over aligned 8-lane groups: DPP row_shr inside the 16-lane rows, a lane whose source
// lies in the previous group adds nothing (three VALU steps, no LDS permutes).
__device__ __forceinline__ int scan8(int v) {
    const int l8 = threadIdx.x & 7;
    int t = __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += l8 >= 1 ? t : 0;
    t = __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += l8 >= 2 ? t : 0;
    t = __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += l8 >= 4 ? t : 0;
    return v;
}

// Tile histogram of one chunk of d.chunk depth-ordered Gaussians: each rect adds +1/-1 at its four
// corners of a (gx+1) x (gy+1) difference array in LDS; a 2-D prefix sum gives the per-tile counts.
// GROUP8 (default): the prefix sums by 8-lane groups, one row (then one column) per group, each lane
// summing a run of ceil(n/8) cells and the 8 run sums scanned with DPP -- every row at once instead
// of one row per wave at a time with a 6-step LDS-permute scan (the kernel's VALU and LDS waits).
template <bool GROUP8>
__global__ __launch_bounds__(kScanBlock) void k_chunk_count(Dims d, GeomArena g) {
    extern __shared__ int diff[];  // (gx+1)*(gy+1)
    if (g.ctrl[kCtrlOverflow]) return;
    const int b = blockIdx.y, c = blockIdx.x;
    const uint32_t V = g.fstat[kFsWords * b + kFsVisible];
    if ((uint32_t)c * d.chunk >= V) return;
    const int W1 = d.gx + 1, H1 = d.gy + 1;
    for (int k = threadIdx.x; k < W1 * H1; k += kScanBlock) diff[k] = 0;
    __syncthreads();
    for (int k = 0; k < d.chunk; k += kScanBlock) {
        const uint32_t j = (uint32_t)c * d.chunk + k + threadIdx.x;
        if (j < V) {
            const uint32_t gi = g.order[(int64_t)b * d.P + j];
            const uint2 r = g.rect[(int64_t)b * d.P + gi];
            const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
            atomicAdd(&diff[y0 * W1 + x0], 1);
            atomicAdd(&diff[y0 * W1 + x1], -1);
            atomicAdd(&diff[y1 * W1 + x0], -1);
            atomicAdd(&diff[y1 * W1 + x1], 1);
        }
    }
    __syncthreads();
    // 2-D inclusive prefix of the difference array, one wave per row (lanes along x), then one wave
    // per column (lanes along y; the odd pitch W1 keeps the column reads conflict-free), 64
    // elements per step with the carry in a register; then the table row is written coalesced
    if (GROUP8) {
        const int g8 = threadIdx.x >> 3, l8 = threadIdx.x & 7;
        const int cx = (d.gx + 7) >> 3, cy = (d.gy + 7) >> 3;
        for (int y = g8; y < d.gy; y += kScanBlock / 8) {  // (whole 8-lane groups take a row or not)
            int* rowp = diff + y * W1;
            const int x0 = l8 * cx, x1 = min(d.gx, x0 + cx);
            int s = 0;
            for (int x = x0; x < x1; x++) s += rowp[x];
            int run = scan8(s) - s;
            for (int x = x0; x < x1; x++) { run += rowp[x]; rowp[x] = run; }
        }
        __syncthreads();
        for (int x = g8; x < d.gx; x += kScanBlock / 8) {
            const int y0 = l8 * cy, y1 = min(d.gy, y0 + cy);
            int s = 0;
            for (int y = y0; y < y1; y++) s += diff[y * W1 + x];
            int run = scan8(s) - s;
            for (int y = y0; y < y1; y++) { run += diff[y * W1 + x]; diff[y * W1 + x] = run; }
        }
        __syncthreads();
        uint32_t* row = g.table + ((int64_t)b * d.nchunk + c) * d.T;
        const int sy = kScanBlock / d.gx, sx = kScanBlock - sy * d.gx;
        int y = threadIdx.x / d.gx, x = threadIdx.x - y * d.gx;
        for (int t = threadIdx.x; t < d.T; t += kScanBlock) {
            row[t] = (uint32_t)diff[y * W1 + x];
            x += sx;
            y += sy;
            if (x >= d.gx) { x -= d.gx; y++; }
        }
        return;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int kWaves = kScanBlock / 64;
    for (int y = wv; y < d.gy; y += kWaves) {
        int carry = 0;
        for (int x0 = 0; x0 < d.gx; x0 += 64) {
            const int x = x0 + lane;
            int v = x < d.gx ? diff[y * W1 + x] : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(v, o);
                if (lane >= o) v += t;
            }
            if (x < d.gx) diff[y * W1 + x] = v + carry;
            carry += __shfl(v, 63);
        }
    }
    __syncthreads();
    for (int x = wv; x < d.gx; x += kWaves) {
        int carry = 0;
        for (int y0 = 0; y0 < d.gy; y0 += 64) {
            const int y = y0 + lane;
            int v = y < d.gy ? diff[y * W1 + x] : 0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(v, o);
                if (lane >= o) v += t;
            }
            if (y < d.gy) diff[y * W1 + x] = v + carry;
            carry += __shfl(v, 63);
        }
    }
    __syncthreads();
    uint32_t* row = g.table + ((int64_t)b * d.nchunk + c) * d.T;
    for (int t = threadIdx.x; t < d.T; t += kScanBlock) {
        const int y = t / d.gx, x = t - y * d.gx;
        row[t] = (uint32_t)diff[y * W1 + x];
    }
}

// Per tile: exclusive scan down the (chunk x tile) count table -> each chunk's base in the tile,
// and the tile's count.  16 waves per 64 tiles: wave w sums its slice of the rows (lane = tile,
// 8 loads in flight), the slice totals are scanned across the waves through LDS, and each wave
// rewrites its slice from its offset (the second read hits L2).  16x the waves of one thread per
// tile walking all rows serially (measured 75 -> 61 us per 32-frame chunk_count stage).
constexpr int kColWaves = 16;
__global__ __launch_bounds__(64 * kColWaves) void k_column_scan_wide(Dims d, GeomArena g, ImageArena im) {
    __shared__ uint32_t tot[kColWaves][64];
    const int b = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int t = blockIdx.x * 64 + lane;
    const bool ok = t < d.T && !g.ctrl[kCtrlOverflow];
    const int nc = (int)((g.fstat[kFsWords * b + kFsVisible] + d.chunk - 1) / d.chunk);
    const int per = (nc + kColWaves - 1) / kColWaves;
    const int c0 = w * per, c1 = min(nc, c0 + per);
    uint32_t* col = g.table + (int64_t)b * d.nchunk * d.T + t;
    uint32_t sum = 0;
    if (ok) {
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = col[(int64_t)(c + u) * d.T];
#pragma unroll
            for (int u = 0; u < 8; u++) sum += v[u];
        }
        for (; c < c1; c++) sum += col[(int64_t)c * d.T];
    }
    tot[w][lane] = sum;
    __syncthreads();
    uint32_t acc = 0, all = 0;
#pragma unroll
    for (int u = 0; u < kColWaves; u++) {
        const uint32_t x = tot[u][lane];
        acc += u < w ? x : 0u;
        all += x;
    }
    if (ok) {
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = col[(int64_t)(c + u) * d.T];
#pragma unroll
            for (int u = 0; u < 8; u++) { col[(int64_t)(c + u) * d.T] = acc; acc += v[u]; }
        }
        for (; c < c1; c++) {
            const uint32_t v = col[(int64_t)c * d.T];
            col[(int64_t)c * d.T] = acc;
            acc += v;
        }
        if (w == 0) im.tile_count[(int64_t)b * d.T + t] = all;
    } else if (t < d.T && w == 0) {
        im.tile_count[(int64_t)b * d.T + t] = 0u;  // overflow: no instances
    }
}

void launch_chunk_count(const Dims& d, const GeomArena& g, const ImageArena& im, hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    const size_t lds = (size_t)(d.gx + 1) * (d.gy + 1) * 4;
    static size_t attr = 0;
    if (lds > 65536 && attr < lds) {
        attr = lds;
        hipFuncSetAttribute((const void*)k_chunk_count<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipFuncSetAttribute((const void*)k_chunk_count<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    static const bool g8 = tune_env("GSR_CHUNK_SCAN8", 1) != 0;
    if (g8) hipLaunchKernelGGL(k_chunk_count<true>, dim3(d.nchunk, d.B), dim3(kScanBlock), lds, s, d, g);
    else hipLaunchKernelGGL(k_chunk_count<false>, dim3(d.nchunk, d.B), dim3(kScanBlock), lds, s, d, g);
    hipLaunchKernelGGL(k_column_scan_wide, dim3((d.T + 63) / 64, d.B), dim3(64 * kColWaves), 0, s, d, g, im);
}

// ---------------------------------------------------------------- 4. tile ranges
// Per frame (one workgroup each): exclusive scan of the tile counts from the frame's batch-wide
// offset -> ranges (empty tiles keep the reference's memset value (0,0), rasterizer_impl.cu:313),
// and a histogram of the tiles over the work-list buckets (clz of the list length).  Then every
// frame places its tiles into the batch-wide render work list, bucket-major (longest lists first,
// empty tiles last), so persistent render workgroups take the longest tiles first.
__global__ __launch_bounds__(1024) void k_tile_scan(Dims d, GeomArena g, ImageArena im) {
    __shared__ uint32_t sh[1024 / 64 + 1];
    __shared__ uint32_t h[kLptBuckets];
    const int b = blockIdx.x;
    const bool ovf = g.ctrl[kCtrlOverflow] != 0;
    if (threadIdx.x < kLptBuckets) h[threadIdx.x] = 0;
    const int per = (d.T + 1023) / 1024;
    const int beg = threadIdx.x * per, end = min(d.T, beg + per);
    const uint32_t* cnt = im.tile_count + (int64_t)b * d.T;
    uint32_t s = 0;
    if (!ovf)
        for (int t = beg; t < end; t++) s += cnt[t];
    uint32_t total;
    uint32_t ex = block_excl_scan<uint32_t, 1024>(s, &total, sh) + (ovf ? 0u : g.fstat[kFsWords * b + kFsRBase]);
    uint2* rg = im.ranges + (int64_t)b * d.T;
    for (int t = beg; t < end; t++) {
        const uint32_t c = ovf ? 0u : cnt[t];
        rg[t] = c ? make_uint2(ex, ex + c) : make_uint2(0u, 0u);
        atomicAdd(&h[c ? __clz(c) : kLptBuckets - 1], 1u);
        ex += c;
    }
    __syncthreads();
    if (threadIdx.x < kLptBuckets) im.lpt_hist[b * kLptBuckets + threadIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(1024) void k_tile_place(Dims d, GeomArena g, ImageArena im) {
    extern __shared__ uint32_t hist[];  // [B][kLptBuckets]
    __shared__ uint32_t cur[kLptBuckets];
    const int b = blockIdx.x;
    for (int i = threadIdx.x; i < d.B * kLptBuckets; i += 1024) hist[i] = im.lpt_hist[i];
    __syncthreads();
    if (threadIdx.x < kLptBuckets) {  // bucket totals over all frames, and this frame's share before it
        const int bk = threadIdx.x;
        uint32_t tot = 0, mine = 0;
        for (int f = 0; f < d.B; f++) {
            const uint32_t v = hist[f * kLptBuckets + bk];
            tot += v;
            if (f < b) mine += v;
        }
        cur[bk] = tot;
        hist[bk] = mine;  // (row 0 is no longer needed)
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // start of this frame's run in each bucket (bucket-major)
        uint32_t acc = 0;
        for (int bk = 0; bk < kLptBuckets; bk++) {
            const uint32_t t = cur[bk];
            if (b == 0 && bk == kLptBuckets - 1) g.ctrl[kCtrlNonEmpty] = acc;  // non-empty tiles
            cur[bk] = acc + hist[bk];
            acc += t;
        }
    }
    __syncthreads();
    const bool ovf = g.ctrl[kCtrlOverflow] != 0;
    const uint32_t* cnt = im.tile_count + (int64_t)b * d.T;
    for (int t = threadIdx.x; t < d.T; t += 1024) {
        const uint32_t c = ovf ? 0u : cnt[t];
        im.work_list[atomicAdd(&cur[c ? __clz(c) : kLptBuckets - 1], 1u)] = (uint32_t)(b * d.T + t);
    }
}

// One frame (the per-frame drop-in path): k_tile_scan and k_tile_place in one workgroup -- the
// work-list bucket starts are this frame's own histogram's prefix (one launch instead of two).
__global__ __launch_bounds__(1024) void k_tile_scan_place1(Dims d, GeomArena g, ImageArena im) {
    __shared__ uint32_t sh[1024 / 64 + 1];
    __shared__ uint32_t h[kLptBuckets];
    const bool ovf = g.ctrl[kCtrlOverflow] != 0;
    if (threadIdx.x < kLptBuckets) h[threadIdx.x] = 0;
    const int per = (d.T + 1023) / 1024;
    const int beg = threadIdx.x * per, end = min(d.T, beg + per);
    const uint32_t* cnt = im.tile_count;
    uint32_t s = 0;
    if (!ovf)
        for (int t = beg; t < end; t++) s += cnt[t];
    uint32_t total;
    uint32_t ex = block_excl_scan<uint32_t, 1024>(s, &total, sh) + (ovf ? 0u : g.fstat[kFsRBase]);
    for (int t = beg; t < end; t++) {
        const uint32_t c = ovf ? 0u : cnt[t];
        im.ranges[t] = c ? make_uint2(ex, ex + c) : make_uint2(0u, 0u);
        atomicAdd(&h[c ? __clz(c) : kLptBuckets - 1], 1u);
        ex += c;
    }
    __syncthreads();
    if (threadIdx.x < kLptBuckets) im.lpt_hist[threadIdx.x] = h[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {  // bucket starts, longest lists first, empty tiles last
        uint32_t acc = 0;
        for (int bk = 0; bk < kLptBuckets; bk++) {
            const uint32_t t = h[bk];
            if (bk == kLptBuckets - 1) g.ctrl[kCtrlNonEmpty] = acc;
            h[bk] = acc;
            acc += t;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += 1024) {
        const uint32_t c = ovf ? 0u : cnt[t];
        im.work_list[atomicAdd(&h[c ? __clz(c) : kLptBuckets - 1], 1u)] = (uint32_t)t;
    }
}

// k_tile_scan_place1's work by one workgroup of NT threads (the single-frame ordered scatter's
// workgroup 0, TS): ranges, the work-list histogram, the longest-first work list, the non-empty count
template <int NT>
__device__ void tile_scan_place_wg(const Dims& d, const GeomArena& g, const ImageArena& im) {
    __shared__ uint32_t sh[NT / 64 + 1];
    __shared__ uint32_t h[kLptBuckets];
    const bool ovf = g.ctrl[kCtrlOverflow] != 0;
    if (threadIdx.x < kLptBuckets) h[threadIdx.x] = 0;
    const int per = (d.T + NT - 1) / NT;
    const int beg = threadIdx.x * per, end = min(d.T, beg + per);
    const uint32_t* cnt = im.tile_count;
    uint32_t sum = 0;
    if (!ovf)
        for (int t = beg; t < end; t++) sum += cnt[t];
    uint32_t total;
    uint32_t ex = block_excl_scan<uint32_t, NT>(sum, &total, sh) + (ovf ? 0u : g.fstat[kFsRBase]);
    for (int t = beg; t < end; t++) {
        const uint32_t c = ovf ? 0u : cnt[t];
        im.ranges[t] = c ? make_uint2(ex, ex + c) : make_uint2(0u, 0u);
        atomicAdd(&h[c ? __clz(c) : kLptBuckets - 1], 1u);
        ex += c;
    }
    __syncthreads();
    if (threadIdx.x < kLptBuckets) im.lpt_hist[threadIdx.x] = h[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {  // bucket starts, longest lists first, empty tiles last
        uint32_t acc = 0;
        for (int bk = 0; bk < kLptBuckets; bk++) {
            const uint32_t t = h[bk];
            if (bk == kLptBuckets - 1) g.ctrl[kCtrlNonEmpty] = acc;
            h[bk] = acc;
            acc += t;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += NT) {
        const uint32_t c = ovf ? 0u : cnt[t];
        im.work_list[atomicAdd(&h[c ? __clz(c) : kLptBuckets - 1], 1u)] = (uint32_t)t;
    }
}

// the single-frame tile scan runs inside the ordered scatter (its workgroup 0, k_ordered_scatter TS;
// the production scatter only: the A/B variants keep the separate launch)
static bool tile_scan_in_scatter(const Dims& d) {
    static const bool on = tune_env("GSR_B1_TILESCAN_FUSED", 1) != 0 && tune_env("GSR_SCATTER_ABLATE", 0) == 0 &&
                           tune_env("GSR_SCATTER_WAVESEARCH", 1) != 0;  // 0: its own launch (A/B)
    return on && d.B == 1 && d.P > 0;
}

void launch_tile_scan(const Dims& d, const GeomArena& g, const ImageArena& im, hipStream_t s) {
    if (tile_scan_in_scatter(d)) return;
    if (d.B == 1) {
        hipLaunchKernelGGL(k_tile_scan_place1, dim3(1), dim3(1024), 0, s, d, g, im);
        return;
    }
    hipLaunchKernelGGL(k_tile_scan, dim3(d.B), dim3(1024), 0, s, d, g, im);
    hipLaunchKernelGGL(k_tile_place, dim3(d.B), dim3(1024), (size_t)d.B * kLptBuckets * 4, s, d, g, im);
}

// ---------------------------------------------------------------- strip masks
// (rect_qmin, strip_pre and box_reach: gsr_cull.h, shared with render_fwd's quad waves)

// Strip mask of one (Gaussian, tile) instance: bit s is set unless no pixel centre of the tile's
// s-th strip (strip_origin, kStripW x kStripH) can give alpha = min(0.99, o*exp(-Q/2)) >= 1/255, i.e. unless Q > 2 ln(255 o)
// on the whole strip.  A cleared bit only ever removes pairs the blend skips anyway (alpha < 1/255,
// forward.cu:362-363), so culling with it is decision-preserving; the slack (1e-4 of the form's
// term magnitudes + 1e-3 relative) covers float rounding of both this test and the blend's power.
// Non-finite or non-positive-definite conics keep every strip.  Host-callable for
// tools/strip_mask_check.cpp (brute force over the strip's 64 pixels: no strip with a pixel at
// Q <= K is ever cleared; 0.4% more strips kept than needed on random conics).
// strip_mask_loop: the four box_reach calls; strip_mask: the same bits from sub_reach4<8> (the 2 x 2
// strips of a tile share their column and row terms, no divergent branches), checked equal to the
// loop by tools/strip_mask_check.cpp (tests/test_cull.py)
__host__ __device__ __forceinline__ uint32_t strip_mask_loop(float4 co, float4 pre, float2 m, int tx, int ty) {
    const uint32_t mode = __builtin_bit_cast(uint32_t, pre.w);
    if (mode == 1u) return 0u;
    if (mode == 2u) return (1u << kStrips) - 1u;
    const float a = co.x, b = co.y, c = co.z;
    const float K = pre.x;
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < kStrips; s++) {
        int sx0, sy0;
        strip_origin(tx, ty, s, sx0, sy0);
        if (box_reach(a, b, c, K, pre.y, pre.z, m, (float)sx0, (float)sy0, (float)kStripW, (float)kStripH))
            bits |= 1u << s;
    }
    return bits;
}

__host__ __device__ __forceinline__ uint32_t strip_mask(float4 co, float4 pre, float2 m, int tx, int ty) {
    if constexpr (kStripW != 8 || kStripH != 8) {
        return strip_mask_loop(co, pre, m, tx, ty);
    } else {
        const uint32_t mode = __builtin_bit_cast(uint32_t, pre.w);
        if (mode == 1u) return 0u;
        if (mode == 2u) return (1u << kStrips) - 1u;
        return sub_reach4<8>(co.x, co.y, co.z, pre.x, pre.y, pre.z, m, (float)(tx * GSR_BX), (float)(ty * GSR_BY));
    }
}

// Quad mask of one instance (single-frame arenas, BinArena.qmask): bit 4 s + q is set when strip s's
// bit is (strip_mask) and quad q (4x4; x offset 4 (q & 1), y offset 4 (q >> 1)) of that strip passes
// box_reach (quad_reach4: the four quads' tests with shared terms).  A cleared bit only drops pairs the
// blend skips; the single-frame quad render waves walk only their quad's entries with it.  (A reach-
// box test in its place costs the scatter 4 us instead of 30 at one frame, but keeps 45% more of the
// longest quad's Gaussians: the render lost more than the scatter saved.)
__device__ __forceinline__ uint32_t quad_mask(float4 co, float4 pre, float2 m, int tx, int ty, uint32_t sm) {
    const uint32_t mode = __builtin_bit_cast(uint32_t, pre.w);
    uint32_t bits = 0;
#pragma unroll
    for (int st = 0; st < kStrips; st++) {
        if (!((sm >> st) & 1u)) continue;
        if (mode == 2u) {
            bits |= 0xFu << (4 * st);
            continue;
        }
        int sx0, sy0;
        strip_origin(tx, ty, st, sx0, sy0);
        bits |= quad_reach4(co.x, co.y, co.z, pre.x, pre.y, pre.z, m, (float)sx0, (float)sy0) << (4 * st);
    }
    return bits;
}

// The quad masks of a single-frame list, in place: the scatter leaves each entry's tile in its qmask
// word, and this flat pass replaces it with quad_mask.  The box tests run on (entry, strip) pairs
// compacted across the wave (an entry keeps ~1.2 of its 4 strips): each wave stages its 64 entries'
// conic, mean and strip origins in LDS, lists the pairs, and evaluates quad_reach4 on 64 pairs at a
// time -- one pass per kept strip instead of the wave running every strip any lane keeps.  (The
// scatter itself runs one workgroup per 256 Gaussians at one frame, latency-bound; computing the
// masks there cost it 2.4x.)
// (Measured: adding k_strip_count's per-tile strip counts here, one atomic per (tile run, strip) of
// each wave's 64 entries, took the pass from 16 to 36 us per C2 frame -- the waves of a long tile
// all add to the same four words -- against 9 us for the separate count launch.)
__global__ __launch_bounds__(256) void k_quad_masks(Dims d, GeomArena g, ImageArena im, BinArena bn) {
    __shared__ float4 s_co[4][64], s_pre[4][64];
    __shared__ float2 s_m[4][64];
    __shared__ int2 s_org[4][64];         // tile (tx, ty) of the entry
    __shared__ uint32_t s_pair[4][256];   // (lane | strip << 8) per pair
    __shared__ uint32_t s_bits[4][64];
    if (g.ctrl[kCtrlOverflow]) return;
    const uint32_t R = g.ctrl[kCtrlRLo];  // (one frame: the list length)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t p0 = (blockIdx.x * 4u + (uint32_t)wv) * 64u; p0 < R; p0 += gridDim.x * 256u) {
        const uint32_t p = p0 + (uint32_t)lane;
        const uint32_t e = p < R ? bn.point_list[p] : 0u;
        const uint32_t t = p < R ? bn.qmask[p] : 0u;
        const uint32_t sm = e >> 28;
        if (sm) {
            const int64_t gi = (int64_t)(e & kIndexMask);
            const float4 r0 = g.rrec[2 * gi], r1 = g.rrec[2 * gi + 1];
            // the scatter's conic / opacity / mean of the render record (exact rescaling)
            const float4 co = make_float4(-2.0f * r1.x, -r1.y, -2.0f * r1.z, r0.z);
            s_co[wv][lane] = co;
            s_pre[wv][lane] = strip_pre(co);
            s_m[wv][lane] = make_float2(r0.x, r0.y);
            s_org[wv][lane] = make_int2((int)(t % (uint32_t)d.gx), (int)(t / (uint32_t)d.gx));
        }
        s_bits[wv][lane] = 0u;
        // the wave's (entry, strip) pairs
        uint32_t np = 0;
#pragma unroll
        for (int st = 0; st < kStrips; st++) {
            const bool has = (sm >> st) & 1u;
            const uint64_t bm = __ballot(has);
            if (has) {
                const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                s_pair[wv][np + rk] = (uint32_t)lane | ((uint32_t)st << 8);
            }
            np += (uint32_t)__popcll(bm);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t k0 = 0; k0 < np; k0 += 64u) {
            if (k0 + (uint32_t)lane < np) {
                const uint32_t pr = s_pair[wv][k0 + lane];
                const int l = (int)(pr & 0xFFu), st = (int)(pr >> 8);
                const float4 co = s_co[wv][l], pre = s_pre[wv][l];
                uint32_t qb;
                if (__builtin_bit_cast(uint32_t, pre.w) == 2u) {
                    qb = 0xFu;
                } else {
                    const int2 og = s_org[wv][l];
                    int sx0, sy0;
                    strip_origin(og.x, og.y, st, sx0, sy0);
                    qb = quad_reach4(co.x, co.y, co.z, pre.x, pre.y, pre.z, s_m[wv][l], (float)sx0, (float)sy0);
                }
                atomicOr(&s_bits[wv][l], qb << (4 * st));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (p < R) bn.qmask[p] = s_bits[wv][lane];
        __builtin_amdgcn_wave_barrier();
    }
}

void launch_quad_masks(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                       hipStream_t s) {
    // 2048 workgroups: 8 per CU, every wave resident with about one 64-entry chunk (the pass is
    // load-latency-bound; 1024 workgroups: 19.6 us per C2 frame, 2048: 17.4, 4096: 17.1; GSR_QMASK_WG A/B)
    static const int wg = tune_env("GSR_QMASK_WG", 2048);
    if (b.qmask && d.B == 1 && d.P > 0) hipLaunchKernelGGL(k_quad_masks, dim3(wg), dim3(256), 0, s, d, g, im, b);
}

// ---------------------------------------------------------------- 5. ordered scatter
// One workgroup per chunk of d.chunk depth-ordered Gaussians (one count-table row), in d.chunk/kSlots
// passes of kSlots Gaussians (one per thread, "slot").  A pass spreads its instances evenly over the
// threads (binary search in the slots' inclusive tile-count scan), so one huge splat does not
// serialise a wave.  An instance (slot o, tile t) lands at
//     base[t] + #(slots o' < o of this pass whose rect covers t)
// with base[t] = ranges[t].x + table[chunk][t] + the pass's earlier slots covering t; the second
// term is a popcount of per-wave ballots of "rect covers tile column tx" and "... row ty" (4 x
// 64-bit masks per column and per row, in LDS), and base[] advances by the pass's per-tile totals.
// The (chunk x tile) table and the per-workgroup base[] load shrink with the chunk, not the pass.
// WS (default; GSR_SCATTER_WAVESEARCH=0 for the per-lane search): each wave expands a contiguous run
// of the pass's instances, 64 at a time; the owner of instance q0 + i is o0 + (slot boundaries in
// (q0, q0 + i]) with o0 the owner of q0 (the previous step's last lane): every lane reads the end of
// slot o0 + lane, marks it in a per-wave 64-entry LDS row when it falls in the window, and one
// ballot of the row gives every lane its count -- in place of an 8-step binary search per instance.
// TS (one frame): k_tile_scan_place1 folded in -- workgroup 0 writes the ranges and the render work
// list (tile_scan_place_wg), and every workgroup takes its list positions from its own exclusive scan
// of the tile counts (the same sums) instead of reading the ranges: one launch fewer per frame.
template <int ABL, bool WS, bool TS = false>  // timing ablations (GSR_SCATTER_ABLATE): 1 = no strip test, 2 = no list store
__global__ __launch_bounds__(kSlots) __attribute__((amdgpu_waves_per_eu(6))) void k_ordered_scatter(Dims d, GeomArena g, ImageArena im, BinArena bn, int xcd_order) {
    uint32_t sink = 0;
    __shared__ uint32_t s_mark[kSlots];  // WS: one 64-entry row per wave
    uint32_t tag = 0;
    extern __shared__ uint64_t masks[];  // colm[gx][4], rowm[gy][4], then uint32 tile bases[T]
    __shared__ uint32_t s_pref[kSlots];
    __shared__ uint32_t s_sh[kSlots / 64 + 1];
    __shared__ uint2 s_rect[kSlots];
    __shared__ uint32_t s_gi[kSlots];
    __shared__ float4 s_co[kSlots];
    __shared__ float4 s_pre[kSlots];
    __shared__ float2 s_m[kSlots];
    if (TS && blockIdx.x == 0) {
        tile_scan_place_wg<kSlots>(d, g, im);
        __syncthreads();
    }
    if (g.ctrl[kCtrlOverflow]) return;
    // XCD-aware order (GSR_SCATTER_XCD, default on): workgroup L runs on XCD L % 8, and XCD x takes
    // the x-th eighth of the (frame, chunk) items in chunk order, so consecutive chunks -- which
    // write adjacent entries of every tile list -- meet in one L2 and leave it as whole lines
    // instead of partial ones from eight L2s.  Off: blockIdx order (chunk-major per frame).
    int b, c;
    if (xcd_order) {
        const uint32_t L = blockIdx.x, N = (uint32_t)d.nchunk * (uint32_t)d.B;
        const uint32_t M = (N + 7u) / 8u;
        const uint32_t item = (L & 7u) * M + (L >> 3);
        if (item >= N) return;
        b = (int)(item / (uint32_t)d.nchunk);
        c = (int)(item - (uint32_t)b * (uint32_t)d.nchunk);
    } else {
        b = blockIdx.y;
        c = blockIdx.x;
    }
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t V = g.fstat[kFsWords * b + kFsVisible];
    if ((uint32_t)c * d.chunk >= V) return;
    uint64_t* colm = masks;
    uint64_t* rowm = masks + 4 * d.gx;
    uint32_t* base = (uint32_t*)(masks + 4 * (d.gx + d.gy));
    // list position of this chunk's first instance in every tile of the frame
    const uint32_t* tbl = g.table + ((int64_t)b * d.nchunk + c) * d.T;
    if constexpr (TS) {  // (one frame) the tile's list start from this workgroup's own scan of the counts
        const int per = (d.T + kSlots - 1) / kSlots;
        const int beg = tid * per, end = min(d.T, beg + per);
        uint32_t sum = 0;
        for (int t = beg; t < end; t++) sum += im.tile_count[t];
        uint32_t total;
        uint32_t ex = block_excl_scan<uint32_t, kSlots>(sum, &total, s_sh) + g.fstat[kFsRBase];
        for (int t = beg; t < end; t++) {
            base[t] = ex + tbl[t];
            ex += im.tile_count[t];
        }
    } else {
        const uint2* rg = im.ranges + (int64_t)b * d.T;
        for (int t = tid; t < d.T; t += kSlots) base[t] = rg[t].x + tbl[t];
    }
    for (int pass = 0; pass < d.chunk / kSlots; pass++) {
        const uint32_t j0 = (uint32_t)c * d.chunk + (uint32_t)pass * kSlots;
        if (j0 >= V) break;  // uniform
        const uint32_t j = j0 + tid;
        uint32_t gi = 0, nt = 0;
        uint2 r = make_uint2(0u, 0u);
        if (j < V) {
            gi = g.order[(int64_t)b * d.P + j];
            const int64_t gid = (int64_t)b * d.P + gi;
            r = g.rect[gid];
            nt = ((r.y & 0xFFFF) - (r.x & 0xFFFF)) * ((r.y >> 16) - (r.x >> 16));
            // conic, opacity and mean from the render record (exact: its conic words are the conic
            // times -1/2 and -1, powers of two), so a GSR_FORWARD_ONLY preprocess need not write them
            const float4 r0 = g.rrec[2 * gid], r1 = g.rrec[2 * gid + 1];
            const float4 co = make_float4(-2.0f * r1.x, -r1.y, -2.0f * r1.z, r0.z);
            s_co[tid] = co;
            s_pre[tid] = strip_pre(co);
            s_m[tid] = make_float2(r0.x, r0.y);
        }
        uint32_t total;
        s_pref[tid] = block_excl_scan<uint32_t, kSlots>(nt, &total, s_sh) + nt;  // (barriers inside)
        s_rect[tid] = r;
        s_gi[tid] = gi;
        const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
        // this wave's column / row words: bit l of colm[4 x + wv] = lane l's rect covers column x.
        // Zero them, then every lane ORs its bit into the few columns and rows its rect spans
        // (ds_or_b64; a wave's LDS operations complete in order) instead of one ballot per column.
        for (int x = lane; x < d.gx; x += 64) colm[4 * x + wv] = 0ull;
        for (int y = lane; y < d.gy; y += 64) rowm[4 * y + wv] = 0ull;
        if (nt) {
            const unsigned long long bit = 1ull << lane;
            for (int x = x0; x < x1; x++) atomicOr((unsigned long long*)&colm[4 * x + wv], bit);
            for (int y = y0; y < y1; y++) atomicOr((unsigned long long*)&rowm[4 * y + wv], bit);
        }
        if (WS && pass == 0) s_mark[tid] = 0u;  // (tags start at 1; the barrier below orders it)
        __syncthreads();
        const uint32_t per = WS ? (total + kSlots - 1) / kSlots * 64u : 0u;  // instances per wave
        const uint32_t qa = WS ? min(total, (uint32_t)wv * per) : (uint32_t)tid;
        const uint32_t qb = WS ? min(total, qa + per) : total;
        int o0 = 0;
        if (WS && qa < qb) {  // owner of the wave's first instance (wave-uniform)
            int lo = 0, hi = kSlots - 1;
#pragma unroll
            for (int step = 0; step < 8; step++) {
                const int mid = (lo + hi) >> 1;
                if (s_pref[mid] > qa) hi = mid; else lo = mid + 1;
            }
            o0 = lo;
        }
        for (uint32_t q0 = qa; q0 < qb; q0 += WS ? 64u : (uint32_t)kSlots) {
            const uint32_t q = WS ? q0 + (uint32_t)lane : q0;
            int o;
            if (WS) {
                uint32_t* mrow = s_mark + 64 * wv;
                ++tag;
                const int os = o0 + lane;
                const uint32_t e = os < kSlots ? s_pref[os] : 0xFFFFFFFFu;  // end of slot os (> q0)
                if (e - q0 < 64u) mrow[e - q0] = tag;  // slot os + 1 starts inside the window
                const uint64_t M = __ballot(mrow[lane] == tag);  // (a wave's LDS ops complete in order)
                const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                o = o0 + __popcll(M & upto);
                o0 = __shfl(o, 63);
                if (q >= qb) continue;
            } else {
                int lo = 0, hi = kSlots - 1;  // first slot whose inclusive count exceeds q
#pragma unroll
                for (int step = 0; step < 8; step++) {
                    const int mid = (lo + hi) >> 1;
                    if (s_pref[mid] > q) hi = mid; else lo = mid + 1;
                }
                o = lo;
            }
            const uint32_t k = q - (o ? s_pref[o - 1] : 0u);
            const uint2 ro = s_rect[o];
            const int ox0 = ro.x & 0xFFFF, oy0 = ro.x >> 16, ow = (ro.y & 0xFFFF) - ox0;
            // k / ow in float: exact, the quotient's fraction is >= 0.5/ow from an integer
            const int dy = (int)(((float)k + 0.5f) * __builtin_amdgcn_rcpf((float)ow));
            const int ty = oy0 + dy, tx = ox0 + (int)k - dy * ow;
            const int t = ty * d.gx + tx;
            const int w_o = o >> 6, l_o = o & 63;
            uint32_t lr = 0;
            for (int w = 0; w < w_o; w++) lr += (uint32_t)__popcll(colm[4 * tx + w] & rowm[4 * ty + w]);
            const uint64_t below = l_o ? (~0ull >> (64 - l_o)) : 0ull;
            lr += (uint32_t)__popcll(colm[4 * tx + w_o] & rowm[4 * ty + w_o] & below);
            const uint32_t sm = (ABL & 1) ? 0xFu : strip_mask(s_co[o], s_pre[o], s_m[o], tx, ty);
            if (ABL & 2) sink += base[t] + lr + sm;
            else bn.point_list[base[t] + lr] = s_gi[o] | (sm << 28);
            if (bn.qmask) bn.qmask[base[t] + lr] = (uint32_t)t;  // (k_quad_masks turns it into the mask)
        }
        if ((pass + 1) * kSlots < d.chunk && j0 + kSlots < V) {  // uniform: advance base[] past this pass
            __syncthreads();
            for (int t = tid; t < d.T; t += kSlots) {
                const int tx = t % d.gx, ty = t / d.gx;
                uint32_t n = 0;
#pragma unroll
                for (int w = 0; w < kSlots / 64; w++) n += (uint32_t)__popcll(colm[4 * tx + w] & rowm[4 * ty + w]);
                base[t] += n;
            }
            __syncthreads();
        }
    }
    if ((ABL & 2) && sink == 0xDEADBEEFu) bn.point_list[0] = sink;
}

void launch_ordered_scatter(const Dims& d, const GeomArena& g, const ImageArena& im,
                            const BinArena& b, hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    const size_t lds = (size_t)(d.gx + d.gy) * 4 * 8 + (size_t)d.T * 4;
    static size_t attr = 0;
    if (lds > 65536 && attr < lds) {
        attr = lds;
        for (const void* f : {(const void*)k_ordered_scatter<0, true>, (const void*)k_ordered_scatter<0, true, true>,
#ifdef GSR_TUNING
                              (const void*)k_ordered_scatter<1, true>, (const void*)k_ordered_scatter<2, true>,
                              (const void*)k_ordered_scatter<3, true>,
#endif
                              (const void*)k_ordered_scatter<0, false>})
            hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    static const int abl = tune_env("GSR_SCATTER_ABLATE", 0);  // timing ablations: GSR_TUNING builds only
    static const int xo = tune_env("GSR_SCATTER_XCD", 1) != 0 ? 1 : 0;
    static const bool ws = tune_env("GSR_SCATTER_WAVESEARCH", 1) != 0;
    const uint32_t N = (uint32_t)d.nchunk * (uint32_t)d.B;
    const dim3 gr = xo ? dim3(8u * ((N + 7u) / 8u)) : dim3(d.nchunk, d.B), bl(kSlots);
#ifdef GSR_TUNING
    if (abl == 1) hipLaunchKernelGGL((k_ordered_scatter<1, true>), gr, bl, lds, s, d, g, im, b, xo);
    else if (abl == 2) hipLaunchKernelGGL((k_ordered_scatter<2, true>), gr, bl, lds, s, d, g, im, b, xo);
    else if (abl == 3) hipLaunchKernelGGL((k_ordered_scatter<3, true>), gr, bl, lds, s, d, g, im, b, xo);
    else
#else
    (void)abl;
#endif
    if (!ws) hipLaunchKernelGGL((k_ordered_scatter<0, false>), gr, bl, lds, s, d, g, im, b, xo);
    else if (tile_scan_in_scatter(d)) hipLaunchKernelGGL((k_ordered_scatter<0, true, true>), gr, bl, lds, s, d, g, im, b, xo);
    else hipLaunchKernelGGL((k_ordered_scatter<0, true>), gr, bl, lds, s, d, g, im, b, xo);
}

// ---------------------------------------------------------------- 6. strip work list
// The render kernels' unit of work is one 64-pixel strip (8x8), and its cost is the number of list entries
// whose strip bit is set (before early termination).  The tile-level longest-first list above
// orders by list length in octaves, which lets strips of 10x the mean work start late and set the
// kernel's length; this orders the strips themselves, 4 buckets per octave of survivors.
__device__ __forceinline__ uint32_t strip_bucket(uint32_t c) {
    if (!c) return kStripBuckets - 1;
    const uint32_t e = 31u - __clz(c);
    const uint32_t sub = e >= 2u ? (c >> (e - 2u)) & 3u : (c << (2u - e)) & 3u;
    return 127u - (e * 4u + sub);
}

// One wave per tile: popcount of each strip bit over the tile's list.
__global__ __launch_bounds__(256) void k_strip_count(Dims d, ImageArena im, BinArena bn) {
    const int tile_g = (int)((blockIdx.x * 256u + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (tile_g >= d.B * d.T) return;
    const uint2 r = im.ranges[tile_g];
    uint32_t c[kStrips] = {};
    // the 16-byte-aligned body as uint4 loads (8 per lane in flight: the longest lists, several
    // thousand entries, bound this kernel by their load round trips), the unaligned ends by lanes
    const uint32_t a4 = min((r.x + 3u) & ~3u, r.y), b4 = max(r.y & ~3u, a4);
    if (r.x + (uint32_t)lane < a4) { const uint32_t e = bn.point_list[r.x + lane];
#pragma unroll
        for (int s = 0; s < kStrips; s++) c[s] += (e >> (28 + s)) & 1u; }
    if (b4 + (uint32_t)lane < r.y) { const uint32_t e = bn.point_list[b4 + lane];
#pragma unroll
        for (int s = 0; s < kStrips; s++) c[s] += (e >> (28 + s)) & 1u; }
    const uint4* __restrict__ q = reinterpret_cast<const uint4*>(bn.point_list + a4);
    const uint32_t n4 = (b4 - a4) >> 2;
    for (uint32_t i = lane; i < n4; i += 512) {
        uint4 e[8];
#pragma unroll
        for (int u = 0; u < 8; u++) e[u] = i + 64u * u < n4 ? q[i + 64u * u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 8; u++)
#pragma unroll
            for (int s = 0; s < kStrips; s++)
                c[s] += ((e[u].x >> (28 + s)) & 1u) + ((e[u].y >> (28 + s)) & 1u) + ((e[u].z >> (28 + s)) & 1u) +
                        ((e[u].w >> (28 + s)) & 1u);
    }
#pragma unroll
    for (int s = 0; s < kStrips; s++) {
        uint32_t v = c[s];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        c[s] = v;
    }
    if (lane < kStrips) {
        uint32_t v = c[0];
#pragma unroll
        for (int s = 1; s < kStrips; s++) v = lane == s ? c[s] : v;
        im.strip_cnt[(int64_t)tile_g * kStrips + lane] = v;
    }
}

// Per frame: histogram of its non-empty tiles' strips over the buckets.
__device__ __forceinline__ uint32_t tile_strip_max(const ImageArena& im, int64_t tg) {
    uint32_t m = 0;
#pragma unroll
    for (int s = 0; s < kStrips; s++) m = max(m, im.strip_cnt[tg * kStrips + s]);
    return m;
}

// Per frame: histogram over the buckets of its non-empty tiles' strips (tile_major = 0) or of the
// tiles themselves keyed by their longest strip (tile_major = 1).
__global__ __launch_bounds__(1024) void k_strip_hist(Dims d, ImageArena im, int tile_major, int map) {
    __shared__ uint32_t h[8 * kStripBuckets];
    const int b = blockIdx.x;
    const int nh = map == 2 ? 8 * kStripBuckets : kStripBuckets;
    for (int i = threadIdx.x; i < nh; i += 1024) h[i] = 0;
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += 1024) {
        const int64_t tg = (int64_t)b * d.T + t;
        if (!im.tile_count[tg]) continue;
        if (map == 2) {  // (tile-major by construction)
            atomicAdd(&h[tile_queue(t, d.gx) * kStripBuckets + strip_bucket(tile_strip_max(im, tg))], 1u);
        } else if (tile_major) {
            atomicAdd(&h[strip_bucket(tile_strip_max(im, tg))], 1u);
        } else {
#pragma unroll
            for (int s = 0; s < kStrips; s++) atomicAdd(&h[strip_bucket(im.strip_cnt[tg * kStrips + s])], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nh; i += 1024) im.strip_hist[(int64_t)b * nh + i] = h[i];
}

// map 2: list offsets of every (frame, queue, bucket) run, in place of the histogram.  The list is
// queue-major (queue q's tiles form one segment), bucket-major inside a segment (most survivors
// first), frame-major inside a bucket; the segment bounds go to ctrl[kCtrlQStart..] for queue_item.
__global__ __launch_bounds__(1024) void k_strip_qscan(Dims d, ImageArena im, uint32_t* ctrl) {
    constexpr int kN = 8 * kStripBuckets;  // (queue, bucket) runs, queue-major
    __shared__ uint32_t tot[kN + 1];
    __shared__ uint32_t sh[1024 / 64 + 1];
    // (frames 8 at a time: eight independent loads in flight per thread instead of a chain of B)
    for (int i = threadIdx.x; i < kN; i += 1024) {
        uint32_t a = 0;
        int f = 0;
        for (; f + 8 <= d.B; f += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = im.strip_hist[(int64_t)(f + u) * kN + i];
#pragma unroll
            for (int u = 0; u < 8; u++) a += v[u];
        }
        for (; f < d.B; f++) a += im.strip_hist[(int64_t)f * kN + i];
        tot[i] = a;
    }
    if (threadIdx.x == 0) tot[kN] = 0;
    __syncthreads();
    // exclusive scan over the runs, two per thread (kN <= 2048)
    const int i0 = 2 * threadIdx.x;
    const uint32_t a0 = i0 < kN ? tot[i0] : 0u, a1 = i0 + 1 < kN ? tot[i0 + 1] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan<uint32_t, 1024>(a0 + a1, &total, sh);  // (barriers inside)
    if (i0 < kN) tot[i0] = ex;
    if (i0 + 1 < kN) tot[i0 + 1] = ex + a0;
    if (threadIdx.x == 0) tot[kN] = total;
    __syncthreads();
    for (int i = threadIdx.x; i < kN; i += 1024) {
        uint32_t run = tot[i];
        int f = 0;
        for (; f + 8 <= d.B; f += 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = im.strip_hist[(int64_t)(f + u) * kN + i];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                im.strip_hist[(int64_t)(f + u) * kN + i] = run;
                run += v[u];
            }
        }
        for (; f < d.B; f++) {
            uint32_t* h = im.strip_hist + (int64_t)f * kN + i;
            const uint32_t c = *h;
            *h = run;
            run += c;
        }
    }
    if (threadIdx.x < 8) {
        const int q = threadIdx.x;
        ctrl[kCtrlQStart + q] = tot[q * kStripBuckets];
        ctrl[kCtrlQStart + 8 + q] = tot[(q + 1) * kStripBuckets] - tot[q * kStripBuckets];
    }
}

// Per frame: place its strips into the batch-wide strip list, bucket-major (most survivors first);
// the order inside a bucket is whatever the LDS atomics give (scheduling only).  tile_major = 1
// places whole tiles (their 4 strips consecutive) by their longest strip, so the render's
// tile-affine queues (queue_item) keep a tile's strips -- which read the same Gaussians -- on one
// XCD and its L2.
__global__ __launch_bounds__(1024) void k_strip_place(Dims d, ImageArena im, int tile_major, int map) {
    extern __shared__ uint32_t hist[];  // [B][kStripBuckets]
    __shared__ uint32_t cur[8 * kStripBuckets];
    __shared__ uint32_t before[kStripBuckets];
    const int b = blockIdx.x;
    if (map == 2) {  // offsets from k_strip_qscan
        for (int i = threadIdx.x; i < 8 * kStripBuckets; i += 1024)
            cur[i] = im.strip_hist[(int64_t)b * 8 * kStripBuckets + i];
        __syncthreads();
        for (int t = threadIdx.x; t < d.T; t += 1024) {
            const int64_t tg = (int64_t)b * d.T + t;
            if (!im.tile_count[tg]) continue;
            const uint32_t pos =
                atomicAdd(&cur[tile_queue(t, d.gx) * kStripBuckets + strip_bucket(tile_strip_max(im, tg))], 1u);
#pragma unroll
            for (int s = 0; s < kStrips; s++) im.strip_list[kStrips * pos + s] = ((uint32_t)tg << 2) | (uint32_t)s;
        }
        return;
    }
    for (int i = threadIdx.x; i < d.B * kStripBuckets; i += 1024) hist[i] = im.strip_hist[i];
    __syncthreads();
    for (int bk = threadIdx.x; bk < kStripBuckets; bk += 1024) {  // bucket totals; this frame's share before it
        uint32_t tot = 0, mine = 0;
        for (int f = 0; f < d.B; f++) {
            const uint32_t v = hist[f * kStripBuckets + bk];
            tot += v;
            if (f < b) mine += v;
        }
        cur[bk] = tot;
        before[bk] = mine;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // start of this frame's run in each bucket (bucket-major)
        uint32_t acc = 0;
        for (int bk = 0; bk < kStripBuckets; bk++) {
            const uint32_t t = cur[bk];
            cur[bk] = acc + before[bk];
            acc += t;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += 1024) {
        const int64_t tg = (int64_t)b * d.T + t;
        if (!im.tile_count[tg]) continue;
        if (tile_major) {
            const uint32_t pos = atomicAdd(&cur[strip_bucket(tile_strip_max(im, tg))], 1u);
#pragma unroll
            for (int s = 0; s < kStrips; s++) im.strip_list[kStrips * pos + s] = ((uint32_t)tg << 2) | (uint32_t)s;
        } else {
#pragma unroll
            for (int s = 0; s < kStrips; s++) {
                const uint32_t bk = strip_bucket(im.strip_cnt[tg * kStrips + s]);
                im.strip_list[atomicAdd(&cur[bk], 1u)] = ((uint32_t)tg << 2) | (uint32_t)s;
            }
        }
    }
}

// One frame, maps 0 / 1: k_strip_hist and k_strip_place in one workgroup (one launch instead of two).
__global__ __launch_bounds__(1024) void k_strip_order1(Dims d, ImageArena im, int tile_major) {
    __shared__ uint32_t h[kStripBuckets];
    for (int i = threadIdx.x; i < kStripBuckets; i += 1024) h[i] = 0;
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += 1024) {
        if (!im.tile_count[t]) continue;
        if (tile_major) {
            atomicAdd(&h[strip_bucket(tile_strip_max(im, t))], 1u);
        } else {
#pragma unroll
            for (int sp = 0; sp < kStrips; sp++) atomicAdd(&h[strip_bucket(im.strip_cnt[(int64_t)t * kStrips + sp])], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kStripBuckets; i += 1024) im.strip_hist[i] = h[i];
    __syncthreads();
    if (threadIdx.x == 0) {  // bucket-major starts, most survivors first
        uint32_t acc = 0;
        for (int bk = 0; bk < kStripBuckets; bk++) {
            const uint32_t c = h[bk];
            h[bk] = acc;
            acc += c;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < d.T; t += 1024) {
        if (!im.tile_count[t]) continue;
        if (tile_major) {
            const uint32_t pos = atomicAdd(&h[strip_bucket(tile_strip_max(im, t))], 1u);
#pragma unroll
            for (int sp = 0; sp < kStrips; sp++) im.strip_list[kStrips * pos + sp] = ((uint32_t)t << 2) | (uint32_t)sp;
        } else {
#pragma unroll
            for (int sp = 0; sp < kStrips; sp++) {
                const uint32_t bk = strip_bucket(im.strip_cnt[(int64_t)t * kStrips + sp]);
                im.strip_list[atomicAdd(&h[bk], 1u)] = ((uint32_t)t << 2) | (uint32_t)sp;
            }
        }
    }
}

void launch_strip_list_tile(const Dims& d, const ImageArena& im, uint32_t* out, hipStream_t s) {
    if (d.B == 0 || d.T == 0) return;
    ImageArena i2 = im;
    i2.strip_list = out;
    hipLaunchKernelGGL(k_strip_hist, dim3(d.B), dim3(1024), 0, s, d, i2, 1, 1);
    const size_t lds = (size_t)d.B * kStripBuckets * 4;
    static size_t attr = 0;
    if (lds > 65536 && attr < lds) {
        attr = lds;
        hipFuncSetAttribute((const void*)k_strip_place, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    hipLaunchKernelGGL(k_strip_place, dim3(d.B), dim3(1024), lds, s, d, i2, 1, 1);
}

void launch_strip_order(const Dims& d, const GeomArena& g, const ImageArena& im, const BinArena& b,
                        hipStream_t s) {
    if (d.B == 0 || d.T == 0) return;
    const int nt = d.B * d.T;
    hipLaunchKernelGGL(k_strip_count, dim3((nt + 3) / 4), dim3(256), 0, s, d, im, b);
    launch_quad_masks(d, g, im, b, s);
    const int tile_major = strip_order_tile_major();
    // (one frame: the tile-affine walk of one longest-first list, measured 1.5% faster there)
    const int map = tile_major ? (d.B == 1 ? 1 : xcd_queue_map()) : 0;
    if (d.B == 1 && map != 2) {
        hipLaunchKernelGGL(k_strip_order1, dim3(1), dim3(1024), 0, s, d, im, tile_major);
        return;
    }
    hipLaunchKernelGGL(k_strip_hist, dim3(d.B), dim3(1024), 0, s, d, im, tile_major, map);
    if (map == 2) {
        // (frame-major segments -- one or two frames' records per XCD L2 at a time -- measured 7%
        // slower render_fwd than bucket-major: the batch-wide longest-first order sets the tail)
        hipLaunchKernelGGL(k_strip_qscan, dim3(1), dim3(1024), 0, s, d, im, g.ctrl);
        hipLaunchKernelGGL(k_strip_place, dim3(d.B), dim3(1024), 0, s, d, im, tile_major, map);
        return;
    }
    const size_t lds = (size_t)d.B * kStripBuckets * 4;
    static size_t attr = 0;
    if (lds > 65536 && attr < lds) {
        attr = lds;
        hipFuncSetAttribute((const void*)k_strip_place, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    hipLaunchKernelGGL(k_strip_place, dim3(d.B), dim3(1024), lds, s, d, im, tile_major, map);
}

}  // namespace gsr
