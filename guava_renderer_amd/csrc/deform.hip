// deform.hip -- per-frame avatar deformation on gfx950: linear-blend skinning (SMPL-X body /
// FLAME head) and GUAVA's Gaussian assembly, B frames per launch set (include/gsr_deform.h).
//
// Reference (restated, not translated):
//   lbs / lbs_wobeta                models/modules/flame/lbs.py:142-229 / :255-333
//   blend_shapes, vertices2joints   lbs.py:355-376, :335-352
//   batch_rodrigues                 lbs.py:379-410
//   batch_rigid_transform           lbs.py:426-482
//   Ubody_Gaussian.forward          models/UbodyAvatar/ubody_gaussian.py:252-278
//   compute_face_orientation        utils/graphics_utils.py:52-80
//   roma 1.5.3 rotmat_to_unitquat / quat_product (third-party, scipy-derived; call sites
//   ubody_gaussian.py:253-254,258,270)
//
// Kernels (all B frames per launch):
//   k_pack_rows      segs x B WGs     the coefficient rows of EHM.forward from their pieces
//   k_lbs_rodrigues  B*J threads      axis-angle -> R, pose feature R - I
//   k_lbs_blend      3V/64 x B/16 WGs (B = 1: one frame, 16 waves per WG) v_shaped = template + shapedirs.betas, v_posed = v_shaped +
//                                     posedirs.feature: the bases are streamed once per 16 frames
//                                     (HBM-bound: 4*(NB + 9(J-1)) bytes per vertex coordinate)
//   k_lbs_blend_mfma 3V/32 x B/32 WGs the same for B > 16 on the matrix cores (f32 MFMA), bases
//                                     streamed once per 32 frames
//   k_lbs_joints     J/4 x B WGs      J_regressor . v_shaped (+ joints_offset)
//   k_lbs_chain      B WGs            the kinematic chain in LDS, one tree level per step
//   k_lbs_skin       V x B            T_v = sum_j w_vj A_j, v = T_v [v_posed; 1]
//   k_deform_gaussians (V+N) x B/8    vertex + UV Gaussians straight into the rasterizer's inputs
//                                     (face frames once per face and frame, in LDS)
// Every sum runs in a fixed order (fmaf chains over k in index order, 3-term dots left to right),
// so results are deterministic run to run.
#include <climits>
#include <cstdlib>
#include <string>

#include "../../include/gsr.h"
#include "../../include/gsr_deform.h"
#include "deform_internal.h"
#include "gsr_internal.h"
#include "preprocess_dev.h"

namespace gsr {

#ifndef GSR_DEFORM_NOSTORE
#define GSR_DEFORM_NOSTORE 0  // timing ablation only: skip the UV rotation and the means/scales stores
#endif

constexpr int kLbsFrames = 16;  // frames per k_lbs_blend workgroup (accumulators per thread)
constexpr int kLbsSplit = 4;    // k_lbs_blend waves per workgroup, each an interleaved slice of k
// single-frame batches (the per-frame drop-in path): one accumulator per thread and 16 waves per
// workgroup, so the K-long stream of every coordinate has 16 slices of loads in flight
constexpr int kLbsSplit1 = 16;

struct Parents {
    int8_t p[GSR_LBS_MAX_JOINTS];
};

// batch_rodrigues (lbs.py:379-410): angle = |r + 1e-8|, dir = r / angle,
// R = I + sin K + (1 - cos) K.K with K the cross-product matrix of dir.
// batch_rodrigues (lbs.py:379-410) of pose entry t (axis-angle, or a rotation matrix when !pose2rot)
__device__ __forceinline__ void rodrigues_one(const float* __restrict__ pose, int t, int pose2rot, float (&R)[9]) {
    if (pose2rot) {
        const float rx = pose[3 * t], ry = pose[3 * t + 1], rz = pose[3 * t + 2];
        const float ex = rx + 1e-8f, ey = ry + 1e-8f, ez = rz + 1e-8f;
        const float angle = sqrtf(ex * ex + ey * ey + ez * ez);
        const float x = rx / angle, y = ry / angle, z = rz / angle;
        const float c = cosf(angle), s = sinf(angle);
        const float K[9] = {0.f, -z, y, z, 0.f, -x, -y, x, 0.f};
        const float omc = 1.0f - c;
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const float kk = K[3 * r] * K[q] + K[3 * r + 1] * K[3 + q] + K[3 * r + 2] * K[6 + q];
                R[3 * r + q] = ((r == q ? 1.0f : 0.0f) + s * K[3 * r + q]) + omc * kk;
            }
    } else {
#pragma unroll
        for (int e = 0; e < 9; e++) R[e] = pose[9 * t + e];
    }
}

__global__ void k_lbs_rodrigues(int B, int J, const float* __restrict__ pose, int pose2rot,
                                float* __restrict__ rot, float* __restrict__ feat) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * J) return;
    const int b = t / J, j = t - b * J;
    float R[9];
    rodrigues_one(pose, t, pose2rot, R);
#pragma unroll
    for (int e = 0; e < 9; e++) rot[9 * t + e] = R[e];
    if (j > 0) {  // pose_feature = (rot_mats[:, 1:] - I).view(B, -1)   (lbs.py:303)
        float* f = feat + (int64_t)b * (J - 1) * 9 + (j - 1) * 9;
#pragma unroll
        for (int e = 0; e < 9; e++) f[e] = R[e] - ((e % 4) == 0 ? 1.0f : 0.0f);
    }
}

// acc[f] += sum over this wave's k-slice (k = w mod kLbsSplit, ascending) of coef[k][f] * base[k][m],
// kLbsBatch loads of the k-major base issued before their FMAs (enough bytes in flight to stream
// from HBM with ~4 waves per SIMD).
constexpr int kLbsBatch = 16;
template <int NF, int SPLIT>
__device__ __forceinline__ void lbs_stream(const float* __restrict__ base, int M, int m, int K, int w,
                                           const float* coef, float (&acc)[NF]) {
    for (int k0 = w; k0 < K; k0 += SPLIT * kLbsBatch) {
        float v[kLbsBatch];
#pragma unroll
        for (int u = 0; u < kLbsBatch; u++) {
            const int k = k0 + u * SPLIT;
            v[u] = k < K ? base[(int64_t)k * M + m] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kLbsBatch; u++) {
            const int k = k0 + u * SPLIT;
            if (k >= K) break;
            if constexpr (NF % 4 == 0) {
                const float4* c = reinterpret_cast<const float4*>(&coef[k * NF]);
#pragma unroll
                for (int q = 0; q < NF / 4; q++) {
                    const float4 cq = c[q];
                    acc[4 * q] = fmaf(cq.x, v[u], acc[4 * q]); acc[4 * q + 1] = fmaf(cq.y, v[u], acc[4 * q + 1]);
                    acc[4 * q + 2] = fmaf(cq.z, v[u], acc[4 * q + 2]); acc[4 * q + 3] = fmaf(cq.w, v[u], acc[4 * q + 3]);
                }
            } else {
#pragma unroll
                for (int f = 0; f < NF; f++) acc[f] = fmaf(coef[k * NF + f], v[u], acc[f]);
            }
        }
    }
}

// v_shaped = v_template + blend_shapes(betas, shapedirs); v_posed = pose_offsets + v_shaped
// (lbs.py:186,201,210 / :305,314): a [3V x K] x [K x B] product streamed from HBM.  A workgroup
// owns 64 vertex coordinates (lane = coordinate) of kLbsFrames frames; its kLbsSplit waves take
// interleaved slices of k (k = w mod kLbsSplit), so each coordinate's K-long stream has 4 waves of
// loads in flight instead of one serial chain, and the slice sums are added in slice order through
// LDS (deterministic).  The frame coefficients sit in LDS (broadcast reads); the k-major bases are
// read coalesced, once per frame group.
inline dim3 lbs_blend_grid(int M, int B, int nf) {
    const int nx8 = ((M + 63) / 64 + 7) / 8 * 8;
    return dim3(nx8 * ((B + nf - 1) / nf));
}

template <int NF, int SPLIT>
__global__ __launch_bounds__(64 * SPLIT) void k_lbs_blend(int B, int M, int NB, int NP,
                                                              const float* __restrict__ vt, int64_t vt_stride,
                                                              const float* __restrict__ betas,
                                                              const float* __restrict__ sd_t,
                                                              const float* __restrict__ feat,
                                                              const float* __restrict__ pd,
                                                              float* __restrict__ v_shaped,
                                                              float* __restrict__ v_posed) {
    extern __shared__ float4 lds4[];  // coef [(NB + NP)][NF], then the slice reduction
    float* coef = reinterpret_cast<float*>(lds4);
    // XCD-aware order (1-D grid, lbs_blend_grid): the frame groups of one coordinate block are
    // dealt to the same XCD back to back, so all but the first read the basis slice from its L2
    const int ng = (B + NF - 1) / NF;
    const int jx = (int)(blockIdx.x >> 3);
    const int by = jx % ng;
    const int bx = (jx / ng) * 8 + (int)(blockIdx.x & 7);
    if (bx * 64 >= M) return;  // padding block (the whole workgroup, before any barrier)
    const int b0 = by * NF;
    const int nk = NB + NP;
    for (int idx = threadIdx.x; idx < nk * NF; idx += blockDim.x) {
        const int k = idx / NF, f = idx - k * NF;
        const int b = b0 + f;
        float v = 0.f;
        if (b < B) v = k < NB ? betas[(int64_t)b * NB + k] : feat[(int64_t)b * NP + (k - NB)];
        coef[idx] = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int m = bx * 64 + lane;
    const bool ok = m < M;
    const int nf = min(NF, B - b0);
    float as[NF], ap[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) { as[f] = 0.f; ap[f] = 0.f; }
    if (ok) {
        lbs_stream<NF, SPLIT>(sd_t, M, m, NB, w, coef, as);
        lbs_stream<NF, SPLIT>(pd, M, m, NP, w, coef + NB * NF, ap);
    }
    // slice reduction through LDS: red[w][f][lane]
    float* red = coef;
    __syncthreads();  // coefficients no longer needed
#pragma unroll
    for (int f = 0; f < NF; f++) red[(w * NF + f) * 64 + lane] = as[f];
    __syncthreads();
    float vs[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) vs[f] = 0.f;
    if (w == 0) {
#pragma unroll
        for (int f = 0; f < NF; f++) {
            float acc = red[f * 64 + lane];
            for (int u = 1; u < SPLIT; u++) acc += red[(u * NF + f) * 64 + lane];
            const int b = b0 + f;
            if (ok && f < nf) {
                const float tv = vt[(int64_t)b * vt_stride + m];
                vs[f] = NB > 0 ? tv + acc : tv;
                v_shaped[(int64_t)b * M + m] = vs[f];
            }
        }
    }
    if (!v_posed) return;  // blend_shapes + joints only (gsr_blend_joints); uniform
    __syncthreads();
#pragma unroll
    for (int f = 0; f < NF; f++) red[(w * NF + f) * 64 + lane] = ap[f];
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int f = 0; f < NF; f++) {
            float acc = red[f * 64 + lane];
            for (int u = 1; u < SPLIT; u++) acc += red[(u * NF + f) * 64 + lane];
            if (ok && f < nf) v_posed[(int64_t)(b0 + f) * M + m] = acc + vs[f];
        }
    }
}

// The same products for batches of more than kLbsFrames frames, on the matrix cores, with the
// bases read ONCE per 32 frames: D[b][m] = sum_k coef[b][k] base[k][m] is a (32 frames x 32
// coordinates) tile per workgroup, v_mfma_f32_32x32x2_f32 (exact f32 products) with A = the
// frames' coefficients (row b, k) and B = the k-major bases (column m, coalesced 128-byte
// half-wave loads).  The 4 waves take interleaved k-steps and their partial tiles are added in
// wave order through LDS (deterministic); each wave then finishes 4 of the 16 output registers:
// v_shaped = template + shape sum, v_posed = v_shaped + pose sum (the VALU kernel's association).
// (Measured variants: 8 waves x 16 loads in flight, and the coefficient block staged transposed
// in LDS, were both slower at B = 32.)
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int kBlendUnroll = 8;  // k-steps whose loads are issued before their MFMAs

__device__ __forceinline__ void blend_mfma_part(floatx16& acc, const float* __restrict__ coef, int ncoef,
                                                const float* __restrict__ base, int M, int K, int bA, bool bok,
                                                int m, bool mok, int w, int hi) {
    const int nsteps = (K + 1) / 2;
    for (int s0 = w; s0 < nsteps; s0 += 4 * kBlendUnroll) {
        float a[kBlendUnroll], bb[kBlendUnroll];
#pragma unroll
        for (int u = 0; u < kBlendUnroll; u++) {
            const int k = 2 * (s0 + 4 * u) + hi;
            const bool kok = s0 + 4 * u < nsteps && k < K;
            a[u] = (bok && kok) ? coef[(int64_t)bA * ncoef + k] : 0.f;
            bb[u] = (mok && kok) ? base[(int64_t)k * M + m] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kBlendUnroll; u++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], bb[u], acc, 0, 0, 0);
    }
}

__global__ __launch_bounds__(256) void k_lbs_blend_mfma(int B, int M, int NB, int NP,
                                                        const float* __restrict__ vt, int64_t vt_stride,
                                                        const float* __restrict__ betas,
                                                        const float* __restrict__ sd_t,
                                                        const float* __restrict__ feat,
                                                        const float* __restrict__ pd,
                                                        float* __restrict__ v_shaped,
                                                        float* __restrict__ v_posed) {
    __shared__ float red[4][2][16][64];  // per-wave partial tiles: [wave][shape/pose][register][lane]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hi = lane >> 5, l32 = lane & 31;
    const int m0 = blockIdx.x * 32, b0 = blockIdx.y * 32;
    const int m = m0 + l32, bA = b0 + l32;
    const bool mok = m < M, bok = bA < B;
    floatx16 as, ap;
#pragma unroll
    for (int r = 0; r < 16; r++) { as[r] = 0.f; ap[r] = 0.f; }
    if (NB > 0) blend_mfma_part(as, betas, NB, sd_t, M, NB, bA, bok, m, mok, w, hi);
    if (NP > 0 && v_posed) blend_mfma_part(ap, feat, NP, pd, M, NP, bA, bok, m, mok, w, hi);
#pragma unroll
    for (int r = 0; r < 16; r++) {
        red[w][0][r][lane] = as[r];
        red[w][1][r][lane] = ap[r];
    }
    __syncthreads();
    // wave w finishes registers 4w..4w+3: row (frame) (r&3) + 8(r>>2) + 4(lane>>5), column m
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int r = 4 * w + i;
        const int b = b0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (!mok || b >= B) continue;
        float S = red[0][0][r][lane], Pz = red[0][1][r][lane];
#pragma unroll
        for (int u = 1; u < 4; u++) { S += red[u][0][r][lane]; Pz += red[u][1][r][lane]; }
        const float tv = vt[(int64_t)b * vt_stride + m];
        const float vs = NB > 0 ? tv + S : tv;
        v_shaped[(int64_t)b * M + m] = vs;
        if (v_posed) v_posed[(int64_t)b * M + m] = Pz + vs;
    }
}

// ---- tiled bases (GsrLbsSparse.shapedirs_tiled / posedirs_tiled, include/gsr_deform.h)
// A base [K][M] re-laid once per avatar as 1-KB tiles of 32 coordinates x 8 k: tile (t, g) holds, as
// float4 (t * nkg + g) * 64 + 32 h + c, component j, the value base[8g + 4h + j][32t + c] (K padded to
// a multiple of 8, M to 32, with zeros).  Every load is then one fully coalesced 16-byte-per-lane
// wave read (1 KB), where the k-major layout gives 4-byte lanes (256 B per load instruction): the
// blend's bases stream at HBM rate with a quarter of the load instructions in flight.
constexpr int kTiledUnroll = 4;  // tile groups whose loads are issued before their products
#ifndef GSR_BLEND_COEF_VEC
#define GSR_BLEND_COEF_VEC 1
#endif

// D[frame][m] over the k of one base: v_mfma_f32_32x32x2_f32 with lane (c, h) holding base[8g + 4h + j]
// [32t + c] (B operand) and coef[frame b0 + c][8g + 4h + j] (A operand) for the j-th MFMA of a group
// (the lane halves' k of one MFMA are 8g + j and 8g + 4 + j); wave w takes the groups g = w mod 4.
// The coefficient gathers (lane = frame row, 4 consecutive k) are 16- or 8-byte loads when the rows'
// stride and base allow (vw = 4 / 2, wave-uniform): 16 scattered dword loads per step were the
// texture path's load (TA 48% / TD 58% busy at 37% of HBM), four times the base tile's loads.
__device__ __forceinline__ int coef_vec_width(const float* coef, int ncoef) {
    if (((uintptr_t)coef & 15) == 0 && (ncoef & 3) == 0) return 4;
    if (((uintptr_t)coef & 7) == 0 && (ncoef & 1) == 0) return 2;
    return 1;
}

__device__ __forceinline__ void blend_tiled_mfma_part(floatx16& acc, const float* __restrict__ coef, int ncoef,
                                                      const float4* __restrict__ tb, int K, int t, int bA,
                                                      bool bok, int w, int hi, int lane, int nw = 4) {
    const int nkg = (K + 7) / 8;
    const int nfull = GSR_BLEND_COEF_VEC ? K / 8 : 0;  // groups whose 8 k are all < K
    const int vw = coef_vec_width(coef, ncoef);
    const float4* __restrict__ p = tb + (int64_t)t * nkg * 64 + lane;
    const float* __restrict__ cr = coef + (int64_t)bA * ncoef;
    for (int g0 = w; g0 < nkg; g0 += nw * kTiledUnroll) {
        float4 v[kTiledUnroll];
        float a[kTiledUnroll][4];
#pragma unroll
        for (int u = 0; u < kTiledUnroll; u++) {
            const int g = g0 + nw * u;
            v[u] = g < nkg ? p[(int64_t)g * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
            const int k0 = 8 * g + 4 * hi;
            if (g < nfull && vw == 4) {
                const float4 c = bok ? *reinterpret_cast<const float4*>(cr + k0) : make_float4(0.f, 0.f, 0.f, 0.f);
                a[u][0] = c.x; a[u][1] = c.y; a[u][2] = c.z; a[u][3] = c.w;
            } else if (g < nfull && vw == 2) {
                const float2 c0 = bok ? *reinterpret_cast<const float2*>(cr + k0) : make_float2(0.f, 0.f);
                const float2 c1 = bok ? *reinterpret_cast<const float2*>(cr + k0 + 2) : make_float2(0.f, 0.f);
                a[u][0] = c0.x; a[u][1] = c0.y; a[u][2] = c1.x; a[u][3] = c1.y;
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int k = k0 + j;
                    a[u][j] = (bok && k < K) ? cr[k] : 0.f;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kTiledUnroll; u++) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][0], v[u].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][1], v[u].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][2], v[u].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][3], v[u].w, acc, 0, 0, 0);
        }
    }
}

// k_lbs_blend_mfma over the tiled bases: one workgroup per 32 coordinates x 32 frames, the same
// wave-order reduction and epilogue.  NW waves split the k groups (g = w mod NW): 8 when the grid
// has at most 512 workgroups (the FLAME head, 471: 4 waves per workgroup left the SIMDs under two
// waves each, every wave a long serial load -> MFMA chain), else 4.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_lbs_blend_tiled(int B, int M, int NB, int NP,
                                                         const float* __restrict__ vt, int64_t vt_stride,
                                                         const float* __restrict__ betas,
                                                         const float4* __restrict__ sd_tiled,
                                                         const float* __restrict__ feat,
                                                         const float4* __restrict__ pd_tiled,
                                                         float* __restrict__ v_shaped,
                                                         float* __restrict__ v_posed) {
    __shared__ float red[NW][2][16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hi = lane >> 5, l32 = lane & 31;
    const int t = blockIdx.x, m0 = t * 32, b0 = blockIdx.y * 32;
    const int m = m0 + l32, bA = b0 + l32;
    const bool mok = m < M, bok = bA < B;
    floatx16 as, ap;
#pragma unroll
    for (int r = 0; r < 16; r++) { as[r] = 0.f; ap[r] = 0.f; }
    if (NB > 0) blend_tiled_mfma_part(as, betas, NB, sd_tiled, NB, t, bA, bok, w, hi, lane, NW);
    if (NP > 0 && v_posed) blend_tiled_mfma_part(ap, feat, NP, pd_tiled, NP, t, bA, bok, w, hi, lane, NW);
#pragma unroll
    for (int r = 0; r < 16; r++) {
        red[w][0][r][lane] = as[r];
        red[w][1][r][lane] = ap[r];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16 / NW; i++) {
        const int r = (16 / NW) * w + i;
        const int b = b0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (!mok || b >= B) continue;
        float S = red[0][0][r][lane], Pz = red[0][1][r][lane];
#pragma unroll
        for (int u = 1; u < NW; u++) { S += red[u][0][r][lane]; Pz += red[u][1][r][lane]; }
        const float tv = vt[(int64_t)b * vt_stride + m];
        const float vs = NB > 0 ? tv + S : tv;
        v_shaped[(int64_t)b * M + m] = vs;
        if (v_posed) v_posed[(int64_t)b * M + m] = Pz + vs;
    }
}

// One frame over the tiled bases (the per-frame drop-in path): lane (c, h) of wave w sums
// coef[8g + 4h + j] base[8g + 4h + j][32t + c] over its groups g = w mod 4 (four fmaf per 16-byte
// load), then the two lane halves and the four waves are added in a fixed order through LDS.
__device__ __forceinline__ float blend_tiled_one(const float* __restrict__ coef, const float4* __restrict__ tb,
                                                 int K, int t, int w, int hi, int lane) {
    const int nkg = (K + 7) / 8;
    const float4* __restrict__ p = tb + (int64_t)t * nkg * 64 + lane;
    float acc = 0.f;
    for (int g0 = w; g0 < nkg; g0 += 4 * kTiledUnroll) {
        float4 v[kTiledUnroll];
        float a[kTiledUnroll][4];
#pragma unroll
        for (int u = 0; u < kTiledUnroll; u++) {
            const int g = g0 + 4 * u;
            v[u] = g < nkg ? p[(int64_t)g * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int k = 8 * g + 4 * hi + j;
                a[u][j] = k < K ? coef[k] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < kTiledUnroll; u++) {
            acc = fmaf(a[u][0], v[u].x, acc);
            acc = fmaf(a[u][1], v[u].y, acc);
            acc = fmaf(a[u][2], v[u].z, acc);
            acc = fmaf(a[u][3], v[u].w, acc);
        }
    }
    return acc;
}

// pose (single-frame LBS, gsr_lbs_sp): the pose features are formed here from the frame's pose
// (rodrigues_one, the same expressions as k_lbs_rodrigues) instead of read from a launch before
__device__ __forceinline__ void blend_tiled1_block(const Blend1Job& j, int t) {
    __shared__ float red[2][4][64];
    __shared__ float sfeat[9 * (GSR_LBS_MAX_JOINTS - 1)];
    const int M = j.M, NB = j.NB, NP = j.NP;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hi = lane >> 5, l32 = lane & 31;
    const int m = t * 32 + l32;
    const float* feat = j.feat;
    if (j.pose && NP > 0 && j.v_posed) {
        const int jn = NP / 9;  // J - 1 posed joints (pose_feature skips the root)
        if ((int)threadIdx.x < jn) {
            float R[9];
            rodrigues_one(j.pose, (int)threadIdx.x + 1, j.pose2rot, R);
#pragma unroll
            for (int e = 0; e < 9; e++) sfeat[9 * threadIdx.x + e] = R[e] - ((e % 4) == 0 ? 1.0f : 0.0f);
        }
        __syncthreads();
        feat = sfeat;
    }
    red[0][w][lane] = NB > 0 ? blend_tiled_one(j.betas, j.sd_tiled, NB, t, w, hi, lane) : 0.f;
    red[1][w][lane] = (NP > 0 && j.v_posed) ? blend_tiled_one(feat, j.pd_tiled, NP, t, w, hi, lane) : 0.f;
    __syncthreads();
    if (w == 0 && hi == 0 && m < M) {
        float S = 0.f, Pz = 0.f;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            S += red[0][u][l32] + red[0][u][l32 + 32];
            Pz += red[1][u][l32] + red[1][u][l32 + 32];
        }
        const float vs = NB > 0 ? j.vt[m] + S : j.vt[m];
        j.v_shaped[m] = vs;
        if (j.v_posed) j.v_posed[m] = Pz + vs;
    }
}

__global__ __launch_bounds__(256) void k_lbs_blend_tiled1(Blend1Job j) { blend_tiled1_block(j, blockIdx.x); }

// Two independent single-frame blends in one launch (EHM's FLAME head blend beside the body's shape
// blend, gsr_ehm_forward at B = 1): workgroups [0, na) take job a, the rest job b.  One launch fewer
// on the serial per-frame path, and the two partial grids share the chip instead of running in turn.
__global__ __launch_bounds__(256) void k_lbs_blend_tiled1_pair(Blend1Job a, int na, Blend1Job b) {
    if ((int)blockIdx.x < na) blend_tiled1_block(a, blockIdx.x);
    else blend_tiled1_block(b, blockIdx.x - na);
}

// blend launcher: the matrix-core kernel for more than kLbsFrames frames, the streaming one otherwise
// (tiled bases, when the caller prepared them: B > kLbsFrames and B = 1)
static void launch_blend(int B, int M, int NB, int NP, const float* vt, int64_t vt_stride, const float* betas,
                         const float* sd_t, const float* feat, const float* pd, float* vs, float* vp,
                         hipStream_t s, const GsrLbsSparse* sp = nullptr, const float* pose = nullptr,
                         int pose2rot = 1);

// the single-frame tiled blend forms the pose features itself (k_lbs_blend_tiled1's pose argument)
static bool blend_takes_pose(int B, int NB, int NP, const float* vp, const GsrLbsSparse* sp) {
    static const bool tiled_on = tune_env("GSR_BLEND_TILED", 1) != 0;
    return B == 1 && tiled_on && sp && (NB == 0 || sp->shapedirs_tiled) && (NP == 0 || !vp || sp->posedirs_tiled) &&
           (NB > 0 || (NP > 0 && vp)) && NP <= 9 * (GSR_LBS_MAX_JOINTS - 1);
}

static size_t lbs_blend_lds(int NB, int NP, int nf, int split) {
    const size_t coef = sizeof(float) * (size_t)(NB + NP) * nf;
    const size_t red = sizeof(float) * (size_t)split * nf * 64;
    return coef > red ? coef : red;
}

static void lbs_blend_attr(size_t lds) {
    static size_t attr = 0;
    if (lds > 65536 && attr < lds) {
        attr = lds;
        hipFuncSetAttribute((const void*)k_lbs_blend<kLbsFrames, kLbsSplit>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipFuncSetAttribute((const void*)k_lbs_blend<1, kLbsSplit1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
    }
}

Blend1Job blend1_job(int M, int NB, int NP, const float* vt, const float* betas, const float* feat, float* vs,
                     float* vp, const GsrLbsSparse* sp, const float* pose, int pose2rot) {
    return Blend1Job{M, NB, vp ? NP : 0, pose2rot, vt, betas, reinterpret_cast<const float4*>(sp->shapedirs_tiled),
                     feat, reinterpret_cast<const float4*>(sp->posedirs_tiled), vs, vp, pose};
}

// whether launch_blend takes the single-frame tiled kernel (k_lbs_blend_tiled1) for these arguments
bool blend_tiled1_applies(int B, int NB, int NP, const float* vp, const GsrLbsSparse* sp) {
    static const bool tiled_on = tune_env("GSR_BLEND_TILED", 1) != 0;
    return B == 1 && tiled_on && sp && (NB == 0 || sp->shapedirs_tiled) && (NP == 0 || !vp || sp->posedirs_tiled) &&
           (NB > 0 || (NP > 0 && vp));
}

static void launch_blend(int B, int M, int NB, int NP, const float* vt, int64_t vt_stride, const float* betas,
                         const float* sd_t, const float* feat, const float* pd, float* vs, float* vp,
                         hipStream_t s, const GsrLbsSparse* sp, const float* pose, int pose2rot) {
    static const bool valu_only = tune_env("GSR_BLEND_VALU", 0) == 1;  // timing A/B only
    // GSR_BLEND_TILED=0: the k-major kernels even with tiled bases (A/B)
    static const bool tiled_on = tune_env("GSR_BLEND_TILED", 1) != 0;
    const bool tiled = tiled_on && sp && (NB == 0 || sp->shapedirs_tiled) &&
                       (NP == 0 || !vp || sp->posedirs_tiled) && (NB > 0 || (NP > 0 && vp));
    if (tiled && B > kLbsFrames && !valu_only) {
        static const int nw_env = tune_env("GSR_BLEND_NW", 0);
        const dim3 grid((M + 31) / 32, (B + 31) / 32);
        const int nw = nw_env == 4 || nw_env == 8 ? nw_env : (grid.x * grid.y <= 512 ? 8 : 4);
        const float4* sdt = reinterpret_cast<const float4*>(sp->shapedirs_tiled);
        const float4* pdt = reinterpret_cast<const float4*>(sp->posedirs_tiled);
        if (nw == 8)
            hipLaunchKernelGGL(k_lbs_blend_tiled<8>, grid, dim3(512), 0, s, B, M, NB, vp ? NP : 0, vt, vt_stride,
                               betas, sdt, feat, pdt, vs, vp);
        else
            hipLaunchKernelGGL(k_lbs_blend_tiled<4>, grid, dim3(256), 0, s, B, M, NB, vp ? NP : 0, vt, vt_stride,
                               betas, sdt, feat, pdt, vs, vp);
        return;
    }
    if (tiled && B == 1) {
        const Blend1Job j = blend1_job(M, NB, NP, vt, betas, feat, vs, vp, sp, pose, pose2rot);
        hipLaunchKernelGGL(k_lbs_blend_tiled1, dim3((M + 31) / 32), dim3(256), 0, s, j);
        return;
    }
    if (B > kLbsFrames && !valu_only) {
        hipLaunchKernelGGL(k_lbs_blend_mfma, dim3((M + 31) / 32, (B + 31) / 32), dim3(256), 0, s, B, M, NB,
                           vp ? NP : 0, vt, vt_stride, betas, sd_t, feat, pd, vs, vp);
        return;
    }
    static const bool single = tune_env("GSR_BLEND_SINGLE", 1) != 0;  // 0: B = 1 on the 16-frame kernel (A/B)
    if (B == 1 && single) {
        const size_t lds = lbs_blend_lds(NB, vp ? NP : 0, 1, kLbsSplit1);
        lbs_blend_attr(lds);
        hipLaunchKernelGGL((k_lbs_blend<1, kLbsSplit1>), lbs_blend_grid(M, B, 1), dim3(64 * kLbsSplit1), lds, s, B, M,
                           NB, vp ? NP : 0, vt, vt_stride, betas, sd_t, feat, pd, vs, vp);
        return;
    }
    const size_t lds = lbs_blend_lds(NB, vp ? NP : 0, kLbsFrames, kLbsSplit);
    lbs_blend_attr(lds);
    hipLaunchKernelGGL((k_lbs_blend<kLbsFrames, kLbsSplit>), lbs_blend_grid(M, B, kLbsFrames), dim3(64 * kLbsSplit),
                       lds, s, B, M, NB, vp ? NP : 0, vt, vt_stride, betas, sd_t, feat, pd, vs, vp);
}

// vertices2joints (lbs.py:335-352): J[b,j,:] = sum_v J_regressor[j,v] v_shaped[b,v,:], plus
// joints_offset (lbs.py:191/:295).  One workgroup per (group of kJointsPerWG joints, frame), so a
// frame's vertices are read once per group rather than once per joint; fixed-shape tree reduction.
constexpr int kJointsPerWG = 4;

__global__ __launch_bounds__(256) void k_lbs_joints(int V, int J, const float* __restrict__ jreg,
                                                    const float* __restrict__ v_shaped,
                                                    const float* __restrict__ joff,
                                                    float* __restrict__ joints) {
    __shared__ float red[3 * kJointsPerWG][256];
    const int j0 = blockIdx.x * kJointsPerWG, b = blockIdx.y;
    const int nj = min(kJointsPerWG, J - j0);
    const float* vs = v_shaped + (int64_t)b * V * 3;
    float acc[kJointsPerWG][3];
#pragma unroll
    for (int q = 0; q < kJointsPerWG; q++) acc[q][0] = acc[q][1] = acc[q][2] = 0.f;
    // four vertices' loads in flight per round; each thread still sums its vertices in index order
    constexpr int kU = 4;
    int v0 = threadIdx.x;
    for (; v0 + 256 * (kU - 1) < V; v0 += 256 * kU) {
        float x[kU], y[kU], z[kU], wv[kU][kJointsPerWG];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int v = v0 + 256 * u;
            x[u] = vs[3 * v]; y[u] = vs[3 * v + 1]; z[u] = vs[3 * v + 2];
#pragma unroll
            for (int q = 0; q < kJointsPerWG; q++) wv[u][q] = q < nj ? jreg[(int64_t)(j0 + q) * V + v] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kU; u++)
#pragma unroll
            for (int q = 0; q < kJointsPerWG; q++) {
                acc[q][0] = fmaf(wv[u][q], x[u], acc[q][0]);
                acc[q][1] = fmaf(wv[u][q], y[u], acc[q][1]);
                acc[q][2] = fmaf(wv[u][q], z[u], acc[q][2]);
            }
    }
    for (int v = v0; v < V; v += 256) {
        const float x = vs[3 * v], y = vs[3 * v + 1], z = vs[3 * v + 2];
#pragma unroll
        for (int q = 0; q < kJointsPerWG; q++) {
            const float wv = q < nj ? jreg[(int64_t)(j0 + q) * V + v] : 0.f;
            acc[q][0] = fmaf(wv, x, acc[q][0]);
            acc[q][1] = fmaf(wv, y, acc[q][1]);
            acc[q][2] = fmaf(wv, z, acc[q][2]);
        }
    }
#pragma unroll
    for (int q = 0; q < kJointsPerWG; q++)
        for (int c = 0; c < 3; c++) red[3 * q + c][threadIdx.x] = acc[q][c];
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h)
#pragma unroll
            for (int e = 0; e < 3 * kJointsPerWG; e++) red[e][threadIdx.x] += red[e][threadIdx.x + h];
        __syncthreads();
    }
    if ((int)threadIdx.x < 3 * nj) {
        const int q = threadIdx.x / 3, c = threadIdx.x - 3 * q;
        float v = red[threadIdx.x][0];
        if (joff) v = v + joff[((int64_t)b * J + j0 + q) * 3 + c];
        joints[((int64_t)b * J + j0 + q) * 3 + c] = v;
    }
}

// vertices2joints over the J_regressor's nonzeros (CSR rows, vertex order; gsr_lbs_sp): one wave
// per (joint, frame), lanes take the row's nonzeros 64 at a time (each lane its own fmaf chain in
// index order), then a fixed xor-tree across the lanes -- deterministic run to run.  SMPL-X / FLAME
// joint regressors are sparse (a joint averages a few dozen vertices), so a frame's joints cost one
// load round instead of the dense kernel's pass over J x V weights.
__global__ __launch_bounds__(256) void k_lbs_joints_csr(int B, int V, int J, const int32_t* __restrict__ row,
                                                        const int32_t* __restrict__ col,
                                                        const float* __restrict__ val,
                                                        const float* __restrict__ v_shaped,
                                                        const float* __restrict__ joff,
                                                        float* __restrict__ joints) {
    const int w = (int)((blockIdx.x * 256u + threadIdx.x) >> 6), lane = threadIdx.x & 63;
    if (w >= B * J) return;
    const int b = w / J, j = w - b * J;
    const float* vs = v_shaped + (int64_t)b * V * 3;
    float x = 0.f, y = 0.f, z = 0.f;
    for (int k = row[j] + lane; k < row[j + 1]; k += 64) {
        const int v = col[k];
        const float wv = val[k];
        x = fmaf(wv, vs[3 * v], x);
        y = fmaf(wv, vs[3 * v + 1], y);
        z = fmaf(wv, vs[3 * v + 2], z);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        x += __shfl_xor(x, off);
        y += __shfl_xor(y, off);
        z += __shfl_xor(z, off);
    }
    if (lane < 3) {
        float v = lane == 0 ? x : lane == 1 ? y : z;
        if (joff) v = v + joff[((int64_t)b * J + j) * 3 + lane];
        joints[((int64_t)b * J + j) * 3 + lane] = v;
    }
}

// batch_rigid_transform (lbs.py:426-482), one frame per workgroup: local transforms
// [R | J_i - J_parent], the chain product chain_i = chain_parent . local_i, posed joints =
// chain[:, :3, 3], A = chain - pad(chain . [J; 0]).  The chain runs level by level of the kinematic
// tree (16 threads per joint, one matrix element each): every joint of a level in one step, so
// SMPL-X's 54 sequential products become its tree depth (~10) barrier steps -- each product is
// the same expression as the sequential chain's, so the results are identical.
// rot == null: each joint's rotation from the pose (rodrigues_one), as the single-frame path does.
// jrow != null (single frame, CSR regressor): the rest joints are regressed here first -- each of the
// 16 waves takes joints w, w + 16, ... with k_lbs_joints_csr's per-lane chains and xor tree (the same
// sums, bit for bit) -- and written to `joints`, one launch fewer per lbs call.
struct ChainJoints {
    const int32_t* row;
    const int32_t* col;
    const float* val;
    const float* vs;    // v_shaped of the frame
    const float* joff;  // or null
};
__global__ __launch_bounds__(16 * GSR_LBS_MAX_JOINTS) void k_lbs_chain(int J, Parents par,
                                                                     const float* __restrict__ rot,
                                                                     float* __restrict__ joints,
                                                                     float* __restrict__ jtrans,
                                                                     float* __restrict__ A,
                                                                     const float* __restrict__ pose, int pose2rot,
                                                                     ChainJoints cj) {
    __shared__ float tm[GSR_LBS_MAX_JOINTS][16];
    __shared__ float ch[GSR_LBS_MAX_JOINTS][16];
    __shared__ int depth[GSR_LBS_MAX_JOINTS];
    __shared__ float sjt[GSR_LBS_MAX_JOINTS * 3];
    __shared__ int maxd;
    const int b = blockIdx.x, t = threadIdx.x;
    const float* Jb = joints + (int64_t)b * J * 3;
    if (cj.row) {
        const int w = t >> 6, lane = t & 63;
        for (int j = w; j < J; j += 16) {
            float x = 0.f, y = 0.f, z = 0.f;
            for (int k = cj.row[j] + lane; k < cj.row[j + 1]; k += 64) {
                const int v = cj.col[k];
                const float wv = cj.val[k];
                x = fmaf(wv, cj.vs[3 * v], x);
                y = fmaf(wv, cj.vs[3 * v + 1], y);
                z = fmaf(wv, cj.vs[3 * v + 2], z);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                x += __shfl_xor(x, off);
                y += __shfl_xor(y, off);
                z += __shfl_xor(z, off);
            }
            if (lane < 3) {
                float v = lane == 0 ? x : lane == 1 ? y : z;
                if (cj.joff) v = v + cj.joff[j * 3 + lane];
                sjt[3 * j + lane] = v;
                joints[j * 3 + lane] = v;
            }
        }
        __syncthreads();
        Jb = sjt;
    }
    if (t == 0) maxd = 0;
    if (t < J) {
        float R[9];
        if (rot) {
#pragma unroll
            for (int e = 0; e < 9; e++) R[e] = rot[((int64_t)b * J + t) * 9 + e];
        } else {
            rodrigues_one(pose, b * J + t, pose2rot, R);
        }
        float rel[3];
        for (int c = 0; c < 3; c++) rel[c] = t == 0 ? Jb[c] : Jb[3 * t + c] - Jb[3 * par.p[t] + c];
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) tm[t][4 * r + c] = R[3 * r + c];
            tm[t][4 * r + 3] = rel[r];
        }
        tm[t][12] = 0.f; tm[t][13] = 0.f; tm[t][14] = 0.f; tm[t][15] = 1.f;
        int dd = 0;
        for (int i = t; i > 0 && dd < GSR_LBS_MAX_JOINTS; i = par.p[i]) dd++;  // (parents precede children)
        depth[t] = dd;
    }
    __syncthreads();
    if (t < J) atomicMax(&maxd, depth[t]);
    if (t < 16) ch[0][t] = tm[0][t];
    __syncthreads();
    const int j = t >> 4, e = t & 15, r = e >> 2, c = e & 3;
    const int dj = j < J ? depth[j] : -1;
    for (int lvl = 1; lvl <= maxd; lvl++) {
        if (dj == lvl) {
            const float* P = ch[par.p[j]];
            const float* L = tm[j];
            ch[j][e] = P[4 * r] * L[c] + P[4 * r + 1] * L[4 + c] + P[4 * r + 2] * L[8 + c] + P[4 * r + 3] * L[12 + c];
        }
        __syncthreads();
    }
    if (t < J) {
        const float* T = ch[t];
        const float jx = Jb[3 * t], jy = Jb[3 * t + 1], jz = Jb[3 * t + 2];
        float* a = A + ((int64_t)b * J + t) * 16;
        for (int rr = 0; rr < 4; rr++) {
            const float tj = T[4 * rr] * jx + T[4 * rr + 1] * jy + T[4 * rr + 2] * jz + T[4 * rr + 3] * 0.0f;
            a[4 * rr] = T[4 * rr];
            a[4 * rr + 1] = T[4 * rr + 1];
            a[4 * rr + 2] = T[4 * rr + 2];
            a[4 * rr + 3] = T[4 * rr + 3] - tj;
        }
        if (jtrans)
            for (int rr = 0; rr < 3; rr++) jtrans[((int64_t)b * J + t) * 3 + rr] = T[4 * rr + 3];
    }
}

// Skinning over each vertex's nonzero weights (ELL: K (joint, weight) pairs per vertex, joints
// increasing, padding weight 0; gsr_lbs_sp): the same fmaf chains in joint order as k_lbs_skin,
// minus its terms with a zero weight (fma(0, a, t) == t), so the results are bit-identical to the
// dense kernel's with K loads per vertex instead of J.
template <int KMAX>
__global__ __launch_bounds__(256) void k_lbs_skin_ell(int V, int J, int K, const int32_t* __restrict__ sj,
                                                      const float* __restrict__ sw,
                                                      const float* __restrict__ A,
                                                      const float* __restrict__ v_posed,
                                                      float* __restrict__ verts,
                                                      float* __restrict__ vtrans) {
    __shared__ float As[GSR_LBS_MAX_JOINTS * 16];
    const int b = blockIdx.y;
    for (int i = threadIdx.x; i < J * 16; i += blockDim.x) As[i] = A[(int64_t)b * J * 16 + i];
    __syncthreads();
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    int jj[KMAX];
    float ww[KMAX];
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        jj[u] = u < K ? min((int)sj[(int64_t)u * V + v], J - 1) : 0;  // (in range by contract; clamped)
        ww[u] = u < K ? sw[(int64_t)u * V + v] : 0.f;
    }
    float T[16];
#pragma unroll
    for (int e = 0; e < 16; e++) T[e] = 0.f;
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        if (u >= K) break;
        const float* Aj = As + 16 * jj[u];
#pragma unroll
        for (int e = 0; e < 16; e++) T[e] = fmaf(ww[u], Aj[e], T[e]);
    }
    const float* vp = v_posed + ((int64_t)b * V + v) * 3;
    const float px = vp[0], py = vp[1], pz = vp[2];
    float* out = verts + ((int64_t)b * V + v) * 3;
#pragma unroll
    for (int r = 0; r < 3; r++) out[r] = T[4 * r] * px + T[4 * r + 1] * py + T[4 * r + 2] * pz + T[4 * r + 3] * 1.0f;
    if (vtrans) {
        float* o = vtrans + ((int64_t)b * V + v) * 16;
#pragma unroll
        for (int e = 0; e < 16; e++) o[e] = T[e];
    }
}

// Skinning (lbs.py:218-227 / :320-331): T = W . A per vertex, v = T [v_posed; 1].
__global__ __launch_bounds__(256) void k_lbs_skin(int V, int J, const float* __restrict__ w_t,
                                                  const float* __restrict__ A,
                                                  const float* __restrict__ v_posed,
                                                  float* __restrict__ verts,
                                                  float* __restrict__ vtrans) {
    __shared__ float As[GSR_LBS_MAX_JOINTS * 16];
    const int b = blockIdx.y;
    for (int i = threadIdx.x; i < J * 16; i += blockDim.x) As[i] = A[(int64_t)b * J * 16 + i];
    __syncthreads();
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    // T = sum_j w_j A_j as 8 packed pairs (v_pk_fma_f32: two independent fmaf chains per
    // instruction, each in j order); four weight loads in flight per round
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 T2[8];
#pragma unroll
    for (int e = 0; e < 8; e++) T2[e] = f2{0.f, 0.f};
    const f2* A2 = reinterpret_cast<const f2*>(As);
    // 16 weight loads in flight per round (the kernel is load-latency bound; J <= 64 is 4 rounds)
    for (int j0 = 0; j0 < J; j0 += 16) {
        float w16[16];
#pragma unroll
        for (int u = 0; u < 16; u++) w16[u] = j0 + u < J ? w_t[(int64_t)(j0 + u) * V + v] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; u++) {
            if (j0 + u >= J) break;
#pragma unroll
            for (int e = 0; e < 8; e++)
                T2[e] = __builtin_elementwise_fma(f2{w16[u], w16[u]}, A2[8 * (j0 + u) + e], T2[e]);
        }
    }
    float T[16];
#pragma unroll
    for (int e = 0; e < 8; e++) { T[2 * e] = T2[e].x; T[2 * e + 1] = T2[e].y; }
    const float* p = v_posed + ((int64_t)b * V + v) * 3;
    const float x = p[0], y = p[1], z = p[2];
    float* o = verts + ((int64_t)b * V + v) * 3;
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = T[4 * r] * x + T[4 * r + 1] * y + T[4 * r + 2] * z + T[4 * r + 3] * 1.0f;
    if (vtrans) {
        float4* tv = reinterpret_cast<float4*>(vtrans + ((int64_t)b * V + v) * 16);
        tv[0] = make_float4(T[0], T[1], T[2], T[3]);
        tv[1] = make_float4(T[4], T[5], T[6], T[7]);
        tv[2] = make_float4(T[8], T[9], T[10], T[11]);
        tv[3] = make_float4(T[12], T[13], T[14], T[15]);
    }
}

// EHM.forward's head splice (EHM.py:72-75, :121-124): the FLAME head vertices (+ eyelid blend
// shapes, times head_scale) replace the body template's FLAME-mapped vertices, re-anchored from the
// mean of head joints [hj0, hj1) to the mean of body joints [bj0, bj1).
__global__ __launch_bounds__(256) void k_splice_head(
    int Vb, int Nh, const int32_t* __restrict__ idx, const float* __restrict__ head,
    const float* __restrict__ r_eyelid, const float* __restrict__ l_eyelid,
    const float* __restrict__ eyelid, const float* __restrict__ head_scale,
    const float* __restrict__ hjoints, int Jh, int hj0, int hj1, const float* __restrict__ bjoints,
    int Jb, int bj0, int bj1, float* __restrict__ body, uint32_t* __restrict__ bad) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Nh) return;
    const int d = idx[i];
    if (d < 0 || d >= Vb) {
        if (bad) atomicOr(bad, 2u);
        return;
    }
    const float* hj = hjoints + (int64_t)b * Jh * 3;
    const float* bjt = bjoints + (int64_t)b * Jb * 3;
    for (int c = 0; c < 3; c++) {
        float h = head[((int64_t)b * Nh + i) * 3 + c];
        if (eyelid) {
            h = h + r_eyelid[3 * i + c] * eyelid[2 * b + 1];
            h = h + l_eyelid[3 * i + c] * eyelid[2 * b];
        }
        if (head_scale) h = h * head_scale[3 * b + c];
        float hs = 0.f, bs = 0.f;
        for (int j = hj0; j < hj1; j++) hs += hj[3 * j + c];
        for (int j = bj0; j < bj1; j++) bs += bjt[3 * j + c];
        body[((int64_t)b * Vb + d) * 3 + c] = (h - hs / (float)(hj1 - hj0)) + bs / (float)(bj1 - bj0);
    }
}

// roma.rotmat_to_unitquat (scipy's from_matrix decision scheme), row-major m -> (x, y, z, w).
// The branch on the largest of (m00, m11, m22, trace) picks one of four candidate quaternions;
// the candidates share their off-diagonal sums, so all four are formed with 7 adds and the choice
// is made with selects (no dynamically indexed arrays, which compile to compare/select ladders).
__device__ __forceinline__ float4 rotmat_to_unitquat(const float m[9]) {
    const float d0 = m[0], d1 = m[4], d2 = m[8];
    const float d3 = (d0 + d1) + d2;
    int ch = 0;
    float best = d0;
    if (d1 > best) { best = d1; ch = 1; }
    if (d2 > best) { best = d2; ch = 2; }
    if (d3 > best) { best = d3; ch = 3; }
    const float t = 1.0f - d3;
    const float s01 = m[1] + m[3], s02 = m[2] + m[6], s12 = m[5] + m[7];  // m[3j+i] + m[3i+j]
    const float r0 = m[7] - m[5], r1 = m[2] - m[6], r2 = m[3] - m[1];     // the w candidates
    float4 q;
    q.x = ch == 0 ? t + 2.0f * m[0] : ch == 1 ? s01 : ch == 2 ? s02 : r0;
    q.y = ch == 0 ? s01 : ch == 1 ? t + 2.0f * m[4] : ch == 2 ? s12 : r1;
    q.z = ch == 0 ? s02 : ch == 1 ? s12 : ch == 2 ? t + 2.0f * m[8] : r2;
    q.w = ch == 0 ? r0 : ch == 1 ? r1 : ch == 2 ? r2 : 1.0f + d3;
    const float n = sqrtf(((q.x * q.x + q.y * q.y) + q.z * q.z) + q.w * q.w);
    return make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}

// roma.quat_product, xyzw: (p_w q_v + q_w p_v + p_v x q_v, p_w q_w - p_v . q_v)
__device__ __forceinline__ float4 quat_product(float4 p, float4 q) {
    float4 o;
    o.x = (p.w * q.x + q.w * p.x) + (p.y * q.z - p.z * q.y);
    o.y = (p.w * q.y + q.w * p.y) + (p.z * q.x - p.x * q.z);
    o.z = (p.w * q.z + q.w * p.z) + (p.x * q.y - p.y * q.x);
    o.w = p.w * q.w - ((p.x * q.x + p.y * q.y) + p.z * q.z);
    return o;
}

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx + ay * by) + az * bz;
}

// compute_face_orientation (graphics_utils.py:61-80, safe_normalize eps 1e-20) of one deformed face
// and the frame's rotmat_to_unitquat (ubody_gaussian.py:257-258): fr = {m[9] (row-major, columns
// a0 a1 a2), s, q.xyzw}.
__device__ __forceinline__ void face_frame(const float* __restrict__ vb, int i0, int i1, int i2, float fr[14]) {
    const float v0x = vb[3 * i0], v0y = vb[3 * i0 + 1], v0z = vb[3 * i0 + 2];
    const float e1x = vb[3 * i1] - v0x, e1y = vb[3 * i1 + 1] - v0y, e1z = vb[3 * i1 + 2] - v0z;
    const float e2x = vb[3 * i2] - v0x, e2y = vb[3 * i2 + 1] - v0y, e2z = vb[3 * i2 + 2] - v0z;
    const float l1 = sqrtf(fmaxf(dot3(e1x, e1y, e1z, e1x, e1y, e1z), 1e-20f));
    const float a0x = e1x / l1, a0y = e1y / l1, a0z = e1z / l1;
    const float c1x = a0y * e2z - a0z * e2y, c1y = a0z * e2x - a0x * e2z, c1z = a0x * e2y - a0y * e2x;
    const float lc1 = sqrtf(fmaxf(dot3(c1x, c1y, c1z, c1x, c1y, c1z), 1e-20f));
    const float a1x = c1x / lc1, a1y = c1y / lc1, a1z = c1z / lc1;
    const float c2x = a1y * a0z - a1z * a0y, c2y = a1z * a0x - a1x * a0z, c2z = a1x * a0y - a1y * a0x;
    const float lc2 = sqrtf(fmaxf(dot3(c2x, c2y, c2z, c2x, c2y, c2z), 1e-20f));
    const float a2x = -(c2x / lc2), a2y = -(c2y / lc2), a2z = -(c2z / lc2);
    const float m[9] = {a0x, a1x, a2x, a0y, a1y, a2y, a0z, a1z, a2z};
    const float4 q = rotmat_to_unitquat(m);
#pragma unroll
    for (int k = 0; k < 9; k++) fr[k] = m[k];
    fr[9] = (l1 + fabsf(dot3(a2x, a2y, a2z, e2x, e2y, e2z))) / 2.0f;
    fr[10] = q.x; fr[11] = q.y; fr[12] = q.z; fr[13] = q.w;
}

constexpr int kDeformFrames = 8;  // frames per workgroup (GSR_DEFORM_FRAMES overrides, timing only)
constexpr int kFrStride = 15;  // LDS floats per face frame (odd: conflict-free per-thread rows)

// Vertex Gaussians (ubody_gaussian.py:252-254): xyz = LBS vertex, rotation =
// normalize(q(T_v[:3,:3]) (x) q_v) in wxyz, scale unchanged.  UV Gaussians (:257-271): frame
// [a0 a1 a2], scale s and q(frame) of the deformed binding face, centre = bary . face vertices,
// xyz = (frame . local) * s + centre, rotation = q(frame) (x) q_uv (not renormalised), scale =
// scale * s.
//
// One thread per Gaussian and fpw frames per workgroup: the frame-independent inputs (binding,
// face vertex indices, barycentrics and, when shared, local offsets / rotations / scales) are read
// once per workgroup instead of once per frame, which is most of the kernel's HBM traffic.  Face
// frames are computed once per (face, frame) as the reference does: GUAVA's UV Gaussians come in
// texel order, so a workgroup's 256 Gaussians bind a short run of faces, and the workgroup
// computes that run's frames into LDS (one thread per face) for its Gaussians to read; a
// workgroup whose faces span more than 256 ids computes per Gaussian (same function, same bits).
__global__ __launch_bounds__(256) void k_deform_gaussians(
    int B, int fpw, int V, int F, int N, const float* __restrict__ verts, const float* __restrict__ vtrans,
    const int32_t* __restrict__ faces, const float* __restrict__ vrot, int64_t s_vrot,
    const float* __restrict__ vscale, int64_t s_vscale, const int32_t* __restrict__ bind,
    const float* __restrict__ bary, const float* __restrict__ lxyz, int64_t s_lxyz,
    const float* __restrict__ urot, int64_t s_urot, const float* __restrict__ uscale,
    int64_t s_uscale, float* __restrict__ means, float* __restrict__ rots, float* __restrict__ scales,
    uint32_t* __restrict__ bad) {
    __shared__ float fr_lds[256 * kFrStride];
    __shared__ int range[2];
    const int P = V + N;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool uv = i >= V && i < P;
    const int n = i - V;
    // binding resolved once (reference: an IndexError; here a flag and NaN outputs)
    int f = -1, j0 = 0, j1 = 0, j2 = 0;
    if (uv) {
        const int bf = bind[n];
        if (bf >= 0 && bf < F) {
            const int a = faces[3 * bf], c = faces[3 * bf + 1], d = faces[3 * bf + 2];
            if (a >= 0 && a < V && c >= 0 && c < V && d >= 0 && d < V) { f = bf; j0 = a; j1 = c; j2 = d; }
        }
        if (f < 0 && bad) atomicOr(bad, 1u);
    }
    float w0 = 0.f, w1 = 0.f, w2 = 0.f;
    if (uv) { w0 = bary[3 * n]; w1 = bary[3 * n + 1]; w2 = bary[3 * n + 2]; }
    // the workgroup's face run
    if (threadIdx.x == 0) { range[0] = INT_MAX; range[1] = -1; }
    __syncthreads();
    if (f >= 0) { atomicMin(&range[0], f); atomicMax(&range[1], f); }
    __syncthreads();
    const int fmin = range[0], nf = range[1] - range[0] + 1;
    const bool shared_frames = range[1] >= 0 && nf <= 256;
    int t0 = -1, t1 = 0, t2 = 0;  // this thread's face in the run (shared mode)
    if (shared_frames && (int)threadIdx.x < nf) {
        const int ff = fmin + threadIdx.x;
        const int a = faces[3 * ff], c = faces[3 * ff + 1], d = faces[3 * ff + 2];
        if (a >= 0 && a < V && c >= 0 && c < V && d >= 0 && d < V) { t0 = a; t1 = c; t2 = d; }
    }
    const int b1 = min(B, (int)(blockIdx.y + 1) * fpw);
    for (int b = blockIdx.y * fpw; b < b1; b++) {
        const float* vb = verts + (int64_t)b * V * 3;
        if (shared_frames) {
            if (b > blockIdx.y * fpw) __syncthreads();  // the previous frame's readers are done
            if (t0 >= 0) face_frame(vb, t0, t1, t2, fr_lds + threadIdx.x * kFrStride);
            __syncthreads();
        }
        if (i >= P) continue;
        const int64_t o = (int64_t)b * P + i;
        if (i < V) {
            const float4* tv = reinterpret_cast<const float4*>(vtrans + ((int64_t)b * V + i) * 16);
            const float4 r0 = tv[0], r1 = tv[1], r2 = tv[2];
            const float m[9] = {r0.x, r0.y, r0.z, r1.x, r1.y, r1.z, r2.x, r2.y, r2.z};
            const float4 qd = rotmat_to_unitquat(m);
            const float* qv = vrot + b * s_vrot + 4 * (int64_t)i;  // wxyz
            const float4 q = quat_product(qd, make_float4(qv[1], qv[2], qv[3], qv[0]));
            // F.normalize over the wxyz vector: x / max(||x||, 1e-12)
            const float nn = fmaxf(sqrtf(((q.w * q.w + q.x * q.x) + q.y * q.y) + q.z * q.z), 1e-12f);
            reinterpret_cast<float4*>(rots)[o] = make_float4(q.w / nn, q.x / nn, q.y / nn, q.z / nn);
            for (int c = 0; c < 3; c++) {
                means[3 * o + c] = vb[3 * i + c];
                scales[3 * o + c] = vscale[b * s_vscale + 3 * (int64_t)i + c];
            }
            continue;
        }
        if (f < 0) {
            const float nan = __int_as_float(0x7fc00000);
            for (int c = 0; c < 3; c++) { means[3 * o + c] = nan; scales[3 * o + c] = nan; }
            reinterpret_cast<float4*>(rots)[o] = make_float4(nan, nan, nan, nan);
            continue;
        }
        float fr[14];
        if (shared_frames) {
            const float* src = fr_lds + (f - fmin) * kFrStride;
#pragma unroll
            for (int k = 0; k < 14; k++) fr[k] = src[k];
        } else {
            face_frame(vb, j0, j1, j2, fr);
        }
        const float s = fr[9];
        const float* qu = urot + b * s_urot + 4 * (int64_t)n;  // wxyz
        const float4 q = quat_product(make_float4(fr[10], fr[11], fr[12], fr[13]), make_float4(qu[1], qu[2], qu[3], qu[0]));
        if (!GSR_DEFORM_NOSTORE || q.w == 12345.f) reinterpret_cast<float4*>(rots)[o] = make_float4(q.w, q.x, q.y, q.z);
        const float* l = lxyz + b * s_lxyz + 3 * (int64_t)n;
        const float lx = l[0], ly = l[1], lz = l[2];
        const float cx = (w0 * vb[3 * j0] + w1 * vb[3 * j1]) + w2 * vb[3 * j2];
        const float cy = (w0 * vb[3 * j0 + 1] + w1 * vb[3 * j1 + 1]) + w2 * vb[3 * j2 + 1];
        const float cz = (w0 * vb[3 * j0 + 2] + w1 * vb[3 * j1 + 2]) + w2 * vb[3 * j2 + 2];
        const float mx = dot3(fr[0], fr[1], fr[2], lx, ly, lz) * s + cx;
        const float my = dot3(fr[3], fr[4], fr[5], lx, ly, lz) * s + cy;
        const float mz = dot3(fr[6], fr[7], fr[8], lx, ly, lz) * s + cz;
        const float* us = uscale + b * s_uscale + 3 * (int64_t)n;
        if (!GSR_DEFORM_NOSTORE || mx == 12345.f) {
            means[3 * o] = mx; means[3 * o + 1] = my; means[3 * o + 2] = mz;
            for (int c = 0; c < 3; c++) scales[3 * o + c] = us[c] * s;
        }
    }
}

// The avatar pipeline's fused forward (gsr_forward_batch_deformed): k_deform_gaussians' assembly of
// each (Gaussian, frame) -- the same face-frame sharing and the same expressions -- handed in
// registers to the projection of k_preprocess (preprocess_dev.h), which writes the geometry rows
// and the per-block summaries of the frame.  Gaussian blocks of kScanBlock = 256 (the workgroup) are
// preprocess's blocks, so the block summaries index as k_preprocess's.
__global__ __launch_bounds__(256) void k_deform_preprocess(int fpw, GsrDeformInputs dg, Dims d, Inputs in,
                                                           GeomArena g, Outputs o) {
    __shared__ float fr_lds[256 * kFrStride];
    __shared__ int range[2];
    const int V = dg.V, F = dg.F, N = dg.N, P = V + N;
    const int32_t* __restrict__ faces = dg.faces;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool uv = i >= V && i < P;
    const int n = i - V;
    int f = -1, j0 = 0, j1 = 0, j2 = 0;
    if (uv) {
        const int bf = dg.binding_face[n];
        if (bf >= 0 && bf < F) {
            const int a = faces[3 * bf], c = faces[3 * bf + 1], e = faces[3 * bf + 2];
            if (a >= 0 && a < V && c >= 0 && c < V && e >= 0 && e < V) { f = bf; j0 = a; j1 = c; j2 = e; }
        }
        if (f < 0 && dg.bad_index_flag) atomicOr(dg.bad_index_flag, 1u);
    }
    float w0 = 0.f, w1 = 0.f, w2 = 0.f;
    if (uv) { w0 = dg.face_bary[3 * n]; w1 = dg.face_bary[3 * n + 1]; w2 = dg.face_bary[3 * n + 2]; }
    if (threadIdx.x == 0) { range[0] = INT_MAX; range[1] = -1; }
    __syncthreads();
    if (f >= 0) { atomicMin(&range[0], f); atomicMax(&range[1], f); }
    __syncthreads();
    const int fmin = range[0], nf = range[1] - range[0] + 1;
    const bool shared_frames = range[1] >= 0 && nf <= 256;
    int t0 = -1, t1 = 0, t2 = 0;
    if (shared_frames && (int)threadIdx.x < nf) {
        const int ff = fmin + threadIdx.x;
        const int a = faces[3 * ff], c = faces[3 * ff + 1], e = faces[3 * ff + 2];
        if (a >= 0 && a < V && c >= 0 && c < V && e >= 0 && e < V) { t0 = a; t1 = c; t2 = e; }
    }
    const int b1 = min(d.B, (int)(blockIdx.y + 1) * fpw);
    for (int b = blockIdx.y * fpw; b < b1; b++) {
        const float* vb = dg.verts + (int64_t)b * V * 3;
        if (shared_frames) {
            if (b > (int)blockIdx.y * fpw) __syncthreads();
            if (t0 >= 0) face_frame(vb, t0, t1, t2, fr_lds + threadIdx.x * kFrStride);
            __syncthreads();
        }
        // the frame's depth-bucket counters (k_preprocess's duty)
        for (int k = i; k <= d.NB; k += d.nblk * kScanBlock) g.bstart[(int64_t)b * (d.NB + 1) + k] = 0u;
        const int64_t gid = (int64_t)b * P + i;
        uint32_t tiles = 0;
        if (i < P) {
            float mo[3], so[3], qq[4];
            if (i < V) {
                const float4* tv = reinterpret_cast<const float4*>(dg.vert_transforms + ((int64_t)b * V + i) * 16);
                const float4 r0 = tv[0], r1 = tv[1], r2 = tv[2];
                const float m[9] = {r0.x, r0.y, r0.z, r1.x, r1.y, r1.z, r2.x, r2.y, r2.z};
                const float4 qd = rotmat_to_unitquat(m);
                const float* qv = dg.vtx_rotations + b * dg.vtx_rot_stride + 4 * (int64_t)i;  // wxyz
                const float4 q = quat_product(qd, make_float4(qv[1], qv[2], qv[3], qv[0]));
                const float nn = fmaxf(sqrtf(((q.w * q.w + q.x * q.x) + q.y * q.y) + q.z * q.z), 1e-12f);
                qq[0] = q.w / nn; qq[1] = q.x / nn; qq[2] = q.y / nn; qq[3] = q.z / nn;
                for (int c = 0; c < 3; c++) {
                    mo[c] = vb[3 * i + c];
                    so[c] = dg.vtx_scales[b * dg.vtx_scale_stride + 3 * (int64_t)i + c];
                }
            } else if (f < 0) {
                const float nan = __int_as_float(0x7fc00000);
                for (int c = 0; c < 3; c++) { mo[c] = nan; so[c] = nan; }
                for (int c = 0; c < 4; c++) qq[c] = nan;
            } else {
                float fr[14];
                if (shared_frames) {
                    const float* src = fr_lds + (f - fmin) * kFrStride;
#pragma unroll
                    for (int k = 0; k < 14; k++) fr[k] = src[k];
                } else {
                    face_frame(vb, j0, j1, j2, fr);
                }
                const float s = fr[9];
                const float* qu = dg.uv_rotations + b * dg.uv_rot_stride + 4 * (int64_t)n;  // wxyz
                const float4 q = quat_product(make_float4(fr[10], fr[11], fr[12], fr[13]),
                                              make_float4(qu[1], qu[2], qu[3], qu[0]));
                qq[0] = q.w; qq[1] = q.x; qq[2] = q.y; qq[3] = q.z;
                const float* l = dg.local_xyz + b * dg.local_stride + 3 * (int64_t)n;
                const float lx = l[0], ly = l[1], lz = l[2];
                const float cx = (w0 * vb[3 * j0] + w1 * vb[3 * j1]) + w2 * vb[3 * j2];
                const float cy = (w0 * vb[3 * j0 + 1] + w1 * vb[3 * j1 + 1]) + w2 * vb[3 * j2 + 1];
                const float cz = (w0 * vb[3 * j0 + 2] + w1 * vb[3 * j1 + 2]) + w2 * vb[3 * j2 + 2];
                mo[0] = dot3(fr[0], fr[1], fr[2], lx, ly, lz) * s + cx;
                mo[1] = dot3(fr[3], fr[4], fr[5], lx, ly, lz) * s + cy;
                mo[2] = dot3(fr[6], fr[7], fr[8], lx, ly, lz) * s + cz;
                const float* us = dg.uv_scales + b * dg.uv_scale_stride + 3 * (int64_t)n;
                for (int c = 0; c < 3; c++) so[c] = us[c] * s;
            }
            tiles = preprocess_one(d, in, g, o, b, gid, mo, nullptr, so, qq, in.opac[in.s_opac * b + i]);
        }
        preprocess_block_sums(d, g, b, blockIdx.x, tiles, gid);
    }
    zero_ctrl_words(d, in, g);  // (in.fwd_only is set: no backward reads this workspace)
}

void launch_deform_preprocess(const Dims& d, const Inputs& in, const GeomArena& g, const Outputs& o,
                              const GsrDeformInputs& dg, hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    // 4 frames per workgroup: 118.9 us per 32 frames vs 169.7 / 132.5 / 121.3 / 131.6 at 1 / 2 / 8 / 16
    // (GSR_FUSED_FRAMES; fewer re-reads of the binding set-up against fewer workgroups in flight)
    static const int fpw = [] {
        const int v = tune_env("GSR_FUSED_FRAMES", 4);
        return v >= 1 && v <= 64 ? v : 1;
    }();
    hipLaunchKernelGGL(k_deform_preprocess, dim3(d.nblk, (d.B + fpw - 1) / fpw), dim3(256), 0, s, fpw, dg, d, in,
                       g, o);
}

struct PackTable {
    GsrRowSegment seg[GSR_PACK_MAX_SEGMENTS];
};

// gsr_pack_rows: one workgroup per (segment, frame); a row piece is at most a few hundred floats
__global__ __launch_bounds__(256) void k_pack_rows(PackTable t) {
    const GsrRowSegment sg = t.seg[blockIdx.x];
    const int b = blockIdx.y;
    for (int c = threadIdx.x; c < sg.width; c += 256)
        sg.dst[b * sg.dst_stride + c] = sg.src ? sg.src[b * sg.src_stride + c] : 0.f;
}

namespace {

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct LbsArena {
    float *rot, *feat, *vs, *vp, *joints, *A;
};

size_t carve_lbs(char* base, int B, int V, int J, LbsArena* a) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return reinterpret_cast<float*>(p);
    };
    const size_t f = sizeof(float);
    LbsArena t;
    t.rot = take(f * (size_t)B * J * 9);
    t.feat = take(f * (size_t)B * (J > 1 ? J - 1 : 1) * 9);
    t.vs = take(f * (size_t)B * V * 3);
    t.vp = take(f * (size_t)B * V * 3);
    t.joints = take(f * (size_t)B * J * 3);
    t.A = take(f * (size_t)B * J * 16);
    if (a) *a = t;
    return off;
}

int hip_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return api_fail(GSR_ERR_HIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    return 0;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

// The tiled layout of a k-major base (GsrLbsSparse.*_tiled): one float4 per thread.
__global__ __launch_bounds__(256) void k_lbs_tile_base(int K, int M, int64_t n4, const float* __restrict__ base,
                                                       float4* __restrict__ tiled) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const int nkg = (K + 7) / 8;
    const int lane = (int)(i & 63);
    const int64_t tg = i >> 6;
    const int g = (int)(tg % nkg), t = (int)(tg / nkg);
    const int m = 32 * t + (lane & 31), k0 = 8 * g + 4 * (lane >> 5);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = (m < M && k0 + j < K) ? base[(int64_t)(k0 + j) * M + m] : 0.f;
    tiled[i] = make_float4(v[0], v[1], v[2], v[3]);
}

extern "C" {

size_t gsr_lbs_workspace_bytes(int B, int V, int J, int NB) {
    (void)NB;
    if (B <= 0 || V <= 0 || J <= 0) return 0;
    return carve_lbs(nullptr, B, V, J, nullptr);
}

}  // extern "C"

namespace {
// the joint regression of gsr_lbs / gsr_blend_joints: CSR rows when given, else the dense kernel
void launch_joints(int B, int V, int J, const float* J_regressor, const GsrLbsSparse* sp, const float* vs,
                   const float* joints_offset, float* joints, hipStream_t s) {
    if (sp && sp->jreg_row) {
        hipLaunchKernelGGL(k_lbs_joints_csr, dim3((B * J + 3) / 4), dim3(256), 0, s, B, V, J, sp->jreg_row,
                           sp->jreg_col, sp->jreg_val, vs, joints_offset, joints);
    } else {
        hipLaunchKernelGGL(k_lbs_joints, dim3((J + kJointsPerWG - 1) / kJointsPerWG, B), dim3(256), 0, s, V, J,
                           J_regressor, vs, joints_offset, joints);
    }
}
// NB: shape coefficients of the call, V: its vertices (the pose base is 9(J-1) x 3V)
int check_sparse(const GsrLbsSparse* sp, int J, int NB, int V, const char* who) {
    if (!sp) return 0;
    if (sp->jreg_row && (!sp->jreg_col || !sp->jreg_val))
        return api_fail(GSR_ERR_ARG, (std::string(who) + ": jreg_row without jreg_col / jreg_val").c_str());
    if (sp->skin_k && (sp->skin_k < 0 || sp->skin_k > GSR_LBS_SKIN_MAX_K || !sp->skin_joint || !sp->skin_weight))
        return api_fail(GSR_ERR_ARG, (std::string(who) + ": skin_k must be in [1, 16] with its arrays").c_str());
    if (((uintptr_t)sp->shapedirs_tiled | (uintptr_t)sp->posedirs_tiled) & 15)
        return api_fail(GSR_ERR_ARG, (std::string(who) + ": tiled bases must be 16-byte aligned").c_str());
    if (sp->shapedirs_tiled && NB > 0 && (sp->shapedirs_tiled_k != NB || sp->shapedirs_tiled_m != 3 * V))
        return api_fail(GSR_ERR_ARG, (std::string(who) + ": shapedirs_tiled was tiled for another NB x 3V").c_str());
    if (sp->posedirs_tiled && J > 1 && (sp->posedirs_tiled_k != 9 * (J - 1) || sp->posedirs_tiled_m != 3 * V))
        return api_fail(GSR_ERR_ARG, (std::string(who) + ": posedirs_tiled was tiled for another 9(J-1) x 3V").c_str());
    return 0;
}
}  // namespace

extern "C" {

int gsr_lbs(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
            const float* betas, const float* shapedirs_t, const float* pose, int pose2rot,
            const float* posedirs, const float* J_regressor, const int32_t* parents_host,
            const float* lbs_weights_t, const float* joints_offset, float* verts,
            float* joints_transformed, float* joints, float* vert_transforms,
            float* joint_transforms, float* v_shaped, char* workspace, void* stream) {
    return gsr_lbs_sp(B, V, J, NB, v_template, v_template_stride, betas, shapedirs_t, pose, pose2rot, posedirs,
                      J_regressor, parents_host, lbs_weights_t, joints_offset, verts, joints_transformed, joints,
                      vert_transforms, joint_transforms, v_shaped, workspace, nullptr, stream);
}

int gsr_lbs_sp(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
               const float* betas, const float* shapedirs_t, const float* pose, int pose2rot,
               const float* posedirs, const float* J_regressor, const int32_t* parents_host,
               const float* lbs_weights_t, const float* joints_offset, float* verts,
               float* joints_transformed, float* joints, float* vert_transforms,
               float* joint_transforms, float* v_shaped, char* workspace, const GsrLbsSparse* sp,
               void* stream) {
    return gsr::lbs_run(B, V, J, NB, v_template, v_template_stride, betas, shapedirs_t, pose, pose2rot, posedirs,
                        J_regressor, parents_host, lbs_weights_t, joints_offset, verts, joints_transformed, joints,
                        vert_transforms, joint_transforms, v_shaped, workspace, sp, stream, true);
}

}  // extern "C"

// gsr_lbs_sp, or (skin = false) everything up to the skinning: the joint transforms A and v_posed stay
// in the workspace (lbs_skin_splice reads them)
int gsr::lbs_run(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                 const float* betas, const float* shapedirs_t, const float* pose, int pose2rot,
                 const float* posedirs, const float* J_regressor, const int32_t* parents_host,
                 const float* lbs_weights_t, const float* joints_offset, float* verts,
                 float* joints_transformed, float* joints, float* vert_transforms,
                 float* joint_transforms, float* v_shaped, char* workspace, const GsrLbsSparse* sp,
                 void* stream, bool skin, const Blend1Job* companion, bool* companion_done) {
    if (companion_done) *companion_done = false;
    if (B <= 0 || V <= 0) return api_fail(GSR_ERR_ARG, "gsr_lbs: B and V must be positive");
    if (int rc = check_sparse(sp, J, betas ? NB : 0, V, "gsr_lbs")) return rc;
    if (J < 1 || J > GSR_LBS_MAX_JOINTS) return api_fail(GSR_ERR_ARG, "gsr_lbs: J must be in [1, 64]");
    if (!v_template || !pose || !J_regressor || !parents_host || !lbs_weights_t || (skin && !verts) || !workspace)
        return api_fail(GSR_ERR_ARG, "gsr_lbs: null required pointer");
    if (J > 1 && !posedirs) return api_fail(GSR_ERR_ARG, "gsr_lbs: posedirs is null");
    if (v_template_stride != 0 && v_template_stride != (int64_t)V * 3)
        return api_fail(GSR_ERR_ARG, "gsr_lbs: v_template stride must be 0 or V*3");
    if (betas) {
        if (NB <= 0 || !shapedirs_t) return api_fail(GSR_ERR_ARG, "gsr_lbs: betas need NB > 0 and shapedirs");
    } else {
        NB = 0;
    }
    Parents par;
    for (int i = 0; i < GSR_LBS_MAX_JOINTS; i++) par.p[i] = -1;
    if (parents_host[0] != -1) return api_fail(GSR_ERR_ARG, "gsr_lbs: parents[0] must be -1");
    for (int i = 1; i < J; i++) {
        if (parents_host[i] < 0 || parents_host[i] >= i)
            return api_fail(GSR_ERR_ARG, "gsr_lbs: parents must satisfy 0 <= parents[i] < i");
        par.p[i] = (int8_t)parents_host[i];
    }
    hipStream_t s = (hipStream_t)stream;
    LbsArena a;
    carve_lbs(workspace, B, V, J, &a);
    float* vs = v_shaped ? v_shaped : a.vs;
    float* jr = joints ? joints : a.joints;
    float* A = joint_transforms ? joint_transforms : a.A;
    const int NP = (J - 1) * 9;
    const int M = V * 3;

    if (lbs_blend_lds(NB, NP, kLbsFrames, kLbsSplit) > 160 * 1024) return api_fail(GSR_ERR_ARG, "gsr_lbs: NB + 9(J-1) too large for LDS");
    // single frame on tiled bases: Rodrigues runs inside the blend (pose features) and the chain
    // (rotations), one launch fewer on the per-frame path; otherwise its own launch feeds both
    const bool fused = blend_takes_pose(B, NB, NP, a.vp, sp);
    if (!fused) {
        hipLaunchKernelGGL(k_lbs_rodrigues, dim3((B * J + 255) / 256), dim3(256), 0, s, B, J, pose,
                           pose2rot, a.rot, a.feat);
        if (int rc = hip_check("lbs_rodrigues")) return rc;
    }
    if (companion && companion_done && blend_tiled1_applies(B, NB, NP, a.vp, sp)) {
        // this blend and the caller's independent one in one launch (k_lbs_blend_tiled1_pair)
        const Blend1Job ja = blend1_job(M, NB, NP, v_template, betas, a.feat, vs, a.vp, sp, fused ? pose : nullptr,
                                        pose2rot);
        const int na = (M + 31) / 32, nb = (companion->M + 31) / 32;
        hipLaunchKernelGGL(k_lbs_blend_tiled1_pair, dim3(na + nb), dim3(256), 0, s, ja, na, *companion);
        *companion_done = true;
    } else {
        launch_blend(B, M, NB, NP, v_template, v_template_stride, betas, shapedirs_t, a.feat, posedirs, vs, a.vp, s,
                     sp, fused ? pose : nullptr, pose2rot);
    }
    if (int rc = hip_check("lbs_blend")) return rc;
    // single frame with the CSR regressor: the joints are regressed inside the chain's workgroup
    // (GSR_CHAIN_JOINTS=0: their own launch, A/B)
    static const bool chain_joints_on = tune_env("GSR_CHAIN_JOINTS", 1) != 0;
    ChainJoints cj{nullptr, nullptr, nullptr, nullptr, nullptr};
    if (B == 1 && sp && sp->jreg_row && chain_joints_on) {
        cj = ChainJoints{sp->jreg_row, sp->jreg_col, sp->jreg_val, vs, joints_offset};
    } else {
        launch_joints(B, V, J, J_regressor, sp, vs, joints_offset, jr, s);
        if (int rc = hip_check("lbs_joints")) return rc;
    }
    hipLaunchKernelGGL(k_lbs_chain, dim3(B), dim3(16 * GSR_LBS_MAX_JOINTS), 0, s, J, par, fused ? nullptr : a.rot,
                       jr, joints_transformed, A, pose, pose2rot, cj);
    if (int rc = hip_check("lbs_chain")) return rc;
    if (!skin) return 0;
    if (sp && sp->skin_k > 0) {
        const dim3 g((V + 255) / 256, B);
        if (sp->skin_k <= 4)
            hipLaunchKernelGGL(k_lbs_skin_ell<4>, g, dim3(256), 0, s, V, J, sp->skin_k, sp->skin_joint,
                               sp->skin_weight, A, a.vp, verts, vert_transforms);
        else if (sp->skin_k <= 8)
            hipLaunchKernelGGL(k_lbs_skin_ell<8>, g, dim3(256), 0, s, V, J, sp->skin_k, sp->skin_joint,
                               sp->skin_weight, A, a.vp, verts, vert_transforms);
        else
            hipLaunchKernelGGL(k_lbs_skin_ell<16>, g, dim3(256), 0, s, V, J, sp->skin_k, sp->skin_joint,
                               sp->skin_weight, A, a.vp, verts, vert_transforms);
    } else {
        hipLaunchKernelGGL(k_lbs_skin, dim3((V + 255) / 256, B), dim3(256), 0, s, V, J, lbs_weights_t, A,
                           a.vp, verts, vert_transforms);
    }
    return hip_check("lbs_skin");
}

// The FLAME head's skinning fused into the splice (EHM.py:67-75, :121-124): per head vertex, the ELL
// skinning of k_lbs_skin_ell (the same fmaf chains and vertex expression, so the same head vertex),
// then k_splice_head's eyelids, head scale and re-anchoring, written straight into the body template:
// the head vertices never reach memory and one launch goes.
template <int KMAX>
__global__ __launch_bounds__(256) void k_skin_splice(int Vh, int Jh, int K, const int32_t* __restrict__ sj,
                                                     const float* __restrict__ sw, const float* __restrict__ A,
                                                     const float* __restrict__ v_posed, int Vb,
                                                     const int32_t* __restrict__ idx,
                                                     const float* __restrict__ r_eyelid,
                                                     const float* __restrict__ l_eyelid,
                                                     const float* __restrict__ eyelid,
                                                     const float* __restrict__ head_scale,
                                                     const float* __restrict__ hjoints, int hj0, int hj1,
                                                     const float* __restrict__ bjoints, int Jb, int bj0, int bj1,
                                                     float* __restrict__ body, uint32_t* __restrict__ bad) {
    __shared__ float As[GSR_LBS_MAX_JOINTS * 16];
    const int b = blockIdx.y;
    for (int i = threadIdx.x; i < Jh * 16; i += blockDim.x) As[i] = A[(int64_t)b * Jh * 16 + i];
    __syncthreads();
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= Vh) return;
    const int d = idx[v];
    if (d < 0 || d >= Vb) {
        if (bad) atomicOr(bad, 2u);
        return;
    }
    int jj[KMAX];
    float ww[KMAX];
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        jj[u] = u < K ? min((int)sj[(int64_t)u * Vh + v], Jh - 1) : 0;
        ww[u] = u < K ? sw[(int64_t)u * Vh + v] : 0.f;
    }
    float T[16];
#pragma unroll
    for (int e = 0; e < 16; e++) T[e] = 0.f;
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        if (u >= K) break;
        const float* Aj = As + 16 * jj[u];
#pragma unroll
        for (int e = 0; e < 16; e++) T[e] = fmaf(ww[u], Aj[e], T[e]);
    }
    const float* vp = v_posed + ((int64_t)b * Vh + v) * 3;
    const float px = vp[0], py = vp[1], pz = vp[2];
    const float* hjb = hjoints + (int64_t)b * Jh * 3;
    const float* bjt = bjoints + (int64_t)b * Jb * 3;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        float h = T[4 * c] * px + T[4 * c + 1] * py + T[4 * c + 2] * pz + T[4 * c + 3] * 1.0f;
        if (eyelid) {
            h = h + r_eyelid[3 * v + c] * eyelid[2 * b + 1];
            h = h + l_eyelid[3 * v + c] * eyelid[2 * b];
        }
        if (head_scale) h = h * head_scale[3 * b + c];
        float hs = 0.f, bs = 0.f;
        for (int j = hj0; j < hj1; j++) hs += hjb[3 * j + c];
        for (int j = bj0; j < bj1; j++) bs += bjt[3 * j + c];
        body[((int64_t)b * Vb + d) * 3 + c] = (h - hs / (float)(hj1 - hj0)) + bs / (float)(bj1 - bj0);
    }
}

// the launch for gsr_ehm_forward: A and v_posed from the head's lbs workspace (lbs_run(skin = false));
// returns 1 (nothing launched) when the head has no ELL skinning weights
int gsr::lbs_skin_splice(int B, int Vh, int Jh, const GsrLbsSparse* sp_h, const char* ws_h, int Vb,
                         const int32_t* head_index, const float* r_eyelid, const float* l_eyelid,
                         const float* eyelid, const float* head_scale, const float* head_joints, int hj0, int hj1,
                         const float* body_joints, int Jb, int bj0, int bj1, float* body_v_shaped,
                         uint32_t* bad_index_flag, void* stream) {
    if (!sp_h || sp_h->skin_k <= 0) return 1;
    if (hj0 < 0 || hj1 <= hj0 || hj1 > Jh || bj0 < 0 || bj1 <= bj0 || bj1 > Jb)
        return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: bad reference joint ranges");
    if (eyelid && (!r_eyelid || !l_eyelid)) return api_fail(GSR_ERR_ARG, "gsr_ehm_forward: eyelid bases missing");
    LbsArena a;
    carve_lbs(const_cast<char*>(ws_h), B, Vh, Jh, &a);
    const dim3 g((Vh + 255) / 256, B);
    hipStream_t s = (hipStream_t)stream;
#define GSR_SKS(KM)                                                                                              \
    hipLaunchKernelGGL(k_skin_splice<KM>, g, dim3(256), 0, s, Vh, Jh, sp_h->skin_k, sp_h->skin_joint,            \
                       sp_h->skin_weight, a.A, a.vp, Vb, head_index, r_eyelid, l_eyelid, eyelid, head_scale,     \
                       head_joints, hj0, hj1, body_joints, Jb, bj0, bj1, body_v_shaped, bad_index_flag)
    if (sp_h->skin_k <= 4) GSR_SKS(4);
    else if (sp_h->skin_k <= 8) GSR_SKS(8);
    else GSR_SKS(16);
#undef GSR_SKS
    return hip_check("skin_splice");
}

extern "C" {

int gsr_blend_joints(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                     const float* betas, const float* shapedirs_t, const float* J_regressor,
                     const float* joints_offset, float* v_shaped, float* joints, void* stream) {
    return gsr_blend_joints_sp(B, V, J, NB, v_template, v_template_stride, betas, shapedirs_t, J_regressor,
                               joints_offset, v_shaped, joints, nullptr, stream);
}

int gsr_blend_joints_sp(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                        const float* betas, const float* shapedirs_t, const float* J_regressor,
                        const float* joints_offset, float* v_shaped, float* joints, const GsrLbsSparse* sp,
                        void* stream) {
    return gsr::blend_joints_run(B, V, J, NB, v_template, v_template_stride, betas, shapedirs_t, J_regressor,
                                 joints_offset, v_shaped, joints, sp, stream, false);
}

}  // extern "C"

// gsr_blend_joints_sp; blend_done: the blend shapes were launched already (k_lbs_blend_tiled1_pair)
int gsr::blend_joints_run(int B, int V, int J, int NB, const float* v_template, int64_t v_template_stride,
                          const float* betas, const float* shapedirs_t, const float* J_regressor,
                          const float* joints_offset, float* v_shaped, float* joints, const GsrLbsSparse* sp,
                          void* stream, bool blend_done) {
    if (B <= 0 || V <= 0 || J < 1) return api_fail(GSR_ERR_ARG, "gsr_blend_joints: bad sizes");
    if (int rc = check_sparse(sp, 1, betas ? NB : 0, V, "gsr_blend_joints")) return rc;
    if (!v_template || !J_regressor || !v_shaped || !joints)
        return api_fail(GSR_ERR_ARG, "gsr_blend_joints: null required pointer");
    if (v_template_stride != 0 && v_template_stride != (int64_t)V * 3)
        return api_fail(GSR_ERR_ARG, "gsr_blend_joints: v_template stride must be 0 or V*3");
    if (betas && (NB <= 0 || !shapedirs_t))
        return api_fail(GSR_ERR_ARG, "gsr_blend_joints: betas need NB > 0 and shapedirs");
    if (!betas) NB = 0;
    if (lbs_blend_lds(NB, 0, kLbsFrames, kLbsSplit) > 160 * 1024) return api_fail(GSR_ERR_ARG, "gsr_blend_joints: NB too large for LDS");
    hipStream_t s = (hipStream_t)stream;
    const int M = V * 3;
    if (!blend_done) {
        launch_blend(B, M, NB, 0, v_template, v_template_stride, betas, shapedirs_t, nullptr, nullptr, v_shaped, nullptr,
                     s, sp);
        if (int rc = hip_check("blend_shapes")) return rc;
    }
    launch_joints(B, V, J, J_regressor, sp, v_shaped, joints_offset, joints, s);
    return hip_check("vertices2joints");
}

extern "C" {

size_t gsr_lbs_tiled_floats(int K, int M) {
    if (K <= 0 || M <= 0) return 0;
    return (size_t)((M + 31) / 32) * (size_t)((K + 7) / 8) * 256;
}

int gsr_lbs_tile_bases(int K, int M, const float* base, float* tiled, void* stream) {
    if (K <= 0 || M <= 0 || !base || !tiled) return api_fail(GSR_ERR_ARG, "gsr_lbs_tile_bases: bad arguments");
    if (((uintptr_t)tiled & 15) != 0) return api_fail(GSR_ERR_ARG, "gsr_lbs_tile_bases: tiled must be 16-byte aligned");
    const int64_t n4 = (int64_t)gsr_lbs_tiled_floats(K, M) / 4;
    hipLaunchKernelGGL(k_lbs_tile_base, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, K, M,
                       n4, base, reinterpret_cast<float4*>(tiled));
    return hip_check("lbs_tile_base");
}

int gsr_splice_head(int B, int V_body, int N_head, const int32_t* head_index, const float* head_verts,
                    const float* r_eyelid, const float* l_eyelid, const float* eyelid_params,
                    const float* head_scale, const float* head_joints, int J_head, int hj0, int hj1,
                    const float* body_joints, int J_body, int bj0, int bj1, float* body_v_shaped,
                    uint32_t* bad_index_flag, void* stream) {
    if (B <= 0 || V_body <= 0 || N_head < 0) return api_fail(GSR_ERR_ARG, "gsr_splice_head: bad sizes");
    if (N_head == 0) return 0;
    if (!head_index || !head_verts || !head_joints || !body_joints || !body_v_shaped)
        return api_fail(GSR_ERR_ARG, "gsr_splice_head: null required pointer");
    if (eyelid_params && (!r_eyelid || !l_eyelid))
        return api_fail(GSR_ERR_ARG, "gsr_splice_head: eyelid_params need both eyelid bases");
    if (hj0 < 0 || hj1 <= hj0 || hj1 > J_head || bj0 < 0 || bj1 <= bj0 || bj1 > J_body)
        return api_fail(GSR_ERR_ARG, "gsr_splice_head: bad reference joint ranges");
    hipLaunchKernelGGL(k_splice_head, dim3((N_head + 255) / 256, B), dim3(256), 0, (hipStream_t)stream,
                       V_body, N_head, head_index, head_verts, r_eyelid, l_eyelid, eyelid_params,
                       head_scale, head_joints, J_head, hj0, hj1, body_joints, J_body, bj0, bj1,
                       body_v_shaped, bad_index_flag);
    return hip_check("splice_head");
}

int gsr_pack_rows(int B, int nseg, const GsrRowSegment* segs, void* stream) {
    if (B <= 0 || nseg < 0 || nseg > GSR_PACK_MAX_SEGMENTS) return api_fail(GSR_ERR_ARG, "gsr_pack_rows: bad sizes");
    if (nseg == 0) return 0;
    if (!segs) return api_fail(GSR_ERR_ARG, "gsr_pack_rows: null segment table");
    PackTable t;
    for (int i = 0; i < nseg; i++) {
        t.seg[i] = segs[i];
        if (!segs[i].dst || segs[i].width < 0 || segs[i].width > 4096 || segs[i].dst_stride < segs[i].width ||
            segs[i].src_stride < 0)
            return api_fail(GSR_ERR_ARG, "gsr_pack_rows: bad segment");
    }
    hipLaunchKernelGGL(k_pack_rows, dim3(nseg, B), dim3(256), 0, (hipStream_t)stream, t);
    return hip_check("pack_rows");
}

int gsr_deform_gaussians(int B, int V, int F, int N, const float* verts,
                         const float* vert_transforms, const int32_t* faces,
                         const float* vtx_rotations, int64_t vtx_rot_stride,
                         const float* vtx_scales, int64_t vtx_scale_stride,
                         const int32_t* binding_face, const float* face_bary,
                         const float* local_xyz, int64_t local_stride,
                         const float* uv_rotations, int64_t uv_rot_stride,
                         const float* uv_scales, int64_t uv_scale_stride, float* means3D,
                         float* rotations, float* scales, uint32_t* bad_index_flag, void* stream) {
    if (B <= 0 || V < 0 || N < 0 || F < 0) return api_fail(GSR_ERR_ARG, "gsr_deform_gaussians: bad sizes");
    if (V + N == 0) return 0;
    if (!verts || !means3D || !rotations || !scales)
        return api_fail(GSR_ERR_ARG, "gsr_deform_gaussians: null required pointer");
    if (V > 0 && (!vert_transforms || !vtx_rotations || !vtx_scales))
        return api_fail(GSR_ERR_ARG, "gsr_deform_gaussians: vertex Gaussians need transforms, rotations, scales");
    if (N > 0 && (!faces || !binding_face || !face_bary || !local_xyz || !uv_rotations || !uv_scales || F == 0))
        return api_fail(GSR_ERR_ARG, "gsr_deform_gaussians: UV Gaussians need faces and binding data");
    auto bad_stride = [](int64_t st, int64_t full) { return st != 0 && st != full; };
    if (bad_stride(vtx_rot_stride, 4LL * V) || bad_stride(vtx_scale_stride, 3LL * V) ||
        bad_stride(local_stride, 3LL * N) || bad_stride(uv_rot_stride, 4LL * N) ||
        bad_stride(uv_scale_stride, 3LL * N))
        return api_fail(GSR_ERR_ARG, "gsr_deform_gaussians: strides must be 0 or a whole frame");
    hipStream_t s = (hipStream_t)stream;
    static const int fpw = [] {
        const int v = tune_env("GSR_DEFORM_FRAMES", kDeformFrames);
        return v >= 1 && v <= 64 ? v : 1;
    }();
    const int P = V + N;
    hipLaunchKernelGGL(k_deform_gaussians, dim3((P + 255) / 256, (B + fpw - 1) / fpw), dim3(256), 0, s, B, fpw,
                       V, F, N, verts, vert_transforms, faces, vtx_rotations, vtx_rot_stride, vtx_scales,
                       vtx_scale_stride, binding_face, face_bary, local_xyz, local_stride, uv_rotations,
                       uv_rot_stride, uv_scales, uv_scale_stride, means3D, rotations, scales,
                       bad_index_flag);
    return hip_check("deform_gaussians");
}

}  // extern "C"
