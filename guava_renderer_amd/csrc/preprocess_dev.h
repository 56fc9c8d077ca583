// preprocess_dev.h -- the per-Gaussian projection of preprocessCUDA (forward.cu:74-269), shared by
// k_preprocess (inputs from HBM) and the fused deform + preprocess kernel of the avatar pipeline
// (inputs straight from the Gaussian assembly's registers, deform.hip): one definition, the same
// bits either way.
#pragma once
#include "gsr_internal.h"

namespace gsr {

// forward.cu:114-148 computeCov3D (quaternion (r,x,y,z) = rot[0..3], not normalized)
__device__ __forceinline__ void cov3d_fwd(const float s[3], float mod, const float q[4], float* cov) {
    mat3 S = mk3(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * s[0];
    S.m[1][1] = mod * s[1];
    S.m[2][2] = mod * s[2];
    const float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = mk3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                 2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                 2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 M = mul3(S, R);
    mat3 Sig = mul3(tr3(M), M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

// One Gaussian of frame b (gid = b * P + i): mean p, and either cp (cov3D_precomp row) or scale sc +
// rotation q (wxyz); opacity op.  Writes its geometry rows (and o.radii) and returns its tile count.
__device__ __forceinline__ uint32_t preprocess_one(const Dims& d, const Inputs& in, const GeomArena& g,
                                                   const Outputs& o, int b, int64_t gid, const float p[3],
                                                   const float* cp, const float sc[3], const float q[4],
                                                   float op) {
    uint32_t tiles = 0;
    const float* view = in.view + 16 * b;
    const float* proj = in.proj + 16 * b;
    const float tanx = in.tan_dev ? in.tan_dev[2 * b] : in.tanx;
    const float tany = in.tan_dev ? in.tan_dev[2 * b + 1] : in.tany;
    // rasterizer_impl.cu:224-225
    const float focal_y = (float)d.H / (2.0f * tany);
    const float focal_x = (float)d.W / (2.0f * tanx);
    int radius = 0;
    uint2 rect = make_uint2(0, 0);
    // in_frustum (auxiliary.h:151-176)
    float ph[4];
    xform4x4(p, proj, ph);
    const float pw = 1.0f / (ph[3] + 0.0000001f);
    float pv[3];
    xform4x3(p, view, pv);
    if (pv[2] <= 0.2f) {
        if (in.prefiltered) atomicOr(&g.ctrl[kCtrlError], 1u);
    } else {
        const float pproj[2] = {ph[0] * pw, ph[1] * pw};
        float c3[6];
        if (cp) {
#pragma unroll
            for (int k = 0; k < 6; k++) c3[k] = cp[k];
        } else {
            cov3d_fwd(sc, in.scale_mod, q, c3);
            if (!in.fwd_only)
#pragma unroll
                for (int k = 0; k < 6; k++) g.cov3D[6 * gid + k] = c3[k];
        }
        // computeCov2D (forward.cu:74-109)
        float t[3];
        xform4x3(p, view, t);
        const float limx = 1.3f * tanx;
        const float limy = 1.3f * tany;
        const float txtz = t[0] / t[2];
        const float tytz = t[1] / t[2];
        t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
        t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
        const mat3 J = mk3(focal_x / t[2], 0.0f, -(focal_x * t[0]) / (t[2] * t[2]),
                           0.0f, focal_y / t[2], -(focal_y * t[1]) / (t[2] * t[2]), 0, 0, 0);
        const mat3 W = mk3(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6],
                           view[10]);
        const mat3 T = mul3(W, J);
        const mat3 V = mk3(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
        const mat3 cv = mul3(mul3(tr3(T), tr3(V)), T);
        float cx = cv.m[0][0], cy = cv.m[0][1], cz = cv.m[1][1];
        // forward.cu:215-245
        const float h_var = 0.3f;
        const float det_cov = cx * cz - cy * cy;
        cx += h_var;
        cz += h_var;
        const float det_cov_plus_h_cov = cx * cz - cy * cy;
        float h_conv = 1.0f;
        if (in.antialiasing) h_conv = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        const float det = det_cov_plus_h_cov;
        if (det != 0.0f) {
            const float det_inv = 1.f / det;
            const float conic0 = cz * det_inv, conic1 = -cy * det_inv, conic2 = cx * det_inv;
            const float mid = 0.5f * (cx + cz);
            const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
            const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
            const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
            const float pix0 = ndc2pix(pproj[0], d.W), pix1 = ndc2pix(pproj[1], d.H);
            uint32_t rmin[2], rmax[2];
            const int ir = f2i(my_radius);
            get_rect(pix0, pix1, ir, d.gx, d.gy, rmin, rmax);
            const uint32_t nt = (rmax[0] - rmin[0]) * (rmax[1] - rmin[1]);
            if (nt != 0) {
                g.depth[gid] = pv[2];
                if (!in.fwd_only) {  // (rows read by the backward only; binning reads the record)
                    g.invdepth[gid] = 1.0f / pv[2];
                    g.means2D[gid] = make_float2(pix0, pix1);
                    g.conic[gid] = make_float4(conic0, conic1, conic2, op * h_conv);
                }
                radius = ir;
                tiles = nt;
                rect = make_uint2(rmin[0] | (rmin[1] << 16), rmax[0] | (rmax[1] << 16));
                // render record (render_fwd.hip): position, opacity, 1/depth, pre-scaled conic
                // (exact power-of-two scalings)
                float4* rr = g.rrec + 2 * gid;
                rr[0] = make_float4(pix0, pix1, op * h_conv, 1.0f / pv[2]);
                rr[1] = make_float4(-0.5f * conic0, -conic1, -0.5f * conic2, 0.f);
            }
        }
    }
    if (!in.fwd_only) g.radii[gid] = radius;
    g.tiles[gid] = tiles;
    g.rect[gid] = rect;
    if (o.radii) o.radii[gid] = radius;
    return tiles;
}

// The per-block summaries of one frame's kScanBlock Gaussians (every thread of the block calls it):
// sum of tiles for the batch-wide scan, depth-key range of the frame for the bucket sort.
__device__ __forceinline__ void preprocess_block_sums(const Dims& d, const GeomArena& g, int b, int blk_x,
                                                      uint32_t tiles, int64_t gid) {
    __shared__ uint32_t red[3][kScanBlock / 64];
    uint32_t v = tiles;
    const uint32_t key = tiles ? __float_as_uint(g.depth[gid]) : 0u;  // depth > 0.2: monotone bits
    uint32_t kmax = key, nkmax = tiles ? ~key : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        v += __shfl_xor(v, off);
        kmax = max(kmax, (uint32_t)__shfl_xor(kmax, off));
        nkmax = max(nkmax, (uint32_t)__shfl_xor(nkmax, off));
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = v;
        red[1][threadIdx.x >> 6] = kmax;
        red[2][threadIdx.x >> 6] = nkmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0, km = 0, nkm = 0;
#pragma unroll
        for (int w = 0; w < kScanBlock / 64; w++) {
            s += red[0][w];
            km = max(km, red[1][w]);
            nkm = max(nkm, red[2][w]);
        }
        const int64_t blk = (int64_t)b * d.nblk + blk_x;
        g.blocksums[blk] = s;
        g.blockkey[2 * blk] = km;
        g.blockkey[2 * blk + 1] = nkm;
    }
    __syncthreads();  // red[] is reused by the next frame of a multi-frame caller
}


// The control words of a forward (ctrl + the per-frame fstat rows) start at zero: the first kernel
// of the forward (k_preprocess / k_deform_preprocess) zeroes them, one strided word per thread,
// instead of a memset launch before it (in.zero_ctrl).  None of those words is read or accumulated
// during that kernel except kCtrlError (a prefiltered forward's atomicOr: the host then keeps the
// memset) and kCtrlFwdOnly (written here from in.fwd_only).
__device__ __forceinline__ void zero_ctrl_words(const Dims& d, const Inputs& in, const GeomArena& g) {
    const int64_t t = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    if (in.zero_ctrl) {
        const int64_t n = (int64_t)kCtrlWords + (int64_t)kFsWords * d.B;
        const int64_t T = (int64_t)gridDim.x * gridDim.y * blockDim.x;
        for (int64_t k = t; k < n; k += T)
            if (k != kCtrlFwdOnly) g.ctrl[k] = 0u;
        if (t == 0) g.ctrl[kCtrlFwdOnly] = in.fwd_only ? 1u : 0u;
    } else if (in.fwd_only && t == 0) {
        g.ctrl[kCtrlFwdOnly] = 1u;
    }
}
}  // namespace gsr
