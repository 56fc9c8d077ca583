// preprocess.hip -- per-Gaussian projection (forward.cu:74-269 of the reference), one thread per
// Gaussian per frame, plus the frustum test of markVisible (rasterizer_impl.cu:54-66).
//
// Roofline: HBM-bound streaming kernel.  Algorithmic bytes per Gaussian: reads means 12, scale 12,
// rotation 16, opacity 4 (=44 B) and writes depth 4, invdepth 4, radii 4+4, means2D 8, cov3D 24,
// conic 16, rect 8, tiles 4 (=76 B); the per-frame view/proj matrices are wave-uniform.
#include "preprocess_dev.h"

namespace gsr {

__global__ __launch_bounds__(kScanBlock) void k_preprocess(Dims d, Inputs in, GeomArena g, Outputs o) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    const int64_t gid = (int64_t)b * d.P + i;
    // the frame's depth-bucket counters start at zero (first read by k_bucket_count, after
    // k_frame_totals): zeroed here instead of by a separate memset launch
    for (int k = i; k <= d.NB; k += d.nblk * kScanBlock) g.bstart[(int64_t)b * (d.NB + 1) + k] = 0u;
    uint32_t tiles = 0;
    if (i < d.P) {
        const float* pm = in.means3D + in.s_means * b + 3 * (int64_t)i;
        const float p[3] = {pm[0], pm[1], pm[2]};
        const float* cp = in.cov3D_pre ? in.cov3D_pre + in.s_cov * b + 6 * (int64_t)i : nullptr;
        float sc[3] = {0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
        if (!cp) {
            const float* sp = in.scales + in.s_scales * b + 3 * (int64_t)i;
            const float* rp = in.rot + in.s_rot * b + 4 * (int64_t)i;
            sc[0] = sp[0]; sc[1] = sp[1]; sc[2] = sp[2];
            q[0] = rp[0]; q[1] = rp[1]; q[2] = rp[2]; q[3] = rp[3];
        }
        tiles = preprocess_one(d, in, g, o, b, gid, p, cp, sc, q, in.opac[in.s_opac * b + i]);
    }
    zero_ctrl_words(d, in, g);
    preprocess_block_sums(d, g, b, blockIdx.x, tiles, gid);
}

void launch_preprocess(const Dims& d, const Inputs& in, const GeomArena& g, const Outputs& o,
                       hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    dim3 grid(d.nblk, d.B);
    hipLaunchKernelGGL(k_preprocess, grid, dim3(kScanBlock), 0, s, d, in, g, o);
}

// checkFrustum (rasterizer_impl.cu:54-66)
__global__ void k_mark_visible(int P, const float* __restrict__ means3D, const float* view,
                               const float* proj, uint8_t* present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float p[3] = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
    float ph[4];
    xform4x4(p, proj, ph);
    float pv[3];
    xform4x3(p, view, pv);
    present[i] = (pv[2] <= 0.2f) ? 0 : 1;
}

void launch_mark_visible(int P, const float* means3D, const float* view, const float* proj,
                         uint8_t* present, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, proj,
                       present);
}

}  // namespace gsr
