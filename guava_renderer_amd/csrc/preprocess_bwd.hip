// preprocess_bwd.hip -- per-Gaussian backward of the projection: computeCov2DCUDA
// (backward.cu:147-326), preprocessCUDA bwd (:398-449) and computeCov3D bwd (:330-393) of the
// reference, fused into one launch (the reference uses two).
#include "gsr_internal.h"

namespace gsr {

__device__ __forceinline__ float sqf(float x) { return x * x; }

// Gradients of Gaussian i in frame b; returns false (outputs untouched) when it was culled there.
// The per-frame outputs (mean2D, conic, cov3D, invdepth) are stored unless gr.reduce; the
// attributes' gradients come back in o_mean / o_op / o_scale / o_rot.
__device__ __forceinline__ bool preprocess_bwd_frame(const Dims& d, const Inputs& in, const GeomArena& g,
                                                     const Grads& gr, int b, int i, float o_mean[3], float& o_op,
                                                     float o_scale[3], float o_rot[4]) {
    const int64_t gid = (int64_t)b * d.P + i;
    if (!(g.radii[gid] > 0)) return false;
    const float* view = in.view + 16 * b;
    const float* proj = in.proj + 16 * b;
    const float tanx = in.tan_dev ? in.tan_dev[2 * b] : in.tanx;
    const float tany = in.tan_dev ? in.tan_dev[2 * b + 1] : in.tany;
    const float h_y = (float)d.H / (2.0f * tany);
    const float h_x = (float)d.W / (2.0f * tanx);
    const float* c3p = in.cov3D_pre ? in.cov3D_pre + in.s_cov * b + 6 * (int64_t)i : g.cov3D + 6 * gid;
    float c3[6];
#pragma unroll
    for (int k = 0; k < 6; k++) c3[k] = c3p[k];
    const float* pm = in.means3D + in.s_means * b + 3 * (int64_t)i;
    const float mean[3] = {pm[0], pm[1], pm[2]};
    // render_bwd's sums for this Gaussian (one 32-byte row), also handed to the caller's buffers
    const float4 gt0 = reinterpret_cast<const float4*>(g.gterm)[2 * gid];
    const float4 gt1 = reinterpret_cast<const float4*>(g.gterm)[2 * gid + 1];
    const float dcx = gt0.z, dcy = gt0.w, dcz = gt1.x;
    if (!gr.reduce) {
        gr.dL_dconic[4 * gid] = dcx;
        gr.dL_dconic[4 * gid + 1] = dcy;
        gr.dL_dconic[4 * gid + 3] = dcz;
        gr.dL_dmean2D[3 * gid] = gt0.x;
        gr.dL_dmean2D[3 * gid + 1] = gt0.y;
        if (gr.dL_dinvdepth_g) gr.dL_dinvdepth_g[gid] = gt1.z;
    }
    o_op = gt1.y;

    // ---- computeCov2DCUDA ----
    float t[3];
    xform4x3(mean, view, t);
    const float limx = 1.3f * tanx;
    const float limy = 1.3f * tany;
    const float txtz = t[0] / t[2];
    const float tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    const mat3 J = mk3(h_x / t[2], 0.0f, -(h_x * t[0]) / (t[2] * t[2]), 0.0f, h_y / t[2],
                       -(h_y * t[1]) / (t[2] * t[2]), 0, 0, 0);
    const mat3 Wm = mk3(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    const mat3 V = mk3(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    const mat3 Tm = mul3(Wm, J);
    const mat3 cov2D = mul3(mul3(tr3(Tm), tr3(V)), Tm);
    float c_xx = cov2D.m[0][0], c_xy = cov2D.m[0][1], c_yy = cov2D.m[1][1];
    const float h_var = 0.3f;
    float d_inside_root = 0.f;
    if (in.antialiasing) {
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
        const float h_conv = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        const float dL_dopacity_v = gt1.y;
        const float d_h_conv = dL_dopacity_v * in.opac[in.s_opac * b + i];
        o_op = dL_dopacity_v * h_conv;
        d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f : d_h_conv / (2 * h_conv);
    } else {
        c_xx += h_var;
        c_yy += h_var;
    }
    float dL_dc_xx = 0, dL_dc_xy = 0, dL_dc_yy = 0;
    if (in.antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float denom_f = d_inside_root / sqf(w * w + w * (x + y) + x * y - z * z);
        dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
        dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
        dL_dc_xy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    const float (*T)[3] = Tm.m;
    float dcov[6];
    if (denom2inv != 0) {
        dL_dc_xx += denom2inv * (-c_yy * c_yy * dcx + 2 * c_xy * c_yy * dcy + (denom - c_xx * c_yy) * dcz);
        dL_dc_yy += denom2inv * (-c_xx * c_xx * dcz + 2 * c_xx * c_xy * dcy + (denom - c_xx * c_yy) * dcx);
        dL_dc_xy += denom2inv * 2 * (c_xy * c_yy * dcx - (denom + 2 * c_xy * c_xy) * dcy + c_xx * c_xy * dcz);
        dcov[0] = (T[0][0] * T[0][0] * dL_dc_xx + T[0][0] * T[1][0] * dL_dc_xy + T[1][0] * T[1][0] * dL_dc_yy);
        dcov[3] = (T[0][1] * T[0][1] * dL_dc_xx + T[0][1] * T[1][1] * dL_dc_xy + T[1][1] * T[1][1] * dL_dc_yy);
        dcov[5] = (T[0][2] * T[0][2] * dL_dc_xx + T[0][2] * T[1][2] * dL_dc_xy + T[1][2] * T[1][2] * dL_dc_yy);
        dcov[1] = 2 * T[0][0] * T[0][1] * dL_dc_xx + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_dc_xy + 2 * T[1][0] * T[1][1] * dL_dc_yy;
        dcov[2] = 2 * T[0][0] * T[0][2] * dL_dc_xx + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_dc_xy + 2 * T[1][0] * T[1][2] * dL_dc_yy;
        dcov[4] = 2 * T[0][2] * T[0][1] * dL_dc_xx + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_dc_xy + 2 * T[1][1] * T[1][2] * dL_dc_yy;
    } else {
#pragma unroll
        for (int k = 0; k < 6; k++) dcov[k] = 0;
    }
    if (!gr.reduce)
#pragma unroll
        for (int k = 0; k < 6; k++) gr.dL_dcov3D[6 * gid + k] = dcov[k];
    const float (*Vr)[3] = V.m;
    const float dL_dT00 = 2 * (T[0][0] * Vr[0][0] + T[0][1] * Vr[0][1] + T[0][2] * Vr[0][2]) * dL_dc_xx +
                          (T[1][0] * Vr[0][0] + T[1][1] * Vr[0][1] + T[1][2] * Vr[0][2]) * dL_dc_xy;
    const float dL_dT01 = 2 * (T[0][0] * Vr[1][0] + T[0][1] * Vr[1][1] + T[0][2] * Vr[1][2]) * dL_dc_xx +
                          (T[1][0] * Vr[1][0] + T[1][1] * Vr[1][1] + T[1][2] * Vr[1][2]) * dL_dc_xy;
    const float dL_dT02 = 2 * (T[0][0] * Vr[2][0] + T[0][1] * Vr[2][1] + T[0][2] * Vr[2][2]) * dL_dc_xx +
                          (T[1][0] * Vr[2][0] + T[1][1] * Vr[2][1] + T[1][2] * Vr[2][2]) * dL_dc_xy;
    const float dL_dT10 = 2 * (T[1][0] * Vr[0][0] + T[1][1] * Vr[0][1] + T[1][2] * Vr[0][2]) * dL_dc_yy +
                          (T[0][0] * Vr[0][0] + T[0][1] * Vr[0][1] + T[0][2] * Vr[0][2]) * dL_dc_xy;
    const float dL_dT11 = 2 * (T[1][0] * Vr[1][0] + T[1][1] * Vr[1][1] + T[1][2] * Vr[1][2]) * dL_dc_yy +
                          (T[0][0] * Vr[1][0] + T[0][1] * Vr[1][1] + T[0][2] * Vr[1][2]) * dL_dc_xy;
    const float dL_dT12 = 2 * (T[1][0] * Vr[2][0] + T[1][1] * Vr[2][1] + T[1][2] * Vr[2][2]) * dL_dc_yy +
                          (T[0][0] * Vr[2][0] + T[0][1] * Vr[2][1] + T[0][2] * Vr[2][2]) * dL_dc_xy;
    const float (*Wr)[3] = Wm.m;
    const float dL_dJ00 = Wr[0][0] * dL_dT00 + Wr[0][1] * dL_dT01 + Wr[0][2] * dL_dT02;
    const float dL_dJ02 = Wr[2][0] * dL_dT00 + Wr[2][1] * dL_dT01 + Wr[2][2] * dL_dT02;
    const float dL_dJ11 = Wr[1][0] * dL_dT10 + Wr[1][1] * dL_dT11 + Wr[1][2] * dL_dT12;
    const float dL_dJ12 = Wr[2][0] * dL_dT10 + Wr[2][1] * dL_dT11 + Wr[2][2] * dL_dT12;
    const float tz = 1.f / t[2];
    const float tz2 = tz * tz;
    const float tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t[0]) * tz3 * dL_dJ02 +
                   (2 * h_y * t[1]) * tz3 * dL_dJ12;
    if (gr.invd) dL_dtz -= gt1.z / (t[2] * t[2]);
    const float dt[3] = {dL_dtx, dL_dty, dL_dtz};
    float dm[3];
    xformvec_t(dt, view, dm);

    // ---- preprocessCUDA bwd: mean2D -> mean3D ----
    float mh[4];
    xform4x4(mean, proj, mh);
    const float m_w = 1.0f / (mh[3] + 0.0000001f);
    const float mul1 = (proj[0] * mean[0] + proj[4] * mean[1] + proj[8] * mean[2] + proj[12]) * m_w * m_w;
    const float mul2 = (proj[1] * mean[0] + proj[5] * mean[1] + proj[9] * mean[2] + proj[13]) * m_w * m_w;
    const float d2x = gt0.x, d2y = gt0.y;
    dm[0] += (proj[0] * m_w - proj[3] * mul1) * d2x + (proj[1] * m_w - proj[3] * mul2) * d2y;
    dm[1] += (proj[4] * m_w - proj[7] * mul1) * d2x + (proj[5] * m_w - proj[7] * mul2) * d2y;
    dm[2] += (proj[8] * m_w - proj[11] * mul1) * d2x + (proj[9] * m_w - proj[11] * mul2) * d2y;
    o_mean[0] = dm[0];
    o_mean[1] = dm[1];
    o_mean[2] = dm[2];

    // ---- computeCov3D bwd ----
    if (in.scales && in.rot && gr.dL_dscale && gr.dL_drot) {
        const float* q = in.rot + in.s_rot * b + 4 * (int64_t)i;
        const float r = q[0], x = q[1], y = q[2], z = q[3];
        const mat3 R = mk3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                           2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                           2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
        mat3 S = mk3(1, 0, 0, 0, 1, 0, 0, 0, 1);
        const float* sc = in.scales + in.s_scales * b + 3 * (int64_t)i;
        const float s[3] = {in.scale_mod * sc[0], in.scale_mod * sc[1], in.scale_mod * sc[2]};
        S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
        const mat3 M = mul3(S, R);
        const mat3 dSig = mk3(dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                              0.5f * dcov[2], 0.5f * dcov[4], dcov[5]);
        mat3 M2;
#pragma unroll
        for (int c = 0; c < 3; c++)
#pragma unroll
            for (int rr = 0; rr < 3; rr++) M2.m[c][rr] = 2.0f * M.m[c][rr];
        const mat3 dM = mul3(M2, dSig);
        const mat3 Rt = tr3(R);
        mat3 dMt = tr3(dM);
#pragma unroll
        for (int k = 0; k < 3; k++)
            o_scale[k] = Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1] + Rt.m[k][2] * dMt.m[k][2];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int rr = 0; rr < 3; rr++) dMt.m[k][rr] *= s[k];
        const float (*D)[3] = dMt.m;
        o_rot[0] = 2 * z * (D[0][1] - D[1][0]) + 2 * y * (D[2][0] - D[0][2]) + 2 * x * (D[1][2] - D[2][1]);
        o_rot[1] = 2 * y * (D[1][0] + D[0][1]) + 2 * z * (D[2][0] + D[0][2]) + 2 * r * (D[1][2] - D[2][1]) - 4 * x * (D[2][2] + D[1][1]);
        o_rot[2] = 2 * x * (D[1][0] + D[0][1]) + 2 * r * (D[2][0] - D[0][2]) + 2 * z * (D[1][2] + D[2][1]) - 4 * y * (D[2][2] + D[0][0]);
        o_rot[3] = 2 * r * (D[0][1] - D[1][0]) + 2 * x * (D[2][0] + D[0][2]) + 2 * y * (D[1][2] + D[2][1]) - 4 * z * (D[1][1] + D[0][0]);
    }
    return true;
}

// Per-frame mode: one thread per (Gaussian, frame), every output per frame.  Frame-reduced mode
// (gr.reduce, the shared attributes of a training batch): one thread per Gaussian sums its frames in
// frame order and writes each attribute gradient once -- no [B][P][k] buffers and no separate sum.
__global__ __launch_bounds__(kScanBlock) void k_preprocess_bwd(Dims d, Inputs in, GeomArena g, Grads gr) {
    const int i = blockIdx.x * kScanBlock + threadIdx.x;
    if (i >= d.P || g.ctrl[kCtrlFwdOnly]) return;  // (a GSR_FORWARD_ONLY workspace: no backward rows)
    const bool geo = in.scales && in.rot && gr.dL_dscale && gr.dL_drot;
    if (!gr.reduce) {
        const int b = blockIdx.y;
        const int64_t gid = (int64_t)b * d.P + i;
        float m[3], sc[3], r[4], op;
        if (!preprocess_bwd_frame(d, in, g, gr, b, i, m, op, sc, r)) return;
        gr.dL_dopacity[gid] = op;
#pragma unroll
        for (int k = 0; k < 3; k++) gr.dL_dmeans3D[3 * gid + k] = m[k];
        if (geo) {
#pragma unroll
            for (int k = 0; k < 3; k++) gr.dL_dscale[3 * gid + k] = sc[k];
#pragma unroll
            for (int k = 0; k < 4; k++) gr.dL_drot[4 * gid + k] = r[k];
        }
        return;
    }
    float am[3] = {0.f, 0.f, 0.f}, as[3] = {0.f, 0.f, 0.f}, ar[4] = {0.f, 0.f, 0.f, 0.f}, aop = 0.f;
    for (int b = 0; b < d.B; b++) {
        float m[3], sc[3] = {0.f, 0.f, 0.f}, r[4] = {0.f, 0.f, 0.f, 0.f}, op;
        if (!preprocess_bwd_frame(d, in, g, gr, b, i, m, op, sc, r)) continue;
        aop += op;
#pragma unroll
        for (int k = 0; k < 3; k++) { am[k] += m[k]; as[k] += sc[k]; }
#pragma unroll
        for (int k = 0; k < 4; k++) ar[k] += r[k];
    }
    gr.dL_dopacity[i] = aop;
#pragma unroll
    for (int k = 0; k < 3; k++) gr.dL_dmeans3D[3 * (int64_t)i + k] = am[k];
    if (geo) {
#pragma unroll
        for (int k = 0; k < 3; k++) gr.dL_dscale[3 * (int64_t)i + k] = as[k];
#pragma unroll
        for (int k = 0; k < 4; k++) gr.dL_drot[4 * (int64_t)i + k] = ar[k];
    }
}

void launch_preprocess_bwd(const Dims& d, const Inputs& in, const GeomArena& g, const Grads& gr,
                           hipStream_t s) {
    if (d.P == 0 || d.B == 0) return;
    hipLaunchKernelGGL(k_preprocess_bwd, dim3(d.nblk, gr.reduce ? 1 : d.B), dim3(kScanBlock), 0, s, d, in, g, gr);
}

}  // namespace gsr
