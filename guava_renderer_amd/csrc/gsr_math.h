// gsr_math.h -- device-side arithmetic shared by the gfx950 kernels.
//
// Every expression follows the evaluation-order contract of DESIGN.md ("Numerics contract"):
// the library is compiled with -ffp-contract=off, so a*b+c is two roundings unless written as
// fmaf().  The preprocess restates forward.cu:74-269 / auxiliary.h:40-176 of the reference
// (submodules/diff-gaussian-rasterization-32) in glm's summation order; the blend uses the
// fused form of the Gaussian exponent and blend_parts() for a bit-reproducible exp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GSR_C 32
#define GSR_BX 16
#define GSR_BY 16
#define GSR_TILE_PIX (GSR_BX * GSR_BY)

namespace gsr {

// float -> int32 as CUDA cvt.rzi.s32.f32: truncate, saturate, NaN -> 0.
__device__ __forceinline__ int f2i(float v) {
    if (v != v) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

// Deterministic exp: same op sequence as gsro_expf (oracle/gsr_oracle.c).
__device__ __forceinline__ float expf_exact(float x) {
    float xc = fmaxf(x, -87.0f);
    xc = fminf(xc, 88.0f);
    float k = rintf(xc * 1.44269504088896341f);
    float r = fmaf(k, -0.693359375f, xc);
    r = fmaf(k, 2.12194440e-4f, r);
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    float r2 = r * r;
    p = fmaf(p, r2, r);
    p = p + 1.0f;
    int ki = (int)k;
    const float r_ = p * __uint_as_float((uint32_t)(ki + 127) << 23);
    return (x != x) ? x : r_;  // NaN passes through (select, no branch)
}

// The blend's exp, split as exp(x) = 2^k (1 + q) (the same op sequence as gsro_blend_parts in
// oracle/gsr_oracle.c): k = rint(x log2e), r = x - k ln2 in one fma (|k| <= 8 wherever alpha can
// reach 1/255, so the single-constant reduction is exact to 2e-8 there), q = r + r^2 P(r) with a
// degree-4 minimax P on [-ln2/2, ln2/2] (exp within 0.97 ulp on [-5.6, 0]).  The opacity is folded
// into the power-of-two scale, alpha = fma(o 2^k, q, o 2^k): one rounding instead of o * exp(x)'s
// two (1.2 ulp from o exp(x) vs 1.8), and two VALU fewer per (pixel, Gaussian) pair than the
// seven-coefficient exp followed by the opacity multiply.
__device__ __forceinline__ void blend_parts(float x, float& q, int& k) {
    const float kf = rintf(x * 1.44269504088896341f);
    const float r = fmaf(kf, -0.693147182464599609375f, x);
    float p = 1.3814539415761828e-3f;
    p = fmaf(p, r, 8.36874544620514e-3f);
    p = fmaf(p, r, 4.166838899254799e-2f);
    p = fmaf(p, r, 1.666652113199234e-1f);
    p = fmaf(p, r, 4.999999403953552e-1f);
    q = fmaf(p, r * r, r);
    k = (int)kf;  // v_cvt_i32_f32: NaN -> 0 (q is then NaN, so alpha is too)
}
// alpha before the 0.99 clamp: o exp(x) for x in [-87, 0]
__device__ __forceinline__ float blend_oexp(float o, float q, int k) {
    const float s = __builtin_amdgcn_ldexpf(o, k);
    return fmaf(s, q, s);
}
// exp(x) itself (the backward's G)
__device__ __forceinline__ float blend_G(float q, int k) {
    return __builtin_amdgcn_ldexpf(q + 1.0f, k);
}

// Hardware exp2 path (v_exp_f32), used in "fast" mode.
__device__ __forceinline__ float expf_fast(float x) {
    return __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
}

// glm mat3, column-major m[col][row].
struct mat3 { float m[3][3]; };

__device__ __forceinline__ mat3 mk3(float a0, float a1, float a2, float a3, float a4, float a5,
                                    float a6, float a7, float a8) {
    mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
// glm operator*(mat3, mat3): Result[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2]
__device__ __forceinline__ mat3 mul3(const mat3& A, const mat3& B) {
    mat3 o;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++)
            o.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return o;
}
__device__ __forceinline__ mat3 tr3(const mat3& A) {
    mat3 o;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 3; r++) o.m[c][r] = A.m[r][c];
    return o;
}

// auxiliary.h:69-99 (column-major 4x4, row-vector convention)
__device__ __forceinline__ void xform4x3(const float p[3], const float* m, float o[3]) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
__device__ __forceinline__ void xform4x4(const float p[3], const float* m, float o[4]) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}
// auxiliary.h:111-119
__device__ __forceinline__ void xformvec_t(const float p[3], const float* m, float o[3]) {
    o[0] = m[0] * p[0] + m[1] * p[1] + m[2] * p[2];
    o[1] = m[4] * p[0] + m[5] * p[1] + m[6] * p[2];
    o[2] = m[8] * p[0] + m[9] * p[1] + m[10] * p[2];
}

// auxiliary.h:40-43: computed in double, rounded to float on return.
__device__ __forceinline__ float ndc2pix(float v, int S) {
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

// auxiliary.h:45-55 getRect(float2 p, int max_radius, ...)
__device__ __forceinline__ void get_rect(float px, float py, int r, int gx, int gy, uint32_t rmin[2],
                                         uint32_t rmax[2]) {
    const float rf = (float)r;
    int a;
    a = f2i((px - rf) / (float)GSR_BX); a = a > 0 ? a : 0; rmin[0] = min((uint32_t)a, (uint32_t)gx);
    a = f2i((py - rf) / (float)GSR_BY); a = a > 0 ? a : 0; rmin[1] = min((uint32_t)a, (uint32_t)gy);
    a = f2i((((px + rf) + (float)GSR_BX) - 1.0f) / (float)GSR_BX); a = a > 0 ? a : 0;
    rmax[0] = min((uint32_t)a, (uint32_t)gx);
    a = f2i((((py + rf) + (float)GSR_BY) - 1.0f) / (float)GSR_BY); a = a > 0 ? a : 0;
    rmax[1] = min((uint32_t)a, (uint32_t)gy);
}

// ---- split-bf16 operands (render_fwd colour accumulation, render_bwd contractions) ----
// x = x_hi + x_lo with x_hi = bf16_rne(x), x_lo = bf16_rne(x - x_hi): |x - x_hi - x_lo| <= 2^-17 |x|,
// and every product of two such halves is exact in f32.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float float2x __attribute__((ext_vector_type(2)));
// v_cvt_pk_bf16_f32 (round to nearest even) of (x, y), x in the low half
__device__ __forceinline__ unsigned cvt_pk_bf16(float x, float y) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector((float2x){x, y}, bf16x2));
}
// (hi, lo) packed low|high: hi = bf16(f), lo = bf16(f - hi)
__device__ __forceinline__ unsigned split_hl(float f) {
    const float hf = __uint_as_float(cvt_pk_bf16(f, f) << 16);
    return cvt_pk_bf16(hf, f - hf);
}
// (hi, hi) and (lo, lo)
__device__ __forceinline__ void split_hh_ll(float w, unsigned& hh, unsigned& ll) {
    hh = cvt_pk_bf16(w, w);
    const float r = w - __uint_as_float(hh << 16);
    ll = cvt_pk_bf16(r, r);
}

// Gaussian exponent of the blend (fused form; A=-cx/2, Bb=-cy, Cq=-cz/2 are exact scalings).
__device__ __forceinline__ float blend_power(float A, float Bb, float Cq, float dx, float dy) {
    return fmaf(dy, fmaf(Cq, dy, Bb * dx), (A * dx) * dx);
}

}  // namespace gsr
