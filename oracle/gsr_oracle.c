/*
 * gsr_oracle.c -- CPU restatement of diff-gaussian-rasterization-32 (TEST INFRASTRUCTURE ONLY).
 * See gsr_oracle.h for scope, citations and the evaluation-order contract.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp).
 */
#include "gsr_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define C GSRO_C
#define BX GSRO_BX
#define BY GSRO_BY

static int g_threads = 0;
void gsro_set_threads(int n) { g_threads = n; }
int gsro_get_threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}

/* float -> int32 with CUDA cvt.rzi.s32.f32 semantics (truncate, saturate, NaN -> 0). */
static inline int f2i(float v) {
    if (v != v) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* Deterministic exp (Cody-Waite reduction + Cephes-style degree-6 polynomial), identical
 * operation sequence in guava_renderer_amd/csrc/gsr_math.h. Used for the blend only. */
float gsro_expf(float x) {
    if (x != x) return x;
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
    return p * bitsf((uint32_t)(ki + 127) << 23);
}

/* The blend's alpha = min(0.99, o * exp(power)) (forward.cu:361, backward.cu:529-531), with exp
 * split as 2^k (1 + q) and the opacity folded into the power-of-two scale -- the op sequence of
 * blend_parts / blend_oexp / blend_G in guava_renderer_amd/csrc/gsr_math.h, so the GPU's alphas are
 * bit-identical.  k = rint(x log2e), r = x - k ln2 (one fma), q = r + r^2 P(r) with a degree-4
 * minimax P on [-ln2/2, ln2/2]; alpha = fma(o 2^k, q, o 2^k).  Accuracy: exp within 0.97 ulp and
 * o exp(x) within 1.2 ulp on [-5.6, 0] (alpha >= 1/255 needs x > -5.54); libm-free.
 * power < -87 never blends (alpha 0, as exp(-87) * o < 1/255); a NaN power gives alpha 0.99. */
static inline void blend_parts(float x, float* q, int* k) {
    const float kf = rintf(x * 1.44269504088896341f);
    const float r = fmaf(kf, -0.693147182464599609375f, x);
    float p = 1.3814539415761828e-3f;
    p = fmaf(p, r, 8.36874544620514e-3f);
    p = fmaf(p, r, 4.166838899254799e-2f);
    p = fmaf(p, r, 1.666652113199234e-1f);
    p = fmaf(p, r, 4.999999403953552e-1f);
    *q = fmaf(p, r * r, r);
    *k = (kf == kf) ? (int)kf : 0; /* v_cvt_i32_f32 gives 0 for NaN; |kf| <= 126 otherwise */
}
/* Blend arithmetic modes (the `exact_exp` argument of the render functions):
 *   1 GSRO_RESTATED  -- the restatement the GPU reproduces bit for bit: fused power, blend_parts exp,
 *                       C = fmaf(f, alpha T, C);
 *   0 GSRO_LIBM_EXP  -- the same arithmetic with libm expf (the reference's exp, forward.cu:360);
 *   2 GSRO_LITERAL   -- the reference's expressions as written, every product and sum rounded
 *                       (C semantics; nvcc may contract some into fma, which this container cannot
 *                       reproduce): power = -0.5f * (a dx dx + c dy dy) - b dx dy (forward.cu:352,
 *                       backward.cu:564), alpha = min(0.99f, o expf(power)) (:360), C += f alpha T
 *                       (:372), invdepth += (1 / depth) alpha T (:375), out = C + T bg (:391). */
float gsro_blend_alpha(float o, float x, int exact) {
    if (exact != 1) return fminf(0.99f, o * expf(x));
    if (x < -87.0f) return 0.0f;
    float q;
    int k;
    blend_parts(x, &q, &k);
    const float s = ldexpf(o, k);
    return fminf(0.99f, fmaf(s, q, s));
}
/* exp(x) = 2^k (1 + q) for the backward's dL/dopacity and dL/dG terms */
float gsro_blend_G(float x, int exact) {
    if (exact != 1) return expf(x);
    if (x < -87.0f) x = -87.0f; /* never used there (alpha is 0); keeps k in range */
    float q;
    int k;
    blend_parts(x, &q, &k);
    return ldexpf(q + 1.0f, k);
}

/* ---- glm-order helpers (glm mat3 is column-major: m[col][row]) ---- */
typedef struct { float m[3][3]; } mat3;

/* glm::mat3(a0..a8): columns (a0,a1,a2), (a3,a4,a5), (a6,a7,a8) */
static inline mat3 mk3(float a0, float a1, float a2, float a3, float a4, float a5,
                       float a6, float a7, float a8) {
    mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
/* glm type_mat3x3.inl:486-519: Result[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2] */
static inline mat3 mul3(mat3 A, mat3 B) {
    mat3 o;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++)
            o.m[c][r] = A.m[0][r] * B.m[c][0] + A.m[1][r] * B.m[c][1] + A.m[2][r] * B.m[c][2];
    return o;
}
static inline mat3 tr3(mat3 A) {
    mat3 o;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) o.m[c][r] = A.m[r][c];
    return o;
}

/* auxiliary.h:69-99 */
static inline void xform4x3(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static inline void xform4x4(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}
/* auxiliary.h:111-119 */
static inline void xformvec_t(const float* p, const float* m, float* o) {
    o[0] = m[0] * p[0] + m[1] * p[1] + m[2] * p[2];
    o[1] = m[4] * p[0] + m[5] * p[1] + m[6] * p[2];
    o[2] = m[8] * p[0] + m[9] * p[1] + m[10] * p[2];
}

/* auxiliary.h:40-43 (double arithmetic, converted to float on return) */
static inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

/* auxiliary.h:45-55 getRect(float2, int, ...) */
static inline void get_rect(float px, float py, int r, int gx, int gy, unsigned rmin[2], unsigned rmax[2]) {
    float rf = (float)r;
    int a;
    a = f2i((px - rf) / (float)BX); a = a > 0 ? a : 0; rmin[0] = (unsigned)a < (unsigned)gx ? (unsigned)a : (unsigned)gx;
    a = f2i((py - rf) / (float)BY); a = a > 0 ? a : 0; rmin[1] = (unsigned)a < (unsigned)gy ? (unsigned)a : (unsigned)gy;
    a = f2i((((px + rf) + (float)BX) - 1.0f) / (float)BX); a = a > 0 ? a : 0; rmax[0] = (unsigned)a < (unsigned)gx ? (unsigned)a : (unsigned)gx;
    a = f2i((((py + rf) + (float)BY) - 1.0f) / (float)BY); a = a > 0 ? a : 0; rmax[1] = (unsigned)a < (unsigned)gy ? (unsigned)a : (unsigned)gy;
}

/* auxiliary.h:151-176 */
static inline int in_frustum(const float* p, const float* view, const float* proj, float* p_view) {
    float ph[4];
    xform4x4(p, proj, ph);
    float pw = 1.0f / (ph[3] + 0.0000001f);
    (void)pw; /* p_proj is computed and unused by the test (lateral cull commented out) */
    xform4x3(p, view, p_view);
    return !(p_view[2] <= 0.2f);
}

void gsro_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present) {
    for (int i = 0; i < P; i++) {
        float pv[3];
        present[i] = (uint8_t)in_frustum(means3D + 3 * i, view, proj, pv);
    }
}

/* forward.cu:114-148 */
static void cov3d_fwd(const float* s, float mod, const float* q, float* cov) {
    mat3 S = mk3(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * s[0];
    S.m[1][1] = mod * s[1];
    S.m[2][2] = mod * s[2];
    float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = mk3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                 2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                 2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 M = mul3(S, R);
    mat3 Sig = mul3(tr3(M), M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

/* forward.cu:74-109 (T, J, W returned for reuse by the backward restatement) */
static void cov2d_core(const float* mean, float fx, float fy, float tanx, float tany, const float* cov3D,
                       const float* view, float* t_out, float* txtz_out, float* tytz_out, float* limx_out,
                       float* limy_out, mat3* Tm, mat3* Wm, mat3* Vrk, mat3* cov) {
    float t[3];
    xform4x3(mean, view, t);
    const float limx = 1.3f * tanx;
    const float limy = 1.3f * tany;
    const float txtz = t[0] / t[2];
    const float tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    mat3 J = mk3(fx / t[2], 0.0f, -(fx * t[0]) / (t[2] * t[2]),
                 0.0f, fy / t[2], -(fy * t[1]) / (t[2] * t[2]),
                 0, 0, 0);
    mat3 W = mk3(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    mat3 T = mul3(W, J);
    mat3 V = mk3(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 cv = mul3(mul3(tr3(T), tr3(V)), T);
    if (t_out) { t_out[0] = t[0]; t_out[1] = t[1]; t_out[2] = t[2]; }
    if (txtz_out) *txtz_out = txtz;
    if (tytz_out) *tytz_out = tytz;
    if (limx_out) *limx_out = limx;
    if (limy_out) *limy_out = limy;
    if (Tm) *Tm = T;
    if (Wm) *Wm = W;
    if (Vrk) *Vrk = V;
    *cov = cv;
}

int gsro_preprocess(int P, const float* means3D, const float* scales, float scale_mod,
                    const float* rot, const float* opac, const float* cov3D_precomp,
                    const float* view, const float* proj, int W, int H,
                    float tanx, float tany, int prefiltered, int antialiasing,
                    int* radii, float* means2D, float* depths, float* cov3D,
                    float* conic_opacity, uint32_t* tiles_touched) {
    /* rasterizer_impl.cu:224-225 */
    const float focal_y = H / (2.0f * tany);
    const float focal_x = W / (2.0f * tanx);
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    int err = 0;
#pragma omp parallel for schedule(static) num_threads(gsro_get_threads()) reduction(| : err)
    for (int idx = 0; idx < P; idx++) {
        radii[idx] = 0;
        tiles_touched[idx] = 0;
        depths[idx] = 0.f;
        means2D[2 * idx] = means2D[2 * idx + 1] = 0.f;
        for (int k = 0; k < 4; k++) conic_opacity[4 * idx + k] = 0.f;
        if (!cov3D_precomp)
            for (int k = 0; k < 6; k++) cov3D[6 * idx + k] = 0.f;
        const float* p = means3D + 3 * idx;
        float p_view[3];
        if (!in_frustum(p, view, proj, p_view)) {
            if (prefiltered) err |= 1;
            continue;
        }
        float ph[4];
        xform4x4(p, proj, ph);
        float pw = 1.0f / (ph[3] + 0.0000001f);
        float pproj[3] = {ph[0] * pw, ph[1] * pw, ph[2] * pw};
        const float* c3;
        if (cov3D_precomp) {
            c3 = cov3D_precomp + 6 * idx;
        } else {
            cov3d_fwd(scales + 3 * idx, scale_mod, rot + 4 * idx, cov3D + 6 * idx);
            c3 = cov3D + 6 * idx;
        }
        mat3 cv;
        cov2d_core(p, focal_x, focal_y, tanx, tany, c3, view, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, &cv);
        float cx = cv.m[0][0], cy = cv.m[0][1], cz = cv.m[1][1];
        const float h_var = 0.3f;
        const float det_cov = cx * cz - cy * cy;
        cx += h_var;
        cz += h_var;
        const float det_cov_plus_h_cov = cx * cz - cy * cy;
        float h_conv = 1.0f;
        if (antialiasing) h_conv = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
        const float det = det_cov_plus_h_cov;
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cz * det_inv, -cy * det_inv, cx * det_inv};
        float mid = 0.5f * (cx + cz);
        float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        float pix[2] = {ndc2pix(pproj[0], W), ndc2pix(pproj[1], H)};
        unsigned rmin[2], rmax[2];
        get_rect(pix[0], pix[1], f2i(my_radius), gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        depths[idx] = p_view[2];
        radii[idx] = f2i(my_radius);
        means2D[2 * idx] = pix[0];
        means2D[2 * idx + 1] = pix[1];
        conic_opacity[4 * idx + 0] = conic[0];
        conic_opacity[4 * idx + 1] = conic[1];
        conic_opacity[4 * idx + 2] = conic[2];
        conic_opacity[4 * idx + 3] = opac[idx] * h_conv;
        tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
    }
    return err ? -1 : 0;
}

/* rasterizer_impl.cu:35-50 */
static uint32_t get_higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

int64_t gsro_bin(int P, int W, int H, const int* radii, const float* means2D, const float* depths,
                 const uint32_t* tiles_touched, uint32_t* point_offsets,
                 uint32_t* point_list, uint64_t* point_keys, uint32_t* ranges, int64_t R_cap) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const int T = gx * gy;
    /* InclusiveSum (rasterizer_impl.cu:280) */
    uint64_t acc = 0;
    for (int i = 0; i < P; i++) { acc += tiles_touched[i]; point_offsets[i] = (uint32_t)acc; }
    int64_t R = (int64_t)acc;
    memset(ranges, 0, sizeof(uint32_t) * 2 * (size_t)T);
    if (R > R_cap) return -R;
    if (R == 0) return 0;
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)R);
    uint32_t* vals = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)R);
    /* duplicateWithKeys (rasterizer_impl.cu:70-111) */
    for (int idx = 0; idx < P; idx++) {
        if (radii[idx] > 0) {
            uint32_t off = (idx == 0) ? 0 : point_offsets[idx - 1];
            unsigned rmin[2], rmax[2];
            get_rect(means2D[2 * idx], means2D[2 * idx + 1], radii[idx], gx, gy, rmin, rmax);
            for (unsigned y = rmin[1]; y < rmax[1]; y++)
                for (unsigned x = rmin[0]; x < rmax[0]; x++) {
                    uint64_t key = (uint64_t)(y * (unsigned)gx + x);
                    key <<= 32;
                    key |= fbits(depths[idx]);
                    keys[off] = key;
                    vals[off] = (uint32_t)idx;
                    off++;
                }
        }
    }
    /* cub::DeviceRadixSort::SortPairs over bits [0, 32+bit): stable LSD radix, 8-bit digits
     * (rasterizer_impl.cu:303-311). */
    int endbit = 32 + (int)get_higher_msb((uint32_t)T);
    uint64_t* k2 = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)R);
    uint32_t* v2 = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)R);
    for (int shift = 0; shift < endbit; shift += 8) {
        size_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        uint64_t mask = 0xFFull;
        int nb = endbit - shift < 8 ? endbit - shift : 8;
        mask = (1ull << nb) - 1ull;
        for (int64_t i = 0; i < R; i++) cnt[((keys[i] >> shift) & mask) + 1]++;
        for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
        for (int64_t i = 0; i < R; i++) {
            size_t d = (size_t)((keys[i] >> shift) & mask);
            size_t pos = cnt[d]++;
            k2[pos] = keys[i];
            v2[pos] = vals[i];
        }
        uint64_t* tk = keys; keys = k2; k2 = tk;
        uint32_t* tv = vals; vals = v2; v2 = tv;
    }
    memcpy(point_list, vals, sizeof(uint32_t) * (size_t)R);
    if (point_keys) memcpy(point_keys, keys, sizeof(uint64_t) * (size_t)R);
    /* identifyTileRanges (rasterizer_impl.cu:116-138) */
    for (int64_t idx = 0; idx < R; idx++) {
        uint32_t cur = (uint32_t)(keys[idx] >> 32);
        if (idx == 0) ranges[2 * cur] = 0;
        else {
            uint32_t prev = (uint32_t)(keys[idx - 1] >> 32);
            if (cur != prev) {
                ranges[2 * prev + 1] = (uint32_t)idx;
                ranges[2 * cur] = (uint32_t)idx;
            }
        }
        if (idx == R - 1) ranges[2 * cur + 1] = (uint32_t)R;
    }
    free(keys); free(vals); free(k2); free(v2);
    return R;
}

/* The blend's Gaussian exponent at d = (dx, dy) = xy - pixel: mode 2 as written at forward.cu:352
 * (left to right, each product rounded); else the fused form of gsr_math.h blend_power (an algebraic
 * rewrite with A = -a/2, B = -b, C = -c/2, exact scalings). */
static inline float blend_power_m(const float* co, float dx, float dy, int mode) {
    if (mode == 2) return -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
    const float A = -0.5f * co[0], Bb = -co[1], Cq = -0.5f * co[2];
    return fmaf(dy, fmaf(Cq, dy, Bb * dx), (A * dx) * dx);
}

void gsro_render(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                 const float* means2D, const float* colors, const float* conic_opacity,
                 const float* depths, const float* bg, int exact_exp,
                 float* out_color, float* out_invdepth, float* final_T, uint32_t* n_contrib) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const int T = gx * gy;
    const size_t HW = (size_t)H * (size_t)W;
#pragma omp parallel for schedule(dynamic, 1) num_threads(gsro_get_threads())
    for (int tile = 0; tile < T; tile++) {
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t start = ranges[2 * tile], end = ranges[2 * tile + 1];
        for (int ly = 0; ly < BY; ly++)
            for (int lx = 0; lx < BX; lx++) {
                const int x = tx * BX + lx, y = ty * BY + ly;
                if (x >= W || y >= H) continue;
                const size_t pix = (size_t)W * (size_t)y + (size_t)x;
                const float pfx = (float)x, pfy = (float)y;
                float Tr = 1.0f;
                uint32_t contributor = 0, last = 0;
                float Cc[C];
                for (int ch = 0; ch < C; ch++) Cc[ch] = 0.f;
                float invd = 0.f;
                for (uint32_t j = start; j < end; j++) {
                    contributor++;
                    const uint32_t g = point_list[j];
                    const float* co = conic_opacity + 4 * (size_t)g;
                    const float dx = means2D[2 * (size_t)g] - pfx;
                    const float dy = means2D[2 * (size_t)g + 1] - pfy;
                    const float power = blend_power_m(co, dx, dy, exact_exp);
                    if (power > 0.0f) continue;
                    const float alpha = gsro_blend_alpha(co[3], power, exact_exp);
                    if (alpha < 1.0f / 255.0f) continue;
                    const float test_T = Tr * (1.0f - alpha);
                    if (test_T < 0.0001f) break; /* done: the reference stops iterating */
                    const float* f = colors + (size_t)g * C;
                    if (exact_exp == 2) {
                        for (int ch = 0; ch < C; ch++) Cc[ch] += f[ch] * alpha * Tr;
                        invd += (1.0f / depths[g]) * alpha * Tr;
                    } else {
                        const float w = alpha * Tr;
                        for (int ch = 0; ch < C; ch++) Cc[ch] = fmaf(f[ch], w, Cc[ch]);
                        invd = fmaf(1.0f / depths[g], w, invd);
                    }
                    Tr = test_T;
                    last = contributor;
                }
                final_T[pix] = Tr;
                n_contrib[pix] = last;
                for (int ch = 0; ch < C; ch++)
                    out_color[(size_t)ch * HW + pix] = exact_exp == 2 ? Cc[ch] + Tr * bg[ch] : fmaf(Tr, bg[ch], Cc[ch]);
                if (out_invdepth) out_invdepth[pix] = invd;
            }
    }
}

/* Work counts of the per-pixel loop above (test infrastructure for gsr_render_counters):
 * out[0] = (pixel, Gaussian) pairs visited (up to and including a terminating Gaussian),
 * out[1] = pairs that contributed. */
void gsro_render_counts(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                        const float* means2D, const float* conic_opacity, int exact_exp,
                        uint64_t* out) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    uint64_t visited = 0, contrib = 0;
    for (int tile = 0; tile < gx * gy; tile++) {
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t start = ranges[2 * tile], end = ranges[2 * tile + 1];
        for (int ly = 0; ly < BY; ly++)
            for (int lx = 0; lx < BX; lx++) {
                const int x = tx * BX + lx, y = ty * BY + ly;
                if (x >= W || y >= H) continue;
                float Tr = 1.0f;
                for (uint32_t j = start; j < end; j++) {
                    visited++;
                    const uint32_t g = point_list[j];
                    const float* co = conic_opacity + 4 * (size_t)g;
                    const float dx = means2D[2 * (size_t)g] - (float)x;
                    const float dy = means2D[2 * (size_t)g + 1] - (float)y;
                    const float power = blend_power_m(co, dx, dy, exact_exp);
                    if (power > 0.0f) continue;
                    const float alpha = gsro_blend_alpha(co[3], power, exact_exp);
                    if (alpha < 1.0f / 255.0f) continue;
                    const float test_T = Tr * (1.0f - alpha);
                    if (test_T < 0.0001f) break;
                    Tr = test_T;
                    contrib++;
                }
            }
    }
    out[0] = visited;
    out[1] = contrib;
}

/* Decision flips between the two blend exps (test infrastructure): per pixel, walks the loop of
 * forward.cu:349-381 twice in lockstep -- once with the restatement's exp (exact_exp = 1), once
 * with libm expf (the nearest this container has to CUDA's expf) -- and sets flags[pix] = 1 when any
 * pair's take decision (alpha >= 1/255) or stop decision (T (1 - alpha) < 1e-4) differs.  Those are
 * the pixels where two exps a few ulp apart legitimately give different colours (SURVEY.md §7,
 * "exp() ulp differences"); everywhere else the images agree to the alphas' rounding.
 * Returns the number of flagged pixels. */
uint64_t gsro_render_decision_flips(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                                    const float* means2D, const float* conic_opacity, uint8_t* flags) {
    return gsro_render_decision_flips_modes(W, H, ranges, point_list, means2D, conic_opacity, 1, 0, flags);
}

/* The same between any two blend modes (mode_a, mode_b: 0 / 1 / 2 as gsro_render). */
uint64_t gsro_render_decision_flips_modes(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                                          const float* means2D, const float* conic_opacity, int mode_a,
                                          int mode_b, uint8_t* flags) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    uint64_t nflip = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(gsro_get_threads()) reduction(+ : nflip)
    for (int tile = 0; tile < gx * gy; tile++) {
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t start = ranges[2 * tile], end = ranges[2 * tile + 1];
        for (int ly = 0; ly < BY; ly++)
            for (int lx = 0; lx < BX; lx++) {
                const int x = tx * BX + lx, y = ty * BY + ly;
                if (x >= W || y >= H) continue;
                float T0 = 1.0f, T1 = 1.0f;
                int done0 = 0, done1 = 0, flip = 0;
                for (uint32_t j = start; j < end && !(done0 && done1) && !flip; j++) {
                    const uint32_t g = point_list[j];
                    const float* co = conic_opacity + 4 * (size_t)g;
                    const float dx = means2D[2 * (size_t)g] - (float)x;
                    const float dy = means2D[2 * (size_t)g + 1] - (float)y;
                    const float p0 = blend_power_m(co, dx, dy, mode_a), p1 = blend_power_m(co, dx, dy, mode_b);
                    const float a0 = p0 > 0.0f ? 0.0f : gsro_blend_alpha(co[3], p0, mode_a);
                    const float a1 = p1 > 0.0f ? 0.0f : gsro_blend_alpha(co[3], p1, mode_b);
                    const int take0 = !(a0 < 1.0f / 255.0f), take1 = !(a1 < 1.0f / 255.0f);
                    if (take0 != take1) { flip = 1; break; }
                    if (!take0) continue;
                    const float t0 = T0 * (1.0f - a0), t1 = T1 * (1.0f - a1);
                    const int stop0 = t0 < 0.0001f, stop1 = t1 < 0.0001f;
                    if (stop0 != stop1) { flip = 1; break; }
                    if (stop0) { done0 = done1 = 1; break; }
                    T0 = t0;
                    T1 = t1;
                }
                flags[(size_t)W * y + x] = (uint8_t)flip;
                nflip += (uint64_t)flip;
            }
    }
    return nflip;
}

/* Accumulation order of gsro_render_backward's per-Gaussian sums (test infrastructure): 0 = tiles,
 * then pixels, in increasing order; 1 = both reversed.  The reference accumulates with float atomics
 * in whatever order its threads arrive (backward.cu:593-635), so the difference between the two orders
 * is the f32 noise floor that any reassociating implementation (the GPU's included) is judged
 * against per element (tests/helpers.py grad_check). */
static int g_bwd_reverse = 0;
void gsro_set_backward_order(int reverse) { g_bwd_reverse = reverse; }

void gsro_render_backward(int W, int H, const uint32_t* ranges, const uint32_t* point_list,
                          const float* bg, const float* means2D, const float* conic_opacity,
                          const float* colors, const float* depths, const float* final_T,
                          const uint32_t* n_contrib, const float* dL_dpix,
                          const float* dL_dinvdepth_pix, int exact_exp,
                          float* dL_dmean2D, float* dL_dconic, float* dL_dopacity,
                          float* dL_dcolors, float* dL_dinvdepth_g) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const int T = gx * gy;
    const size_t HW = (size_t)H * (size_t)W;
    const float ddelx_dx = (float)(0.5 * W);
    const float ddely_dy = (float)(0.5 * H);
    const int use_invd = (dL_dinvdepth_pix != NULL && dL_dinvdepth_g != NULL);
    for (int tile_i = 0; tile_i < T; tile_i++) {
        const int tile = g_bwd_reverse ? T - 1 - tile_i : tile_i;
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t start = ranges[2 * tile], end = ranges[2 * tile + 1];
        for (int pi = 0; pi < BX * BY; pi++) {
                const int pp = g_bwd_reverse ? BX * BY - 1 - pi : pi;
                const int lx = pp % BX, ly = pp / BX;
                const int x = tx * BX + lx, y = ty * BY + ly;
                if (x >= W || y >= H) continue;
                const size_t pix = (size_t)W * (size_t)y + (size_t)x;
                const float pfx = (float)x, pfy = (float)y;
                const float T_final = final_T[pix];
                float Tr = T_final;
                uint32_t contributor = end - start;
                const uint32_t last_contributor = n_contrib[pix];
                float accum_rec[C], dL_dpixel[C], last_color[C];
                for (int ch = 0; ch < C; ch++) {
                    accum_rec[ch] = 0.f;
                    last_color[ch] = 0.f;
                    dL_dpixel[ch] = dL_dpix[(size_t)ch * HW + pix];
                }
                const float dL_invdepth = use_invd ? dL_dinvdepth_pix[pix] : 0.f;
                float accum_invdepth_rec = 0.f, last_alpha = 0.f, last_invdepth = 0.f;
                float bg_dot_dpixel = 0.f;
                for (int i = 0; i < C; i++) bg_dot_dpixel += bg[i] * dL_dpixel[i];
                for (uint32_t jj = end; jj > start; jj--) {
                    const uint32_t j = jj - 1;
                    contributor--;
                    if (contributor >= last_contributor) continue;
                    const uint32_t g = point_list[j];
                    const float* co = conic_opacity + 4 * (size_t)g;
                    const float dx = means2D[2 * (size_t)g] - pfx;
                    const float dy = means2D[2 * (size_t)g + 1] - pfy;
                    const float power = blend_power_m(co, dx, dy, exact_exp);
                    if (power > 0.0f) continue;
                    const float G = gsro_blend_G(power, exact_exp);
                    const float alpha = gsro_blend_alpha(co[3], power, exact_exp);
                    if (alpha < 1.0f / 255.0f) continue;
                    Tr = Tr / (1.f - alpha);
                    const float dchannel_dcolor = alpha * Tr;
                    float dL_dalpha = 0.0f;
                    const float* f = colors + (size_t)g * C;
                    for (int ch = 0; ch < C; ch++) {
                        const float c = f[ch];
                        accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                        last_color[ch] = c;
                        const float dL_dchannel = dL_dpixel[ch];
                        dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
                        dL_dcolors[(size_t)g * C + ch] += dchannel_dcolor * dL_dchannel;
                    }
                    if (use_invd) {
                        const float invd = 1.f / depths[g];
                        accum_invdepth_rec = last_alpha * last_invdepth + (1.f - last_alpha) * accum_invdepth_rec;
                        last_invdepth = invd;
                        dL_dalpha += (invd - accum_invdepth_rec) * dL_invdepth;
                        dL_dinvdepth_g[g] += dchannel_dcolor * dL_invdepth;
                    }
                    dL_dalpha *= Tr;
                    last_alpha = alpha;
                    dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
                    const float dL_dG = co[3] * dL_dalpha;
                    const float gdx = G * dx;
                    const float gdy = G * dy;
                    const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                    const float dG_ddely = -gdy * co[2] - gdx * co[1];
                    dL_dmean2D[3 * (size_t)g + 0] += dL_dG * dG_ddelx * ddelx_dx;
                    dL_dmean2D[3 * (size_t)g + 1] += dL_dG * dG_ddely * ddely_dy;
                    dL_dconic[4 * (size_t)g + 0] += -0.5f * gdx * dx * dL_dG;
                    dL_dconic[4 * (size_t)g + 1] += -0.5f * gdx * dy * dL_dG;
                    dL_dconic[4 * (size_t)g + 3] += -0.5f * gdy * dy * dL_dG;
                    dL_dopacity[g] += G * dL_dalpha;
                }
            }
    }
}

static inline float sq(float x) { return x * x; }

void gsro_preprocess_backward(int P, int W, int H, const float* means3D, const int* radii,
                              const float* scales, float scale_mod, const float* rot,
                              const float* opac, const float* cov3D, const float* view,
                              const float* proj, float tanx, float tany,
                              const float* dL_dmean2D, const float* dL_dconic,
                              const float* dL_dinvdepth_g, int antialiasing,
                              float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D,
                              float* dL_dscale, float* dL_drot) {
    const float h_y = H / (2.0f * tany);
    const float h_x = W / (2.0f * tanx);
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        /* ---- computeCov2DCUDA (backward.cu:147-326) ---- */
        const float* c3 = cov3D + 6 * (size_t)idx;
        const float* mean = means3D + 3 * (size_t)idx;
        const float dcx = dL_dconic[4 * (size_t)idx], dcy = dL_dconic[4 * (size_t)idx + 1],
                    dcz = dL_dconic[4 * (size_t)idx + 3];
        float t[3], txtz, tytz, limx, limy;
        mat3 Tm, Wm, V, cov2D;
        cov2d_core(mean, h_x, h_y, tanx, tany, c3, view, t, &txtz, &tytz, &limx, &limy, &Tm, &Wm, &V, &cov2D);
        const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
        const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
        float c_xx = cov2D.m[0][0], c_xy = cov2D.m[0][1], c_yy = cov2D.m[1][1];
        const float h_var = 0.3f;
        float d_inside_root = 0.f;
        if (antialiasing) {
            const float det_cov = c_xx * c_yy - c_xy * c_xy;
            c_xx += h_var;
            c_yy += h_var;
            const float det_cov_plus_h_cov = c_xx * c_yy - c_xy * c_xy;
            const float h_conv = sqrtf(fmaxf(0.000025f, det_cov / det_cov_plus_h_cov));
            const float dL_dopacity_v = dL_dopacity[idx];
            const float d_h_conv = dL_dopacity_v * opac[idx];
            dL_dopacity[idx] = dL_dopacity_v * h_conv;
            d_inside_root = (det_cov / det_cov_plus_h_cov) <= 0.000025f ? 0.f : d_h_conv / (2 * h_conv);
        } else {
            c_xx += h_var;
            c_yy += h_var;
        }
        float dL_dc_xx = 0, dL_dc_xy = 0, dL_dc_yy = 0;
        if (antialiasing) {
            const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
            const float denom_f = d_inside_root / sq(w * w + w * (x + y) + x * y - z * z);
            dL_dc_xx = w * (w * y + y * y + z * z) * denom_f;
            dL_dc_yy = w * (w * x + x * x + z * z) * denom_f;
            dL_dc_xy = -2.f * w * z * (w + x + y) * denom_f;
        }
        float denom = c_xx * c_yy - c_xy * c_xy;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float* dcov = dL_dcov3D + 6 * (size_t)idx;
        const float (*T)[3] = Tm.m;
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
            for (int i = 0; i < 6; i++) dcov[i] = 0;
        }
        const float (*Vr)[3] = V.m;
        float dL_dT00 = 2 * (T[0][0] * Vr[0][0] + T[0][1] * Vr[0][1] + T[0][2] * Vr[0][2]) * dL_dc_xx +
                        (T[1][0] * Vr[0][0] + T[1][1] * Vr[0][1] + T[1][2] * Vr[0][2]) * dL_dc_xy;
        float dL_dT01 = 2 * (T[0][0] * Vr[1][0] + T[0][1] * Vr[1][1] + T[0][2] * Vr[1][2]) * dL_dc_xx +
                        (T[1][0] * Vr[1][0] + T[1][1] * Vr[1][1] + T[1][2] * Vr[1][2]) * dL_dc_xy;
        float dL_dT02 = 2 * (T[0][0] * Vr[2][0] + T[0][1] * Vr[2][1] + T[0][2] * Vr[2][2]) * dL_dc_xx +
                        (T[1][0] * Vr[2][0] + T[1][1] * Vr[2][1] + T[1][2] * Vr[2][2]) * dL_dc_xy;
        float dL_dT10 = 2 * (T[1][0] * Vr[0][0] + T[1][1] * Vr[0][1] + T[1][2] * Vr[0][2]) * dL_dc_yy +
                        (T[0][0] * Vr[0][0] + T[0][1] * Vr[0][1] + T[0][2] * Vr[0][2]) * dL_dc_xy;
        float dL_dT11 = 2 * (T[1][0] * Vr[1][0] + T[1][1] * Vr[1][1] + T[1][2] * Vr[1][2]) * dL_dc_yy +
                        (T[0][0] * Vr[1][0] + T[0][1] * Vr[1][1] + T[0][2] * Vr[1][2]) * dL_dc_xy;
        float dL_dT12 = 2 * (T[1][0] * Vr[2][0] + T[1][1] * Vr[2][1] + T[1][2] * Vr[2][2]) * dL_dc_yy +
                        (T[0][0] * Vr[2][0] + T[0][1] * Vr[2][1] + T[0][2] * Vr[2][2]) * dL_dc_xy;
        const float (*Wr)[3] = Wm.m;
        float dL_dJ00 = Wr[0][0] * dL_dT00 + Wr[0][1] * dL_dT01 + Wr[0][2] * dL_dT02;
        float dL_dJ02 = Wr[2][0] * dL_dT00 + Wr[2][1] * dL_dT01 + Wr[2][2] * dL_dT02;
        float dL_dJ11 = Wr[1][0] * dL_dT10 + Wr[1][1] * dL_dT11 + Wr[1][2] * dL_dT12;
        float dL_dJ12 = Wr[2][0] * dL_dT10 + Wr[2][1] * dL_dT11 + Wr[2][2] * dL_dT12;
        float tz = 1.f / t[2];
        float tz2 = tz * tz;
        float tz3 = tz2 * tz;
        float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
        float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
        float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t[0]) * tz3 * dL_dJ02 +
                       (2 * h_y * t[1]) * tz3 * dL_dJ12;
        if (dL_dinvdepth_g) dL_dtz -= dL_dinvdepth_g[idx] / (t[2] * t[2]);
        float dt[3] = {dL_dtx, dL_dty, dL_dtz};
        float dmean[3];
        xformvec_t(dt, view, dmean);
        float* dm = dL_dmeans3D + 3 * (size_t)idx;
        dm[0] = dmean[0]; dm[1] = dmean[1]; dm[2] = dmean[2];

        /* ---- preprocessCUDA bwd (backward.cu:398-449) ---- */
        const float* m = mean;
        float mh[4];
        xform4x4(m, proj, mh);
        float m_w = 1.0f / (mh[3] + 0.0000001f);
        float mul1 = (proj[0] * m[0] + proj[4] * m[1] + proj[8] * m[2] + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m[0] + proj[5] * m[1] + proj[9] * m[2] + proj[13]) * m_w * m_w;
        const float d2x = dL_dmean2D[3 * (size_t)idx], d2y = dL_dmean2D[3 * (size_t)idx + 1];
        float dx_ = (proj[0] * m_w - proj[3] * mul1) * d2x + (proj[1] * m_w - proj[3] * mul2) * d2y;
        float dy_ = (proj[4] * m_w - proj[7] * mul1) * d2x + (proj[5] * m_w - proj[7] * mul2) * d2y;
        float dz_ = (proj[8] * m_w - proj[11] * mul1) * d2x + (proj[9] * m_w - proj[11] * mul2) * d2y;
        dm[0] += dx_; dm[1] += dy_; dm[2] += dz_;

        /* ---- computeCov3D bwd (backward.cu:330-393) ---- */
        if (scales && rot) {
            const float* q = rot + 4 * (size_t)idx;
            float r = q[0], x = q[1], y = q[2], z = q[3];
            mat3 R = mk3(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                         2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                         2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
            mat3 S = mk3(1, 0, 0, 0, 1, 0, 0, 0, 1);
            const float* sc = scales + 3 * (size_t)idx;
            float s[3] = {scale_mod * sc[0], scale_mod * sc[1], scale_mod * sc[2]};
            S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
            mat3 M = mul3(S, R);
            const float* dc3 = dL_dcov3D + 6 * (size_t)idx;
            mat3 dSig = mk3(dc3[0], 0.5f * dc3[1], 0.5f * dc3[2], 0.5f * dc3[1], dc3[3], 0.5f * dc3[4],
                            0.5f * dc3[2], 0.5f * dc3[4], dc3[5]);
            mat3 M2;
            for (int c = 0; c < 3; c++)
                for (int rr = 0; rr < 3; rr++) M2.m[c][rr] = 2.0f * M.m[c][rr];
            mat3 dM = mul3(M2, dSig);
            mat3 Rt = tr3(R);
            mat3 dMt = tr3(dM);
            float* dsc = dL_dscale + 3 * (size_t)idx;
            for (int k = 0; k < 3; k++)
                dsc[k] = Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1] + Rt.m[k][2] * dMt.m[k][2];
            for (int k = 0; k < 3; k++)
                for (int rr = 0; rr < 3; rr++) dMt.m[k][rr] *= s[k];
            float (*D)[3] = dMt.m;
            float* dq = dL_drot + 4 * (size_t)idx;
            dq[0] = 2 * z * (D[0][1] - D[1][0]) + 2 * y * (D[2][0] - D[0][2]) + 2 * x * (D[1][2] - D[2][1]);
            dq[1] = 2 * y * (D[1][0] + D[0][1]) + 2 * z * (D[2][0] + D[0][2]) + 2 * r * (D[1][2] - D[2][1]) - 4 * x * (D[2][2] + D[1][1]);
            dq[2] = 2 * x * (D[1][0] + D[0][1]) + 2 * r * (D[2][0] - D[0][2]) + 2 * z * (D[1][2] + D[2][1]) - 4 * y * (D[2][2] + D[0][0]);
            dq[3] = 2 * r * (D[0][1] - D[1][0]) + 2 * x * (D[2][0] + D[0][2]) + 2 * y * (D[1][2] + D[2][1]) - 4 * z * (D[1][1] + D[0][0]);
        }
    }
}
