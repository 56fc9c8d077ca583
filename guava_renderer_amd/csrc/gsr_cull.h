// gsr_cull.h -- the exact, conservative "can this Gaussian reach alpha >= 1/255 anywhere in this
// pixel rectangle" test: binning's per-strip masks (binning.hip strip_mask) and render_fwd's
// per-quad cull of the single-frame quad waves.  A rejected (rectangle, Gaussian) pair only ever
// removes pairs the blend skips anyway (alpha < 1/255, forward.cu:362-363), so culling with it is
// decision-preserving.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace gsr {

// Minimum over the pixel-centre rectangle dx in [dxl, dxh], dy in [dyl, dyh] (dx = mean - pixel)
// of the conic's quadratic form Q = a dx^2 + 2b dx dy + c dy^2 (power = -Q/2 in the blend).  Q is
// convex (a, c > 0, ac > b^2), so the minimum is 0 if the mean lies inside, else it lies on an edge:
// each edge is a 1-D quadratic minimised by clamping its vertex.
// Only the edges FACING the mean can hold that minimum: from a point of any other edge the segment
// towards the mean enters the rectangle and Q falls along it (convexity).  So at most one vertical
// edge (the column nearest the mean, when the mean is left or right of the rectangle) and one
// horizontal edge are evaluated -- half of the four-edge form's work, the same minimum.
__host__ __device__ __forceinline__ float rect_qmin(float a, float b, float c, float ia, float ic, float dxl, float dxh,
                                           float dyl, float dyh) {
    const bool xin = dxl <= 0.f && dxh >= 0.f, yin = dyl <= 0.f && dyh >= 0.f;
    if (xin && yin) return 0.f;
    float q = 3.0e38f;
    if (!xin) {  // the facing column: dx = dxl (mean right of it) or dxh (mean left of it)
        const float X = dxl > 0.f ? dxl : dxh;
        const float y = fminf(fmaxf(-b * X * ic, dyl), dyh);
        q = a * X * X + 2.f * b * X * y + c * y * y;
    }
    if (!yin) {  // the facing row
        const float Y = dyl > 0.f ? dyl : dyh;
        const float x = fminf(fmaxf(-b * Y * ia, dxl), dxh);
        q = fminf(q, a * x * x + 2.f * b * x * Y + c * Y * Y);
    }
    return q;
}

// Per-Gaussian part of the strip test, computed once per Gaussian (not once per instance):
// (K = 2 ln(255 o), 1/a, 1/c, mode) with mode 0 = test the strips, 1 = no strip (o < 1/255:
// alpha <= o < 1/255 at every pixel), 2 = every strip (non-finite or non-positive-definite conic).
__host__ __device__ __forceinline__ float4 strip_pre(float4 co) {
    const float a = co.x, b = co.y, c = co.z, o = co.w;
    if (o < 1.0f / 255.0f) return make_float4(0.f, 0.f, 0.f, __builtin_bit_cast(float, 1u));
    if (!(a > 0.f) || !(c > 0.f) || !(a * c - b * b > 0.f) || !(o <= 3.0e38f))
        return make_float4(0.f, 0.f, 0.f, __builtin_bit_cast(float, 2u));
    return make_float4(2.0f * logf(255.0f * o), 1.0f / a, 1.0f / c, __builtin_bit_cast(float, 0u));
}

// Whether the Gaussian (conic a, b, c; pre = strip_pre's K, 1/a, 1/c) can give alpha >= 1/255 at
// some pixel centre of the w x h rectangle at (x0, y0): not (Q > K) on the whole rectangle, with a
// slack of 1e-4 of the form's term magnitudes + 1e-3 relative that covers float rounding of both
// this test and the blend's power (tools/strip_mask_check.cpp brute-forces it).
__host__ __device__ __forceinline__ bool box_reach(float a, float b, float c, float K, float ia, float ic, float2 m,
                                                   float x0, float y0, float w, float h) {
    const float dxl = m.x - (x0 + (w - 1.0f)), dxh = m.x - x0;
    const float mx = fmaxf(fabsf(dxl), fabsf(dxh));
    const float dyl = m.y - (y0 + (h - 1.0f)), dyh = m.y - y0;
    const float my = fmaxf(fabsf(dyl), fabsf(dyh));
    const float slack = 1e-4f * (a * mx * mx + 2.f * fabsf(b) * mx * my + c * my * my) + 1e-3f * K + 1e-3f;
    const float q = rect_qmin(a, b, c, ia, ic, dxl, dxh, dyl, dyh);
    return !(q > K + slack);
}

// The pixel-centre bounding box (xmin, ymin, xmax, ymax) of where a Gaussian can reach alpha >=
// 1/255, for the single-frame quad masks: the ellipse Q <= K has half-extents sqrt(K c / det) and
// sqrt(K a / det) (det = ac - b^2), taken here for K' = 1.01 K + 0.01 -- a 1% margin that exceeds the
// float rounding of the blend's power by orders of magnitude for any conic with |b| <= 0.995
// sqrt(ac) (terms at most 400x Q there).  Flatter conics (and mode 2) get an unbounded box: every
// quad of their kept strips stays.  Per Gaussian, once.
__host__ __device__ __forceinline__ float4 reach_bbox(float4 co, float4 pre, float2 m) {
    const float a = co.x, b = co.y, c = co.z;
    const uint32_t mode = __builtin_bit_cast(uint32_t, pre.w);
    const float det = a * c - b * b;
    if (mode != 0u || !(b * b <= 0.990025f * (a * c)) || !(det > 0.f))
        return make_float4(-3.0e38f, -3.0e38f, 3.0e38f, 3.0e38f);
    const float K2 = 1.01f * pre.x + 0.01f;
    const float hx = sqrtf(K2 * c / det) * 1.001f + 1e-3f, hy = sqrtf(K2 * a / det) * 1.001f + 1e-3f;
    return make_float4(m.x - hx, m.y - hy, m.x + hx, m.y + hy);
}
// The four quads (bit q: x offset 4 (q & 1), y offset 4 (q >> 1)) of the 8x8 strip at (sx0, sy0)
// whose pixel centres meet the box.
__host__ __device__ __forceinline__ uint32_t quad_bits_bbox(float4 bb, float sx0, float sy0) {
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const float x0 = sx0 + 4.0f * (float)(q & 1), y0 = sy0 + 4.0f * (float)(q >> 1);
        bits |= (bb.x <= x0 + 3.0f && bb.z >= x0 && bb.y <= y0 + 3.0f && bb.w >= y0) ? (1u << q) : 0u;
    }
    return bits;
}

// box_reach of the four S x S sub-rectangles of the 2S x 2S block at (x0b, y0b) at once, bit q =
// sub-rectangle q (x offset S (q & 1), y offset S (q >> 1)): the same expressions as box_reach /
// rect_qmin on each (so the same bits), with the per-column and per-row terms shared between them
// and rect_qmin's branches turned into selects of the same values (no divergent paths).  S = 4: the
// quads of an 8x8 strip (quad_reach4); S = 8: the strips of a 16x16 tile (binning's strip_mask).
template <int S>
__host__ __device__ __forceinline__ uint32_t sub_reach4(float a, float b, float c, float K, float ia, float ic,
                                                        float2 m, float x0b, float y0b) {
    float dxl[2], dxh[2], mx[2], dyl[2], dyh[2], my[2];
    bool xin[2], yin[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const float x0 = x0b + (float)S * (float)h, y0 = y0b + (float)S * (float)h;
        dxl[h] = m.x - (x0 + ((float)S - 1.0f));
        dxh[h] = m.x - x0;
        mx[h] = fmaxf(fabsf(dxl[h]), fabsf(dxh[h]));
        dyl[h] = m.y - (y0 + ((float)S - 1.0f));
        dyh[h] = m.y - y0;
        my[h] = fmaxf(fabsf(dyl[h]), fabsf(dyh[h]));
        xin[h] = dxl[h] <= 0.f && dxh[h] >= 0.f;
        yin[h] = dyl[h] <= 0.f && dyh[h] >= 0.f;
    }
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int hx = q & 1, hy = q >> 1;
        const float slack = 1e-4f * (a * mx[hx] * mx[hx] + 2.f * fabsf(b) * mx[hx] * my[hy] + c * my[hy] * my[hy]) +
                            1e-3f * K + 1e-3f;
        const float X = dxl[hx] > 0.f ? dxl[hx] : dxh[hx];
        const float y = fminf(fmaxf(-b * X * ic, dyl[hy]), dyh[hy]);
        const float qx = a * X * X + 2.f * b * X * y + c * y * y;
        const float Y = dyl[hy] > 0.f ? dyl[hy] : dyh[hy];
        const float x = fminf(fmaxf(-b * Y * ia, dxl[hx]), dxh[hx]);
        const float qy = a * x * x + 2.f * b * x * Y + c * Y * Y;
        float qm = xin[hx] ? 3.0e38f : qx;
        qm = yin[hy] ? qm : fminf(qm, qy);
        qm = (xin[hx] && yin[hy]) ? 0.f : qm;
        bits |= (!(qm > K + slack)) ? (1u << q) : 0u;
    }
    return bits;
}

// the four 4x4 quads of the 8x8 strip at (sx0, sy0)
__host__ __device__ __forceinline__ uint32_t quad_reach4(float a, float b, float c, float K, float ia, float ic,
                                                         float2 m, float sx0, float sy0) {
    return sub_reach4<4>(a, b, c, K, ia, ic, m, sx0, sy0);
}

}  // namespace gsr
