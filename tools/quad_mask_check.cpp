// Host check of the single-frame quad tests (gsr_cull.h): (1) quad_reach4 -- the quad masks binning
// stores (binning.hip k_quad_masks) -- equals box_reach on each 4x4 quad (the shared-term form
// computes the same values) and never clears a quad with a pixel centre at Q <= K = 2 ln(255 o)
// (float64 brute force over its 16 pixels): it only drops pairs the blend skips anyway; (2) the
// conservative reach boxes (reach_bbox + quad_bits_bbox: A/B and analysis only, not stored by the
// product) never clear such a quad either.  Random conics around strips near the origin and around
// pixel (1600, 1024) (float slack at large coordinates), including means inside, on the edges and far
// away, and thin rotated ellipses:
//   hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I guava_renderer_amd/csrc \
//         tools/quad_mask_check.cpp -o /tmp/qmc && /tmp/qmc
#include "gsr_cull.h"
#include <cmath>
#include <cstdio>
#include <random>

int main() {
    using namespace gsr;
    std::mt19937 rng(11);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    long n = 0, mismatch = 0, missed = 0, need = 0, kept = 0, bb_missed = 0, bb_kept = 0;
    for (int it = 0; it < 400000; it++) {
        const float sx0 = 8.f * (float)(it % 5) + ((it >> 4) & 1 ? 1600.f : 0.f),
                    sy0 = 8.f * (float)((it / 5) % 3) + ((it >> 5) & 1 ? 1024.f : 0.f);
        const float s1 = std::exp(-3.f + 6.f * U(rng)), s2 = std::exp(-3.f + 6.f * U(rng));
        const float th = 6.2831853f * U(rng);
        const float cs = std::cos(th), sn = std::sin(th);
        // conic = inverse covariance of R diag(s1^2, s2^2) R^T
        const double i1 = 1.0 / ((double)s1 * s1), i2 = 1.0 / ((double)s2 * s2);
        const float a = (float)(cs * cs * i1 + sn * sn * i2), b = (float)(cs * sn * (i1 - i2)),
                    c = (float)(sn * sn * i1 + cs * cs * i2);
        const float o = 0.004f + U(rng);
        const float span = 8.f + 6.f * std::max(s1, s2);
        const float2 m = make_float2(sx0 + 4.f - span + 2.f * span * U(rng), sy0 + 4.f - span + 2.f * span * U(rng));
        const float4 pre = strip_pre(make_float4(a, b, c, o));
        if (__builtin_bit_cast(uint32_t, pre.w) != 0u) continue;
        const uint32_t bits = quad_reach4(a, b, c, pre.x, pre.y, pre.z, m, sx0, sy0);
        const uint32_t bbits = quad_bits_bbox(reach_bbox(make_float4(a, b, c, o), pre, m), sx0, sy0);
        for (int q = 0; q < 4; q++) {
            const float x0 = sx0 + 4.f * (q & 1), y0 = sy0 + 4.f * (q >> 1);
            const bool ref = box_reach(a, b, c, pre.x, pre.y, pre.z, m, x0, y0, 4.f, 4.f);
            const bool got = (bits >> q) & 1u;
            n++;
            mismatch += ref != got;
            kept += got;
            bool reach = false;
            for (int py = 0; py < 4; py++)
                for (int px = 0; px < 4; px++) {
                    const double dx = (double)m.x - (x0 + px), dy = (double)m.y - (y0 + py);
                    const double Q = a * dx * dx + 2.0 * b * dx * dy + c * dy * dy;
                    reach |= Q <= 2.0 * std::log(255.0 * o);
                }
            need += reach;
            missed += reach && !got;
            const bool bgot = (bbits >> q) & 1u;
            bb_kept += bgot;
            bb_missed += reach && !bgot;
        }
    }
    std::printf("quads %ld: mismatches vs box_reach %ld, missed %ld, needed %ld, kept %ld; "
                "reach boxes: missed %ld, kept %ld\n", n, mismatch, missed, need, kept, bb_missed, bb_kept);
    return (mismatch || missed || bb_missed) ? 1 : 0;
}
