// Host check of the scatter's strip test (binning.hip: strip_mask): it never clears a strip that
// has a pixel centre with Q <= K = 2 ln(255 o) (brute force over the strip's 64 pixels, float64),
// and how many strips it keeps beyond those; and that strip_mask (sub_reach4<8>) gives the bits of the
// four box_reach calls (strip_mask_loop).  Random conics around tiles near the origin and far from it:
//   hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I guava_renderer_amd/csrc \
//         -I include tools/strip_mask_check.cpp -o /tmp/smc && /tmp/smc
#include "../guava_renderer_amd/csrc/binning.hip"
#include <cmath>
#include <cstdio>
#include <random>

namespace gsr {  // link stand-ins for the launch helpers binning.hip uses (host check only)
int persistent_grid(int) { return 1; }
int strip_order_tile_major() { return 1; }
int xcd_queue_map() { return 2; }
}  // namespace gsr

int main() {
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    long n = 0, kept = 0, missed = 0, need = 0, mism = 0;
    for (int it = 0; it < 2000000; it++) {
        // tiles near the origin and around pixel (1600, 1024): float slack at large coordinates
        const int tx = (it & 1) ? 100 : 3, ty = (it & 2) ? 64 : 5;
        // conic of a 2D covariance with random axes and angle, mean near the tile
        const float s1 = 0.3f + 12.f * U(rng) * U(rng), s2 = 0.3f + 12.f * U(rng) * U(rng), th = 6.2831853f * U(rng);
        const float cs = cosf(th), sn = sinf(th);
        const double cxx = s1 * s1 * cs * cs + s2 * s2 * sn * sn, cyy = s1 * s1 * sn * sn + s2 * s2 * cs * cs;
        const double cxy = (s1 * s1 - s2 * s2) * cs * sn;
        const double det = cxx * cyy - cxy * cxy;
        const float4 co = make_float4((float)(cyy / det), (float)(-cxy / det), (float)(cxx / det), 0.004f + 0.996f * U(rng));
        const float2 m = make_float2(tx * 16 - 20.f + 56.f * U(rng), ty * 16 - 20.f + 56.f * U(rng));
        const float4 pre = gsr::strip_pre(co);
        const uint32_t a = gsr::strip_mask(co, pre, m, tx, ty);
        mism += a != gsr::strip_mask_loop(co, pre, m, tx, ty);  // the shared-term form: same bits
        for (int s = 0; s < gsr::kStrips; s++) {
            int x0, y0;
            gsr::strip_origin(tx, ty, s, x0, y0);
            bool hit = false;
            for (int p = 0; p < 64 && !hit; p++) {
                const double dx = m.x - (x0 + p % gsr::kStripW), dy = m.y - (y0 + p / gsr::kStripW);
                const double Q = co.x * dx * dx + 2.0 * co.y * dx * dy + co.z * dy * dy;
                hit = Q <= 2.0 * log(255.0 * co.w);
            }
            n++;
            need += hit;
            kept += (a >> s) & 1;
            missed += hit && !((a >> s) & 1);
        }
    }
    printf("strips %ld, with a pixel at Q <= K %ld, kept %ld, wrongly cleared %ld, mismatches vs the box_reach loop %ld\n",
           n, need, kept, missed, mism);
    return (missed || mism) ? 1 : 0;
}
