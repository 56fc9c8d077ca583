// Do v_mfma_f32_32x32x2_f32 and plain f32 VALU work overlap on one SIMD (gfx950)?
// Each workgroup = 8 waves (2 per SIMD).  Modes:
//   0: every wave runs only MFMAs (NM per iteration, 2 independent accumulators)
//   1: every wave runs only VALU FMAs (NV per iteration, 8 independent chains)
//   2: waves 0-3 MFMA-only, waves 4-7 VALU-only (one of each per SIMD)
//   3: every wave interleaves NM MFMAs and NV VALU FMAs per iteration
//   4: as 1 with bf16 MFMAs 32x32x8 (NM per iteration) in mode-2 layout (reference)
// Prints the kernel time of each mode; overlap <=> mode 2 ~ max(mode 0, mode 1) at matched work.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short shortx4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void k(int iters, float seed, float* out) {
    const int w = threadIdx.x >> 6;
    floatx16 a0 = {}, a1 = {};
    float v[8];
    for (int i = 0; i < 8; i++) v[i] = seed + i * threadIdx.x;
    const float x = seed * threadIdx.x, y = seed + threadIdx.x;
    const bool do_m = MODE == 0 || MODE == 3 || ((MODE == 2 || MODE == 4) && w < 4);
    const bool do_v = MODE == 1 || MODE == 3 || ((MODE == 2 || MODE == 4) && w >= 4);
    for (int it = 0; it < iters; it++) {
        if (do_m) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if (MODE == 4) {
                    const shortx4 aa = {1, 2, 3, 4};
                    a0 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(aa, aa, a0, 0, 0, 0);
                    a1 = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(aa, aa, a1, 0, 0, 0);
                } else {
                    a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
                    a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, a1, 0, 0, 0);
                }
            }
        }
        if (do_v) {
#pragma unroll
            for (int j = 0; j < 16; j++)
#pragma unroll
                for (int c = 0; c < 8; c++) v[c] = fmaf(v[c], x, y);
        }
    }
    float s = 0.f;
    for (int i = 0; i < 16; i++) s += a0[i] + a1[i];
    for (int i = 0; i < 8; i++) s += v[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
    float* o;
    hipMalloc(&o, 4096 * 512 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256, iters = 4000;  // one 8-wave workgroup per CU
    for (int rep = 0; rep < 2; rep++) {
        for (int mode = 0; mode < 5; mode++) {
            auto run = [&](auto kern) {
                kern<<<grid, 512>>>(iters, 1.0001f, o);
                hipDeviceSynchronize();
                hipEventRecord(e0);
                kern<<<grid, 512>>>(iters, 1.0001f, o);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                return ms;
            };
            float ms = mode == 0 ? run(k<0>) : mode == 1 ? run(k<1>) : mode == 2 ? run(k<2>) : mode == 3 ? run(k<3>) : run(k<4>);
            // per SIMD: mode 0: 2 waves x 8 MFMA (64 cyc) per iter; mode 1: 2 waves x 128 VALU
            printf("mode %d: %.3f ms\n", mode, ms);
        }
    }
    return 0;
}
