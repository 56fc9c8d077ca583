// Residency microbenchmark: how many 256-thread workgroups run concurrently for a given LDS /
// register footprint and launch pattern.  Each workgroup spins ~SPIN_US and records its 100 MHz
// realtime start/end; the host reports the average number resident.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int LDS_BYTES, int NREG>
__global__ __launch_bounds__(256) void k_spin(unsigned long long* out, int spin_ticks, int empty_mod) {
    __shared__ float lds[LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1];
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float acc[NREG];
#pragma unroll
    for (int i = 0; i < NREG; i++) acc[i] = threadIdx.x * (i + 1);
    bool empty = empty_mod > 0 && (blockIdx.x % empty_mod) != 0;
    if (!empty) {
        while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks) {
#pragma unroll
            for (int i = 0; i < NREG; i++) acc[i] = acc[i] * 1.0001f + 0.5f;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < NREG; i++) s += acc[i];
    lds[threadIdx.x % (LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1)] = s;
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = t0; out[2 * blockIdx.x + 1] = t1 + (lds[0] == 12345.f); }
}

template <int LDS, int NREG>
void run(const char* name, int nblk, int spin_us, int empty_mod) {
    unsigned long long* d;
    hipMalloc(&d, sizeof(unsigned long long) * 2 * nblk);
    hipLaunchKernelGGL((k_spin<LDS, NREG>), dim3(nblk), dim3(256), 0, 0, d, spin_us * 100, empty_mod);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((k_spin<LDS, NREG>), dim3(nblk), dim3(256), 0, 0, d, spin_us * 100, empty_mod);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * nblk);
    hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * nblk, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, t1 = 0; double sum = 0; int busy = 0;
    for (int i = 0; i < nblk; i++) {
        t0 = std::min(t0, h[2 * i]); t1 = std::max(t1, h[2 * i + 1]);
        bool e = empty_mod > 0 && (i % empty_mod) != 0;
        if (!e) { sum += (double)(h[2 * i + 1] - h[2 * i]); busy++; }
    }
    hipFuncAttributes a; hipFuncGetAttributes(&a, (const void*)k_spin<LDS, NREG>);
    printf("%-28s regs=%3d lds=%6d blocks=%6d busy=%6d span=%8.1fus avg_resident_busy_WGs=%.1f\n", name,
           a.numRegs, (int)a.sharedSizeBytes, nblk, busy, (t1 - t0) / 100.0, sum / (double)(t1 - t0));
    hipFree(d);
}

int main() {
    run<1024, 8>("small", 16384, 20, 0);
    run<11440, 8>("lds11k", 16384, 20, 0);
    run<11440, 64>("lds11k_reg64", 16384, 20, 0);
    run<11440, 96>("lds11k_reg96", 16384, 20, 0);
    run<11440, 8>("lds11k_half_empty", 32768, 20, 2);
    run<11440, 8>("lds11k_3of4_empty", 32768, 20, 4);
    return 0;
}
