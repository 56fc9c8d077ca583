// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE on gfx950 for the load shapes render_fwd uses,
// against an exactly known byte count (MI355X_MICROARCH.md: FETCH_SIZE is exactly half the bytes of
// a 16-B/lane streaming read; other widths uncalibrated).  Each kernel reads a 1 GiB buffer (4x the
// Infinity Cache, so the reads reach HBM) exactly once:
//   k_b32      : buffer_load_dword, 4 B per lane, a wave reads 256 contiguous bytes (render_fwd's
//                feature operand: lanes 0-31 one Gaussian's 128-B row, lanes 32-63 another's)
//   k_b128     : 16 B per lane (the guide's calibrated case)
//   k_uni_b128 : wave-uniform 16-B loads (render_fwd's render-record loads: every lane the same
//                address), consecutive 16-B pieces per load
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/fetch_calib.hip -o tools/micro/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE -- tools/micro/fetch_calib   (prints the byte count per kernel)
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = size_t(1) << 30;

__global__ __launch_bounds__(256) void k_b32(const float* __restrict__ src, float* sink, size_t n) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7FFFFFFF, 0x00020000);
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(i * 4 % 0x7FFFFFF0u), 0, 0));
    if (acc == 12345.f) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_b128(const float4* __restrict__ src, float* sink, size_t n4) {
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const float4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;
}

// each wave walks its own contiguous 1/nwaves slice in 16-B steps, every lane loading the same 16 B
__global__ __launch_bounds__(256) void k_uni_b128(const float4* __restrict__ src, float* sink, size_t n4) {
    const size_t nw = (size_t)gridDim.x * (blockDim.x / 64);
    const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const size_t per = n4 / nw;
    float acc = 0.f;
    for (size_t i = w * per; i < (w + 1) * per; i++) {
        const float4 v = src[__builtin_amdgcn_readfirstlane((unsigned)(i & 0xFFFFFFFFu)) + (i & ~size_t(0xFFFFFFFF))];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;
}

int main() {
    float* buf = nullptr;
    float* sink = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(buf, 0, kBytes);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t n = kBytes / 4;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_b32, dim3(cus * 8), dim3(256), 0, 0, buf, sink, n / 4);  // 256 MiB: the b32 path wraps at 2 GiB offsets
        hipLaunchKernelGGL(k_b128, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink, n / 4);
        hipLaunchKernelGGL(k_uni_b128, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<const float4*>(buf), sink,
                           n / 16);  // 64 MiB of uniform 16-B pieces
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("k_b32 bytes %zu\nk_b128 bytes %zu\nk_uni_b128 bytes %zu\n", kBytes / 4, kBytes, kBytes / 4);
    return 0;
}
