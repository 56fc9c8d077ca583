// Does the buffer range check of a raw (stride 0) buffer load include the SGPR offset?
// Loads at byte offset 256 of a 64-byte resource, once through voffset and once through soffset.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* p, float* out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 64, 0x00020000);
    const int lane = threadIdx.x;
    out[lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, 256 + lane * 4, 0, 0));
    out[64 + lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 256, 0));
}
int main() {
    float h[1024], *d, *o;
    for (int i = 0; i < 1024; i++) h[i] = 1.0f + i;
    hipMalloc(&d, sizeof h); hipMalloc(&o, 128 * 4);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(d, o);
    float r[128];
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("voffset past range: %g %g   soffset past range: %g %g\n", r[0], r[1], r[64], r[65]);
    return 0;
}
