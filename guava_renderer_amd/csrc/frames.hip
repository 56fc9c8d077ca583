// frames.hip -- the consumer-side frame encoding of the multi-GPU exchange.
//
// GUAVA's consumer of a rendered frame writes 8-bit images: main/test.py:85 stacks
// to8b(render) = (255 * np.clip(img, 0, 1)).astype(np.uint8) (utils/general_utils.py:316-317) into
// the video, :81-82 saves PNGs.  Gathering those bytes instead of f32 planes cuts the per-frame
// all-gather payload 4x (3 x H x W bytes per frame).  One pass over the first
// `channels` planes of each [C_src, H, W] frame: 4 pixels per thread (16-B loads, 4-B stores).
#include "../../include/gsr.h"
#include "gsr_internal.h"

namespace gsr {

// 255 * clip(x, 0, 1) truncated toward zero, as numpy's float -> uint8 cast of a value in [0, 255];
// NaN -> 0 (fmaxf returns the non-NaN operand).
__device__ __forceinline__ uint32_t to8(float x) {
    const float c = fminf(fmaxf(x, 0.0f), 1.0f);
    return (uint32_t)(255.0f * c);
}

__global__ __launch_bounds__(256) void k_frames_to8b(int64_t n4, int64_t plane4, int channels,
                                                     const float* __restrict__ src, int64_t frame_stride,
                                                     int64_t plane, uint32_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 4-pixel group of the output
    if (i >= n4) return;
    const int64_t fc = i / plane4;               // frame * channels + channel
    const int64_t q = i - fc * plane4;
    const int64_t f = fc / channels;
    const int64_t c = fc - f * channels;
    const float4 v = *reinterpret_cast<const float4*>(src + f * frame_stride + c * plane + 4 * q);
    dst[i] = to8(v.x) | (to8(v.y) << 8) | (to8(v.z) << 16) | (to8(v.w) << 24);
}

__global__ __launch_bounds__(256) void k_frames_to8b_scalar(int64_t n, int64_t plane, int channels,
                                                            const float* __restrict__ src,
                                                            int64_t frame_stride, uint8_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t fc = i / plane;
    const int64_t p = i - fc * plane;
    const int64_t f = fc / channels;
    const int64_t c = fc - f * channels;
    dst[i] = (uint8_t)to8(src[f * frame_stride + c * plane + p]);
}

}  // namespace gsr

extern "C" int gsr_frames_to8b(int B, int channels, int height, int width, const float* src,
                               int64_t frame_stride, uint8_t* dst, void* stream) {
    using namespace gsr;
    if (B < 0 || channels <= 0 || height <= 0 || width <= 0 || frame_stride < (int64_t)channels * height * width)
        return api_fail(GSR_ERR_ARG, "gsr_frames_to8b: bad shape or frame stride");
    if (B == 0) return 0;
    if (!src || !dst) return api_fail(GSR_ERR_ARG, "gsr_frames_to8b: null buffer");
    const int64_t plane = (int64_t)height * width;
    const int64_t n = (int64_t)B * channels * plane;
    hipStream_t s = (hipStream_t)stream;
    const bool vec = (plane % 4) == 0 && (frame_stride % 4) == 0 && ((uintptr_t)src & 15) == 0 &&
                     ((uintptr_t)dst & 3) == 0;
    if (vec) {
        const int64_t n4 = n / 4;
        hipLaunchKernelGGL(k_frames_to8b, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, n4, plane / 4,
                           channels, src, frame_stride, plane, reinterpret_cast<uint32_t*>(dst));
    } else {
        hipLaunchKernelGGL(k_frames_to8b_scalar, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, plane,
                           channels, src, frame_stride, dst);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return api_fail(GSR_ERR_HIP, hipGetErrorString(e));
    return 0;
}
