// rs_post.h -- post-frame streaming kernels: the producer loop's per-frame block
// after produceRestir (pg/simpleguidx11.cpp:246-333) minus OIDN:
//   accumulator = glm::mix(accumulator, frame, 1/(accFrameCtr+1))               (:246-253)
//   display = vec4(compress(aces(accumulator)), 1)  with the tonemap / gammaCorrect switches (:266-294)
//   mean / variance of the accumulator's per-pixel channel mean (float mean, double sums) (:304-327)
// One pass over the band: 12 B frame + 12 B accumulator read, 12 B accumulator + 16 B display written
// = 52 B/px (HBM-bound streaming, ~15 us at 1080p); per-workgroup double partials reduced in a fixed
// order so the statistics are deterministic.
#pragma once
#include "rs_device.h"

namespace rs {

struct PostConst {
    int W, y0, y1;
    float a;              // 1 / (accFrameCtr + 1)
    int tonemap, gamma;
};

// Utils::aces (pg/utils.cpp:191-198) per channel, glm::clamp = min(max(x, 0), 1) in select form
__device__ __forceinline__ float post_aces(float x) {
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    float v = (x * (a * x + b)) / (x * (c * x + d) + e);
    return gmin(gmax(v, 0.0f), 1.0f);
}
// Utils::compress (pg/utils.cpp:219-229); the linear-segment test compares with the double 0.0031308
__device__ __forceinline__ float post_compress(float u) {
    if (u <= 0.0f) return 0.0f;
    if (u >= 1.0f) return 1.0f;
    if ((double)u <= 0.0031308) return u * 12.92f;
    return 1.055f * rs_powf(u, 1.0f / 2.4f) - 0.055f;
}

__global__ void __launch_bounds__(256) k_post(const float* __restrict__ frame, float* __restrict__ acc,
                                              float4* __restrict__ display, PostConst P, double2* __restrict__ part) {
    __shared__ double ss[256], sq[256];
    const size_t n = (size_t)(P.y1 - P.y0) * P.W;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    double s = 0.0, q = 0.0;
    if (i < n) {
        const size_t p = (size_t)P.y0 * P.W + i;
        float px[3], m[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            m[k] = acc[3 * p + k] * (1.0f - P.a) + frame[3 * p + k] * P.a;   // compute_mix_scalar
            float v = m[k];
            if (P.tonemap) v = post_aces(v);
            if (P.gamma) v = post_compress(v);
            px[k] = v;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[3 * p + k] = m[k];
        display[p] = make_float4(px[0], px[1], px[2], 1.0f);
        const float mean = (m[0] + m[1] + m[2]) / 3.0f;
        s = mean;
        q = (double)(mean * mean);
    }
    ss[threadIdx.x] = s; sq[threadIdx.x] = q;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) { ss[threadIdx.x] += ss[threadIdx.x + w]; sq[threadIdx.x] += sq[threadIdx.x + w]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = make_double2(ss[0], sq[0]);
}

// display from the denoised accumulator when RenderParams::denoise (pg/simpleguidx11.cpp:277-292)
__global__ void __launch_bounds__(256) k_post_display(const float* __restrict__ img, float4* __restrict__ display,
                                                      PostConst P) {
    const size_t n = (size_t)(P.y1 - P.y0) * P.W;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t p = (size_t)P.y0 * P.W + i;
    float px[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float v = img[3 * p + k];
        if (P.tonemap) v = post_aces(v);
        if (P.gamma) v = post_compress(v);
        px[k] = v;
    }
    display[p] = make_float4(px[0], px[1], px[2], 1.0f);
}

// one workgroup: partials -> (sum, sqr_sum), fixed order
__global__ void __launch_bounds__(256) k_post_reduce(const double2* __restrict__ part, int n, double2* out) {
    __shared__ double ss[256], sq[256];
    double s = 0.0, q = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) { s += part[i].x; q += part[i].y; }
    ss[threadIdx.x] = s; sq[threadIdx.x] = q;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) { ss[threadIdx.x] += ss[threadIdx.x + w]; sq[threadIdx.x] += sq[threadIdx.x + w]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = make_double2(ss[0], sq[0]);
}

}  // namespace rs
