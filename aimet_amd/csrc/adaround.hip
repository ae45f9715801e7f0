// adaround.hip -- fused AdaRound soft-quantization forward and backward for gfx950.
//
// Reference (pure torch, ~6 elementwise kernels forward and ~10 backward per iteration, each a
// full pass over the weight): AdaroundWrapper.apply_adaround (v1/adaround/adaround_wrapper.py:124-149)
// and AdaroundLoss.compute_round_loss (v1/adaround/adaround_loss.py:83-110), ZETA = 1.1,
// GAMMA = -0.1 (aimet_common/defs.py:302-306).
//
// Here: one pass forward (reads W, alpha; writes Wq: 12 B/elem) and one pass backward (reads
// grad_Wq, W, alpha; writes grad_alpha: 16 B/elem) that also produces the rounding-loss term
// and its gradient. Floating-point results follow torch float32 op order (tolerance-checked).
#include "common.hpp"

namespace aimet_amd
{
namespace
{

constexpr float kGamma = -0.1f;
// python: (ZETA - GAMMA) = 1.2000000000000002 -> float32 scalar 1.2f in the torch op
constexpr float kZmG = (float) (1.1 - (-0.1));

struct AdaChannel
{
    FastDiv divK, divC;
    uint32_t C;
    __device__ __forceinline__ uint32_t channel(uint32_t i) const
    {
        if (C == 1)
            return 0;
        uint32_t row = divK.div(i);
        return row - divC.div(row) * C;
    }
};

__device__ __forceinline__ float sigmoidf(float a)
{
    return 1.0f / (1.0f + expf(-a));
}

__global__ __launch_bounds__(kBlock) void adaround_fwd_kernel(const float* __restrict__ w,
                                                              const float* __restrict__ alpha, float* __restrict__ wq,
                                                              uint32_t n, AdaChannel map,
                                                              const float* __restrict__ delta,
                                                              const float* __restrict__ offset, float qmax, int soft)
{
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    {
        uint32_t c = map.channel(i);
        float d = delta[c], o = offset[c];
        float t = __builtin_floorf(w[i] / d);
        float a = alpha[i];
        float h;
        if (soft)
        {
            float pre = sigmoidf(a) * kZmG + kGamma;
            h         = fminf(fmaxf(pre, 0.0f), 1.0f);
        }
        else
            h = a >= 0.0f ? 1.0f : 0.0f;
        float q = fminf(fmaxf(t + h - o, 0.0f), qmax);
        wq[i]   = (q + o) * d;
    }
}

__device__ __forceinline__ float block_sum(float v)
{
    __shared__ float s[kBlock / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0)
        s[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kBlock / 64; ++i)
            r += s[i];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kBlock) void adaround_bwd_kernel(const float* __restrict__ w,
                                                              const float* __restrict__ alpha,
                                                              const float* __restrict__ g, float* __restrict__ ga,
                                                              uint32_t n, AdaChannel map,
                                                              const float* __restrict__ delta,
                                                              const float* __restrict__ offset, float qmax, float reg,
                                                              float beta, float* __restrict__ round_loss)
{
    float loss = 0.0f;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    {
        uint32_t c = map.channel(i);
        float d = delta[c], o = offset[c];
        float t   = __builtin_floorf(w[i] / d);
        float a   = alpha[i];
        float sg  = sigmoidf(a);
        float pre = sg * kZmG + kGamma;
        float h   = fminf(fmaxf(pre, 0.0f), 1.0f);
        float u   = t + h - o;
        // d wq / d h = delta inside the clamp window (torch clamp_backward: min <= x <= max)
        float gh = (u >= 0.0f && u <= qmax) ? g[i] * d : 0.0f;
        if (reg != 0.0f)
        {
            float x  = 2.0f * h - 1.0f;
            float ax = fabsf(x);
            float p  = powf(ax, beta);
            loss += 1.0f - p;
            // d/dh [reg * (1 - |2h-1|^beta)] = -reg * beta * |x|^(beta-1) * sign(x) * 2
            float dp = (ax > 0.0f) ? beta * powf(ax, beta - 1.0f) * (x > 0.0f ? 1.0f : -1.0f) : 0.0f;
            gh += -reg * dp * 2.0f;
        }
        // h = clamp(pre, 0, 1); pre = sigmoid(a) * (zeta - gamma) + gamma
        float gpre = (pre >= 0.0f && pre <= 1.0f) ? gh : 0.0f;
        ga[i]      = gpre * kZmG * (1.0f - sg) * sg;
    }
    if (reg != 0.0f && round_loss)
    {
        float s = block_sum(loss);
        if (threadIdx.x == 0)
            atomicAdd(round_loss, reg * s);
    }
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

int aimet_adaround_forward(const float* w, const float* alpha, float* wq, int64_t outer, int64_t C, int64_t K,
                           const float* delta, const float* offset, int32_t bw, int soft, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "AdaRound weight too large (>= 2^31 elements)");
        require_device_ptr(w, "weight");
        require_device_ptr(alpha, "alpha");
        require_device_ptr(wq, "output");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        AdaChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        float qmax = (float) ((1ull << bw) - 1);
        adaround_fwd_kernel<<<stream_blocks(n, kBlock), kBlock, 0, as_stream(stream)>>>(
            w, alpha, wq, (uint32_t) n, map, delta, offset, qmax, soft);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_backward(const float* w, const float* alpha, const float* g, float* ga, int64_t outer, int64_t C,
                            int64_t K, const float* delta, const float* offset, int32_t bw, float reg, float beta,
                            float* round_loss, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "AdaRound weight too large (>= 2^31 elements)");
        require_device_ptr(w, "weight");
        require_device_ptr(alpha, "alpha");
        require_device_ptr(g, "grad");
        require_device_ptr(ga, "grad_alpha");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        AdaChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        float qmax = (float) ((1ull << bw) - 1);
        adaround_bwd_kernel<<<stream_blocks(n, kBlock), kBlock, 0, as_stream(stream)>>>(
            w, alpha, g, ga, (uint32_t) n, map, delta, offset, qmax, reg, beta, round_loss);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
