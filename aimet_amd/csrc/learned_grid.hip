// learned_grid.hip -- range-learning (LearnedGrid) QAT quantize-dequantize, fused, for gfx950.
//
// Reference: quantsim_straight_through_grad.py:191-249 calculate_forward_pass and :252-328
// asymmetric_gradients / symmetric_gradients, driven by QuantizeDequantizeFunc
// (v1/tensor_quantizer.py:896-986): ~10 torch kernels per tensor per step, saving x, an uint8
// x_quant and a bool mask for the backward.
//
// Here: forward = one pass (x -> y, 8 B/elem, nothing saved but x); backward = one pass that
// recomputes x_round from x and produces grad_x = mask * grad AND the three per-channel sums the
// encoding gradients need (12 B/elem):
//   A = sum((x_quant + offset) * g)        B = sum(mask * (x / delta) * g)      D = sum(!mask * g)
// asymmetric: grad_min = -(A-B)/steps + max * steps/(max-min)^2 * delta*D ; grad_max = (A-B)/steps - min * (...)
// symmetric:  grad_max = (A - B) / floor(steps/2), grad_min = -grad_max
// (assembled from the C-vectors on the torch side). Float32; torch.round = round-half-even.
#include "common.hpp"

namespace aimet_amd
{
namespace
{

typedef float f4 __attribute__((ext_vector_type(4)));

struct LgChannel
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

// x_round = round(x / delta) - offset ; x_quant = clamp(x_round, 0, steps) ; y = (x_quant + offset) * delta
__device__ __forceinline__ float lg_qdq(float x, float d, float o, float steps)
{
    float xr = __builtin_rintf(x / d) - o;
    float xq = fminf(fmaxf(xr, 0.0f), steps);
    return (xq + o) * d;
}

__global__ __launch_bounds__(kBlock) void lg_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                        uint32_t n, LgChannel map, const float* __restrict__ delta,
                                                        const float* __restrict__ offset, float steps, int vec)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (vec)
    {
        if (t >= n / 4)
            return;
        uint32_t c = map.channel(t * 4);
        float d = delta[c], o = offset[c];
        f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + t), r;
        r.x = lg_qdq(v.x, d, o, steps);
        r.y = lg_qdq(v.y, d, o, steps);
        r.z = lg_qdq(v.z, d, o, steps);
        r.w = lg_qdq(v.w, d, o, steps);
        __builtin_nontemporal_store(r, reinterpret_cast<f4*>(y) + t);
    }
    else
    {
        if (t >= n)
            return;
        uint32_t c = map.channel(t);
        y[t]       = lg_qdq(x[t], delta[c], offset[c], steps);
    }
}

struct Sums
{
    float a, b, d;
};

__device__ __forceinline__ void lg_bwd_elem(float x, float g, float dl, float o, float steps, float& gx, Sums& s)
{
    float xr   = __builtin_rintf(x / dl) - o;
    bool mask  = (xr >= 0.0f) && (xr <= steps);
    float xq   = fminf(fmaxf(xr, 0.0f), steps);
    gx         = mask ? g : 0.0f * g;      // mask_tensor * grad (keeps -0 / NaN behaviour of a multiply)
    s.a += (xq + o) * g;
    s.b += mask ? (x / dl) * g : 0.0f;
    s.d += mask ? 0.0f : g;
}

__device__ __forceinline__ Sums block_reduce(Sums s)
{
    __shared__ float sh[3][kBlock / 64];
#pragma unroll
    for (int k = 32; k > 0; k >>= 1)
    {
        s.a += __shfl_xor(s.a, k, 64);
        s.b += __shfl_xor(s.b, k, 64);
        s.d += __shfl_xor(s.d, k, 64);
    }
    int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
    {
        sh[0][w] = s.a;
        sh[1][w] = s.b;
        sh[2][w] = s.d;
    }
    __syncthreads();
    Sums r {0, 0, 0};
    if (threadIdx.x == 0)
        for (int i = 0; i < kBlock / 64; ++i)
        {
            r.a += sh[0][i];
            r.b += sh[1][i];
            r.d += sh[2][i];
        }
    __syncthreads();
    return r;
}

// per-tensor (C == 1): grid-stride, block partial sums -> 3 float atomics per workgroup
__global__ __launch_bounds__(kBlock) void lg_bwd_tensor_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ g, float* __restrict__ gx,
                                                               int64_t n, const float* __restrict__ delta,
                                                               const float* __restrict__ offset, float steps,
                                                               float* __restrict__ sums, int vec)
{
    const float dl = delta[0], o = offset[0];
    Sums s {0, 0, 0};
    if (vec)
    {
        const int64_t nv = n / 4;
        for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < nv; i += (int64_t) gridDim.x * kBlock)
        {
            f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + i);
            f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + i);
            float r0, r1, r2, r3;
            lg_bwd_elem(a.x, b.x, dl, o, steps, r0, s);
            lg_bwd_elem(a.y, b.y, dl, o, steps, r1, s);
            lg_bwd_elem(a.z, b.z, dl, o, steps, r2, s);
            lg_bwd_elem(a.w, b.w, dl, o, steps, r3, s);
            f4 r = {r0, r1, r2, r3};
            if (gx)
                __builtin_nontemporal_store(r, reinterpret_cast<f4*>(gx) + i);
        }
        for (int64_t i = nv * 4 + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
        {
            float r;
            lg_bwd_elem(x[i], g[i], dl, o, steps, r, s);
            if (gx)
                gx[i] = r;
        }
    }
    else
    {
        for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
        {
            float r;
            lg_bwd_elem(x[i], g[i], dl, o, steps, r, s);
            if (gx)
                gx[i] = r;
        }
    }
    Sums t = block_reduce(s);
    if (threadIdx.x == 0)
    {
        atomicAdd(&sums[0], t.a);
        atomicAdd(&sums[1], t.b);
        atomicAdd(&sums[2], t.d);
    }
}

// per-channel: one workgroup per channel of [outer][C][K], sums written directly
__global__ __launch_bounds__(kBlock) void lg_bwd_channel_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ g, float* __restrict__ gx,
                                                                int64_t outer, int64_t C, int64_t K,
                                                                const float* __restrict__ delta,
                                                                const float* __restrict__ offset, float steps,
                                                                float* __restrict__ sums)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        const float dl = delta[c], o = offset[c];
        Sums s {0, 0, 0};
        for (int64_t r = 0; r < outer; ++r)
        {
            const int64_t base = (r * C + c) * K;
            for (int64_t k = threadIdx.x; k < K; k += kBlock)
            {
                float v;
                lg_bwd_elem(x[base + k], g[base + k], dl, o, steps, v, s);
                if (gx)
                    gx[base + k] = v;
            }
        }
        Sums t = block_reduce(s);
        if (threadIdx.x == 0)
        {
            sums[3 * c + 0] = t.a;
            sums[3 * c + 1] = t.b;
            sums[3 * c + 2] = t.d;
        }
    }
}

// per-channel, 16-B form (K % 4 == 0, aligned): a (channel, slice) grid; with one slice the sums
// are stored (deterministic), with several (few channels: fill the chip) they are added atomically
// into the zeroed sums.
__global__ __launch_bounds__(kBlock) void lg_bwd_channel_vec_kernel(const f4* __restrict__ x, const f4* __restrict__ g,
                                                                    f4* __restrict__ gx, int64_t outer, int64_t C,
                                                                    int64_t K4, FastDiv divK4,
                                                                    const float* __restrict__ delta,
                                                                    const float* __restrict__ offset, float steps,
                                                                    float* __restrict__ sums)
{
    const int splits = gridDim.y;
    const int64_t Q  = outer * K4;
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        const float dl = delta[c], o = offset[c];
        Sums s {0, 0, 0};
        for (int64_t j = (int64_t) blockIdx.y * kBlock + threadIdx.x; j < Q; j += (int64_t) splits * kBlock)
        {
            const int64_t r = outer == 1 ? 0 : divK4.div((uint32_t) j);
            const int64_t i = (r * C + c) * K4 + (j - r * K4);
            f4 a = __builtin_nontemporal_load(x + i);
            f4 b = __builtin_nontemporal_load(g + i);
            float r0, r1, r2, r3;
            lg_bwd_elem(a.x, b.x, dl, o, steps, r0, s);
            lg_bwd_elem(a.y, b.y, dl, o, steps, r1, s);
            lg_bwd_elem(a.z, b.z, dl, o, steps, r2, s);
            lg_bwd_elem(a.w, b.w, dl, o, steps, r3, s);
            if (gx)
            {
                f4 rv = {r0, r1, r2, r3};
                __builtin_nontemporal_store(rv, gx + i);
            }
        }
        Sums t = block_reduce(s);
        if (threadIdx.x == 0)
        {
            if (splits == 1)
            {
                sums[3 * c + 0] = t.a;
                sums[3 * c + 1] = t.b;
                sums[3 * c + 2] = t.d;
            }
            else
            {
                atomicAdd(&sums[3 * c + 0], t.a);
                atomicAdd(&sums[3 * c + 1], t.b);
                atomicAdd(&sums[3 * c + 2], t.d);
            }
        }
    }
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

int aimet_lg_forward(const float* x, float* y, int64_t outer, int64_t C, int64_t K, const float* delta,
                     const float* offset, float num_steps, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "learned-grid QDQ needs < 2^31 elements per call");
        require_device_ptr(x, "x");
        require_device_ptr(y, "y");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        LgChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        bool vec     = (C == 1 || K % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0
                       && n % 4 == 0;
        int64_t work = vec ? n / 4 : n;
        lg_fwd_kernel<<<(unsigned) ceil_div(work, kBlock), kBlock, 0, as_stream(stream)>>>(
            x, y, (uint32_t) n, map, delta, offset, num_steps, vec ? 1 : 0);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_lg_backward(const float* x, const float* grad, float* grad_x, float* sums, int64_t outer, int64_t C,
                      int64_t K, const float* delta, const float* offset, float num_steps, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        require_device_ptr(sums, "sums");
        hipStream_t s = as_stream(stream);
        AIMET_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(float) * 3 * C, s));
        if (n == 0)
            return;
        require_device_ptr(x, "x");
        require_device_ptr(grad, "grad");
        if (grad_x)
            require_device_ptr(grad_x, "grad_x");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        if (C == 1)
        {
            bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad) |
                         reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0;
            lg_bwd_tensor_kernel<<<stream_blocks(n, (int64_t) kBlock * 16), kBlock, 0, s>>>(
                x, grad, grad_x, n, delta, offset, num_steps, sums, vec ? 1 : 0);
        }
        else if (K % 4 == 0 && outer * (K / 4) < (int64_t(1) << 32) &&
                 ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad) |
                   reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0)
        {
            // >= 2048 workgroups in flight: slice channels when there are fewer than that
            const int64_t K4  = K / 4;
            int64_t splits    = C >= 2048 ? 1 : (2048 + C - 1) / C;
            const int64_t per = ceil_div(outer * K4, kBlock);   // enough quads for every slice
            if (splits > per)
                splits = per > 0 ? per : 1;
            dim3 grid((unsigned) (C < 65536 ? C : 65536), (unsigned) splits);
            lg_bwd_channel_vec_kernel<<<grid, kBlock, 0, s>>>(
                reinterpret_cast<const f4*>(x), reinterpret_cast<const f4*>(grad), reinterpret_cast<f4*>(grad_x),
                outer, C, K4, FastDiv((uint32_t) (K4 > 0 ? K4 : 1)), delta, offset, num_steps, sums);
        }
        else
        {
            int grid = (int) (C < 65536 ? C : 65536);
            lg_bwd_channel_kernel<<<grid, kBlock, 0, s>>>(x, grad, grad_x, outer, C, K, delta, offset, num_steps,
                                                          sums);
        }
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
