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
constexpr int kAdaBwdGrid = 8192;   // 32 workgroups per CU; bounds the round-loss atomics

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

typedef float f4 __attribute__((ext_vector_type(4)));

// sigmoid with the hardware exp2 and reciprocal (v_exp_f32, v_rcp_f32, ~1 ulp each): within a
// few ulp of torch's 1/(1+expf(-a)); h enters Wq additively inside the clamp (no rounding after
// it), so Wq stays within the tests' 1e-6 absolute tolerance, and dL/dalpha within 1e-5 relative.
__device__ __forceinline__ float sigmoidf(float a)
{
    return __builtin_amdgcn_rcpf(1.0f + __expf(-a));
}

// floor(w / d) exactly as the IEEE division gives it, from q = w * rcp (rcp = v_rcp_f32(d), within
// 1 ulp): |q - RN(w/d)| <= 3.5 ulp(q) < 2^-21 (|q| + 1), so when q lies farther than that from
// every integer both floors agree; otherwise (and for non-finite q) the division decides.
__device__ __forceinline__ float floor_div(float w, float d, float rcp)
{
    const float q   = w * rcp;
    const float f   = __builtin_floorf(q);
    const float thr = (__builtin_fabsf(q) + 1.0f) * 4.76837158203125e-7f;   // 2^-21
    if (q - f > thr && (f + 1.0f) - q > thr)
        return f;
    return __builtin_floorf(w / d);
}

// |x|^beta for x in [0, 1] (the rounding-loss power): exp2(beta * log2 x) on the hardware
// transcendental unit; the reference's (torch) powf differs by a few ulp
__device__ __forceinline__ float pow01(float ax, float beta)
{
    return ax > 0.0f ? exp2f(beta * __log2f(ax)) : (beta == 0.0f ? 1.0f : 0.0f);
}

struct AdaParams
{
    float qmax, reg, beta;
    int soft;
};

__device__ __forceinline__ float ada_fwd(float w, float a, float d, float o, const AdaParams& p, float rcp)
{
    float t = floor_div(w, d, rcp);   // == floor of the IEEE division (floor is sensitive to the last ulp)
    float h;
    if (p.soft)
    {
        float pre = sigmoidf(a) * kZmG + kGamma;
        h         = fminf(fmaxf(pre, 0.0f), 1.0f);
    }
    else
        h = a >= 0.0f ? 1.0f : 0.0f;
    float q = fminf(fmaxf(t + h - o, 0.0f), p.qmax);
    return (q + o) * d;
}

// dL/dalpha of Wq (clamp pass-through masks as torch autograd) + the rounding-loss gradient
__device__ __forceinline__ float ada_bwd(float w, float a, float g, float d, float o, const AdaParams& p, float rcp,
                                         float& loss)
{
    float t   = floor_div(w, d, rcp);
    float sg  = sigmoidf(a);
    float pre = sg * kZmG + kGamma;
    float h   = fminf(fmaxf(pre, 0.0f), 1.0f);
    float u   = t + h - o;
    // d wq / d h = delta inside the clamp window (torch clamp_backward: min <= x <= max)
    float gh = (u >= 0.0f && u <= p.qmax) ? g * d : 0.0f;
    if (p.reg != 0.0f)
    {
        float x  = 2.0f * h - 1.0f;
        float ax = fabsf(x);
        float pw = pow01(ax, p.beta);
        loss += 1.0f - pw;
        // d/dh [reg * (1 - |2h-1|^beta)] = -reg * beta * |x|^(beta-1) * sign(x) * 2
        float dp = (ax > 0.0f) ? p.beta * (pw * __builtin_amdgcn_rcpf(ax)) * (x > 0.0f ? 1.0f : -1.0f) : 0.0f;
        gh += -p.reg * dp * 2.0f;
    }
    // h = clamp(pre, 0, 1); pre = sigmoid(a) * (zeta - gamma) + gamma
    float gpre = (pre >= 0.0f && pre <= 1.0f) ? gh : 0.0f;
    return gpre * kZmG * (1.0f - sg) * sg;
}

// 16-B streaming form: four consecutive elements share a channel (K % 4 == 0 or C == 1);
// one quad per lane, one tile per workgroup (the QDQ kernels' measured-best shape)
__global__ __launch_bounds__(kBlock) void adaround_fwd_vec_kernel(const f4* __restrict__ w, const f4* __restrict__ alpha,
                                                                  f4* __restrict__ wq, uint32_t nq, AdaChannel map,
                                                                  const float* __restrict__ delta,
                                                                  const float* __restrict__ offset, AdaParams p)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq)
        return;
    const uint32_t c = map.channel(4 * i);
    const float d = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(d);
    f4 wv = __builtin_nontemporal_load(w + i), av = __builtin_nontemporal_load(alpha + i), r;
    r.x = ada_fwd(wv.x, av.x, d, o, p, rcp);
    r.y = ada_fwd(wv.y, av.y, d, o, p, rcp);
    r.z = ada_fwd(wv.z, av.z, d, o, p, rcp);
    r.w = ada_fwd(wv.w, av.w, d, o, p, rcp);
    __builtin_nontemporal_store(r, wq + i);
}

__global__ __launch_bounds__(kBlock) void adaround_fwd_kernel(const float* __restrict__ w,
                                                              const float* __restrict__ alpha, float* __restrict__ wq,
                                                              uint32_t n, AdaChannel map,
                                                              const float* __restrict__ delta,
                                                              const float* __restrict__ offset, AdaParams p)
{
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    {
        uint32_t c = map.channel(i);
        wq[i]      = ada_fwd(w[i], alpha[i], delta[c], offset[c], p, __builtin_amdgcn_rcpf(delta[c]));
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

// backward: grid-stride over quads (bounded grid: one round-loss atomic per workgroup)
__global__ __launch_bounds__(kBlock) void adaround_bwd_vec_kernel(const f4* __restrict__ w, const f4* __restrict__ alpha,
                                                                  const f4* __restrict__ g, f4* __restrict__ ga,
                                                                  uint32_t nq, AdaChannel map,
                                                                  const float* __restrict__ delta,
                                                                  const float* __restrict__ offset, AdaParams p,
                                                                  float* __restrict__ round_loss,
                                                                  const float* __restrict__ reg_beta)
{
    if (reg_beta)   // device-resident {reg, beta}: a HIP-graph replay per iteration
    {
        p.reg  = reg_beta[0];
        p.beta = reg_beta[1];
    }
    float loss = 0.0f;
    constexpr int U       = 4;   // quads in flight per lane (3 x 16-B loads each)
    const uint32_t stride = gridDim.x * kBlock * U;
    for (uint32_t base = blockIdx.x * kBlock * U + threadIdx.x; base < nq; base += stride)
    {
        f4 wv[U], av[U], gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t i = base + u * kBlock;
            const uint32_t j = i < nq ? i : nq - 1;   // clamped (never stored)
            wv[u] = __builtin_nontemporal_load(w + j);
            av[u] = __builtin_nontemporal_load(alpha + j);
            gv[u] = __builtin_nontemporal_load(g + j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t i = base + u * kBlock;
            if (i >= nq)
                break;
            const uint32_t c = map.channel(4 * i);
            const float d = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(d);
            f4 r;
            r.x = ada_bwd(wv[u].x, av[u].x, gv[u].x, d, o, p, rcp, loss);
            r.y = ada_bwd(wv[u].y, av[u].y, gv[u].y, d, o, p, rcp, loss);
            r.z = ada_bwd(wv[u].z, av[u].z, gv[u].z, d, o, p, rcp, loss);
            r.w = ada_bwd(wv[u].w, av[u].w, gv[u].w, d, o, p, rcp, loss);
            __builtin_nontemporal_store(r, ga + i);
        }
    }
    if (p.reg != 0.0f && round_loss)
    {
        float s = block_sum(loss);
        if (threadIdx.x == 0)
            atomicAdd(round_loss, p.reg * s);
    }
}

__global__ __launch_bounds__(kBlock) void adaround_bwd_kernel(const float* __restrict__ w,
                                                              const float* __restrict__ alpha,
                                                              const float* __restrict__ g, float* __restrict__ ga,
                                                              uint32_t n, AdaChannel map,
                                                              const float* __restrict__ delta,
                                                              const float* __restrict__ offset, AdaParams p,
                                                              float* __restrict__ round_loss,
                                                              const float* __restrict__ reg_beta)
{
    if (reg_beta)
    {
        p.reg  = reg_beta[0];
        p.beta = reg_beta[1];
    }
    float loss = 0.0f;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    {
        uint32_t c = map.channel(i);
        ga[i]      = ada_bwd(w[i], alpha[i], g[i], delta[c], offset[c], p, __builtin_amdgcn_rcpf(delta[c]), loss);
    }
    if (p.reg != 0.0f && round_loss)
    {
        float s = block_sum(loss);
        if (threadIdx.x == 0)
            atomicAdd(round_loss, p.reg * s);
    }
}

bool aligned16(const void* p)
{
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

// ---- reconstruction-loss gradient (adaround_loss.py:70-80) ------------------------------------
// loss = mean over (N, spatial) of ||act(q) - act(t)||^2 over dim 1, so
// dloss/dq = scale * (act(q) - act(t)) * act'(q) with scale = 2 / (N * spatial): one elementwise
// pass (12 B/elem) for the ~12 torch kernels of act / sub / norm / pow / mean and their backward.
// act: 0 none, 1 ReLU (torch threshold_backward: x > 0), 2 ReLU6 (hardtanh(0, 6) backward:
// 0 < x < 6).
__device__ __forceinline__ float recon_g(float q, float t, float scale, int act)
{
    float a = q, b = t, m = 1.0f;
    if (act == 1)
    {
        a = fmaxf(q, 0.0f);
        b = fmaxf(t, 0.0f);
        m = q > 0.0f ? 1.0f : 0.0f;
    }
    else if (act == 2)
    {
        a = fminf(fmaxf(q, 0.0f), 6.0f);
        b = fminf(fmaxf(t, 0.0f), 6.0f);
        m = (q > 0.0f && q < 6.0f) ? 1.0f : 0.0f;
    }
    return scale * (a - b) * m;
}

__global__ __launch_bounds__(kBlock) void recon_grad_vec_kernel(const f4* __restrict__ q, const f4* __restrict__ t,
                                                                f4* __restrict__ g, int64_t nq, float scale, int act)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq)
        return;
    const f4 a = __builtin_nontemporal_load(q + i), b = __builtin_nontemporal_load(t + i);
    f4 r;
    r.x = recon_g(a.x, b.x, scale, act);
    r.y = recon_g(a.y, b.y, scale, act);
    r.z = recon_g(a.z, b.z, scale, act);
    r.w = recon_g(a.w, b.w, scale, act);
    __builtin_nontemporal_store(r, g + i);
}

__global__ __launch_bounds__(kBlock) void recon_grad_kernel(const float* __restrict__ q, const float* __restrict__ t,
                                                            float* __restrict__ g, int64_t begin, int64_t n,
                                                            float scale, int act)
{
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
        g[i] = recon_g(q[i], t[i], scale, act);
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
        AdaParams p {(float) ((1ull << bw) - 1), 0.0f, 0.0f, soft};
        if ((C == 1 || K % 4 == 0) && n % 4 == 0 && aligned16(w) && aligned16(alpha) && aligned16(wq))
        {
            uint32_t nq = (uint32_t) (n / 4);
            adaround_fwd_vec_kernel<<<ceil_div(nq, kBlock), kBlock, 0, as_stream(stream)>>>(
                reinterpret_cast<const f4*>(w), reinterpret_cast<const f4*>(alpha), reinterpret_cast<f4*>(wq), nq,
                map, delta, offset, p);
        }
        else
            adaround_fwd_kernel<<<stream_blocks(n, kBlock), kBlock, 0, as_stream(stream)>>>(
                w, alpha, wq, (uint32_t) n, map, delta, offset, p);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"

namespace
{

int adaround_backward(const float* w, const float* alpha, const float* g, float* ga, int64_t outer, int64_t C,
                      int64_t K, const float* delta, const float* offset, int32_t bw, float reg, float beta,
                      const float* reg_beta, float* round_loss, void* stream)
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
        AdaParams p {(float) ((1ull << bw) - 1), reg, beta, 1};
        if ((C == 1 || K % 4 == 0) && n % 4 == 0 && aligned16(w) && aligned16(alpha) && aligned16(g) &&
            aligned16(ga))
        {
            uint32_t nq = (uint32_t) (n / 4);
            int64_t blocks = ceil_div(nq, kBlock * 4);
            adaround_bwd_vec_kernel<<<(unsigned) (blocks < kAdaBwdGrid ? blocks : kAdaBwdGrid), kBlock, 0,
                                      as_stream(stream)>>>(
                reinterpret_cast<const f4*>(w), reinterpret_cast<const f4*>(alpha), reinterpret_cast<const f4*>(g),
                reinterpret_cast<f4*>(ga), nq, map, delta, offset, p, round_loss, reg_beta);
        }
        else
            adaround_bwd_kernel<<<stream_blocks(n, kBlock), kBlock, 0, as_stream(stream)>>>(
                w, alpha, g, ga, (uint32_t) n, map, delta, offset, p, round_loss, reg_beta);
        AIMET_LAUNCH_CHECK();
    });
}

}   // namespace

extern "C" {

int aimet_adaround_backward(const float* w, const float* alpha, const float* g, float* ga, int64_t outer, int64_t C,
                            int64_t K, const float* delta, const float* offset, int32_t bw, float reg, float beta,
                            float* round_loss, void* stream)
{
    return adaround_backward(w, alpha, g, ga, outer, C, K, delta, offset, bw, reg, beta, nullptr, round_loss, stream);
}

int aimet_adaround_recon_grad(const float* q, const float* t, float* g, int64_t n, int64_t reduced, int act,
                              void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(n >= 0 && reduced > 0, "invalid shape");
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        if (n == 0)
            return;
        require_device_ptr(q, "quant_out");
        require_device_ptr(t, "orig_out");
        require_device_ptr(g, "grad");
        AIMET_REQUIRE(n % reduced == 0, "element count is not a multiple of the reduced dimension");
        // torch: mean over n / reduced values of the dim-1 squared norm; d/dq = 2 (a - b) / count
        const float scale = (float) (2.0 / (double) (n / reduced));
        hipStream_t s     = as_stream(stream);
        int64_t done      = 0;
        if (aligned16(q) && aligned16(t) && aligned16(g))
        {
            const int64_t nq = n / 4;
            if (nq)
            {
                AIMET_REQUIRE(ceil_div(nq, kBlock) < (int64_t(1) << 31), "tensor too large");
                recon_grad_vec_kernel<<<(unsigned) ceil_div(nq, kBlock), kBlock, 0, s>>>(
                    reinterpret_cast<const f4*>(q), reinterpret_cast<const f4*>(t), reinterpret_cast<f4*>(g), nq,
                    scale, act);
                AIMET_LAUNCH_CHECK();
            }
            done = nq * 4;
        }
        if (done < n)
        {
            recon_grad_kernel<<<stream_blocks(n - done, kBlock), kBlock, 0, s>>>(q, t, g, done, n, scale, act);
            AIMET_LAUNCH_CHECK();
        }
    });
}

int aimet_adaround_backward_dev(const float* w, const float* alpha, const float* g, float* ga, int64_t outer,
                                int64_t C, int64_t K, const float* delta, const float* offset, int32_t bw,
                                const float* reg_beta_dev, float* round_loss, void* stream)
{
    const int rc = guarded([&] {
        AIMET_REQUIRE(reg_beta_dev != nullptr, "reg_beta_dev is null");
        require_device_ptr(reg_beta_dev, "reg_beta");
    });
    if (rc != AIMET_OK)
        return rc;
    return adaround_backward(w, alpha, g, ga, outer, C, K, delta, offset, bw, 0.0f, 0.0f, reg_beta_dev, round_loss,
                             stream);
}

}   // extern "C"
