// Where the channel-major MFMA forward's time goes (aimet_amd/csrc/pwcm.hip, pw_cm_forward_kernel
// SK = 1): the same kernel body with parts removed, timed with HIP events over 200 launches.
//   V0 full; V1 no MFMA (the loads kept alive by a VALU add); V2 no operand loads in the K loop;
//   V3 no epilogue (targets not read, g not written); V4 epilogue only; V5 V0 with 2x the waves
//   (16 output channels per wave: half the MFMA columns wasted, twice the latency hiding);
//   fwd2 V5: the targets prefetched before the K loop; V6: + 32 x 32 per wave (twice the waves).
// Standalone (no aimet_amd library):
//   hipcc -O3 --offload-arch=gfx950 -o build/pw_cm_probe tools/studies/pw_cm_probe.hip && ./build/pw_cm_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                   \
    do                                                                             \
    {                                                                              \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess)                                                      \
        {                                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

struct FastDiv
{
    uint32_t d, mul, shr;
    explicit FastDiv(uint32_t divisor) : d(divisor), mul(0), shr(0)
    {
        if (d > 1)
        {
            uint32_t l = 32 - __builtin_clz(d - 1);
            uint32_t p = 31 + l;
            mul        = (uint32_t) (((1ull << p) + d - 1) / d);
            shr        = p - 32;
        }
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const { return d == 1 ? n : (__umulhi(n, mul) >> shr); }
};

struct Batch
{
    const float* x;
    const int64_t* idx;
    uint32_t nb, Cin, Cout, hw, P;
    FastDiv div_hw;
};

template <int V>
__global__ __launch_bounds__(64) void fwd(Batch B, const float* __restrict__ target, const float* __restrict__ w,
                                          float* __restrict__ g, float* __restrict__ sink)
{
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const uint32_t co0 = blockIdx.y * 32, p0 = blockIdx.x * 64;
    const uint32_t pa = min(p0 + i, B.P - 1), pb = min(p0 + 32 + i, B.P - 1);
    const uint32_t ba = B.div_hw.div(pa), bb = B.div_hw.div(pb);
    const size_t ra = (size_t) B.idx[ba], rb = (size_t) B.idx[bb];
    const float* xa = B.x + ra * B.Cin * B.hw + (pa - ba * B.hw);
    const float* xb = B.x + rb * B.Cin * B.hw + (pb - bb * B.hw);
    const float* wr = w + (size_t) min(co0 + i, B.Cout - 1) * B.Cin;
    const uint32_t nch = B.Cin / 32;
    float a0[16], x0[16], y0[16], a1[16], x1[16], y1[16];
    auto load = [&](uint32_t c, float (&a)[16], float (&xv)[16], float (&yv)[16]) {
        const uint32_t k0 = c * 32;
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
        {
            const uint32_t k = k0 + 4 * s2 + 2 * h;
            if (V == 2)
            {
                a[2 * s2] = a[2 * s2 + 1] = (float) k;
                xv[2 * s2] = xv[2 * s2 + 1] = yv[2 * s2] = yv[2 * s2 + 1] = (float) lane;
                continue;
            }
            const float2 v = *reinterpret_cast<const float2*>(wr + k);
            a[2 * s2]      = v.x;
            a[2 * s2 + 1]  = v.y;
#pragma unroll
            for (int e = 0; e < 2; ++e)
            {
                xv[2 * s2 + e] = xa[(size_t) (k + e) * B.hw];
                yv[2 * s2 + e] = xb[(size_t) (k + e) * B.hw];
            }
        }
    };
    f32x16 acc0 = {}, acc1 = {};
    auto mfma = [&](const float (&a)[16], const float (&xv)[16], const float (&yv)[16]) {
#pragma unroll
        for (int st = 0; st < 16; ++st)
        {
            if (V == 1)
            {
                acc0[st] += a[st] * xv[st];
                acc1[st] += a[st] * yv[st];
            }
            else
            {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], xv[st], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], yv[st], acc1, 0, 0, 0);
            }
        }
    };
    if (V != 4)
    {
        uint32_t c = 0;
        load(c, a0, x0, y0);
        for (; c < nch; c += 2)
        {
            if (c + 1 < nch)
                load(c + 1, a1, x1, y1);
            mfma(a0, x0, y0);
            if (c + 1 >= nch)
                break;
            if (c + 2 < nch)
                load(c + 2, a0, x0, y0);
            mfma(a1, x1, y1);
        }
    }
    if (V == 3)
    {
        float s = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            s += acc0[r] + acc1[r];
        sink[blockIdx.y * gridDim.x * 64 + blockIdx.x * 64 + lane] = s;
        return;
    }
    const float* ta = target + ra * B.Cout * B.hw + (pa - ba * B.hw);
    const float* tb = target + rb * B.Cout * B.hw + (pb - bb * B.hw);
#pragma unroll
    for (int r = 0; r < 16; ++r)
    {
        const uint32_t co = co0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= B.Cout)
            continue;
        const float t0 = ta[(size_t) co * B.hw], t1 = tb[(size_t) co * B.hw];
        if (p0 + i < B.P)
            g[(size_t) co * B.P + p0 + i] = acc0[r] - t0;
        if (p0 + 32 + i < B.P)
            g[(size_t) co * B.P + p0 + 32 + i] = acc1[r] - t1;
    }
}

template <int V>
float time_it(const Batch& B, const float* t, const float* w, float* g, float* sink, int reps)
{
    dim3 grid((B.P + 63) / 64, (B.Cout + 31) / 32);
    for (int r = 0; r < 5; ++r)
        fwd<V><<<grid, 64>>>(B, t, w, g, sink);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
        fwd<V><<<grid, 64>>>(B, t, w, g, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / reps;
}


// V5/V6: targets prefetched before the K loop; V6 additionally 32 x 32 per wave (one accumulator,
// twice the waves)
template <int V>
__global__ __launch_bounds__(64) void fwd2(Batch B, const float* __restrict__ target, const float* __restrict__ w,
                                           float* __restrict__ g)
{
    constexpr int NP = V == 6 ? 32 : 64;   // positions per wave
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const uint32_t co0 = blockIdx.y * 32, p0 = blockIdx.x * NP;
    const uint32_t pa = min(p0 + i, B.P - 1), pb = min(p0 + 32 + i, B.P - 1);
    const uint32_t ba = B.div_hw.div(pa), bb = B.div_hw.div(pb);
    const size_t ra = (size_t) B.idx[ba], rb = (size_t) B.idx[bb];
    const float* xa = B.x + ra * B.Cin * B.hw + (pa - ba * B.hw);
    const float* xb = B.x + rb * B.Cin * B.hw + (pb - bb * B.hw);
    const float* wr = w + (size_t) min(co0 + i, B.Cout - 1) * B.Cin;
    const uint32_t nch = B.Cin / 32;
    float t0[16], t1[16];
    {
        const float* ta = target + ra * B.Cout * B.hw + (pa - ba * B.hw);
        const float* tb = target + rb * B.Cout * B.hw + (pb - bb * B.hw);
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const uint32_t co = min(co0 + (r & 3) + 8 * (r >> 2) + 4 * h, B.Cout - 1);
            t0[r]             = ta[(size_t) co * B.hw];
            if (NP == 64)
                t1[r] = tb[(size_t) co * B.hw];
        }
    }
    float a0[16], x0[16], y0[16], a1[16], x1[16], y1[16];
    auto load = [&](uint32_t c, float (&a)[16], float (&xv)[16], float (&yv)[16]) {
        const uint32_t k0 = c * 32;
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
        {
            const uint32_t k = k0 + 4 * s2 + 2 * h;
            const float2 v = *reinterpret_cast<const float2*>(wr + k);
            a[2 * s2]      = v.x;
            a[2 * s2 + 1]  = v.y;
#pragma unroll
            for (int e = 0; e < 2; ++e)
            {
                xv[2 * s2 + e] = xa[(size_t) (k + e) * B.hw];
                if (NP == 64)
                    yv[2 * s2 + e] = xb[(size_t) (k + e) * B.hw];
            }
        }
    };
    f32x16 acc0 = {}, acc1 = {};
    auto mfma = [&](const float (&a)[16], const float (&xv)[16], const float (&yv)[16]) {
#pragma unroll
        for (int st = 0; st < 16; ++st)
        {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], xv[st], acc0, 0, 0, 0);
            if (NP == 64)
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], yv[st], acc1, 0, 0, 0);
        }
    };
    uint32_t c = 0;
    load(c, a0, x0, y0);
    for (; c < nch; c += 2)
    {
        if (c + 1 < nch)
            load(c + 1, a1, x1, y1);
        mfma(a0, x0, y0);
        if (c + 1 >= nch)
            break;
        if (c + 2 < nch)
            load(c + 2, a0, x0, y0);
        mfma(a1, x1, y1);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r)
    {
        const uint32_t co = co0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= B.Cout)
            continue;
        if (p0 + i < B.P)
            g[(size_t) co * B.P + p0 + i] = acc0[r] - t0[r];
        if (NP == 64 && p0 + 32 + i < B.P)
            g[(size_t) co * B.P + p0 + 32 + i] = acc1[r] - t1[r];
    }
}

template <int V>
float time_it2(const Batch& B, const float* t, const float* w, float* g, int reps)
{
    constexpr int NP = V == 6 ? 32 : 64;
    dim3 grid((B.P + NP - 1) / NP, (B.Cout + 31) / 32);
    for (int r = 0; r < 5; ++r)
        fwd2<V><<<grid, 64>>>(B, t, w, g);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
        fwd2<V><<<grid, 64>>>(B, t, w, g);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / reps;
}

int main()
{
    const uint32_t shapes[][3] = {{64, 384, 196}, {384, 64, 196}, {160, 960, 49}, {960, 160, 49}};
    const uint32_t nb = 32, rows = 256;
    for (auto& sh : shapes)
    {
        const uint32_t Cin = sh[0], Cout = sh[1], hw = sh[2], P = nb * hw;
        float *x, *t, *w, *g, *sink;
        int64_t* idx;
        CHECK(hipMalloc(&x, sizeof(float) * rows * Cin * hw));
        CHECK(hipMalloc(&t, sizeof(float) * rows * Cout * hw));
        CHECK(hipMalloc(&w, sizeof(float) * Cout * Cin));
        CHECK(hipMalloc(&g, sizeof(float) * Cout * P));
        CHECK(hipMalloc(&sink, sizeof(float) * 64 * ((P + 63) / 64) * ((Cout + 31) / 32)));
        CHECK(hipMalloc(&idx, sizeof(int64_t) * nb));
        CHECK(hipMemset(x, 0, sizeof(float) * rows * Cin * hw));
        CHECK(hipMemset(t, 0, sizeof(float) * rows * Cout * hw));
        CHECK(hipMemset(w, 0, sizeof(float) * Cout * Cin));
        std::vector<int64_t> hidx(nb);
        for (uint32_t b = 0; b < nb; ++b)
            hidx[b] = (b * 97) % rows;
        CHECK(hipMemcpy(idx, hidx.data(), sizeof(int64_t) * nb, hipMemcpyHostToDevice));
        Batch B {x, idx, nb, Cin, Cout, hw, P, FastDiv(hw)};
        const int reps = 200;
        printf("{\"cin\": %u, \"cout\": %u, \"hw\": %u, \"waves\": %u, \"full_us\": %.2f, \"no_mfma_us\": %.2f, "
               "\"no_loads_us\": %.2f, \"no_epilogue_us\": %.2f, \"epilogue_only_us\": %.2f, \"prefetch_t_us\": %.2f, "
               "\"tile32x32_us\": %.2f}\n",
               Cin, Cout, hw, ((P + 63) / 64) * ((Cout + 31) / 32), time_it<0>(B, t, w, g, sink, reps),
               time_it<1>(B, t, w, g, sink, reps), time_it<2>(B, t, w, g, sink, reps),
               time_it<3>(B, t, w, g, sink, reps), time_it<4>(B, t, w, g, sink, reps), time_it2<5>(B, t, w, g, reps),
               time_it2<6>(B, t, w, g, reps));
        fflush(stdout);
        CHECK(hipFree(x));
        CHECK(hipFree(t));
        CHECK(hipFree(w));
        CHECK(hipFree(g));
        CHECK(hipFree(sink));
        CHECK(hipFree(idx));
    }
    return 0;
}
