// Exhaustive check of the library's fast pow (aimet_amd/csrc/fast_pow.hpp: pow01_fast, the
// table-driven f32 form; round 6's first form evaluated ln / exp in f64: pow_fast_check_f64.txt)
// against the bit-exact emulation of torch's CPU pow (aimet_amd/csrc/sleef_pow.hpp: pow01_log over
// sleef_logkf, equal to torch.pow on the CPU: tests/test_adaround_golden.py,
// tools/studies/sleef_powf_check.py).
//
// For every f32 x in (0, 1) (1,065,353,215 values: subnormals included) and every exponent of
//   * the default AdaRound schedule (10,000 iterations, warm start 0.2, beta 20 -> 2: the 8,000
//     post-warm-start betas and beta - 1, as float),
//   * a 1,000-iteration schedule (800 betas and beta - 1),
//   * 4,000 exponents drawn uniformly from [0.5, 25] (seed 1),
// it counts the (x, e) pairs where the two results are equal, 1 ulp apart, or farther (must be 0),
// and -- for the first `cr_exps` exponents -- how far each lies from the correctly rounded x^e
// (double-precision exp(e log x), rounded once). Then times both forms on 2^26 random x.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         --offload-arch=gfx950 -I aimet_amd/csrc tools/studies/pow_fast_check.hip -o tools/studies/pow_fast_check
//   tools/studies/pow_fast_check [max_exponents] [cr_exps]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "fast_pow.hpp"
#include "sleef_pow.hpp"

using namespace aimet_amd;

#define CK(x)                                                                                                  \
    do                                                                                                         \
    {                                                                                                          \
        hipError_t e_ = (x);                                                                                   \
        if (e_ != hipSuccess)                                                                                  \
        {                                                                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                     \
            std::exit(1);                                                                                      \
        }                                                                                                      \
    } while (0)

struct Stats
{
    unsigned long long pairs, equal, one, more;          // fast vs Sleef
    unsigned long long cr_pairs, fast_cr, sleef_cr;     // != the correctly rounded value (cr exponents)
    unsigned max_ulp, max_fast_cr, max_sleef_cr;
    unsigned bad_x, bad_e;                              // a pair more than 1 ulp apart
};

constexpr int kThreads    = 256;
constexpr uint32_t kXEnd  = 0x3F800000u;   // x bits in [1, 0x3F800000): every f32 in (0, 1)

__device__ __forceinline__ unsigned ulps(float a, float b)
{
    const int d = (int) __float_as_uint(a) - (int) __float_as_uint(b);   // a, b >= 0 finite (or +inf)
    return (unsigned) (d < 0 ? -d : d);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ unsigned wave_maxu(unsigned v)
{
    for (int o = 32; o > 0; o >>= 1)
        v = max(v, (unsigned) __shfl_xor((int) v, o));
    return v;
}

__global__ __launch_bounds__(kThreads) void check_kernel(const float* __restrict__ exps, int ne, int ncr, uint32_t x0,
                                                         Stats* st)
{
    pow_tab_fill<kThreads>();
    __syncthreads();
    const uint32_t xb = x0 + blockIdx.x * kThreads + threadIdx.x;
    unsigned long long pairs = 0, eq = 0, one = 0, more = 0, crp = 0, fcr = 0, scr = 0;
    unsigned mx = 0, mf = 0, ms = 0;
    if (xb >= 1u && xb < kXEnd)
    {
        const float x  = __uint_as_float(xb);
        const F2 l     = sleef_logkf(x);
        const double L = log((double) x);
        for (int k = 0; k < ne; ++k)
        {
            const float e = exps[k];
            const float s = pow01_log(x, e, false, l);
            const float f = pow01_fast(x, e);
            const unsigned u = ulps(f, s);
            ++pairs;
            eq += u == 0;
            one += u == 1;
            if (u > 1)
            {
                ++more;
                st->bad_x = xb;
                st->bad_e = __float_as_uint(e);
            }
            mx = max(mx, u);
            if (k < ncr)
            {
                const float c = (float) exp((double) e * L);
                ++crp;
                const unsigned uf = ulps(f, c), us = ulps(s, c);
                fcr += uf != 0;
                scr += us != 0;
                mf = max(mf, uf);
                ms = max(ms, us);
            }
        }
    }
    __shared__ unsigned long long ssum[7][kThreads / 64];
    __shared__ unsigned smax[3][kThreads / 64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned long long v[7] = {wave_sum(pairs), wave_sum(eq), wave_sum(one), wave_sum(more),
                                     wave_sum(crp), wave_sum(fcr), wave_sum(scr)};
    const unsigned m[3] = {wave_maxu(mx), wave_maxu(mf), wave_maxu(ms)};
    if (lane == 0)
    {
        for (int j = 0; j < 7; ++j)
            ssum[j][w] = v[j];
        for (int j = 0; j < 3; ++j)
            smax[j][w] = m[j];
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        unsigned long long S[7] = {};
        unsigned M[3] = {};
        for (int i = 0; i < kThreads / 64; ++i)
        {
            for (int j = 0; j < 7; ++j)
                S[j] += ssum[j][i];
            for (int j = 0; j < 3; ++j)
                M[j] = max(M[j], smax[j][i]);
        }
        atomicAdd(&st->pairs, S[0]);
        atomicAdd(&st->equal, S[1]);
        atomicAdd(&st->one, S[2]);
        atomicAdd(&st->more, S[3]);
        atomicAdd(&st->cr_pairs, S[4]);
        atomicAdd(&st->fast_cr, S[5]);
        atomicAdd(&st->sleef_cr, S[6]);
        atomicMax(&st->max_ulp, M[0]);
        atomicMax(&st->max_fast_cr, M[1]);
        atomicMax(&st->max_sleef_cr, M[2]);
    }
}

__global__ __launch_bounds__(kThreads) void time_sleef(const float* __restrict__ x, float* __restrict__ y, int n, float e)
{
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n)
        y[i] = pow01_log(x[i], e, false, sleef_logkf(x[i]));
}
__global__ __launch_bounds__(kThreads) void time_fast(const float* __restrict__ x, float* __restrict__ y, int n, float e)
{
    pow_tab_fill<kThreads>();
    __syncthreads();
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n)
        y[i] = pow01_fast(x[i], e);
}

static std::vector<float> schedule(int iters, double warm, double b0, double b1)
{
    std::vector<float> v;
    const double ws = warm * iters;
    for (int it = (int) std::ceil(ws); it < iters; ++it)
    {
        const double rel  = (it - ws) / (iters - ws);
        const double beta = b1 + 0.5 * (b0 - b1) * (1.0 + std::cos(rel * M_PI));
        for (float e : {(float) beta, (float) (beta - 1.0)})
            if (e != 2.0f && e != 3.0f && e != 0.0f)
                v.push_back(e);
    }
    return v;
}

int main(int argc, char** argv)
{
    std::vector<float> exps = schedule(10000, 0.2, 20.0, 2.0);
    const size_t n_default  = exps.size();
    for (float e: schedule(1000, 0.2, 20.0, 2.0))
        exps.push_back(e);
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(0.5f, 25.0f);
    for (int i = 0; i < 4000; ++i)
    {
        const float e = U(rng);
        if (e != 2.0f && e != 3.0f)
            exps.push_back(e);
    }
    if (argc > 1)
        exps.resize(std::min(exps.size(), (size_t) std::atol(argv[1])));
    const int ncr = argc > 2 ? std::atoi(argv[2]) : 64;
    // the correctly-rounded comparison takes exponents spread over the whole list
    std::vector<float> ordered;
    const size_t stride = std::max<size_t>(1, exps.size() / std::max(1, ncr));
    std::vector<char> taken(exps.size(), 0);
    for (size_t i = 0; i < exps.size() && (int) ordered.size() < ncr; i += stride)
    {
        ordered.push_back(exps[i]);
        taken[i] = 1;
    }
    for (size_t i = 0; i < exps.size(); ++i)
        if (!taken[i])
            ordered.push_back(exps[i]);
    std::printf("exponents: %zu (default schedule %zu; the first %d also against the correctly rounded value), "
                "x values: %u\n", ordered.size(), n_default, ncr, kXEnd - 1);
    float* d_exps;
    Stats* d_st;
    CK(hipMalloc(&d_exps, ordered.size() * sizeof(float)));
    CK(hipMemcpy(d_exps, ordered.data(), ordered.size() * sizeof(float), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_st, sizeof(Stats)));
    CK(hipMemset(d_st, 0, sizeof(Stats)));
    // exponents in chunks, x in slices: every launch bounded (a few seconds at most)
    const int kChunk       = 256;
    const uint32_t kSlice  = 1u << 26;
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventRecord(t0, nullptr));
    for (size_t e0 = 0; e0 < ordered.size(); e0 += kChunk)
    {
        const int ne  = (int) std::min<size_t>(kChunk, ordered.size() - e0);
        const int ncr_chunk = (int) std::max<long>(0, std::min<long>(ne, (long) ncr - (long) e0));
        for (uint32_t x0 = 0; x0 < kXEnd; x0 += kSlice)
        {
            const uint32_t n = std::min(kSlice, kXEnd - x0);
            check_kernel<<<(n + kThreads - 1) / kThreads, kThreads>>>(d_exps + e0, ne, ncr_chunk, x0, d_st);
            CK(hipGetLastError());
        }
        CK(hipDeviceSynchronize());
        if ((e0 / kChunk) % 16 == 0)
        {
            Stats h;
            CK(hipMemcpy(&h, d_st, sizeof(Stats), hipMemcpyDeviceToHost));
            std::printf("  exponents done %zu: pairs %llu, 1 ulp apart %llu, farther %llu\n",
                        e0 + ne, h.pairs, h.one, h.more);
            std::fflush(stdout);
        }
    }
    CK(hipEventRecord(t1, nullptr));
    CK(hipEventSynchronize(t1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t0, t1));
    Stats h;
    CK(hipMemcpy(&h, d_st, sizeof(Stats), hipMemcpyDeviceToHost));
    std::printf("pairs %llu in %.1f s\n", h.pairs, ms / 1e3);
    std::printf("fast == Sleef: %llu (%.4f %%); 1 ulp apart: %llu (%.4f %%); farther: %llu; max %u ulp\n", h.equal,
                100.0 * h.equal / h.pairs, h.one, 100.0 * h.one / h.pairs, h.more, h.max_ulp);
    if (h.more)
        std::printf("  e.g. x = %a, e = %a\n", (double) __builtin_bit_cast(float, h.bad_x),
                    (double) __builtin_bit_cast(float, h.bad_e));
    std::printf("against the correctly rounded x^e (%llu pairs): fast differs %llu (%.4f %%, max %u ulp), "
                "Sleef differs %llu (%.4f %%, max %u ulp)\n", h.cr_pairs, h.fast_cr, 100.0 * h.fast_cr / h.cr_pairs,
                h.max_fast_cr, h.sleef_cr, 100.0 * h.sleef_cr / h.cr_pairs, h.max_sleef_cr);
    // timing: 2^26 x uniform in (0.01, 0.99)
    const int N = 1 << 26;
    std::vector<float> hx(N);
    std::uniform_real_distribution<float> X(0.01f, 0.99f);
    for (auto& v: hx)
        v = X(rng);
    float *dx, *dy;
    CK(hipMalloc(&dx, N * sizeof(float)));
    CK(hipMalloc(&dy, N * sizeof(float)));
    CK(hipMemcpy(dx, hx.data(), N * sizeof(float), hipMemcpyHostToDevice));
    for (float e: {19.0f, 10.5f, 1.25f})
    {
        float best[2] = {1e30f, 1e30f};
        for (int rep = 0; rep < 5; ++rep)
            for (int form = 0; form < 2; ++form)
            {
                CK(hipEventRecord(t0, nullptr));
                if (form == 0)
                    time_sleef<<<N / kThreads, kThreads>>>(dx, dy, N, e);
                else
                    time_fast<<<N / kThreads, kThreads>>>(dx, dy, N, e);
                CK(hipEventRecord(t1, nullptr));
                CK(hipEventSynchronize(t1));
                CK(hipEventElapsedTime(&ms, t0, t1));
                best[form] = std::min(best[form], ms);
            }
        std::printf("e = %g: Sleef emulation %.3f ms, fast pow %.3f ms for 2^26 pows\n", e, best[0], best[1]);
    }
    return h.more ? 2 : 0;
}
