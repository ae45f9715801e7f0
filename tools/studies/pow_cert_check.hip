// A certified f64 evaluation of torch's CPU pow (cert_logk / cert_expk / pow01_cert, below) checked
// exhaustively against the library's exact Sleef emulation (aimet_amd/csrc/sleef_pow.hpp: sleef_logkf /
// sleef_expkf / pow01_log, itself bit-equal to torch's CPU pow: tests/test_adaround_golden.py,
// tools/studies/sleef_powf_check.py). Result (profiles/r05/pow_cert_check.txt): bit-exact wherever it
// certifies, 99.8 % certified on x uniform in (0, 1) -- and no faster than the exact emulation on
// MI355X, where an f64 FMA and an f32 <-> f64 conversion each issue at half the f32 FMA's rate
// (tools/studies/valu_rates.hip), so it stays out of the library.
//
// For every f32 x in (0, 1) (1,065,353,215 values) and every exponent of
//   * the default AdaRound schedule (10,000 iterations, warm start 0.2, beta 20 -> 2: the 8,000
//     post-warm-start betas and beta - 1, as float),
//   * a 1,000-iteration schedule (800 betas and beta - 1),
//   * 4,000 exponents drawn uniformly from [0.5, 25] (seed 1),
// it counts the certified inputs and those whose certified result differs from pow01_log (must be 0),
// and records the largest deviation of the f64 values from Sleef's double-float values relative to
// the bounds the certification assumes (< 1 needed; the margin is what the bound argument leaves).
// Then times both forms on 2^26 random x in (0.01, 0.99).
//
//   hipcc -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         --offload-arch=gfx950 -I aimet_amd/csrc tools/studies/pow_cert_check.hip -o tools/studies/pow_cert_check
//   tools/studies/pow_cert_check [max_exponents]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "sleef_pow.hpp"

using namespace aimet_amd;

namespace
{
// ---- certified evaluation: the same powf mostly in f64 ----------------------------------------
// MI355X issues an f64 FMA at the rate of an f32 one, so the double-float pairs of Sleef's logkf /
// expkf (3-10 f32 operations per step) cost more than f64 arithmetic holding the same value to
// 2^-53. The certified form evaluates Sleef's formula with
//   * every f32 step whose result Sleef feeds to an f32 polynomial or to its exponent choice done
//     exactly as sleef_logkf / sleef_expkf do it (the divisor's reciprocal, x.x, x2.x and the
//     polynomial t; q; the polynomial u), and
//   * the double-float accumulations in f64: D ~ d = logkf(x) * e, S ~ s = d - q ln2, T ~ t = 1 + s +
//     s^2 u, the value Sleef rounds to f32 last.
// Bounds on the distance to Sleef's double-float values:
//   |D - d| <= 2^-43 |D|       -- |L - logkf(x)| <= 2^-45 |L| over EVERY f32 x in (0, 1) (measured
//                                 exhaustively), plus the product's own 2^-46.9
//   |S - s| <= bS = 2^-42.5 |D| + 2^-52        (the two Cody-Waite steps add <= 2^-45.8 |D|)
//   |T - t| <= 1.5 bS + 2^-44 [+ s^2 2^-22.3 when s.x is not certified, below]
// Sleef rounds d to f32 (for q), s (for the polynomial u) and t (the result). Wherever D lies
// farther than its bound from an f32 rounding midpoint, q is Sleef's; wherever S does, u is Sleef's
// bit for bit -- otherwise the two u differ by at most 2^-22.3 (two f32 Horner evaluations of the
// same polynomial on neighbouring inputs), which moves t by at most s^2 2^-22.3 (small exactly where
// s's own rounding is uncertain: small |s|); and wherever T lies farther than its bound from a
// midpoint, Sleef's final rounding gives (float) T. Then the result is Sleef's bit for bit (`ok`);
// otherwise (~0.2 % of the inputs of an AdaRound backward) the caller evaluates pow01_log.
// This file checks every f32 x in (0, 1) x 21,600 exponents (the default
// schedule's among them): certified == pow01_log wherever certified, and the measured deviations
// sit inside the bounds (profiles/r05/pow_cert_check.txt).
constexpr double kCertLn2 = (double) 0.69314718246459960938f + (double) -1.904654323148236017e-09f;   // exact sum
constexpr double kCertC   = (double) 0.66666662693023681640625f + (double) 3.69183861259614332084311e-09f;

// distance of v's f64 mantissa from the f32 rounding midpoint of its binade, in units of v's f64
// ulp (0 .. 2^28). For a bound K < 2^27 of those units (so that a value below a power of two stays
// above the midpoint under it), dist > K means every value within K ulps of v rounds to f32 as v.
__device__ __forceinline__ float cert_dist(double v)
{
    const int lo = (int) ((uint32_t) __double_as_longlong(v) & 0x1FFFFFFFu) - 0x10000000;
    return (float) (lo < 0 ? -lo : lo);
}

// Sleef's logkf(x) for x in (0, 1) as an f64 value (sleef_logkf's formula, f32 steps exact)
__device__ __forceinline__ double cert_logk(float d)
{
    int ee;
    (void) __builtin_frexpf(d * (1.0f / 0.75f), &ee);
    const float e = (float) (ee - 1);
    int em;
    float m = __builtin_frexpf(d, &em) * 2.0f;
    if (m >= 1.5f)
        m *= 0.5f;
    const float n   = -1.0f + m;                                 // exact
    const float dx  = 1.0f + m;                                  // the divisor's f32 part
    const float r0  = __builtin_amdgcn_rcpf(dx);
    const float t   = __builtin_fmaf(__builtin_fmaf(-dx, r0, 1.0f), r0, r0);   // 1 / dx (df_div)
    const float s   = n * t;                                     // Sleef's x.x
    const float x2x = s * s;                                     // Sleef's x2.x
    float tp        = __builtin_fmaf(0.240320354700088500976562f, x2x, 0.285112679004669189453125f);
    tp              = __builtin_fmaf(tp, x2x, 0.400007992982864379882812f);
    // x = n / (1 + m): one Newton correction of s in f64 (n - s (1 + m) is exact), |X - x| < 2^-46 |x|
    const double sd = (double) s;
    const double X  = fma(fma(-sd, (double) m + 1.0, (double) n), (double) t, sd);
    const double X2 = X * X;
    return fma((double) e, kCertLn2, fma(2.0, X, X2 * X * fma(X2, (double) tp, kCertC)));
}

// the f64 values behind cert_expk's result (for tools/studies/pow_cert_check.hip)
struct CertTrace
{
    double S, T;
    int q;
    bool s_cert;   // S certified (u is Sleef's bit for bit)
    int why;       // 0 certified, 1 D / range, 2 T
};
// Sleef's expkf for d ~ D (f64), certified: ok when the result is provably sleef_expkf(d)
__device__ __forceinline__ float cert_expk(double D, bool& ok, CertTrace* tr = nullptr)
{
    const float dd = (float) D;                                  // Sleef: d.x + d.y in f32
    const float ad = __builtin_fabsf(dd);
    const int q    = (int) __builtin_rintf(dd * 1.442695040888963407359924681001892137426645954152985934135449406931f);
    const float qf = (float) q;
    const double S = fma((double) qf, -0.693145751953125, D) + (double) (qf * -1.428606765330187045e-06f);
    const float sx = (float) S;                                  // Sleef's s.x when certified
    float u        = 0.00136324646882712841033936f;
    u              = __builtin_fmaf(u, sx, 0.00836596917361021041870117f);
    u              = __builtin_fmaf(u, sx, 0.0416710823774337768554688f);
    u              = __builtin_fmaf(u, sx, 0.166665524244308471679688f);
    u              = __builtin_fmaf(u, sx, 0.499999850988388061523438f);
    const double T = fma(S * S, (double) u, S) + 1.0;
    // the roundings against their bounds in f64-ulp units (ulp64(v) >= |v| 2^-53; T >= 0.7):
    // D: 2^-43 |D| -> 2^10; S: bS 2^53 / |S| = (2^10.5 |D| + 2) / |S|; T: (1.5 bS + 2^-44) 2^53 / 0.7,
    // + s^2 2^-22.3 2^53 / 0.7 = s^2 2^31.2 when S is not certified
    const float as     = __builtin_fabsf(sx);
    const float kS     = __builtin_fmaf(1448.155f, ad, 2.0f);
    const bool s_cert  = kS < 0x1p26f * as && cert_dist(S) * as > kS;
    const float kT     = __builtin_fmaf(3103.2f, ad, 736.0f) + (s_cert ? 0.0f : sx * sx * 2.5e9f);
    // q <= 126 (the result is finite); |D| < 2^7 keeps q * ln2's f32 split exact; D away from -104,
    // Sleef's flush to zero (decided on d.x, within 2^-23 |d| of D)
    const bool d_cert = ad < 128.0f && q <= 126 && __builtin_fabsf(dd + 104.0f) > 0.001f && cert_dist(D) > 1024.0f;
    const bool t_cert = kT < 0x1p26f && cert_dist(T) > kT;
    ok                = d_cert && t_cert;
    if (tr)
        *tr = CertTrace {S, T, q, s_cert, !d_cert ? 1 : (!t_cert ? 2 : 0)};
    const float tv = (float) T;
    const float r  = q >= -125 ? __builtin_ldexpf(tv, q) : sleef_ldexp(tv, q);
    return dd < -104.0f ? 0.0f : r;
}

// pow01_log(x, e, false, .) for x in (0, 1) and e not in {0, 2, 3}, certified (see above); L = cert_logk(x)
__device__ __forceinline__ float pow01_cert(double L, float e, bool& ok)
{
    return cert_expk(L * (double) e, ok);
}
}   // namespace

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
    unsigned long long evaluated, certified, mismatched, q_mismatched_certified, why_d, why_t;
    unsigned rL, rD, rS, rT;   // float bit patterns of the largest ratios (non-negative: uint order)
    unsigned bad_x, bad_e;     // first mismatch found (bit patterns)
};

constexpr int kThreads = 256;
constexpr uint32_t kXEnd = 0x3F800000u;   // x in [2^-149, 1)

__device__ __forceinline__ float wave_max(float v)
{
    for (int o = 32; o > 0; o >>= 1)
        v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}

// grid = false: x = every f32 bit pattern in (0, 1); grid = true: x = k 2^-24, k = 1 .. 2^24 - 1 (uniform
// in value, as |2h - 1| of an AdaRound alpha roughly is)
__global__ __launch_bounds__(kThreads) void check_kernel(const float* __restrict__ exps, int ne, Stats* st, bool grid)
{
    const uint32_t k0 = 1u + blockIdx.x * kThreads + threadIdx.x;
    const uint32_t xb = grid ? __float_as_uint((float) k0 * 0x1p-24f) : k0;
    unsigned long long ev = 0, ce = 0, mm = 0, qm = 0, wd = 0, wt = 0;
    float rL = 0.0f, rD = 0.0f, rS = 0.0f, rT = 0.0f;
    if (grid ? k0 < (1u << 24) : k0 < kXEnd)
    {
        const float x   = __uint_as_float(xb);
        const F2 l      = sleef_logkf(x);
        const double L  = cert_logk(x);
        const double ls = (double) l.x + (double) l.y;
        rL              = (float) (fabs(L - ls) / (0x1p-41 * fabs(L)));
        for (int k = 0; k < ne; ++k)
        {
            const float e = exps[k];
            const F2 d    = df_mul_f2f(l, e);
            ExpkTrace te;
            float exact = sleef_expkf(d, &te);
            exact       = exact != exact ? __builtin_inff() : exact;
            bool ok;
            CertTrace tc;
            const double D  = L * (double) e;
            const float c   = cert_expk(D, ok, &tc);
            const double ds = (double) d.x + (double) d.y;
            const double bS = 0x1p-43 * 1.4142135623730951 * fabs(D) + 0x1p-52;
            if (fabs(D) < 128.0 && tc.q <= 126)
                rD = fmaxf(rD, (float) (fabs(D - ds) / (0x1p-43 * fabs(D))));
            if (tc.q == te.q && fabs(D) < 128.0 && tc.q <= 126)
            {
                const double sx = (double) (float) tc.S;
                rS = fmaxf(rS, (float) (fabs(tc.S - te.s) / bS));
                rT = fmaxf(rT, (float) (fabs(tc.T - te.t) /
                                        (1.5 * bS + 0x1p-44 + (tc.s_cert ? 0.0 : sx * sx * 0x1p-22 * 0.8122523963562356))));
            }
            wd += tc.why == 1;
            wt += tc.why == 2;
            ++ev;
            if (ok)
            {
                ++ce;
                if (__float_as_uint(c) != __float_as_uint(exact))
                {
                    ++mm;
                    st->bad_x = xb;
                    st->bad_e = __float_as_uint(e);
                }
                if (tc.q != te.q)
                    ++qm;
            }
        }
    }
    __shared__ float smax[4][kThreads / 64];
    __shared__ unsigned long long ssum[6][kThreads / 64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float m0 = wave_max(rL), m1 = wave_max(rD), m2 = wave_max(rS), m3 = wave_max(rT);
    const unsigned long long s0 = wave_sum(ev), s1 = wave_sum(ce), s2 = wave_sum(mm), s3 = wave_sum(qm), s4 = wave_sum(wd),
                             s5 = wave_sum(wt);
    if (lane == 0)
    {
        smax[0][w] = m0, smax[1][w] = m1, smax[2][w] = m2, smax[3][w] = m3;
        ssum[0][w] = s0, ssum[1][w] = s1, ssum[2][w] = s2, ssum[3][w] = s3, ssum[4][w] = s4, ssum[5][w] = s5;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float M[4] = {0, 0, 0, 0};
        unsigned long long S[6] = {0, 0, 0, 0, 0, 0};
        for (int i = 0; i < kThreads / 64; ++i)
        {
            for (int j = 0; j < 4; ++j)
                M[j] = fmaxf(M[j], smax[j][i]);
            for (int j = 0; j < 6; ++j)
                S[j] += ssum[j][i];
        }
        atomicAdd(&st->evaluated, S[0]);
        atomicAdd(&st->certified, S[1]);
        atomicAdd(&st->mismatched, S[2]);
        atomicAdd(&st->q_mismatched_certified, S[3]);
        atomicAdd(&st->why_d, S[4]);
        atomicAdd(&st->why_t, S[5]);
        atomicMax(&st->rL, __float_as_uint(M[0]));
        atomicMax(&st->rD, __float_as_uint(M[1]));
        atomicMax(&st->rS, __float_as_uint(M[2]));
        atomicMax(&st->rT, __float_as_uint(M[3]));
    }
}

__global__ __launch_bounds__(kThreads) void time_exact(const float* __restrict__ x, float* __restrict__ y, int n, float e)
{
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n)
        y[i] = pow01_log(x[i], e, false, sleef_logkf(x[i]));
}
__global__ __launch_bounds__(kThreads) void time_cert(const float* __restrict__ x, float* __restrict__ y, int n, float e)
{
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n)
    {
        bool ok;
        float r = pow01_cert(cert_logk(x[i]), e, ok);
        if (!ok)
            r = pow01_log(x[i], e, false, sleef_logkf(x[i]));
        y[i] = r;
    }
}

__global__ __launch_bounds__(kThreads) void time_cert_only(const float* __restrict__ x, float* __restrict__ y, int n, float e)
{
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n)
    {
        bool ok;
        const float r = pow01_cert(cert_logk(x[i]), e, ok);
        y[i]          = ok ? r : -r;
    }
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
    const size_t n_default = exps.size();
    for (float e : schedule(1000, 0.2, 20.0, 2.0))
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
    // the f64 constants are the exact sums of Sleef's pairs
    if (kCertLn2 - (double) 0.69314718246459960938f != (double) -1.904654323148236017e-09f ||
        kCertC - (double) 0.66666662693023681640625f != (double) 3.69183861259614332084311e-09f)
    {
        std::printf("constant pair not exact\n");
        return 1;
    }
    std::printf("exponents: %zu (default schedule %zu), x values: %u\n", exps.size(), n_default, kXEnd - 1);
    float* d_exps;
    Stats* d_st;
    CK(hipMalloc(&d_exps, exps.size() * sizeof(float)));
    CK(hipMemcpy(d_exps, exps.data(), exps.size() * sizeof(float), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_st, sizeof(Stats)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto f = [](unsigned u) {
        float v;
        std::memcpy(&v, &u, 4);
        return v;
    };
    unsigned long long total_mismatched = 0;
    for (int grid_mode = 1; grid_mode >= 0; --grid_mode)
    {
        std::printf("== x = %s\n", grid_mode ? "k 2^-24, k = 1 .. 2^24 - 1 (uniform in value)" : "every f32 in (0, 1)");
        CK(hipMemset(d_st, 0, sizeof(Stats)));
        const int chunk     = grid_mode ? 1024 : 64;
        const unsigned nx   = grid_mode ? (1u << 24) - 1 : kXEnd - 1;
        const unsigned grid = (nx + kThreads - 1) / kThreads;
        CK(hipEventRecord(a));
        for (size_t k0 = 0; k0 < exps.size(); k0 += chunk)
        {
            const int ne = (int) std::min((size_t) chunk, exps.size() - k0);
            check_kernel<<<grid, kThreads>>>(d_exps + k0, ne, d_st, grid_mode != 0);
            CK(hipGetLastError());
            if ((k0 / chunk) % 16 == 15 || k0 + chunk >= exps.size())
            {
                CK(hipDeviceSynchronize());
                Stats s;
                CK(hipMemcpy(&s, d_st, sizeof(Stats), hipMemcpyDeviceToHost));
                std::printf("  exponents done %zu: evaluated %llu certified %llu mismatched %llu\n", k0 + ne, s.evaluated,
                            s.certified, s.mismatched);
                std::fflush(stdout);
                if (s.mismatched)
                    break;
            }
        }
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        Stats s;
        CK(hipMemcpy(&s, d_st, sizeof(Stats), hipMemcpyDeviceToHost));
        total_mismatched += s.mismatched;
        std::printf("evaluated %llu (x, e) pairs in %.1f s\n", s.evaluated, ms / 1e3);
        std::printf("certified %llu (%.4f %%); rejected on D / range %.4f %%, on T %.4f %%\n", s.certified,
                    100.0 * s.certified / s.evaluated, 100.0 * s.why_d / s.evaluated, 100.0 * s.why_t / s.evaluated);
        std::printf("certified but != pow01_log: %llu", s.mismatched);
        if (s.mismatched)
            std::printf(" (first: x bits 0x%08x, e %.9g)", s.bad_x, f(s.bad_e));
        std::printf("\ncertified with q != Sleef's q: %llu\n", s.q_mismatched_certified);
        std::printf("largest |L - logkf| / (2^-41 |L|)                 : %.4g\n", f(s.rL));
        std::printf("largest |D - d| / (2^-43 |D|)                      : %.4g  (|D| < 128, q <= 126; assumed <= 1)\n", f(s.rD));
        std::printf("largest |S - s| / (2^-42.5 |D| + 2^-52)            : %.4g  (same q; assumed <= 1)\n", f(s.rS));
        std::printf("largest |T - t| / (1.5 bS + 2^-44 [+ s^2 2^-22.3]) : %.4g  (same q; assumed <= 1)\n", f(s.rT));
        std::fflush(stdout);
        if (s.mismatched)
            break;
    }

    // throughput of the two forms
    const int n = 1 << 26;
    std::vector<float> hx(n);
    std::uniform_real_distribution<float> X(0.01f, 0.99f);
    for (auto& v : hx)
        v = X(rng);
    float *dx, *y0, *y1;
    CK(hipMalloc(&dx, n * sizeof(float)));
    CK(hipMalloc(&y0, n * sizeof(float)));
    CK(hipMalloc(&y1, n * sizeof(float)));
    CK(hipMemcpy(dx, hx.data(), n * sizeof(float), hipMemcpyHostToDevice));
    for (float e : {19.0f, 10.5f, 1.25f})
    {
        float t[3];
        for (int form = 0; form < 3; ++form)
        {
            auto kern = form == 0 ? time_exact : (form == 1 ? time_cert : time_cert_only);
            float* y  = form == 0 ? y0 : y1;
            for (int rep = 0; rep < 2; ++rep)
                kern<<<n / kThreads, kThreads>>>(dx, y, n, e);
            CK(hipEventRecord(a));
            for (int rep = 0; rep < 20; ++rep)
                kern<<<n / kThreads, kThreads>>>(dx, y, n, e);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&t[form], a, b));
            t[form] /= 20;
            if (form == 1)
            {
                std::vector<float> h0(n), h1(n);
                CK(hipMemcpy(h0.data(), y0, n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h1.data(), y1, n * 4, hipMemcpyDeviceToHost));
                if (std::memcmp(h0.data(), h1.data(), (size_t) n * 4) != 0)
                    std::printf("e = %g: OUTPUTS DIFFER\n", e);
            }
        }
        std::vector<float> h1(n);
        CK(hipMemcpy(h1.data(), y1, n * 4, hipMemcpyDeviceToHost));
        size_t rej = 0;
        for (float v : h1)
            rej += std::signbit(v);
        std::printf("e = %g: exact %.3f ms, certified + fallback %.3f ms, certified alone %.3f ms for 2^26 pows "
                    "(rejected %.4f %%)\n", e, t[0], t[1], t[2], 100.0 * rej / n);
    }
    return total_mismatched ? 2 : 0;
}
