// fast_pow.hpp -- x^e for x in (0, 1) in f32 arithmetic with small tables: the AdaRound rounding
// loss's pow (adaround_loss.py:83-110; torch's CPU pow = Sleef powf_u10) within 1 ulp of torch's.
//
// torch's CPU pow is Sleef's powf_u10: expkf(logkf(x) * e) in double-float (f32 pairs), ~142 f32
// instructions per element (sleef_pow.hpp reproduces it bit for bit). The result only has to be
// within 1 ulp of Sleef's, and Sleef's error is below 1 ulp, so any pow whose own error stays below
// 1 ulp qualifies (two results on the f32 grid closer than 2 ulps to the same value differ by at
// most 1 ulp); this one keeps its error below ~0.3 ulp before the final rounding, in ~33 f32
// instructions and 2 LDS reads:
//   ln x = k ln2 + ln m (x = m 2^k, m in [0.5, 1)); m's top 7 fraction bits pick c = 1 / m_j and
//   tau = -ln c from a 128-entry table, so ln m = tau + ln(1 + r), r = m c - 1 (one FMA, rounded:
//   |r| <= 2^-8, error <= 2^-33), ln(1 + r) = r + r^2 (-1/2 + r/3 - r^2/4) (truncation 2^-42);
//   A = k LN2_HI + tau_hi is exact in f32 (both multiples of 2^-17, |A| < 2^7), the rest
//   L = (r + p) + (k LN2_LO + tau_lo) carries ~2^-32 of error;
//   y = e ln x as yh + yl = e A (exact two-product) + e L; exp(y) = 2^n 2^(i/32) exp(rr) with
//   N = rint((yh + yl) 32 / ln2) = 32 n + i, rr = yh - N ln2/32 + yl (|rr| <= ~ln2/64, error
//   ~2^-28), exp(rr) - 1 = rr + rr^2 (1/2 + rr/6) (truncation 2^-31), and the result
//   eh + (eh em1 + el) rounded once, scaled by 2^n (exact unless subnormal, like Sleef's own
//   final scaling).
// For e <= 20 the value before the final rounding is within ~2^-26.5 of x^e (relative). Checked
// exhaustively -- every f32 x in (0, 1) x the AdaRound exponent schedules -- against the
// bit-exact Sleef emulation by tools/studies/pow_fast_check.hip (profiles/r06/pow_fast_check.txt).
// The tables (fast_pow_tab.hpp, tools/gen_pow_tab.py: exact decimal arithmetic) are copied into
// LDS once per workgroup (pow_tab_load / pow_tab_store) and read per element with per-lane indices.
#pragma once

#include <hip/hip_runtime.h>

#include "fast_pow_tab.hpp"

namespace aimet_amd
{
namespace
{

typedef float f4t __attribute__((ext_vector_type(4)));
typedef float f2t __attribute__((ext_vector_type(2)));

// the tables in LDS: every kernel that evaluates the fast pow fills them first (pow_tab_fill or
// pow_tab_load + pow_tab_store, then a workgroup barrier)
__shared__ __attribute__((aligned(16))) PowTab g_pow_tab;

// the workgroup's BLOCK threads copy the tables into LDS in two halves, so that a kernel can issue
// its own first loads between them: pow_tab_load (global -> registers), then pow_tab_store
// (registers -> LDS); the caller synchronises the workgroup after the store
template <int BLOCK>
struct PowTabPart
{
    static constexpr int kParts = (kPowTabFloats + BLOCK - 1) / BLOCK;
    float v[kParts];
};

template <int BLOCK>
__device__ __forceinline__ PowTabPart<BLOCK> pow_tab_load()
{
    const float* src = reinterpret_cast<const float*>(&kPowTab);
    PowTabPart<BLOCK> t;
#pragma unroll
    for (int k = 0; k < PowTabPart<BLOCK>::kParts; ++k)
    {
        const int i = (int) threadIdx.x + k * BLOCK;
        t.v[k]      = i < kPowTabFloats ? src[i] : 0.0f;
    }
    return t;
}

template <int BLOCK>
__device__ __forceinline__ void pow_tab_store(const PowTabPart<BLOCK>& t)
{
    float* dst = reinterpret_cast<float*>(&g_pow_tab);
#pragma unroll
    for (int k = 0; k < PowTabPart<BLOCK>::kParts; ++k)
    {
        const int i = (int) threadIdx.x + k * BLOCK;
        if (i < kPowTabFloats)
            dst[i] = t.v[k];
    }
}

template <int BLOCK>
__device__ __forceinline__ void pow_tab_fill()
{
    pow_tab_store<BLOCK>(pow_tab_load<BLOCK>());
}

// ln x = a + l for x in (0, 1) (normal or subnormal), a exact, |error| <= ~2^-31
struct LnSplit
{
    float a, l;
};

__device__ __forceinline__ LnSplit ln01(float x)
{
    const int k     = __builtin_amdgcn_frexp_expf(x);
    const float m   = __builtin_amdgcn_frexp_mantf(x);   // [0.5, 1)
    const uint32_t j = (__float_as_uint(m) >> 16) & 127u;
    const f4t e     = *reinterpret_cast<const f4t*>(g_pow_tab.ln[j]);   // one 16-B LDS read
    const float r   = __builtin_fmaf(m, e.x, -1.0f);
    float t         = __builtin_fmaf(r, -0.25f, 0.333333343f);
    t               = __builtin_fmaf(r, t, -0.5f);
    const float p   = (r * r) * t;
    const float kf  = (float) k;
    const float a   = __builtin_fmaf(kf, kLn2Hi, e.y);   // exact
    const float b   = __builtin_fmaf(kf, kLn2Lo, e.z);
    return LnSplit {a, (r + p) + b};
}

// exp(e ln x) rounded to f32, for ln x = l.a + l.l and e in (0, 64] (the error bound above holds
// for e <= 20; it grows with e)
__device__ __forceinline__ float exp_ln(LnSplit l, float e)
{
    const float yh = e * l.a;
    float yl       = __builtin_fmaf(e, l.a, -yh);   // exact: e A = yh + this
    yl             = __builtin_fmaf(e, l.l, yl);
    const float nf = __builtin_rintf((yh + yl) * kK32Ln2);
    const int n    = (int) nf;
    float rr       = __builtin_fmaf(nf, -kCh, yh);
    rr             = rr + yl;
    rr             = __builtin_fmaf(nf, -kCl, rr);
    const float t  = __builtin_fmaf(rr, 0.166666672f, 0.5f);
    const float em = __builtin_fmaf(rr * rr, t, rr);   // exp(rr) - 1
    const f2t x    = *reinterpret_cast<const f2t*>(g_pow_tab.ex[(uint32_t) n & 31u]);   // {eh, el}: one 8-B read
    const float v  = x.x + __builtin_fmaf(x.x, em, x.y);
    // y >= 64 ln(2^-149), so n > -10000: below 2^-149 the scaled value is +0, as x^e is
    return __builtin_ldexpf(v, n >> 5);
}

// x^e for x in (0, 1), e in (0, 64]
__device__ __forceinline__ float powf01_fast(float x, float e)
{
    return exp_ln(ln01(x), e);
}

// x^e with x = |2h - 1| in [0, 1] (or NaN) for the rounding loss, `l` = ln01(x) (any value where
// x is 0 or 1): the exact cases of torch's pow as sleef_pow.hpp's pow01_log returns them (e == 2 /
// 3: ATen's x*x / x*x*x; x == 0; e == 0 or x == 1: 1; a NaN result: inf), the rest exp_ln (the
// reference's scalar tail too: within 1 ulp of glibc powf's correctly rounded value as of Sleef's)
__device__ __forceinline__ float pow01_fast_l(float x, float e, LnSplit l)
{
    if (e == 2.0f)
        return x * x;
    if (e == 3.0f)
        return x * x * x;
    if (x == 0.0f)
        return e == 0.0f ? 1.0f : 0.0f;
    if (e == 0.0f || x == 1.0f)
        return 1.0f;
    const float r = exp_ln(l, e);
    return r != r ? __builtin_inff() : r;
}

__device__ __forceinline__ float pow01_fast(float x, float e)
{
    return pow01_fast_l(x, e, ln01(x));
}

}   // namespace
}   // namespace aimet_amd
