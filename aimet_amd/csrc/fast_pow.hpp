// fast_pow.hpp -- x^e for x in (0, 1) in f64 arithmetic: the AdaRound rounding loss's pow
// (adaround_loss.py:83-110; torch's CPU pow = Sleef powf_u10) within 1 ulp of torch's result.
//
// torch's CPU pow is Sleef's powf_u10: expkf(logkf(x) * e) in double-float (f32 pairs), ~142 f32
// instructions per element (sleef_pow.hpp reproduces it bit for bit). On MI355X an f64 FMA issues
// at half the rate of an f32 one (profiles/r05/valu_rates.txt) and carries 53 bits, so the same
// function in plain f64 arithmetic is ~30 instructions: x = 2^k m, m in [sqrt(1/2), sqrt(2)),
// ln m = 2 atanh(t) with t = (m - 1) / (m + 1) (a degree-4 polynomial in t^2, |t| <= 0.1716),
// y = e (k ln 2 + ln m), then exp(y) = 2^n exp(r), |r| <= ln2 / 2 (a degree-7 polynomial), rounded
// to f32 once. The coefficients are Chebyshev fits (mpmath.chebyfit, 40 digits, rounded to double):
// |ln m error| <= 1.5e-12, |exp(r) relative error| <= 6e-11, so for e <= 25 the value before the
// final rounding lies within ~2^-33 of x^e (relative): the f32 result is the correctly rounded one
// except within 2^-9 ulp of a rounding midpoint, and within 1 ulp of Sleef's (whose error is < 1
// ulp). Checked exhaustively -- every f32 x in (0, 1) x the AdaRound exponent schedules -- against
// the bit-exact Sleef emulation by tools/studies/pow_fast_check.hip (profiles/r06/pow_fast_check.txt).
#pragma once

#include <hip/hip_runtime.h>

namespace aimet_amd
{
namespace
{

// ln x for x in (0, 1) (normal or subnormal), |error| <= 1.5e-12 + 2^-52 |ln x|
__device__ __forceinline__ double ln01(float x)
{
    int k;
    float mf = __builtin_frexpf(x, &k);   // x = mf 2^k, mf in [0.5, 1)
    if (mf < 0.70710678f)
    {
        mf *= 2.0f;
        k -= 1;
    }
    const double m = (double) mf;            // [sqrt(1/2), sqrt(2))
    const double a = m + 1.0, b = m - 1.0;   // exact
    double r       = __builtin_amdgcn_rcp(a);
    r              = __builtin_fma(__builtin_fma(-a, r, 1.0), r, r);   // one Newton step: 2^-50
    const double t = b * r;
    const double s = t * t;
    double p       = 0.23616359099145984;
    p              = __builtin_fma(p, s, 0.2853505103781631);
    p              = __builtin_fma(p, s, 0.4000038467237519);
    p              = __builtin_fma(p, s, 0.6666666524748752);
    p              = __builtin_fma(p, s, 2.0000000000083595);
    return __builtin_fma((double) k, 0.6931471805599453, t * p);
}

// exp(l e) rounded to f32, for l = ln01(x) and e in (0, 64] (l e <= 0)
__device__ __forceinline__ float exp_ln(double l, float e)
{
    const double y = l * (double) e;
    // exp(y) = 2^n exp(rr): n = rint(y / ln 2), rr = y - n ln2 (ln 2 split: n ln2_hi exact for |n| < 2^11)
    const double n = __builtin_rint(y * 1.4426950408889634);
    double rr      = __builtin_fma(n, -6.93147180369123816490e-01, y);
    rr             = __builtin_fma(n, -1.90821492927058770002e-10, rr);
    double q       = 0.00019907569310848288;
    q              = __builtin_fma(q, rr, 0.0013948578326459795);
    q              = __builtin_fma(q, rr, 0.008333283538708528);
    q              = __builtin_fma(q, rr, 0.041666218319291945);
    q              = __builtin_fma(q, rr, 0.16666666786308587);
    q              = __builtin_fma(q, rr, 0.5000000107729166);
    q              = __builtin_fma(q, rr, 0.999999999995509);
    q              = __builtin_fma(q, rr, 0.9999999999595618);
    // 2^n: y >= 64 ln(2^-149) > -6700, so n > -9700 and the scaled value underflows to +0 in
    // double (and then in float) below 2^-1074, as x^e does below f32's 2^-150
    return (float) __builtin_ldexp(q, n < -2000.0 ? -2000 : (int) n);
}

// x^e for x in (0, 1), e in (0, 64]: x^e rounded from f64
__device__ __forceinline__ float powf01_f64(float x, float e)
{
    return exp_ln(ln01(x), e);
}

// x^e with x = |2h - 1| in [0, 1] (or NaN) for the rounding loss, `l` = ln01(x) (any value where
// x is 0 or 1): the exact cases of torch's pow as sleef_pow.hpp's pow01_log returns them (e == 2 /
// 3: ATen's x*x / x*x*x; x == 0; e == 0 or x == 1: 1; a NaN result: inf), the rest exp_ln (the
// reference's scalar tail too: within glibc powf's 0.82 ulp of the correctly rounded value as the
// vector part is within Sleef's)
__device__ __forceinline__ float pow01_fast_l(float x, float e, double l)
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
