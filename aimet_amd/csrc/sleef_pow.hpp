// sleef_pow.hpp -- torch's CPU pow(tensor, scalar) for float on the device, bit for bit: the
// emulation of Sleef_powf_u10 used by the AdaRound backward's rounding loss (adaround.hip).
// Device-only; also included by tools/studies/pow_cert_check.hip (ExpkTrace exposes the
// double-float values behind a result to that check).
#pragma once

#include <hip/hip_runtime.h>

namespace aimet_amd
{
namespace
{

// ---- torch's CPU pow(tensor, scalar) for float: Vectorized<float>::pow = Sleef_powf16_u10 (the
// AVX512F build: logkf with getexp / getmant in [0.75, 1.5), double-float arithmetic in FMA form,
// expkf), applied to all but the last (n mod 32) elements of the contiguous loop, which take the
// scalar std::pow (within glibc powf's 0.82 ulp: the correctly rounded result from double here).
// Every step below is an IEEE op, so the vector part is Sleef's bit for bit: 4.5 M elements x 40
// exponents equal to torch.pow on the CPU (tools/studies/sleef_powf_check.py).
struct F2
{
    float x, y;
};
__device__ __forceinline__ F2 f2(float x, float y)
{
    return F2 {x, y};
}
__device__ __forceinline__ float fmapn(float x, float y, float z)   // x * y - z
{
    return __builtin_fmaf(x, y, -z);
}
__device__ __forceinline__ float fmanp(float x, float y, float z)   // z - x * y
{
    return __builtin_fmaf(-x, y, z);
}
__device__ __forceinline__ F2 df_normalize(F2 t)
{
    const float s = t.x + t.y;
    return f2(s, (t.x - s) + t.y);
}
__device__ __forceinline__ F2 df_scale(F2 d, float s)
{
    return f2(d.x * s, d.y * s);
}
__device__ __forceinline__ F2 df_add2_ff(float x, float y)
{
    const float s = x + y, v = s - x;
    return f2(s, (x - (s - v)) + (y - v));
}
__device__ __forceinline__ F2 df_add2_f2f(F2 x, float y)
{
    const float s = x.x + y, v = s - x.x;
    const float t = (x.x - (s - v)) + (y - v);
    return f2(s, t + x.y);
}
__device__ __forceinline__ F2 df_add_f2f2(F2 x, F2 y)
{
    const float s = x.x + y.x;
    return f2(s, (((x.x - s) + y.x) + x.y) + y.y);
}
__device__ __forceinline__ F2 df_add2_f2f2(F2 x, F2 y)
{
    const float s = x.x + y.x, v = s - x.x;
    const float t = (x.x - (s - v)) + (y.x - v);
    return f2(s, t + (x.y + y.y));
}
__device__ __forceinline__ F2 df_add_ff2(float x, F2 y)
{
    const float s = x + y.x;
    return f2(s, ((x - s) + y.x) + y.y);
}
__device__ __forceinline__ F2 df_squ(F2 x)
{
    const float s = x.x * x.x;
    return f2(s, __builtin_fmaf(x.x + x.x, x.y, fmapn(x.x, x.x, s)));
}
__device__ __forceinline__ F2 df_mul_f2f2(F2 x, F2 y)
{
    const float s = x.x * y.x;
    return f2(s, __builtin_fmaf(x.x, y.y, __builtin_fmaf(x.y, y.x, fmapn(x.x, y.x, s))));
}
__device__ __forceinline__ F2 df_mul_f2f(F2 x, float y)
{
    const float s = x.x * y;
    return f2(s, __builtin_fmaf(x.y, y, fmapn(x.x, y, s)));
}
// Sleef's vrec (1.0f / d.x, the IEEE division) as v_rcp_f32 + one Newton step: equal to the
// division for every d.x in [1.5, 3] -- logkf's divisor 1 + m, m in [0.75, 1.5), lies in [1.75,
// 2.5] -- exhaustively over those 8,388,609 bit patterns on the MI355X
// (tools/studies/rcp_newton_check.hip; not for general d: it differs where 1/d is subnormal).
__device__ __forceinline__ F2 df_div(F2 n, F2 d)
{
    const float r0 = __builtin_amdgcn_rcpf(d.x);
    const float t  = __builtin_fmaf(__builtin_fmaf(-d.x, r0, 1.0f), r0, r0), s = n.x * t;
    const float u = fmapn(t, n.x, s);
    const float v = fmanp(d.y, t, fmanp(d.x, t, 1.0f));
    return f2(s, __builtin_fmaf(s, v, __builtin_fmaf(n.y, t, u)));
}
// logkf (AVX512 form) for a positive finite d
__device__ __forceinline__ F2 sleef_logkf(float d)
{
    int ee;
    (void) __builtin_frexpf(d * (1.0f / 0.75f), &ee);   // getexp: floor(log2(d / 0.75))
    const float e = (float) (ee - 1);
    int em;
    float m = __builtin_frexpf(d, &em) * 2.0f;          // getmant into [0.75, 1.5)
    if (m >= 1.5f)
        m *= 0.5f;
    // -1 + m is exact for m in [0.75, 1.5) (Sterbenz), so df_add2_ff(-1, m)'s error term is +0
    const F2 x  = df_div(f2(-1.0f + m, 0.0f), df_add2_ff(1.0f, m));
    const F2 x2 = df_squ(x);
    float t     = 0.240320354700088500976562f;
    t           = __builtin_fmaf(t, x2.x, 0.285112679004669189453125f);
    t           = __builtin_fmaf(t, x2.x, 0.400007992982864379882812f);
    const F2 c  = f2(0.66666662693023681640625f, 3.69183861259614332084311e-09f);
    F2 s        = df_mul_f2f(f2(0.69314718246459960938f, -1.904654323148236017e-09f), e);
    s           = df_add_f2f2(s, df_scale(x, 2.0f));
    return df_add_f2f2(s, df_mul_f2f2(df_mul_f2f2(x2, x), df_add2_f2f2(df_mul_f2f(x2, t), c)));
}
__device__ __forceinline__ float sleef_ldexp(float x, int q)
{
    int m = q >> 31;
    m     = (((m + q) >> 6) - m) << 4;
    q     = q - (m << 2);
    m     = 0x7f + m;
    m     = m < 0 ? 0 : (m > 0xff ? 0xff : m);
    float u = __int_as_float(m << 23);
    x       = x * u * u * u * u;
    return x * __int_as_float((q + 0x7f) << 23);
}
// the double-float values behind sleef_expkf's result, for the certification's check
// (tools/studies/pow_cert_check.hip): s after the reduction, t before its final f32 rounding
struct ExpkTrace
{
    double s, t;
    int q;
};
__device__ __forceinline__ float sleef_expkf(F2 d, ExpkTrace* tr = nullptr)
{
    float u     = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
    const int q = (int) __builtin_rintf(u);
    F2 s        = df_add2_f2f(d, (float) q * -0.693145751953125f);
    s           = df_add2_f2f(s, (float) q * -1.428606765330187045e-06f);
    s           = df_normalize(s);
    u           = 0.00136324646882712841033936f;
    u           = __builtin_fmaf(u, s.x, 0.00836596917361021041870117f);
    u           = __builtin_fmaf(u, s.x, 0.0416710823774337768554688f);
    u           = __builtin_fmaf(u, s.x, 0.166665524244308471679688f);
    u           = __builtin_fmaf(u, s.x, 0.499999850988388061523438f);
    F2 t        = df_add_f2f2(s, df_mul_f2f(df_squ(s), u));
    t           = df_add_ff2(1.0f, t);
    if (tr)
        *tr = ExpkTrace {(double) s.x + (double) s.y, (double) t.x + (double) t.y, q};
    // t in [0.7, 1.42]: for q in [-125, 126] the result is normal, where every step of
    // sleef_ldexp is an exact power-of-two scaling, i.e. the one-step ldexp
    u           = (q >= -125 && q <= 126) ? __builtin_ldexpf(t.x + t.y, q) : sleef_ldexp(t.x + t.y, q);
    return d.x < -104.0f ? 0.0f : u;
}

// x^e for x in [0, 1] as torch's CPU pow: e == 2 / 3 -> x*x / x*x*x (ATen's optimized kernel);
// Sleef_powf_u10 in the vectorized part, the correctly rounded value in the scalar tail (`tail`).
// Sleef's powf is expkf(logkf(|x|) * e): `l` = sleef_logkf(x), shared by the two exponents of the
// rounding loss and its gradient (one logkf per element instead of two; the same values).
__device__ __forceinline__ float pow01_log(float x, float e, bool tail, F2 l)
{
    if (e == 2.0f)
        return x * x;
    if (e == 3.0f)
        return x * x * x;
    if (x == 0.0f)
        return e == 0.0f ? 1.0f : 0.0f;
    if (e == 0.0f || x == 1.0f)
        return 1.0f;
    if (tail)
        return (float) exp((double) e * log((double) x));
    const float r = sleef_expkf(df_mul_f2f(l, e));
    return r != r ? __builtin_inff() : r;
}

// ---- the same pow for two elements at once (packed f32: v_pk_fma / v_pk_mul / v_pk_add) ------
// Every operation below is the scalar path's, component by component (packed f32 instructions are
// the IEEE ops per component), so each component is bit-identical to pow01_log / sleef_logkf /
// sleef_expkf; the few non-arithmetic steps (frexp, rint, ldexp, rcp) run per component. ~110 of the
// ~142 VALU instructions of one scalar pow are packable adds, multiplies and FMAs, so a pair costs
// ~87 per element instead of 142: the dense waves of the backward (alpha mostly unsaturated, early
// in an AdaRound loop) evaluate their elements two at a time.
typedef float fl2 __attribute__((ext_vector_type(2)));
struct V2
{
    fl2 x, y;
};
__device__ __forceinline__ fl2 vfma(fl2 a, fl2 b, fl2 c)
{
    return __builtin_elementwise_fma(a, b, c);
}
__device__ __forceinline__ fl2 vsplat(float v)
{
    return fl2 {v, v};
}
__device__ __forceinline__ V2 v2(fl2 x, fl2 y)
{
    return V2 {x, y};
}
__device__ __forceinline__ V2 vdf_normalize(V2 t)
{
    const fl2 s = t.x + t.y;
    return v2(s, (t.x - s) + t.y);
}
__device__ __forceinline__ V2 vdf_add2_ff(fl2 x, fl2 y)
{
    const fl2 s = x + y, v = s - x;
    return v2(s, (x - (s - v)) + (y - v));
}
__device__ __forceinline__ V2 vdf_add2_f2f(V2 x, fl2 y)
{
    const fl2 s = x.x + y, v = s - x.x;
    const fl2 t = (x.x - (s - v)) + (y - v);
    return v2(s, t + x.y);
}
__device__ __forceinline__ V2 vdf_add_f2f2(V2 x, V2 y)
{
    const fl2 s = x.x + y.x;
    return v2(s, (((x.x - s) + y.x) + x.y) + y.y);
}
__device__ __forceinline__ V2 vdf_add2_f2f2(V2 x, V2 y)
{
    const fl2 s = x.x + y.x, v = s - x.x;
    const fl2 t = (x.x - (s - v)) + (y.x - v);
    return v2(s, t + (x.y + y.y));
}
__device__ __forceinline__ V2 vdf_add_ff2(fl2 x, V2 y)
{
    const fl2 s = x + y.x;
    return v2(s, ((x - s) + y.x) + y.y);
}
__device__ __forceinline__ V2 vdf_squ(V2 x)
{
    const fl2 s = x.x * x.x;
    return v2(s, vfma(x.x + x.x, x.y, vfma(x.x, x.x, -s)));
}
__device__ __forceinline__ V2 vdf_mul_f2f2(V2 x, V2 y)
{
    const fl2 s = x.x * y.x;
    return v2(s, vfma(x.x, y.y, vfma(x.y, y.x, vfma(x.x, y.x, -s))));
}
__device__ __forceinline__ V2 vdf_mul_f2f(V2 x, fl2 y)
{
    const fl2 s = x.x * y;
    return v2(s, vfma(x.y, y, vfma(x.x, y, -s)));
}
__device__ __forceinline__ V2 vdf_div(V2 n, V2 d)
{
    const fl2 r0 = fl2 {__builtin_amdgcn_rcpf(d.x.x), __builtin_amdgcn_rcpf(d.x.y)};
    const fl2 t  = vfma(vfma(-d.x, r0, vsplat(1.0f)), r0, r0), s = n.x * t;
    const fl2 u  = vfma(t, n.x, -s);
    const fl2 v  = vfma(-d.y, t, vfma(-d.x, t, vsplat(1.0f)));
    return v2(s, vfma(s, v, vfma(n.y, t, u)));
}
__device__ __forceinline__ V2 vsleef_logkf(fl2 d)
{
    fl2 e, m;
#pragma unroll
    for (int c = 0; c < 2; ++c)
    {
        int ee, em;
        (void) __builtin_frexpf(d[c] * (1.0f / 0.75f), &ee);
        e[c]     = (float) (ee - 1);
        float mc = __builtin_frexpf(d[c], &em) * 2.0f;
        m[c]     = mc >= 1.5f ? mc * 0.5f : mc;
    }
    const V2 x  = vdf_div(v2(vsplat(-1.0f) + m, vsplat(0.0f)), vdf_add2_ff(vsplat(1.0f), m));
    const V2 x2 = vdf_squ(x);
    fl2 t       = vsplat(0.240320354700088500976562f);
    t           = vfma(t, x2.x, vsplat(0.285112679004669189453125f));
    t           = vfma(t, x2.x, vsplat(0.400007992982864379882812f));
    const V2 c  = v2(vsplat(0.66666662693023681640625f), vsplat(3.69183861259614332084311e-09f));
    V2 s        = vdf_mul_f2f(v2(vsplat(0.69314718246459960938f), vsplat(-1.904654323148236017e-09f)), e);
    s           = vdf_add_f2f2(s, v2(x.x * 2.0f, x.y * 2.0f));
    return vdf_add_f2f2(s, vdf_mul_f2f2(vdf_mul_f2f2(x2, x), vdf_add2_f2f2(vdf_mul_f2f(x2, t), c)));
}
__device__ __forceinline__ fl2 vsleef_expkf(V2 d)
{
    const fl2 u0 = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
    fl2 qf;
    int q[2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
    {
        q[c]  = (int) __builtin_rintf(u0[c]);
        qf[c] = (float) q[c];
    }
    V2 s = vdf_add2_f2f(d, qf * -0.693145751953125f);
    s    = vdf_add2_f2f(s, qf * -1.428606765330187045e-06f);
    s    = vdf_normalize(s);
    fl2 u = vsplat(0.00136324646882712841033936f);
    u     = vfma(u, s.x, vsplat(0.00836596917361021041870117f));
    u     = vfma(u, s.x, vsplat(0.0416710823774337768554688f));
    u     = vfma(u, s.x, vsplat(0.166665524244308471679688f));
    u     = vfma(u, s.x, vsplat(0.499999850988388061523438f));
    V2 t  = vdf_add_f2f2(s, vdf_mul_f2f(vdf_squ(s), u));
    t     = vdf_add_ff2(vsplat(1.0f), t);
    const fl2 tv = t.x + t.y;
    fl2 r;
#pragma unroll
    for (int c = 0; c < 2; ++c)
    {
        const float rc = (q[c] >= -125 && q[c] <= 126) ? __builtin_ldexpf(tv[c], q[c]) : sleef_ldexp(tv[c], q[c]);
        r[c]           = d.x[c] < -104.0f ? 0.0f : rc;
    }
    return r;
}
// pow01_log for two elements known to need the logarithm or the tail's double pow (|x| not 0 or
// 1): `l` = vsleef_logkf(x); components marked `tail` take the double pow
__device__ __forceinline__ fl2 vpow01_log(fl2 x, float e, bool tail0, bool tail1, V2 l)
{
    fl2 r;
    if (e == 2.0f)
        r = x * x;
    else if (e == 3.0f)
        r = x * x * x;
    else
    {
        r = vsleef_expkf(vdf_mul_f2f(l, vsplat(e)));
#pragma unroll
        for (int c = 0; c < 2; ++c)
        {
            const float xc = x[c];
            float rc       = r[c] != r[c] ? __builtin_inff() : r[c];
            if (xc == 0.0f)
                rc = e == 0.0f ? 1.0f : 0.0f;
            else if (e == 0.0f || xc == 1.0f)
                rc = 1.0f;
            else if (c == 0 ? tail0 : tail1)
                rc = (float) exp((double) e * log((double) xc));
            r[c] = rc;
        }
    }
    return r;
}

}   // namespace
}   // namespace aimet_amd
