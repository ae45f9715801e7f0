// entropy_core.hpp -- the entropy analyzer's histogram arithmetic (TensorProfilingParams,
// math_functions.cpp:470-560), shared by the device statistics kernels (stats.hip) and the host
// KL search (encodings.cpp).
//
// The reference bins with static_cast<size_t>((value - min) / binWidth) in float and clamps to
// the last bin (getBin, math_functions.cpp:470-474). Its results for out-of-range quotients are
// those of the x86-64 float -> uint64 conversion gcc emits (cvttss2si, with a 2^63 bias branch):
// NaN and quotients <= -1 land in the LAST bin, quotients >= 2^64 in bin 0. Those conversions are
// restated here explicitly so the device reproduces them.
#pragma once

#include <cstdint>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define AIMET_ENT_HD __host__ __device__ __forceinline__
#else
#define AIMET_ENT_HD inline
#endif

namespace aimet_amd
{
namespace entropy
{

constexpr int kBins = 512;   // PDF_SIZE

// (size_t) f on x86-64 (gcc): f < 2^63 (or NaN) -> cvttss2si(f); else cvttss2si(f - 2^63) ^ 2^63.
// cvttss2si yields 0x8000000000000000 for NaN and out-of-range inputs.
AIMET_ENT_HD uint64_t x86_f2u64(float f)
{
    const uint64_t indefinite = 0x8000000000000000ull;
    if (f >= 9223372036854775808.0f)
    {
        float r = f - 9223372036854775808.0f;   // exact
        return (r >= 9223372036854775808.0f) ? 0ull : ((uint64_t) (int64_t) r ^ indefinite);
    }
    if (f >= -9223372036854775808.0f)           // false for NaN
        return (uint64_t) (int64_t) f;
    return indefinite;
}

// the same for double (cvttsd2si)
AIMET_ENT_HD uint64_t x86_d2u64(double f)
{
    const uint64_t indefinite = 0x8000000000000000ull;
    if (f >= 9223372036854775808.0)
    {
        double r = f - 9223372036854775808.0;
        return (r >= 9223372036854775808.0) ? 0ull : ((uint64_t) (int64_t) r ^ indefinite);
    }
    if (f >= -9223372036854775808.0)
        return (uint64_t) (int64_t) f;
    return indefinite;
}

// min((size_t) q, 511) for the quotient q = (value - min) / binWidth
AIMET_ENT_HD int bin_of_quotient(float q)
{
    if (q > -1.0f && q < (float) kBins)
        return (int) q;   // truncation toward zero: (-1, 0] -> 0
    uint64_t b = x86_f2u64(q);
    return b < (uint64_t) (kBins - 1) ? (int) b : kBins - 1;
}

// getBin(PDF_SIZE, binWidth, minValue, value), math_functions.cpp:470-474
AIMET_ENT_HD int get_bin(float binWidth, float minValue, float value)
{
    if (binWidth == 0)
        return 0;
    return bin_of_quotient((value - minValue) / binWidth);
}

#ifdef __HIPCC__
// getBin for a channel's fixed (binWidth, min) with the division replaced by a reciprocal
// multiply where that cannot change the result. q' = RN(s * RN(1/w)) is within 3.0001 ulp of the
// reference's q* = RN(s / w); truncation (and the -1 / 512 clamps) can only differ when an integer
// lies between them, so whenever q' is farther than 2^-20 (|q'| + 1) from the nearest integer the
// bin is the same. Otherwise -- and for every non-finite quotient -- the IEEE division decides.
struct Binner
{
    float width, lo, rcp;
    int zero_width;
    __device__ Binner(float w, float mn) : width(w), lo(mn), rcp(1.0f / w), zero_width(w == 0.0f) {}
    __device__ __forceinline__ int bin(float x) const
    {
        if (zero_width)
            return 0;
        const float s   = x - lo;
        const float q   = s * rcp;
        const float fr  = __builtin_fabsf(q - __builtin_rintf(q));
        const float thr = (__builtin_fabsf(q) + 1.0f) * 9.5367431640625e-7f;   // 2^-20
        if (__builtin_expect(fr > thr, 1))   // q finite and off every integer
            return (q > -1.0f && q < (float) kBins) ? (int) q : (q >= 18446744073709551616.0f ? 0 : kBins - 1);
        return bin_of_quotient(s / width);
    }
};
#endif

}   // namespace entropy
}   // namespace aimet_amd
