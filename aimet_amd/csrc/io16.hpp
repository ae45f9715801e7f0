// io16.hpp -- fp16 / bf16 <-> fp32 element conversions of the 16-bit I/O kernels, exactly as
// torch's .to(torch.float32) (exact) and .to(torch.float16 / torch.bfloat16) (round to nearest
// even; bf16 NaN -> 0x7FC0) compute them.
#pragma once

#include <hip/hip_fp16.h>

#include <cstdint>

namespace aimet_amd
{

enum IoType
{
    IO_F32  = 0,
    IO_F16  = 1,
    IO_BF16 = 2
};

template <int IO>
__device__ __forceinline__ float to_f32(unsigned short u)
{
    if constexpr (IO == IO_F16)
        return __half2float(__ushort_as_half(u));
    else
        return __uint_as_float((uint32_t) u << 16);
}

// MAYBE_NAN = false: the caller knows f is not NaN (a QDQ output with finite delta and offset is
// delta * (integer + offset): finite or +-inf), so the bf16 NaN canonicalisation is skipped
template <int IO, bool MAYBE_NAN = true>
__device__ __forceinline__ unsigned short from_f32(float f)
{
    // The empty asm pins f as an fp32 VGPR value: without it the backend folds
    // fptrunc(fmul(a, b)) into v_fma_mix{lo,hi}_f16(a, b, 0), which rounds the exact product
    // straight to fp16 (no fp32 rounding first: differs from torch's two-step cast near fp16
    // rounding boundaries) and adds +0 (turns a -0 result into +0).
    asm("" : "+v"(f));
    if constexpr (IO == IO_F16)
        return __half_as_ushort(__float2half_rn(f));
    else
    {
        // c10::BFloat16 round_to_nearest_even (c10/util/BFloat16.h): RNE = gfx950's
        // v_cvt_pk_bf16_f32; torch maps every NaN to 0x7FC0
        const unsigned short h = __builtin_bit_cast(unsigned short, (__bf16) f);
        if constexpr (!MAYBE_NAN)
            return h;
        return f != f ? (unsigned short) 0x7FC0 : h;
    }
}


}   // namespace aimet_amd
