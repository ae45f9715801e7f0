// qdq16.hip -- fp16 / bf16 I/O variants of the QDQ and STE kernels.
//
// Reference: a half / bfloat16 tensor is upcast (`tensor.to(torch.float32)`), quantize-dequantized
// by the fp32 kernel and cast back (`.to(orig dtype)`): v1/tensor_quantizer.py:1116-1139 and
// :1141-1168, i.e. three full passes (2+4, 4+4, 4+2 B/elem = 20 B/elem). Here the conversions
// happen in registers: 2 B in + 2 B out per element (4 B/elem), one 16-B vector of
// eight elements per lane. Results are identical to the three-pass sequence: the upcast is exact,
// the fp32 arithmetic is the same (common.hpp), and the downcast is round-to-nearest-even as
// torch's (c10::Half via the hardware cvt, c10::BFloat16 round_to_nearest_even with NaN -> 0x7FC0).
// The STE backward compares float(x) with the float32 bounds (torch type promotion) and returns
// grad * mask in the grad dtype.
#include "common.hpp"
#include "io16.hpp"

#include <cstdlib>

namespace aimet_amd
{
namespace
{

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// thr = qdq_round_thr(p, rcp) (common.hpp), hoisted by the callers out of their element loops
template <bool STOCHASTIC>
__device__ __forceinline__ float qdq(float x, const QdqParams& p, uint64_t seed, uint64_t idx, float rcp, float thr)
{
    float q;
    if constexpr (STOCHASTIC)
        q = quantize_stochastic(x, p, seed, idx);
    else
        q = qdq_round_fast(glibc_fmaxf(glibc_fminf(x, p.max), p.min), p, rcp, thr);
    return dequantize(q, p);
}

struct ChannelMap16
{
    FastDiv divK, divC;
    uint32_t C;
    __device__ __forceinline__ uint32_t channel(uint32_t i) const
    {
        uint32_t row = divK.div(i);
        return row - divC.div(row) * C;
    }
};

__device__ __forceinline__ QdqParams table_params(const float* __restrict__ t, uint32_t C, uint32_t c)
{
    return QdqParams {t[c], t[C + c], t[2 * C + c], t[3 * C + c]};
}

// per-tensor (CH = false, params in SGPRs) / per-channel (CH = true, K % 8 == 0): one 8-element
// 16-B vector per lane, one tile per workgroup, streaming loads/stores
template <int IO, bool CH, bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void qdq16_vec_kernel(const u16x8* __restrict__ in, u16x8* __restrict__ out,
                                                           int64_t nvec, QdqParams p, ChannelMap16 map,
                                                           const float* __restrict__ table, uint64_t seed)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    if constexpr (CH)
        p = table_params(table, map.C, map.channel((uint32_t) (i * 8)));
    u16x8 v = __builtin_nontemporal_load(in + i), r;
    const uint64_t e = (uint64_t) i * 8;
    const float rcp  = 1.0f / p.delta;
    const float thr  = qdq_round_thr(p, rcp);
    if (__builtin_isfinite(p.delta) && __builtin_isfinite(p.offset))
    {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            r[k] = from_f32<IO, false>(qdq<STOCHASTIC>(to_f32<IO>(v[k]), p, seed, e + k, rcp, thr));
    }
    else
    {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            r[k] = from_f32<IO>(qdq<STOCHASTIC>(to_f32<IO>(v[k]), p, seed, e + k, rcp, thr));
    }
    __builtin_nontemporal_store(r, out + i);
}

template <int IO, bool CH, bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void qdq16_scalar_kernel(const unsigned short* __restrict__ in,
                                                              unsigned short* __restrict__ out, int64_t begin,
                                                              int64_t n, QdqParams p, int64_t C, int64_t K,
                                                              const float* __restrict__ table, uint64_t seed)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    {
        QdqParams q = p;
        if constexpr (CH)
            q = table_params(table, (uint32_t) C, (uint32_t) ((i / K) % C));
        const float rcp = 1.0f / q.delta;
        out[i] = from_f32<IO>(qdq<STOCHASTIC>(to_f32<IO>(in[i]), q, seed, (uint64_t) i, rcp, qdq_round_thr(q, rcp)));
    }
}

template <int IO>
__device__ __forceinline__ unsigned short ste16(unsigned short x, unsigned short g, float mn, float mx)
{
    const float xf = to_f32<IO>(x);
    return from_f32<IO>(to_f32<IO>(g) * ((mn <= xf && xf <= mx) ? 1.0f : 0.0f));
}

template <int IO, bool CH>
__global__ __launch_bounds__(kBlock) void ste16_vec_kernel(const u16x8* __restrict__ x, const u16x8* __restrict__ g,
                                                           u16x8* __restrict__ gi, int64_t nvec, float smin,
                                                           float smax, ChannelMap16 map,
                                                           const float* __restrict__ mins,
                                                           const float* __restrict__ maxs)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    float mn = smin, mx = smax;
    if constexpr (CH)
    {
        const uint32_t c = map.channel((uint32_t) (i * 8));
        mn               = mins[c];
        mx               = maxs[c];
    }
    u16x8 a = __builtin_nontemporal_load(x + i), b = __builtin_nontemporal_load(g + i), r;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        r[k] = ste16<IO>(a[k], b[k], mn, mx);
    __builtin_nontemporal_store(r, gi + i);
}

template <int IO, bool CH>
__global__ __launch_bounds__(kBlock) void ste16_scalar_kernel(const unsigned short* __restrict__ x,
                                                              const unsigned short* __restrict__ g,
                                                              unsigned short* __restrict__ gi, int64_t begin,
                                                              int64_t n, float smin, float smax, int64_t C, int64_t K,
                                                              const float* __restrict__ mins,
                                                              const float* __restrict__ maxs)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    {
        float mn = smin, mx = smax;
        if constexpr (CH)
        {
            const int64_t c = (i / K) % C;
            mn              = mins[c];
            mx              = maxs[c];
        }
        gi[i] = ste16<IO>(x[i], g[i], mn, mx);
    }
}

bool aligned16(const void* a, const void* b, const void* c = nullptr)
{
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) ==
           0;
}

// vector part over [0, nvec*8), scalar tail (per-tensor) or everything scalar (K % 8 != 0)
template <int IO, bool CH, bool STO>
void launch_qdq16(const void* in, void* out, int64_t n, const QdqParams& p, int64_t C, int64_t K, const float* table,
                  uint64_t seed, hipStream_t s)
{
    const bool vec_ok = aligned16(in, out) && (!CH || (K % 8 == 0 && n < (int64_t(1) << 32)));
    int64_t nvec      = vec_ok ? n / 8 : 0;
    if (nvec > 0)
    {
        ChannelMap16 map {FastDiv((uint32_t) (CH ? K : 1)), FastDiv((uint32_t) (CH ? C : 1)), (uint32_t) C};
        qdq16_vec_kernel<IO, CH, STO><<<(unsigned) ceil_div(nvec, kBlock), kBlock, 0, s>>>(
            reinterpret_cast<const u16x8*>(in), reinterpret_cast<u16x8*>(out), nvec, p, map, table, seed);
        AIMET_LAUNCH_CHECK();
    }
    if (nvec * 8 < n)
    {
        qdq16_scalar_kernel<IO, CH, STO><<<stream_blocks(n - nvec * 8, kBlock), kBlock, 0, s>>>(
            static_cast<const unsigned short*>(in), static_cast<unsigned short*>(out), nvec * 8, n, p, C, K, table,
            seed);
        AIMET_LAUNCH_CHECK();
    }
}

template <int IO, bool CH>
void launch_ste16(const void* x, const void* g, void* gi, int64_t n, float mn, float mx, int64_t C, int64_t K,
                  const float* mins, const float* maxs, hipStream_t s)
{
    const bool vec_ok = aligned16(x, g, gi) && (!CH || (K % 8 == 0 && n < (int64_t(1) << 32)));
    int64_t nvec      = vec_ok ? n / 8 : 0;
    if (nvec > 0)
    {
        ChannelMap16 map {FastDiv((uint32_t) (CH ? K : 1)), FastDiv((uint32_t) (CH ? C : 1)), (uint32_t) C};
        ste16_vec_kernel<IO, CH><<<(unsigned) ceil_div(nvec, kBlock), kBlock, 0, s>>>(
            reinterpret_cast<const u16x8*>(x), reinterpret_cast<const u16x8*>(g), reinterpret_cast<u16x8*>(gi), nvec,
            mn, mx, map, mins, maxs);
        AIMET_LAUNCH_CHECK();
    }
    if (nvec * 8 < n)
    {
        ste16_scalar_kernel<IO, CH><<<stream_blocks(n - nvec * 8, kBlock), kBlock, 0, s>>>(
            static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(g),
            static_cast<unsigned short*>(gi), nvec * 8, n, mn, mx, C, K, mins, maxs);
        AIMET_LAUNCH_CHECK();
    }
}

template <bool CH>
void dispatch_qdq16(int io, bool sto, const void* in, void* out, int64_t n, const QdqParams& p, int64_t C, int64_t K,
                    const float* table, uint64_t seed, hipStream_t s)
{
    if (io == IO_F16)
        sto ? launch_qdq16<IO_F16, CH, true>(in, out, n, p, C, K, table, seed, s)
            : launch_qdq16<IO_F16, CH, false>(in, out, n, p, C, K, table, seed, s);
    else
        sto ? launch_qdq16<IO_BF16, CH, true>(in, out, n, p, C, K, table, seed, s)
            : launch_qdq16<IO_BF16, CH, false>(in, out, n, p, C, K, table, seed, s);
}

void check_io(int io)
{
    AIMET_REQUIRE(io == IO_F16 || io == IO_BF16, "io_dtype must be 1 (float16) or 2 (bfloat16)");
}

void check_round_mode(int round_mode)
{
    AIMET_REQUIRE(round_mode == AIMET_ROUND_NEAREST || round_mode == AIMET_ROUND_STOCHASTIC, "Unknown rounding mode.");
}

}   // namespace

QdqParams tensor_params(const aimet_tf_encoding& enc);   // qdq.hip

}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

int aimet_qdq_per_tensor_16(const void* in, void* out, int64_t n, int io_dtype, const aimet_tf_encoding* enc,
                            int round_mode, uint64_t seed, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(enc != nullptr, "encoding is null");
        AIMET_REQUIRE(n >= 0, "negative element count");
        check_io(io_dtype);
        check_round_mode(round_mode);
        if (n == 0)
            return;
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        dispatch_qdq16<false>(io_dtype, round_mode == AIMET_ROUND_STOCHASTIC, in, out, n, tensor_params(*enc), 1, 1,
                              nullptr, seed, as_stream(stream));
    });
}

int aimet_qdq_per_channel_16(const void* in, void* out, int64_t outer, int64_t C, int64_t K, int io_dtype,
                             const float* table, int round_mode, uint64_t seed, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid per-channel shape");
        check_io(io_dtype);
        check_round_mode(round_mode);
        const int64_t n = outer * C * K;
        if (n == 0)
            return;
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        require_device_ptr(table, "table");
        dispatch_qdq16<true>(io_dtype, round_mode == AIMET_ROUND_STOCHASTIC, in, out, n, QdqParams {}, C, K, table,
                             seed, as_stream(stream));
    });
}

int aimet_ste_backward_16(const void* x, const void* grad, void* grad_in, int64_t outer, int64_t C, int64_t K,
                          int io_dtype, const float* mins, const float* maxs, float enc_min, float enc_max,
                          void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        check_io(io_dtype);
        const int64_t n = outer * C * K;
        if (n == 0)
            return;
        require_device_ptr(x, "x");
        require_device_ptr(grad, "grad");
        require_device_ptr(grad_in, "grad_in");
        const bool ch = mins != nullptr;
        if (ch)
        {
            require_device_ptr(mins, "mins");
            require_device_ptr(maxs, "maxs");
        }
        hipStream_t s = as_stream(stream);
        if (io_dtype == IO_F16)
            ch ? launch_ste16<IO_F16, true>(x, grad, grad_in, n, 0, 0, C, K, mins, maxs, s)
               : launch_ste16<IO_F16, false>(x, grad, grad_in, n, enc_min, enc_max, 1, 1, nullptr, nullptr, s);
        else
            ch ? launch_ste16<IO_BF16, true>(x, grad, grad_in, n, 0, 0, C, K, mins, maxs, s)
               : launch_ste16<IO_BF16, false>(x, grad, grad_in, n, enc_min, enc_max, 1, 1, nullptr, nullptr, s);
    });
}

}   // extern "C"
