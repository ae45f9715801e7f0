// learned_grid.hip -- range-learning (LearnedGrid) QAT quantize-dequantize, fused, for gfx950.
//
// Reference: quantsim_straight_through_grad.py:191-249 calculate_forward_pass and :252-328
// asymmetric_gradients / symmetric_gradients, driven by QuantizeDequantizeFunc
// (v1/tensor_quantizer.py:896-986): ~10 torch kernels per tensor per step, saving x, an uint8
// x_quant and a bool mask for the backward.
//
// Here: forward = one pass (x -> y, 8 B/elem, nothing saved but x); backward = one pass that
// recomputes x_round from x and produces grad_x = mask * grad AND the three per-channel sums the
// encoding gradients need (12 B/elem):
//   A = sum((x_quant + offset) * g)        B = sum(mask * (x / delta) * g)      D = sum(!mask * g)
// asymmetric: grad_min = -(A-B)/steps + max * steps/(max-min)^2 * delta*D ; grad_max = (A-B)/steps - min * (...)
// symmetric:  grad_max = (A - B) / floor(steps/2), grad_min = -grad_max
// (assembled from the C-vectors on the torch side). Float32; torch.round = round-half-even.
#include "common.hpp"
#include <cmath>
#include "io16.hpp"

namespace aimet_amd
{
namespace
{

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kLgUnroll = 4;

struct LgChannel
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

// x_round = round(x / delta) - offset ; x_quant = clamp(x_round, 0, steps) ; y = (x_quant + offset) * delta
__device__ __forceinline__ float lg_qdq(float x, float d, float o, float steps)
{
    float xr = __builtin_rintf(x / d) - o;
    float xq = fminf(fmaxf(xr, 0.0f), steps);
    return (xq + o) * d;
}

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

// torch's maximum / minimum: a NaN operand is returned
__device__ __forceinline__ float t_maximum(float a, float b)
{
    return a != a ? a : (b != b ? b : fmaxf(a, b));
}
__device__ __forceinline__ float t_minimum(float a, float b)
{
    return a != a ? a : (b != b ? b : fminf(a, b));
}

// get_computed_encodings (quantsim_straight_through_grad.py:121-160) of channel c, element by
// element as the reference's torch ops on the C-vectors: computed in the forward kernel itself
// when `emin` is set (the thread holding the first element of a channel's first row stores
// them for the backward), else read from precomputed delta / offset
struct LgEnc
{
    const float* emin;
    const float* emax;
    float* delta_out;
    float* offset_out;
    float* range_out;   // optional [2][C]: the range as the forward read it (saved for the backward)
    float steps, half_floor, neg_half_ceil;
    int mode;        // 0 symmetric signed, 1 symmetric unsigned, 2 asymmetric
    uint32_t K;      // elements per row (the store condition)
    uint32_t C;
    __device__ __forceinline__ void of(float mn, float mx, float& d, float& o) const
    {
        if (mode == 0)
        {
            d = mx / half_floor;
            o = neg_half_ceil;
        }
        else
        {
            d = (mx - mn) / steps;
            if (mode == 1)
                o = mn / d;
            else
                o = -t_minimum(steps, t_maximum(0.0f, __builtin_rintf(-mn / d)));
        }
    }
    // delta / offset of channel c for element e (flat index): from the range or the tables
    __device__ __forceinline__ void get(uint32_t c, uint32_t e, const float* delta, const float* offset, float& d,
                                        float& o) const
    {
        if (emin == nullptr)
        {
            d = delta[c];
            o = offset[c];
            return;
        }
        const float mn = emin[c], mx = emax[c];
        of(mn, mx, d, o);
        if (e == c * K)
        {
            delta_out[c]  = d;
            offset_out[c] = o;
            if (range_out)
            {
                range_out[c]     = mn;
                range_out[C + c] = mx;
            }
        }
    }
};

// OUT = IO_F32: y float32. OUT = IO_F16 / IO_BF16: y written in 16 bits with torch's rounding --
// the float32 result cast as autocast casts a weight for its matmul, fused into the store.
template <int OUT>
__device__ __forceinline__ void lg_store4(void* __restrict__ y, uint32_t q, f4 r)
{
    if constexpr (OUT == IO_F32)
        __builtin_nontemporal_store(r, static_cast<f4*>(y) + q);
    else
    {
        const u16x4 h = {from_f32<OUT>(r.x), from_f32<OUT>(r.y), from_f32<OUT>(r.z), from_f32<OUT>(r.w)};
        __builtin_nontemporal_store(h, static_cast<u16x4*>(y) + q);
    }
}

// OUT = IO_F32: y float32. OUT = IO_F16 / IO_BF16: y written in 16 bits with torch's rounding --
// the float32 result cast as autocast casts a weight for its matmul, fused into the store.
// Q quads per lane (vec form), kBlock apart: their loads are issued together and a channel's
// encoding is computed once for consecutive quads of that channel (quad q with q * 4 == c * K
// is never preceded by a quad of channel c, so the store of the first one still happens)
template <int OUT, int Q>
__global__ __launch_bounds__(kBlock) void lg_fwd_kernel(const float* __restrict__ x, void* __restrict__ y,
                                                        uint32_t n, LgChannel map, const float* __restrict__ delta,
                                                        const float* __restrict__ offset, float steps, int vec,
                                                        LgEnc enc)
{
    if (vec)
    {
        const uint32_t nq = n / 4;
        const uint32_t q0 = blockIdx.x * (kBlock * Q) + threadIdx.x;
        f4 v[Q];
#pragma unroll
        for (int u = 0; u < Q; ++u)
            if (q0 + u * kBlock < nq)
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + q0 + u * kBlock);
        uint32_t pc = 0xffffffffu;
        float d = 0.0f, o = 0.0f;
#pragma unroll
        for (int u = 0; u < Q; ++u)
        {
            const uint32_t q = q0 + u * kBlock;
            if (q >= nq)
                return;
            const uint32_t c = map.channel(q * 4);
            if (c != pc)
            {
                enc.get(c, q * 4, delta, offset, d, o);
                pc = c;
            }
            f4 r;
            r.x = lg_qdq(v[u].x, d, o, steps);
            r.y = lg_qdq(v[u].y, d, o, steps);
            r.z = lg_qdq(v[u].z, d, o, steps);
            r.w = lg_qdq(v[u].w, d, o, steps);
            lg_store4<OUT>(y, q, r);
        }
    }
    else
    {
        const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
        if (t >= n)
            return;
        uint32_t c = map.channel(t);
        float d, o;
        enc.get(c, t, delta, offset, d, o);
        const float r = lg_qdq(x[t], d, o, steps);
        if constexpr (OUT == IO_F32)
            static_cast<float*>(y)[t] = r;
        else
            static_cast<unsigned short*>(y)[t] = from_f32<OUT>(r);
    }
}

// quads per lane of lg_fwd_kernel's vec form (1, 2 or 4; AIMET_TUNE_LG_FWD_QUADS for experiments)
int lg_fwd_quads()
{
    static int v = [] {
        const char* e = getenv("AIMET_TUNE_LG_FWD_QUADS");   // tuning experiments only
        const int q   = e ? atoi(e) : 2;
        return (q == 1 || q == 4) ? q : 2;
    }();
    return v;
}

template <int OUT>
void launch_lg_fwd(const float* x, void* y, int64_t n, LgChannel map, const float* delta, const float* offset,
                   float steps, bool vec, LgEnc enc, hipStream_t st)
{
    if (vec && lg_fwd_quads() == 4)
        lg_fwd_kernel<OUT, 4><<<(unsigned) ceil_div(n / 4, kBlock * 4), kBlock, 0, st>>>(x, y, (uint32_t) n, map, delta,
                                                                                       offset, steps, 1, enc);
    else if (vec && lg_fwd_quads() == 2)
        lg_fwd_kernel<OUT, 2><<<(unsigned) ceil_div(n / 4, kBlock * 2), kBlock, 0, st>>>(x, y, (uint32_t) n, map, delta,
                                                                                       offset, steps, 1, enc);
    else
        lg_fwd_kernel<OUT, 1><<<(unsigned) ceil_div(vec ? n / 4 : n, kBlock), kBlock, 0, st>>>(
            x, y, (uint32_t) n, map, delta, offset, steps, vec ? 1 : 0, enc);
    AIMET_LAUNCH_CHECK();
}

// four gradient elements of quad i: float32, or 16-bit upcast (exact)
template <int GIO>
__device__ __forceinline__ f4 load_grad4(const void* __restrict__ g, uint32_t i)
{
    if constexpr (GIO == IO_F32)
        return __builtin_nontemporal_load(static_cast<const f4*>(g) + i);
    else
    {
        const u16x4 h = __builtin_nontemporal_load(static_cast<const u16x4*>(g) + i);
        return f4 {to_f32<GIO>(h.x), to_f32<GIO>(h.y), to_f32<GIO>(h.z), to_f32<GIO>(h.w)};
    }
}

struct Sums
{
    float a, b, d;
};

// q = x / dl from the reciprocal (rcp = v_rcp_f32(dl), within 1 ulp): |q - RN(x/dl)| <= 3.5 ulp(q).
// rint(q) equals rint of the IEEE quotient unless a half-integer lies within 2^-21 (|q| + 1) of q
// (ties-to-even only acts exactly on half-integers); then -- and for non-finite q -- the division
// decides. The returned quotient feeds only the tolerance-checked sum B.
__device__ __forceinline__ float rint_div(float x, float dl, float rcp, float& q)
{
    q               = x * rcp;
    const float h   = q - __builtin_floorf(q);
    const float thr = (__builtin_fabsf(q) + 1.0f) * 4.76837158203125e-7f;   // 2^-21
    if (__builtin_fabsf(h - 0.5f) > thr)                                     // false for NaN / inf
        return __builtin_rintf(q);
    q = x / dl;
    return __builtin_rintf(q);
}

__device__ __forceinline__ void lg_bwd_elem(float x, float g, float dl, float o, float steps, float rcp, float& gx,
                                            Sums& s)
{
    float q;
    float xr   = rint_div(x, dl, rcp, q) - o;
    bool mask  = (xr >= 0.0f) && (xr <= steps);
    float xq   = fminf(fmaxf(xr, 0.0f), steps);
    gx         = mask ? g : 0.0f * g;      // mask_tensor * grad (keeps -0 / NaN behaviour of a multiply)
    s.a += (xq + o) * g;
    s.b += mask ? q * g : 0.0f;
    s.d += mask ? 0.0f : g;
}

__device__ __forceinline__ Sums block_reduce(Sums s)
{
    __shared__ float sh[3][kBlock / 64];
#pragma unroll
    for (int k = 32; k > 0; k >>= 1)
    {
        s.a += __shfl_xor(s.a, k, 64);
        s.b += __shfl_xor(s.b, k, 64);
        s.d += __shfl_xor(s.d, k, 64);
    }
    int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
    {
        sh[0][w] = s.a;
        sh[1][w] = s.b;
        sh[2][w] = s.d;
    }
    __syncthreads();
    Sums r {0, 0, 0};
    if (threadIdx.x == 0)
        for (int i = 0; i < kBlock / 64; ++i)
        {
            r.a += sh[0][i];
            r.b += sh[1][i];
            r.d += sh[2][i];
        }
    __syncthreads();
    return r;
}

// per-tensor (C == 1): grid-stride, block partial sums -> partial[block][3] (folded in a fixed order
// by lg_bwd_fold_one: the encoding gradients are reproducible run to run)
__global__ __launch_bounds__(kBlock) void lg_bwd_tensor_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ g, float* __restrict__ gx,
                                                               int64_t n, const float* __restrict__ delta,
                                                               const float* __restrict__ offset, float steps,
                                                               float* __restrict__ sums, int vec)
{
    const float dl = delta[0], o = offset[0], rcp = __builtin_amdgcn_rcpf(dl);
    Sums s {0, 0, 0};
    if (vec)
    {
        // eight elements (two quads) per lane and step, then the < 8 trailing ones: the order of
        // lg_bwd16_tensor_kernel, so the 16-bit path sums exactly what this one sums
        const int64_t no = n / 8;
        for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < no; i += (int64_t) gridDim.x * kBlock)
        {
            const f4 a0 = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + 2 * i);
            const f4 a1 = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + 2 * i + 1);
            const f4 b0 = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + 2 * i);
            const f4 b1 = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + 2 * i + 1);
            float r[8];
            lg_bwd_elem(a0.x, b0.x, dl, o, steps, rcp, r[0], s);
            lg_bwd_elem(a0.y, b0.y, dl, o, steps, rcp, r[1], s);
            lg_bwd_elem(a0.z, b0.z, dl, o, steps, rcp, r[2], s);
            lg_bwd_elem(a0.w, b0.w, dl, o, steps, rcp, r[3], s);
            lg_bwd_elem(a1.x, b1.x, dl, o, steps, rcp, r[4], s);
            lg_bwd_elem(a1.y, b1.y, dl, o, steps, rcp, r[5], s);
            lg_bwd_elem(a1.z, b1.z, dl, o, steps, rcp, r[6], s);
            lg_bwd_elem(a1.w, b1.w, dl, o, steps, rcp, r[7], s);
            if (gx)
            {
                const f4 r0 = {r[0], r[1], r[2], r[3]}, r1 = {r[4], r[5], r[6], r[7]};
                __builtin_nontemporal_store(r0, reinterpret_cast<f4*>(gx) + 2 * i);
                __builtin_nontemporal_store(r1, reinterpret_cast<f4*>(gx) + 2 * i + 1);
            }
        }
        for (int64_t i = no * 8 + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
        {
            float r;
            lg_bwd_elem(x[i], g[i], dl, o, steps, rcp, r, s);
            if (gx)
                gx[i] = r;
        }
    }
    else
    {
        for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
        {
            float r;
            lg_bwd_elem(x[i], g[i], dl, o, steps, rcp, r, s);
            if (gx)
                gx[i] = r;
        }
    }
    Sums t = block_reduce(s);
    if (threadIdx.x == 0)
    {
        sums[3 * blockIdx.x + 0] = t.a;
        sums[3 * blockIdx.x + 1] = t.b;
        sums[3 * blockIdx.x + 2] = t.d;
    }
}

// the encoding gradients of channel c from its sums {A, B, D} (asymmetric / symmetric_gradients,
// the reference's torch expressions element by element); gmin == nullptr: not requested
struct LgRange
{
    const float* emin;
    const float* emax;
    const float* delta;
    float* gmin;
    float* gmax;
    float steps, half_floor;
    int sym;
};

__device__ __forceinline__ void range_grads_one(float A, float B, float D, uint32_t c, const LgRange& r)
{
    const float gss = A - B;
    if (r.sym)
    {
        const float g = gss / r.half_floor;
        r.gmax[c]     = g;
        r.gmin[c]     = -g;
        return;
    }
    const float mn = r.emin[c], mx = r.emax[c];
    const float term1 = gss / r.steps;
    const float w     = mx - mn;
    const float term2 = (r.steps / (w * w)) * (r.delta[c] * D);
    r.gmin[c]         = -term1 + mx * term2;
    r.gmax[c]         = term1 - mn * term2;
}

// sums[0..2] = the nparts partial triples, lane i taking parts i, i + kBlock, ... in order, then
// the fixed shuffle tree of block_reduce: one result whatever the scheduling; the range
// gradients follow in the same launch when requested
__global__ __launch_bounds__(kBlock) void lg_bwd_fold_one(const float* __restrict__ partial, int nparts,
                                                          float* __restrict__ sums, LgRange range)
{
    Sums s {0, 0, 0};
    for (int i = threadIdx.x; i < nparts; i += kBlock)
    {
        s.a += partial[3 * i + 0];
        s.b += partial[3 * i + 1];
        s.d += partial[3 * i + 2];
    }
    Sums t = block_reduce(s);
    if (threadIdx.x == 0)
    {
        sums[0] = t.a;
        sums[1] = t.b;
        sums[2] = t.d;
        if (range.gmin)
            range_grads_one(t.a, t.b, t.d, 0, range);
    }
}

// per-channel: one workgroup per channel of [outer][C][K], sums written directly
__global__ __launch_bounds__(kBlock) void lg_bwd_channel_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ g, float* __restrict__ gx,
                                                                int64_t outer, int64_t C, int64_t K,
                                                                const float* __restrict__ delta,
                                                                const float* __restrict__ offset, float steps,
                                                                float* __restrict__ sums)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        const float dl = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(dl);
        Sums s {0, 0, 0};
        for (int64_t r = 0; r < outer; ++r)
        {
            const int64_t base = (r * C + c) * K;
            for (int64_t k = threadIdx.x; k < K; k += kBlock)
            {
                float v;
                lg_bwd_elem(x[base + k], g[base + k], dl, o, steps, rcp, v, s);
                if (gx)
                    gx[base + k] = v;
            }
        }
        Sums t = block_reduce(s);
        if (threadIdx.x == 0)
        {
            sums[3 * c + 0] = t.a;
            sums[3 * c + 1] = t.b;
            sums[3 * c + 2] = t.d;
        }
    }
}

// per-channel, 16-B form (K % 4 == 0, aligned): a (channel, slice) grid; with one slice the sums
// are stored, with several (few channels: fill the chip) each slice stores its triple at
// sums[(c * splits + slice) * 3] and lg_bwd_tile_fold adds them per channel in slice order.
__global__ __launch_bounds__(kBlock) void lg_bwd_channel_vec_kernel(const f4* __restrict__ x, const f4* __restrict__ g,
                                                                    f4* __restrict__ gx, int64_t outer, int64_t C,
                                                                    int64_t K4, FastDiv divK4,
                                                                    const float* __restrict__ delta,
                                                                    const float* __restrict__ offset, float steps,
                                                                    float* __restrict__ sums)
{
    const int splits = gridDim.y;
    const int64_t Q  = outer * K4;
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        const float dl = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(dl);
        Sums s {0, 0, 0};
        // kLgUnroll quads (2 x 16-B loads each) in flight per lane
        const int64_t step = (int64_t) splits * kBlock;
        for (int64_t j0 = (int64_t) blockIdx.y * kBlock + threadIdx.x; j0 < Q; j0 += step * kLgUnroll)
        {
            f4 a[kLgUnroll], b[kLgUnroll];
            int64_t idx[kLgUnroll];
#pragma unroll
            for (int u = 0; u < kLgUnroll; ++u)
            {
                const int64_t j = j0 + u * step;
                const int64_t jj = j < Q ? j : Q - 1;   // clamped (neither summed nor stored)
                const int64_t r  = outer == 1 ? 0 : divK4.div((uint32_t) jj);
                idx[u]           = (r * C + c) * K4 + (jj - r * K4);
                a[u]             = __builtin_nontemporal_load(x + idx[u]);
                b[u]             = __builtin_nontemporal_load(g + idx[u]);
            }
#pragma unroll
            for (int u = 0; u < kLgUnroll; ++u)
            {
                if (j0 + u * step >= Q)
                    break;
                float r0, r1, r2, r3;
                lg_bwd_elem(a[u].x, b[u].x, dl, o, steps, rcp, r0, s);
                lg_bwd_elem(a[u].y, b[u].y, dl, o, steps, rcp, r1, s);
                lg_bwd_elem(a[u].z, b[u].z, dl, o, steps, rcp, r2, s);
                lg_bwd_elem(a[u].w, b[u].w, dl, o, steps, rcp, r3, s);
                if (gx)
                {
                    f4 rv = {r0, r1, r2, r3};
                    __builtin_nontemporal_store(rv, gx + idx[u]);
                }
            }
        }
        Sums t = block_reduce(s);
        if (threadIdx.x == 0)
        {
            if (splits == 1)
            {
                sums[3 * c + 0] = t.a;
                sums[3 * c + 1] = t.b;
                sums[3 * c + 2] = t.d;
            }
            else
            {
                const int64_t p = c * splits + blockIdx.y;
                sums[3 * p + 0] = t.a;
                sums[3 * p + 1] = t.b;
                sums[3 * p + 2] = t.d;
            }
        }
    }
}

// per-channel, tile form (K/4 a multiple of 256*U): workgroup b covers the U*256 consecutive quads
// [b*U*256, (b+1)*U*256) of the flat tensor -- inside one row, so one channel -- in address order,
// like the streaming QDQ kernels (the (channel, slice) grid above streams from as many places as
// there are channels in flight). Per-workgroup sums go to partial[b][3]; lg_bwd_tile_fold adds them
// per channel in a fixed order (deterministic).
template <int U, int GIO>
__global__ __launch_bounds__(kBlock) void lg_bwd_tile_kernel(const f4* __restrict__ x, const void* __restrict__ g,
                                                             f4* __restrict__ gx, FastDiv divK4, FastDiv divC,
                                                             uint32_t C, const float* __restrict__ delta,
                                                             const float* __restrict__ offset, float steps,
                                                             float* __restrict__ partial)
{
    const uint32_t q0  = blockIdx.x * (uint32_t) (kBlock * U);
    const uint32_t row = divK4.div(q0);
    const uint32_t c   = row - divC.div(row) * C;
    const float dl = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(dl);
    f4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        a[u] = __builtin_nontemporal_load(x + q0 + u * kBlock + threadIdx.x);
        b[u] = load_grad4<GIO>(g, q0 + u * kBlock + threadIdx.x);
    }
    Sums s {0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
        float r0, r1, r2, r3;
        lg_bwd_elem(a[u].x, b[u].x, dl, o, steps, rcp, r0, s);
        lg_bwd_elem(a[u].y, b[u].y, dl, o, steps, rcp, r1, s);
        lg_bwd_elem(a[u].z, b[u].z, dl, o, steps, rcp, r2, s);
        lg_bwd_elem(a[u].w, b[u].w, dl, o, steps, rcp, r3, s);
        if (gx)
        {
            f4 rv = {r0, r1, r2, r3};
            __builtin_nontemporal_store(rv, gx + q0 + u * kBlock + threadIdx.x);
        }
    }
    Sums t = block_reduce(s);
    if (threadIdx.x == 0)
    {
        partial[3 * blockIdx.x + 0] = t.a;
        partial[3 * blockIdx.x + 1] = t.b;
        partial[3 * blockIdx.x + 2] = t.d;
    }
}

// sums[c] = sum over the rows r of channel c and their workgroups w (in that order)
__global__ __launch_bounds__(kBlock) void lg_bwd_tile_fold(const float* __restrict__ partial, float* __restrict__ sums,
                                                           uint32_t outer, uint32_t C, uint32_t per_row, LgRange range)
{
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= C)
        return;
    float a = 0, b = 0, d = 0;
    for (uint32_t r = 0; r < outer; ++r)
        for (uint32_t w = 0; w < per_row; ++w)
        {
            const float* p = partial + 3 * ((size_t) (r * C + c) * per_row + w);
            a += p[0];
            b += p[1];
            d += p[2];
        }
    sums[3 * c + 0] = a;
    sums[3 * c + 1] = b;
    sums[3 * c + 2] = d;
    if (range.gmin)
        range_grads_one(a, b, d, c, range);
}

// ---- fp16 / bf16 I/O, per tensor (C == 1): the conversions in registers ------------------------
// Identical results to x.to(float32) -> the fp32 kernels -> .to(dtype): the upcast is exact, the
// arithmetic and the element -> lane -> workgroup order of the backward's sums are those of
// lg_bwd_tensor_kernel (quads, then the tail), and the downcast is torch's (io16.hpp). 4 B/elem
// forward and 6 B/elem backward instead of 20 and 24 for the three-pass chains.

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// vec: eight elements (one 16-B load) per lane; otherwise one element per lane
template <int IO>
__global__ __launch_bounds__(kBlock) void lg_fwd16_kernel(const unsigned short* __restrict__ x,
                                                          unsigned short* __restrict__ y, uint32_t n,
                                                          const float* __restrict__ delta,
                                                          const float* __restrict__ offset, float steps, int vec,
                                                          LgEnc enc)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    float d, o;
    enc.get(0, t, delta, offset, d, o);   // element 0's thread stores them
    if (vec)
    {
        if (t >= n / 8)
            return;
        const u16x8 v = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(x) + t);
        u16x8 r;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            r[k] = from_f32<IO>(lg_qdq(to_f32<IO>(v[k]), d, o, steps));
        __builtin_nontemporal_store(r, reinterpret_cast<u16x8*>(y) + t);
    }
    else if (t < n)
        y[t] = from_f32<IO>(lg_qdq(to_f32<IO>(x[t]), d, o, steps));
}

// the element -> lane -> workgroup order of lg_bwd_tensor_kernel (eight per lane and step, then
// the tail), so the sums equal the float32 kernel's on the upcast tensors
template <int IO>
__global__ __launch_bounds__(kBlock) void lg_bwd16_tensor_kernel(const unsigned short* __restrict__ x,
                                                                 const unsigned short* __restrict__ g,
                                                                 unsigned short* __restrict__ gx, int64_t n,
                                                                 const float* __restrict__ delta,
                                                                 const float* __restrict__ offset, float steps,
                                                                 float* __restrict__ partial, int vec)
{
    const float dl = delta[0], o = offset[0], rcp = __builtin_amdgcn_rcpf(dl);
    Sums s {0, 0, 0};
    int64_t done = 0;
    if (vec)
    {
        const int64_t no = n / 8;
        for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < no; i += (int64_t) gridDim.x * kBlock)
        {
            const u16x8 a = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(x) + i);
            const u16x8 b = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(g) + i);
            float r[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                lg_bwd_elem(to_f32<IO>(a[k]), to_f32<IO>(b[k]), dl, o, steps, rcp, r[k], s);
            if (gx)
            {
                u16x8 h;
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    h[k] = from_f32<IO>(r[k]);
                __builtin_nontemporal_store(h, reinterpret_cast<u16x8*>(gx) + i);
            }
        }
        done = no * 8;
    }
    for (int64_t i = done + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
    {
        float r;
        lg_bwd_elem(to_f32<IO>(x[i]), to_f32<IO>(g[i]), dl, o, steps, rcp, r, s);
        if (gx)
            gx[i] = from_f32<IO>(r);
    }
    Sums t = block_reduce(s);
    if (threadIdx.x == 0)
    {
        partial[3 * blockIdx.x + 0] = t.a;
        partial[3 * blockIdx.x + 1] = t.b;
        partial[3 * blockIdx.x + 2] = t.d;
    }
}

// ---- the small per-channel vectors around the passes, one launch each -----------------------
// Each expression is the reference's torch op sequence on float32 C-vectors, element by element,
// with torch's NaN rules (clamp keeps a NaN input, maximum / minimum return the NaN operand) and
// no contraction: results are those of the torch ops, bit for bit (tests/test_gpu_parity.py).

// set_encoding_min_max_gating_threshold (v1/tensor_quantizer.py:1347-1359), in place
__global__ __launch_bounds__(kBlock) void lg_gate_kernel(float* __restrict__ emin, float* __restrict__ emax,
                                                         uint32_t C)
{
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= C)
        return;
    float mn = emin[c], mx = emax[c];
    mn = mn != mn ? mn : fminf(mn, 0.0f);   // clamp_(max=0)
    mx = mx != mx ? mx : fmaxf(mx, 0.0f);   // clamp_(min=0)
    emin[c] = mn;
    emax[c] = t_maximum(mx, mn + 1e-5f);
}

// the gate over up to kGateRanges ranges in one launch (a wrapper's quantizers): range r owns the
// threads [start[r], start[r + 1])
constexpr int kGateRanges = 8;
struct LgGateSet
{
    float* emin[kGateRanges];
    float* emax[kGateRanges];
    uint32_t start[kGateRanges + 1];
    int n;
};

__global__ __launch_bounds__(kBlock) void lg_gate_many_kernel(LgGateSet set)
{
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= set.start[set.n])
        return;
    int r = 0;
    while (r + 1 < set.n && t >= set.start[r + 1])
        ++r;
    const uint32_t c = t - set.start[r];
    float* emin = set.emin[r];
    float* emax = set.emax[r];
    float mn = emin[c], mx = emax[c];
    mn = mn != mn ? mn : fminf(mn, 0.0f);   // the expressions of lg_gate_kernel
    mx = mx != mx ? mx : fmaxf(mx, 0.0f);
    emin[c] = mn;
    emax[c] = t_maximum(mx, mn + 1e-5f);
}

// get_computed_encodings (quantsim_straight_through_grad.py:121-160)
__global__ __launch_bounds__(kBlock) void lg_encodings_kernel(const float* __restrict__ emin,
                                                              const float* __restrict__ emax, uint32_t C,
                                                              float steps, int mode, float half_floor,
                                                              float neg_half_ceil, float* __restrict__ delta,
                                                              float* __restrict__ offset, float* __restrict__ range_out)
{
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= C)
        return;
    const float mn = emin[c], mx = emax[c];
    if (range_out)
    {
        range_out[c]     = mn;
        range_out[C + c] = mx;
    }
    float d, o;
    if (mode == 0)   // symmetric, signed
    {
        d = mx / half_floor;
        o = neg_half_ceil;
    }
    else
    {
        d = (mx - mn) / steps;
        if (mode == 1)   // symmetric, unsigned
            o = mn / d;
        else             // asymmetric: -min(steps, max(0, round(-min / delta)))
            o = -t_minimum(steps, t_maximum(0.0f, __builtin_rintf(-mn / d)));
    }
    delta[c]  = d;
    offset[c] = o;
}

// the encoding gradients from the backward's sums {A, B, D} (asymmetric / symmetric_gradients)
__global__ __launch_bounds__(kBlock) void lg_range_grads_kernel(const float* __restrict__ sums, uint32_t C,
                                                                LgRange range)
{
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c < C)
        range_grads_one(sums[3 * c], sums[3 * c + 1], sums[3 * c + 2], c, range);
}

LgRange range_of(const aimet_lg_range_spec* spec, float steps)
{
    LgRange r {};
    if (spec == nullptr)
        return r;
    AIMET_REQUIRE(spec->grad_min && spec->grad_max && spec->encoding_min && spec->encoding_max && spec->delta,
                  "aimet_lg_range_spec: every pointer must be set");
    r = LgRange {spec->encoding_min, spec->encoding_max, spec->delta, spec->grad_min, spec->grad_max, steps,
                 (float) std::floor(steps / 2.0), spec->use_symmetric};
    return r;
}

// the range gradients as their own launch (backward paths whose sums come without a fold)
void launch_range_grads(const float* sums, int64_t C, const LgRange& r, hipStream_t s)
{
    if (r.gmin == nullptr || C == 0)
        return;
    lg_range_grads_kernel<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, s>>>(sums, (uint32_t) C, r);
    AIMET_LAUNCH_CHECK();
}

template <int GIO>
void launch_bwd_tile(int U, int64_t wg, const f4* x, const void* g, f4* gx, FastDiv dk, FastDiv dc, int64_t C,
                     const float* delta, const float* offset, float steps, float* partial, hipStream_t s)
{
    if (U == 4)
        lg_bwd_tile_kernel<4, GIO><<<(unsigned) wg, kBlock, 0, s>>>(x, g, gx, dk, dc, (uint32_t) C, delta, offset,
                                                                    steps, partial);
    else if (U == 2)
        lg_bwd_tile_kernel<2, GIO><<<(unsigned) wg, kBlock, 0, s>>>(x, g, gx, dk, dc, (uint32_t) C, delta, offset,
                                                                    steps, partial);
    else
        lg_bwd_tile_kernel<1, GIO><<<(unsigned) wg, kBlock, 0, s>>>(x, g, gx, dk, dc, (uint32_t) C, delta, offset,
                                                                    steps, partial);
    AIMET_LAUNCH_CHECK();
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

int aimet_lg_forward(const float* x, float* y, int64_t outer, int64_t C, int64_t K, const float* delta,
                     const float* offset, float num_steps, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "learned-grid QDQ needs < 2^31 elements per call");
        require_device_ptr(x, "x");
        require_device_ptr(y, "y");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        LgChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        bool vec     = (C == 1 || K % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0
                       && n % 4 == 0;
        launch_lg_fwd<IO_F32>(x, y, n, map, delta, offset, num_steps, vec, LgEnc {}, as_stream(stream));
    });
}

}   // extern "C"

namespace
{

LgEnc enc_of(const float* emin, const float* emax, int64_t C, int64_t K, int bw, int sym, int strict, int unsign,
             float* delta, float* offset, float* range_out)
{
    AIMET_REQUIRE(bw > 0 && bw < 32, "invalid bitwidth");
    require_device_ptr(emin, "encoding_min");
    require_device_ptr(emax, "encoding_max");
    require_device_ptr(delta, "delta");
    require_device_ptr(offset, "offset");
    double steps = std::ldexp(1.0, bw) - 1;
    if (sym && strict)
        steps -= 1;
    const double half = steps / 2;
    if (range_out)
        require_device_ptr(range_out, "range_out");
    return LgEnc {emin, emax, delta, offset, range_out, (float) steps, (float) std::floor(half),
                  (float) -std::ceil(half), (sym && !unsign) ? 0 : (sym ? 1 : 2), (uint32_t) K, (uint32_t) C};
}

void forward_cast(const float* x, void* y, int64_t outer, int64_t C, int64_t K, int out_dtype, const float* delta,
                  const float* offset, float num_steps, LgEnc enc, hipStream_t st);

}   // namespace

extern "C" {

int aimet_lg_forward_range(const float* x, void* y, int64_t outer, int64_t C, int64_t K, int out_dtype,
                           const float* emin, const float* emax, int bw, int sym, int strict, int unsign,
                           float* delta_out, float* offset_out, float* range_out, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        const LgEnc enc = enc_of(emin, emax, C, K, bw, sym, strict, unsign, delta_out, offset_out, range_out);
        if (outer * C * K == 0)
        {
            // no element to carry the encodings: compute them on their own
            lg_encodings_kernel<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, as_stream(stream)>>>(
                emin, emax, (uint32_t) C, enc.steps, enc.mode, enc.half_floor, enc.neg_half_ceil, delta_out,
                offset_out, range_out);
            AIMET_LAUNCH_CHECK();
            return;
        }
        forward_cast(x, y, outer, C, K, out_dtype, nullptr, nullptr, enc.steps, enc, as_stream(stream));
    });
}

int aimet_lg_forward_cast(const float* x, void* y, int64_t outer, int64_t C, int64_t K, int out_dtype,
                          const float* delta, const float* offset, float num_steps, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(out_dtype == IO_F16 || out_dtype == IO_BF16, "out_dtype must be 1 (float16) or 2 (bfloat16)");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        forward_cast(x, y, outer, C, K, out_dtype, delta, offset, num_steps, LgEnc {}, as_stream(stream));
    });
}

}   // extern "C"

namespace
{

// out_dtype IO_F32: float32 result (aimet_lg_forward's arithmetic), else the 16-bit cast of it
void forward_cast(const float* x, void* y, int64_t outer, int64_t C, int64_t K, int out_dtype, const float* delta,
                  const float* offset, float num_steps, LgEnc enc, hipStream_t st)
{
    {
        AIMET_REQUIRE(out_dtype == IO_F32 || out_dtype == IO_F16 || out_dtype == IO_BF16, "invalid out_dtype");
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "learned-grid QDQ needs < 2^31 elements per call");
        require_device_ptr(x, "x");
        require_device_ptr(y, "y");
        LgChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        const int ya = out_dtype == IO_F32 ? 15 : 7;
        bool vec = (C == 1 || K % 4 == 0) && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(y) & ya) == 0 && n % 4 == 0;
        if (out_dtype == IO_F32)
            launch_lg_fwd<IO_F32>(x, y, n, map, delta, offset, num_steps, vec, enc, st);
        else if (out_dtype == IO_F16)
            launch_lg_fwd<IO_F16>(x, y, n, map, delta, offset, num_steps, vec, enc, st);
        else
            launch_lg_fwd<IO_BF16>(x, y, n, map, delta, offset, num_steps, vec, enc, st);
    }
}

}   // namespace

extern "C" {

int aimet_lg_backward(const float* x, const float* grad, float* grad_x, float* sums, int64_t outer, int64_t C,
                      int64_t K, const float* delta, const float* offset, float num_steps,
                      const aimet_lg_range_spec* range_spec, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        require_device_ptr(sums, "sums");
        hipStream_t s = as_stream(stream);
        const LgRange range = range_of(range_spec, num_steps);
        if (n == 0)
        {
            AIMET_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(float) * 3 * C, s));
            launch_range_grads(sums, C, range, s);
            return;
        }
        require_device_ptr(x, "x");
        require_device_ptr(grad, "grad");
        if (grad_x)
            require_device_ptr(grad_x, "grad_x");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        if (C == 1)
        {
            bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad) |
                         reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0;
            const unsigned nb = stream_blocks(n, (int64_t) kBlock * 16);
            float* partial    = static_cast<float*>(scratch_alloc(sizeof(float) * 3 * nb, s));
            lg_bwd_tensor_kernel<<<nb, kBlock, 0, s>>>(x, grad, grad_x, n, delta, offset, num_steps, partial,
                                                       vec ? 1 : 0);
            AIMET_LAUNCH_CHECK();
            lg_bwd_fold_one<<<1, kBlock, 0, s>>>(partial, (int) nb, sums, range);
            AIMET_LAUNCH_CHECK();
            scratch_free(partial, s);
            return;
        }
        else if (K % 1024 == 0 && n < (int64_t(1) << 31) && C < 65536 &&
                 ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad) |
                   reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0)
        {
            const int64_t K4 = K / 4;
            const int U      = K4 % (kBlock * 4) == 0 ? 4 : K4 % (kBlock * 2) == 0 ? 2 : 1;
            const int64_t wg = n / 4 / (kBlock * U);
            float* partial   = nullptr;
            partial = static_cast<float*>(scratch_alloc(sizeof(float) * 3 * wg, s));
            auto xv = reinterpret_cast<const f4*>(x);
            auto gv = reinterpret_cast<const f4*>(grad);
            auto ov = reinterpret_cast<f4*>(grad_x);
            FastDiv dk((uint32_t) K4), dc((uint32_t) C);
            launch_bwd_tile<IO_F32>(U, wg, xv, gv, ov, dk, dc, C, delta, offset, num_steps, partial, s);
            lg_bwd_tile_fold<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, s>>>(
                partial, sums, (uint32_t) outer, (uint32_t) C, (uint32_t) (K4 / (kBlock * U)), range);
            AIMET_LAUNCH_CHECK();
            scratch_free(partial, s);
            return;
        }
        else if (K % 4 == 0 && outer * (K / 4) < (int64_t(1) << 32) &&
                 ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad) |
                   reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0)
        {
            // >= 2048 workgroups in flight: slice channels when there are fewer than that
            const int64_t K4  = K / 4;
            int64_t splits    = C >= 2048 ? 1 : (2048 + C - 1) / C;
            const int64_t per = ceil_div(outer * K4, kBlock);   // enough quads for every slice
            if (splits > per)
                splits = per > 0 ? per : 1;
            dim3 grid((unsigned) (C < 65536 ? C : 65536), (unsigned) splits);
            float* partial = splits > 1 ? static_cast<float*>(scratch_alloc(sizeof(float) * 3 * C * splits, s))
                                        : sums;
            lg_bwd_channel_vec_kernel<<<grid, kBlock, 0, s>>>(
                reinterpret_cast<const f4*>(x), reinterpret_cast<const f4*>(grad), reinterpret_cast<f4*>(grad_x),
                outer, C, K4, FastDiv((uint32_t) (K4 > 0 ? K4 : 1)), delta, offset, num_steps, partial);
            if (splits > 1)
            {
                AIMET_LAUNCH_CHECK();
                lg_bwd_tile_fold<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, s>>>(partial, sums, 1u, (uint32_t) C,
                                                                                   (uint32_t) splits, range);
                AIMET_LAUNCH_CHECK();
                scratch_free(partial, s);
                return;
            }
        }
        else
        {
            int grid = (int) (C < 65536 ? C : 65536);
            lg_bwd_channel_kernel<<<grid, kBlock, 0, s>>>(x, grad, grad_x, outer, C, K, delta, offset, num_steps,
                                                          sums);
        }
        AIMET_LAUNCH_CHECK();
        launch_range_grads(sums, C, range, s);
    });
}

}   // extern "C"

extern "C" {

}   // extern "C"

namespace
{

void forward_16(const void* x, void* y, int64_t n, int io_dtype, const float* delta, const float* offset,
                float num_steps, LgEnc enc, hipStream_t st)
{
    AIMET_REQUIRE(io_dtype == IO_F16 || io_dtype == IO_BF16, "io_dtype must be 1 (float16) or 2 (bfloat16)");
    AIMET_REQUIRE(n >= 0 && n < (int64_t(1) << 31), "learned-grid QDQ needs < 2^31 elements per call");
    if (n == 0)
        return;
    require_device_ptr(x, "x");
    require_device_ptr(y, "y");
    const bool vec = n % 8 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
    const int64_t work = vec ? n / 8 : n;
    auto xs = static_cast<const unsigned short*>(x);
    auto ys = static_cast<unsigned short*>(y);
    if (io_dtype == IO_F16)
        lg_fwd16_kernel<IO_F16><<<(unsigned) ceil_div(work, kBlock), kBlock, 0, st>>>(
            xs, ys, (uint32_t) n, delta, offset, num_steps, vec ? 1 : 0, enc);
    else
        lg_fwd16_kernel<IO_BF16><<<(unsigned) ceil_div(work, kBlock), kBlock, 0, st>>>(
            xs, ys, (uint32_t) n, delta, offset, num_steps, vec ? 1 : 0, enc);
    AIMET_LAUNCH_CHECK();
}

}   // namespace

extern "C" {

int aimet_lg_forward_16(const void* x, void* y, int64_t n, int io_dtype, const float* delta, const float* offset,
                        float num_steps, void* stream)
{
    return guarded([&] {
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        forward_16(x, y, n, io_dtype, delta, offset, num_steps, LgEnc {}, as_stream(stream));
    });
}

int aimet_lg_forward_16_range(const void* x, void* y, int64_t n, int io_dtype, const float* emin, const float* emax,
                              int bw, int sym, int strict, int unsign, float* delta_out, float* offset_out,
                              float* range_out, void* stream)
{
    return guarded([&] {
        const LgEnc enc = enc_of(emin, emax, 1, n > 0 ? n : 1, bw, sym, strict, unsign, delta_out, offset_out,
                                 range_out);
        if (n == 0)
        {
            lg_encodings_kernel<<<1, kBlock, 0, as_stream(stream)>>>(emin, emax, 1u, enc.steps, enc.mode,
                                                                      enc.half_floor, enc.neg_half_ceil, delta_out,
                                                                      offset_out, range_out);
            AIMET_LAUNCH_CHECK();
            return;
        }
        forward_16(x, y, n, io_dtype, nullptr, nullptr, enc.steps, enc, as_stream(stream));
    });
}

int aimet_lg_gate_range(float* emin, float* emax, int64_t C, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(C >= 0 && C < (int64_t(1) << 31), "invalid channel count");
        if (C == 0)
            return;
        lg_gate_kernel<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, as_stream(stream)>>>(emin, emax, (uint32_t) C);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_lg_gate_ranges(float* const* emin, float* const* emax, const int64_t* C, int n, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(n >= 0 && n <= kGateRanges, "aimet_lg_gate_ranges takes at most 8 ranges");
        AIMET_REQUIRE(n == 0 || (emin && emax && C), "null range table");
        LgGateSet set {};
        int64_t total = 0;
        for (int r = 0; r < n; ++r)
        {
            AIMET_REQUIRE(C[r] >= 0, "invalid channel count");
            require_device_ptr(emin[r], "encoding_min");
            require_device_ptr(emax[r], "encoding_max");
            set.emin[r]  = emin[r];
            set.emax[r]  = emax[r];
            set.start[r] = (uint32_t) total;
            total += C[r];
            AIMET_REQUIRE(total < (int64_t(1) << 31), "too many channels");
        }
        set.start[n] = (uint32_t) total;
        set.n        = n;
        if (total == 0)
            return;
        lg_gate_many_kernel<<<(unsigned) ceil_div(total, kBlock), kBlock, 0, as_stream(stream)>>>(set);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_lg_encodings(const float* emin, const float* emax, int64_t C, int bw, int sym, int strict, int unsign,
                       float* delta, float* offset, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(C >= 0 && C < (int64_t(1) << 31), "invalid channel count");
        AIMET_REQUIRE(bw > 0 && bw < 32, "invalid bitwidth");
        if (C == 0)
            return;
        double steps = std::ldexp(1.0, bw) - 1;
        if (sym && strict)
            steps -= 1;
        const double half = steps / 2;
        const int mode    = (sym && !unsign) ? 0 : (sym ? 1 : 2);
        lg_encodings_kernel<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, as_stream(stream)>>>(
            emin, emax, (uint32_t) C, (float) steps, mode, (float) std::floor(half), (float) -std::ceil(half), delta,
            offset, nullptr);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_lg_range_grads(const float* sums, const float* emin, const float* emax, const float* delta, int64_t C,
                         float num_steps, int sym, float* grad_min, float* grad_max, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(C >= 0 && C < (int64_t(1) << 31), "invalid channel count");
        const aimet_lg_range_spec spec {emin, emax, delta, grad_min, grad_max, sym};
        launch_range_grads(sums, C, range_of(&spec, num_steps), as_stream(stream));
    });
}

int aimet_lg_backward_grad16(const float* x, const void* grad, float* grad_x, float* sums, int64_t outer, int64_t C,
                             int64_t K, int grad_dtype, const float* delta, const float* offset, float num_steps,
                             const aimet_lg_range_spec* range_spec, void* stream)
{
    return guarded([&] {
        const LgRange range = range_of(range_spec, num_steps);
        AIMET_REQUIRE(grad_dtype == IO_F16 || grad_dtype == IO_BF16, "grad_dtype must be 1 (float16) or 2 (bfloat16)");
        AIMET_REQUIRE(outer >= 0 && C > 1 && K >= 0, "invalid shape (per-channel tensors only)");
        const int64_t n = outer * C * K;
        require_device_ptr(sums, "sums");
        hipStream_t s = as_stream(stream);
        if (n == 0)
        {
            AIMET_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(float) * 3 * C, s));
            launch_range_grads(sums, C, range, s);
            return;
        }
        AIMET_REQUIRE(aimet_lg_backward_grad16_supported(outer, C, K, x, grad, grad_x),
                      "16-bit gradient backward: rows must be multiples of 1024 elements, 16-B / 8-B aligned");
        require_device_ptr(x, "x");
        require_device_ptr(grad, "grad");
        if (grad_x)
            require_device_ptr(grad_x, "grad_x");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        // the tile path of aimet_lg_backward with the gradient upcast in registers (exact): the same
        // arithmetic and summation order as aimet_lg_backward on grad.to(float32)
        const int64_t K4 = K / 4;
        const int U      = K4 % (kBlock * 4) == 0 ? 4 : K4 % (kBlock * 2) == 0 ? 2 : 1;
        const int64_t wg = n / 4 / (kBlock * U);
        float* partial   = static_cast<float*>(scratch_alloc(sizeof(float) * 3 * wg, s));
        FastDiv dk((uint32_t) K4), dc((uint32_t) C);
        auto xv = reinterpret_cast<const f4*>(x);
        auto ov = reinterpret_cast<f4*>(grad_x);
        if (grad_dtype == IO_F16)
            launch_bwd_tile<IO_F16>(U, wg, xv, grad, ov, dk, dc, C, delta, offset, num_steps, partial, s);
        else
            launch_bwd_tile<IO_BF16>(U, wg, xv, grad, ov, dk, dc, C, delta, offset, num_steps, partial, s);
        lg_bwd_tile_fold<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, s>>>(
            partial, sums, (uint32_t) outer, (uint32_t) C, (uint32_t) (K4 / (kBlock * U)), range);
        AIMET_LAUNCH_CHECK();
        scratch_free(partial, s);
    });
}

int aimet_lg_backward_grad16_supported(int64_t outer, int64_t C, int64_t K, const void* x, const void* grad,
                                       const void* grad_x)
{
    const int64_t n = outer * C * K;
    return C > 1 && K % 1024 == 0 && n > 0 && n < (int64_t(1) << 31) && C < 65536 &&
           ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(grad) & 7) == 0;
}

int aimet_lg_backward_16(const void* x, const void* grad, void* grad_x, float* sums, int64_t n, int io_dtype,
                         const float* delta, const float* offset, float num_steps,
                         const aimet_lg_range_spec* range_spec, void* stream)
{
    return guarded([&] {
        const LgRange range = range_of(range_spec, num_steps);
        AIMET_REQUIRE(io_dtype == IO_F16 || io_dtype == IO_BF16, "io_dtype must be 1 (float16) or 2 (bfloat16)");
        AIMET_REQUIRE(n >= 0, "invalid size");
        require_device_ptr(sums, "sums");
        hipStream_t s = as_stream(stream);
        if (n == 0)
        {
            AIMET_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(float) * 3, s));
            launch_range_grads(sums, 1, range, s);
            return;
        }
        require_device_ptr(x, "x");
        require_device_ptr(grad, "grad");
        if (grad_x)
            require_device_ptr(grad_x, "grad_x");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(grad) |
                           reinterpret_cast<uintptr_t>(grad_x)) & 15) == 0;
        const unsigned nb = stream_blocks(n, (int64_t) kBlock * 16);   // the fp32 kernel's grid
        float* partial    = static_cast<float*>(scratch_alloc(sizeof(float) * 3 * nb, s));
        auto xs = static_cast<const unsigned short*>(x);
        auto gs = static_cast<const unsigned short*>(grad);
        auto os = static_cast<unsigned short*>(grad_x);
        if (io_dtype == IO_F16)
            lg_bwd16_tensor_kernel<IO_F16><<<nb, kBlock, 0, s>>>(xs, gs, os, n, delta, offset, num_steps, partial,
                                                                 vec ? 1 : 0);
        else
            lg_bwd16_tensor_kernel<IO_BF16><<<nb, kBlock, 0, s>>>(xs, gs, os, n, delta, offset, num_steps, partial,
                                                                  vec ? 1 : 0);
        AIMET_LAUNCH_CHECK();
        lg_bwd_fold_one<<<1, kBlock, 0, s>>>(partial, (int) nb, sums, range);
        AIMET_LAUNCH_CHECK();
        scratch_free(partial, s);
    });
}

}   // extern "C"
