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
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>
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

// The quotient x / d without the IEEE division's ~10 instructions. y = lg_recip(d) = RN(1/d) is
// computed once per encoding; then q0 = RN(x * y) is a faithful quotient, r = x - d * q0 is exact
// (fma), and RN(q0 + r * y) is the correctly rounded quotient (Markstein's theorem) while nothing
// under- or overflows: |d| in [2^-40, 2^40] (else y = NaN and the kernels divide) and |q| in
// [2^-60, 2^60), so |x| and r stay far from the subnormal range. Bit-identical to x / d there:
// tools/studies/markstein_div_check.c (754 M operand pairs, quotients at half-integers +-3 ulp and
// all-ones mantissas included; the same bounds fail only for |x| < 2^-100). Outside that range the
// consumers below need less than the exact quotient (lg_rint_quot, lg_quot), so no element takes
// a slow path: 3 VALU plus one compare per element (the 16-bit kernels are VALU co-bound).
__device__ __forceinline__ float lg_recip(float d)
{
    const float a = __builtin_fabsf(d);
    return (a >= 0x1p-40f && a <= 0x1p40f) ? 1.0f / d : __builtin_nanf("");
}

// torch's NaN: the op chain passes a NaN input through (quieted)
__device__ __forceinline__ float quiet_nan(float x)
{
    return __uint_as_float(__float_as_uint(x) | 0x00400000u);
}

// torch's clamp(v, lo, hi) = minimum(maximum(v, lo), hi): a NaN passes through (gfx950's
// v_maximum3 / v_minimum3, IEEE 754-2019). It differs from torch only in the sign of a zero
// (maximum(-0, +0) = +0), which every use below adds an offset to, where -0 + o == +0 + o.
__device__ __forceinline__ float t_clamp(float v, float lo, float hi)
{
    return __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, lo), hi);
}

// the reference's forward with the division: encodings that lg_recip refuses (or a non-finite
// offset)
__device__ __forceinline__ float lg_qdq_div(float x, float d, float o, float steps)
{
    return (t_clamp(__builtin_rintf(x / d) - o, 0.0f, steps) + o) * d;
}

__device__ __forceinline__ bool lg_fast_enc(float o, float rd)
{
    return rd == rd && __builtin_fabsf(o) <= 0x1p32f;
}

// The forward's element for an encoding lg_fast_enc accepts, never NaN: x is first clamped to
// +-2^59 |d| (med3), inside which |x * y| < 2^60 and the Markstein quotient needs no range test;
// a clamped x gives rint(q) ~ +-2^59, beyond every clamp bound on the same side as the division's
// (+-inf included). A NaN x is the caller's to map (torch's clamp passes it through).
__device__ __forceinline__ float lg_qdq_fast(float x, float d, float o, float steps, float rd, float xmax)
{
    const float xc = __builtin_amdgcn_fmed3f(x, -xmax, xmax);
    const float q0 = xc * rd;
    const float q  = __builtin_fmaf(__builtin_fmaf(-q0, d, xc), rd, q0);
    return (__builtin_amdgcn_fmed3f(__builtin_rintf(q) - o, 0.0f, steps) + o) * d;
}

// x_round = round(x / delta) - offset ; x_quant = clamp(x_round, 0, steps) ; y = (x_quant + offset) * delta
// (rd = lg_recip(d)); a NaN x gives NaN as torch's clamp does
__device__ __forceinline__ float lg_qdq(float x, float d, float o, float steps, float rd)
{
    if (!lg_fast_enc(o, rd))
        return lg_qdq_div(x, d, o, steps);
    const float y = lg_qdq_fast(x, d, o, steps, rd, 0x1p59f * __builtin_fabsf(d));
    return x != x ? quiet_nan(x) : y;
}
template <int N>
__device__ __forceinline__ void lg_qdq_n(const float* x, float d, float o, float steps, float rd, float* y)
{
    if (!lg_fast_enc(o, rd))
    {
#pragma unroll
        for (int k = 0; k < N; ++k)
            y[k] = lg_qdq_div(x[k], d, o, steps);
        return;
    }
    const float xmax = 0x1p59f * __builtin_fabsf(d);
#pragma unroll
    for (int k = 0; k < N; ++k)
    {
        const float v = lg_qdq_fast(x[k], d, o, steps, rd, xmax);
        y[k]          = x[k] != x[k] ? quiet_nan(x[k]) : v;
    }
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
        float d = 0.0f, o = 0.0f, rd = 0.0f;
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
                rd = lg_recip(d);
                pc = c;
            }
            const float xin[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            float yo[4];
            lg_qdq_n<4>(xin, d, o, steps, rd, yo);
            const f4 r = {yo[0], yo[1], yo[2], yo[3]};
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
        const float r = lg_qdq(x[t], d, o, steps, lg_recip(d));
        if constexpr (OUT == IO_F32)
            static_cast<float*>(y)[t] = r;
        else
            static_cast<unsigned short*>(y)[t] = from_f32<OUT>(r);
    }
}

template <int OUT>
void launch_lg_fwd(const float* x, void* y, int64_t n, LgChannel map, const float* delta, const float* offset,
                   float steps, bool vec, LgEnc enc, hipStream_t st)
{
    // two quads per lane in the vec form (one: 4.4 vs 5.4 TB/s on the Llama-3-8B weights; four: no
    // faster, profiles/r02/llama_qat_kernel_stats*.csv)
    if (vec)
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

// One element of the backward (calculate_forward_pass + the gradient expressions of
// QuantizeDequantizeFunc.backward / asymmetric_gradients / symmetric_gradients), with
// q = RN(x / dl) (lg_quot, rcp = lg_recip(dl)), the reference's x / delta:
//   m = mask (0 / 1) ; grad_x = m * grad ;
//   MODE 1 (symmetric_gradients): A += (x_quant + offset) * grad ; B += (m * (x / delta)) * grad
//     (the reference's two sums, :311-314);
//   MODE 2 (asymmetric_gradients): A += (x_quant + offset - (x * m) / delta) * grad, the
//     reference's one grad_scale sum (:283-286, B stays 0), and D += grad where !m (grad_offset
//     without its delta factor, applied to the sum);
//   MODE 0 (no range gradients requested): A, B as MODE 1 and D as MODE 2.
// Where !m, (x * m) / delta is 0 * x (NaN for a non-finite x) and m * (x / delta) is 0 * (x /
// delta) (NaN also when the quotient overflows), as the reference evaluates them. mask is
// x_quant == x_round with x_quant = med3(x_round, 0, steps) (one compare instead of two; false
// for a NaN round); a NaN x makes the sums NaN through those 0 * NaN terms, as the reference's,
// so x_quant need not pass the NaN through. Every kernel forms the same values.
template <int MODE>
__device__ __forceinline__ void lg_bwd_term_m(float x, float q, float g, float o, float steps, float& gx, Sums& s)
{
    const float xr = __builtin_rintf(q) - o;
    const float xq = __builtin_amdgcn_fmed3f(xr, 0.0f, steps);
    const bool in  = xq == xr;
    const float m  = in ? 1.0f : 0.0f;
    gx = m * g;
    if constexpr (MODE == 2)
    {
        s.a += ((xq + o) - m * (in ? q : x)) * g;
        s.d += in ? 0.0f : g;
    }
    else
    {
        s.a += (xq + o) * g;
        s.b += (m * q) * g;
        if constexpr (MODE == 0)
            s.d += in ? 0.0f : g;
    }
}
__device__ __forceinline__ void lg_bwd_term(float x, float q, float g, float o, float steps, int mode, float& gx,
                                            Sums& s)
{
    if (mode == 2)
        lg_bwd_term_m<2>(x, q, g, o, steps, gx, s);
    else if (mode == 1)
        lg_bwd_term_m<1>(x, q, g, o, steps, gx, s);
    else
        lg_bwd_term_m<0>(x, q, g, o, steps, gx, s);
}

// RN(x / d) for the backward from y = lg_recip(d) (not NaN), no branch: the Markstein quotient
// while |q0| < 2^60 -- RN(x / d) itself except for |x| < 2^-100, where it is off by a few ulps of
// a quotient below 2^-59 -- else q0 = RN(x * y) (infinite exactly when x is, or when x / d is
// within an ulp of overflowing). rint(q) and the mask are therefore the division's (grad_x is
// bit-exact); B's terms can differ only in those two corners, at the encoding gradients' tolerance.
__device__ __forceinline__ float lg_quot(float x, float d, float y)
{
    const float q0 = x * y;
    const float q  = __builtin_fmaf(__builtin_fmaf(-q0, d, x), y, q0);
    return __builtin_fabsf(q0) < 0x1p60f ? q : q0;
}

__device__ __forceinline__ void lg_bwd_elem(float x, float g, float dl, float o, float steps, float rcp, float& gx,
                                            Sums& s, int mode)
{
    lg_bwd_term(x, lg_fast_enc(o, rcp) ? lg_quot(x, dl, rcp) : x / dl, g, o, steps, mode, gx, s);
}

// lg_bwd_elem over N elements in order (the same sums)
template <int N>
__device__ __forceinline__ void lg_bwd_elems(const float* x, const float* g, float dl, float o, float steps,
                                             float rcp, float* gx, Sums& s, int mode)
{
    float q[N];
    if (lg_fast_enc(o, rcp))
    {
#pragma unroll
        for (int k = 0; k < N; ++k)
            q[k] = lg_quot(x[k], dl, rcp);
    }
    else
    {
#pragma unroll
        for (int k = 0; k < N; ++k)
            q[k] = x[k] / dl;
    }
#pragma unroll
    for (int k = 0; k < N; ++k)
        lg_bwd_term(x[k], q[k], g[k], o, steps, mode, gx[k], s);
}

// lg_bwd_elems for an encoding lg_fast_enc accepts: no division code in the caller's vector path
// (its registers are then the streaming loads' and the sums', not the division's temporaries)
template <int N, int MODE>
__device__ __forceinline__ void lg_bwd_elems_fast(const float* x, const float* g, float dl, float o, float steps,
                                                  float rcp, float* gx, Sums& s)
{
#pragma unroll
    for (int k = 0; k < N; ++k)
        lg_bwd_term_m<MODE>(x[k], lg_quot(x[k], dl, rcp), g[k], o, steps, gx[k], s);
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

// The per-tensor backward's ntiles partial triples folded as one triple, whichever kernel folds
// them (lg_bwd_fold_one, or the kernel's last workgroup): lane l sums tiles l, l + kBlock, ... in
// order, then the fixed shuffle tree of block_reduce -- one result whatever the scheduling; the
// range gradients follow when requested. Called by every thread of one workgroup.
// (A fold in two levels -- each group of tiles folded by its last-arriving workgroup -- summed in
// another order whose error on Llama-3-8B's lm_head output range gradient reached 2.45 units of the
// stated bound, above the 2 the tests assert, and was no faster: profiles/r04/README.md.)
__device__ __forceinline__ void fold_partials(const float* __restrict__ partial, int64_t nparts,
                                              float* __restrict__ sums, const LgRange& range)
{
    // each lane's parts in ascending order, kFoldBatch triples of loads in flight at a time (one
    // dependent round trip per part made a 3,342-part fold 5 us long)
    constexpr int kFoldBatch = 8;
    Sums s {0, 0, 0};
    for (int64_t i0 = threadIdx.x; i0 < nparts; i0 += (int64_t) kBlock * kFoldBatch)
    {
        float a[kFoldBatch], b[kFoldBatch], d[kFoldBatch];
#pragma unroll
        for (int u = 0; u < kFoldBatch; ++u)
        {
            const int64_t i = i0 + (int64_t) u * kBlock;
            const float* p  = partial + 3 * (i < nparts ? i : 0);
            a[u]            = p[0];
            b[u]            = p[1];
            d[u]            = p[2];
        }
#pragma unroll
        for (int u = 0; u < kFoldBatch; ++u)
            if (i0 + (int64_t) u * kBlock < nparts)
            {
                s.a += a[u];
                s.b += b[u];
                s.d += d[u];
            }
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

// a tile's partial triple (folded by the next launch)
__device__ __forceinline__ void store_sums(float* p, const Sums& t)
{
    p[0] = t.a;
    p[1] = t.b;
    p[2] = t.d;
}

// per-tensor (C == 1), tile form: workgroup b owns the kLgTile consecutive elements
// [b * kLgTile, (b + 1) * kLgTile); lane l of it takes the 8-element groups u * kBlock + l
// (u < kLgTileSteps), every load of the tile issued before any arithmetic. The per-lane sums run
// in (u, element) order, then the fixed shuffle tree of block_reduce, one partial triple per
// workgroup, folded in workgroup order by lg_bwd_fold_one (deterministic; the fold in the kernel's
// last-arriving workgroup measured 7-8 us slower per call than its own 4 us launch -- every
// workgroup draining its stores and taking a ticket, profiles/r04/README.md -- and was removed).
// lg_bwd16_tensor_kernel maps elements to lanes and workgroups identically, so the 16-bit path sums exactly what this one
// sums. (A grid-stride form with one pair of loads per lane in flight ran at 0.47 of HBM peak on
// the 16-bit Llama-3-8B activations.)
constexpr int kLgTileSteps = 2;

// a tile's element e of lane `lane` in step u, k-th of its 8
__device__ __forceinline__ int64_t lg_tile_elem(int64_t base, int u, int k)
{
    return base + ((int64_t) u * kBlock + threadIdx.x) * 8 + k;
}

// Tiles per launch: tile b is processed by workgroup b % gridDim.x (grid = the tile count unless
// a tuning cap is set); its partial triple goes to sums[3 * b], so the fold sees the same partials
// in the same order whatever the grid.
template <int STEPS, int MODE>
__global__ __launch_bounds__(kBlock) void lg_bwd_tensor_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ g, float* __restrict__ gx,
                                                               int64_t n, const float* __restrict__ delta,
                                                               const float* __restrict__ offset, float steps,
                                                               float* __restrict__ sums, int vec, int64_t ntiles)
{
    constexpr int64_t kTile = (int64_t) kBlock * 8 * STEPS;
    const float dl = delta[0], o = offset[0], rcp = lg_recip(dl);
    const bool fast = lg_fast_enc(o, rcp);   // else every tile takes the element path (the division)
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x)
    {
        const int64_t base = tile * kTile;
        Sums s {0, 0, 0};
        if (fast && vec && base + kTile <= n)
        {
            f4 a[STEPS][2], b[STEPS][2];
#pragma unroll
            for (int u = 0; u < STEPS; ++u)
            {
                const int64_t q = lg_tile_elem(base, u, 0) / 4;
                a[u][0] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + q);
                a[u][1] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(x) + q + 1);
                b[u][0] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + q);
                b[u][1] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + q + 1);
            }
#pragma unroll
            for (int u = 0; u < STEPS; ++u)
            {
                float r[8];
                const float xv[8] = {a[u][0].x, a[u][0].y, a[u][0].z, a[u][0].w,
                                     a[u][1].x, a[u][1].y, a[u][1].z, a[u][1].w};
                const float gv[8] = {b[u][0].x, b[u][0].y, b[u][0].z, b[u][0].w,
                                     b[u][1].x, b[u][1].y, b[u][1].z, b[u][1].w};
                lg_bwd_elems_fast<8, MODE>(xv, gv, dl, o, steps, rcp, r, s);
                if (gx)
                {
                    const int64_t q = lg_tile_elem(base, u, 0) / 4;
                    const f4 r0 = {r[0], r[1], r[2], r[3]}, r1 = {r[4], r[5], r[6], r[7]};
                    __builtin_nontemporal_store(r0, reinterpret_cast<f4*>(gx) + q);
                    __builtin_nontemporal_store(r1, reinterpret_cast<f4*>(gx) + q + 1);
                }
            }
        }
        else
        {
            // the last (partial) tile, unaligned pointers or an encoding for the division: element
            // by element, the same order
            for (int u = 0; u < STEPS; ++u)
                for (int k = 0; k < 8; ++k)
                {
                    const int64_t e = lg_tile_elem(base, u, k);
                    if (e >= n)
                        break;
                    float r;
                    lg_bwd_elem(x[e], g[e], dl, o, steps, rcp, r, s, MODE);
                    if (gx)
                        gx[e] = r;
                }
        }
        Sums t = block_reduce(s);
        if (threadIdx.x == 0)
            store_sums(sums + 3 * tile, t);
    }
}

// Launch shape of the per-tensor backward kernels (fp32 and 16-bit use the same, so their sums
// stay identical): kLgTileSteps 8-element groups per lane and tile, one workgroup per tile (fp32) or
// kLgBwd16Grid workgroups looping over the tiles (16-bit, pipelined)
struct LgBwdLaunch
{
    int64_t ntiles;
    unsigned grid, grid16;
};
constexpr int64_t kLgBwd16Grid = 2048;

LgBwdLaunch lg_bwd_launch(int64_t n)
{
    LgBwdLaunch L;
    // (one 8-element group per lane and tile for calls of <= 4 M elements -- twice the workgroups --
    // measured no faster, 5.5 vs 5.2 us at 2 M elements, and its summation order put Llama-3-8B's
    // lm_head output range gradient at 2.45 units of the stated bound: not used; four groups kept
    // the bound but ran slower, profiles/r04/lg16_steps2_vs_steps4.jsonl)
    L.ntiles = ceil_div(n, (int64_t) kBlock * 8 * kLgTileSteps);
    AIMET_REQUIRE(L.ntiles < (int64_t(1) << 31), "too many elements");
    L.grid   = (unsigned) L.ntiles;
    L.grid16 = (unsigned) (L.ntiles > kLgBwd16Grid ? kLgBwd16Grid : L.ntiles);
    return L;
}

// f(integral_constant<MODE>) for the backward mode: the per-tensor kernels are compiled per mode
// (lg_bwd_term_m), so their element loops carry only the sums that mode needs
template <class F>
void lg_bwd_dispatch(int mode, F&& f)
{
    if (mode == 2)
        f(std::integral_constant<int, 2> {});
    else if (mode == 1)
        f(std::integral_constant<int, 1> {});
    else
        f(std::integral_constant<int, 0> {});
}

// the per-tensor backward's fold, its own launch
__global__ __launch_bounds__(kBlock) void lg_bwd_fold_one(const float* __restrict__ partial, int64_t ntiles,
                                                          float* __restrict__ sums, LgRange range)
{
    fold_partials(partial, ntiles, sums, range);
}

// per-channel: one workgroup per channel of [outer][C][K], sums written directly
__global__ __launch_bounds__(kBlock) void lg_bwd_channel_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ g, float* __restrict__ gx,
                                                                int64_t outer, int64_t C, int64_t K,
                                                                const float* __restrict__ delta,
                                                                const float* __restrict__ offset, float steps, int mode,
                                                                float* __restrict__ sums)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        const float dl = delta[c], o = offset[c], rcp = lg_recip(dl);
        Sums s {0, 0, 0};
        for (int64_t r = 0; r < outer; ++r)
        {
            const int64_t base = (r * C + c) * K;
            for (int64_t k = threadIdx.x; k < K; k += kBlock)
            {
                float v;
                lg_bwd_elem(x[base + k], g[base + k], dl, o, steps, rcp, v, s, mode);
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
                                                                    const float* __restrict__ offset, float steps, int mode,
                                                                    float* __restrict__ sums)
{
    const int splits = gridDim.y;
    const int64_t Q  = outer * K4;
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        const float dl = delta[c], o = offset[c], rcp = lg_recip(dl);
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
                float rr[4];
                const float xv[4] = {a[u].x, a[u].y, a[u].z, a[u].w}, gv[4] = {b[u].x, b[u].y, b[u].z, b[u].w};
                lg_bwd_elems<4>(xv, gv, dl, o, steps, rcp, rr, s, mode);
                if (gx)
                {
                    f4 rv = {rr[0], rr[1], rr[2], rr[3]};
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
                                                             const float* __restrict__ offset, float steps, int mode,
                                                             float* __restrict__ partial)
{
    const uint32_t q0  = blockIdx.x * (uint32_t) (kBlock * U);
    const uint32_t row = divK4.div(q0);
    const uint32_t c   = row - divC.div(row) * C;
    const float dl = delta[c], o = offset[c], rcp = lg_recip(dl);
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
        float rr[4];
        const float xv[4] = {a[u].x, a[u].y, a[u].z, a[u].w}, gv[4] = {b[u].x, b[u].y, b[u].z, b[u].w};
        lg_bwd_elems<4>(xv, gv, dl, o, steps, rcp, rr, s, mode);
        if (gx)
        {
            f4 rv = {rr[0], rr[1], rr[2], rr[3]};
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

// lg_fwd16_kernel's default shape: kLgFwd16Vecs 16-B vectors (8 elements) per lane and tile,
// kLgFwd16Grid workgroups looping over the tiles (other shapes measured slower, profiles/r03/
// lg16_kernel_stats.csv, profiles/r04/lg16_*.jsonl)
constexpr int kLgFwd16Vecs     = 1;
constexpr int64_t kLgFwd16Grid  = 2048;   // workgroups: 8 per CU, one resident round
constexpr int64_t kLgFwd16Tile = (int64_t) kBlock * 8 * kLgFwd16Vecs;

// 16-B loads / stores of the 16-bit kernels: nontemporal (NT, the streaming default) or through
// the caches (measured no faster for activations still resident in the MALL, profiles/r04)
template <bool NT>
__device__ __forceinline__ u16x8 ld16(const u16x8* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(u16x8 v, u16x8* p)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <int IO, int V, int BLOCK, bool NT>
__device__ __forceinline__ void lg_fwd16_load(const unsigned short* __restrict__ x, int64_t tile, u16x8* v)
{
    constexpr int64_t kTile = (int64_t) BLOCK * 8 * V;
#pragma unroll
    for (int u = 0; u < V; ++u)
        v[u] = ld16<NT>(reinterpret_cast<const u16x8*>(x) + tile * kTile / 8 + u * BLOCK + threadIdx.x);
}

// Workgroup b takes tiles b, b + grid, ... (grid capped near one resident wave of workgroups per
// SIMD slot): the next tile's loads are issued before the current tile is computed, so each wave
// keeps its 16-B loads in flight through its own arithmetic (a wave that loaded, waited and then
// computed left the memory pipe idle during the ~20 VALU per element). Full tiles only; the
// partial last tile, unaligned pointers and encodings for the division take the element loop.
template <int IO, int V, int BLOCK, bool NT = true>
__global__ __launch_bounds__(BLOCK) void lg_fwd16_kernel(const unsigned short* __restrict__ x,
                                                         unsigned short* __restrict__ y, int64_t n,
                                                         const float* __restrict__ delta,
                                                         const float* __restrict__ offset, float steps, int vec,
                                                         LgEnc enc, int64_t ntiles)
{
    constexpr int64_t kTile = (int64_t) BLOCK * 8 * V;
    // the first tile's loads go out before the encoding is read (they do not depend on it; on a
    // small call the two latencies in a row were most of the kernel)
    const int64_t nvec = vec ? n / kTile : 0;
    int64_t tile       = blockIdx.x;
    u16x8 cur[V];
    if (tile < nvec)
        lg_fwd16_load<IO, V, BLOCK, NT>(x, tile, cur);
    float d, o;
    // element 0's thread (tile 0 is workgroup 0's first) stores the encoding
    enc.get(0, blockIdx.x == 0 && threadIdx.x == 0 ? 0u : 1u, delta, offset, d, o);
    const float rd   = lg_recip(d);
    const float xmax = 0x1p59f * __builtin_fabsf(d);
    const bool fast  = lg_fast_enc(o, rd);
    const int64_t nfull = fast ? nvec : 0;
    if (tile < nfull)
    {
        auto compute = [&](const u16x8 (&v)[V], int64_t t) {
#pragma unroll
            for (int u = 0; u < V; ++u)
            {
                u16x8 r;
#pragma unroll
                for (int k = 0; k < 8; ++k)
                {
                    // never NaN for a fast encoding; a NaN input -> the 16-bit NaN torch's cast
                    // of the passed-through NaN gives (one select, no NaN test of the result)
                    const float xf = to_f32<IO>(v[u][k]);
                    const float yq = lg_qdq_fast(xf, d, o, steps, rd, xmax);
                    r[k] = xf != xf ? from_f32<IO>(quiet_nan(xf)) : from_f32<IO, false>(yq);
                }
                st16<NT>(r, reinterpret_cast<u16x8*>(y) + t * kTile / 8 + u * BLOCK + threadIdx.x);
            }
        };
        // two register buffers in turn (no copy of the next tile's registers, which made the
        // compiler wait for its loads at the end of every tile); the next tile's loads are
        // unconditional -- the last tile reloads itself, unused -- so the same number of loads is
        // outstanding on every path and the wait at each tile's first use leaves them in flight
        u16x8 nxt[V];
        for (;;)
        {
            int64_t tn = tile + gridDim.x < nfull ? tile + gridDim.x : tile;
            lg_fwd16_load<IO, V, BLOCK, NT>(x, tn, nxt);
            compute(cur, tile);
            tile += gridDim.x;
            if (tile >= nfull)
                break;
            tn = tile + gridDim.x < nfull ? tile + gridDim.x : tile;
            lg_fwd16_load<IO, V, BLOCK, NT>(x, tn, cur);
            compute(nxt, tile);
            tile += gridDim.x;
            if (tile >= nfull)
                break;
        }
    }
    // the rest element by element: tiles from nfull on (all of them when not vec / not fast)
    for (; tile < ntiles; tile += gridDim.x)
        for (int64_t e = tile * kTile + threadIdx.x; e < (tile + 1) * kTile && e < n; e += BLOCK)
            y[e] = from_f32<IO>(lg_qdq(to_f32<IO>(x[e]), d, o, steps, rd));
}

// the element -> lane -> workgroup order of lg_bwd_tensor_kernel (tiles of kLgTile, 8 elements per
// lane and step), so the sums equal the float32 kernel's on the upcast tensors
template <int STEPS, bool NT>
__device__ __forceinline__ void lg_bwd16_load(const unsigned short* __restrict__ x, const unsigned short* __restrict__ g,
                                              int64_t base, u16x8* a, u16x8* b)
{
#pragma unroll
    for (int u = 0; u < STEPS; ++u)
    {
        const int64_t q = lg_tile_elem(base, u, 0) / 8;
        a[u] = ld16<NT>(reinterpret_cast<const u16x8*>(x) + q);
        b[u] = ld16<NT>(reinterpret_cast<const u16x8*>(g) + q);
    }
}

// Tiles b, b + grid, ... per workgroup with the next tile's loads issued before the current tile is
// computed and reduced (see lg_fwd16_kernel); each tile's partial triple still goes to
// partial[3 * tile], so the sums are those of any other grid.
template <int IO, int STEPS, int MODE, bool NT = true>
__global__ __launch_bounds__(kBlock) void lg_bwd16_tensor_kernel(const unsigned short* __restrict__ x,
                                                                 const unsigned short* __restrict__ g,
                                                                 unsigned short* __restrict__ gx, int64_t n,
                                                                 const float* __restrict__ delta,
                                                                 const float* __restrict__ offset, float steps,
                                                                 float* __restrict__ partial, int vec, int64_t ntiles)
{
    constexpr int64_t kTile = (int64_t) kBlock * 8 * STEPS;
    // the first tile's loads go out before the encoding is read: they do not depend on it, and on
    // a small call (a few tiles per CU) the two latencies in a row were most of the kernel
    const int64_t nvec = vec ? n / kTile : 0;
    int64_t tile = blockIdx.x;
    u16x8 a[STEPS], b[STEPS];
    if (tile < nvec)
        lg_bwd16_load<STEPS, NT>(x, g, tile * kTile, a, b);
    const float dl = delta[0], o = offset[0], rcp = lg_recip(dl);
    // full tiles of an encoding lg_fast_enc accepts take the vector path; the rest (the partial
    // last tile, unaligned pointers, an encoding for the division) the element path
    const int64_t nfull = lg_fast_enc(o, rcp) ? nvec : 0;
    // full tiles: two register buffers in turn, the next tile's loads unconditional (see
    // lg_fwd16_kernel), each tile's partial triple published as before
    auto full_tile = [&](const u16x8 (&a_)[STEPS], const u16x8 (&b_)[STEPS], int64_t t) {
        const int64_t base = t * kTile;
        Sums s {0, 0, 0};
#pragma unroll
        for (int u = 0; u < STEPS; ++u)
        {
            float r[8], xv[8], gv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
            {
                xv[k] = to_f32<IO>(a_[u][k]);
                gv[k] = to_f32<IO>(b_[u][k]);
            }
            lg_bwd_elems_fast<8, MODE>(xv, gv, dl, o, steps, rcp, r, s);
            if (gx)
            {
                u16x8 h;
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    h[k] = from_f32<IO>(r[k]);
                st16<NT>(h, reinterpret_cast<u16x8*>(gx) + lg_tile_elem(base, u, 0) / 8);
            }
        }
        Sums t3 = block_reduce(s);
        if (threadIdx.x == 0)
            store_sums(partial + 3 * t, t3);
    };
    if (tile < nfull)
    {
        u16x8 an[STEPS], bn[STEPS];
        for (;;)
        {
            int64_t tn = tile + gridDim.x < nfull ? tile + gridDim.x : tile;
            lg_bwd16_load<STEPS, NT>(x, g, tn * kTile, an, bn);
            full_tile(a, b, tile);
            tile += gridDim.x;
            if (tile >= nfull)
                break;
            tn = tile + gridDim.x < nfull ? tile + gridDim.x : tile;
            lg_bwd16_load<STEPS, NT>(x, g, tn * kTile, a, b);
            full_tile(an, bn, tile);
            tile += gridDim.x;
            if (tile >= nfull)
                break;
        }
    }
    // the rest element by element (the partial last tile, unaligned pointers, an encoding for the
    // division), the same order
    for (; tile < ntiles; tile += gridDim.x)
    {
        const int64_t base = tile * kTile;
        Sums s {0, 0, 0};
        for (int u = 0; u < STEPS; ++u)
            for (int k = 0; k < 8; ++k)
            {
                const int64_t e = lg_tile_elem(base, u, k);
                if (e >= n)
                    break;
                float r;
                lg_bwd_elem(to_f32<IO>(x[e]), to_f32<IO>(g[e]), dl, o, steps, rcp, r, s, MODE);
                if (gx)
                    gx[e] = from_f32<IO>(r);
            }
        Sums t3 = block_reduce(s);
        if (threadIdx.x == 0)
            store_sums(partial + 3 * tile, t3);
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
                     const float* delta, const float* offset, float steps, int mode, float* partial, hipStream_t s)
{
    if (U == 4)
        lg_bwd_tile_kernel<4, GIO><<<(unsigned) wg, kBlock, 0, s>>>(x, g, gx, dk, dc, (uint32_t) C, delta, offset,
                                                                    steps, mode, partial);
    else if (U == 2)
        lg_bwd_tile_kernel<2, GIO><<<(unsigned) wg, kBlock, 0, s>>>(x, g, gx, dk, dc, (uint32_t) C, delta, offset,
                                                                    steps, mode, partial);
    else
        lg_bwd_tile_kernel<1, GIO><<<(unsigned) wg, kBlock, 0, s>>>(x, g, gx, dk, dc, (uint32_t) C, delta, offset,
                                                                    steps, mode, partial);
    AIMET_LAUNCH_CHECK();
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

namespace
{

// sub-problems of a [outer][C][K] learned-grid pass with <= lg_chunk_elems() elements each (the
// fp32 forward's element -> channel map is 32-bit): whole rows when a row of C x K fits, else
// channel ranges of one row, else pieces of one channel's K (a multiple of 16 elements, so every
// piece keeps the 16-B alignment). fn(first element, outer', first channel, C', K').
// aimet_lg_set_chunk_limit (tests only) lowers the bound to exercise the chunking on small tensors.
std::atomic<int64_t> g_lg_chunk {int64_t(1) << 30};
int64_t lg_chunk_elems()
{
    return g_lg_chunk.load(std::memory_order_relaxed);
}

template <class F>
void for_each_lg_chunk(int64_t outer, int64_t C, int64_t K, F fn)
{
    const int64_t lim = lg_chunk_elems();
    if (C * K <= lim)
    {
        const int64_t rows = lim / (C * K);
        for (int64_t r = 0; r < outer; r += rows)
            fn(r * C * K, std::min(rows, outer - r), 0, C, K);
        return;
    }
    for (int64_t r = 0; r < outer; ++r)
    {
        if (K <= lim)
        {
            const int64_t cs = lim / K;
            for (int64_t c = 0; c < C; c += cs)
                fn((r * C + c) * K, 1, c, std::min(cs, C - c), K);
        }
        else
            for (int64_t c = 0; c < C; ++c)
                for (int64_t k = 0; k < K; k += lim)
                    fn((r * C + c) * K + k, 1, c, 1, std::min(lim, K - k));
    }
}

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

int aimet_lg_forward(const float* x, float* y, int64_t outer, int64_t C, int64_t K, const float* delta,
                     const float* offset, float num_steps, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        forward_cast(x, y, outer, C, K, IO_F32, delta, offset, num_steps, LgEnc {}, as_stream(stream));
    });
}

}   // extern "C"


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
        require_device_ptr(x, "x");
        require_device_ptr(y, "y");
        if (n > lg_chunk_elems())
        {
            // past 2^31 elements the kernels' 32-bit element -> channel arithmetic would wrap: the
            // encodings first (when the kernel was to form them), then sub-problems of whole rows
            // (or channel ranges, or row pieces) of <= lg_chunk_elems() elements each
            if (enc.emin)
            {
                lg_encodings_kernel<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, st>>>(
                    enc.emin, enc.emax, (uint32_t) C, enc.steps, enc.mode, enc.half_floor, enc.neg_half_ceil,
                    enc.delta_out, enc.offset_out, enc.range_out);
                AIMET_LAUNCH_CHECK();
                delta  = enc.delta_out;
                offset = enc.offset_out;
            }
            const size_t ysz = out_dtype == IO_F32 ? 4 : 2;
            for_each_lg_chunk(outer, C, K, [&](int64_t first, int64_t o2, int64_t c0, int64_t C2, int64_t K2) {
                forward_cast(x + first, static_cast<char*>(y) + first * ysz, o2, C2, K2, out_dtype, delta + c0,
                             offset + c0, num_steps, LgEnc {}, st);
            });
            return;
        }
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
        const int mode      = range.gmin == nullptr ? 0 : range.sym ? 1 : 2;   // lg_bwd_term_m
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
            const LgBwdLaunch L = lg_bwd_launch(n);
            float* partial      = static_cast<float*>(scratch_alloc(sizeof(float) * 3 * L.ntiles, s));
            const int v         = vec ? 1 : 0;
            lg_bwd_dispatch(mode, [&](auto md) {
                lg_bwd_tensor_kernel<kLgTileSteps, decltype(md)::value><<<L.grid, kBlock, 0, s>>>(
                    x, grad, grad_x, n, delta, offset, num_steps, partial, v, L.ntiles);
            });
            AIMET_LAUNCH_CHECK();
            lg_bwd_fold_one<<<1, kBlock, 0, s>>>(partial, L.ntiles, sums, range);
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
            launch_bwd_tile<IO_F32>(U, wg, xv, gv, ov, dk, dc, C, delta, offset, num_steps, mode, partial, s);
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
                outer, C, K4, FastDiv((uint32_t) (K4 > 0 ? K4 : 1)), delta, offset, num_steps, mode, partial);
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
                                                          mode, sums);
        }
        AIMET_LAUNCH_CHECK();
        launch_range_grads(sums, C, range, s);
    });
}

}   // extern "C"

namespace
{

void forward_16(const void* x, void* y, int64_t n, int io_dtype, const float* delta, const float* offset,
                float num_steps, LgEnc enc, hipStream_t st)
{
    AIMET_REQUIRE(io_dtype == IO_F16 || io_dtype == IO_BF16, "io_dtype must be 1 (float16) or 2 (bfloat16)");
    AIMET_REQUIRE(n >= 0 && ceil_div(n, kLgFwd16Tile) < (int64_t(1) << 31), "too many elements");
    if (n == 0)
        return;
    require_device_ptr(x, "x");
    require_device_ptr(y, "y");
    const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
    auto xs = static_cast<const unsigned short*>(x);
    auto ys = static_cast<unsigned short*>(y);
    // kLgFwd16Vecs 16-B vectors per lane, kLgFwd16Grid workgroups looping over the tiles
    const int64_t ntiles = ceil_div(n, kLgFwd16Tile);
    const unsigned grid  = (unsigned) (ntiles > kLgFwd16Grid ? kLgFwd16Grid : ntiles);
    const int v          = vec ? 1 : 0;
    if (io_dtype == IO_F16)
        lg_fwd16_kernel<IO_F16, kLgFwd16Vecs, kBlock><<<grid, kBlock, 0, st>>>(xs, ys, n, delta, offset, num_steps, v,
                                                                              enc, ntiles);
    else
        lg_fwd16_kernel<IO_BF16, kLgFwd16Vecs, kBlock><<<grid, kBlock, 0, st>>>(xs, ys, n, delta, offset, num_steps, v,
                                                                               enc, ntiles);
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

int aimet_lg_set_chunk_limit(int64_t elems)
{
    return guarded([&] {
        AIMET_REQUIRE(elems == 0 || (elems >= 1024 && elems <= (int64_t(1) << 30)),
                      "chunk limit: 0 (default) or 1024 .. 2^30 elements");
        g_lg_chunk.store(elems == 0 ? (int64_t(1) << 30) : (elems / 16) * 16, std::memory_order_relaxed);
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
        const int mode      = range.gmin == nullptr ? 0 : range.sym ? 1 : 2;   // lg_bwd_term_m
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
            launch_bwd_tile<IO_F16>(U, wg, xv, grad, ov, dk, dc, C, delta, offset, num_steps, mode, partial, s);
        else
            launch_bwd_tile<IO_BF16>(U, wg, xv, grad, ov, dk, dc, C, delta, offset, num_steps, mode, partial, s);
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
        const int mode      = range.gmin == nullptr ? 0 : range.sym ? 1 : 2;   // lg_bwd_term_m
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
        const LgBwdLaunch L = lg_bwd_launch(n);   // the fp32 kernel's tiles
        float* partial      = static_cast<float*>(scratch_alloc(sizeof(float) * 3 * L.ntiles, s));
        auto xs = static_cast<const unsigned short*>(x);
        auto gs = static_cast<const unsigned short*>(grad);
        auto os = static_cast<unsigned short*>(grad_x);
        const int v = vec ? 1 : 0;
        lg_bwd_dispatch(mode, [&](auto md) {
            constexpr int MD = decltype(md)::value;
            if (io_dtype == IO_F16)
                lg_bwd16_tensor_kernel<IO_F16, kLgTileSteps, MD><<<L.grid16, kBlock, 0, s>>>(
                    xs, gs, os, n, delta, offset, num_steps, partial, v, L.ntiles);
            else
                lg_bwd16_tensor_kernel<IO_BF16, kLgTileSteps, MD><<<L.grid16, kBlock, 0, s>>>(
                    xs, gs, os, n, delta, offset, num_steps, partial, v, L.ntiles);
        });
        AIMET_LAUNCH_CHECK();
        lg_bwd_fold_one<<<1, kBlock, 0, s>>>(partial, L.ntiles, sums, range);
        AIMET_LAUNCH_CHECK();
        scratch_free(partial, s);
    });
}

}   // extern "C"
