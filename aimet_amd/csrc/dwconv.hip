// dwconv.hip -- depthwise 2-D convolution forward and weight gradient for gfx950: the layer math
// of the AdaRound loop on MobileNet-class depthwise layers (aimet_amd.adaround_optimizer).
//
// AdaRound's per-iteration work on a depthwise layer (adaround_optimizer.py:181-218) is
// q_out = conv(x, Wq) and dL/dWq = conv_weight_grad(x, dL/dq_out) over a 32-sample batch; the
// input gradient is never needed. PyTorch's native depthwise kernels take 36 us (forward) and
// 100 us (weight gradient) per MobileNet-v2 depthwise layer-iteration (profiles/r02
// adaround_loop_kernels_v1.csv); both are HBM-bound elementwise-plus-reduction work:
//   forward:     reads x once (neighbours from L1/L2), writes y:   (|x| + |y|) * 4 B
//   weight grad: reads x and dy once:                               (|x| + |dy|) * 4 B
//
// Layout NCHW fp32, square kernel K (3 or 5), square stride / padding / dilation, groups == C
// (one filter per channel), weights [C][1][K][K].
//
// Forward: one lane per output in NCHW order (coalesced stores), y = bias + sum_kh sum_kw
// w * x in that order with fused multiply-adds (PyTorch's conv_depthwise2d_forward_kernel order).
// Weight grad: the (n, oh, ow) positions of a channel are split into S contiguous slices, one
// workgroup each; every lane keeps K*K partial sums, reduced in the workgroup by a fixed shuffle
// tree, stored per slice; a fold kernel adds the slices in order -- deterministic.
#include "common.hpp"
#include "recon.hpp"

#include <cstdlib>

namespace aimet_amd
{
namespace
{

struct DwShape
{
    uint32_t N, C, H, W, OH, OW;
    int stride, pad, dil;
    FastDiv div_ow, div_ohow, div_c;
};

template <int K>
__global__ __launch_bounds__(kBlock) void dw_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        DwShape s, uint32_t total)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= total)
        return;
    const uint32_t nc  = s.div_ohow.div(i);
    const uint32_t rem = i - nc * (s.OH * s.OW);
    const uint32_t oh  = s.div_ow.div(rem);
    const uint32_t ow  = rem - oh * s.OW;
    const uint32_t n   = s.div_c.div(nc);
    const uint32_t c   = nc - n * s.C;
    const float* xp    = x + ((size_t) n * s.C + c) * s.H * s.W;
    const float* wp    = w + c * K * K;
    float v            = bias ? bias[c] : 0.0f;
    const int ih0 = (int) oh * s.stride - s.pad, iw0 = (int) ow * s.stride - s.pad;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
    {
        const int ih = ih0 + kh * s.dil;
        if (ih < 0 || ih >= (int) s.H)
            continue;
#pragma unroll
        for (int kw = 0; kw < K; ++kw)
        {
            const int iw = iw0 + kw * s.dil;
            if (iw >= 0 && iw < (int) s.W)
                v = __builtin_fmaf(wp[kh * K + kw], xp[ih * (int) s.W + iw], v);
        }
    }
    y[i] = v;
}

// partial[(c * S + slice) * K*K + k]: channel c, positions [slice * per, (slice + 1) * per) of its
// N*OH*OW outputs (position p = (n * OH + oh) * OW + ow)
template <int K>
__global__ __launch_bounds__(kBlock) void dw_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                                          float* __restrict__ partial, DwShape s, uint32_t per)
{
    constexpr int KK  = K * K;
    const uint32_t c  = blockIdx.y;
    const uint32_t S  = gridDim.x;
    const uint32_t np = s.N * s.OH * s.OW;
    const uint32_t p0 = blockIdx.x * per;
    const uint32_t p1 = p0 + per < np ? p0 + per : np;
    float acc[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k)
        acc[k] = 0.0f;
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += kBlock)
    {
        const uint32_t n   = s.div_ohow.div(p);
        const uint32_t rem = p - n * (s.OH * s.OW);
        const uint32_t oh  = s.div_ow.div(rem);
        const uint32_t ow  = rem - oh * s.OW;
        const size_t plane = (size_t) n * s.C + c;
        const float g      = gy[plane * s.OH * s.OW + rem];
        const float* xp    = x + ((size_t) n * s.C + c) * s.H * s.W;
        const int ih0 = (int) oh * s.stride - s.pad, iw0 = (int) ow * s.stride - s.pad;
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
        {
            const int ih     = ih0 + kh * s.dil;
            const bool rowin = ih >= 0 && ih < (int) s.H;
#pragma unroll
            for (int kw = 0; kw < K; ++kw)
            {
                const int iw = iw0 + kw * s.dil;
                if (rowin && iw >= 0 && iw < (int) s.W)
                    acc[kh * K + kw] = __builtin_fmaf(g, xp[ih * (int) s.W + iw], acc[kh * K + kw]);
            }
        }
    }
    // workgroup reduction of the K*K sums: wave shuffles, then the waves in order
    __shared__ float sh[KK][kBlock / 64];
#pragma unroll
    for (int k = 0; k < KK; ++k)
    {
        float v = acc[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0)
            sh[k][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < KK)
    {
        float v = 0.0f;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i)
            v += sh[threadIdx.x][i];
        partial[((size_t) c * S + blockIdx.x) * KK + threadIdx.x] = v;
    }
}

// ---- quad forms (K = 3, dilation 1, stride 1 (2 instantiated, not taken), OW % 4 == 0) -----------
// A lane takes 4 consecutive outputs of one row (a quad; OW % 4 == 0 keeps a quad inside its row):
// their 3 x (3 ST + 3) input window is loaded once (18 or 27 loads for 36 taps), the index
// divisions are done once per quad, and the weight-gradient partials accumulate quad by quad,
// output j = 0..3 in order, taps (kh, kw) in order -- in the weight-gradient kernel and in the
// one-pass step alike, so the two stay bit-identical. Taps outside the plane are dropped by selects.
template <int ST>
constexpr int kDwWin = 3 * ST + 3;

template <int ST>
__device__ __forceinline__ void dw_quad_window(const float* __restrict__ xp, int ih0, int iw0, const DwShape& s,
                                               float (&xw)[3][kDwWin<ST>], uint32_t& rowv, uint32_t& colv)
{
    const int H = (int) s.H, W = (int) s.W;
    int iwc[kDwWin<ST>];
    colv = 0;
#pragma unroll
    for (int c = 0; c < kDwWin<ST>; ++c)
    {
        const int iw = iw0 + c;
        colv |= (iw >= 0 && iw < W ? 1u : 0u) << c;
        iwc[c] = iw < 0 ? 0 : (iw >= W ? W - 1 : iw);
    }
    rowv = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
    {
        const int ih   = ih0 + kh;
        const bool rok = ih >= 0 && ih < H;
        rowv |= (rok ? 1u : 0u) << kh;
        const float* xr = xp + (ih < 0 ? 0 : (ih >= H ? H - 1 : ih)) * W;
#pragma unroll
        for (int c = 0; c < kDwWin<ST>; ++c)
        {
            const float v = xr[iwc[c]];
            xw[kh][c]     = rok && ((colv >> c) & 1u) ? v : 0.0f;
        }
    }
}

// acc[k] += g[j] * tap(j, k) for the quad's outputs j = 0..3 in order (taps outside the plane skipped)
template <int ST>
__device__ __forceinline__ void dw_quad_accumulate(const float (&xw)[3][kDwWin<ST>], uint32_t rowv, uint32_t colv,
                                                   const float (&g)[4], float (&acc)[9])
{
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw)
            {
                const int c   = j * ST + kw;
                const bool ok = ((rowv >> kh) & 1u) && ((colv >> c) & 1u);
                const float f = __builtin_fmaf(g[j], xw[kh][c], acc[kh * 3 + kw]);
                acc[kh * 3 + kw] = ok ? f : acc[kh * 3 + kw];
            }
}

__device__ __forceinline__ void dw_block_partial(const float (&acc)[9], float* __restrict__ partial, uint32_t c,
                                                 uint32_t S)
{
    __shared__ float sh[9][kBlock / 64];
#pragma unroll
    for (int k = 0; k < 9; ++k)
    {
        float v = acc[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0)
            sh[k][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < 9)
    {
        float v = 0.0f;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i)
            v += sh[threadIdx.x][i];
        partial[((size_t) c * S + blockIdx.x) * 9 + threadIdx.x] = v;
    }
}

// dw_wgrad_kernel in quads (positions [blockIdx.x * per, ...) of channel c, per % 4 == 0)
template <int ST>
__global__ __launch_bounds__(kBlock) void dw_wgrad_quad_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                                               float* __restrict__ partial, DwShape s, uint32_t per)
{
    const uint32_t c  = blockIdx.y;
    const uint32_t np = s.N * s.OH * s.OW;
    const uint32_t p0 = blockIdx.x * per;
    const uint32_t p1 = p0 + per < np ? p0 + per : np;
    float acc[9];
#pragma unroll
    for (int k = 0; k < 9; ++k)
        acc[k] = 0.0f;
    for (uint32_t qb = p0 / 4 + threadIdx.x; qb < p1 / 4; qb += kBlock)
    {
        const uint32_t p   = 4 * qb;
        const uint32_t n   = s.div_ohow.div(p);
        const uint32_t rem = p - n * (s.OH * s.OW);
        const uint32_t oh  = s.div_ow.div(rem);
        const uint32_t ow  = rem - oh * s.OW;
        const size_t plane = (size_t) n * s.C + c;
        const float4 g4    = *reinterpret_cast<const float4*>(gy + plane * s.OH * s.OW + rem);
        const float g[4]   = {g4.x, g4.y, g4.z, g4.w};
        float xw[3][kDwWin<ST>];
        uint32_t rowv, colv;
        dw_quad_window<ST>(x + plane * s.H * s.W, (int) oh * ST - s.pad, (int) ow * ST - s.pad, s, xw, rowv, colv);
        dw_quad_accumulate<ST>(xw, rowv, colv, g, acc);
    }
    dw_block_partial(acc, partial, c, gridDim.x);
}

// The AdaRound iteration of a depthwise layer up to dL/dWq in ONE pass over the batch
// (aimet_adaround_dw_step). For the positions of dw_wgrad_kernel's slices, sample n's input plane
// and fp target are read in place from the caches (row idx_all[it][n]); q = dw_fwd_kernel's sum,
// g = recon_grad_idx_kernel's gradient of q (recon_g), and the K*K products g * x accumulate in
// dw_wgrad_kernel's order: the partials -- and grad_w after dw_wgrad_fold -- are bit-identical to
// gather -> dw_fwd -> recon_grad_idx -> dw_wgrad, with no batch copy of the input and neither q nor
// g in HBM (the caches are read once: |x| + |target| bytes per iteration instead of ~9 passes).
struct DwStep
{
    const float* x_cache;     // [rows][C][H][W]
    const float* t_cache;     // [rows][C][OH][OW]
    const int64_t* idx_all;   // [iterations][N]
    const int64_t* it_cur;
    int64_t* it_next;         // workgroup (0, 0) writes it + 1 (as adaround_gather_kernel)
    const float* w;           // [C][K][K]
    const float* bias;        // nullable
    float scale;              // 2 / (N * OH * OW)
    int act;
};

// U positions per lane in flight (their taps, target and sample row loaded before any of them is
// reduced; the accumulation order stays p, p + kBlock, ...), the batch's cache rows in LDS: the
// loop is otherwise a chain of dependent loads per position
template <int K, int UU>
constexpr int kDwStepU = UU > 0 ? UU : (K == 3 ? 4 : 2);
constexpr int kDwStepRows = 1024;   // batches up to this size keep their row table in LDS

template <int K, int UU = 0>
__global__ __launch_bounds__(kBlock) void dw_step_kernel(DwStep a, float* __restrict__ partial, DwShape s,
                                                         uint32_t per)
{
    constexpr int KK  = K * K;
    constexpr int U   = kDwStepU<K, UU>;
    const uint32_t c  = blockIdx.y;
    const uint32_t S  = gridDim.x;
    const uint32_t np = s.N * s.OH * s.OW;
    const uint32_t p0 = blockIdx.x * per;
    const uint32_t p1 = p0 + per < np ? p0 + per : np;
    // the channel's taps and bias first: they do not depend on the iteration counter, so their
    // loads overlap its round trip and the batch-row table's
    float wk[KK], acc[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k)
    {
        wk[k]  = a.w[c * KK + k];
        acc[k] = 0.0f;
    }
    const float b0    = a.bias ? a.bias[c] : 0.0f;
    const int64_t it  = a.it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        a.it_next[0] = it + 1;
    const int64_t* rows = a.idx_all + it * (int64_t) s.N;
    __shared__ int64_t srows[kDwStepRows];
    const bool lds_rows = s.N <= (uint32_t) kDwStepRows;
    if (lds_rows)
        for (uint32_t i = threadIdx.x; i < s.N; i += kBlock)
            srows[i] = rows[i];
    __syncthreads();
    for (uint32_t pb = p0 + threadIdx.x; pb < p1; pb += kBlock * U)
    {
        float xv[U][KK], tv[U];
        int ih0[U], iw0[U];
        uint32_t valid[U];   // bit k: tap k inside the plane
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = pb + u * kBlock;
            ih0[u]   = 0;
            iw0[u]   = 0;
            valid[u] = 0;   // an out-of-range position: every tap skipped, nothing added
            tv[u]    = 0.0f;
#pragma unroll
            for (int k = 0; k < KK; ++k)
                xv[u][k] = 0.0f;
            if (p < p1)
            {
                const uint32_t n   = s.div_ohow.div(p);
                const uint32_t rem = p - n * (s.OH * s.OW);
                const uint32_t oh  = s.div_ow.div(rem);
                const uint32_t ow  = rem - oh * s.OW;
                const size_t plane = (size_t) (lds_rows ? srows[n] : rows[n]) * s.C + c;
                const float* xp    = a.x_cache + plane * s.H * s.W;
                tv[u]  = a.t_cache[plane * s.OH * s.OW + rem];
                ih0[u] = (int) oh * s.stride - s.pad;
                iw0[u] = (int) ow * s.stride - s.pad;
                // branch-free taps: every load reads an in-plane address (clamped) and a tap outside
                // the plane is dropped by a select on a validity bit, never by control flow (per-tap
                // branches cost ~300 scalar instructions per 4 positions); the FMAs and their order
                // are the four-launch chain's
                uint32_t m = 0;
#pragma unroll
                for (int kh = 0; kh < K; ++kh)
                {
                    const int ih   = ih0[u] + kh * s.dil;
                    const bool rin = ih >= 0 && ih < (int) s.H;
                    const int ihc  = ih < 0 ? 0 : (ih >= (int) s.H ? (int) s.H - 1 : ih);
#pragma unroll
                    for (int kw = 0; kw < K; ++kw)
                    {
                        const int iw  = iw0[u] + kw * s.dil;
                        const bool ok = rin && iw >= 0 && iw < (int) s.W;
                        const int iwc = iw < 0 ? 0 : (iw >= (int) s.W ? (int) s.W - 1 : iw);
                        const float xval = xp[ihc * (int) s.W + iwc];
                        xv[u][kh * K + kw] = ok ? xval : 0.0f;
                        m |= (ok ? 1u : 0u) << (kh * K + kw);
                    }
                }
                valid[u] = m;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (pb + u * kBlock >= p1)
                break;
            const uint32_t m = valid[u];
            float v = b0;
#pragma unroll
            for (int k = 0; k < KK; ++k)
            {
                const float f = __builtin_fmaf(wk[k], xv[u][k], v);
                v = (m >> k) & 1u ? f : v;
            }
            // recon_grad_idx_kernel adds the (absent) bias as + 0.0f: the same here
            const float g = recon_g(v + 0.0f, tv[u], a.scale, a.act);
#pragma unroll
            for (int k = 0; k < KK; ++k)
            {
                const float f = __builtin_fmaf(g, xv[u][k], acc[k]);
                acc[k] = (m >> k) & 1u ? f : acc[k];
            }
        }
    }
    __shared__ float sh[KK][kBlock / 64];
#pragma unroll
    for (int k = 0; k < KK; ++k)
    {
        float v = acc[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
            v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0)
            sh[k][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < KK)
    {
        float v = 0.0f;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i)
            v += sh[threadIdx.x][i];
        partial[((size_t) c * S + blockIdx.x) * KK + threadIdx.x] = v;
    }
}

// aimet_adaround_dw_step in quads: q of the quad's 4 outputs (dw_fwd_kernel's FMA order), their
// gradients, and dw_wgrad_quad_kernel's accumulation -- bit-identical to gather + dw_fwd_kernel +
// recon_grad_idx_kernel + dw_wgrad_quad_kernel; 2 quads per lane in flight
template <int ST>
__global__ __launch_bounds__(kBlock) void dw_step_quad_kernel(DwStep a, float* __restrict__ partial, DwShape s,
                                                              uint32_t per)
{
    constexpr int U   = 2;
    const uint32_t c  = blockIdx.y;
    const uint32_t np = s.N * s.OH * s.OW;
    const uint32_t p0 = blockIdx.x * per;
    const uint32_t p1 = p0 + per < np ? p0 + per : np;
    // the taps and bias ahead of the iteration counter (see dw_step_kernel)
    float wk[9], acc[9];
#pragma unroll
    for (int k = 0; k < 9; ++k)
    {
        wk[k]  = a.w[c * 9 + k];
        acc[k] = 0.0f;
    }
    const float b0    = a.bias ? a.bias[c] : 0.0f;
    const int64_t it  = a.it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        a.it_next[0] = it + 1;
    const int64_t* rows = a.idx_all + it * (int64_t) s.N;
    __shared__ int64_t srows[kDwStepRows];
    const bool lds_rows = s.N <= (uint32_t) kDwStepRows;
    if (lds_rows)
        for (uint32_t i = threadIdx.x; i < s.N; i += kBlock)
            srows[i] = rows[i];
    __syncthreads();
    const uint32_t q1 = p1 / 4;
    for (uint32_t qbb = p0 / 4 + threadIdx.x; qbb < q1; qbb += kBlock * U)
    {
        float xw[U][3][kDwWin<ST>], tq[U][4];
        uint32_t rowv[U], colv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t qb = qbb + u * kBlock;
            rowv[u] = colv[u] = 0;
            if (qb < q1)
            {
                const uint32_t p   = 4 * qb;
                const uint32_t n   = s.div_ohow.div(p);
                const uint32_t rem = p - n * (s.OH * s.OW);
                const uint32_t oh  = s.div_ow.div(rem);
                const uint32_t ow  = rem - oh * s.OW;
                const size_t plane = (size_t) (lds_rows ? srows[n] : rows[n]) * s.C + c;
                const float4 t4    = *reinterpret_cast<const float4*>(a.t_cache + plane * s.OH * s.OW + rem);
                tq[u][0] = t4.x;
                tq[u][1] = t4.y;
                tq[u][2] = t4.z;
                tq[u][3] = t4.w;
                dw_quad_window<ST>(a.x_cache + plane * s.H * s.W, (int) oh * ST - s.pad, (int) ow * ST - s.pad, s,
                                   xw[u], rowv[u], colv[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            if (qbb + u * kBlock >= q1)
                break;
            float g[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
            {
                float v = b0;
#pragma unroll
                for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                    for (int kw = 0; kw < 3; ++kw)
                    {
                        const int cc  = j * ST + kw;
                        const bool ok = ((rowv[u] >> kh) & 1u) && ((colv[u] >> cc) & 1u);
                        const float f = __builtin_fmaf(wk[kh * 3 + kw], xw[u][kh][cc], v);
                        v = ok ? f : v;
                    }
                // recon_grad_idx_kernel adds the (absent) bias as + 0.0f: the same here
                g[j] = recon_g(v + 0.0f, tq[u][j], a.scale, a.act);
            }
            dw_quad_accumulate<ST>(xw[u], rowv[u], colv[u], g, acc);
        }
    }
    dw_block_partial(acc, partial, c, gridDim.x);
}

__global__ __launch_bounds__(kBlock) void dw_wgrad_fold(const float* __restrict__ partial, float* __restrict__ gw,
                                                        uint32_t C, uint32_t S, uint32_t KK)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;   // (c, k)
    if (i >= C * KK)
        return;
    const uint32_t c = i / KK, k = i - c * KK;
    float v          = 0.0f;
    for (uint32_t sl = 0; sl < S; ++sl)
        v += partial[((size_t) c * S + sl) * KK + k];
    gw[i] = v;
}

// slices of >= 16 positions per lane, and enough workgroups (~2048) to fill the chip
inline bool aligned16(const void* p)
{
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

// the quad forms apply (dw_wgrad_quad_kernel, dw_step_quad_kernel)
// (stride 2 measured slower in quads: 84 -> 125 us on 96 channels at 112^2, profiles/r03/dw_step_tune.jsonl;
// the kernels keep the stride-2 instantiation for that comparison)
bool dw_quads(int64_t K, int64_t stride, int64_t dil, int64_t OW)
{
    return K == 3 && dil == 1 && stride == 1 && OW % 4 == 0;
}

int64_t wgrad_slices(int64_t N, int64_t C, int64_t OH, int64_t OW, uint32_t* per_out, bool quads = false)
{
    const int64_t np   = N * OH * OW;
    // positions per lane per slice (it sets the summation order of the weight gradient, for the
    // fused and the unfused path alike)
    constexpr int64_t ppl = 16;
    int64_t S          = ceil_div(np, (int64_t) kBlock * ppl);
    const int64_t want = ceil_div(2048, C);
    if (S < want)
        S = want < ceil_div(np, kBlock) ? want : ceil_div(np, kBlock);
    if (S < 1)
        S = 1;
    uint32_t per = (uint32_t) ceil_div(np, S);
    if (quads)
        per = (per + 3) / 4 * 4;   // slices of whole quads (np % 4 == 0 when OW % 4 == 0)
    if (per_out)
        *per_out = per;
    return ceil_div(np, per);
}

DwShape make_shape(int64_t N, int64_t C, int64_t H, int64_t W, int64_t OH, int64_t OW, int K, int stride, int pad,
                   int dil)
{
    AIMET_REQUIRE(K == 3 || K == 5, "depthwise kernel size must be 3 or 5");
    AIMET_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && OH > 0 && OW > 0, "invalid depthwise shape");
    AIMET_REQUIRE(stride > 0 && pad >= 0 && dil > 0, "invalid stride / padding / dilation");
    AIMET_REQUIRE((OH - 1) * stride - 2 * pad + dil * (K - 1) + 1 <= H && (OW - 1) * stride - 2 * pad + dil * (K - 1) + 1 <= W,
                  "output size inconsistent with the input size");
    AIMET_REQUIRE(N * C * H * W < (int64_t(1) << 31) && N * C * OH * OW < (int64_t(1) << 31),
                  "depthwise tensors must have < 2^31 elements");
    DwShape s;
    s.N = (uint32_t) N, s.C = (uint32_t) C, s.H = (uint32_t) H, s.W = (uint32_t) W, s.OH = (uint32_t) OH;
    s.OW = (uint32_t) OW, s.stride = stride, s.pad = pad, s.dil = dil;
    s.div_ow   = FastDiv((uint32_t) OW);
    s.div_ohow = FastDiv((uint32_t) (OH * OW));
    s.div_c    = FastDiv((uint32_t) C);
    return s;
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

namespace
{

void dw_forward(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C, int64_t H,
                int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride, int32_t pad, int32_t dilation,
                hipStream_t st)
{
    DwShape s = make_shape(N, C, H, W, OH, OW, K, stride, pad, dilation);
    require_device_ptr(x, "x");
    require_device_ptr(w, "weight");
    require_device_ptr(y, "y");
    if (bias)
        require_device_ptr(bias, "bias");
    const uint32_t total = (uint32_t) (N * C * OH * OW);
    const unsigned grid  = (unsigned) ceil_div(total, kBlock);
    if (K == 3)
        dw_fwd_kernel<3><<<grid, kBlock, 0, st>>>(x, w, bias, y, s, total);
    else
        dw_fwd_kernel<5><<<grid, kBlock, 0, st>>>(x, w, bias, y, s, total);
    AIMET_LAUNCH_CHECK();
}

void dw_grad_weight(const float* x, const float* grad_y, float* grad_w, float* workspace, int64_t N, int64_t C,
                    int64_t H, int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride, int32_t pad,
                    int32_t dilation, hipStream_t st)
{
    DwShape s = make_shape(N, C, H, W, OH, OW, K, stride, pad, dilation);
    require_device_ptr(x, "x");
    require_device_ptr(grad_y, "grad_y");
    require_device_ptr(grad_w, "grad_w");
    AIMET_REQUIRE(C <= 65535, "depthwise weight gradient: at most 65535 channels");
    uint32_t per      = 0;
    const bool quads  = dw_quads(K, stride, dilation, OW) && aligned16(grad_y);
    const int64_t S   = wgrad_slices(N, C, OH, OW, &per, quads);
    // a caller-owned workspace (aimet_dwconv2d_grad_weight_workspace elements) keeps the call
    // free of allocations, e.g. inside a HIP-graph capture
    if (workspace)
        require_device_ptr(workspace, "workspace");
    float* partial = workspace ? workspace
                               : static_cast<float*>(scratch_alloc(sizeof(float) * (size_t) (C * S * K * K), st));
    dim3 grid((unsigned) S, (unsigned) C);
    if (quads && stride == 1)
        dw_wgrad_quad_kernel<1><<<grid, kBlock, 0, st>>>(x, grad_y, partial, s, per);
    else if (quads)
        dw_wgrad_quad_kernel<2><<<grid, kBlock, 0, st>>>(x, grad_y, partial, s, per);
    else if (K == 3)
        dw_wgrad_kernel<3><<<grid, kBlock, 0, st>>>(x, grad_y, partial, s, per);
    else
        dw_wgrad_kernel<5><<<grid, kBlock, 0, st>>>(x, grad_y, partial, s, per);
    AIMET_LAUNCH_CHECK();
    dw_wgrad_fold<<<(unsigned) ceil_div(C * K * K, kBlock), kBlock, 0, st>>>(partial, grad_w, (uint32_t) C,
                                                                            (uint32_t) S, (uint32_t) (K * K));
    AIMET_LAUNCH_CHECK();
    if (!workspace)
        scratch_free(partial, st);
}

void dw_step(const float* x_cache, const float* t_cache, const int64_t* idx_all, const int64_t* it_cur,
             int64_t* it_next, const float* w, const float* bias, float* grad_w, float* workspace, int64_t N,
             int64_t C, int64_t H, int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride, int32_t pad,
             int32_t dilation, int32_t act, hipStream_t st)
{
    DwShape s = make_shape(N, C, H, W, OH, OW, K, stride, pad, dilation);
    AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
    AIMET_REQUIRE(C <= 65535, "depthwise weight gradient: at most 65535 channels");
    require_device_ptr(x_cache, "x_cache");
    require_device_ptr(t_cache, "target_cache");
    require_device_ptr(idx_all, "idx_all");
    require_device_ptr(it_cur, "it_cur");
    require_device_ptr(it_next, "it_next");
    require_device_ptr(w, "weight");
    AIMET_REQUIRE(grad_w || workspace, "grad_w may be null only with a workspace (the slices stay there)");
    if (grad_w)
        require_device_ptr(grad_w, "grad_w");
    if (bias)
        require_device_ptr(bias, "bias");
    uint32_t per     = 0;
    // the quad form exactly when aimet_dwconv2d_grad_weight takes it (the gradient's buffer there
    // is a 16-B aligned torch / scratch allocation; the target cache here is checked)
    const bool quads = dw_quads(K, stride, dilation, OW) && aligned16(t_cache);
    const int64_t S  = wgrad_slices(N, C, OH, OW, &per, quads);
    if (workspace)
        require_device_ptr(workspace, "workspace");
    float* partial = workspace ? workspace
                               : static_cast<float*>(scratch_alloc(sizeof(float) * (size_t) (C * S * K * K), st));
    // aimet_adaround_recon_grad_indexed's scale: 2 / (number of dim-1 norms)
    DwStep a {x_cache, t_cache, idx_all, it_cur, it_next, w, bias, (float) (2.0 / (double) (N * OH * OW)), act};
    dim3 grid((unsigned) S, (unsigned) C);
    // (1, 2 or 8 positions per lane in flight instead of the default measured no faster:
    // profiles/r03/dw_step_tune.jsonl)
    if (quads && stride == 1)
        dw_step_quad_kernel<1><<<grid, kBlock, 0, st>>>(a, partial, s, per);
    else if (quads)
        dw_step_quad_kernel<2><<<grid, kBlock, 0, st>>>(a, partial, s, per);
    else if (K == 3)
        dw_step_kernel<3><<<grid, kBlock, 0, st>>>(a, partial, s, per);
    else
        dw_step_kernel<5><<<grid, kBlock, 0, st>>>(a, partial, s, per);
    AIMET_LAUNCH_CHECK();
    if (grad_w)   // else the Adam step folds the [C][S][K K] slices (aimet_adaround_backward_adam_parts)
    {
        dw_wgrad_fold<<<(unsigned) ceil_div(C * K * K, kBlock), kBlock, 0, st>>>(partial, grad_w, (uint32_t) C,
                                                                                (uint32_t) S, (uint32_t) (K * K));
        AIMET_LAUNCH_CHECK();
    }
    if (!workspace)
        scratch_free(partial, st);
}

}   // namespace

extern "C" {

int aimet_dwconv2d_forward(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C,
                           int64_t H, int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride, int32_t pad,
                           int32_t dilation, void* stream)
{
    return guarded([&] {
        dw_forward(x, w, bias, y, N, C, H, W, OH, OW, K, stride, pad, dilation, as_stream(stream));
    });
}

int aimet_dwconv2d_grad_weight_workspace(int64_t N, int64_t C, int64_t OH, int64_t OW, int32_t K, int64_t* elems)
{
    return guarded([&] {
        AIMET_REQUIRE(elems != nullptr, "elems is null");
        AIMET_REQUIRE(N > 0 && C > 0 && OH > 0 && OW > 0 && (K == 3 || K == 5), "invalid depthwise shape");
        *elems = C * wgrad_slices(N, C, OH, OW, nullptr) * K * K;
    });
}

int aimet_dwconv2d_grad_weight(const float* x, const float* grad_y, float* grad_w, float* workspace, int64_t N,
                               int64_t C, int64_t H, int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride,
                               int32_t pad, int32_t dilation, void* stream)
{
    return guarded([&] {
        dw_grad_weight(x, grad_y, grad_w, workspace, N, C, H, W, OH, OW, K, stride, pad, dilation,
                       as_stream(stream));
    });
}

int aimet_adaround_dw_step(const float* x_cache, const float* target_cache, const int64_t* idx_all,
                           const int64_t* it_cur, int64_t* it_next, const float* w, const float* bias, float* grad_w,
                           float* workspace, int64_t N, int64_t C, int64_t H, int64_t W, int64_t OH, int64_t OW,
                           int32_t K, int32_t stride, int32_t pad, int32_t dilation, int32_t act, void* stream)
{
    return guarded([&] {
        dw_step(x_cache, target_cache, idx_all, it_cur, it_next, w, bias, grad_w, workspace, N, C, H, W, OH, OW, K,
                stride, pad, dilation, act, as_stream(stream));
    });
}

int aimet_adaround_dw_step_slices(const float* target_cache, int64_t N, int64_t C, int64_t OH, int64_t OW, int32_t K,
                                  int32_t stride, int32_t dilation, int64_t* slices)
{
    return guarded([&] {
        AIMET_REQUIRE(slices != nullptr, "slices is null");
        AIMET_REQUIRE(N > 0 && C > 0 && OH > 0 && OW > 0 && (K == 3 || K == 5), "invalid depthwise shape");
        const bool quads = dw_quads(K, stride, dilation, OW) && aligned16(target_cache);
        uint32_t per     = 0;
        *slices          = wgrad_slices(N, C, OH, OW, &per, quads);
    });
}

}   // extern "C"
