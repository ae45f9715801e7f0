// pwstep.hip -- the AdaRound iteration of a 1x1 convolution with few channels, up to dL/dWq, in
// one pass over the cached rows (aimet_adaround_pw_step).
//
// The GEMM form of the loop (adaround_optimizer.py: gather -> torch.matmul -> the fused
// reconstruction gradient -> a weight-gradient GEMM) moves the batch through HBM ~7 times:
// the input copy (2|x|), q written and read (2|q|), the target (|q|), g written and read (2|q|),
// x again (|x|). On MobileNet-v2's high-resolution 1x1 layers (16..192 channels at 28^2..112^2,
// batch 32) that is 0.1-0.24 ms per iteration. Here one kernel reads x and the fp target once
// (|x| + |q| bytes) and keeps q, g and the weight-gradient partials on chip:
//
//   per tile of T = 32 positions of one sample (rows idx_all[it][n] of the caches):
//     XT[t][ci]   <- x_cache[row][ci][hw0 + t]                         (LDS)
//     q[co][t]     = sum_ci W[co][ci] * XT[t][ci]  (ci ascending, fmaf) (registers)
//     GT[t][co]    = recon_g(q + bias[co], target[row][co][hw0 + t])    (LDS; recon.hpp, as
//                    aimet_adaround_recon_grad_indexed with the bias: the GEMM form's arithmetic)
//     acc[co][ci] += sum_t GT[t][co] * XT[t][ci]   (t ascending, fmaf)  (registers, per lane)
//   each workgroup walks tiles blockIdx.x, + gridDim.x, ... and stores its Cout x Cin partial;
//   a fold adds the partials in workgroup order: deterministic.
//
// Sizes: Cin <= 192; a workgroup covers R output rows (blockIdx.y: row range) with R * Cin <= 6144
// and at most 512 4 x 4 gradient blocks (two per lane) -- all of C_out when it fits, else several
// row ranges, each reading the input tile again; fp32, NCHW caches with HW = H * W positions per
// channel plane, HW % 4 == 0.
//
// Measured (profiles/r03/adaround_pw_fused_forms.txt): faster than the GEMM form on MobileNet-v2's
// expanding layers and the stem (0.24 -> 0.16 ms per iteration at 16 -> 96 x 112^2), even at
// 56^2 on projecting ones, slower on projecting layers below 56^2, which the loop's shape rule
// leaves to the GEMM form (adaround_optimizer.py: _PW_FUSED). The kernel is LDS-bound; its LDS
// images are position-major so the dL/dW phase's 16-B reads are contiguous across lanes (the
// ci-major first version was 1.2-1.9x slower).
#include "common.hpp"
#include "recon.hpp"

#include <algorithm>
#include <cstdlib>

namespace aimet_amd
{
namespace
{

constexpr int kPwT     = 32;                    // positions per tile
constexpr int kPwMaxC  = 192;
constexpr int kPwPairs = 6144;

struct PwStep
{
    const float* x_cache;     // [rows][Cin][HW]
    const float* t_cache;     // [rows][Cout][HW]
    const int64_t* idx_all;   // [iterations][N]
    const int64_t* it_cur;
    int64_t* it_next;         // workgroup 0 writes it + 1 (as adaround_gather_kernel)
    const float* w;           // [Cout][Cin]
    const float* bias;        // nullable: added to q before the gradient (the GEMM form's recon)
    float scale;              // 2 / (N * HW)
    int act;
    uint32_t N, Cin, Cout, HW, tiles_per_sample, tiles;
    uint32_t R;               // output rows per workgroup row range (blockIdx.y): [y R, y R + R)
};

// one tile's input quads of this lane: q = threadIdx.x + kBlock k (ci = q / (T / 4), t = 4 (q % (T / 4)));
// issued for the next tile while the current one is computed. HW % 4 == 0 and 16-B aligned
// planes (checked by the host), so a quad is entirely inside or outside the plane.
constexpr int kPwQuads = kPwMaxC * kPwT / 4 / kBlock;   // 6

__device__ __forceinline__ void pw_load_x(const PwStep& a, const int64_t* rows, uint32_t tile, float4 (&x)[kPwQuads])
{
    const uint32_t n   = tile / a.tiles_per_sample;
    const uint32_t hw0 = (tile - n * a.tiles_per_sample) * kPwT;
    const float* xr    = a.x_cache + (size_t) rows[n] * a.Cin * a.HW;   // uniform base
#pragma unroll
    for (int k = 0; k < kPwQuads; ++k)
    {
        const uint32_t q = threadIdx.x + kBlock * k, ci = q / (kPwT / 4), t = 4 * (q % (kPwT / 4));
        const uint32_t off = ci * a.HW + hw0 + t;
        x[k] = q < a.Cin * (kPwT / 4) && hw0 + t < a.HW ? *reinterpret_cast<const float4*>(xr + off)
                                                         : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// Register blocking, position-major LDS images (XT[t][ci], GT[t][co]; row stride kPwRow floats):
//   q / g:  lane (tq, cr) = (lane % 8, lane / 8) computes t = 4 tq .. 4 tq + 3 of rows
//           co = cr + 32 j: per 4 input channels four 16-B reads of XT (its 4 positions) and one
//           16-B read of W per row for 16 FMAs per row (ci ascending);
//   dL/dW:  lane b owns blocks b and b + 256 of 4 x 4 (co, ci) pairs (blocks row-major over
//           ceil(Cout / 4) x ceil(Cin / 4)): per position one 16-B read of GT and one of XT for 16
//           FMAs (t ascending); consecutive lanes read consecutive 16-B chunks of an XT row.
// Columns of XT / GT / W past Cin / Cout up to the next multiple of 4 are zero.
constexpr int kPwJ      = kPwMaxC / 32;     // 6 output rows per lane in the q / g phase
constexpr int kPwBlocks = 2;                // 4 x 4 gradient blocks per lane
constexpr int kPwRow    = kPwMaxC + 4;      // XT / GT row stride (16-B aligned)

__global__ __launch_bounds__(kBlock, 2) void pw_step_kernel(PwStep a, float* __restrict__ partial)
{
    __shared__ __attribute__((aligned(16))) float XT[kPwT * kPwRow];
    __shared__ __attribute__((aligned(16))) float GT[kPwT * kPwRow];
    __shared__ __attribute__((aligned(16))) float Ws[kPwPairs + 3 * kPwMaxC];
    // this workgroup's output rows [r0, r0 + Cout) of the layer's a.Cout (blockIdx.y: row range)
    const uint32_t r0 = blockIdx.y * a.R;
    const uint32_t Cin = a.Cin, Cout = a.Cout - r0 < a.R ? a.Cout - r0 : a.R, pairs = Cin * a.Cout;
    const uint32_t Cin4 = (Cin + 3) / 4, Cout4 = (Cout + 3) / 4, wrow = 4 * Cin4;
    // W first: it does not depend on the iteration counter, so its loads overlap that round trip
    for (uint32_t e = threadIdx.x; e < Cout * wrow; e += kBlock)
    {
        const uint32_t co = e / wrow, ci = e - co * wrow;
        Ws[e] = ci < Cin ? a.w[(r0 + co) * Cin + ci] : 0.0f;
    }
    const int64_t it = a.it_cur[0];
    if (blockIdx.x == 0 && threadIdx.x == 0)
        a.it_next[0] = it + 1;
    const int64_t* rows = a.idx_all + it * (int64_t) a.N;
    for (uint32_t e = threadIdx.x; e < kPwT * (wrow - Cin); e += kBlock)
        XT[(e / (wrow - Cin)) * kPwRow + Cin + e % (wrow - Cin)] = 0.0f;
    for (uint32_t e = threadIdx.x; e < kPwT * (4 * Cout4 - Cout); e += kBlock)
        GT[(e / (4 * Cout4 - Cout)) * kPwRow + Cout + e % (4 * Cout4 - Cout)] = 0.0f;
    const uint32_t tq = threadIdx.x % 8, cr = threadIdx.x / 8;
    float acc[kPwBlocks][16];
#pragma unroll
    for (int bl = 0; bl < kPwBlocks; ++bl)
#pragma unroll
        for (int k = 0; k < 16; ++k)
            acc[bl][k] = 0.0f;
    float4 nxt[kPwQuads];
    if (blockIdx.x < a.tiles)
        pw_load_x(a, rows, blockIdx.x, nxt);
    for (uint32_t tile = blockIdx.x; tile < a.tiles; tile += gridDim.x)
    {
        const uint32_t n   = tile / a.tiles_per_sample;
        const uint32_t hw0 = (tile - n * a.tiles_per_sample) * kPwT;
        const bool t_in    = hw0 + 4 * tq < a.HW;   // HW % 4 == 0: the quad is in or out
        const float* tr    = a.t_cache + ((size_t) rows[n] * a.Cout + r0) * a.HW;   // uniform base
        __syncthreads();   // the previous tile's XT / GT are consumed (and W / the pads written)
#pragma unroll
        for (int k = 0; k < kPwQuads; ++k)
        {
            const uint32_t q = threadIdx.x + kBlock * k;
            if (q < Cin * (kPwT / 4))
            {
                const uint32_t ci = q / (kPwT / 4), t = 4 * (q % (kPwT / 4));
                XT[t * kPwRow + ci]       = nxt[k].x;
                XT[(t + 1) * kPwRow + ci] = nxt[k].y;
                XT[(t + 2) * kPwRow + ci] = nxt[k].z;
                XT[(t + 3) * kPwRow + ci] = nxt[k].w;
            }
        }
        __syncthreads();
        if (tile + gridDim.x < a.tiles)
            pw_load_x(a, rows, tile + gridDim.x, nxt);
        // the targets of this lane's outputs, issued before the sums
        float4 tv[kPwJ];
#pragma unroll
        for (int j = 0; j < kPwJ; ++j)
        {
            const uint32_t co = cr + 32 * j;
            tv[j] = co < Cout && t_in ? *reinterpret_cast<const float4*>(tr + co * a.HW + hw0 + 4 * tq)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float q[kPwJ][4];
#pragma unroll
        for (int j = 0; j < kPwJ; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                q[j][k] = 0.0f;
        for (uint32_t c4 = 0; c4 < Cin4; ++c4)
        {
            float4 xv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                xv[k] = *reinterpret_cast<const float4*>(XT + (4 * tq + k) * kPwRow + 4 * c4);
#pragma unroll
            for (int j = 0; j < kPwJ; ++j)
            {
                const uint32_t co = cr + 32 * j;
                if (co < Cout)
                {
                    const float4 wv = *reinterpret_cast<const float4*>(Ws + co * wrow + 4 * c4);
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                    {
                        float v = q[j][k];
                        v = __builtin_fmaf(wv.x, xv[k].x, v);
                        v = __builtin_fmaf(wv.y, xv[k].y, v);
                        v = __builtin_fmaf(wv.z, xv[k].z, v);
                        v = __builtin_fmaf(wv.w, xv[k].w, v);
                        q[j][k] = v;
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kPwJ; ++j)
        {
            const uint32_t co = cr + 32 * j;
            if (co < Cout)
            {
                const float bs = a.bias ? a.bias[r0 + co] : 0.0f;
                const float tk[4] = {tv[j].x, tv[j].y, tv[j].z, tv[j].w};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    GT[(4 * tq + k) * kPwRow + co] = t_in ? recon_g(q[j][k] + bs, tk[k], a.scale, a.act) : 0.0f;
            }
        }
        __syncthreads();
        // dL/dW blocks: 4 output rows x 4 input rows, positions t ascending
#pragma unroll
        for (int bl = 0; bl < kPwBlocks; ++bl)
        {
            const uint32_t b = threadIdx.x + kBlock * bl;
            if (b < Cout4 * Cin4)
            {
                const uint32_t cb = b / Cin4, ib = b - cb * Cin4;
#pragma unroll 4
                for (int t = 0; t < kPwT; ++t)
                {
                    const float4 gv = *reinterpret_cast<const float4*>(GT + t * kPwRow + 4 * cb);
                    const float4 xv = *reinterpret_cast<const float4*>(XT + t * kPwRow + 4 * ib);
                    const float g4[4] = {gv.x, gv.y, gv.z, gv.w}, x4[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            acc[bl][r * 4 + c] = __builtin_fmaf(g4[r], x4[c], acc[bl][r * 4 + c]);
                }
            }
        }
    }
#pragma unroll
    for (int bl = 0; bl < kPwBlocks; ++bl)
    {
        const uint32_t b = threadIdx.x + kBlock * bl;
        if (b < Cout4 * Cin4)
        {
            const uint32_t cb = b / Cin4, ib = b - cb * Cin4;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                {
                    const uint32_t co = 4 * cb + r, ci = 4 * ib + c;
                    if (co < Cout && ci < Cin)
                        partial[(size_t) blockIdx.x * pairs + (r0 + co) * Cin + ci] = acc[bl][r * 4 + c];
                }
        }
    }
}

// ---- the same step on the f32 matrix cores ------------------------------------------------
// pw_step_kernel spends its time on LDS operand reads for VALU FMAs (16 FMAs per two 16-B reads).
// Here both contractions are v_mfma_f32_32x32x2_f32 (A[i][k] from lane (i, h) = (lane & 31,
// lane >> 5) at k = 2 st + h, B[k][j] at j = i; C row (r & 3) + 8 (r >> 2) + 4 h, column i):
//   per tile of 32 positions of one sample, X[ci][p] staged in LDS (rows padded to 33 floats: the
//   column reads of the second product hit distinct banks), W[co][ci] staged once;
//   Q (Cp x 32, Cp = rows rounded up to 32) = W X, one 32 x 32 block per wave (blocks w, w + 4);
//   G = recon_g(Q + bias, target) into LDS (zero past the sample's end); the next tile's X and
//   targets are loaded while this tile's weight gradient runs;
//   dW (Cp x Kp, Kp = Cin rounded up to 32) += G X^T over the 32 positions, the 32 x 32 output
//   blocks spread over the waves (<= 3 each) and kept in accumulators across the workgroup's
//   tiles; the partial per workgroup is folded as pw_step_kernel's (pw_fold_slices / _final).
// Sums in a fixed order (deterministic); not bit-identical to pw_step_kernel's FMA chains.
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kPmT   = 32;   // positions per tile
constexpr int kPmLd  = 33;   // X / G row stride (floats)
constexpr int kPmMaxT = 3;   // weight-gradient blocks per wave

struct PmShape
{
    uint32_t Cp, Kw, Kx, nblk1, nblk3n, nblk3;   // rows padded, W row stride, X rows, block counts
};

template <int XB, int TB>
__global__ __launch_bounds__(kBlock, 2) void pw_mfma_step_kernel(PwStep a, PmShape m, float* __restrict__ partial)
{
    extern __shared__ float lds[];
    float* Ws = lds;                         // [Cp][Kw]
    float* Xs = Ws + m.Cp * m.Kw;            // [Kx][33]
    float* Gs = Xs + m.Kx * kPmLd;           // [Cp][33]
    const uint32_t r0 = blockIdx.y * a.R;
    const uint32_t Cin = a.Cin, Cout = a.Cout - r0 < a.R ? a.Cout - r0 : a.R, pairs = Cin * a.Cout;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    // W (zero past Cin / the range's rows) and the X rows past Cin (zero, never rewritten), ahead
    // of the iteration counter (independent of it)
    for (uint32_t e = threadIdx.x; e < m.Cp * m.Kw; e += kBlock)
    {
        const uint32_t co = e / m.Kw, ci = e - co * m.Kw;
        Ws[e] = (co < Cout && ci < Cin) ? a.w[(size_t) (r0 + co) * Cin + ci] : 0.0f;
    }
    for (uint32_t e = Cin * kPmLd + threadIdx.x; e < m.Kx * kPmLd; e += kBlock)
        Xs[e] = 0.0f;
    const int64_t it = a.it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        a.it_next[0] = it + 1;
    const int64_t* rows = a.idx_all + it * (int64_t) a.N;
    // this tile's X (XB per lane: element q = threadIdx.x + kBlock j -> ci = q / 32, p = q % 32)
    // and this wave's targets (its GEMM1 blocks w, w + 4, ...: 16 per block)
    float xr[XB], tr[TB][16];
    auto load = [&](uint32_t tile) {
        const uint32_t n   = tile / a.tiles_per_sample;
        const uint32_t hw0 = (tile - n * a.tiles_per_sample) * kPmT;
        const size_t row   = (size_t) rows[n];
        const float* xb    = a.x_cache + row * Cin * a.HW + hw0;
#pragma unroll
        for (int j = 0; j < XB; ++j)
        {
            const uint32_t q = threadIdx.x + kBlock * j, ci = q / kPmT, p = q % kPmT;
            const bool in    = ci < Cin && hw0 + p < a.HW;
            xr[j]            = in ? xb[(size_t) ci * a.HW + p] : 0.0f;
        }
        const float* tb = a.t_cache + (row * a.Cout + r0) * a.HW + hw0 + i;
        const bool pin  = hw0 + i < a.HW;
#pragma unroll
        for (int b = 0; b < TB; ++b)
        {
            const uint32_t mb = wave + 4 * b;
#pragma unroll
            for (int r = 0; r < 16; ++r)
            {
                const uint32_t co = mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                tr[b][r]          = (mb < m.nblk1 && co < Cout && pin) ? tb[(size_t) co * a.HW] : 0.0f;
            }
        }
    };
    f32x16 acc3[kPmMaxT];
#pragma unroll
    for (int t = 0; t < kPmMaxT; ++t)
        acc3[t] = f32x16 {};
    if (blockIdx.x < a.tiles)
        load(blockIdx.x);
    for (uint32_t tile = blockIdx.x; tile < a.tiles; tile += gridDim.x)
    {
        const uint32_t n   = tile / a.tiles_per_sample;
        const uint32_t hw0 = (tile - n * a.tiles_per_sample) * kPmT;
        __syncthreads();   // the previous tile's products are done with Xs / Gs (and Ws is written)
#pragma unroll
        for (int j = 0; j < XB; ++j)
        {
            const uint32_t q = threadIdx.x + kBlock * j, ci = q / kPmT, p = q % kPmT;
            if (ci < Cin)
                Xs[ci * kPmLd + p] = xr[j];
        }
        __syncthreads();
        // Q = W X for this wave's blocks, then G into LDS
        const bool pin = hw0 + i < a.HW;
#pragma unroll
        for (int b = 0; b < TB; ++b)
        {
            const uint32_t mb = wave + 4 * b;
            if (mb >= m.nblk1)
                continue;
            f32x16 q = {};
            const float* wrow = Ws + (mb * 32 + i) * m.Kw;
            for (uint32_t st = 0; 2 * st < Cin; ++st)   // k = 2 st + h < Cin rounded up to even (zero pad)
                q = __builtin_amdgcn_mfma_f32_32x32x2f32(wrow[2 * st + h], Xs[(2 * st + h) * kPmLd + i], q, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r)
            {
                const uint32_t co = mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                float gv          = 0.0f;
                if (co < Cout && pin)
                    gv = recon_g(q[r] + (a.bias ? a.bias[r0 + co] : 0.0f), tr[b][r], a.scale, a.act);
                Gs[co * kPmLd + i] = gv;
            }
        }
        if (tile + gridDim.x < a.tiles)
            load(tile + gridDim.x);   // in flight through the weight gradient below
        __syncthreads();
        // dW += G X^T over the tile's 32 positions
#pragma unroll
        for (int t = 0; t < kPmMaxT; ++t)
        {
            const uint32_t blk = wave + 4 * t;
            if (blk >= m.nblk3)
                continue;
            const uint32_t mb = blk / m.nblk3n, nbk = blk - mb * m.nblk3n;
            const float* grow = Gs + (mb * 32 + i) * kPmLd;
            const float* xrow = Xs + (nbk * 32 + i) * kPmLd;
#pragma unroll 4
            for (int st = 0; st < kPmT / 2; ++st)
                acc3[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(grow[2 * st + h], xrow[2 * st + h], acc3[t], 0, 0, 0);
        }
    }
#pragma unroll
    for (int t = 0; t < kPmMaxT; ++t)
    {
        const uint32_t blk = wave + 4 * t;
        if (blk >= m.nblk3)
            continue;
        const uint32_t mb = blk / m.nblk3n, nbk = blk - mb * m.nblk3n, ci = nbk * 32 + i;
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const uint32_t co = mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (co < Cout && ci < Cin)
                partial[(size_t) blockIdx.x * pairs + (size_t) (r0 + co) * Cin + ci] = acc3[t][r];
        }
    }
}

// The fold of the workgroups' partials, in two levels so that ~512 partials of up to 6144 pairs
// are read by enough lanes: level 1 sums workgroups [s * chunk, (s + 1) * chunk) of pair e in
// order into part2[s][e]; level 2 sums the kPwSlices slices in order (deterministic).
constexpr uint32_t kPwSlices = 32;

__global__ __launch_bounds__(kBlock) void pw_fold_slices(const float* __restrict__ partial, float* __restrict__ part2,
                                                         uint32_t pairs, uint32_t nparts, uint32_t chunk)
{
    const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= pairs)
        return;
    const uint32_t b0 = blockIdx.y * chunk, b1 = b0 + chunk < nparts ? b0 + chunk : nparts;
    float v = 0.0f;
    for (uint32_t b = b0; b < b1; ++b)
        v += partial[(size_t) b * pairs + e];
    part2[(size_t) blockIdx.y * pairs + e] = v;
}

__global__ __launch_bounds__(kBlock) void pw_fold_final(const float* __restrict__ part2, float* __restrict__ gw,
                                                        uint32_t pairs, uint32_t nslices)
{
    const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= pairs)
        return;
    float v = 0.0f;
    for (uint32_t s = 0; s < nslices; ++s)
        v += part2[(size_t) s * pairs + e];
    gw[e] = v;
}

// workgroups: at least ~4 tiles each (fewer partials to fold), at most 2 per CU (~78 KiB of LDS
// each)
constexpr int64_t kPwGrid = 512;

uint32_t pw_grid(int64_t tiles)
{
    int64_t g = ceil_div(tiles, (int64_t) 4);
    g         = g < 1 ? 1 : (g > kPwGrid ? kPwGrid : g);
    return (uint32_t) g;
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

// the matrix-core form's padded shape for a row range of R rows (pw_mfma_step_kernel)
static PmShape pm_shape(int64_t Cin, int64_t R)
{
    PmShape m;
    m.Cp     = (uint32_t) (ceil_div(R, (int64_t) 32) * 32);
    const uint32_t cin2 = (uint32_t) (ceil_div(Cin, (int64_t) 2) * 2);
    m.Kw     = cin2 + 1;
    m.nblk1  = m.Cp / 32;
    m.nblk3n = (uint32_t) ceil_div(Cin, (int64_t) 32);
    m.Kx     = std::max<uint32_t>(cin2, m.nblk3n * 32);
    m.nblk3  = m.nblk1 * m.nblk3n;
    return m;
}

// the matrix-core form's row ranges: at most 128 rows (one 32-row output block per wave), as few
// ranges as that allows, each a multiple of 32 rows but the last
static int64_t pm_rows(int64_t Cin, int64_t Cout)
{
    const int64_t nr = ceil_div(Cout, (int64_t) 128);
    (void) Cin;
    return ceil_div(ceil_div(Cout, nr), (int64_t) 32) * 32;
}

// the matrix-core form for C_in >= 32 where its staging fits (W, X and G in <= 64 KiB of LDS,
// <= 3 weight-gradient blocks per wave), else the VALU form. Below 32 input channels the weight
// gradient's 32-wide blocks are mostly padding and the forward's sums 8-16 steps deep: MobileNet-v2's
// stem and its 16 / 24-channel expanding layers ran 16-40 % slower there, the C_in >= 32 layers
// 9-20 % faster (profiles/r04/README.md)
static bool pw_uses_mfma(int64_t Cin, int64_t Cout, PmShape* shape = nullptr, size_t* lds_bytes = nullptr)
{
    const PmShape pm = pm_shape(Cin, pm_rows(Cin, Cout));
    const size_t lds = sizeof(float) * ((size_t) pm.Cp * pm.Kw + (size_t) pm.Kx * kPmLd + (size_t) pm.Cp * kPmLd);
    if (shape)
        *shape = pm;
    if (lds_bytes)
        *lds_bytes = lds;
    return Cin >= 32 && lds <= 65536 && pm.nblk1 <= 4 && pm.nblk3 <= 4 * kPmMaxT;
}

// output rows per workgroup row range: all of them when they fit (C_out <= 192, C_in C_out <= 6144),
// else the most that do, a multiple of 4
static int64_t pw_rows(int64_t Cin, int64_t Cout)
{
    int64_t r = kPwPairs / Cin;
    r         = r > kPwMaxC ? kPwMaxC : r;
    if (Cout <= r)
        return Cout;
    return r - r % 4;
}

int aimet_adaround_pw_step_uses_mfma(int64_t Cin, int64_t Cout, int* uses)
{
    return guarded([&] {
        AIMET_REQUIRE(Cin > 0 && Cout > 0 && uses != nullptr, "invalid argument");
        *uses = pw_uses_mfma(Cin, Cout) ? 1 : 0;
    });
}

int aimet_adaround_pw_step_workspace(int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int64_t* elems)
{
    return guarded([&] {
        AIMET_REQUIRE(elems != nullptr, "elems is null");
        AIMET_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && HW > 0, "invalid shape");
        const int64_t tiles = N * ceil_div(HW, (int64_t) kPwT);
        *elems              = ((int64_t) pw_grid(tiles) + kPwSlices) * Cin * Cout;
    });
}

// where aimet_adaround_pw_step leaves its second-level slices when grad_w is NULL: workspace
// elements [offset, offset + slices * C_in * C_out), [slices][C_out][C_in], added in slice order
// from +0 by pw_fold_final (aimet_adaround_backward_adam_parts with part_kk = C_in * C_out: the same
// sum)
int aimet_adaround_pw_step_slices(int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int64_t* offset, int64_t* slices)
{
    return guarded([&] {
        AIMET_REQUIRE(offset != nullptr && slices != nullptr, "null output");
        AIMET_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && HW > 0, "invalid shape");
        const int64_t tiles  = N * ceil_div(HW, (int64_t) kPwT);
        const uint32_t grid  = pw_grid(tiles);
        const uint32_t chunk = (uint32_t) ceil_div((int64_t) grid, (int64_t) kPwSlices);
        *offset              = (int64_t) grid * Cin * Cout;
        *slices              = ceil_div((int64_t) grid, (int64_t) chunk);
    });
}

int aimet_adaround_pw_step(const float* x_cache, const float* target_cache, const int64_t* idx_all,
                           const int64_t* it_cur, int64_t* it_next, const float* w, const float* bias, float* grad_w,
                           float* workspace, int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int32_t act,
                           void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && HW > 0, "invalid shape");
        AIMET_REQUIRE(Cin <= kPwMaxC, "pointwise step: Cin <= 192");
        AIMET_REQUIRE(Cout < (int64_t(1) << 24), "pointwise step: too many output channels");
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        AIMET_REQUIRE(N * HW < (int64_t(1) << 31) / kPwT, "batch too large");
        AIMET_REQUIRE(HW % 4 == 0 && (reinterpret_cast<uintptr_t>(x_cache) & 15) == 0 &&
                          (reinterpret_cast<uintptr_t>(target_cache) & 15) == 0,
                      "pointwise step: HW % 4 == 0 and 16-B aligned caches");
        require_device_ptr(x_cache, "x_cache");
        require_device_ptr(target_cache, "target_cache");
        require_device_ptr(idx_all, "idx_all");
        require_device_ptr(it_cur, "it_cur");
        require_device_ptr(it_next, "it_next");
        require_device_ptr(w, "weight");
        AIMET_REQUIRE(grad_w || workspace, "grad_w may be null only with a workspace (the slices stay there)");
        if (grad_w)
            require_device_ptr(grad_w, "grad_w");
        if (bias)
            require_device_ptr(bias, "bias");
        PmShape pm {};
        size_t lds      = 0;
        const bool mfma = pw_uses_mfma(Cin, Cout, &pm, &lds);
        const int64_t R   = mfma ? pm_rows(Cin, Cout) : pw_rows(Cin, Cout);
        AIMET_REQUIRE(mfma || ((R >= 4 || R == Cout) && R * Cin <= kPwPairs &&
                               ceil_div(Cin, (int64_t) 4) * ceil_div(R, (int64_t) 4) <= (int64_t) kBlock * kPwBlocks),
                      "pointwise step: at most 512 4x4 weight-gradient blocks per row range");
        const int64_t tps    = ceil_div(HW, (int64_t) kPwT);
        const int64_t tiles  = N * tps;
        const uint32_t grid  = pw_grid(tiles);
        const int64_t ranges = ceil_div(Cout, R);
        AIMET_REQUIRE(ranges <= 65535, "pointwise step: too many row ranges");
        const int64_t pairs = Cin * Cout;
        hipStream_t st      = as_stream(stream);
        if (workspace)
            require_device_ptr(workspace, "workspace");
        const size_t ws_elems = ((size_t) grid + kPwSlices) * (size_t) pairs;
        float* part = workspace ? workspace : static_cast<float*>(scratch_alloc(sizeof(float) * ws_elems, st));
        float* part2 = part + (size_t) grid * pairs;
        PwStep a {x_cache, target_cache, idx_all, it_cur, it_next, w, bias,
                  (float) (2.0 / (double) (N * HW)), act, (uint32_t) N, (uint32_t) Cin, (uint32_t) Cout,
                  (uint32_t) HW, (uint32_t) tps, (uint32_t) tiles, (uint32_t) R};
        if (mfma)
        {
            // X loads per lane (Cin x 32 / 256, bucketed) sized per layer, so a small layer holds no
            // idle registers; one target block per wave (row ranges of <= 128 rows, pm_rows)
            const dim3 g2(grid, (unsigned) ranges);
            auto go = [&](auto xb) {
                pw_mfma_step_kernel<decltype(xb)::value, 1><<<g2, kBlock, lds, st>>>(a, pm, part);
            };
            if (Cin <= 32)
                go(std::integral_constant<int, 4> {});
            else if (Cin <= 64)
                go(std::integral_constant<int, 8> {});
            else if (Cin <= 96)
                go(std::integral_constant<int, 12> {});
            else if (Cin <= 144)
                go(std::integral_constant<int, 18> {});
            else
                go(std::integral_constant<int, 24> {});
        }
        else
            pw_step_kernel<<<dim3(grid, (unsigned) ranges), kBlock, 0, st>>>(a, part);
        AIMET_LAUNCH_CHECK();
        const uint32_t chunk   = (uint32_t) ceil_div((int64_t) grid, (int64_t) kPwSlices);
        const uint32_t nslices = (uint32_t) ceil_div((int64_t) grid, (int64_t) chunk);
        const unsigned gx      = (unsigned) ceil_div(pairs, (int64_t) kBlock);
        pw_fold_slices<<<dim3(gx, nslices), kBlock, 0, st>>>(part, part2, (uint32_t) pairs, grid, chunk);
        AIMET_LAUNCH_CHECK();
        if (grad_w)   // else the Adam step adds the slices (aimet_adaround_pw_step_slices)
        {
            pw_fold_final<<<gx, kBlock, 0, st>>>(part2, grad_w, (uint32_t) pairs, nslices);
            AIMET_LAUNCH_CHECK();
        }
        if (!workspace)
            scratch_free(part, st);
    });
}

}   // extern "C"
