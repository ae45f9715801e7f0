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
//     Xs[ci][t]   <- x_cache[row][ci][hw0 + t]                         (LDS)
//     q[co][t]     = sum_ci W[co][ci] * Xs[ci][t]  (ci ascending, fmaf) (registers)
//     Gs[co][t]    = recon_g(q + bias[co], target[row][co][hw0 + t])    (LDS; recon.hpp, as
//                    aimet_adaround_recon_grad_indexed with the bias: the GEMM form's arithmetic)
//     acc[co][ci] += sum_t Gs[co][t] * Xs[ci][t]   (t ascending, fmaf)  (registers, per lane)
//   each workgroup walks tiles blockIdx.x, + gridDim.x, ... and stores its Cout x Cin partial;
//   a fold adds the partials in workgroup order: deterministic.
//
// Sizes: Cin, Cout <= 192, Cin * Cout <= 6144 and at most 512 4 x 4 gradient blocks (two per
// lane); fp32, NCHW caches with HW = H * W positions per channel plane, HW % 4 == 0.
//
// Measured (profiles/r03/adaround_pw_fused_forms.txt): faster than the GEMM form on expanding
// layers (C_out >= 4 C_in) at >= 56^2 positions, slower on projecting layers, so the loop takes
// it by that shape rule (adaround_optimizer.py: _PW_FUSED). The kernel is LDS-bound; the dL/dW
// phase's 16-B reads of Xs rows 4 apart (stride 144 floats = 16 banks) conflict 4-way, and a
// position-major copy of Xs / Gs for that phase is the next step.
#include "common.hpp"
#include "recon.hpp"

namespace aimet_amd
{
namespace
{

constexpr int kPwT     = 32;                    // positions per tile
constexpr int kPwPad   = kPwT + 4;              // LDS row stride (16-B aligned rows)
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

// Register blocking (LDS operand traffic, not HBM, bounded the first version: 2 LDS reads per FMA):
//   q / g:  lane (tq, cr) = (lane % 8, lane / 8) computes t = 4 tq .. 4 tq + 3 of rows
//           co = cr + 32 j: per ci one 16-B read of Xs and one read of W per row for 4 FMAs per row;
//   dL/dW:  lane b owns blocks b and b + 256 of 4 x 4 (co, ci) pairs (blocks row-major over
//           ceil(Cout / 4) x ceil(Cin / 4)): per 4 positions 8 16-B reads for 64 FMAs.
// Rows of Xs / Gs past Cin / Cout up to the next multiple of 4 are zero, so partial blocks add 0.
constexpr int kPwJ      = kPwMaxC / 32;   // 6 output rows per lane in the q / g phase
constexpr int kPwBlocks = 2;              // 4 x 4 gradient blocks per lane

__global__ __launch_bounds__(kBlock, 2) void pw_step_kernel(PwStep a, float* __restrict__ partial)
{
    __shared__ __attribute__((aligned(16))) float Xs[kPwMaxC * kPwPad];
    __shared__ __attribute__((aligned(16))) float Gs[kPwMaxC * kPwPad];
    __shared__ float Ws[kPwPairs];
    const uint32_t Cin = a.Cin, Cout = a.Cout, pairs = Cin * Cout;
    const uint32_t Cin4 = (Cin + 3) / 4, Cout4 = (Cout + 3) / 4;
    const int64_t it = a.it_cur[0];
    if (blockIdx.x == 0 && threadIdx.x == 0)
        a.it_next[0] = it + 1;
    const int64_t* rows = a.idx_all + it * (int64_t) a.N;
    for (uint32_t e = threadIdx.x; e < pairs; e += kBlock)
        Ws[e] = a.w[e];
    for (uint32_t e = threadIdx.x; e < (4 * Cin4 - Cin) * kPwPad; e += kBlock)
        Xs[Cin * kPwPad + e] = 0.0f;
    for (uint32_t e = threadIdx.x; e < (4 * Cout4 - Cout) * kPwPad; e += kBlock)
        Gs[Cout * kPwPad + e] = 0.0f;
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
        const float* tr    = a.t_cache + (size_t) rows[n] * Cout * a.HW;   // uniform base
        __syncthreads();   // the previous tile's Xs / Gs are consumed (and Ws / the pads written)
#pragma unroll
        for (int k = 0; k < kPwQuads; ++k)
        {
            const uint32_t q = threadIdx.x + kBlock * k;
            if (q < Cin * (kPwT / 4))
                *reinterpret_cast<float4*>(Xs + (q / (kPwT / 4)) * kPwPad + 4 * (q % (kPwT / 4))) = nxt[k];
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
        float4 q[kPwJ];
#pragma unroll
        for (int j = 0; j < kPwJ; ++j)
            q[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (uint32_t ci = 0; ci < Cin; ++ci)
        {
            const float4 xv = *reinterpret_cast<const float4*>(Xs + ci * kPwPad + 4 * tq);
#pragma unroll
            for (int j = 0; j < kPwJ; ++j)
            {
                const uint32_t co = cr + 32 * j;
                if (co < Cout)
                {
                    const float wv = Ws[co * Cin + ci];
                    q[j].x = __builtin_fmaf(wv, xv.x, q[j].x);
                    q[j].y = __builtin_fmaf(wv, xv.y, q[j].y);
                    q[j].z = __builtin_fmaf(wv, xv.z, q[j].z);
                    q[j].w = __builtin_fmaf(wv, xv.w, q[j].w);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < kPwJ; ++j)
        {
            const uint32_t co = cr + 32 * j;
            if (co < Cout)
            {
                const float bs = a.bias ? a.bias[co] : 0.0f;
                float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
                if (t_in)
                {
                    g.x = recon_g(q[j].x + bs, tv[j].x, a.scale, a.act);
                    g.y = recon_g(q[j].y + bs, tv[j].y, a.scale, a.act);
                    g.z = recon_g(q[j].z + bs, tv[j].z, a.scale, a.act);
                    g.w = recon_g(q[j].w + bs, tv[j].w, a.scale, a.act);
                }
                *reinterpret_cast<float4*>(Gs + co * kPwPad + 4 * tq) = g;
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
                const float* g0 = Gs + 4 * cb * kPwPad;
                const float* x0 = Xs + 4 * ib * kPwPad;
#pragma unroll 2
                for (int t4 = 0; t4 < kPwT / 4; ++t4)
                {
                    float4 gv[4], xv[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                    {
                        gv[r] = *reinterpret_cast<const float4*>(g0 + r * kPwPad + 4 * t4);
                        xv[r] = *reinterpret_cast<const float4*>(x0 + r * kPwPad + 4 * t4);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                        {
                            float v = acc[bl][r * 4 + c];
                            v = __builtin_fmaf(gv[r].x, xv[c].x, v);
                            v = __builtin_fmaf(gv[r].y, xv[c].y, v);
                            v = __builtin_fmaf(gv[r].z, xv[c].z, v);
                            v = __builtin_fmaf(gv[r].w, xv[c].w, v);
                            acc[bl][r * 4 + c] = v;
                        }
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
                        partial[(size_t) blockIdx.x * pairs + co * Cin + ci] = acc[bl][r * 4 + c];
                }
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

int aimet_adaround_pw_step_workspace(int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int64_t* elems)
{
    return guarded([&] {
        AIMET_REQUIRE(elems != nullptr, "elems is null");
        AIMET_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && HW > 0, "invalid shape");
        const int64_t tiles = N * ceil_div(HW, (int64_t) kPwT);
        *elems              = ((int64_t) pw_grid(tiles) + kPwSlices) * Cin * Cout;
    });
}

int aimet_adaround_pw_step(const float* x_cache, const float* target_cache, const int64_t* idx_all,
                           const int64_t* it_cur, int64_t* it_next, const float* w, const float* bias, float* grad_w,
                           float* workspace, int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int32_t act,
                           void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && HW > 0, "invalid shape");
        AIMET_REQUIRE(Cin <= kPwMaxC && Cout <= kPwMaxC && Cin * Cout <= kPwPairs,
                      "pointwise step: Cin, Cout <= 192 and Cin * Cout <= 6144");
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        AIMET_REQUIRE(N * HW < (int64_t(1) << 31) / kPwT, "batch too large");
        AIMET_REQUIRE(HW % 4 == 0 && (reinterpret_cast<uintptr_t>(x_cache) & 15) == 0 &&
                          (reinterpret_cast<uintptr_t>(target_cache) & 15) == 0,
                      "pointwise step: HW % 4 == 0 and 16-B aligned caches");
        AIMET_REQUIRE(ceil_div(Cin, (int64_t) 4) * ceil_div(Cout, (int64_t) 4) <= (int64_t) kBlock * kPwBlocks,
                      "pointwise step: at most 512 4x4 weight-gradient blocks");
        require_device_ptr(x_cache, "x_cache");
        require_device_ptr(target_cache, "target_cache");
        require_device_ptr(idx_all, "idx_all");
        require_device_ptr(it_cur, "it_cur");
        require_device_ptr(it_next, "it_next");
        require_device_ptr(w, "weight");
        require_device_ptr(grad_w, "grad_w");
        if (bias)
            require_device_ptr(bias, "bias");
        const int64_t tps   = ceil_div(HW, (int64_t) kPwT);
        const int64_t tiles = N * tps;
        const uint32_t grid = pw_grid(tiles);
        const int64_t pairs = Cin * Cout;
        hipStream_t st      = as_stream(stream);
        if (workspace)
            require_device_ptr(workspace, "workspace");
        const size_t ws_elems = ((size_t) grid + kPwSlices) * (size_t) pairs;
        float* part = workspace ? workspace : static_cast<float*>(scratch_alloc(sizeof(float) * ws_elems, st));
        float* part2 = part + (size_t) grid * pairs;
        PwStep a {x_cache, target_cache, idx_all, it_cur, it_next, w, bias,
                  (float) (2.0 / (double) (N * HW)), act, (uint32_t) N, (uint32_t) Cin, (uint32_t) Cout,
                  (uint32_t) HW, (uint32_t) tps, (uint32_t) tiles};
        pw_step_kernel<<<grid, kBlock, 0, st>>>(a, part);
        AIMET_LAUNCH_CHECK();
        const uint32_t chunk   = (uint32_t) ceil_div((int64_t) grid, (int64_t) kPwSlices);
        const uint32_t nslices = (uint32_t) ceil_div((int64_t) grid, (int64_t) chunk);
        const unsigned gx      = (unsigned) ceil_div(pairs, (int64_t) kBlock);
        pw_fold_slices<<<dim3(gx, nslices), kBlock, 0, st>>>(part, part2, (uint32_t) pairs, grid, chunk);
        AIMET_LAUNCH_CHECK();
        pw_fold_final<<<gx, kBlock, 0, st>>>(part2, grad_w, (uint32_t) pairs, nslices);
        AIMET_LAUNCH_CHECK();
        if (!workspace)
            scratch_free(part, st);
    });
}

}   // extern "C"
