// pwcm.hip -- the AdaRound loop's iteration for 1x1 layers with many channels at small spatial
// sizes (MobileNet-v2's 14x14 / 7x7 expand and project layers), channel-major over the batch's
// nb * hw positions, on the f32-input matrix cores.
//
// Reference: adaround_optimizer.py:181-218 runs, per iteration, the batch draw (index_select of
// the cached inputs and fp outputs), the wrapped layer's forward, the reconstruction loss and
// autograd's weight gradient. The GEMM form of that (aimet_adaround_gather_cm, a library GEMM,
// aimet_adaround_recon_grad_indexed_cm, a second library GEMM) is five graph nodes of tiny work
// each. Here it is two kernels (and the Adam step, which folds the weight gradient's slices):
//
//  * aimet_adaround_pw_cm_forward: g[co][p] = recon_g(sum_ci W[co][ci] x[ci][p] + bias[co],
//    target) for p = b * hw + t over the batch, x[ci][p] gathered in place from row
//    idx_all[it][b] of the input cache (no channel-major copy), the target read in place; 64 x 64
//    output tiles, 32-deep K chunks staged in LDS, one 32 x 32 v_mfma_f32_32x32x2_f32 accumulator
//    per wave (the f32 matrix instruction: exact fmaf chains in ci order, deterministic);
//  * aimet_adaround_pw_cm_wgrad: part[s][co][ci] = sum over the positions of slice s of
//    g[co][p] x[ci][p] (x gathered again), slices over the positions so that the small
//    [Cout][Cin] output still fills the chip; aimet_adaround_backward_adam_parts adds the slices
//    in slice order.
//
// Results are fp32 GEMM sums in a fixed order: deterministic, equal to the library GEMMs to fp32
// summation tolerance (not bit for bit).
#include "common.hpp"
#include "recon.hpp"

namespace aimet_amd
{
namespace
{

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kT  = 64;   // output tile (rows x columns), 2 x 2 waves of 32 x 32
constexpr int kKc = 32;   // K chunk staged in LDS per step
constexpr int kLdA = kKc + 1;    // [64][33]: lanes reading one k column hit distinct banks
constexpr int kLdB = kT + 4;     // [32][68]

struct CmBatch
{
    const float* x;          // [rows][Cin][hw]
    const int64_t* idx_all;  // [iterations][nb]
    const int64_t* it_cur;
    uint32_t nb, Cin, Cout, hw, P;   // P = nb * hw
    FastDiv div_hw;
};

// x[ci][p] of this iteration's batch (0 outside the problem)
__device__ __forceinline__ float load_x(const CmBatch& B, const int64_t* rows, uint32_t ci, uint32_t p)
{
    if (ci >= B.Cin || p >= B.P)
        return 0.0f;
    const uint32_t b = B.div_hw.div(p), t = p - b * B.hw;
    return B.x[((size_t) rows[b] * B.Cin + ci) * B.hw + t];
}

// acc += A[64 x kKc] . B[kKc x 64] for this wave's 32 x 32 quarter (wr, wc): 16 MFMA steps of k = 2
__device__ __forceinline__ void mfma_chunk(const float (*As)[kLdA], const float (*Bs)[kLdB], int wr, int wc, f32x16& acc)
{
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < kKc / 2; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[wr * 32 + i][2 * s + h], Bs[2 * s + h][wc * 32 + i], acc, 0, 0, 0);
}

// forward + reconstruction gradient: tile (blockIdx.y: 64 output channels, blockIdx.x: 64 positions)
__global__ __launch_bounds__(256) void pw_cm_forward_kernel(CmBatch B, const float* __restrict__ target,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            float* __restrict__ g, int64_t* __restrict__ it_next,
                                                            float scale, int act)
{
    __shared__ float As[kT][kLdA];   // W[co][ci]
    __shared__ float Bs[kKc][kLdB];  // x[ci][p]
    const int64_t it = B.it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        it_next[0] = it + 1;
    const int64_t* rows = B.idx_all + it * B.nb;
    const uint32_t p0 = blockIdx.x * kT, co0 = blockIdx.y * kT;
    const int tid = threadIdx.x, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
    f32x16 acc = {};
    for (uint32_t k0 = 0; k0 < B.Cin; k0 += kKc)
    {
#pragma unroll
        for (int j = 0; j < kT * kKc / 256; ++j)   // A: 64 x 32, consecutive ci across lanes
        {
            const int e = tid + 256 * j, r = e / kKc, k = e % kKc;
            const uint32_t co = co0 + r, ci = k0 + k;
            As[r][k] = (co < B.Cout && ci < B.Cin) ? w[(size_t) co * B.Cin + ci] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < kT * kKc / 256; ++j)   // B: 32 x 64, consecutive positions across lanes
        {
            const int e = tid + 256 * j, k = e / kT, c = e % kT;
            Bs[k][c] = load_x(B, rows, k0 + k, p0 + c);
        }
        __syncthreads();
        mfma_chunk(As, Bs, wr, wc, acc);
        __syncthreads();
    }
    // C/D map of the 32 x 32 f32 MFMA: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int lane = tid & 63;
    const uint32_t p = p0 + wc * 32 + (lane & 31);
    if (p >= B.P)
        return;
    const uint32_t b = B.div_hw.div(p), t = p - b * B.hw;
    const float* trow = target + (size_t) rows[b] * B.Cout * B.hw + t;
#pragma unroll
    for (int r = 0; r < 16; ++r)
    {
        const uint32_t co = co0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (co < B.Cout)
            g[(size_t) co * B.P + p] = recon_g(acc[r] + (bias ? bias[co] : 0.0f), trow[(size_t) co * B.hw], scale, act);
    }
}

// weight-gradient slice s (blockIdx.z) for the tile (blockIdx.y: 64 output channels, blockIdx.x:
// 64 input channels): sum over the slice's positions in order, K chunks of 32 positions
__global__ __launch_bounds__(256) void pw_cm_wgrad_kernel(CmBatch B, const float* __restrict__ g,
                                                          float* __restrict__ part, uint32_t per_slice)
{
    __shared__ float As[kT][kLdA];   // g[co][p]
    __shared__ float Bs[kKc][kLdB];  // x[ci][p], stored [p][ci]
    const int64_t it    = B.it_cur[0];
    const int64_t* rows = B.idx_all + it * B.nb;
    const uint32_t ci0 = blockIdx.x * kT, co0 = blockIdx.y * kT;
    const uint32_t ps = blockIdx.z * per_slice, pe = ps + per_slice < B.P ? ps + per_slice : B.P;
    const int tid = threadIdx.x, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
    f32x16 acc = {};
    for (uint32_t k0 = ps; k0 < pe; k0 += kKc)
    {
#pragma unroll
        for (int j = 0; j < kT * kKc / 256; ++j)   // A: g rows, consecutive positions across lanes
        {
            const int e = tid + 256 * j, r = e / kKc, k = e % kKc;
            const uint32_t co = co0 + r, p = k0 + k;
            As[r][k] = (co < B.Cout && p < pe) ? g[(size_t) co * B.P + p] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < kT * kKc / 256; ++j)   // B: x^T, consecutive positions across lanes
        {
            const int e = tid + 256 * j, c = e / kKc, k = e % kKc;
            Bs[k][c] = k0 + k < pe ? load_x(B, rows, ci0 + c, k0 + k) : 0.0f;
        }
        __syncthreads();
        mfma_chunk(As, Bs, wr, wc, acc);
        __syncthreads();
    }
    const int lane = tid & 63;
    const uint32_t ci = ci0 + wc * 32 + (lane & 31);
    if (ci >= B.Cin)
        return;
    float* out = part + (size_t) blockIdx.z * B.Cout * B.Cin;
#pragma unroll
    for (int r = 0; r < 16; ++r)
    {
        const uint32_t co = co0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (co < B.Cout)
            out[(size_t) co * B.Cin + ci] = acc[r];
    }
}

CmBatch cm_batch(const float* x, const int64_t* idx_all, const int64_t* it_cur, int64_t nb, int64_t Cin, int64_t Cout,
                 int64_t hw)
{
    AIMET_REQUIRE(nb > 0 && Cin > 0 && Cout > 0 && hw > 0, "invalid shape");
    AIMET_REQUIRE(nb * hw < (int64_t(1) << 31) && Cout * nb * hw < (int64_t(1) << 40) && Cin < (1 << 24) &&
                      Cout < (1 << 24),
                  "channel-major batch too large");
    require_device_ptr(x, "x_cache");
    require_device_ptr(idx_all, "idx_all");
    require_device_ptr(it_cur, "it_cur");
    return CmBatch {x, idx_all, it_cur, (uint32_t) nb, (uint32_t) Cin, (uint32_t) Cout, (uint32_t) hw,
                    (uint32_t) (nb * hw), FastDiv((uint32_t) hw)};
}

}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

int aimet_adaround_pw_cm_forward(const float* x_cache, const float* target_cache, const int64_t* idx_all,
                                 const int64_t* it_cur, int64_t* it_next, const float* w, const float* bias,
                                 float* grad_q, int64_t nb, int64_t Cin, int64_t Cout, int64_t hw, int32_t act,
                                 void* stream)
{
    return guarded([&] {
        const CmBatch B = cm_batch(x_cache, idx_all, it_cur, nb, Cin, Cout, hw);
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        require_device_ptr(target_cache, "target_cache");
        require_device_ptr(it_next, "it_next");
        require_device_ptr(w, "weight");
        require_device_ptr(grad_q, "grad_q");
        if (bias)
            require_device_ptr(bias, "bias");
        const float scale = (float) (2.0 / (double) (nb * hw));   // as aimet_adaround_recon_grad_indexed_cm
        const dim3 grid((unsigned) ceil_div(B.P, kT), (unsigned) ceil_div(Cout, kT));
        AIMET_REQUIRE(grid.y <= 65535, "too many output channels");
        pw_cm_forward_kernel<<<grid, 256, 0, as_stream(stream)>>>(B, target_cache, w, bias, grad_q, it_next, scale, act);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_pw_cm_wgrad_slices(int64_t nb, int64_t Cin, int64_t Cout, int64_t hw, int64_t* slices)
{
    return guarded([&] {
        AIMET_REQUIRE(slices != nullptr, "slices is null");
        AIMET_REQUIRE(nb > 0 && Cin > 0 && Cout > 0 && hw > 0, "invalid shape");
        // enough slices for ~2 workgroups per CU, each at least 8 K chunks of positions deep
        const int64_t tiles = ceil_div(Cin, kT) * ceil_div(Cout, kT), P = nb * hw;
        int64_t s = ceil_div(512, tiles);
        const int64_t smax = std::max<int64_t>(1, P / (8 * kKc));
        *slices = std::min<int64_t>(std::min<int64_t>(s, smax), 64);
    });
}

int aimet_adaround_pw_cm_wgrad(const float* x_cache, const int64_t* idx_all, const int64_t* it_cur,
                               const float* grad_q, float* parts, int64_t slices, int64_t nb, int64_t Cin, int64_t Cout,
                               int64_t hw, void* stream)
{
    return guarded([&] {
        const CmBatch B = cm_batch(x_cache, idx_all, it_cur, nb, Cin, Cout, hw);
        require_device_ptr(grad_q, "grad_q");
        require_device_ptr(parts, "parts");
        AIMET_REQUIRE(slices >= 1 && slices <= 65535, "slices out of range");
        // slice boundaries on K-chunk multiples: every slice but the last holds whole chunks
        const int64_t per = ceil_div(ceil_div((int64_t) B.P, slices), (int64_t) kKc) * kKc;
        AIMET_REQUIRE(ceil_div((int64_t) B.P, per) <= slices, "slices");
        const dim3 grid((unsigned) ceil_div(Cin, kT), (unsigned) ceil_div(Cout, kT), (unsigned) slices);
        AIMET_REQUIRE(grid.y <= 65535, "too many output channels");
        pw_cm_wgrad_kernel<<<grid, 256, 0, as_stream(stream)>>>(B, grad_q, parts, (uint32_t) per);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
