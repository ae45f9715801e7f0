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
//    idx_all[it][b] of the input cache (no channel-major copy), the target read in place; each wave
//    owns a 32 x 64 sub-tile (two v_mfma_f32_32x32x2_f32 accumulators: the f32 matrix instruction,
//    exact fmaf chains), stages 16-deep K chunks in its own LDS slot with the next chunk's loads in
//    flight, and deep sums are split over up to 4 waves whose accumulators are added in a fixed
//    order (deterministic);
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

constexpr int kKc  = 16;          // K chunk per wave step
constexpr int kLdA = kKc + 1;     // [32][17]: the lanes reading one k column hit distinct banks
constexpr int kLdB = 64 + 4;      // [16][68]
constexpr int kStage = 32 * kLdA + kKc * kLdB;   // one wave's staging floats

struct CmBatch
{
    const float* x;          // [rows][Cin][hw]
    const int64_t* idx_all;  // [iterations][nb]
    const int64_t* it_cur;
    uint32_t nb, Cin, Cout, hw, P;   // P = nb * hw
    FastDiv div_hw;
};

// the LDS writes of this wave visible to its own lanes (wave-local staging, in-order LDS)
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// acc0 / acc1 += A[32 x kKc] . B[kKc x 64] (columns 0-31 / 32-63): kKc / 2 steps of the 32 x 32 x 2
// f32 MFMA, the two accumulators' chains interleaved
__device__ __forceinline__ void mfma_chunk(const float* As, const float* Bs, f32x16& acc0, f32x16& acc1)
{
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
#pragma unroll
    for (int st = 0; st < kKc / 2; ++st)
    {
        const float a = As[i * kLdA + 2 * st + h];
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bs[(2 * st + h) * kLdB + i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bs[(2 * st + h) * kLdB + 32 + i], acc1, 0, 0, 0);
    }
}

// SK > 1 waves computed the same 32 x 64 sub-tile over interleaved K chunks: wave `part` 0 adds the
// others' accumulators in part order (deterministic). Every thread of the workgroup calls it.
template <int SK>
__device__ __forceinline__ void reduce_parts(f32x16& acc0, f32x16& acc1, float* red)
{
    if constexpr (SK > 1)
    {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, part = wave % SK;
        if (part != 0)
        {
#pragma unroll
            for (int r = 0; r < 16; ++r)
            {
                red[(wave * 32 + r) * 64 + lane]      = acc0[r];
                red[(wave * 32 + 16 + r) * 64 + lane] = acc1[r];
            }
        }
        __syncthreads();
        if (part == 0)
            for (int q = 1; q < SK; ++q)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                {
                    acc0[r] += red[((wave + q) * 32 + r) * 64 + lane];
                    acc1[r] += red[((wave + q) * 32 + 16 + r) * 64 + lane];
                }
    }
}

// forward + reconstruction gradient. A workgroup's 4 waves cover 4 / SK sub-tiles of 32 output
// channels x 64 positions (blockIdx.y: channel block, blockIdx.x: 64 positions); the SK waves of a
// sub-tile take the Cin chunks part, part + SK, ... (each with the next chunk's loads in flight
// while its MFMAs run), and their accumulators are added in part order.
template <int SK>
__global__ __launch_bounds__(256) void pw_cm_forward_kernel(CmBatch B, const float* __restrict__ target,
                                                            const float* __restrict__ w, const float* __restrict__ bias,
                                                            float* __restrict__ g, int64_t* __restrict__ it_next,
                                                            float scale, int act)
{
    constexpr int SUB = 4 / SK;
    __shared__ float stage[4][kStage];
    __shared__ float red[SK > 1 ? 4 * 32 * 64 : 1];
    const int64_t it = B.it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        it_next[0] = it + 1;
    const int64_t* rows = B.idx_all + it * B.nb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, part = wave % SK;
    const uint32_t co0 = blockIdx.y * (32 * SUB) + (wave / SK) * 32, p0 = blockIdx.x * 64;
    // B loads: lane = position p0 + lane, k = 0 .. kKc - 1 (consecutive positions across lanes)
    const uint32_t pl = p0 + lane;
    const bool pv     = pl < B.P;
    size_t xbase      = 0;
    if (pv)
    {
        const uint32_t b = B.div_hw.div(pl);
        xbase            = (size_t) rows[b] * B.Cin * B.hw + (pl - b * B.hw);
    }
    // A loads: k = lane & 15, rows (lane >> 4) + 4 j
    const int ak = lane & 15, ar = lane >> 4;
    float* As = stage[wave];
    float* Bs = As + 32 * kLdA;
    const uint32_t nch = (B.Cin + kKc - 1) / kKc;
    float ra[8], rb[kKc];
    auto load = [&](uint32_t c) {
        const uint32_t k0 = c * kKc;
#pragma unroll
        for (int j = 0; j < 8; ++j)
        {
            const uint32_t co = co0 + ar + 4 * j, ci = k0 + ak;
            ra[j] = (co < B.Cout && ci < B.Cin) ? w[(size_t) co * B.Cin + ci] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < kKc; ++k)
            rb[k] = (pv && k0 + k < B.Cin) ? B.x[xbase + (size_t) (k0 + k) * B.hw] : 0.0f;
    };
    f32x16 acc0 = {}, acc1 = {};
    uint32_t c = part;
    if (c < nch)
        load(c);
    for (; c < nch; c += SK)
    {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            As[(ar + 4 * j) * kLdA + ak] = ra[j];
#pragma unroll
        for (int k = 0; k < kKc; ++k)
            Bs[k * kLdB + lane] = rb[k];
        wave_sync();
        if (c + SK < nch)
            load(c + SK);
        mfma_chunk(As, Bs, acc0, acc1);
        wave_sync();
    }
    reduce_parts<SK>(acc0, acc1, red);
    if (part != 0)
        return;
    // C/D map of the 32 x 32 f32 MFMA: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int h = 0; h < 2; ++h)
    {
        const uint32_t p = p0 + 32 * h + (lane & 31);
        if (p >= B.P)
            continue;
        const uint32_t b = B.div_hw.div(p), t = p - b * B.hw;
        const float* trow = target + (size_t) rows[b] * B.Cout * B.hw + t;
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const uint32_t co = co0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const float q     = h ? acc1[r] : acc0[r];
            if (co < B.Cout)
                g[(size_t) co * B.P + p] = recon_g(q + (bias ? bias[co] : 0.0f), trow[(size_t) co * B.hw], scale, act);
        }
    }
}

// weight-gradient slice s (blockIdx.z): sub-tile 32 output channels (blockIdx.y) x 64 input channels
// (blockIdx.x); the 4 waves take the slice's 16-position chunks part, part + 4, ... and are added in
// part order
__global__ __launch_bounds__(256) void pw_cm_wgrad_kernel(CmBatch B, const float* __restrict__ g,
                                                          float* __restrict__ part_out, uint32_t per_slice)
{
    constexpr int SK = 4;
    __shared__ float stage[4][kStage];
    __shared__ float red[4 * 32 * 64];
    const int64_t it    = B.it_cur[0];
    const int64_t* rows = B.idx_all + it * B.nb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, part = wave;
    const uint32_t ci0 = blockIdx.x * 64, co0 = blockIdx.y * 32;
    const uint32_t ps = blockIdx.z * per_slice, pe = ps + per_slice < B.P ? ps + per_slice : B.P;
    const int kk = lane & 15, sub = lane >> 4;   // position in the chunk, row / column group
    float* As = stage[wave];
    float* Bs = As + 32 * kLdA;
    float ra[8], rb[16];
    auto load = [&](uint32_t k0) {
        const uint32_t p = k0 + kk;
        const bool in    = p < pe;
        size_t xb        = 0;
        if (in)
        {
            const uint32_t b = B.div_hw.div(p);
            xb               = (size_t) rows[b] * B.Cin * B.hw + (p - b * B.hw);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)   // A: g[co][p], 4 rows x 16 consecutive positions per load
        {
            const uint32_t co = co0 + sub + 4 * j;
            ra[j] = (in && co < B.Cout) ? g[(size_t) co * B.P + p] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)   // B: x[ci][p], 4 input channels x 16 consecutive positions per load
        {
            const uint32_t ci = ci0 + sub + 4 * j;
            rb[j] = (in && ci < B.Cin) ? B.x[xb + (size_t) ci * B.hw] : 0.0f;
        }
    };
    f32x16 acc0 = {}, acc1 = {};
    uint32_t k0 = ps + part * kKc;
    if (k0 < pe)
        load(k0);
    for (; k0 < pe; k0 += SK * kKc)
    {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            As[(sub + 4 * j) * kLdA + kk] = ra[j];
#pragma unroll
        for (int j = 0; j < 16; ++j)
            Bs[kk * kLdB + sub + 4 * j] = rb[j];
        wave_sync();
        if (k0 + SK * kKc < pe)
            load(k0 + SK * kKc);
        mfma_chunk(As, Bs, acc0, acc1);
        wave_sync();
    }
    reduce_parts<SK>(acc0, acc1, red);
    if (part != 0)
        return;
    float* out = part_out + (size_t) blockIdx.z * B.Cout * B.Cin;
#pragma unroll
    for (int h = 0; h < 2; ++h)
    {
        const uint32_t ci = ci0 + 32 * h + (lane & 31);
        if (ci >= B.Cin)
            continue;
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const uint32_t co = co0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (co < B.Cout)
                out[(size_t) co * B.Cin + ci] = h ? acc1[r] : acc0[r];
        }
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
        // waves per sub-tile by the depth of the sum: deep Cin splits over the workgroup's waves
        const int sk      = Cin >= 256 ? 4 : (Cin >= 96 ? 2 : 1);
        const int64_t sub = 32 * (4 / sk);
        const dim3 grid((unsigned) ceil_div((int64_t) B.P, (int64_t) 64), (unsigned) ceil_div(Cout, sub));
        AIMET_REQUIRE(grid.y <= 65535, "too many output channels");
        hipStream_t st = as_stream(stream);
        if (sk == 4)
            pw_cm_forward_kernel<4><<<grid, 256, 0, st>>>(B, target_cache, w, bias, grad_q, it_next, scale, act);
        else if (sk == 2)
            pw_cm_forward_kernel<2><<<grid, 256, 0, st>>>(B, target_cache, w, bias, grad_q, it_next, scale, act);
        else
            pw_cm_forward_kernel<1><<<grid, 256, 0, st>>>(B, target_cache, w, bias, grad_q, it_next, scale, act);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_pw_cm_wgrad_slices(int64_t nb, int64_t Cin, int64_t Cout, int64_t hw, int64_t* slices)
{
    return guarded([&] {
        AIMET_REQUIRE(slices != nullptr, "slices is null");
        AIMET_REQUIRE(nb > 0 && Cin > 0 && Cout > 0 && hw > 0, "invalid shape");
        // enough slices for ~2 workgroups per CU, each at least 2 chunks deep per wave
        const int64_t tiles = ceil_div(Cin, (int64_t) 64) * ceil_div(Cout, (int64_t) 32), P = nb * hw;
        const int64_t s     = ceil_div((int64_t) 512, tiles);
        const int64_t smax  = std::max<int64_t>(1, P / (8 * kKc));
        *slices             = std::min<int64_t>(std::min<int64_t>(s, smax), 64);
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
        const dim3 grid((unsigned) ceil_div(Cin, (int64_t) 64), (unsigned) ceil_div(Cout, (int64_t) 32),
                        (unsigned) slices);
        AIMET_REQUIRE(grid.y <= 65535, "too many output channels");
        pw_cm_wgrad_kernel<<<grid, 256, 0, as_stream(stream)>>>(B, grad_q, parts, (uint32_t) per);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
