// pw_cm_mfma.hip (study; was aimet_amd/csrc/pwcm.hip until round 5) -- NOT part of libaimet_amd.so:
// measured slower than the library-GEMM channel-major form it was meant to replace
// (profiles/r04/pw_cm_mfma_vs_library_v4.jsonl), so it was moved out of the product (VERDICT r04
// weak item 6). It builds against aimet_amd/csrc's headers (-I aimet_amd/csrc) if needed again.
//
// The AdaRound loop's iteration for 1x1 layers with many channels at small spatial
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
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kKc = 32;   // K per chunk: 16 steps of the 32 x 32 x 2 f32 MFMA

struct CmBatch
{
    const float* x;          // [rows][Cin][hw]
    const int64_t* idx_all;  // [iterations][nb]
    const int64_t* it_cur;
    uint32_t nb, Cin, Cout, hw, P;   // P = nb * hw
    FastDiv div_hw;
};

// The operands go from memory straight into the MFMA's register layout (no LDS staging): lane
// (i, h) = (lane & 31, lane >> 5) supplies A[i][k] and B[k][i] of step st at
// k = kk(st, h), so every lane loads only its own values. Both operands use the same k map, so
// each step still adds the products of one k pair; the order over a chunk is fixed
// (deterministic).
//   forward (K = input channels):  kk = 4 (st / 2) + 2 h + st % 2 -- W[co][k0 + kk] as float2 pairs
//   wgrad   (K = positions):       kk = 8 (st / 4) + 4 h + st % 4 -- 4 consecutive positions per load
//                                  (hw % 4 == 0), else kk = 16 h + st (the sample followed incrementally)

// forward + reconstruction gradient. One 32 x NP sub-tile (32 output channels x NP = 32 or 64
// positions) per workgroup of SK waves; wave `part` takes the K chunks part, part + SK, ... with
// the next chunk's loads in flight while its MFMAs run; the waves' accumulators are added in part
// order through LDS (deterministic). EVEN: Cin % 32 == 0 (no ragged chunk: W read as float2
// pairs, no zeroing). Wave 0 issues its outputs' targets and biases before the first chunk's loads
// (tools/studies/pw_cm_probe.hip: loading them in the epilogue doubled the kernel); NP = 32 gives
// twice the waves of NP = 64 for layers with few output tiles (one wave per SIMD left the loads'
// latency exposed).
template <int SK, bool EVEN, int NP>
__global__ __launch_bounds__(64 * SK) void pw_cm_forward_kernel(CmBatch B, const float* __restrict__ target,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ bias, float* __restrict__ g,
                                                                int64_t* __restrict__ it_next, float scale, int act)
{
    constexpr bool TWO = NP == 64;   // two accumulators (positions i and 32 + i)
    __shared__ float red[SK > 1 ? (SK - 1) * 32 * NP : 1];
    const int64_t it = B.it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        it_next[0] = it + 1;
    const int64_t* rows = B.idx_all + it * B.nb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const uint32_t co0 = blockIdx.y * 32, p0 = blockIdx.x * NP;
    // this lane's B columns (positions p0 + i and, NP = 64, p0 + 32 + i; clamped into the batch: a
    // column past P is computed from real data and never stored)
    const uint32_t pa = min(p0 + i, B.P - 1), pb = min(p0 + (TWO ? 32 : 0) + i, B.P - 1);
    const uint32_t ba = B.div_hw.div(pa), bb = B.div_hw.div(pb);
    const size_t ra = (size_t) rows[ba], rb = (size_t) rows[bb];
    const float* xa = B.x + ra * B.Cin * B.hw + (pa - ba * B.hw);
    const float* xb = B.x + rb * B.Cin * B.hw + (pb - bb * B.hw);
    const float* wr = w + (size_t) min(co0 + i, B.Cout - 1) * B.Cin;
    const uint32_t nch = (B.Cin + kKc - 1) / kKc;
    // wave 0's epilogue operands first: C/D map of the 32 x 32 f32 MFMA, element r of lane (i, h)
    // is row (r & 3) + 8 (r >> 2) + 4 h, column i
    float t0[16], t1[TWO ? 16 : 1], bs[16];
    if (wave == 0)
    {
        const float* ta = target + ra * B.Cout * B.hw + (pa - ba * B.hw);
        const float* tb = target + rb * B.Cout * B.hw + (pb - bb * B.hw);
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const uint32_t co = min(co0 + (r & 3) + 8 * (r >> 2) + 4 * h, B.Cout - 1);
            t0[r]             = ta[(size_t) co * B.hw];
            if constexpr (TWO)
                t1[r] = tb[(size_t) co * B.hw];
            bs[r] = bias ? bias[co] : 0.0f;
        }
    }
    float a0[16], x0[16], y0[TWO ? 16 : 1], a1[16], x1[16], y1[TWO ? 16 : 1];
    auto load = [&](uint32_t c, float (&a)[16], float (&xv)[16], auto& yv) {
        const uint32_t k0 = c * kKc;
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
        {
            const uint32_t k = k0 + 4 * s2 + 2 * h;   // steps 2 s2 (k) and 2 s2 + 1 (k + 1)
            if constexpr (EVEN)
            {
                const float2 v = *reinterpret_cast<const float2*>(wr + k);
                a[2 * s2]      = v.x;
                a[2 * s2 + 1]  = v.y;
#pragma unroll
                for (int e = 0; e < 2; ++e)
                {
                    xv[2 * s2 + e] = xa[(size_t) (k + e) * B.hw];
                    if constexpr (TWO)
                        yv[2 * s2 + e] = xb[(size_t) (k + e) * B.hw];
                }
            }
            else
            {
#pragma unroll
                for (int e = 0; e < 2; ++e)
                {
                    const uint32_t ke = k + e, kc = min(ke, B.Cin - 1);
                    const bool in     = ke < B.Cin;
                    const float av = wr[kc], xv_ = xa[(size_t) kc * B.hw];
                    a[2 * s2 + e]  = in ? av : 0.0f;
                    xv[2 * s2 + e] = in ? xv_ : 0.0f;
                    if constexpr (TWO)
                    {
                        const float yv_ = xb[(size_t) kc * B.hw];
                        yv[2 * s2 + e]  = in ? yv_ : 0.0f;
                    }
                }
            }
        }
    };
    f32x16 acc0 = {}, acc1 = {};
    auto mfma = [&](const float (&a)[16], const float (&xv)[16], const auto& yv) {
#pragma unroll
        for (int st = 0; st < 16; ++st)
        {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], xv[st], acc0, 0, 0, 0);
            if constexpr (TWO)
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], yv[st], acc1, 0, 0, 0);
        }
    };
    uint32_t c = wave;
    if (c < nch)
        load(c, a0, x0, y0);
    for (; c < nch; c += 2 * SK)
    {
        if (c + SK < nch)
            load(c + SK, a1, x1, y1);
        mfma(a0, x0, y0);
        if (c + SK >= nch)
            break;
        if (c + 2 * SK < nch)
            load(c + 2 * SK, a0, x0, y0);
        mfma(a1, x1, y1);
    }
    if constexpr (SK > 1)
    {
        if (wave != 0)
        {
            float* rd = red + (wave - 1) * 32 * NP;
#pragma unroll
            for (int r = 0; r < 16; ++r)
            {
                rd[r * 64 + lane] = acc0[r];
                if constexpr (TWO)
                    rd[(16 + r) * 64 + lane] = acc1[r];
            }
        }
        __syncthreads();
        if (wave != 0)
            return;
        for (int q = 0; q < SK - 1; ++q)
        {
            const float* rd = red + q * 32 * NP;
#pragma unroll
            for (int r = 0; r < 16; ++r)
            {
                acc0[r] += rd[r * 64 + lane];
                if constexpr (TWO)
                    acc1[r] += rd[(16 + r) * 64 + lane];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r)
    {
        const uint32_t co = co0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= B.Cout)
            continue;
        if (p0 + i < B.P)
            g[(size_t) co * B.P + p0 + i] = recon_g(acc0[r] + bs[r], t0[r], scale, act);
        if constexpr (TWO)
            if (p0 + 32 + i < B.P)
                g[(size_t) co * B.P + p0 + 32 + i] = recon_g(acc1[r] + bs[r], t1[r], scale, act);
    }
}

constexpr int kMaxRowsLds = 256;   // the batch's row table in LDS (wgrad) up to this nb

// weight-gradient slice s (blockIdx.z): one wave per 32 output channels (blockIdx.y) x 64 input
// channels (blockIdx.x) over positions [s per_slice, (s + 1) per_slice), 32-position chunks with
// the next chunk's loads in flight. V4: hw % 4 == 0 (4 consecutive positions are one sample's, so
// x comes as float4; per_slice and the chunks are multiples of 8, so the groups stay aligned).
template <bool V4>
__global__ __launch_bounds__(64) void pw_cm_wgrad_kernel(CmBatch B, const float* __restrict__ g,
                                                         float* __restrict__ part_out, uint32_t per_slice)
{
    __shared__ int64_t srows[kMaxRowsLds];
    const int64_t it    = B.it_cur[0];
    const int64_t* rows = B.idx_all + it * B.nb;
    const bool lds_rows = B.nb <= kMaxRowsLds;
    if (lds_rows)
        for (uint32_t b = threadIdx.x; b < B.nb; b += 64)
            srows[b] = rows[b];
    __syncthreads();
    const int lane = threadIdx.x, i = lane & 31, h = lane >> 5;
    const uint32_t ci0 = blockIdx.x * 64, co0 = blockIdx.y * 32;
    const uint32_t ps = blockIdx.z * per_slice, pe = min(ps + per_slice, B.P);
    const float* gr   = g + (size_t) min(co0 + i, B.Cout - 1) * B.P;
    const uint32_t cia = min(ci0 + i, B.Cin - 1), cib = min(ci0 + 32 + i, B.Cin - 1);
    const size_t plane = (size_t) B.Cin * B.hw;
    // x[ci][q] for a position q of the batch
    auto xrow = [&](uint32_t b) -> size_t { return (size_t) (lds_rows ? srows[b] : rows[b]) * plane; };
    float a0[16], x0[16], y0[16], a1[16], x1[16], y1[16];
    auto load = [&](uint32_t q0, float (&a)[16], float (&xv)[16], float (&yv)[16]) {
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
        {
            const uint32_t q = q0 + 8 * s4 + 4 * h;   // steps 4 s4 .. 4 s4 + 3: positions q .. q + 3
            if constexpr (V4)
            {
                const uint32_t qc = min(q, pe - 4);   // pe - ps is a multiple of 4 (P = nb hw, hw % 4 == 0)
                const uint32_t b = B.div_hw.div(qc), t = qc - b * B.hw;
                const size_t base = xrow(b) + t;
                const f4 gv = *reinterpret_cast<const f4*>(gr + qc);
                const f4 xv4 = *reinterpret_cast<const f4*>(B.x + base + (size_t) cia * B.hw);
                const f4 yv4 = *reinterpret_cast<const f4*>(B.x + base + (size_t) cib * B.hw);
                const bool in = q < pe;
                const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, xa[4] = {xv4.x, xv4.y, xv4.z, xv4.w},
                            ya[4] = {yv4.x, yv4.y, yv4.z, yv4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                {
                    a[4 * s4 + e]  = in ? ga[e] : 0.0f;
                    xv[4 * s4 + e] = in ? xa[e] : 0.0f;
                    yv[4 * s4 + e] = in ? ya[e] : 0.0f;
                }
            }
        }
    };
    // hw % 4 != 0 (7 x 7 layers): lane h takes positions q0 + 16 h .. + 15 (step st: q0 + 16 h + st),
    // following the sample boundary incrementally instead of a division per position
    auto load_s = [&](uint32_t q0, float (&a)[16], float (&xv)[16], float (&yv)[16]) {
        const uint32_t qs = q0 + 16 * h, qc0 = min(qs, pe - 1);
        uint32_t b = B.div_hw.div(qc0), t = qc0 - b * B.hw;
        size_t base = xrow(b);
#pragma unroll
        for (int e = 0; e < 16; ++e)
        {
            const uint32_t q = qs + e;
            const bool in    = q < pe;
            const float gv = gr[min(q, pe - 1)], xv_ = B.x[base + (size_t) cia * B.hw + t],
                        yv_ = B.x[base + (size_t) cib * B.hw + t];
            a[e]  = in ? gv : 0.0f;
            xv[e] = in ? xv_ : 0.0f;
            yv[e] = in ? yv_ : 0.0f;
            if (++t == B.hw)
            {
                t    = 0;
                b    = min(b + 1, B.nb - 1);
                base = xrow(b);
            }
        }
    };
    f32x16 acc0 = {}, acc1 = {};
    auto mfma = [&](const float (&a)[16], const float (&xv)[16], const float (&yv)[16]) {
#pragma unroll
        for (int st = 0; st < 16; ++st)
        {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], xv[st], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[st], yv[st], acc1, 0, 0, 0);
        }
    };
    auto ld = [&](uint32_t q, float (&a)[16], float (&xv)[16], float (&yv)[16]) {
        if constexpr (V4)
            load(q, a, xv, yv);
        else
            load_s(q, a, xv, yv);
    };
    uint32_t q0 = ps;
    if (q0 < pe)
        ld(q0, a0, x0, y0);
    for (; q0 < pe; q0 += 2 * kKc)
    {
        if (q0 + kKc < pe)
            ld(q0 + kKc, a1, x1, y1);
        mfma(a0, x0, y0);
        if (q0 + kKc >= pe)
            break;
        if (q0 + 2 * kKc < pe)
            ld(q0 + 2 * kKc, a0, x0, y0);
        mfma(a1, x1, y1);
    }
    // part[s][co][ci]: element r of lane (i, h) is output channel co0 + (r & 3) + 8 (r >> 2) + 4 h,
    // input channel ci0 + i (acc0) / ci0 + 32 + i (acc1)
    float* out = part_out + (size_t) blockIdx.z * B.Cout * B.Cin;
#pragma unroll
    for (int r = 0; r < 16; ++r)
    {
        const uint32_t co = co0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= B.Cout)
            continue;
        if (ci0 + i < B.Cin)
            out[(size_t) co * B.Cin + ci0 + i] = acc0[r];
        if (ci0 + 32 + i < B.Cin)
            out[(size_t) co * B.Cin + ci0 + 32 + i] = acc1[r];
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
        const bool even   = Cin % kKc == 0 && (reinterpret_cast<uintptr_t>(w) & 7) == 0;
        // positions per wave and waves per sub-tile: enough waves to give every SIMD one (the sums
        // are latency-bound at one wave per SIMD) -- 32-position tiles first, then the K chunks split
        // over up to 4 waves
        const int64_t ctiles = ceil_div(Cout, (int64_t) 32);
        const int np         = ceil_div((int64_t) B.P, (int64_t) 64) * ctiles >= 1024 ? 64 : 32;
        const int64_t tiles  = ceil_div((int64_t) B.P, (int64_t) np) * ctiles;
        const int64_t nch    = ceil_div(Cin, (int64_t) kKc);
        int sk               = 1;
        while (sk < 4 && tiles * sk < 1024 && 2 * sk <= nch)   // 8 waves of ~200 VGPRs would spill
            sk *= 2;
        const dim3 grid((unsigned) ceil_div((int64_t) B.P, (int64_t) np), (unsigned) ctiles);
        AIMET_REQUIRE(grid.y <= 65535, "too many output channels");
        hipStream_t st = as_stream(stream);
        auto go = [&](auto skc, auto evc, auto npc) {
            constexpr int SK    = decltype(skc)::value;
            constexpr bool EVEN = decltype(evc)::value;
            constexpr int NP    = decltype(npc)::value;
            pw_cm_forward_kernel<SK, EVEN, NP><<<grid, 64 * SK, 0, st>>>(B, target_cache, w, bias, grad_q, it_next,
                                                                          scale, act);
        };
        auto with_np = [&](auto skc, auto evc) {
            if (np == 64)
                go(skc, evc, std::integral_constant<int, 64> {});
            else
                go(skc, evc, std::integral_constant<int, 32> {});
        };
        auto with_even = [&](auto skc) {
            if (even)
                with_np(skc, std::true_type {});
            else
                with_np(skc, std::false_type {});
        };
        if (sk == 4)
            with_even(std::integral_constant<int, 4> {});
        else if (sk == 2)
            with_even(std::integral_constant<int, 2> {});
        else
            with_even(std::integral_constant<int, 1> {});
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_pw_cm_wgrad_slices(int64_t nb, int64_t Cin, int64_t Cout, int64_t hw, int64_t* slices)
{
    return guarded([&] {
        AIMET_REQUIRE(slices != nullptr, "slices is null");
        AIMET_REQUIRE(nb > 0 && Cin > 0 && Cout > 0 && hw > 0, "invalid shape");
        // one wave per (32 x 64 tile, slice): about one wave per SIMD (1024), each slice at least
        // two 32-position chunks deep; at most 64 slices (the Adam step adds them per element)
        const int64_t tiles = ceil_div(Cin, (int64_t) 64) * ceil_div(Cout, (int64_t) 32), P = nb * hw;
        const int64_t s     = ceil_div((int64_t) 1024, tiles);
        const int64_t smax  = std::max<int64_t>(1, P / (2 * kKc));
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
        // slice boundaries on multiples of 8 positions (the float4 groups stay inside one sample
        // and aligned when hw % 4 == 0)
        const int64_t per = ceil_div(ceil_div((int64_t) B.P, slices), (int64_t) 8) * 8;
        const dim3 grid((unsigned) ceil_div(Cin, (int64_t) 64), (unsigned) ceil_div(Cout, (int64_t) 32),
                        (unsigned) slices);
        AIMET_REQUIRE(grid.y <= 65535, "too many output channels");
        const bool v4 = hw % 4 == 0 && (reinterpret_cast<uintptr_t>(x_cache) & 15) == 0 &&
                        (reinterpret_cast<uintptr_t>(grad_q) & 15) == 0;
        if (v4)
            pw_cm_wgrad_kernel<true><<<grid, 64, 0, as_stream(stream)>>>(B, grad_q, parts, (uint32_t) per);
        else
            pw_cm_wgrad_kernel<false><<<grid, 64, 0, as_stream(stream)>>>(B, grad_q, parts, (uint32_t) per);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
