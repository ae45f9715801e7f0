// stats.hip -- encoding-statistics kernels (TF min/max; TF-E / percentile / MSE histograms).
//
// Reference: math_functions.cu:52-64 (two thrust reductions, each ending in a blocking D2H),
// :125-211 (a private 512-bin histogram per THREAD in a <=32 MiB global scratch, reduced by ONE
// 512-thread block, then a blocking cudaMemcpy), math_functions.cpp:207-288 (range init and PDF
// averaging on the host). Per-channel statistics were gathered by a Python loop over channels
// (v1/tensor_quantizer.py:567-570), one select().contiguous() copy + one analyzer per channel.
//
// MI355X design:
//   * min/max: one fused pass, 16-B loads, wave64 shuffle + LDS block reduction, per-block
//     partials combined by one small block (no atomics: deterministic).
//   * histogram: LDS-privatised 512-bin histograms (one per wave, ds_add_u32), a register counter
//     for exact zeros (ReLU outputs put ~half of all elements into one bin), then one 64-bit
//     global atomic per non-empty bin per workgroup.
//   * range init and the double-precision PDF running average run on the device, so an
//     updateStats call is 2-4 stream-ordered launches with no host synchronisation.
//   * per-channel: all channels in one launch, one workgroup per channel.
// Arithmetic follows the reference CPU code bit for bit (DTYPE = float; see common.hpp).
#include "entropy_core.hpp"
#include "tq_state.hpp"

#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <vector>

namespace aimet_amd
{

namespace
{

constexpr int kWaves      = kBlock / 64;
constexpr int kHistUnroll = 4;
constexpr int kHistGrid   = 2048;   // 8 workgroups per CU: enough 16-B loads in flight for HBM
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_min(float v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_max(float v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide min/max; result valid in thread 0. NaNs never enter (fminf/fmaxf drop them),
// matching GetMin_cpu/GetMax_cpu (std::min/std::max skip NaN, math_functions.cpp:327-347).
// The sign of a zero extremum is immaterial downstream (TfEncodingAnalyzer.cpp:87-88 and
// InitializePdf produce identical results for +0 and -0).
__device__ __forceinline__ void block_minmax(float& mn, float& mx)
{
    __shared__ float smn[kWaves], smx[kWaves];
    mn       = wave_min(mn);
    mx       = wave_max(mx);
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0)
    {
        smn[w] = mn;
        smx[w] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
#pragma unroll
        for (int i = 1; i < kWaves; ++i)
        {
            mn = fminf(mn, smn[i]);
            mx = fmaxf(mx, smx[i]);
        }
    }
}

__device__ __forceinline__ void accum4(const float4& v, float& mn, float& mx)
{
    mn = fminf(fminf(mn, v.x), fminf(v.y, fminf(v.z, v.w)));
    mx = fmaxf(fmaxf(mx, v.x), fmaxf(v.y, fmaxf(v.z, v.w)));
}

// ---- per-tensor min/max: partials[block] = {-min, max} --------------------------------------
// One workgroup's share (block `blk` of `nblk`) of the min/max pass over x[0, n).
__device__ __forceinline__ void minmax_part(const float* __restrict__ x, int64_t n, int vec, int64_t blk,
                                            int64_t nblk, float2* __restrict__ partials)
{
    float mn = INFINITY, mx = -INFINITY;
    if (vec)
    {
        // streaming 16-B loads, 4 in flight per lane (tools/studies/hist_variants.hip: 6.8 TB/s)
        const f4* x4         = reinterpret_cast<const f4*>(x);
        int64_t nvec         = n / 4;
        const int64_t stride = nblk * kBlock * 4;
        for (int64_t b = blk * kBlock * 4 + threadIdx.x; b < nvec; b += stride)
        {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)   // NaN padding is ignored by fminf/fmaxf
                v[u] = b + u * kBlock < nvec ? __builtin_nontemporal_load(x4 + b + u * kBlock)
                                             : f4 {NAN, NAN, NAN, NAN};
#pragma unroll
            for (int u = 0; u < 4; ++u)
                accum4(make_float4(v[u].x, v[u].y, v[u].z, v[u].w), mn, mx);
        }
        for (int64_t i = nvec * 4 + blk * kBlock + threadIdx.x; i < n; i += nblk * kBlock)
        {
            mn = fminf(mn, x[i]);
            mx = fmaxf(mx, x[i]);
        }
    }
    else
    {
        for (int64_t i = blk * kBlock + threadIdx.x; i < n; i += nblk * kBlock)
        {
            mn = fminf(mn, x[i]);
            mx = fmaxf(mx, x[i]);
        }
    }
    block_minmax(mn, mx);
    if (threadIdx.x == 0)
        partials[blk] = make_float2(-mn, mx);
}

__global__ __launch_bounds__(kBlock) void minmax_tensor_kernel(const float* __restrict__ x, int64_t n, int vec,
                                                               float2* __restrict__ partials,
                                                               const int32_t* __restrict__ pdf_init, int skip_if_init)
{
    if (skip_if_init && pdf_init[0])
        return;
    minmax_part(x, n, vec, blockIdx.x, gridDim.x, partials);
}

// Combine per-block partials {-min, max} into minmax[0].
__global__ __launch_bounds__(kBlock) void minmax_combine_max_kernel(const float2* __restrict__ partials, int nparts,
                                                                    float2* __restrict__ minmax,
                                                                    const int32_t* __restrict__ pdf_init,
                                                                    int skip_if_init)
{
    if (skip_if_init && pdf_init[0])
        return;
    float a = -INFINITY, b = -INFINITY;
    for (int i = threadIdx.x; i < nparts; i += kBlock)
    {
        a = fmaxf(a, partials[i].x);
        b = fmaxf(b, partials[i].y);
    }
    float na = -a;            // min over -(partials.x) == global min
    block_minmax(na, b);      // na: block min of mins, b: block max of maxes
    if (threadIdx.x == 0)
        minmax[0] = make_float2(-na, b);
}

// ---- per-channel min/max: one workgroup per channel of [outer][C][K] -----------------------
__global__ __launch_bounds__(kBlock) void minmax_channel_kernel(const float* __restrict__ x, int64_t outer, int64_t C,
                                                                int64_t K, int vec, float2* __restrict__ minmax,
                                                                const int32_t* __restrict__ pdf_init,
                                                                int skip_if_init)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        if (skip_if_init && pdf_init[c])
            continue;
        float mn = INFINITY, mx = -INFINITY;
        for (int64_t o = 0; o < outer; ++o)
        {
            const float* row = x + (o * C + c) * K;
            if (vec)
            {
                const float4* r4 = reinterpret_cast<const float4*>(row);
                for (int64_t k = threadIdx.x; k < K / 4; k += kBlock)
                    accum4(r4[k], mn, mx);
            }
            else
            {
                for (int64_t k = threadIdx.x; k < K; k += kBlock)
                {
                    mn = fminf(mn, row[k]);
                    mx = fmaxf(mx, row[k]);
                }
            }
        }
        block_minmax(mn, mx);
        if (threadIdx.x == 0)
            minmax[c] = make_float2(-mn, mx);
        __syncthreads();
    }
}

// ---- fold: TF running min/max, or PDF range initialisation --------------------------------
// InitializePdf<float>(pdf, min, max, signed=true), math_functions.cpp:207-241.
__device__ void initialize_pdf(const TqDevice& d, int64_t c, float min_val, float max_val)
{
    if (min_val == max_val)
        max_val = (max_val < min_val + 0.01f) ? min_val + 0.01f : max_val;
    float center = (max_val + min_val) / 2.0f;
    float lo     = center - 3.0f * (center - min_val);
    float hi     = center + 3.0f * (max_val - center);
    min_val      = (-FLT_MAX < lo) ? lo : -FLT_MAX;   // std::max(lowest, lo)
    max_val      = (hi < FLT_MAX) ? hi : FLT_MAX;     // std::min(max, hi)
    double bs    = ((double) max_val - (double) min_val) / kPdfSize;
    double x0    = (double) min_val + (double) 0 * bs;
    double x1    = (double) min_val + (double) 1 * bs;
    float bucket = (float) (x1 - x0);                 // UpdatePdf:264
    float mv     = (float) x0;                        // UpdatePdf:265 (signed)
    d.hist_min[c]    = min_val;
    d.bucket_size[c] = bs;
    d.bin_bucket[c]  = bucket;
    d.bin_offset[c]  = mv / bucket;                   // UpdatePdf:267
    d.iterations[c]  = 0;                             // pdf[] is zero since the last reset
    d.pdf_init[c]    = 1;
}

// TfEncodingAnalyzer.cpp:63-71 (TF: running min/max in double) or UpdatePdf's first-batch range
// initialisation (histogram schemes), for channel c from minmax[c] = {-min, max}
__device__ __forceinline__ void fold_one(const TqDevice& d, int64_t c, bool tf_scheme)
{
    float2 m = reinterpret_cast<const float2*>(d.minmax)[c];
    float mn = -m.x, mx = m.y;
    if (tf_scheme)
    {
        // std::min/std::max in double
        double cmin = (double) mn, cmax = (double) mx;
        double2* acc = reinterpret_cast<double2*>(d.acc);
        double2 a    = acc[c];
        a.x          = (cmin < a.x) ? cmin : a.x;
        a.y          = (a.y < cmax) ? cmax : a.y;
        acc[c]       = a;
    }
    else if (!d.pdf_init[c])
    {
        // UpdatePdf:254-259: an all-zero tensor does not initialise the PDF (batch ignored)
        if (mn == 0 && mx == 0)
            return;
        initialize_pdf(d, c, mn, mx);
    }
}

__global__ __launch_bounds__(kBlock) void fold_minmax_kernel(TqDevice d, int64_t C, int tf_scheme)
{
    int64_t c = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (c < C)
        fold_one(d, c, tf_scheme != 0);
}

// ---- entropy analyzer: TensorProfilingParams (math_functions.cpp:476-560) ---------------------
// Per batch, for channel c and the (exchanged) batch min/max: an all-zero batch is skipped
// (:482-487), the first batch fixes the range (:496-501), a batch outside the range widens it and
// redistributes the 512 bins (:503-550), and the batch is binned with the float (binWidth, min)
// of :552-558. Bin counts are integers (doubles < 2^53 in the reference), so the redistribution is
// accumulated in 64-bit integers: exact and independent of the order of the adds. Any blockDim;
// mnf / mxf must be uniform over the block.
__device__ void ent_fold_one(const TqDevice& d, int64_t c, float mnf, float mxf)
{
    using entropy::get_bin;
    using entropy::x86_d2u64;
    __shared__ unsigned long long scaled[kPdfSize];
    double minInput = mnf, maxInput = mxf;
    if (minInput == 0 && maxInput == 0)
    {
        if (threadIdx.x == 0)
            d.active[c] = 0;
        return;
    }
    if (minInput == maxInput)
    {
        double t = minInput + (double) 0.01f;   // minInput + (DTYPE) 0.01
        maxInput = (maxInput < t) ? t : maxInput;
    }
    double2* acc = reinterpret_cast<double2*>(d.acc);
    double2 a    = acc[c];
    if (!d.pdf_init[c])
    {
        a.x = minInput;
        a.y = maxInput;
    }
    if (minInput < a.x || maxInput > a.y)
    {
        const double newMin = (a.x < minInput) ? a.x : minInput;    // std::min(minInput, tpp.min)
        const double newMax = (maxInput < a.y) ? a.y : maxInput;    // std::max(maxInput, tpp.max)
        const double dstW   = (newMax - newMin) / kPdfSize;
        const double srcW   = (a.y - a.x) / kPdfSize;
        const float dstWf = (float) dstW, newMinf = (float) newMin;
        for (int i = threadIdx.x; i < kPdfSize; i += blockDim.x)
            scaled[i] = 0;
        __syncthreads();
        double* hist = d.pdf + c * kPdfSize;
        for (int i = threadIdx.x; i < kPdfSize; i += blockDim.x)
        {
            const double h = hist[i];
            if (h == 0)
                continue;
            const double begin  = a.x + srcW * (double) i;
            const uint64_t dbin = x86_d2u64((begin - newMin) / dstW);
            const double dend   = newMin + dstW * (double) (dbin + 1);
            double cnt          = __builtin_round((dend - begin) / srcW * h);
            cnt                 = (h < cnt) ? h : cnt;
            if (!(__builtin_fabs(cnt) < 9.0e15))   // non-finite ranges (inf inputs): see DESIGN.md
                cnt = h;
            atomicAdd(&scaled[get_bin(dstWf, newMinf, (float) begin)], (unsigned long long) (long long) cnt);
            if (cnt < h)
                atomicAdd(&scaled[get_bin(dstWf, newMinf, (float) (begin + dstW))],
                          (unsigned long long) (long long) (h - cnt));
        }
        __syncthreads();
        for (int i = threadIdx.x; i < kPdfSize; i += blockDim.x)
            hist[i] = (double) (long long) scaled[i];
        a.x = newMin;
        a.y = newMax;
    }
    __syncthreads();   // every lane has read acc / pdf_init
    if (threadIdx.x == 0)
    {
        acc[c]          = a;
        d.pdf_init[c]   = 1;
        d.bin_bucket[c] = (float) ((a.y - a.x) / kPdfSize);   // float binWidth
        d.bin_offset[c] = (float) a.x;                        // getBin's float minValue
        d.active[c]     = 1;
    }
}

__global__ __launch_bounds__(kBlock) void ent_fold_minmax_kernel(TqDevice d, int64_t C)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        float2 m = reinterpret_cast<const float2*>(d.minmax)[c];
        ent_fold_one(d, c, -m.x, m.y);
        __syncthreads();
    }
}

// histogram += this batch's counts; iterations++ (math_functions.cpp:554-559). Any blockDim.
__device__ __forceinline__ void ent_fold_hist_one(const TqDevice& d, int64_t c)
{
    for (int i = threadIdx.x; i < kPdfSize; i += blockDim.x)
    {
        int64_t idx   = c * kPdfSize + i;
        d.pdf[idx]    = d.pdf[idx] + (double) d.counts[idx];
        d.counts[idx] = 0;
    }
    if (threadIdx.x == 0)
        d.iterations[c] += 1;
}

// ---- histogram ----------------------------------------------------------------------------
// GetHistogram_cpu, math_functions.cpp:367-384: index = round(x / bucket - offset) in float,
// out-of-range (and NaN) dropped.
struct PdfBinner
{
    float bucket, offset, rcp, thr;
    // thr: round_div_sub's threshold 2^-21 (|q| + |off| + 1) bounded once for every element whose
    // bin can be in range (|v| <= 512, so |q| <= 512 + |off| + 1): hoisted out of the element loop.
    // An element beyond that bound lies out of range whichever way it rounds, and a zero code's
    // sign does not matter for a bin index, so the fast path needs no other test.
    __device__ PdfBinner(float b, float o)
        : bucket(b), offset(o), rcp(1.0f / b),
          thr((2.0f * __builtin_fabsf(o) + 514.0f) * 4.76837158203125e-7f)
    {
    }
    __device__ __forceinline__ int bin(float x) const
    {
        // == roundf(x / bucket - offset) bit for bit (round_div_sub, common.hpp), in range
        const float v = x * rcp - offset;
        float r;
        if (__builtin_fabsf(__builtin_amdgcn_fractf(v) - 0.5f) > thr)   // false for NaN
            r = __builtin_rintf(v);
        else
            r = __builtin_roundf(x / bucket - offset);
        return (r >= 0.0f && r < (float) kPdfSize) ? (int) r : -1;
    }
};

// The binner of channel c: the PDF's (TF-E / percentile / MSE) or the entropy analyzer's
template <bool ENT>
struct BinnerOf;
template <>
struct BinnerOf<false>
{
    typedef PdfBinner type;
    __device__ static bool live(const TqDevice& d, int64_t c) { return d.pdf_init[c] != 0; }
};
template <>
struct BinnerOf<true>
{
    typedef entropy::Binner type;
    __device__ static bool live(const TqDevice& d, int64_t c) { return d.active[c] != 0; }
};

// per-tensor: many workgroups over one tensor, atomics into counts[0][:]. One workgroup's share
// (block `blk` of `nblk`) of the pass over x[0, n).
//
// The workgroup's LDS histogram is [bin][32]: lane l adds into column l & 31, so the 32 lanes that
// a ds_add_u32 services together always address 32 different banks. With one [512] histogram per
// wave, bins of ordinary activations (a few dozen bins around the bulk) put ~4 lanes on one bank
// per group -- 73% of the kernel's LDS cycles were bank-conflict cycles on ViT-L/16's activations
// (round 3's SQ_LDS_BANK_CONFLICT pass) -- and lanes adding to one bin serialise. The columns of a bin are
// folded once, when the workgroup ends.
// COLS = 16 halves the LDS (32 KiB, more workgroups per CU): lanes l and l + 16 then share a
// column, a conflict only when their bins have the same parity.
template <int BLOCK, bool ENT, int COLS = 32>
__device__ __forceinline__ void histogram_part(const float* __restrict__ x, int64_t n, int vec, int64_t blk,
                                               int64_t nblk, const TqDevice& d)
{
    constexpr int kHistCols = COLS;
    __shared__ uint32_t lds[kPdfSize * kHistCols];   // 64 KiB (32 columns)
    typename BinnerOf<ENT>::type bn {d.bin_bucket[0], d.bin_offset[0]};
    const uint32_t col = threadIdx.x & (kHistCols - 1);
    for (int i = threadIdx.x; i < kPdfSize * kHistCols / 4; i += BLOCK)
        reinterpret_cast<uint4*>(lds)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int zbin = bn.bin(0.0f);
    uint32_t zc    = 0;
    auto add = [&](float v) {
        if (v == 0.0f)
        {
            ++zc;
            return;
        }
        int b = bn.bin(v);
        if (b >= 0)
            atomicAdd(&lds[b * kHistCols + col], 1u);
    };
    int64_t done = 0;
    if (vec)
    {
        // 4 x 16-B streaming loads in flight per lane (tools/studies/hist_variants.hip: 5.6-5.8 TB/s)
        const f4* x4         = reinterpret_cast<const f4*>(x);
        const int64_t nv     = n / 4;
        const int64_t stride = nblk * BLOCK * kHistUnroll;
        for (int64_t base = blk * BLOCK * kHistUnroll + threadIdx.x; base < nv; base += stride)
        {
            f4 v[kHistUnroll];
#pragma unroll
            for (int u = 0; u < kHistUnroll; ++u)
            {
                // padding: NaN is dropped by the PDF binner; the entropy binner counts NaN (last
                // bin, as the reference), so there the padding is zeros, taken back from the
                // register zero counter
                int64_t i = base + (int64_t) u * BLOCK;
                if (ENT && i >= nv)
                    zc -= 4;
                v[u] = i < nv ? __builtin_nontemporal_load(x4 + i)
                              : (ENT ? f4 {0.f, 0.f, 0.f, 0.f} : f4 {NAN, NAN, NAN, NAN});
            }
#pragma unroll
            for (int u = 0; u < kHistUnroll; ++u)
            {
                add(v[u].x);
                add(v[u].y);
                add(v[u].z);
                add(v[u].w);
            }
        }
        done = nv * 4;
    }
    for (int64_t i = done + blk * BLOCK + threadIdx.x; i < n; i += nblk * BLOCK)
        add(x[i]);
    zc = wave_sum(zc);
    if ((threadIdx.x & 63) == 0 && zbin >= 0 && zc)
        atomicAdd(&lds[zbin * kHistCols + col], zc);
    __syncthreads();
    for (int b = threadIdx.x; b < kPdfSize; b += BLOCK)
    {
        // the bin's 32 columns as 8 16-B reads, started at a lane-dependent quarter so that the
        // 16 lanes of a ds_read_b128 group spread over the banks
        const uint4* row = reinterpret_cast<const uint4*>(lds + b * kHistCols);
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < kHistCols / 4; ++j)
        {
            const uint4 q = row[(j + b) & (kHistCols / 4 - 1)];
            s += q.x + q.y + q.z + q.w;
        }
        if (s)
            atomicAdd(&d.counts[b], (unsigned long long) s);
    }
}

template <int BLOCK, bool ENT, int COLS>
__global__ __launch_bounds__(BLOCK) void histogram_tensor_kernel(const float* __restrict__ x, int64_t n, int vec,
                                                                 TqDevice d)
{
    if (!BinnerOf<ENT>::live(d, 0))
        return;
    histogram_part<BLOCK, ENT, COLS>(x, n, vec, blockIdx.x, gridDim.x, d);
}

// per-channel: one workgroup per channel, counts written directly
template <bool ENT>
__global__ __launch_bounds__(kBlock) void histogram_channel_kernel(const float* __restrict__ x, int64_t outer,
                                                                   int64_t C, int64_t K, int vec, TqDevice d)
{
    __shared__ uint32_t lds[kWaves][kPdfSize];
    const int w = threadIdx.x >> 6;
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        if (!BinnerOf<ENT>::live(d, c))
            continue;
        typename BinnerOf<ENT>::type bn {d.bin_bucket[c], d.bin_offset[c]};
        for (int i = threadIdx.x; i < kWaves * kPdfSize; i += kBlock)
            (&lds[0][0])[i] = 0;
        __syncthreads();
        const int zbin = bn.bin(0.0f);
        uint32_t zc    = 0;
        auto add = [&](float v) {
            if (v == 0.0f)
            {
                ++zc;
                return;
            }
            int b = bn.bin(v);
            if (b >= 0)
                atomicAdd(&lds[w][b], 1u);
        };
        for (int64_t o = 0; o < outer; ++o)
        {
            const float* row = x + (o * C + c) * K;
            if (vec)
            {
                const float4* r4 = reinterpret_cast<const float4*>(row);
                for (int64_t k = threadIdx.x; k < K / 4; k += kBlock)
                {
                    float4 v = r4[k];
                    add(v.x);
                    add(v.y);
                    add(v.z);
                    add(v.w);
                }
            }
            else
            {
                for (int64_t k = threadIdx.x; k < K; k += kBlock)
                    add(row[k]);
            }
        }
        zc = wave_sum(zc);
        if ((threadIdx.x & 63) == 0 && zbin >= 0 && zc)
            atomicAdd(&lds[w][zbin], zc);
        __syncthreads();
        for (int b = threadIdx.x; b < kPdfSize; b += kBlock)
        {
            uint32_t s = 0;
#pragma unroll
            for (int i = 0; i < kWaves; ++i)
                s += lds[i][b];
            d.counts[c * kPdfSize + b] = s;
        }
        __syncthreads();
    }
}

// UpdatePdf:277-287 -- pdf = (pdf * it + count / N) / (it + 1), double, per bin.
// UpdatePdf:280-287 for channel c (one 512-lane workgroup): pdf = (pdf*it + cnt/N)/(it+1) in
// double; counts cleared for the next batch
__device__ __forceinline__ void fold_hist_one(const TqDevice& d, int64_t c, int64_t count)
{
    int it        = d.iterations[c];
    int64_t idx   = c * kPdfSize + threadIdx.x;
    double prob   = (double) d.counts[idx] / (double) count;
    // first batch: (0 * 0 + prob) / 1 == prob exactly (the PDF is zero since the reset), so the
    // old PDF is not read
    d.pdf[idx]    = it == 0 ? prob : (d.pdf[idx] * it + prob) / (it + 1);
    d.counts[idx] = 0;
    __syncthreads();
    if (threadIdx.x == 0)
        d.iterations[c] = it + 1;
    __syncthreads();
}

__global__ __launch_bounds__(kPdfSize) void fold_histogram_kernel(TqDevice d, int64_t C, int64_t count)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        if (!d.pdf_init[c])
            continue;
        fold_hist_one(d, c, count);
    }
}

__global__ __launch_bounds__(kPdfSize) void ent_fold_histogram_kernel(TqDevice d, int64_t C)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
        if (d.active[c])
            ent_fold_hist_one(d, c);
}

__global__ __launch_bounds__(kBlock) void reset_acc_kernel(double* acc, int64_t C)
{
    int64_t c = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (c < C)
    {
        acc[2 * c]     = DBL_MAX;    // TfEncodingAnalyzer.h:88
        acc[2 * c + 1] = -DBL_MAX;   // TfEncodingAnalyzer.h:89
    }
}

// one workgroup per quantizer
__global__ __launch_bounds__(kBlock) void reset_acc_many_kernel(const ResetJob* __restrict__ jobs)
{
    const ResetJob J = jobs[blockIdx.x];
    for (int64_t c = threadIdx.x; c < J.C; c += kBlock)
    {
        J.acc[2 * c]     = DBL_MAX;    // TfEncodingAnalyzer.h:88
        J.acc[2 * c + 1] = -DBL_MAX;   // TfEncodingAnalyzer.h:89
    }
}

// ---- many per-tensor quantizers in one launch per phase ---------------------------------------
// A calibration batch updates every activation quantizer of the model: per quantizer the single
// launches are min/max + combine + fold + histogram + PDF fold (5 launches, ~5 us each); for
// ViT-L's 99 quantizers that is ~500 launches per batch. Here each phase is ONE launch over all
// quantizers: workgroup -> quantizer = the last quantizer whose first workgroup is <= blockIdx.x.
// Every wave finds it with ONE round of loads (lane i reads quantizer i's first workgroup, a ballot
// counts those <= b) instead of a binary search's chain of dependent loads: under a full HBM queue
// each dependent load costs microseconds during which the new workgroup has no data load in flight.
template <class Job, class First>
__device__ __forceinline__ int find_job_ballot(const Job* __restrict__ jobs, int njobs, uint32_t b, First first)
{
    const int lane = threadIdx.x & 63;
    int count      = 0;
    for (int base = 0; base < njobs; base += 64)
    {
        const int i            = base + lane;
        const bool le          = i < njobs && first(jobs[i]) <= b;
        const unsigned long long m = __ballot(le);
        count += __popcll(m);
        if (m != ~0ull)
            break;   // first workgroups ascend: no later quantizer starts at or before b
    }
    return count - 1;
}

__device__ __forceinline__ int find_job(const StatsJob* __restrict__ jobs, int njobs, uint32_t b, bool hist)
{
    return hist ? find_job_ballot(jobs, njobs, b, [](const StatsJob& j) { return j.h_block0; })
                : find_job_ballot(jobs, njobs, b, [](const StatsJob& j) { return j.mm_block0; });
}

// One 16-KiB tile per step (4 x 16-B nontemporal loads per lane), the tiles of every quantizer in
// address order, one {-min, max} partial per tile: the workgroups in flight read one contiguous
// window of HBM (6.7 vs 5.9 TB/s for grid-stride workgroups inside each tensor,
// tools/studies/read_ceiling.py). A first batch of <= 64 quantizers runs one workgroup per tile (1.64 ms
// on ResNet-50's activations); later batches of PDF schemes, where every quantizer's range is
// fixed, and larger tables run kMmGrid workgroups that walk the tiles and skip a fixed quantizer
// at once (ViT-L/16 calibration: 900 -> 1016 Gelem/s; profiles/r02/compute_encodings_study.txt).
constexpr int64_t kMmTile = (int64_t) kBlock * 16;   // elements per tile
constexpr int kMmGrid     = 2048;                    // 256 CUs x 8 workgroups of 256 lanes
typedef const __attribute__((address_space(1))) f4* gf4p;

__device__ __forceinline__ float2 minmax_tile(const float* __restrict__ x, int64_t n, int vec, int64_t tile,
                                              bool last_tile)
{
    float mn = INFINITY, mx = -INFINITY;
    if (vec)
    {
        gf4p x4            = (gf4p) x;
        const int64_t nvec = n / 4;
        const int64_t base = tile * (kMmTile / 4) + threadIdx.x;
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)   // NaN padding is ignored by fminf/fmaxf
            v[u] = base + u * kBlock < nvec ? __builtin_nontemporal_load(x4 + base + u * kBlock)
                                            : f4 {NAN, NAN, NAN, NAN};
#pragma unroll
        for (int u = 0; u < 4; ++u)
            accum4(make_float4(v[u].x, v[u].y, v[u].z, v[u].w), mn, mx);
        if (last_tile)   // the last tile also takes the < 4 trailing elements
            for (int64_t i = nvec * 4 + threadIdx.x; i < n; i += kBlock)
            {
                mn = fminf(mn, x[i]);
                mx = fmaxf(mx, x[i]);
            }
    }
    else
    {
        const int64_t end = (tile + 1) * kMmTile < n ? (tile + 1) * kMmTile : n;
        for (int64_t i = tile * kMmTile + threadIdx.x; i < end; i += kBlock)
        {
            mn = fminf(mn, x[i]);
            mx = fmaxf(mx, x[i]);
        }
    }
    block_minmax(mn, mx);   // ends with the result in thread 0 (and an LDS barrier inside)
    return make_float2(-mn, mx);
}

// one tile per workgroup (the first batch: every tile is read)
__global__ __launch_bounds__(kBlock) void minmax_many_kernel(const StatsJob* __restrict__ jobs, int njobs)
{
    const StatsJob& J = jobs[find_job(jobs, njobs, blockIdx.x, false)];
    if (J.hist && !J.ent && !J.fresh && J.d.pdf_init[0])
        return;   // PDF schemes take min/max on the first (non-zero) batch only
    const int64_t tile = blockIdx.x - J.mm_block0;
    const float2 r     = minmax_tile(J.x, J.n, J.vec, tile, tile + 1 == (int64_t) J.mm_blocks);
    if (threadIdx.x == 0)
        reinterpret_cast<float2*>(J.mm_part)[tile] = r;
}

// kMmGrid workgroups walking the tiles (later batches of PDF schemes, whose quantizers all skip
// unless a range is still unset: a skip per quantizer instead of a workgroup per tile)
__global__ __launch_bounds__(kBlock) void minmax_walk_kernel(const StatsJob* __restrict__ jobs, int njobs,
                                                             uint32_t tiles)
{
    uint32_t t = blockIdx.x;
    if (t >= tiles)
        return;
    int ji = find_job(jobs, njobs, t, false);
    // the current quantizer's fields live in registers; tiles only grow, so the quantizer index
    // only steps forward and a tile costs no table load
    const float* x = nullptr;
    int64_t n = 0;
    float2* part = nullptr;
    uint32_t b0 = 0, next_b0 = 0;
    int vec = 0;
    bool skip = false;
    auto enter = [&](int j) {
        const StatsJob& J = jobs[j];
        x       = J.x;
        n       = J.n;
        vec     = J.vec;
        part    = reinterpret_cast<float2*>(J.mm_part);
        b0      = J.mm_block0;
        next_b0 = j + 1 < njobs ? jobs[j + 1].mm_block0 : tiles;
        // PDF schemes take min/max on the first (non-zero) batch only
        skip = J.hist && !J.ent && !J.fresh && J.d.pdf_init[0];
    };
    // the first quantizer after `from` that is not skipped (njobs if none): 64 job entries per
    // round of parallel loads, instead of one dependent load per skipped quantizer (a later ViT-L/16
    // batch, all 318 quantizers fixed, spent 417 us stepping through the table one job at a time)
    auto next_live = [&](int from) {
        const int lane = threadIdx.x & 63;
        for (int base = from; base < njobs; base += 64)
        {
            const int j = base + lane;
            bool live   = false;
            if (j < njobs)
            {
                const StatsJob& J = jobs[j];
                live              = !(J.hist && !J.ent && !J.fresh && J.d.pdf_init[0]);
            }
            const unsigned long long m = __ballot(live);
            if (m)
                return base + (int) __builtin_ctzll(m);
        }
        return njobs;
    };
    enter(ji);
    while (t < tiles)
    {
        while (t >= next_b0)
            enter(++ji);
        if (skip)
        {
            const int nj = next_live(ji + 1);
            if (nj >= njobs)
                break;
            const uint32_t b0n = jobs[nj].mm_block0;   // > t: every tile before it is skipped
            t += (b0n - t + gridDim.x - 1) / gridDim.x * gridDim.x;
            if (t >= tiles)
                break;
            ji = nj;
            enter(ji);
            continue;
        }
        const int64_t tile = t - b0;
        const float2 r     = minmax_tile(x, n, vec, tile, t + 1 == next_b0);
        if (threadIdx.x == 0)
            part[tile] = r;
        __syncthreads();   // the block reduction's LDS is reused by the next tile
        t += gridDim.x;
    }
}

// one workgroup per quantizer: partials -> minmax[0] = {-min, max}; optionally the fold
__global__ __launch_bounds__(kBlock) void combine_many_kernel(const StatsJob* __restrict__ jobs, int fold)
{
    const StatsJob& J = jobs[blockIdx.x];
    if (J.count_out && threadIdx.x == 0)
        *J.count_out = J.n;   // this rank's element count, summed over ranks with the bin counts
    if (J.hist && !J.ent && !J.fresh && J.d.pdf_init[0])
        return;
    const float2* partials = reinterpret_cast<const float2*>(J.mm_part);
    float a = -INFINITY, b = -INFINITY;
    // a 205-MB tensor leaves 12.5 K tile partials: 24 independent loads in flight per lane, so the
    // largest quantizer's partials arrive in two rounds of latency (8 per lane took ~22 us for
    // ResNet-50's 55 quantizers, the call's critical path between the two passes)
    constexpr int kU  = 24;
    const uint32_t nb = J.mm_blocks;
    for (uint32_t i0 = threadIdx.x; i0 < nb; i0 += kBlock * kU)
    {
        float2 p[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
            p[u] = i0 + u * kBlock < nb ? partials[i0 + u * kBlock] : make_float2(-INFINITY, -INFINITY);
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            a = fmaxf(a, p[u].x);
            b = fmaxf(b, p[u].y);
        }
    }
    float na = -a;
    block_minmax(na, b);
    __shared__ float2 res;
    if (threadIdx.x == 0)
    {
        res = make_float2(-na, b);
        reinterpret_cast<float2*>(J.d.minmax)[0] = res;
        if (fold && !J.ent)
            fold_one(J.d, 0, !J.hist);
    }
    if (fold && J.ent)
    {
        __syncthreads();
        ent_fold_one(J.d, 0, -res.x, res.y);
    }
}

// one workgroup per quantizer (the entropy fold redistributes 512 bins)
__global__ __launch_bounds__(kBlock) void fold_minmax_many_kernel(const StatsJob* __restrict__ jobs)
{
    const StatsJob& J = jobs[blockIdx.x];
    if (J.ent)
    {
        float2 m = reinterpret_cast<const float2*>(J.d.minmax)[0];
        ent_fold_one(J.d, 0, -m.x, m.y);
    }
    else if (threadIdx.x == 0)
        fold_one(J.d, 0, !J.hist);
}

template <int BLOCK, int COLS>
__global__ __launch_bounds__(BLOCK) void histogram_many_kernel(const StatsJob* __restrict__ jobs, int njobs)
{
    const StatsJob& J = jobs[find_job(jobs, njobs, blockIdx.x, true)];
    if (!J.hist)
        return;
    if (J.ent)
    {
        if (J.d.active[0])
            histogram_part<BLOCK, true, COLS>(J.x, J.n, J.vec, blockIdx.x - J.h_block0, J.h_blocks, J.d);
    }
    else if (J.d.pdf_init[0])
        histogram_part<BLOCK, false, COLS>(J.x, J.n, J.vec, blockIdx.x - J.h_block0, J.h_blocks, J.d);
}

__global__ __launch_bounds__(kPdfSize) void fold_histogram_many_kernel(const StatsJob* __restrict__ jobs)
{
    const StatsJob& J = jobs[blockIdx.x];
    if (!J.hist)
        return;
    if (J.ent)
    {
        if (J.d.active[0])
            ent_fold_hist_one(J.d, 0);
    }
    else if (J.d.pdf_init[0])
        fold_hist_one(J.d, 0, J.count_dev ? *J.count_dev : J.count);
}

// ---- many per-channel quantizers: updateStats in two launches ------------------------------
// ResNet-50's 54 weight quantizers took 4-5 launches each (min/max, fold, histogram, fold, and
// the PDF fold of every channel); a channel's fold depends only on its own statistics, so here
// the workgroup that reduces channel c also folds it.
__device__ __forceinline__ int find_channel_job(const ChannelJob* __restrict__ jobs, int njobs, uint32_t b)
{
    return find_job_ballot(jobs, njobs, b, [](const ChannelJob& j) { return j.block0; });
}

__device__ __forceinline__ void channel_minmax(const ChannelJob& J, int64_t c, float& mn, float& mx)
{
    mn = INFINITY;
    mx = -INFINITY;
    for (int64_t o = 0; o < J.outer; ++o)
    {
        const float* row = J.x + (o * J.C + c) * J.K;
        if (J.vec)
        {
            const float4* r4 = reinterpret_cast<const float4*>(row);
            for (int64_t k = threadIdx.x; k < J.K / 4; k += kBlock)
                accum4(r4[k], mn, mx);
        }
        else
        {
            for (int64_t k = threadIdx.x; k < J.K; k += kBlock)
            {
                mn = fminf(mn, row[k]);
                mx = fmaxf(mx, row[k]);
            }
        }
    }
}

// min/max of channel c + fold_one / ent_fold_one (fold_minmax_kernel, ent_fold_minmax_kernel)
__global__ __launch_bounds__(kBlock) void channel_minmax_fold_many_kernel(const ChannelJob* __restrict__ jobs,
                                                                          int njobs)
{
    const ChannelJob& J = jobs[find_channel_job(jobs, njobs, blockIdx.x)];
    const int64_t c     = blockIdx.x - J.block0;
    if (J.kind == kKindPdf && J.d.pdf_init[c])
        return;   // PDF schemes take min/max on the first (non-zero) batch only
    float mn, mx;
    channel_minmax(J, c, mn, mx);
    block_minmax(mn, mx);
    __shared__ float2 res;
    if (threadIdx.x == 0)
    {
        res = make_float2(-mn, mx);
        reinterpret_cast<float2*>(J.d.minmax)[c] = res;
        if (J.kind != kKindEntropy)
            fold_one(J.d, c, J.kind == kKindTf);
    }
    if (J.kind == kKindEntropy)
    {
        __syncthreads();
        ent_fold_one(J.d, c, -res.x, res.y);
    }
}

// histogram of channel c + the PDF fold (fold_hist_one) / entropy accumulation (ent_fold_hist_one),
// straight from the LDS counts
template <bool ENT>
__device__ __forceinline__ void channel_hist_fold(const ChannelJob& J, int64_t c)
{
    __shared__ uint32_t lds[kWaves][kPdfSize];
    const TqDevice& d = J.d;
    if (!BinnerOf<ENT>::live(d, c))
        return;
    const int w = threadIdx.x >> 6;
    typename BinnerOf<ENT>::type bn {d.bin_bucket[c], d.bin_offset[c]};
    for (int i = threadIdx.x; i < kWaves * kPdfSize; i += kBlock)
        (&lds[0][0])[i] = 0;
    __syncthreads();
    const int zbin = bn.bin(0.0f);
    uint32_t zc    = 0;
    auto add = [&](float v) {
        if (v == 0.0f)
        {
            ++zc;
            return;
        }
        int b = bn.bin(v);
        if (b >= 0)
            atomicAdd(&lds[w][b], 1u);
    };
    for (int64_t o = 0; o < J.outer; ++o)
    {
        const float* row = J.x + (o * J.C + c) * J.K;
        if (J.vec)
        {
            const float4* r4 = reinterpret_cast<const float4*>(row);
            for (int64_t k = threadIdx.x; k < J.K / 4; k += kBlock)
            {
                float4 v = r4[k];
                add(v.x);
                add(v.y);
                add(v.z);
                add(v.w);
            }
        }
        else
        {
            for (int64_t k = threadIdx.x; k < J.K; k += kBlock)
                add(row[k]);
        }
    }
    zc = wave_sum(zc);
    if ((threadIdx.x & 63) == 0 && zbin >= 0 && zc)
        atomicAdd(&lds[w][zbin], zc);
    __syncthreads();
    const int it       = d.iterations[c];
    const double count = (double) (J.outer * J.K);
    for (int b = threadIdx.x; b < kPdfSize; b += kBlock)
    {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < kWaves; ++i)
            s += lds[i][b];
        const int64_t idx = c * kPdfSize + b;
        if (ENT)
            d.pdf[idx] = d.pdf[idx] + (double) s;                        // math_functions.cpp:554-559
        else if (it == 0)   // (0 * 0 + p) / 1 == p exactly: the PDF is zero since the reset
            d.pdf[idx] = (double) s / count;
        else
            d.pdf[idx] = (d.pdf[idx] * it + (double) s / count) / (it + 1);   // UpdatePdf:280-287
    }
    __syncthreads();   // every lane has read iterations[c]
    if (threadIdx.x == 0)
        d.iterations[c] = it + 1;
}

__global__ __launch_bounds__(kBlock) void channel_hist_fold_many_kernel(const ChannelJob* __restrict__ jobs,
                                                                        int njobs)
{
    const ChannelJob& J = jobs[find_channel_job(jobs, njobs, blockIdx.x)];
    const int64_t c     = blockIdx.x - J.block0;
    if (J.kind == kKindEntropy)
        channel_hist_fold<true>(J, c);
    else if (J.kind == kKindPdf)
        channel_hist_fold<false>(J, c);
}

inline int grid_for_channels(int64_t C)
{
    return (int) (C < 65536 ? C : 65536);
}

}   // namespace

void launch_batch_minmax(const TqDevice& d, const float* x, int64_t outer, int64_t C, int64_t K, int skip_if_init,
                         hipStream_t s)
{
    bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    if (C == 1)
    {
        int64_t n  = outer * K;
        int blocks = stream_blocks(n, (int64_t) kBlock * 16);
        if (blocks > kMinmaxParts)
            blocks = kMinmaxParts;
        minmax_tensor_kernel<<<blocks, kBlock, 0, s>>>(x, n, al ? 1 : 0, reinterpret_cast<float2*>(d.partials),
                                                       d.pdf_init, skip_if_init);
        AIMET_LAUNCH_CHECK();
        minmax_combine_max_kernel<<<1, kBlock, 0, s>>>(reinterpret_cast<const float2*>(d.partials), blocks,
                                                       reinterpret_cast<float2*>(d.minmax), d.pdf_init, skip_if_init);
        AIMET_LAUNCH_CHECK();
    }
    else
    {
        int vec = (al && K % 4 == 0) ? 1 : 0;
        minmax_channel_kernel<<<grid_for_channels(C), kBlock, 0, s>>>(x, outer, C, K, vec,
                                                                      reinterpret_cast<float2*>(d.minmax), d.pdf_init,
                                                                      skip_if_init);
        AIMET_LAUNCH_CHECK();
    }
}

void launch_fold_minmax(const TqDevice& d, int64_t C, StatsKind kind, hipStream_t s)
{
    if (kind == kKindEntropy)
        ent_fold_minmax_kernel<<<grid_for_channels(C), kBlock, 0, s>>>(d, C);
    else
        fold_minmax_kernel<<<(int) ceil_div(C, kBlock), kBlock, 0, s>>>(d, C, kind == kKindTf ? 1 : 0);
    AIMET_LAUNCH_CHECK();
}

template <bool ENT>
static void launch_hist_tensor(unsigned grid, const float* x, int64_t n, int vec, const TqDevice& d, hipStream_t s)
{
    histogram_tensor_kernel<1024, ENT, 16><<<grid, 1024, 0, s>>>(x, n, vec, d);
}

template <bool ENT>
static void batch_histogram(const TqDevice& d, const float* x, int64_t outer, int64_t C, int64_t K, hipStream_t s)
{
    bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    if (C == 1)
    {
        int64_t n = outer * K;
        // workgroups of 1024 lanes sharing one [512][16] LDS histogram (32 KiB: two per CU), each
        // a contiguous share of ~128 K elements, the grid capped at 2 per CU (256 / 512-lane and
        // 8 / 32-column shapes measured slower, tools/studies/hist_many_tune.py)
        const int64_t per = (int64_t) 1024 * kHistUnroll * 4 * 8;
        int64_t blocks    = ceil_div(n, per);
        const int64_t cap = 256 * 2;
        blocks            = blocks < 1 ? 1 : (blocks > cap ? cap : blocks);
        launch_hist_tensor<ENT>((unsigned) blocks, x, n, al ? 1 : 0, d, s);
        AIMET_LAUNCH_CHECK();
    }
    else
    {
        int vec = (al && K % 4 == 0) ? 1 : 0;
        histogram_channel_kernel<ENT><<<grid_for_channels(C), kBlock, 0, s>>>(x, outer, C, K, vec, d);
    }
    AIMET_LAUNCH_CHECK();
}

void launch_batch_histogram(const TqDevice& d, const float* x, int64_t outer, int64_t C, int64_t K, StatsKind kind,
                            hipStream_t s)
{
    if (kind == kKindEntropy)
        batch_histogram<true>(d, x, outer, C, K, s);
    else if (kind == kKindPdf)
        batch_histogram<false>(d, x, outer, C, K, s);
}

void launch_fold_histogram(const TqDevice& d, int64_t C, int64_t count, StatsKind kind, hipStream_t s)
{
    if (kind == kKindEntropy)
        ent_fold_histogram_kernel<<<grid_for_channels(C), kPdfSize, 0, s>>>(d, C);
    else if (kind == kKindPdf)
        fold_histogram_kernel<<<grid_for_channels(C), kPdfSize, 0, s>>>(d, C, count);
    else
        return;
    AIMET_LAUNCH_CHECK();
}

// elements per workgroup of the batched histogram pass; 1024 lanes sharing one [512][16] LDS
// histogram (profiles/r03: ViT-L/16 later batches 2.8-2.9 ms vs 3.1-3.2 with 512 lanes and 4.7 with
// 512 lanes x 32 columns)
constexpr int64_t kHistElemsPerBlock = 131072;

void stats_layout(std::vector<StatsJob>& jobs, uint64_t* mm_out, uint64_t* hb_out)
{
    uint64_t mm = 0, hb = 0;
    for (auto& j: jobs)
    {
        j.mm_block0 = (uint32_t) mm;
        j.mm_blocks = (uint32_t) std::max<int64_t>(1, ceil_div(j.n, kMmTile));
        j.h_block0  = (uint32_t) hb;
        j.h_blocks  = (uint32_t) (j.hist ? std::max<int64_t>(1, std::min<int64_t>(kHistGrid,
                                                                               ceil_div(j.n, kHistElemsPerBlock)))
                                         : 0);
        mm += j.mm_blocks;
        hb += j.h_blocks;
    }
    AIMET_REQUIRE(mm < (uint64_t(1) << 31) && hb < (uint64_t(1) << 31), "too many workgroups");
    *mm_out = mm;
    *hb_out = hb;
}

// walk the tiles when every quantizer is a PDF scheme that has seen a batch (its range is almost
// surely fixed) or when the job table needs more than one ballot round per workgroup (> 64
// quantizers: ViT-L/16's 318 read their first batch in 5.8 ms walking vs 7.1 ms one tile per
// workgroup)
bool stats_walk(const StatsJob* jobs, int n)
{
    bool fixed = true;
    for (int i = 0; i < n; ++i)
        fixed = fixed && jobs[i].hist && !jobs[i].ent && jobs[i].seen;
    return n > 64 || fixed;
}

void launch_stats_table(const StatsJob* dj, int n, uint64_t mm, uint64_t hb, bool walk, int phases, hipStream_t s,
                        const std::function<void()>& between)
{
    if (n == 0)
        return;
    if (phases & kPhaseMinmax)
    {
        if (walk)
            minmax_walk_kernel<<<(unsigned) std::min<uint64_t>(mm, kMmGrid), kBlock, 0, s>>>(dj, n, (uint32_t) mm);
        else
            minmax_many_kernel<<<(unsigned) mm, kBlock, 0, s>>>(dj, n);
        AIMET_LAUNCH_CHECK();
    }
    if (between)
        between();
    if (phases & kPhaseMinmax)
    {
        combine_many_kernel<<<n, kBlock, 0, s>>>(dj, (phases & kPhaseFoldMinmax) ? 1 : 0);
        AIMET_LAUNCH_CHECK();
    }
    else if (phases & kPhaseFoldMinmax)
    {
        fold_minmax_many_kernel<<<(unsigned) n, kBlock, 0, s>>>(dj);
        AIMET_LAUNCH_CHECK();
    }
    if ((phases & kPhaseHistogram) && hb > 0)
    {
        histogram_many_kernel<1024, 16><<<(unsigned) hb, 1024, 0, s>>>(dj, n);
        AIMET_LAUNCH_CHECK();
    }
    if (phases & kPhaseFoldHistogram)
    {
        fold_histogram_many_kernel<<<n, kPdfSize, 0, s>>>(dj);
        AIMET_LAUNCH_CHECK();
    }
}

void launch_stats_many(std::vector<StatsJob>& jobs, int phases, hipStream_t s, const std::function<void()>& between)
{
    if (jobs.empty())
        return;
    uint64_t mm = 0, hb = 0;
    stats_layout(jobs, &mm, &hb);
    const int n = (int) jobs.size();
    float* parts = nullptr;
    if (phases & kPhaseMinmax)
    {
        parts = static_cast<float*>(scratch_alloc(sizeof(float) * 2 * mm, s));
        for (auto& j: jobs)
            j.mm_part = parts + 2 * (int64_t) j.mm_block0;
    }
    auto* dj = static_cast<StatsJob*>(upload_async(jobs.data(), sizeof(StatsJob) * n, s));
    try
    {
        launch_stats_table(dj, n, mm, hb, stats_walk(jobs.data(), n), phases, s, between);
    }
    catch (...)
    {
        if (parts)
            scratch_free(parts, s);
        scratch_free(dj, s);
        throw;
    }
    if (parts)
        scratch_free(parts, s);
    scratch_free(dj, s);
}

uint64_t channel_layout(std::vector<ChannelJob>& jobs, bool* any_hist)
{
    uint64_t blocks = 0;
    bool hist       = false;
    for (auto& j: jobs)
    {
        j.block0 = (uint32_t) blocks;
        blocks += (uint64_t) j.C;
        hist = hist || j.kind != kKindTf;
    }
    AIMET_REQUIRE(blocks < (uint64_t(1) << 31), "too many channels");
    *any_hist = hist;
    return blocks;
}

void launch_channel_table(const ChannelJob* dj, int n, uint64_t blocks, bool any_hist, hipStream_t s)
{
    if (n == 0 || blocks == 0)
        return;
    channel_minmax_fold_many_kernel<<<(unsigned) blocks, kBlock, 0, s>>>(dj, n);
    AIMET_LAUNCH_CHECK();
    if (any_hist)
    {
        channel_hist_fold_many_kernel<<<(unsigned) blocks, kBlock, 0, s>>>(dj, n);
        AIMET_LAUNCH_CHECK();
    }
}

void launch_channel_stats_many(std::vector<ChannelJob>& jobs, hipStream_t s)
{
    if (jobs.empty())
        return;
    bool any_hist         = false;
    const uint64_t blocks = channel_layout(jobs, &any_hist);
    const int n           = (int) jobs.size();
    auto* dj              = static_cast<ChannelJob*>(upload_async(jobs.data(), sizeof(ChannelJob) * n, s));
    launch_channel_table(dj, n, blocks, any_hist, s);
    scratch_free(dj, s);
}

void launch_reset_table(const ResetJob* dj, int n, hipStream_t s)
{
    if (n == 0)
        return;
    reset_acc_many_kernel<<<(unsigned) n, kBlock, 0, s>>>(dj);
    AIMET_LAUNCH_CHECK();
}

void launch_reset_state_many(const std::vector<ResetJob>& jobs, hipStream_t s)
{
    if (jobs.empty())
        return;
    auto* dj = static_cast<ResetJob*>(upload_async(jobs.data(), sizeof(ResetJob) * jobs.size(), s));
    launch_reset_table(dj, (int) jobs.size(), s);
    scratch_free(dj, s);
}

// blockIdx.y = job; the workgroups along x stride over the job's 16-B words, then its tail bytes
// any byte range: the 16-B aligned middle with vector stores, the unaligned head (e.g. a
// quantizer's {-min, max} inside a packed exchange buffer) and tail byte by byte
__global__ __launch_bounds__(kBlock) void zero_many_kernel(const ZeroJob* __restrict__ jobs)
{
    const ZeroJob J   = jobs[blockIdx.y];
    unsigned char* b  = static_cast<unsigned char*>(J.p);
    const int64_t mis = (int64_t) (reinterpret_cast<uintptr_t>(b) & 15);
    const int64_t head = mis ? (16 - mis < J.bytes ? 16 - mis : J.bytes) : 0;
    const int64_t nq  = (J.bytes - head) / 16;
    f4* q             = reinterpret_cast<f4*>(b + head);
    const f4 z        = {0.f, 0.f, 0.f, 0.f};
    const int64_t str = (int64_t) gridDim.x * kBlock;
    for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < nq; i += str)
        q[i] = z;
    if (blockIdx.x == 0)
    {
        for (int64_t i = threadIdx.x; i < head; i += kBlock)
            b[i] = 0;
        for (int64_t i = head + nq * 16 + threadIdx.x; i < J.bytes; i += kBlock)
            b[i] = 0;
    }
}

void launch_zero_table(const ZeroJob* dj, int n, int64_t most, hipStream_t s)
{
    if (n == 0)
        return;
    AIMET_REQUIRE(n < 65536, "too many ranges to zero in one launch");
    const int64_t bx = std::max<int64_t>(1, std::min<int64_t>(64, ceil_div(most / 16, (int64_t) kBlock * 8)));
    zero_many_kernel<<<dim3((unsigned) bx, (unsigned) n), kBlock, 0, s>>>(dj);
    AIMET_LAUNCH_CHECK();
}

void launch_zero_many(const std::vector<ZeroJob>& jobs, hipStream_t s)
{
    if (jobs.empty())
        return;
    AIMET_REQUIRE(jobs.size() < 65536, "too many ranges to zero in one launch");
    int64_t most = 0;
    for (const ZeroJob& j: jobs)
        most = std::max(most, j.bytes);
    auto* dj = static_cast<ZeroJob*>(upload_async(jobs.data(), sizeof(ZeroJob) * jobs.size(), s));
    launch_zero_table(dj, (int) jobs.size(), most, s);
    scratch_free(dj, s);
}

void launch_reset_state(const TqDevice& d, int64_t C, bool hist, hipStream_t s)
{
    (void) hist;
    reset_acc_kernel<<<(int) ceil_div(C, kBlock), kBlock, 0, s>>>(d.acc, C);
    AIMET_LAUNCH_CHECK();
}

}   // namespace aimet_amd
